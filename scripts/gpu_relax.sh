#!/bin/bash
# flood relaxation: parity subset, then single-stream kernel times of CTWS_RELAX=1 (LDS tiles) vs 0 (frontier)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_config_blocks.py tests/test_from_seeds_gpu.py} -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_relax.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_relax.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for c in ${CONFIGS:-3}; do
for v in ${VALUES:-1 0}; do
  CTWS_RELAX=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/relax_c${c}_$v -o run --output-format csv -- \
    python3 -u bench.py --config $c --streams 1 --steps 1 --warmup 1 --no-cpu-baseline --no-host > gpurun_out/relax_c${c}_$v.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "relax=$v rc=$rc"; tail -3 gpurun_out/relax_c${c}_$v.log; exit $rc; }
  python3 scripts/prof_table.py 2 gpurun_out/relax_c${c}_$v > gpurun_out/relax_c${c}_$v.table 2>&1
  echo "== c$c CTWS_RELAX=$v: $(grep -o '"value": [0-9.]*' gpurun_out/relax_c${c}_$v.log | head -1) $(grep -o '"flood_relax": [0-9.]*' gpurun_out/relax_c${c}_$v.log | tail -1)"
  grep -E "k_tile_relax|k_frontier|k_flood_verify|k_descent|k_regrow|k_output" gpurun_out/relax_c${c}_$v.table
done
done
exit 0
