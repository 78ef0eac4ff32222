#!/bin/bash
# Round 6: the masked plateau fill's scans with more loads in flight (x: whole rows of up to 512
# voxels in registers; y / z: 16 positions per step): parity on the experimental build
# (libctws_exp.so as CTWS_LIB), then config 5 A/B against the current build.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06r
mkdir -p $O
export TMPDIR=/tmp
CTWS_LIB=$PWD/cluster_tools_amd/libctws_exp.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_config_blocks.py tests/test_corridor_gpu.py tests/test_frontier_variants.py tests/test_gpu_pass2.py tests/test_from_seeds_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for k in 1 2; do
  for v in exp cur; do
    unset CTWS_LIB
    [ $v = exp ] && export CTWS_LIB=$PWD/cluster_tools_amd/libctws_exp.so
    timeout -k 10 200 python -u bench.py --config 5 --streams 1 --steps 2 --warmup 1 --no-host --no-cpu-baseline --no-e2e --no-strong --no-threshcc --no-config5 > $O/c5_${v}_$k.json 2> $O/c5_${v}_$k.err || { tail -5 $O/c5_${v}_$k.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c5_${v}_$k.json').read().strip().splitlines()[-1]); s=d['stage_ms_1stream']; print('c5 $v', d['ms_per_step'], {k: round(v, 2) for k, v in s.items() if k in ('flood_relax', 'flood_verify', 'seeds')})"
  done
done
