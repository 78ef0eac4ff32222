#!/bin/bash
# Round 6: seed members with 8 words in flight, 2-D seed components from the classes
# (k_seed_union2): parity (pass 2, parity, variants incl. the tile-CC seeds), then the A/B on
# configs 3 / 4 / 5 against the previous build (libctws_prev.so).
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_pass2.py tests/test_from_seeds_gpu.py tests/test_golden_gpu.py tests/test_gpu_parity.py tests/test_config_blocks.py tests/test_frontier_variants.py tests/test_corridor_gpu.py tests/test_pass2_ranks.py tests/test_bench_two_pass_ranks.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for c in 3 4 5; do
  for k in 1 2; do
    for v in new prev; do
      unset CTWS_LIB
      [ $v = prev ] && export CTWS_LIB=$PWD/cluster_tools_amd/libctws_prev.so
      timeout -k 10 200 python -u bench.py --config $c --streams 1 --steps 2 --warmup 1 --no-host --no-cpu-baseline --no-e2e --no-strong --no-threshcc --no-config5 > $O/c${c}_${v}_$k.json 2> $O/c${c}_${v}_$k.err || { tail -5 $O/c${c}_${v}_$k.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/c${c}_${v}_$k.json').read().strip().splitlines()[-1]); s=d['stage_ms_1stream']; print('c$c $v', d['ms_per_step'], {k: round(v, 2) for k, v in s.items() if k in ('seeds', 'flood_relax', 'size_filter')})"
    done
  done
done
