#!/bin/bash
# Round 6: seed components from the classes (k_seed_members, 2-D k_seed_union2): parity (seeds bit-exact,
# the tile-CC path as a variant), then the A/B on the same build (CTWS_SEED_TILECC=1 = tiles).
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_config_blocks.py tests/test_golden_gpu.py tests/test_gpu_pass2.py tests/test_frontier_variants.py tests/test_from_seeds_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for c in 3 4 5; do
  for k in 1 2; do
    for v in 0 1; do
      CTWS_SEED_TILECC=$v timeout -k 10 200 python -u bench.py --config $c --streams 1 --steps 2 --warmup 1 --no-host --no-cpu-baseline --no-e2e --no-strong --no-threshcc --no-config5 > $O/c${c}_t${v}_$k.json 2> $O/c${c}_t${v}_$k.err || { tail -5 $O/c${c}_t${v}_$k.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/c${c}_t${v}_$k.json').read().strip().splitlines()[-1]); s=d['stage_ms_1stream']; print('c$c tilecc=$v', d['ms_per_step'], {k: round(v, 2) for k, v in s.items() if k in ('seeds', 'crop_cc', 'flood_relax')})"
    done
  done
done
