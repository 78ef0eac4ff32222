#!/bin/bash
# Round 6: seed members carrying their labels (k_member_label): parity, then the descent-tile A/B
# (CTWS_MEMBER_LABEL=0 = the previous path on the same build).
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_config_blocks.py tests/test_golden_gpu.py tests/test_gpu_pass2.py tests/test_from_seeds_gpu.py tests/test_corridor_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for c in 3 4; do
  for k in 1 2; do
    for v in 1 0; do
      CTWS_MEMBER_LABEL=$v timeout -k 10 200 python -u bench.py --config $c --streams 1 --steps 2 --warmup 1 --no-host --no-cpu-baseline --no-e2e --no-strong --no-threshcc --no-config5 > $O/c${c}_ml${v}_$k.json 2> $O/c${c}_ml${v}_$k.err || { tail -5 $O/c${c}_ml${v}_$k.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/c${c}_ml${v}_$k.json').read().strip().splitlines()[-1]); s=d['stage_ms_1stream']; print('c$c ml$v', d['ms_per_step'], {k: round(v, 2) for k, v in s.items() if k in ('seeds', 'descent_tile', 'flood_descent', 'flood_relax')})"
    done
  done
done
