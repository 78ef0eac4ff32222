#!/bin/bash
# Round 6: the whole GPU suite, then A/B of the gauss_yx interior staging vs the round-5 build.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for c in 3 4; do
  for k in 1 2; do
    for v in new old; do
      if [ $v = old ]; then export CTWS_LIB=$PWD/cluster_tools_amd/libctws_old.so; else unset CTWS_LIB; fi
      timeout -k 10 200 python -u bench.py --config $c --streams 1 --steps 2 --warmup 1 --no-host --no-cpu-baseline --no-e2e --no-strong --no-threshcc --no-config5 > $O/c${c}_${v}_$k.json 2> $O/c${c}_${v}_$k.err || { tail -5 $O/c${c}_${v}_$k.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/c${c}_${v}_$k.json').read().strip().splitlines()[-1]); s=d['stage_ms_1stream']; print('c$c $v', d['ms_per_step'], {k: round(v, 2) for k, v in s.items() if k in ('flood_relax', 'crop_cc', 'seeds', 'edt_yz', 'smooth_seeds', 'hmap')})"
    done
  done
done
