#!/bin/bash
# Round 6: 2-D seeds back on the tile CC, the masked plateau fill's register scans; the whole GPU
# suite + smoke on this build, then configs 3 / 5 A/B against the previous build (libctws_prev.so),
# then the default bench line.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06s
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
for c in 3 5; do
  for v in cur prev; do
    unset CTWS_LIB
    [ $v = prev ] && export CTWS_LIB=$PWD/cluster_tools_amd/libctws_prev.so
    timeout -k 10 200 python -u bench.py --config $c --streams 1 --steps 2 --warmup 1 --no-host --no-cpu-baseline --no-e2e --no-strong --no-threshcc --no-config5 > $O/c${c}_${v}.json 2> $O/c${c}_${v}.err || { tail -5 $O/c${c}_${v}.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c${c}_${v}.json').read().strip().splitlines()[-1]); s=d['stage_ms_1stream']; print('c$c $v', d['ms_per_step'], {k: round(v, 2) for k, v in s.items() if k in ('seeds', 'plateau', 'flood_relax')})"
  done
done
unset CTWS_LIB
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-400
