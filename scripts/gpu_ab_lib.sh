#!/bin/bash
# Same-box A/B of two library builds (CTWS_LIB=$ALT vs the default libctws.so), alternating,
# single-stream flood stage times.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/ab_lib${TAG:+_$TAG}
mkdir -p $O
export TMPDIR=/tmp
ALT=${ALT:-cluster_tools_amd/libctws_old.so}
for c in ${CONFIGS:-4 3}; do
  for k in 1 2; do
    for v in new old; do
      if [ $v = old ]; then export CTWS_LIB=$PWD/$ALT; else unset CTWS_LIB; fi
      timeout -k 10 200 python -u bench.py --config $c --streams 1 --steps 2 --warmup 1 --no-host --no-cpu-baseline --no-e2e --no-strong --no-threshcc --no-config5 > $O/c${c}_${v}_$k.json 2> $O/c${c}_${v}_$k.err || { tail -5 $O/c${c}_${v}_$k.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/c${c}_${v}_$k.json').read().strip().splitlines()[-1]); s=d['stage_ms_1stream']; print('c$c $v', d['ms_per_step'], {k: v for k, v in s.items() if k in ('flood_relax', 'size_filter', 'descent_tile', 'crop_cc')})"
    done
  done
done
