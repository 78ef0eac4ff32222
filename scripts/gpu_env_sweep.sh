#!/bin/bash
# Single-stream stage times of configs over environment knob settings (VARIANTS, comma-joined).
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/env_sweep${TAG:+_$TAG}
mkdir -p $O
export TMPDIR=/tmp
for c in ${CONFIGS:-4 3}; do
  for v in ${VARIANTS:-CTWS_FRONTIER_REPS=32}; do
    tag=$(echo "$v" | tr '=, ' '___')
    ( export $(echo $v | tr ',' ' '); timeout -k 10 200 python -u bench.py --config $c --streams 1 --steps 2 --warmup 1 --no-host --no-cpu-baseline --no-e2e --no-strong --no-threshcc --no-config5 > $O/c${c}_$tag.json 2> $O/c${c}_$tag.err ) || { tail -5 $O/c${c}_$tag.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c${c}_$tag.json').read().strip().splitlines()[-1]); s=d['stage_ms_1stream']; print('c$c $v', d['ms_per_step'], {k: v for k, v in s.items() if k in ('flood_relax', 'size_filter', 'frontier_iters', 'regrow_iters')})"
  done
done
