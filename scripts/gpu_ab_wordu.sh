#!/bin/bash
# A/B: words in flight per wave step of k_descent_init / k_regrow_init (CTWS_WORD_U 4 / 8),
# single-stream stage times of configs 3 and 4.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ab
for c in 3 4; do
  for u in 4 8 4 8; do
    CTWS_WORD_U=$u timeout -k 10 200 python -u bench.py --config $c --streams 1 --steps 3 --warmup 1 --no-host --no-cpu-baseline --no-e2e --no-strong > gpurun_out/ab/wu_c${c}_u$u.json 2> gpurun_out/ab/wu_c${c}_u$u.err || { tail -5 gpurun_out/ab/wu_c${c}_u$u.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab/wu_c${c}_u$u.json').read().strip().splitlines()[-1]); s=d['stage_ms_1stream']; print('c$c U$u', d['ms_per_step'], 'descent', s['flood_descent'], 'size_filter', s['size_filter'])"
  done
done
