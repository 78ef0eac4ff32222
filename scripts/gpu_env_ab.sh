#!/bin/bash
# A/B of environment settings (arguments, e.g. CTWS_FRONTIER_GRID=768): single-stream stage
# times of config ${C:-3}, each setting run twice in alternation.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/envab
c=${C:-3}
for rep in 1 2; do
  for v in "$@"; do
    tag=$(echo "$v" | tr '=, ' '___')
    env ${v//,/ } timeout -k 10 200 python -u bench.py --config $c --streams 1 --steps 3 --warmup 1 --no-host --no-cpu-baseline --no-e2e --no-strong > gpurun_out/envab/c${c}_${tag}_$rep.json 2> gpurun_out/envab/c${c}_${tag}_$rep.err || { tail -5 gpurun_out/envab/c${c}_${tag}_$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/envab/c${c}_${tag}_$rep.json').read().strip().splitlines()[-1]); s=d['stage_ms_1stream']; print('$v', d['ms_per_step'], 'relax', s['flood_relax'], 'size_filter', s['size_filter'])"
  done
done
