#!/bin/bash
# Single-stream stage times of CONFIGS (no tests): timing experiments only.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/st
for c in ${CONFIGS:-3 4}; do
  timeout -k 10 200 python -u bench.py --config $c --streams 1 --steps 3 --warmup 1 --no-host --no-cpu-baseline --no-e2e --no-strong > gpurun_out/st/c$c.json 2> gpurun_out/st/c$c.err || { tail -5 gpurun_out/st/c$c.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/st/c$c.json').read().strip().splitlines()[-1]); s=d['stage_ms_1stream']; print('c$c', d['ms_per_step'], {k: v for k, v in s.items() if v >= 0.5 and k not in ('frontier_iters', 'regrow_iters', 'flood_packed')})"
done
