#!/bin/bash
# Frontier statistics (CTWS_TRACE=1): open voxels, visits, key writes per step, configs 3/4/5.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06_fstats
mkdir -p $O
export TMPDIR=/tmp
for c in ${CONFIGS:-3 4 5}; do
  CTWS_TRACE=1 timeout -k 10 300 python -u bench.py --config $c --streams 1 --steps 1 --warmup 0 --no-host --no-cpu-baseline --no-e2e --no-strong --no-threshcc --no-config5 > $O/c$c.json 2> $O/c$c.err || { tail -5 $O/c$c.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c$c.json').read().strip().splitlines()[-1]); s=d['stage_ms_1stream']; print('c$c', {k: s.get(k) for k in ('open_voxels', 'frontier_visits', 'frontier_key_writes', 'flood_relax', 'frontier_iters')})"
done
