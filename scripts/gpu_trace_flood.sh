#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for c in ${CONFIGS:-3 4}; do
  CTWS_TRACE=1 timeout -k 10 300 python3 -u bench.py --config $c --steps 1 --warmup 0 --streams 1 --no-cpu-baseline --no-host > gpurun_out/trace_c$c.log 2> gpurun_out/trace_c$c.err
  rc=$?; [ $rc -ne 0 ] && { tail -3 gpurun_out/trace_c$c.err; exit $rc; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/trace_c$c.log').read().strip().splitlines()[-1])
s=d['stage_ms_1stream']; o=d['config']['outer_voxels_per_gpu']
print('c$c open', s.get('open_voxels'), 'frac %.3f' % (s.get('open_voxels',0)/o/2), 'visits', s.get('frontier_visits'), 'visits/open %.2f' % (s.get('frontier_visits',0)/max(1,s.get('open_voxels',1))))"
done
exit 0
