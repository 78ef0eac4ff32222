#!/bin/bash
# flood schedule sweep on config 3 (and 4): frontier iterations before the tile flood, local sweeps
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for v in "CTWS_FRONTIER_ITERS=0" "CTWS_FRONTIER_ITERS=2" "CTWS_FRONTIER_REPS=8" "CTWS_FRONTIER_REPS=16" "CTWS_VERIFY_UNFUSED=1" "CTWS_VERIFY=0"; do
  for c in ${CONFIGS:-3}; do
    env $v timeout -k 10 300 python3 -u bench.py --config $c --steps 2 --warmup 1 --streams 1 --no-cpu-baseline --no-host > gpurun_out/exp_flood.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "$v rc=$rc"; tail -3 gpurun_out/exp_flood.log; exit $rc; }
    python3 -c "
import json
d=json.loads(open('gpurun_out/exp_flood.log').read().strip().splitlines()[-1])
s=d['stage_ms_1stream']
print('$v c$c', d['value'], d['ms_per_step'], 'relax', s.get('flood_relax'), 'verify', s.get('flood_verify'), 'sf', s.get('size_filter'), 'it', s.get('frontier_iters'), 'rounds', s.get('flood_rounds'), 'fb', s.get('flood_fallback'))"
  done
done
exit 0
