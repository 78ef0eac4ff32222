#!/bin/bash
# streams 2 vs 3 (twice each), then one traced run (open voxels, frontier visits)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/st
export TMPDIR=/tmp
for s in 2 3 2 3 4; do
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --streams $s > gpurun_out/st/s$s.log 2>&1
  rc=$?; echo "streams $s rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/st/s$s.log)"
  [ $rc -ne 0 ] && exit $rc
done
CTWS_TRACE=1 timeout -k 10 200 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --streams 1 > gpurun_out/st/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; python -c "import json; d=json.loads([l for l in open('gpurun_out/st/trace.log') if l.startswith('{')][0]); print({k:v for k,v in d['stage_ms'].items() if 'open' in k or 'visit' in k or 'iters' in k})"
exit $rc
