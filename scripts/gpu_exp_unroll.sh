#!/bin/bash
# frontier list entries in flight per lane (CTWS_FRONTIER_UNROLL) x local sweeps (CTWS_FRONTIER_REPS):
# parity of the variants, then single-stream flood_relax time
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/un
export TMPDIR=/tmp
for u in 1; do
  CTWS_FRONTIER_UNROLL=$u timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/un/pytest_u$u.log 2>&1
  rc=$?; echo "pytest u$u rc=$rc $(tail -1 gpurun_out/un/pytest_u$u.log)"
  [ $rc -ne 0 ] && exit $rc
done
for u in 1 2; do for r in 4 8 16; do
  CTWS_FRONTIER_UNROLL=$u CTWS_FRONTIER_REPS=$r timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --streams 1 > gpurun_out/un/u${u}r$r.log 2>&1
  rc=$?; echo "u$u r$r rc=$rc $(python -c "import json; d=json.loads([l for l in open('gpurun_out/un/u${u}r$r.log') if l.startswith('{')][0]); print(d['value'], d['stage_ms']['flood_relax'])")"
  [ $rc -ne 0 ] && exit $rc
done; done
exit 0
