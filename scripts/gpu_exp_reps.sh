#!/bin/bash
# parity of the frontier with local sweeps, then a sweep of CTWS_FRONTIER_REPS on the bench
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/reps
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_golden_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/reps/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/reps/pytest.log
[ $rc -ne 0 ] && exit $rc
for r in 1 2 4 8 16; do
  CTWS_FRONTIER_REPS=$r timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --streams ${STREAMS:-2} > gpurun_out/reps/r$r.log 2>&1
  rc=$?; echo "reps $r rc=$rc"; python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/reps/r$r.log') if l.startswith('{')][0]); s=d['stage_ms']; print(d['value'], s['flood_relax'], s['frontier_iters'])"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
