#!/bin/bash
# parity of the flood kernels, then the bench on 1 and 3 streams
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/q
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_golden_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/q/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/q/pytest.log)"
[ $rc -ne 0 ] && exit $rc
for s in 1 3; do
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --streams $s > gpurun_out/q/s$s.log 2>&1
  rc=$?; echo "streams $s rc=$rc $(python -c "import json; d=json.loads([l for l in open('gpurun_out/q/s$s.log') if l.startswith('{')][0]); s=d['stage_ms_1stream']; print(d['value'], s['descent_tile'], s['flood_relax'])")"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
