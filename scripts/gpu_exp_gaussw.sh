#!/bin/bash
# Gaussian sliding-window column tile width (CTWS_GAUSS_W): parity, then single-stream smooth_seeds time
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/gw
export TMPDIR=/tmp
CTWS_GAUSS_W=16 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gw/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/gw/pytest.log)"
[ $rc -ne 0 ] && exit $rc
for w in 32 16 8; do
  CTWS_GAUSS_W=$w timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --streams 1 > gpurun_out/gw/w$w.log 2>&1
  rc=$?; echo "w $w rc=$rc $(python -c "import json; d=json.loads([l for l in open('gpurun_out/gw/w$w.log') if l.startswith('{')][0]); s=d['stage_ms_1stream']; print(d['value'], s['smooth_seeds'], s['hmap'])")"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
