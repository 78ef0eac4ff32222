#!/bin/bash
# ThresholdedComponents GPU tests (k_threshcc.hip), then the quick parity suite + config 3.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/threshcc
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_threshcc_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/threshcc/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/threshcc/pytest.log; [ $rc -ne 0 ] && exit $rc
CONFIGS=${CONFIGS:-3} bash scripts/gpu_quick.sh
