#!/bin/bash
# Round 6: the seed-stage and whole-block repeatability tests at 40 runs x 3 blocks per case.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06w
mkdir -p $O
export TMPDIR=/tmp
CTWS_TEST_REPS=40 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -k "repeatable" > $O/pytest.log 2>&1
echo "rc=$?"; grep -E "passed|failed|Mismatch|FAILED" $O/pytest.log | head -20
