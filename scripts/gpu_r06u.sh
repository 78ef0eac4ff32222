#!/bin/bash
# Round 6: the seed-stage repeatability test on the current build, then on the previous build with
# the 2-D listed-maxima seed union (libctws_union.so), 8 x 3 runs per case.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06u
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "repeatable" > $O/pytest_cur.log 2>&1
rc=$?; tail -2 $O/pytest_cur.log; [ $rc -ne 0 ] && exit $rc
CTWS_LIB=$PWD/cluster_tools_amd/libctws_union.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread -k "repeatable" > $O/pytest_union.log 2>&1
echo "union rc=$?"; grep -E "passed|failed|Mismatch|FAILED" $O/pytest_union.log | head -20
