#!/bin/bash
# Round 6: the seed-stage repeatability test (8 runs x 3 blocks per case) and the stage parity.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06t
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "repeatable or stages_bit_exact or deterministic" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; exit $rc
