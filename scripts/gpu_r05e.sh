#!/bin/bash
# Round 5: threshcc end-to-end timeline (job logs), then the descent change's parity and stage times.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/e2e_threshcc.py --merge-in-job 1 --keep-logs $O/tc_logs > $O/e2e_tc_1.json 2> $O/e2e_tc_1.err || { tail -5 $O/e2e_tc_1.err; exit 1; }
cat $O/e2e_tc_1.json
EXTRA_TESTS="tests/test_frontier_variants.py" CONFIGS="3 4" bash scripts/gpu_quick.sh
