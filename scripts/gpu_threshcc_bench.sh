#!/bin/bash
# BlockComponents throughput (scripts/bench_threshcc.py) and its rocprofv3 kernel statistics.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/tcbench
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/bench_threshcc.py > gpurun_out/tcbench/bench.jsonl 2> gpurun_out/tcbench/bench.err
rc=$?; cat gpurun_out/tcbench/bench.jsonl; [ $rc -ne 0 ] && { tail -5 gpurun_out/tcbench/bench.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tcbench/prof -o tc -- python3 scripts/bench_threshcc.py --no-cpu --reps 10 > gpurun_out/tcbench/prof.log 2>&1
rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/tcbench/prof.log; exit $rc; }
find gpurun_out/tcbench/prof -name '*kernel_stats.csv' | head -3
