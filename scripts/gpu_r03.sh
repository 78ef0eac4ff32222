#!/bin/bash
# Round-3 GPU steps: each GPU step under its own time limit, chained with && (a failing step
# ends the call).  Usage: scripts/gpu_r03.sh <mode> [args]
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
mode=$1; shift
case "$mode" in
  tests)  # GPU test files (all when none given)
    timeout -k 10 1100 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu "$@" \
        > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; exit $rc ;;
  bench)  # bench.py args
    timeout -k 10 600 python -u bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
    tail -3 gpurun_out/bench.err; cat gpurun_out/bench.json; exit $rc ;;
  tests_bench)
    timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu "$@" \
        > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log
    [ $rc -eq 0 ] || exit $rc
    timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
    tail -3 gpurun_out/bench.err; cat gpurun_out/bench.json; exit $rc ;;
  prof)  # single-stream kernel trace of a config: prof <tag> <bench args>
    tag=$1; shift
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run -- \
        python3 bench.py --streams 1 --no-host --no-cpu-baseline "$@" > gpurun_out/prof_$tag.json 2> gpurun_out/prof_$tag.err
    rc=$?; tail -3 gpurun_out/prof_$tag.err; cat gpurun_out/prof_$tag.json; exit $rc ;;
  *) echo "unknown mode $mode"; exit 2 ;;
esac
