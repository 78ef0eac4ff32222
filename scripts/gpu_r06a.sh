#!/bin/bash
# Round 6: the new GPU tests (corridor / wide keys, big blocks, retry, 2-rank two-pass, spill),
# then the whole GPU suite's core files.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r06a
export TMPDIR=/tmp
run() {  # name, timeout, pytest args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python -u -m pytest "$@" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06a/$n.log 2>&1
  local rc=$?; echo "$n rc=$rc: $(tail -1 gpurun_out/r06a/$n.log)"; return $rc
}
run corridor 300 tests/test_corridor_gpu.py -v &&
run parity 400 tests/test_gpu_parity.py tests/test_from_seeds_gpu.py &&
run variants 500 tests/test_frontier_variants.py &&
run ranks 300 tests/test_bench_two_pass_ranks.py &&
run workflow 600 tests/test_workflow_gpu.py -k "retry or roi" &&
run threshcc 400 tests/test_threshcc_gpu.py -k workflow
