#!/bin/bash
# Round 6: the remaining new GPU tests (2-rank two-pass, retry workflow, spill merge).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r06b
export TMPDIR=/tmp
run() {  # name, timeout, pytest args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python -u -m pytest "$@" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06b/$n.log 2>&1
  local rc=$?; echo "$n rc=$rc: $(tail -1 gpurun_out/r06b/$n.log)"; return $rc
}
run ranks 300 tests/test_bench_two_pass_ranks.py &&
run workflow 600 tests/test_workflow_gpu.py -k "retry or roi" &&
run threshcc 400 tests/test_threshcc_gpu.py -k workflow
