#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r06c
export TMPDIR=/tmp
run() {  # name, timeout, pytest args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python -u -m pytest "$@" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06c/$n.log 2>&1
  local rc=$?; echo "$n rc=$rc: $(tail -1 gpurun_out/r06c/$n.log)"; return $rc
}
run workflow 600 tests/test_workflow_gpu.py -k "retry" &&
run threshcc 400 tests/test_threshcc_gpu.py -k workflow &&
run golden 400 tests/test_golden_gpu.py tests/test_gpu_pass2.py tests/test_config_blocks.py
