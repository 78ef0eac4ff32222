#!/bin/bash
# e2e after the job-relabel I/O changes (chunk cache, consecutive blocks, pooled writes), and
# the PMC passes (calibration microkernel + per-stage traffic of configs 3 and 4).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "[$(date +%T)] GPU test suite"
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r04e.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r04e.log; [ $rc -ne 0 ] && exit $rc
echo "[$(date +%T)] e2e probe, full config 3"
timeout -k 10 400 python -u scripts/e2e_probe.py 256 4 1 > gpurun_out/e2e_probe_c3_injob2.txt 2>&1 || { tail -20 gpurun_out/e2e_probe_c3_injob2.txt; exit 1; }
grep -v "^      " gpurun_out/e2e_probe_c3_injob2.txt | tail -6; grep "^      " gpurun_out/e2e_probe_c3_injob2.txt | sed -n '1,4p;18,22p;34,40p'
echo "[$(date +%T)] single-stream config 3"
CONFIG=3 STEPS=2 BENCH_ARGS="--streams 1 --no-e2e --no-strong" SETTINGS="CTWS_X=0" bash scripts/gpu_ab.sh || exit 1
echo "[$(date +%T)] PMC"
bash scripts/gpu_pmc_r04.sh || exit 1
echo "[$(date +%T)] done"
