#!/bin/bash
# LDS-resident iteration 0 of the frontier (k_frontier_lds): parity, A/B, trace.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "[$(date +%T)] parity"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_config_blocks.py tests/test_frontier_variants.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_lds.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_lds.log; [ $rc -ne 0 ] && exit $rc
export BENCH_ARGS="--streams 1 --no-e2e --no-strong" STEPS=2
echo "[$(date +%T)] config 3 A/B"
CONFIG=3 SETTINGS="CTWS_FRONTIER_LDS=0;CTWS_FRONTIER_LDS=1;CTWS_FRONTIER_LDS_GRID=512;CTWS_FRONTIER_LDS_GRID=1536;CTWS_FRONTIER_LDS_REPS=32;CTWS_FRONTIER_LDS=2;CTWS_FRONTIER_GRID=1024" bash scripts/gpu_ab.sh || exit 1
echo "[$(date +%T)] trace c3"
CTWS_TRACE=1 timeout -k 10 300 python -u bench.py --streams 1 --steps 1 --warmup 0 --no-host --no-cpu-baseline --no-e2e --no-strong > gpurun_out/trace_lds_c3.json 2> gpurun_out/trace_lds_c3.err || exit 1
grep "frontier it" gpurun_out/trace_lds_c3.err | head -12
echo "[$(date +%T)] done"
