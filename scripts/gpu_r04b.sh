#!/bin/bash
# Flood schedule experiments: tile-flood round before the frontier (parity + A/B), frontier
# grid sizes, tile flood only; configs 3 and 4 single stream.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "[$(date +%T)] parity with CTWS_TILE_FIRST=1"
CTWS_TILE_FIRST=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_config_blocks.py tests/test_gpu_pass2.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_tilefirst.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_tilefirst.log; [ $rc -ne 0 ] && exit $rc
export BENCH_ARGS="--streams 1 --no-e2e --no-strong" STEPS=2
echo "[$(date +%T)] config 3 A/B"
CONFIG=3 SETTINGS="CTWS_X=0;CTWS_TILE_FIRST=1;CTWS_FRONTIER_GRID=1024;CTWS_FRONTIER_GRID=512;CTWS_FRONTIER_ITERS=0;CTWS_TILE_FIRST=1 CTWS_FRONTIER_GRID=1024;CTWS_VERIFY=0" bash scripts/gpu_ab.sh || exit 1
echo "[$(date +%T)] config 4 A/B"
CONFIG=4 SETTINGS="CTWS_X=0;CTWS_TILE_FIRST=1;CTWS_FRONTIER_GRID=1024;CTWS_FRONTIER_ITERS=0" bash scripts/gpu_ab.sh || exit 1
echo "[$(date +%T)] trace c3 tile-first"
CTWS_TILE_FIRST=1 CTWS_TRACE=1 timeout -k 10 300 python -u bench.py --streams 1 --steps 1 --warmup 0 --no-host --no-cpu-baseline --no-e2e --no-strong > gpurun_out/trace_tf_c3.json 2> gpurun_out/trace_tf_c3.err || exit 1
grep "frontier it\|tile round" gpurun_out/trace_tf_c3.err | head -30
echo "[$(date +%T)] done"
