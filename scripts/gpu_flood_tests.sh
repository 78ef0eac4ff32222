#!/bin/bash
# Flood parity on the GPU: smoke, the parity cases, every frontier / basin variant, the config blocks.
cd /root/repo; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo smoke rc=$rc; tail -3 gpurun_out/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_frontier_variants.py tests/test_config_blocks.py > gpurun_out/pytest_basin.log 2>&1; rc=$?; echo pytest rc=$rc; tail -5 gpurun_out/pytest_basin.log; exit $rc
