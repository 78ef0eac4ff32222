#!/bin/bash
# round-2 GPU session: smoke, parity tests, bench (default config), single-stream profiles
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
[ $rc -ne 0 ] && exit $rc
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [ "${SKIP_BENCH:-0}" != "1" ]; then
timeout -k 10 600 python3 -u bench.py --steps 3 --warmup 1 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench.log
[ $rc -ne 0 ] && exit $rc
fi
if [ -n "${PROF_CONFIGS:-}" ]; then
  CONFIGS="$PROF_CONFIGS" STEPS=1 bash scripts/gpu_prof_cfg.sh
fi
exit 0
