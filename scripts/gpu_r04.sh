#!/bin/bash
# Round-4 GPU session: smoke, the flood/pass-2/sharded parity subset, the default bench line
# (with strong config 4), a 2-rank self-launched bench on one GPU (gloo group, z-halo exchange
# across processes), and a frontier trace of config 3.  Each GPU step under its own time limit;
# the first failure ends the call.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $1"; }
step smoke
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
if [ "${TESTS:-subset}" != "none" ]; then
  step tests
  T="tests/test_gpu_parity.py tests/test_frontier_variants.py tests/test_gpu_pass2.py tests/test_sharded_gpu.py tests/test_config_blocks.py"
  [ "${TESTS}" = "all" ] && T=tests
  timeout -k 10 900 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
fi
if [ "${BENCH:-1}" = "1" ]; then
  step bench
  timeout -k 10 420 python -u bench.py --steps 10 --warmup 3 ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['strong_config4'] and d['strong_config4']['value'], {k: d['stage_ms_1stream'].get(k) for k in ('descent_tile','flood_descent','flood_relax','flood_verify','size_filter','crop_cc','output')})"
fi
if [ "${MULTI:-1}" = "1" ]; then
  step "2-rank bench (one GPU, gloo)"
  timeout -k 10 420 python -u bench.py --gpus 2 --config 5 --streams 1 --steps 2 --warmup 1 --no-strong > gpurun_out/bench_2rank_c5.json 2> gpurun_out/bench_2rank_c5.err || { tail -20 gpurun_out/bench_2rank_c5.err; exit 1; }
  tail -c 700 gpurun_out/bench_2rank_c5.json
fi
if [ "${TRACE:-1}" = "1" ]; then
  step "frontier trace c3"
  CTWS_TRACE=1 timeout -k 10 300 python -u bench.py --streams 1 --steps 1 --warmup 1 --no-host --no-cpu-baseline --no-e2e --no-strong > gpurun_out/trace_c3.json 2> gpurun_out/trace_c3.err || { tail -20 gpurun_out/trace_c3.err; exit 1; }
  grep -c "frontier it" gpurun_out/trace_c3.err || true
fi
step done
