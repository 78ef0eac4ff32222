#!/bin/bash
# Quick check after a kernel change: the parity / golden / from-seeds GPU tests, then the
# single-stream stage times of configs 3 and 4 (CONFIGS to override).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/quick
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden_gpu.py tests/test_from_seeds_gpu.py tests/test_gpu_pass2.py ${EXTRA_TESTS:-} -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/quick/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/quick/pytest.log; [ $rc -ne 0 ] && exit $rc
for c in ${CONFIGS:-3 4}; do
  timeout -k 10 200 python -u bench.py --config $c --streams 1 --steps 3 --warmup 1 --no-host --no-cpu-baseline --no-e2e --no-strong > gpurun_out/quick/c$c.json 2> gpurun_out/quick/c$c.err || { tail -5 gpurun_out/quick/c$c.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/quick/c$c.json').read().strip().splitlines()[-1]); s=d['stage_ms_1stream']; print('c$c', d['ms_per_step'], {k: v for k, v in s.items() if v >= 0.5 and k not in ('frontier_iters', 'regrow_iters', 'flood_packed')})"
done
