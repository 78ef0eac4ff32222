#!/bin/bash
# The whole GPU suite (as the driver runs it), then single-stream stage times of configs 3 / 4.
cd "${GRAFT_REPO_ROOT:-.}"
tag=${TAG:-full}
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$tag/pytest.log 2>&1
rc=$?; tail -4 gpurun_out/$tag/pytest.log; [ $rc -ne 0 ] && exit $rc
for c in ${CONFIGS-3 4}; do
  timeout -k 10 200 python -u bench.py --config $c --streams 1 --steps 3 --warmup 1 --no-host --no-cpu-baseline --no-e2e --no-strong --no-threshcc --no-config5 > gpurun_out/$tag/c$c.json 2> gpurun_out/$tag/c$c.err || { tail -5 gpurun_out/$tag/c$c.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/$tag/c$c.json').read().strip().splitlines()[-1]); s=d['stage_ms_1stream']; print('c$c', d['ms_per_step'], {k: v for k, v in s.items() if v >= 0.5 and k not in ('frontier_iters', 'regrow_iters', 'flood_packed')})"
done
# E2E_TC=1: the ThresholdedComponentsWorkflow end to end, merge tail in the jobs and as tasks
if [ -n "$E2E_TC" ]; then
  for m in 1 0; do
    timeout -k 10 400 python -u scripts/e2e_threshcc.py --merge-in-job $m > gpurun_out/$tag/e2e_tc_$m.json 2> gpurun_out/$tag/e2e_tc_$m.err || { tail -5 gpurun_out/$tag/e2e_tc_$m.err; exit 1; }
    cat gpurun_out/$tag/e2e_tc_$m.json
  done
fi
