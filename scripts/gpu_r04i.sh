#!/bin/bash
# Round-4: kernel traces of configs 3 and 4 (stage table), then the e2e probe with batched reads.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TRACE_CONFIGS="3 4" bash scripts/gpu_r04g_traces.sh || exit 1
echo "[$(date +%T)] workflow tests"
timeout -k 10 400 python -u -m pytest tests/test_workflow_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r04i.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r04i.log; [ $rc -ne 0 ] && exit $rc
echo "[$(date +%T)] e2e probe, full config 3"
timeout -k 10 300 python -u scripts/e2e_probe.py 256 4 1 > gpurun_out/e2e_probe_c3_r04i.txt 2>&1 || { tail -20 gpurun_out/e2e_probe_c3_r04i.txt; exit 1; }
grep -v "processing block\|processed block [1-9]" gpurun_out/e2e_probe_c3_r04i.txt | head -12
grep "start processing block" gpurun_out/e2e_probe_c3_r04i.txt | head -16 | awk '{print $1}' | tr '\n' ' '; echo
for ns in 2 4 6; do
  timeout -k 10 200 python -u bench.py --config 3 --streams $ns --steps 5 --warmup 2 --no-host --no-cpu-baseline --no-e2e --no-strong > gpurun_out/bench_c3_s$ns.json 2> gpurun_out/bench_c3_s$ns.err || { tail -5 gpurun_out/bench_c3_s$ns.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_c3_s$ns.json').read().strip().splitlines()[-1]); print('streams $ns', d['value'], d['ms_per_step'])"
done
echo "[$(date +%T)] done"
