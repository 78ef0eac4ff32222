#!/bin/bash
# In-job relabel (process-group offset scan) in the product path: workflow parity, e2e timelines
# of the full config-3 volume (both relabel modes), the default bench line.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "[$(date +%T)] tests"
timeout -k 10 900 python -u -m pytest tests/test_workflow_gpu.py tests/test_config1_testcfgs.py tests/test_frontier_variants.py tests/test_relabel_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r04d.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r04d.log; [ $rc -ne 0 ] && exit $rc
echo "[$(date +%T)] e2e probe, full config 3, relabel in job"
timeout -k 10 600 python -u scripts/e2e_probe.py 256 4 1 > gpurun_out/e2e_probe_c3_injob.txt 2>&1 || { tail -20 gpurun_out/e2e_probe_c3_injob.txt; exit 1; }
grep -v "^      " gpurun_out/e2e_probe_c3_injob.txt | tail -12
echo "[$(date +%T)] e2e probe, full config 3, three-task relabel"
timeout -k 10 600 python -u scripts/e2e_probe.py 256 4 0 > gpurun_out/e2e_probe_c3_tasks.txt 2>&1 || { tail -20 gpurun_out/e2e_probe_c3_tasks.txt; exit 1; }
grep -v "^      " gpurun_out/e2e_probe_c3_tasks.txt | tail -22
echo "[$(date +%T)] bench"
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_r04d.json 2> gpurun_out/bench_r04d.err || { tail -20 gpurun_out/bench_r04d.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_r04d.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['strong_config4']['value'], d['end_to_end'])"
echo "[$(date +%T)] done"
