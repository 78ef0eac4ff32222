#!/bin/bash
# Round-4 end-to-end I/O: libdeflate codec + HBM-resident in-job relabel.  Workflow GPU tests,
# the full-volume e2e timeline, the job teardown probe, the default bench line.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "[$(date +%T)] workflow tests"
timeout -k 10 400 python -u -m pytest tests/test_workflow_gpu.py tests/test_relabel_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r04h.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r04h.log; [ $rc -ne 0 ] && exit $rc
echo "[$(date +%T)] e2e probe, full config 3"
timeout -k 10 300 python -u scripts/e2e_probe.py 256 4 1 > gpurun_out/e2e_probe_c3_r04h.txt 2>&1 || { tail -20 gpurun_out/e2e_probe_c3_r04h.txt; exit 1; }
head -12 gpurun_out/e2e_probe_c3_r04h.txt | grep -v "start processing block"
echo "[$(date +%T)] teardown probe"
timeout -k 10 120 python -u scripts/teardown_probe.py > gpurun_out/teardown_r04h.txt 2>&1 || { tail -20 gpurun_out/teardown_r04h.txt; exit 1; }
cat gpurun_out/teardown_r04h.txt
echo "[$(date +%T)] bench"
timeout -k 10 420 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_r04h.json 2> gpurun_out/bench_r04h.err || { tail -20 gpurun_out/bench_r04h.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_r04h.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['end_to_end'], d['host_resident']['value'])"
echo "[$(date +%T)] done"
