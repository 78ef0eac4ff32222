#!/bin/bash
# Round-4 final validation after the thresholded-components tuning: smoke, the whole GPU test
# suite, the default bench line, the BlockComponents throughput table + its kernel trace.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "[$(date +%T)] smoke"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r04m.log 2>&1 || { tail -20 gpurun_out/smoke_r04m.log; exit 1; }
tail -1 gpurun_out/smoke_r04m.log
echo "[$(date +%T)] GPU test suite"
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r04m.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r04m.log; [ $rc -ne 0 ] && exit $rc
echo "[$(date +%T)] bench"
timeout -k 10 500 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_r04m.json 2> gpurun_out/bench_r04m.err || { tail -20 gpurun_out/bench_r04m.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_r04m.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['end_to_end']['value'], d['host_resident']['value'], d['vi_vs_oracle']['bit_exact'], d['cpu_baseline']['value']); print(d['thresholded_components'])"
echo "[$(date +%T)] thresholded components table"
bash scripts/gpu_threshcc_bench.sh
echo "[$(date +%T)] done"
