#!/bin/bash
# Round-4 validation + headline: the whole GPU test suite, the default bench line (with
# strong_config4 and end_to_end), the full-volume e2e timeline, a 2-rank self-launched bench.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "[$(date +%T)] smoke"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r04.log 2>&1 || { tail -20 gpurun_out/smoke_r04.log; exit 1; }
tail -1 gpurun_out/smoke_r04.log
echo "[$(date +%T)] GPU test suite"
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r04f.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r04f.log; [ $rc -ne 0 ] && exit $rc
echo "[$(date +%T)] bench"
timeout -k 10 420 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_r04f.json 2> gpurun_out/bench_r04f.err || { tail -20 gpurun_out/bench_r04f.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_r04f.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['pipeline_roofline']['frac'], d['strong_config4']['value'], d['end_to_end']['value'], d['host_resident']['value'], d['vi_vs_oracle']['bit_exact'])"
echo "[$(date +%T)] e2e probe, full config 3"
timeout -k 10 300 python -u scripts/e2e_probe.py 256 4 1 > gpurun_out/e2e_probe_c3_r04f.txt 2>&1 || { tail -20 gpurun_out/e2e_probe_c3_r04f.txt; exit 1; }
grep "workflow rc" gpurun_out/e2e_probe_c3_r04f.txt
echo "[$(date +%T)] 2-rank bench (one GPU, gloo), config 5"
timeout -k 10 300 python -u bench.py --gpus 2 --config 5 --streams 1 --steps 2 --warmup 1 --no-strong > gpurun_out/bench_2rank_c5_r04f.json 2> gpurun_out/bench_2rank_c5_r04f.err || { tail -20 gpurun_out/bench_2rank_c5_r04f.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_2rank_c5_r04f.json').read().strip().splitlines()[-1]); print(d['value'], d['n_gpus'], d['ms_per_step_ranks'], d['config']['dist_backend'], d['config']['pass2_order'])"
echo "[$(date +%T)] done"
