#!/bin/bash
# Round-4 validation after the thresholded components: the whole GPU test suite, smoke, the default bench
# line (end_to_end now on the whole config-3 volume), a 2-rank self-launched bench.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "[$(date +%T)] smoke"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r04l.log 2>&1 || { tail -20 gpurun_out/smoke_r04l.log; exit 1; }
tail -1 gpurun_out/smoke_r04l.log
echo "[$(date +%T)] GPU test suite"
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r04l.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r04l.log; [ $rc -ne 0 ] && exit $rc
echo "[$(date +%T)] bench"
timeout -k 10 500 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_r04l.json 2> gpurun_out/bench_r04l.err || { tail -20 gpurun_out/bench_r04l.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_r04l.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['pipeline_roofline']['frac'], d['strong_config4']['value'], d['end_to_end'], d['host_resident']['value'], d['vi_vs_oracle']['bit_exact'], d['cpu_baseline']['value'])"
echo "[$(date +%T)] 2-rank bench (one GPU, gloo), config 3"
timeout -k 10 300 python -u bench.py --gpus 2 --config 3 --steps 3 --warmup 1 --no-strong > gpurun_out/bench_2rank_c3_r04l.json 2> gpurun_out/bench_2rank_c3_r04l.err || { tail -20 gpurun_out/bench_2rank_c3_r04l.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_2rank_c3_r04l.json').read().strip().splitlines()[-1]); print(d['value'], d['n_gpus'], d['ms_per_step_ranks'], d['config']['dist_backend'])"
echo "[$(date +%T)] done"
