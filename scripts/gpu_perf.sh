#!/bin/bash
# Performance pass: single-stream rocprofv3 kernel trace + stage table per config, then the
# default bench line.  Every GPU step under its own time limit, chained with && (a failing step
# ends the call).  Usage: scripts/gpu_perf.sh <tag> [configs...]   (default configs: 3 4 5)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-perf}; shift
cfgs=${*:-3 4 5}
for c in $cfgs; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_c$c -o run --output-format csv -- \
      python3 -u bench.py --config $c --streams 1 --steps 2 --warmup 1 --no-host --no-cpu-baseline --no-e2e \
      > gpurun_out/prof_${tag}_c$c.json 2> gpurun_out/prof_${tag}_c$c.err || { echo "prof c$c failed"; tail -5 gpurun_out/prof_${tag}_c$c.err; exit 1; }
  echo "c$c: $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/prof_${tag}_c$c.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], {k: d['stage_ms_1stream'].get(k) for k in ('descent_tile','flood_descent','flood_relax','flood_verify','size_filter','crop_cc','output')})")"
done
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 400 python3 -u bench.py --steps 5 --warmup 2 > gpurun_out/bench_${tag}.json 2> gpurun_out/bench_${tag}.err || { echo "bench failed"; tail -5 gpurun_out/bench_${tag}.err; exit 1; }
  tail -c 600 gpurun_out/bench_${tag}.json
fi
