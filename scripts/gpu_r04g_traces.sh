#!/bin/bash
# Round-4 single-stream rocprofv3 kernel traces (stage table + trace roofline) of TRACE_CONFIGS.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in ${TRACE_CONFIGS:-3 4 5}; do
  echo "[$(date +%T)] trace c$c"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r04_c$c -o run --output-format csv -- \
      python3 -u bench.py --config $c --streams 1 --steps 2 --warmup 1 --no-host --no-cpu-baseline --no-e2e --no-strong \
      > gpurun_out/prof_r04_c$c.json 2> gpurun_out/prof_r04_c$c.err || { echo "prof c$c failed"; tail -5 gpurun_out/prof_r04_c$c.err; exit 1; }
  tr=$(ls gpurun_out/prof_r04_c$c/run_kernel_trace.csv gpurun_out/prof_r04_c$c/*/run_kernel_trace.csv 2>/dev/null | head -1); st=$(ls gpurun_out/prof_r04_c$c/run_kernel_stats.csv gpurun_out/prof_r04_c$c/*/run_kernel_stats.csv 2>/dev/null | head -1)
  [ -n "$tr" ] && cp "$tr" gpurun_out/r04_kernel_trace_c$c.csv; [ -n "$st" ] && cp "$st" gpurun_out/r04_kernel_stats_c$c.csv
  [ -n "$tr" ] && python3 scripts/roofline_from_trace.py gpurun_out/r04_kernel_trace_c$c.csv gpurun_out/prof_r04_c$c.json 3 > gpurun_out/r04_roofline_recompute_c$c.json
  python3 -c "import json; d=json.load(open('gpurun_out/r04_roofline_recompute_c$c.json')); print('c$c', d['flood_kernel_ms_per_step'], d['frac'], d['agreement'], d['stage_ms_per_step'])"
  rm -rf gpurun_out/prof_r04_c$c
done
