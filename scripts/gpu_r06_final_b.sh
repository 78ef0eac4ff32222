#!/bin/bash
# Round 6 final (2/2): single-stream rocprofv3 kernel traces of configs 3 / 4 / 5 (stage table +
# trace roofline), then FETCH_SIZE / WRITE_SIZE passes of configs 3 / 4 (HBM bytes per stage).
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${FINAL_DIR:-r06_final}
mkdir -p $O
export TMPDIR=/tmp
for c in ${TRACE_CONFIGS:-3 4 5}; do
  echo "[$(date +%T)] trace c$c"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c$c -o run --output-format csv -- \
      python3 -u bench.py --config $c --streams 1 --steps 2 --warmup 1 --no-host --no-cpu-baseline --no-e2e --no-strong --no-threshcc --no-config5 \
      > $O/prof_c$c.json 2> $O/prof_c$c.err || { echo "prof c$c failed"; tail -5 $O/prof_c$c.err; exit 1; }
  tr=$(find $O/prof_c$c -name 'run_kernel_trace.csv' | head -1); st=$(find $O/prof_c$c -name 'run_kernel_stats.csv' | head -1)
  cp "$st" $O/kernel_stats_c${c}_1stream.csv
  gzip -c "$tr" > $O/kernel_trace_c${c}_1stream.csv.gz
  python3 scripts/roofline_from_trace.py "$tr" $O/prof_c$c.json 3 > $O/roofline_recompute_c$c.json
  python3 -c "import json; d=json.load(open('$O/roofline_recompute_c$c.json')); print('c$c', d['flood_kernel_ms_per_step'], d['frac'], d['agreement'])"
  rm -rf $O/prof_c$c
done
for c in ${PMC_CONFIGS:-3 4}; do
  mkdir -p $O/pmc_c$c
  for grp in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $grp --kernel-include-regex ctws --output-format csv -d $O/pmc_c$c/$grp -o p -- python3 -u bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline --no-host --no-e2e --no-strong --no-threshcc --no-config5 --streams 1 > $O/pmc_c$c/$grp.log 2>&1 || { echo "pmc c$c $grp failed"; tail -5 $O/pmc_c$c/$grp.log; exit 1; }
  done
  python3 scripts/pmc_traffic.py $O/pmc_c$c > $O/pmc_traffic_c$c.json
  python3 -c "import json; d=json.load(open('$O/pmc_traffic_c$c.json')); print('c$c', {k: round(v/1e9,2) for k, v in d.items() if isinstance(v, float)})"
  rm -rf $O/pmc_c$c
done
echo "[$(date +%T)] done"
