#!/bin/bash
# bench lines for the BASELINE.json configs (single-GPU shares); each step under its own limit
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for c in ${CONFIGS:-2 3 4 5}; do
  timeout -k 10 400 python -u bench.py --config $c --steps ${STEPS:-3} --warmup 1 ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/bench_c$c.log 2>&1
  rc=$?; echo "config $c rc=$rc"; tail -1 gpurun_out/bench_c$c.log | cut -c1-600
  [ $rc -ne 0 ] && exit $rc
done
exit 0
