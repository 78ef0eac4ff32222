#!/bin/bash
# bench lines for the BASELINE configs (one-GPU shares), each under its own limit
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for c in ${CONFIGS:-2 4 5}; do
  timeout -k 10 500 python3 -u bench.py --config $c --steps ${STEPS:-3} --warmup 1 ${BENCH_ARGS:---no-cpu-baseline --no-host} > gpurun_out/bench_c$c.log 2>&1
  rc=$?; echo "config $c rc=$rc"; tail -c 600 gpurun_out/bench_c$c.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
