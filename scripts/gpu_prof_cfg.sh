#!/bin/bash
# single-stream kernel trace of one bench config: summaries into gpurun_out/prof_c<N>
#   CONFIGS="3 4" STEPS=2 bash scripts/gpu_prof_cfg.sh
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in ${CONFIGS:-3}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c$c -o run --output-format csv -- \
    python3 -u bench.py --config $c --streams 1 --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline --no-host ${BENCH_ARGS:-} \
    > gpurun_out/prof_c$c.log 2>&1
  rc=$?; echo "config $c rc=$rc"; tail -1 gpurun_out/prof_c$c.log | cut -c1-400
  [ $rc -ne 0 ] && exit $rc
  python3 scripts/prof_table.py $((${STEPS:-2} + 1)) gpurun_out/prof_c$c > gpurun_out/prof_c$c.table 2>&1 || true
done
exit 0
