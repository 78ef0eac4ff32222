#!/bin/bash
# kernel-time sweep of one CTWS_* knob on a bench config (single stream, rocprofv3 kernel trace)
#   VAR=CTWS_WORDS_PER_WAVE VALUES="1 8 32" CONFIG=3 KERNELS="k_localmax|k_output" bash scripts/gpu_sweep_env.sh
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in $VALUES; do
  export $VAR=$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sweep_$v -o run --output-format csv -- \
    python3 -u bench.py --config ${CONFIG:-3} --streams 1 --steps 1 --warmup 1 --no-cpu-baseline --no-host \
    > gpurun_out/sweep_$v.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "$VAR=$v rc=$rc"; tail -3 gpurun_out/sweep_$v.log; exit $rc; }
  python3 scripts/prof_table.py 3 gpurun_out/sweep_$v > gpurun_out/sweep_$v.table 2>&1
  echo "== $VAR=$v: $(grep -o '"value": [0-9.]*' gpurun_out/sweep_$v.log | head -1)"
  grep -E "${KERNELS:-.}" gpurun_out/sweep_$v.table
done
exit 0
