#!/bin/bash
# flood diagnostics on one config: per-iteration frontier trace, then one SQ counter pass
#   CONFIG=3 bash scripts/gpu_diag.sh
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/diag
export TMPDIR=/tmp
c=${CONFIG:-3}
CTWS_TRACE=1 timeout -k 10 300 python3 -u bench.py --config $c --steps 1 --warmup 0 --streams 1 --no-cpu-baseline \
  --no-host ${BENCH_ARGS:-} > gpurun_out/diag/trace_c$c.log 2> gpurun_out/diag/trace_c$c.err
rc=$?; echo "trace rc=$rc"; grep -c frontier gpurun_out/diag/trace_c$c.err; [ $rc -ne 0 ] && exit $rc
if [ "${PMC:-1}" = "1" ]; then
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d gpurun_out/diag/pmc -o sq -- \
  python3 -u bench.py --config $c --steps 1 --warmup 0 --streams 1 --no-cpu-baseline --no-host \
  > gpurun_out/diag/pmc_c$c.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 scripts/pmc_summary.py gpurun_out/diag/pmc > /dev/null
fi
exit 0
