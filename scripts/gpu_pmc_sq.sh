#!/bin/bash
# Issue/stall PMC pass (SQ + GRBM counters, one run, single stream): per kernel, the share of
# wave time spent issuing VALU / any instruction and parked on memory or barriers.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE \
  --kernel-include-regex ctws --output-format csv -d gpurun_out/pmc/SQ -o p -- \
  python -u bench.py --config ${CONFIG:-3} --steps 1 --warmup 0 --no-cpu-baseline --no-host --no-e2e --streams 1 > gpurun_out/pmc/SQ.log 2>&1
rc=$?; echo "pmc SQ rc=$rc"
[ $rc -ne 0 ] && exit $rc
python scripts/pmc_sq.py gpurun_out/pmc/SQ > gpurun_out/pmc/sq_c${CONFIG:-3}.txt && head -40 gpurun_out/pmc/sq_c${CONFIG:-3}.txt
