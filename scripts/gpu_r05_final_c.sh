#!/bin/bash
# Round 5 final (3/3): SQ issue / stall counters of one single-stream config-3 step (one pass).
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05_final
mkdir -p $O/pmc_sq
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE \
  --kernel-include-regex ctws --output-format csv -d $O/pmc_sq/SQ -o p -- \
  python3 -u bench.py --config ${CONFIG:-3} --steps 1 --warmup 0 --no-cpu-baseline --no-host --no-e2e --no-strong --no-threshcc --no-config5 --streams 1 > $O/pmc_sq/SQ.log 2>&1
rc=$?; echo "pmc SQ rc=$rc"
[ $rc -ne 0 ] && exit $rc
python3 scripts/pmc_sq.py $O/pmc_sq/SQ > $O/pmc_sq_c${CONFIG:-3}.txt && head -24 $O/pmc_sq_c${CONFIG:-3}.txt
rm -rf $O/pmc_sq
