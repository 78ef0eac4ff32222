#!/bin/bash
# Round 6 final (3/3): rocprofv3 kernel stats of the default bench command (without the
# end-to-end leg) and the SQ issue / stall counters of one single-stream config-3 step.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${FINAL_DIR:-r06_final}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $O/prof_default -o run --output-format csv -- python3 -u bench.py --no-e2e > $O/bench_prof.json 2> $O/bench_prof.err || { tail -5 $O/bench_prof.err; exit 1; }
cp $(find $O/prof_default -name 'run_kernel_stats.csv' | head -1) $O/kernel_stats_default_bench.csv
rm -rf $O/prof_default
tail -1 $O/bench_prof.json | cut -c1-300
mkdir -p $O/pmc_sq
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE \
  --kernel-include-regex ctws --output-format csv -d $O/pmc_sq/SQ -o p -- \
  python3 -u bench.py --config 3 --steps 1 --warmup 0 --no-cpu-baseline --no-host --no-e2e --no-strong --no-threshcc --no-config5 --streams 1 > $O/pmc_sq/SQ.log 2>&1
rc=$?; echo "pmc SQ rc=$rc"
[ $rc -ne 0 ] && exit $rc
python3 scripts/pmc_sq.py $O/pmc_sq/SQ > $O/pmc_sq_c3.txt && head -16 $O/pmc_sq_c3.txt
rm -rf $O/pmc_sq
