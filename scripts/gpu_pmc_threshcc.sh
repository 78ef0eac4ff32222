#!/bin/bash
# HBM traffic of the BlockComponents kernels: FETCH_SIZE and WRITE_SIZE in separate runs.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_tc
for grp in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex k_tc_ --output-format csv -d gpurun_out/pmc_tc/$grp -o p -- python -u scripts/bench_threshcc.py --no-cpu --only blobs_128x512 --reps 3 > gpurun_out/pmc_tc/$grp.log 2>&1
  rc=$?; echo "pmc $grp rc=$rc"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc_tc/$grp.log; exit $rc; }
done
python scripts/pmc_threshcc.py gpurun_out/pmc_tc > gpurun_out/pmc_tc/traffic.json && cat gpurun_out/pmc_tc/traffic.json
