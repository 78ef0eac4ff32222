#!/bin/bash
# HBM traffic PMC passes (FETCH_SIZE and WRITE_SIZE in separate runs, single stream)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
for grp in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-include-regex ctws --output-format csv -d gpurun_out/pmc/$grp -o p -- python -u bench.py --config ${CONFIG:-3} --steps 1 --warmup 0 --no-cpu-baseline --no-host --streams 1 ${BENCH_ARGS:-} > gpurun_out/pmc/$grp.log 2>&1
  rc=$?; echo "pmc $grp rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
python scripts/pmc_traffic.py gpurun_out/pmc > gpurun_out/pmc/traffic_c${CONFIG:-3}.json
