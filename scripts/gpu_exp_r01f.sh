#!/bin/bash
# stream-count sweep of the bench, then the HBM traffic PMC passes (FETCH_SIZE and WRITE_SIZE in
# separate runs, single stream so the per-kernel counters are not mixed across streams)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/sweep
export TMPDIR=/tmp
for s in 1 3 4; do
  timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --streams $s > gpurun_out/sweep/s$s.log 2>&1
  rc=$?; echo "streams $s rc=$rc"; grep -o '"value": [0-9.]*' gpurun_out/sweep/s$s.log
  [ $rc -ne 0 ] && exit $rc
done
mkdir -p gpurun_out/pmc
for grp in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc/$grp -o p -- python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --streams 1 > gpurun_out/pmc/$grp.log 2>&1
  rc=$?; echo "pmc $grp rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
python scripts/pmc_traffic.py gpurun_out/pmc > gpurun_out/pmc/traffic.json
exit 0
