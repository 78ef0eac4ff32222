#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/st3
export TMPDIR=/tmp
for cfg in "3 4" "2 4" "4 4" "3 2" "1 2"; do set -- $cfg
  CTWS_FRONTIER_REPS=$2 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --streams $1 > gpurun_out/st3/s$1r$2.log 2>&1
  rc=$?; echo "streams $1 reps $2 rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/st3/s$1r$2.log)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
