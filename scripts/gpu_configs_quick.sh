#!/bin/bash
# the other bench configurations on one GPU (no CPU baseline), current defaults
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/cfg
export TMPDIR=/tmp
for c in 3 4 5; do
  timeout -k 10 240 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/cfg/c$c.log 2>&1
  rc=$?; echo "config $c rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/cfg/c$c.log)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
