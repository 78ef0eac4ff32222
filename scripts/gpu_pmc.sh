#!/bin/bash
# PMC passes on the bench (one counter group per run, as the microarch guide prescribes)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc -o pass$i -- python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc/pass$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"; python scripts/pmc_summary.py gpurun_out/pmc > /dev/null; mv gpurun_out/pmc/pmc_summary.json gpurun_out/pmc/summary_pass$i.json
  [ $rc -ne 0 ] && exit $rc
done
exit 0
