#!/bin/bash
# Config 3 bench line over batch budgets (CTWS_BATCH_VOXELS) and stream counts.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/batch_sweep
mkdir -p $O
export TMPDIR=/tmp
for spec in ${SPECS:-536870912:3 268435456:3 134217728:3 134217728:6 67108864:6}; do
  b=${spec%%:*}; s=${spec##*:}
  CTWS_BATCH_VOXELS=$b timeout -k 10 200 python -u bench.py --config 3 --streams $s --steps 5 --warmup 2 --no-host --no-cpu-baseline --no-e2e --no-strong --no-threshcc --no-config5 > $O/b${b}_s$s.json 2> $O/b${b}_s$s.err || { tail -5 $O/b${b}_s$s.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b${b}_s$s.json').read().strip().splitlines()[-1]); print('batch $b streams $s', d['value'], d['ms_per_step'])"
done
