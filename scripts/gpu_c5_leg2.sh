#!/bin/bash
# Which leg slows the bench line's config-5 leg: the CPU baseline or the host path?
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/c5_leg2
mkdir -p $O
export TMPDIR=/tmp
for v in "--no-cpu-baseline" "--no-host" "--no-host --no-cpu-baseline"; do
  tag=$(echo $v | tr -d ' -')
  timeout -k 10 500 python -u bench.py $v --no-e2e --no-strong --no-threshcc > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], 'c5', d['config5']['ms_per_step'])"
done
