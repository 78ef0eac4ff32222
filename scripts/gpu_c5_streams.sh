#!/bin/bash
# Config 5 (two-pass) timed steps over the stream count.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/c5_streams
mkdir -p $O
export TMPDIR=/tmp
for s in ${STREAMS:-1 2 3 1}; do
  timeout -k 10 300 python -u bench.py --config 5 --streams $s --steps 3 --warmup 1 --no-host --no-cpu-baseline --no-e2e --no-strong --no-threshcc > $O/s$s.json 2> $O/s$s.err || { tail -5 $O/s$s.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/s$s.json').read().strip().splitlines()[-1]); print('c5 streams $s', d['value'], d['ms_per_step'])"
done
