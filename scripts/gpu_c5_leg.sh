#!/bin/bash
# The bench line's config-5 leg (after the config-3 workload in the same process) against config 5
# run alone, same box.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/c5_leg
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --config 3 --steps 2 --warmup 1 --no-host --no-cpu-baseline --no-e2e --no-strong --no-threshcc > $O/leg.json 2> $O/leg.err || { tail -5 $O/leg.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/leg.json').read().strip().splitlines()[-1]); print('c3', d['value'], d['ms_per_step'], 'c5 leg', d['config5']['value'], d['config5']['ms_per_step'])"
timeout -k 10 300 python -u bench.py --config 5 --streams 3 --steps 2 --warmup 1 --no-host --no-cpu-baseline --no-e2e --no-strong --no-threshcc > $O/alone.json 2> $O/alone.err || { tail -5 $O/alone.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/alone.json').read().strip().splitlines()[-1]); print('c5 alone', d['value'], d['ms_per_step'])"
timeout -k 10 300 python -u bench.py --config 5 --streams 3 --steps 4 --warmup 2 --no-host --no-cpu-baseline --no-e2e --no-strong --no-threshcc > $O/alone4.json 2> $O/alone4.err || { tail -5 $O/alone4.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/alone4.json').read().strip().splitlines()[-1]); print('c5 alone 4 steps', d['value'], d['ms_per_step'])"
