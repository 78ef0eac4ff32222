#!/bin/bash
# Per-iteration frontier times (CTWS_TRACE=1) of config $C (default 3), one step, single stream,
# for the env settings given as arguments (e.g. CTWS_FRONTIER_LDS=0).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ftrace
c=${C:-3}
for v in "$@"; do
  tag=$(echo "$v" | tr '=, ' '___')
  env CTWS_TRACE=1 ${v//,/ } timeout -k 10 200 python -u bench.py --config $c --streams 1 --steps 1 --warmup 0 --no-host --no-cpu-baseline --no-e2e --no-strong > gpurun_out/ftrace/c${c}_$tag.json 2> gpurun_out/ftrace/c${c}_$tag.err || { tail -5 gpurun_out/ftrace/c${c}_$tag.err; exit 1; }
  echo "== $v"; grep "frontier it" gpurun_out/ftrace/c${c}_$tag.err | head -14
  python3 -c "import json; d=json.loads(open('gpurun_out/ftrace/c${c}_$tag.json').read().strip().splitlines()[-1]); s=d['stage_ms_1stream']; print('relax', s['flood_relax'], 'size_filter', s['size_filter'])"
done
