#!/bin/bash
# Round 5: LDS iteration-0 frontier -- parity suites (flood variants incl. the LDS knobs,
# threshcc), then single-stream stage times of configs 3 / 4 and per-iteration frontier traces.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r05b
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_frontier_variants.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05b/pytest.log 2>&1
rc=$?; tail -4 gpurun_out/r05b/pytest.log; [ $rc -ne 0 ] && exit $rc
for c in ${CONFIGS:-3 4}; do
  for v in ${VARIANTS:-CTWS_FRONTIER_LDS=4 CTWS_FRONTIER_LDS=0}; do
    tag=$(echo "$v" | tr '=, ' '___')
    env CTWS_TRACE=1 $v timeout -k 10 200 python -u bench.py --config $c --streams 1 --steps 1 --warmup 1 --no-host --no-cpu-baseline --no-e2e --no-strong --no-threshcc > gpurun_out/r05b/c${c}_$tag.json 2> gpurun_out/r05b/c${c}_$tag.err || { tail -5 gpurun_out/r05b/c${c}_$tag.err; exit 1; }
    echo "== c$c $v"; grep "frontier it" gpurun_out/r05b/c${c}_$tag.err | tail -12 | head -6
    python3 -c "import json; d=json.loads(open('gpurun_out/r05b/c${c}_$tag.json').read().strip().splitlines()[-1]); s=d['stage_ms_1stream']; print('ms', d['ms_per_step'], {k: v for k, v in s.items() if k.startswith('flood') or k in ('descent_tile', 'size_filter')})"
  done
done
