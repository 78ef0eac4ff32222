#!/bin/bash
# Round 5: workgroup-per-chunk frontier (CTWS_FRONTIER_WPC=4) -- parity of the variants, then
# single-stream flood stage times of configs 3 / 4 per variant.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_frontier_variants.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for c in ${CONFIGS:-3 4}; do
  for v in ${VARIANTS:-CTWS_FRONTIER_WPC=1 CTWS_FRONTIER_WPC=4,CTWS_FRONTIER_GRID_WPC=1024 CTWS_FRONTIER_WPC=4,CTWS_FRONTIER_GRID_WPC=2048 CTWS_FRONTIER_WPC=4,CTWS_FRONTIER_GRID_WPC=4096}; do
    tag=$(echo "$v" | tr '=, ' '___')
    ( export $(echo $v | tr ',' ' '); timeout -k 10 200 python -u bench.py --config $c --streams 1 --steps 2 --warmup 1 --no-host --no-cpu-baseline --no-e2e --no-strong --no-threshcc --no-config5 > $O/c${c}_$tag.json 2> $O/c${c}_$tag.err ) || { tail -5 $O/c${c}_$tag.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c${c}_$tag.json').read().strip().splitlines()[-1]); s=d['stage_ms_1stream']; print('c$c $v', d['ms_per_step'], {k: v for k, v in s.items() if k.startswith('flood') or k in ('descent_tile', 'size_filter')})"
  done
done
