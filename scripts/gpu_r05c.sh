#!/bin/bash
# Round 5: pass-2 word tiles + crop shortcut A/B -- parity tests, then kernel stats of one
# single-stream step of config 3 (crop shortcut on / off) and config 5.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05c
mkdir -p $O
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pass2.py tests/test_config_blocks.py tests/test_frontier_variants.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
run() {  # tag config env...
  tag=$1; c=$2; shift 2
  ( export "$@"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$tag -o run --output-format csv -- python3 bench.py --config $c --streams 1 --steps 1 --warmup 1 --no-host --no-cpu-baseline --no-e2e --no-strong --no-threshcc --no-config5 > $O/$tag.json 2> $O/$tag.err ) || { tail -5 $O/$tag.err; exit 1; }
  echo "== $tag"; python3 scripts/prof_table.py 3 $O/prof_$tag > $O/table_$tag.txt; sed -n 1,26p $O/table_$tag.txt
  cp $(find $O/prof_$tag -name '*kernel_stats.csv') $O/stats_$tag.csv
  gzip -c $(find $O/prof_$tag -name '*kernel_trace.csv') > $O/trace_$tag.csv.gz
  rm -rf $O/prof_$tag
}
run c3_short 3 CTWS_CROP_SHORT=1
run c3_noshort 3 CTWS_CROP_SHORT=0
[ -n "$NO_C5" ] || run c5 5 CTWS_CROP_SHORT=1
[ -z "$C4" ] || run c4_short 4 CTWS_CROP_SHORT=1
[ -z "$C4" ] || run c4_noshort 4 CTWS_CROP_SHORT=0
