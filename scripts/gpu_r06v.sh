#!/bin/bash
# Round 6: the 2-D listed-maxima seed union with device-scope parent loads and no path halving
# (libctws_union.so): the seed repeatability test at 40 runs x 3 blocks per case, then config 3
# A/B against the current build.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06v
mkdir -p $O
export TMPDIR=/tmp
CTWS_TEST_REPS=40 CTWS_LIB=$PWD/cluster_tools_amd/libctws_union.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -k "repeatable" > $O/pytest_union.log 2>&1
echo "union rc=$?"; grep -E "passed|failed|Mismatch|FAILED" $O/pytest_union.log | head -20
for v in cur union cur union; do
  unset CTWS_LIB
  [ $v = union ] && export CTWS_LIB=$PWD/cluster_tools_amd/libctws_union.so
  timeout -k 10 200 python -u bench.py --config 3 --streams 1 --steps 2 --warmup 1 --no-host --no-cpu-baseline --no-e2e --no-strong --no-threshcc --no-config5 > $O/c3_$v.json 2> $O/c3_$v.err || { tail -5 $O/c3_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c3_$v.json').read().strip().splitlines()[-1]); s=d['stage_ms_1stream']; print('c3 $v', d['ms_per_step'], s['seeds'])"
done
