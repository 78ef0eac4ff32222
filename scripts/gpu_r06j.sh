#!/bin/bash
# Round 6: the frontier filtered by the final C (experiment), then the wide-key pass-2 mismatch (debug, traced).
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06j
mkdir -p $O
export TMPDIR=/tmp
for c in 3 4; do
  CTWS_TRACE=1 CTWS_CTRUE_EXP=1 timeout -k 10 300 python -u bench.py --config $c --streams 1 --steps 1 --warmup 0 --no-host --no-cpu-baseline --no-e2e --no-strong --no-threshcc --no-config5 > $O/c$c.json 2> $O/c$c.err || { tail -5 $O/c$c.err; exit 1; }
  grep -E "ctrue exp|verify" $O/c$c.err | head -20
done
CTWS_TRACE=1 timeout -k 10 150 python -u scripts/dbg/wide_pass2.py 2d > $O/wide_pass2.log 2> $O/wide_pass2.err; echo "wide rc=$?"; tail -5 $O/wide_pass2.log; grep -c "flood round" $O/wide_pass2.err; grep -v "flood round" $O/wide_pass2.err | tail -20
