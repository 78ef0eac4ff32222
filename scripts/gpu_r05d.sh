#!/bin/bash
# Round 5: threshcc workflow tests + end to end (threaded chunk I/O, table write), then the
# config-3 stream-count sweep.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_threshcc_gpu.py tests/test_threshcc.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for m in 1 0; do
  timeout -k 10 400 python -u scripts/e2e_threshcc.py --merge-in-job $m > $O/e2e_tc_$m.json 2> $O/e2e_tc_$m.err || { tail -5 $O/e2e_tc_$m.err; exit 1; }
  cat $O/e2e_tc_$m.json
done
for s in ${STREAMS-2 4 6}; do
  timeout -k 10 300 python -u bench.py --config 3 --streams $s --steps 4 --warmup 1 --no-host --no-cpu-baseline --no-e2e --no-strong --no-threshcc --no-config5 > $O/c3_s$s.json 2> $O/c3_s$s.err || { tail -5 $O/c3_s$s.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c3_s$s.json').read().strip().splitlines()[-1]); print('streams $s', d['value'], d['ms_per_step'])"
done
