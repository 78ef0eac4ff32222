cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -3 gpurun_out/t.log; grep -E "FAIL|Error" gpurun_out/t.log | head -20
[ $rc -ne 0 ] && exit $rc
CTWS_TRACE=${TRACE:-0} timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/b.log 2>&1; rc=$?; grep "\[ctws\]" gpurun_out/b.log | tail -12; tail -1 gpurun_out/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step']); print(d['stage_ms'])"
exit $rc
