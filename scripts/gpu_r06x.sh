#!/bin/bash
# Round 6 (measurement only): the global union-find with device-scope parent loads and no path
# halving everywhere (libctws_coh.so): parity + repeatability on it, then configs 3 / 4 A/B.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06x
mkdir -p $O
export TMPDIR=/tmp
CTWS_LIB=$PWD/cluster_tools_amd/libctws_coh.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_config_blocks.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for c in 3 4; do
  for v in cur coh cur coh; do
    unset CTWS_LIB
    [ $v = coh ] && export CTWS_LIB=$PWD/cluster_tools_amd/libctws_coh.so
    timeout -k 10 200 python -u bench.py --config $c --streams 1 --steps 2 --warmup 1 --no-host --no-cpu-baseline --no-e2e --no-strong --no-threshcc --no-config5 > $O/c${c}_$v.json 2> $O/c${c}_$v.err || { tail -5 $O/c${c}_$v.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c${c}_$v.json').read().strip().splitlines()[-1]); s=d['stage_ms_1stream']; print('c$c $v', d['ms_per_step'], {k: round(s[k], 2) for k in ('seeds', 'crop_cc', 'size_filter')})"
  done
done
