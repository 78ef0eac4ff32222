#!/bin/bash
# Round 6: the Gaussians' two interleaved FP64 sums per step (gauss_run / gauss_win) and the EDT
# column search on two voxels at once, the crop merge loads in one round trip: parity, then the
# A/B: new (all), gauss (the Gaussians
# only, libctws_gauss.so), prev (neither, libctws_prev.so) as CTWS_LIB.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_config_blocks.py tests/test_golden_gpu.py tests/test_from_seeds_gpu.py tests/test_gpu_pass2.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for c in 3 4; do
  for k in 1 2; do
    for v in new gauss prev; do
      unset CTWS_LIB
      [ $v != new ] && export CTWS_LIB=$PWD/cluster_tools_amd/libctws_$v.so
      timeout -k 10 200 python -u bench.py --config $c --streams 1 --steps 2 --warmup 1 --no-host --no-cpu-baseline --no-e2e --no-strong --no-threshcc --no-config5 > $O/c${c}_${v}_$k.json 2> $O/c${c}_${v}_$k.err || { tail -5 $O/c${c}_${v}_$k.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/c${c}_${v}_$k.json').read().strip().splitlines()[-1]); s=d['stage_ms_1stream']; print('c$c $v', d['ms_per_step'], {k: round(v, 2) for k, v in s.items() if k in ('smooth_seeds', 'hmap', 'edt_yz', 'crop_cc', 'output')})"
    done
  done
done
