#!/bin/bash
# Round 6: the frontier back at round 5's registers (no per-write statistics / saturation test in
# its loop; d saturation detected on the final keys by k_flood_verify): parity incl. the corridor
# (d > 4095) cases, the A/B against the previous build (libctws_prev.so), then the EDT column
# tile widths (64 new) on configs 4 / 3.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06o
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_corridor_gpu.py tests/test_gpu_parity.py tests/test_config_blocks.py tests/test_frontier_variants.py tests/test_from_seeds_gpu.py tests/test_gpu_pass2.py tests/test_golden_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
CTWS_EDT_W=64 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "stages_bit_exact or config2" --timeout 120 --timeout-method thread > $O/pytest_w64.log 2>&1
rc=$?; tail -1 $O/pytest_w64.log; [ $rc -ne 0 ] && exit $rc
for c in 4 3 5; do
  for k in 1 2; do
    for v in new prev; do
      unset CTWS_LIB
      [ $v = prev ] && export CTWS_LIB=$PWD/cluster_tools_amd/libctws_prev.so
      timeout -k 10 200 python -u bench.py --config $c --streams 1 --steps 2 --warmup 1 --no-host --no-cpu-baseline --no-e2e --no-strong --no-threshcc --no-config5 > $O/c${c}_${v}_$k.json 2> $O/c${c}_${v}_$k.err || { tail -5 $O/c${c}_${v}_$k.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/c${c}_${v}_$k.json').read().strip().splitlines()[-1]); s=d['stage_ms_1stream']; print('c$c $v', d['ms_per_step'], {k: round(v, 2) for k, v in s.items() if k in ('flood_relax', 'flood_verify', 'size_filter', 'seeds')})"
    done
  done
done
unset CTWS_LIB
for c in 4 3; do
  for v in CTWS_EDT_WZ=64 CTWS_EDT_WZ=16 CTWS_EDT_W=32 CTWS_EDT_W=64 CTWS_EDT_W=8; do
    tag=$(echo "$v" | tr '=, ' '___')
    ( export $v; timeout -k 10 200 python -u bench.py --config $c --streams 1 --steps 2 --warmup 1 --no-host --no-cpu-baseline --no-e2e --no-strong --no-threshcc --no-config5 > $O/c${c}_$tag.json 2> $O/c${c}_$tag.err ) || { tail -5 $O/c${c}_$tag.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c${c}_$tag.json').read().strip().splitlines()[-1]); s=d['stage_ms_1stream']; print('c$c $v', d['ms_per_step'], {k: v for k, v in s.items() if k in ('prep_edt_x', 'edt_yz')})"
  done
done
