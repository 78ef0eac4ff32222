#!/bin/bash
# A/B of env settings on one config: one bench line per setting (no CPU baseline, no host pass)
#   CONFIG=3 SETTINGS="A=1 B=2;A=2" bash scripts/gpu_ab.sh    (settings separated by ';')
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
c=${CONFIG:-3}
i=0
IFS=';' read -ra SETS <<< "${SETTINGS:-}"
[ ${#SETS[@]} -eq 0 ] && SETS=("")
for s in "${SETS[@]}"; do
  i=$((i+1))
  env $s timeout -k 10 300 python3 -u bench.py --config $c --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-host \
    ${BENCH_ARGS:-} > gpurun_out/ab/c${c}_$i.log 2> gpurun_out/ab/c${c}_$i.err
  rc=$?
  python3 - "$s" gpurun_out/ab/c${c}_$i.log <<'EOF'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
s = d['stage_ms_1stream']
keys = ['descent_tile', 'flood_descent', 'flood_relax', 'flood_verify', 'seeds', 'size_filter', 'crop_cc', 'frontier_iters', 'regrow_iters']
print('[%s] %.3f Gvox/s %.2f ms/step | ' % (sys.argv[1], d['value'], d['ms_per_step']) + ' '.join('%s %.2f' % (k, s.get(k, 0)) for k in keys))
EOF
  [ $rc -ne 0 ] && { echo "rc=$rc"; tail -3 gpurun_out/ab/c${c}_$i.err; exit $rc; }
done
exit 0
