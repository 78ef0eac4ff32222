cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
# k_frontier variants: CTWS_FRONTIER_MODE bit0 = no XCD chunk order, bit1 = full neighbour reads
for m in ${MODES:-0 1 2 3}; do
  for tr in 0 1; do
  CTWS_TRACE=$tr CTWS_FRONTIER_MODE=$m timeout -k 10 120 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/exp_$m.log 2>&1 || exit $?
  python -c "
import json; d=json.loads(open('gpurun_out/exp_$m.log').read().strip().splitlines()[-1]); s=d['stage_ms']
print('mode=$m trace=$tr', d['value'], {k: s[k] for k in ('descent_tile','flood_descent','flood_relax','frontier_iters','open_voxels','frontier_visits','frontier_full_launches') if k in s})"
  done
done
