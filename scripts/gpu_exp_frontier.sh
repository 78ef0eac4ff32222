cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for it in 256 0 8 16; do
  CTWS_FRONTIER_ITERS=$it timeout -k 10 120 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/exp_$it.log 2>&1 || exit $?
  python -c "
import json; d=json.loads(open('gpurun_out/exp_$it.log').read().strip().splitlines()[-1]); s=d['stage_ms']
print('iters=$it', d['value'], {k: s[k] for k in ('descent_tile','flood_descent','flood_relax','frontier_iters','flood_rounds','flood_tiles_solved')})"
done
