cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for s in ${STREAMS:-1 2 4}; do
  timeout -k 10 120 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --streams $s ${BENCH_ARGS:-} > gpurun_out/exp_s$s.log 2>&1 || exit $?
  python -c "
import json; d=json.loads(open('gpurun_out/exp_s$s.log').read().strip().splitlines()[-1])
print('streams=$s', d['value'], d['ms_per_step'], d['roofline']['ms_per_step'])"
done
