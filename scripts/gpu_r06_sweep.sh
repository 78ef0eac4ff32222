#!/bin/bash
# Single-stream stage times over knob settings (VARIANTS, comma-joined; "base" = defaults),
# twice each, alternating; STAGES = the stage keys printed.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06_sweep${TAG:+_$TAG}
mkdir -p $O
export TMPDIR=/tmp
STAGES=${STAGES:-edt_yz smooth_seeds hmap}
for c in ${CONFIGS:-3 4}; do
  for k in 1 2; do
    for v in ${VARIANTS:-base}; do
      tag=$(echo "$v" | tr '=, ' '___')
      ( [ "$v" != base ] && export $(echo $v | tr ',' ' '); timeout -k 10 200 python -u bench.py --config $c --streams 1 --steps 2 --warmup 1 --no-host --no-cpu-baseline --no-e2e --no-strong --no-threshcc --no-config5 > $O/c${c}_${tag}_$k.json 2> $O/c${c}_${tag}_$k.err ) || { tail -5 $O/c${c}_${tag}_$k.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/c${c}_${tag}_$k.json').read().strip().splitlines()[-1]); s=d['stage_ms_1stream']; print('c$c $v', d['ms_per_step'], {k: round(s.get(k, -1), 3) for k in '$STAGES'.split()})"
    done
  done
done
