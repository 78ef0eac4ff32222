#!/bin/bash
# PMC passes (one counter group per run, kernel trace off): the gather calibration microkernel,
# then HBM bytes per stage of configs 3 and 4 with the dispatch-order stage map.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_cal
./scripts/micro/gather_bytes > gpurun_out/pmc_cal/known.json || exit 1
for grp in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc_cal/$grp -o p -- ./scripts/micro/gather_bytes > gpurun_out/pmc_cal/$grp.log 2>&1 || { echo "cal $grp failed"; tail -5 gpurun_out/pmc_cal/$grp.log; exit 1; }
done
python3 scripts/pmc_gather_calibration.py gpurun_out/pmc_cal gpurun_out/pmc_cal/known.json > gpurun_out/pmc_cal/calibration.json && cat gpurun_out/pmc_cal/calibration.json
for c in ${CONFIGS:-3 4}; do
  mkdir -p gpurun_out/pmc_c$c
  for grp in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $grp --kernel-include-regex ctws --output-format csv -d gpurun_out/pmc_c$c/$grp -o p -- python3 -u bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline --no-host --no-e2e --no-strong --streams 1 > gpurun_out/pmc_c$c/$grp.log 2>&1 || { echo "pmc c$c $grp failed"; tail -5 gpurun_out/pmc_c$c/$grp.log; exit 1; }
  done
  python3 scripts/pmc_traffic.py gpurun_out/pmc_c$c > gpurun_out/pmc_c$c/traffic_c$c.json
  python3 -c "import json; d=json.load(open('gpurun_out/pmc_c$c/traffic_c$c.json')); print('c$c', {k: round(v/1e9,2) for k, v in d.items() if isinstance(v, float)})"
  rm -rf gpurun_out/pmc_c$c/FETCH_SIZE gpurun_out/pmc_c$c/WRITE_SIZE
done
