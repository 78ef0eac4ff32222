#!/bin/bash
# host-resident path rate for several CTWS_D2H_WGS values (bench config 3)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for v in ${VALUES:-0 16 32 64}; do
  export ${VAR:-CTWS_D2H_WGS}=$v; timeout -k 10 300 python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/host_$v.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { tail -3 gpurun_out/host_$v.log; exit $rc; }
  echo "${VAR:-CTWS_D2H_WGS}=$v $(grep -o '"host_resident": {[^}]*}' gpurun_out/host_$v.log | cut -c1-120)"
done
exit 0
