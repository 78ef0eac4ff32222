#!/bin/bash
# Round-4 profiles: single-stream rocprofv3 kernel traces of configs 3, 4, 5 (stage table +
# trace roofline), then the PMC passes (calibration + per-stage traffic of configs 3 and 4).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_r04g_traces.sh || exit 1
echo "[$(date +%T)] PMC"
bash scripts/gpu_pmc_r04.sh || exit 1
echo "[$(date +%T)] done"
