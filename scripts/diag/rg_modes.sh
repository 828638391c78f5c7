#!/bin/bash
# Diagnostic: per-kernel durations of config 2 at B = 8192 with the row-group backward's
# DGPRF_DBG_RG switches (1: no prologue loads, 2: no chunk compute, 4: no dX reduction/store).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/rg_modes
for m in 0 1 2 4 7; do
  DGPRF_DBG_RG=$m timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/rg_modes/m$m -o kt -- \
    python scripts/diag/step_graph.py 2 ${B:-8192} 200 > gpurun_out/rg_modes/m$m.log 2>&1 || exit $?
done
echo done
