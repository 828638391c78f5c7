#!/bin/bash
# gpu_check.sh, then the stamped diagnostic build (only if the checks did not fault).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash scripts/gpu_check.sh
rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
DGPRF_LIB=scripts/microbench/libdgprf_stamps.so timeout -k 10 200 python scripts/microbench/stamps.py > gpurun_out/stamps.log 2>&1
rc2=$?; echo "stamps rc=$rc2"; cat gpurun_out/stamps.log | grep -v amdgpu.ids
exit $rc2
