#!/bin/bash
# Predictive us/sample of the default library and of each build under scripts/variants/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for lib in dgp-rf-mcmc_amd/dgprf/libdgprf.so scripts/variants/*.so; do
  echo -n "$lib: "
  DGPRF_LIB=$PWD/$lib timeout -k 10 120 python3 scripts/prof_predict.py --samples 20 2>&1 | tail -1 || exit $?
done
