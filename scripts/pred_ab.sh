#!/bin/bash
# A/B of the predictive kernel: default library vs scripts/variants/*.so, interleaved, 3 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for rep in 1 2 3; do
  for lib in dgp-rf-mcmc_amd/dgprf/libdgprf.so scripts/variants/*.so; do
    echo -n "$lib: "
    DGPRF_LIB=$PWD/$lib timeout -k 10 120 python3 scripts/prof_predict.py --samples 20 2>&1 | tail -1 || exit $?
  done
done
