#!/bin/bash
# Predictive us/sample of the default library and of each build under scripts/variants/, at the
# config-2 test-set size and at 65536 rows (one round of 4096 resident waves).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for lib in dgp-rf-mcmc_amd/dgprf/libdgprf.so scripts/variants/*.so; do
  for n in 100000 65536; do
    echo -n "$lib n=$n: "
    DGPRF_LIB=$PWD/$lib timeout -k 10 120 python3 scripts/prof_predict.py --samples 20 --n-test $n 2>&1 | tail -1 || exit $?
  done
done
