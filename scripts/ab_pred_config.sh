#!/bin/bash
# A/B of variant builds (scripts/variants/<name>/libdgprf.so) on the predictive add_samples time of
# BASELINE configs (default 4 and 3), interleaved over REPS rounds; checksums must match.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for rep in $(seq 1 ${REPS:-2}); do
  for lib in dgp-rf-mcmc_amd/dgprf/libdgprf.so scripts/variants/*/libdgprf.so; do
    n=$(basename $(dirname $lib))
    for c in ${CONFIGS:-4 3}; do
      echo -n "$n: "
      DGPRF_LIB=$PWD/$lib timeout -k 10 200 python3 scripts/diag/pred_config.py $c ${SAMPLES:-10} 5 || exit $?
    done
  done
done
