#!/bin/bash
# A/B of variant builds (scripts/variants/<name>/) against the product library, interleaved over
# REPS rounds: config-2 predictive (40 samples in one add_samples call, 1e5 test rows) and
# graph-replayed SGHMC steps of CONFIGS at B = 200.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for rep in $(seq 1 ${REPS:-2}); do
  for lib in dgp-rf-mcmc_amd/dgprf/libdgprf.so ${VARIANTS:-scripts/variants/*/libdgprf.so}; do
    n=$(basename $(dirname $lib))
    echo "== $n (round $rep)"
    if [ -z "${NO_PRED}" ]; then
      DGPRF_LIB=$PWD/$lib timeout -k 10 120 python3 scripts/prof_predict.py --samples 40 --batch || exit $?
    fi
    for c in ${CONFIGS:-2}; do
      DGPRF_LIB=$PWD/$lib timeout -k 10 200 python3 scripts/diag/step_graph.py $c 200 ${STEPS:-3000} || exit $?
    done
  done
done
