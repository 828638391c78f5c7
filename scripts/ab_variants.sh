#!/bin/bash
# A/B timing of variant builds (scripts/variants/<name>/{libdgprf.so,libdgprf_torch.so}) against
# the default library, interleaved over REPS rounds: config-2 predictive us/sample (1e5 test rows)
# and graph-replayed SGHMC steps of the CONFIGS at B = 200.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for rep in $(seq 1 ${REPS:-2}); do
  for lib in dgp-rf-mcmc_amd/dgprf/libdgprf.so scripts/variants/*/libdgprf.so; do
    n=$(basename $(dirname $lib))
    echo "== $n (round $rep)"
    if [ -z "${NO_PRED}" ]; then
      DGPRF_LIB=$PWD/$lib timeout -k 10 120 python3 scripts/prof_predict.py --samples 20 || exit $?
      DGPRF_LIB=$PWD/$lib timeout -k 10 120 python3 scripts/prof_predict.py --samples 20 --pairs || exit $?
    fi
    for c in ${CONFIGS:-2 4 5}; do
      DGPRF_LIB=$PWD/$lib timeout -k 10 200 python3 scripts/diag/step_graph.py $c 200 ${STEPS:-2000} || exit $?
    done
  done
done
