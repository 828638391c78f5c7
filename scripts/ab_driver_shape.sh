#!/bin/bash
# The driver's bench shape (--steps 20 --warmup 5, extra legs off) for the product library and
# each variant, interleaved over REPS rounds: the line's value and ms_per_step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for rep in $(seq 1 ${REPS:-3}); do
  for lib in dgp-rf-mcmc_amd/dgprf/libdgprf.so ${VARIANTS:-scripts/variants/*/libdgprf.so}; do
    n=$(basename $(dirname $lib))
    DGPRF_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline \
      --multi-chains 0 --full-bayes-steps 0 --other-configs 0 --b-sweep 0 --eager-calls 0 \
      --driver-epochs 0 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$n', d['value'], d['ms_per_step'], d['roofline']['step_us_events'])" || exit 3
  done
done
