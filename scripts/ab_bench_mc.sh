#!/bin/bash
# A/B of variant builds on the bench's config-2 step rate and its 64-chain leg (short bench runs,
# every other leg off), interleaved over REPS rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for rep in $(seq 1 ${REPS:-2}); do
  for lib in dgp-rf-mcmc_amd/dgprf/libdgprf.so scripts/variants/*/libdgprf.so; do
    n=$(basename $(dirname $lib))
    DGPRF_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --steps 4000 --warmup 200 --other-configs 0 \
      --b-sweep 0 --eager-calls 0 --no-cpu-baseline --full-bayes-steps 0 --pred-samples 2 \
      --profile-reps 20 > gpurun_out/ab_mc_$n.json 2>gpurun_out/ab_mc_$n.err || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'steps/s', d['value'], 'chain-steps/s', d['multi_chain']['chain_steps_per_s'])" gpurun_out/ab_mc_$n.json $n || exit 5
  done
done
