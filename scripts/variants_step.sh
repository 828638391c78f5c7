#!/bin/bash
# Single-chain steps/s and 64-chain chain-steps/s of the default library and each variant build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for lib in dgp-rf-mcmc_amd/dgprf/libdgprf.so scripts/variants/*.so; do
  echo -n "$lib: "
  DGPRF_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --steps 4000 --pred-samples 2 --multi-chains 64 \
    --full-bayes-steps 0 --other-configs 0 --no-cpu-baseline --profile-reps 20 2>/dev/null | \
    python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['multi_chain'])" || exit $?
done
