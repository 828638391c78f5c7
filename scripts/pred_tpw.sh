#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for tpw in 1 2; do
  echo -n "TPW=$tpw: "
  DGPRF_TILE_TPW=$tpw timeout -k 10 120 python3 scripts/prof_predict.py --samples 20 2>&1 | tail -1 || exit $?
done
