#!/bin/bash
# Predictive us/sample at test-set sizes that fill 1, 1.5 and 2 rounds of 4096 resident waves.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for n in 65536 100000 131072 262144; do
  echo -n "n_test=$n: "
  timeout -k 10 120 python3 scripts/prof_predict.py --samples 20 --n-test $n 2>&1 | tail -1 || exit $?
done
