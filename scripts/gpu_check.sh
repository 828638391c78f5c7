#!/bin/bash
# Working check: targeted tests first, then the GPU suite, the fold A/B and a bench run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/${TAG:-chk}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_configs.py -k "folded or resident or dataset_a1 or full_bayes_graph" > $O/pytest_new.log 2>&1 \
  || { tail -30 $O/pytest_new.log; exit 3; }
tail -3 $O/pytest_new.log
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 4; }
tail -3 $O/pytest_gpu.log
[ -n "$NO_AB" ] || { CONFIGS="2 3 5" REPS=2 STEPS=3000 timeout -k 10 600 bash scripts/ab_variants.sh > $O/ab.log 2>&1 || { tail $O/ab.log; exit 5; }; cat $O/ab.log; }
[ -n "$NO_BENCH" ] || { timeout -k 10 500 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 6; }; tail -c 400 $O/bench.json; }
