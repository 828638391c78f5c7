#!/bin/bash
# GPU check: the GPU test suite, then (only if it is green) a bench run.
#   TAG=... PYTEST_ARGS="-k ..." BENCH_ARGS="..." scripts/gpu_check.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/${TAG:-r4}
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  ${PYTEST_ARGS} > $O/pytest_gpu.log 2>&1
rc=$?
tail -5 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
[ -n "${NO_BENCH}" ] && exit 0
timeout -k 10 500 python bench.py ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err || exit $?
tail -c 1500 $O/bench.json
