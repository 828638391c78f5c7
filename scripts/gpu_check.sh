#!/bin/bash
# One gpurun call: smoke -> GPU parity tests -> bench.  Each GPU step has its own time limit;
# anything other than success / ordinary test failure (exit 0/1) ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
BENCH_ARGS=${BENCH_ARGS:-"--steps 2000 --warmup 200 --cpu-runs 5"}
PYTEST_ARGS=${PYTEST_ARGS:-"tests -m gpu -q"}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 1200 python -m pytest $PYTEST_ARGS --timeout 600 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
exit $rc
