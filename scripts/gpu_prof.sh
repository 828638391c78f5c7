#!/bin/bash
# rocprofv3 kernel-trace summary of the bench (no PMC counters in this pass).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
TAG=${TAG:-r01}
BENCH_ARGS=${BENCH_ARGS:-"--steps 2000 --warmup 200 --no-cpu-baseline --multi-chains 0"}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/$TAG -o run \
  -- python3 bench.py $BENCH_ARGS > gpurun_out/prof/${TAG}_bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof/${TAG}_bench.log
find gpurun_out/prof/$TAG -name "*stats*" | head
exit $rc
