#!/bin/bash
# rocprofv3 kernel-trace summary of the full-Bayes step driver.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
TAG=${TAG:-fb}
timeout -k 10 300 python3 scripts/prof_fb.py > gpurun_out/prof/${TAG}_plain.log 2>&1
rc=$?; tail -3 gpurun_out/prof/${TAG}_plain.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/$TAG -o run \
  -- python3 scripts/prof_fb.py > gpurun_out/prof/${TAG}_rocprof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof/${TAG}_rocprof.log
exit $rc
