#!/bin/bash
# Quick GPU iteration: selected parity tests, the config-2 B-sweep, a kernel trace at B = 8192 / 65536.
#   OUT=gpurun_out/x TESTS="tests/test_gpu_large_batch.py" bash scripts/gpu_quick.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=${OUT:-gpurun_out/quick}
TESTS=${TESTS:-"tests/test_gpu_large_batch.py tests/test_gpu_full_bayes.py"}
mkdir -p $OUT && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -5 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/diag/step_graph.py 2 ${SWEEP:-200,1024,8192,65536} 1000 > $OUT/sweep.log 2>&1 || exit $?
grep config $OUT/sweep.log
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof -o kt -- python scripts/diag/step_graph.py 2 ${TRACE_B:-8192} 200 > $OUT/prof.log 2>&1
echo prof rc=$?
