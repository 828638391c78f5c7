#!/bin/bash
# Large-batch parity tests, the config-2 B-sweep and a kernel trace at B = 8192 / 65536.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=${OUT:-gpurun_out/r03d}
mkdir -p $OUT && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_new.log 2>&1
rc=$?; tail -5 $OUT/pytest_new.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/diag/step_graph.py 2 200,1024,8192,65536 1000 > $OUT/sweep.log 2>&1 || exit $?
grep config $OUT/sweep.log
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof -o kt -- python scripts/diag/step_graph.py 2 8192,65536 200 > $OUT/prof.log 2>&1
echo prof rc=$?
bash scripts/diag/agemm_cmp.sh
