#!/bin/bash
# GPU suite, predictive test-set size sweep, config-2 B-sweep and the full bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=${OUT:-gpurun_out/r03g}
mkdir -p $OUT && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/pred_sizes.sh > $OUT/pred_sizes.log 2>&1 || exit $?
cat $OUT/pred_sizes.log
timeout -k 10 300 python scripts/diag/step_graph.py 2 200,8192,65536 1000 > $OUT/sweep.log 2>&1 || exit $?
grep config $OUT/sweep.log
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
tail -c 300 $OUT/bench.json
