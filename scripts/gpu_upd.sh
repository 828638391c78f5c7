#!/bin/bash
# Update kernel with the mass / step-counter / layer-bound loads issued with the partial loads:
# full GPU suite, then the B = 200 steps of configs 2-5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=${OUT:-gpurun_out/upd}
mkdir -p $OUT && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for c in 2 3 4 5; do
  timeout -k 10 200 python scripts/diag/step_graph.py $c 200 3000 > $OUT/step_c$c.log 2>&1 || exit $?
  grep -h config $OUT/step_c$c.log
done
