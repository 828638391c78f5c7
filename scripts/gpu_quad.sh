#!/bin/bash
# Small-minibatch one-launch forward (k_step_fwd_quad): GPU suite, step A/B against the per-layer
# forward (DGPRF_NO_QUAD=1), kernel trace of config 2's step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=${OUT:-gpurun_out/quad}
mkdir -p $OUT && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -5 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for c in 2 3; do
  timeout -k 10 200 python scripts/diag/step_graph.py $c 200 3000 > $OUT/quad_c$c.log 2>&1 || exit $?
  DGPRF_NO_QUAD=1 timeout -k 10 200 python scripts/diag/step_graph.py $c 200 3000 > $OUT/layer_c$c.log 2>&1 || exit $?
  grep -h config $OUT/quad_c$c.log $OUT/layer_c$c.log
done
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/kt -o run \
  -- python3 $GRAFT_REPO_ROOT/scripts/diag/step_graph.py 2 200 2000 > $GRAFT_REPO_ROOT/$OUT/kt.log 2>&1 || exit $?
grep -E "k_step|Name" $GRAFT_REPO_ROOT/$OUT/kt/run_kernel_stats.csv | cut -c1-160
