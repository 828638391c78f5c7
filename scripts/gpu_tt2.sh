#!/bin/bash
# Two-tile row-kernel workgroups (forward_cfg rows_tt = 2): parity tests, config-3 predictive and
# config-2 B = 8,192 step A/B against the one-tile 8-wave form (DGPRF_ROWS_TT1=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=${OUT:-gpurun_out/tt2}
mkdir -p $OUT && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_large_batch.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  if [ $v = 1 ]; then export DGPRF_ROWS_TT1=1; fi
  timeout -k 10 120 python scripts/diag/pred_paths.py 3 auto > $OUT/pred3_$v.log 2>&1 || exit $?
  timeout -k 10 120 python scripts/diag/pred_paths.py 2 auto 8192 > $OUT/pred2_$v.log 2>&1 || exit $?
  timeout -k 10 200 python scripts/diag/step_graph.py 2 2048,8192 1000 > $OUT/step_$v.log 2>&1 || exit $?
  echo "TT1=$v"; grep -h config $OUT/pred3_$v.log $OUT/pred2_$v.log $OUT/step_$v.log
done
