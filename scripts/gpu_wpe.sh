#!/bin/bash
# 16-wave row kernel budgeted for one workgroup per CU (4 waves per SIMD, no spills) when the
# tiles fit the CUs: parity tests and A/B against the 8-wave-per-SIMD budget (DGPRF_ROWS16_WPE8=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=${OUT:-gpurun_out/wpe}
mkdir -p $OUT && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_large_batch.py tests/test_gpu_predictive.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  if [ $v = 1 ]; then export DGPRF_ROWS16_WPE8=1; fi
  timeout -k 10 120 python scripts/diag/pred_paths.py 3 auto 4000 > $OUT/pred3_$v.log 2>&1 || exit $?
  timeout -k 10 120 python scripts/diag/pred_paths.py 2 auto 4000 > $OUT/pred2_$v.log 2>&1 || exit $?
  timeout -k 10 200 python scripts/diag/step_graph.py 2 2048,4096 1000 > $OUT/step_$v.log 2>&1 || exit $?
  echo "WPE8=$v"; grep -h config $OUT/pred3_$v.log $OUT/pred2_$v.log $OUT/step_$v.log
done
