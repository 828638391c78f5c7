#!/bin/bash
# Diagnostic: the hand-written A_1 GEMM (agemm.hip, default) against the cached hipBLASLt kernel
# (DGPRF_AGEMM=lib) on config 4's two shapes — the step (B = 200 rows x 784 x 4096) and the
# predictive forward (10k test rows x 784 x 4096) — per-kernel durations from a rocprofv3 kernel
# trace of each arm, plus each arm's step and predictive wall times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/agemm_cmp}
mkdir -p $OUT
for arm in own lib; do
  DGPRF_AGEMM=$arm timeout -k 10 200 python scripts/diag/step_graph.py 4 200 1000 > $OUT/step_$arm.log 2>&1 || exit $?
  DGPRF_AGEMM=$arm timeout -k 10 200 python scripts/diag/pred_paths.py 4 auto 10000 > $OUT/pred_$arm.log 2>&1 || exit $?
  DGPRF_AGEMM=$arm timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/kt_$arm -o kt -- python scripts/diag/step_graph.py 4 200 300 > $OUT/kt_step_$arm.log 2>&1 || exit $?
  DGPRF_AGEMM=$arm timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/ktp_$arm -o kt -- python scripts/diag/pred_paths.py 4 auto 10000 > $OUT/kt_pred_$arm.log 2>&1 || exit $?
  grep -h "config\|us/sample" $OUT/step_$arm.log $OUT/pred_$arm.log | sed "s/^/$arm: /"
done
