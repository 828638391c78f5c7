#!/bin/bash
# Predictive-kernel experiment: variants, test-set sizes, per-wave stamps, then the GPU tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/pred_exp.txt
bash scripts/variants_pred.sh > $O 2>&1 || exit $?
bash scripts/pred_sizes.sh >> $O 2>&1 || exit $?
for n in 65536 100000; do
  DGPRF_LIB=$PWD/scripts/microbench/libdgprf_pstamps.so timeout -k 10 120 python3 scripts/microbench/pred_stamps.py $n >> $O 2>&1 || exit $?
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
tail -3 gpurun_out/pytest_gpu.log
