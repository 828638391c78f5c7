#!/bin/bash
# End-of-round evidence in one gpurun call: the GPU test suite, the bench evidence
# (scripts/gpu_profile_round.sh: kernel trace, HBM PMC passes, plain bench), rocprofv3 kernel
# traces of the config 4 / 5 steps, FETCH_SIZE / WRITE_SIZE passes of the config 4 / 5 steps and
# SQ counters of the predictive pair kernel.  Each step has its own time limit; the first failure
# ends it.  PART=1: suite + bench evidence only; PART=2: the config / counter profiles only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD
TAG=${TAG:-r06}
O=$R/gpurun_out/final_$TAG
P=$R/profiles/$TAG
mkdir -p $O $P
if [ "${PART:-1}" = 1 ]; then
  timeout -k 10 700 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests \
    > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 3; }
  tail -3 $O/pytest_gpu.log
  cp $O/pytest_gpu.log $P/pytest_gpu.log
  TAG=$TAG bash scripts/gpu_profile_round.sh > $O/profile_round.log 2>&1 || { tail -20 $O/profile_round.log; exit 4; }
  cp $P/* $O/ 2>/dev/null
  tail -c 800 $O/profile_round.log
  exit 0
fi
export TMPDIR=/tmp
for c in 4 5; do
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt$c -o run \
    -- python3 $R/scripts/diag/step_graph.py $c 200 300 > $O/kt$c.log 2>&1) || exit 5
  f=$(find $O/kt$c -name "*kernel_stats.csv" | head -1)
  cp "$f" $P/kernel_stats_step_config$c.csv
  cut -d, -f1-5 "$f" | cut -c1-150 | head -12
  # HBM-side bytes of the step kernels: FETCH_SIZE and WRITE_SIZE in passes of their own
  for ctr in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $O/pmc${c}_${ctr} -o run \
      -- python3 $R/scripts/diag/step_graph.py $c 200 100 > $O/pmc${c}_$ctr.log 2>&1) || exit 6
  done
  python3 $R/scripts/pmc_summary.py $P/pmc_traffic_step_config$c.csv $O/pmc${c}_FETCH_SIZE $O/pmc${c}_WRITE_SIZE > /dev/null || exit 7
done
# SQ counters of the predictive pair kernel (issue port / MFMA pipe)
NAME=pred_pairs CMD="python3 $R/scripts/prof_predict.py --samples 60 --batch" bash scripts/gpu_pmc.sh \
  > $O/pmc_pred_pairs.log 2>&1 || { tail $O/pmc_pred_pairs.log; exit 8; }
cp $R/gpurun_out/pmc_pred_pairs/summary.csv $P/pmc_sq_predictive_pairs.csv
cp $P/* $O/ 2>/dev/null
grep -i "pairs\|tiles" $P/pmc_sq_predictive_pairs.csv | head -20
