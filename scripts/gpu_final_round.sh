#!/bin/bash
# End-of-round evidence in one gpurun call: the GPU test suite, the bench evidence
# (scripts/gpu_profile_round.sh: kernel trace, HBM PMC passes, plain bench), and rocprofv3 kernel
# traces of the config 4 / 5 steps.  Each step has its own time limit; the first failure ends it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD
TAG=${TAG:-r05}
O=$R/gpurun_out/final_$TAG
P=$R/profiles/$TAG
mkdir -p $O $P
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests \
  > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 3; }
tail -3 $O/pytest_gpu.log
cp $O/pytest_gpu.log $P/pytest_gpu.log
TAG=$TAG bash scripts/gpu_profile_round.sh > $O/profile_round.log 2>&1 || { tail -20 $O/profile_round.log; exit 4; }
export TMPDIR=/tmp
for c in 4 5; do
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt$c -o run \
    -- python3 $R/scripts/diag/step_graph.py $c 200 300 > $O/kt$c.log 2>&1) || exit 5
  f=$(find $O/kt$c -name "*kernel_stats.csv" | head -1)
  cp "$f" $P/kernel_stats_step_config$c.csv
  cut -d, -f1-5 "$f" | cut -c1-150 | head -12
done
cp $P/* $O/ 2>/dev/null
tail -c 800 $O/profile_round.log
