#!/bin/bash
# SQ counter passes of the step kernels (scripts/gpu_pmc.sh, two passes each): configs 4 / 5
# at 64 chains per launch (the compute-bound regime) and config 2 / 4 / 5 with one chain.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD
for job in "mc64_c4|python3 $R/scripts/diag/mc_rate.py 64 4" "mc64_c5|python3 $R/scripts/diag/mc_rate.py 64 5" \
           "mc64_c2|python3 $R/scripts/diag/mc_rate.py 64 2" "step_c2|python3 $R/scripts/diag/step_graph.py 2 200 600" \
           "step_c4|python3 $R/scripts/diag/step_graph.py 4 200 300" "step_c5|python3 $R/scripts/diag/step_graph.py 5 200 300"; do
  NAME=${job%%|*} CMD=${job#*|} PASS_LIMIT=150 bash $R/scripts/gpu_pmc.sh > $R/gpurun_out/pmc_${job%%|*}.log 2>&1 || { tail $R/gpurun_out/pmc_${job%%|*}.log; exit 3; }
  mkdir -p $R/gpurun_out/pmc_r06
  cp $R/gpurun_out/pmc_${job%%|*}/summary.csv $R/gpurun_out/pmc_r06/${job%%|*}.csv
  rm -rf $R/gpurun_out/pmc_${job%%|*}  # raw per-dispatch CSVs: only the summary comes back
  echo "== ${job%%|*} done"
done
