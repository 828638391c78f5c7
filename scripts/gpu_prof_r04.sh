#!/bin/bash
# Round-4 profile evidence in one call: rocprofv3 kernel traces of configs 4 and 5 (graph-replayed
# steps at B = 200), then SQ / LDS counter passes of the config-2 predictive forward and of the
# config-4 step (the A_1 GEMM and the backward kernels).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD
O=$R/gpurun_out/prof_r04
mkdir -p $O
export TMPDIR=/tmp
for c in 4 5; do
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt$c -o run \
    -- python3 $R/scripts/diag/step_graph.py $c 200 300 > $O/kt$c.log 2>&1) || exit $?
  f=$(find $O/kt$c -name "*kernel_stats.csv" | head -1)
  echo "== config $c kernel stats"; cut -d, -f1-5 "$f" | cut -c1-150 | head -16
done
NAME=pred CMD="python3 $R/scripts/prof_predict.py --samples 3" FILTER=forward_tiles scripts/gpu_pmc.sh || exit $?
NAME=c4 CMD="python3 $R/scripts/diag/step_graph.py 4 200 100" FILTER="agemm\|step_bwd\|step_update" scripts/gpu_pmc.sh || exit $?
