#!/bin/bash
# Config 4 / 5 steps at B = 200 with k row tiles per backward workgroup (DGPRF_RT_PER_GROUP, row-group
# kernel: ceil(13 / k) gW partial rows instead of 13).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=${OUT:-gpurun_out/rpg}
mkdir -p $OUT && export TMPDIR=/tmp
for c in 4 5 2; do
  for k in 1 2 3 4 7; do
    if [ $k = 1 ]; then unset DGPRF_RT_PER_GROUP; else export DGPRF_RT_PER_GROUP=$k; fi
    timeout -k 10 120 python scripts/diag/step_graph.py $c 200 1000 > $OUT/c${c}_k$k.log 2>&1 || exit $?
    echo -n "k=$k "; grep config $OUT/c${c}_k$k.log
  done
done
