#!/bin/bash
# Per-kernel durations of the config 4 / 5 steps at B = 200 (rocprofv3 kernel trace of
# graph-replayed steps) and the per-kernel event times of dgprf_profile_step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD; OUT=$R/gpurun_out/kt45
mkdir -p $OUT && export TMPDIR=/tmp
for c in 4 5; do
  timeout -k 10 200 python scripts/diag/prof_config.py $c > $OUT/prof_c$c.log 2>&1 || exit $?
  cat $OUT/prof_c$c.log
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt$c -o run \
     -- python3 $R/scripts/diag/step_graph.py $c 200 1000 > $OUT/kt$c.log 2>&1) || exit $?
  f=$(find $OUT/kt$c -name "*kernel_stats.csv" | head -1)
  cut -d, -f1-4 "$f" | cut -c1-150 | head -16
done
