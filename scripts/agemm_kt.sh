#!/bin/bash
# Kernel-trace of the config-4 step/predictive diagnostic: per-kernel average durations.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD; export TMPDIR=/tmp
for lib in ${LIBS:-dgp-rf-mcmc_amd/dgprf/libdgprf.so}; do
  t=$(basename $lib .so)
  cd /tmp && DGPRF_LIB=$R/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $R/gpurun_out/kt4_$t -o run -- python3 $R/scripts/diag/prof_config.py 4 > $R/gpurun_out/kt4_$t.log 2>&1 || exit $?
  f=$(find $R/gpurun_out/kt4_$t -name "*kernel_stats.csv" | head -1)
  echo "== $t"; cut -d, -f1-8 "$f" | cut -c1-200 | head -14
done
