#!/bin/bash
# Round evidence in one gpurun call, in the order the bench line needs it:
#  1. rocprofv3 kernel-trace summary of the bench (-> profiles/$TAG/kernel_stats_bench.csv),
#  2. HBM-traffic PMC passes (FETCH_SIZE / WRITE_SIZE in separate passes, no trace domains)
#     (-> profiles/$TAG/pmc_traffic_summary.csv, pmc_traffic.json),
#  3. the plain bench, which reads 1 and 2 as its cross-check fields (-> bench_plain.json).
# Everything is also written under gpurun_out/prof_$TAG (the only part that comes back).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD
TAG=${TAG:-r06}
O=$R/gpurun_out/prof_$TAG
P=$R/profiles/$TAG
mkdir -p $O $P
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run \
  -- python3 $R/bench.py --steps 2000 --no-cpu-baseline --multi-chains 0 --full-bayes-steps 0 --other-configs 0 --b-sweep 0 --eager-calls 0 --driver-epochs 0 \
  > $O/bench_under_rocprof.json 2> $O/kt.err || exit $?
cp "$(find $O/kt -name '*kernel_stats.csv' | head -1)" $P/kernel_stats_bench.csv || exit 2
cp $O/bench_under_rocprof.json $P/bench_under_rocprof.json || exit 2
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pf -o run \
  -- python3 $R/bench.py --steps 100 --warmup 20 --pred-samples 60 --no-cpu-baseline --multi-chains 0 \
  --full-bayes-steps 0 --other-configs 0 --b-sweep 0 --eager-calls 0 --driver-epochs 0 --profile-reps 20 > $O/pf.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pw -o run \
  -- python3 $R/bench.py --steps 100 --warmup 20 --pred-samples 60 --no-cpu-baseline --multi-chains 0 \
  --full-bayes-steps 0 --other-configs 0 --b-sweep 0 --eager-calls 0 --driver-epochs 0 --profile-reps 20 > $O/pw.log 2>&1 || exit $?
python3 $R/scripts/pmc_summary.py $P/pmc_traffic_summary.csv $O/pf $O/pw > /dev/null || exit 2
python3 $R/scripts/pmc_traffic_json.py $P > /dev/null || exit 2
cp $P/* $O/
cd $R
timeout -k 10 500 python3 bench.py ${BENCH_ARGS} > $O/bench_plain.json 2> $O/bench_plain.err || exit $?
cp $O/bench_plain.json $P/bench_plain.json
tail -c 600 $O/bench_plain.json
