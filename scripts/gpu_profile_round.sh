#!/bin/bash
# Round evidence in one gpurun call: plain bench, rocprofv3 kernel-trace summary of the bench, and
# HBM-traffic PMC passes (FETCH_SIZE / WRITE_SIZE in separate passes, no trace domains).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD
TAG=${TAG:-r04}
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py > $O/bench_plain.json 2> $O/bench_plain.err || exit $?
tail -c 400 $O/bench_plain.json
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run \
  -- python3 $R/bench.py --steps 2000 --no-cpu-baseline --multi-chains 0 --full-bayes-steps 0 --other-configs 0 --b-sweep 0 \
  > $O/bench_under_rocprof.json 2> $O/kt.err || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pf -o run \
  -- python3 $R/bench.py --steps 100 --warmup 20 --pred-samples 3 --no-cpu-baseline --multi-chains 0 \
  --full-bayes-steps 0 --other-configs 0 --b-sweep 0 --profile-reps 20 > $O/pf.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pw -o run \
  -- python3 $R/bench.py --steps 100 --warmup 20 --pred-samples 3 --no-cpu-baseline --multi-chains 0 \
  --full-bayes-steps 0 --other-configs 0 --b-sweep 0 --profile-reps 20 > $O/pw.log 2>&1 || exit $?
python3 $R/scripts/pmc_summary.py $O/pmc_traffic_summary.csv $O/pf $O/pw > /dev/null
find $O -name "*stats*.csv" | head
