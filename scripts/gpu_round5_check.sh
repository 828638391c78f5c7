#!/bin/bash
# GPU suite, then (only if green) the A/B of scripts/variants/* against the current library on the
# configs' steps, and a short bench line.  Each GPU step under its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/${TAG:-chk}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  ${PYTEST_ARGS} > $O/pytest_gpu.log 2>&1
rc=$?
tail -15 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
CONFIGS="${AB_CONFIGS:-2 4 5}" REPS=2 STEPS=2000 timeout -k 10 400 bash scripts/ab_variants.sh > $O/ab.log 2>&1 || { cat $O/ab.log; exit 5; }
cat $O/ab.log
timeout -k 10 300 python bench.py --steps 2000 --no-cpu-baseline --other-configs 0 --b-sweep 0 \
  --multi-chains 0 --full-bayes-steps 0 --eager-calls 0 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 6; }
python3 -c "
import json; l=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('value', l['value'], 'pred/s', l['predictive_samples_per_s'])
r=l['roofline_predictive']; print('pred', r['avg_us_per_sample'], r['frac'], r['single_sample'])
print('roof', l['roofline']['kernel'], l['roofline']['live_in_kernel_us'], l['roofline']['step_kernel_us'])"
