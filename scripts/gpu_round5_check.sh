#!/bin/bash
# GPU suite, then (only if green) config steps (config 4 with and without the resident first-layer
# projection), the predictive forms, and a bench line with the other configs.  Each GPU step under
# its own time limit; the first failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/${TAG:-chk}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  ${PYTEST_ARGS} > $O/pytest_gpu.log 2>&1
rc=$?
tail -15 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
{
  for c in ${CONFIGS:-2 4 5}; do
    timeout -k 10 200 python3 scripts/diag/step_graph.py $c 200 2000 || exit $?
  done
  DGPRF_DIAG_NO_A1=1 timeout -k 10 200 python3 scripts/diag/step_graph.py 4 200 2000 || exit $?
  timeout -k 10 120 python3 scripts/prof_predict.py --samples 20 || exit $?
  timeout -k 10 120 python3 scripts/prof_predict.py --samples 20 --pairs || exit $?
} > $O/steps.log 2>&1 || { cat $O/steps.log; exit 5; }
grep -v amdgpu.ids $O/steps.log
timeout -k 10 400 python bench.py --steps 2000 --no-cpu-baseline --b-sweep 0 --other-steps 500 \
  --multi-chains 0 --full-bayes-steps 0 --eager-calls 0 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 6; }
python3 -c "
import json; l=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('value', l['value'], 'pred/s', l['predictive_samples_per_s'])
r=l['roofline_predictive']; print('pred', r['avg_us_per_sample'], r['frac'], r['single_sample'])
for k, v in l['other_configs'].items(): print(k, v['us_per_step'], v['step_mfma_frac'], v['predictive_samples_per_s'], v['predictive_mfma_frac'], v.get('predictive_finalize_ms'), v['a1_gemm'])"
