#!/bin/bash
# One GPU-box pass: GPU tests, then the driver-shaped bench (--steps 20 --warmup 5) and the default
# bench.  Each GPU step has its own time limit; a crash, abort or timeout ends the script there
# (pytest's rc 1 = failed assertions still lets the benches run).
set -u
mkdir -p gpurun_out
out=gpurun_out/${TAG:-r02}
mkdir -p "$out"
timeout -k 10 ${PYTEST_LIMIT:-1000} python -u -m pytest tests -m gpu -v --timeout 300 \
    --timeout-method thread ${PYTEST_ARGS:-} > "$out/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$out/pytest_gpu.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
[ "${NO_BENCH:-0}" = 1 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > "$out/bench_driver.json" 2> "$out/bench_driver.err" || { echo "bench_driver rc=$?"; exit 2; }
cat "$out/bench_driver.json"
timeout -k 10 500 python -u bench.py > "$out/bench_default.json" 2> "$out/bench_default.err" || { echo "bench_default rc=$?"; exit 2; }
cat "$out/bench_default.json"
exit $rc
