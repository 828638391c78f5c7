O=gpurun_out/r03h; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 200 python scripts/diag/step_graph.py 2 8192,65536 1000 > $O/base.log 2>&1 || exit $?
DGPRF_DBG_RW=8 timeout -k 10 200 python scripts/diag/step_graph.py 2 8192,65536 1000 > $O/one.log 2>&1 || exit $?
grep -h config $O/base.log $O/one.log
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/kt_base -o kt -- python scripts/diag/step_graph.py 2 8192 200 > $O/ktb.log 2>&1 || exit $?
DGPRF_DBG_RW=8 timeout -k 10 200 rocprofv3 --kernel-trace -d $O/kt_one -o kt -- python scripts/diag/step_graph.py 2 8192 200 > $O/kto.log 2>&1 || exit $?
