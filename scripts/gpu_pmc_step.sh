#!/bin/bash
# SQ / LDS counters of the step kernels (config 2 at minibatch B, graph-replayed steps), separate
# passes:  B=8192 bash scripts/gpu_pmc_step.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD
cd /tmp && export TMPDIR=/tmp
B=${B:-8192}
O=$R/gpurun_out/pmc_step_$B
mkdir -p $O
CMD="python3 $R/scripts/diag/step_graph.py 2 $B 200"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d $O/p1 -o run -- $CMD > $O/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_VMEM --output-format csv -d $O/p2 -o run -- $CMD > $O/p2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/p3 -o run -- $CMD > $O/p3.log 2>&1 || exit $?
python3 $R/scripts/pmc_summary.py $O/summary.csv $O/p1 $O/p2 $O/p3 > /dev/null
grep -i "step_bwd\|forward_rows\|step_update" $O/summary.csv | cut -c1-200
