#!/bin/bash
# PMC passes over the predictive forward (separate passes; no trace domains with --pmc).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/pmc_pred
mkdir -p $O
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d $O/p1 -o run -- python3 $R/scripts/prof_predict.py --samples 3 > $O/p1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_VMEM --output-format csv -d $O/p2 -o run -- python3 $R/scripts/prof_predict.py --samples 3 > $O/p2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/scripts/prof_predict.py --samples 20 > $O/kt.log 2>&1
