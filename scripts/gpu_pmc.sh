#!/bin/bash
# SQ / LDS / cache counter passes over one command (one rocprofv3 --pmc run per pass, no trace
# domains, each under its own hard time limit), summarised per kernel by scripts/pmc_summary.py.
#   NAME=pred CMD="python3 scripts/prof_predict.py --samples 3" scripts/gpu_pmc.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD
O=$R/gpurun_out/pmc_${NAME:-run}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_VMEM"
i=0
for P in "$P1" "$P2" ${EXTRA_PASSES}; do
  i=$((i + 1))
  timeout -s KILL ${PASS_LIMIT:-120} rocprofv3 --pmc $P --output-format csv -d $O/p$i -o run -- $CMD \
    > $O/p$i.log 2>&1 || exit $?
done
python3 $R/scripts/pmc_summary.py $O/summary.csv $O/p* > /dev/null
cut -c1-160 $O/summary.csv | grep -v "^kernel" | grep -i "${FILTER:-.}" | head -60
