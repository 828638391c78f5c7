#!/bin/bash
# One SQ PMC pass (8 counters, no trace domains) over the config-4 diagnostic; per-kernel means
# of the step-size A_1 GEMM (B = 200) and the other config-4 step kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD; export TMPDIR=/tmp; O=$R/gpurun_out/pmc4
mkdir -p $O
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --output-format csv \
  -d $O -o run -- python3 $R/scripts/diag/prof_config.py 4 > $O/run.log 2>&1 || exit $?
python3 - "$O" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    k = (r["Kernel_Name"][:60], r.get("Grid_Size", ""))
    acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(acc.items(), key=lambda kv: -sum(kv[1].get("SQ_WAVE_CYCLES", [0]))):
    m = {c: sum(v) / len(v) for c, v in d.items()}
    wc = m.get("SQ_WAVE_CYCLES", 1) or 1
    print(k, "n", len(d.get("SQ_WAVES", [])), "waves", int(m.get("SQ_WAVES", 0)),
          "wave_cyc(q)", int(wc), "wait_any %.2f" % (m.get("SQ_WAIT_ANY", 0) / wc),
          "wait_inst %.2f" % (m.get("SQ_WAIT_INST_ANY", 0) / wc),
          "active %.2f" % (m.get("SQ_ACTIVE_INST_ANY", 0) / wc),
          "wait_lds %.2f" % (m.get("SQ_WAIT_INST_LDS", 0) / wc),
          "mfma_busy", int(m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)), "busy", int(m.get("SQ_BUSY_CYCLES", 0)))
PY
