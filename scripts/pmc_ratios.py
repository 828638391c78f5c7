"""Per-kernel ratios from a scripts/pmc_summary.py CSV (the two SQ passes of scripts/gpu_pmc.sh):
fraction of wave cycles waiting on memory / barriers (SQ_WAIT_ANY), on instruction dependencies
(SQ_WAIT_INST_ANY) and issuing (SQ_ACTIVE_INST_ANY); MFMA pipe utilisation =
SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs); waves per dispatch; LDS bank
conflicts per LDS-active cycle.

  python scripts/pmc_ratios.py SUMMARY.csv [...]
"""
import csv
import sys
from collections import defaultdict


def ratios(path):
    d = defaultdict(dict)
    with open(path) as fh:
        for r in csv.DictReader(fh):
            d[r["kernel"]][r["counter"]] = float(r["mean_per_dispatch"])
    out = []
    for k, c in sorted(d.items()):
        wc = c.get("SQ_WAVE_CYCLES")
        if not wc:
            continue
        ga = c.get("GRBM_GUI_ACTIVE", 0.0)
        out.append((k, c.get("SQ_WAIT_ANY", 0) / wc, c.get("SQ_WAIT_INST_ANY", 0) / wc,
                    c.get("SQ_ACTIVE_INST_ANY", 0) / wc,
                    c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (1024 * ga / 8) if ga else float("nan"),
                    c.get("SQ_WAVES", 0), c.get("SQ_LDS_BANK_CONFLICT", 0) /
                    max(c.get("SQ_LDS_IDX_ACTIVE", 0), 1.0), ga / 8))
    return out


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print(f"== {p}")
        print(f"  {'kernel':58s} wait  dep   issue mfma  waves/disp ldsconf gpu_cycles")
        for k, w, dep, iss, mf, wv, lc, cyc in ratios(p):
            print(f"  {k[:58]:58s} {w:.2f}  {dep:.2f}  {iss:.2f}  {mf:.3f} {wv:10.0f} {lc:7.2f} {cyc:10.0f}")
