"""Per-kernel summary of a rocprofv3 --kernel-trace database (rocpd sqlite, ROCm 7.2 default output)
or kernel_trace.csv: calls, average / total duration, grid and registers, grouped by kernel name
(template arguments kept) and grid size.

  python scripts/kt_summary.py <kt_results.db | kernel_trace.csv> [--csv out.csv] [--match SUBSTR]
"""
import argparse
import csv
import os
import re
import sqlite3
import sys


def short(name):
    name = name.replace("void ", "").replace("(anonymous namespace)::", "").replace("dgprf_sk::", "")
    return re.sub(r"\(.*\)$", "", name)


def rows_db(path):
    c = sqlite3.connect(path)
    q = ("select name, duration, grid_x, grid_y, grid_z, workgroup_x, lds_size, vgpr_count, "
         "accum_vgpr_count, sgpr_count, scratch_size from kernels")
    for r in c.execute(q):
        yield {"name": r[0], "dur": r[1], "grid": (r[2], r[3], r[4]), "wg": r[5], "lds": r[6],
               "vgpr": r[7], "agpr": r[8], "sgpr": r[9], "scratch": r[10]}


def rows_csv(path):
    with open(path) as fh:
        for r in csv.DictReader(fh):
            yield {"name": r["Kernel_Name"], "dur": int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                   "grid": (int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"])),
                   "wg": int(r["Workgroup_Size_X"]), "lds": int(r.get("LDS_Block_Size", 0) or 0),
                   "vgpr": int(r.get("VGPR_Count", 0) or 0), "agpr": int(r.get("Accum_VGPR_Count", 0) or 0),
                   "sgpr": int(r.get("SGPR_Count", 0) or 0), "scratch": int(r.get("Scratch_Size", 0) or 0)}


def summarize(path, match=None):
    it = rows_db(path) if path.endswith(".db") else rows_csv(path)
    agg = {}
    for r in it:
        n = short(r["name"])
        if match and match not in n:
            continue
        key = (n, r["grid"])
        a = agg.setdefault(key, {"calls": 0, "tot": 0, "min": None, "max": 0, "wg": r["wg"],
                                 "lds": r["lds"], "vgpr": r["vgpr"], "agpr": r["agpr"],
                                 "sgpr": r["sgpr"], "scratch": r["scratch"]})
        a["calls"] += 1
        a["tot"] += r["dur"]
        a["min"] = r["dur"] if a["min"] is None else min(a["min"], r["dur"])
        a["max"] = max(a["max"], r["dur"])
    return agg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--csv")
    ap.add_argument("--match")
    args = ap.parse_args()
    agg = summarize(args.path, args.match)
    out = []
    for (n, grid), a in sorted(agg.items(), key=lambda kv: -kv[1]["tot"]):
        out.append({"Name": n, "Grid": "x".join(map(str, grid)), "Workgroup": a["wg"],
                    "Calls": a["calls"], "AverageNs": round(a["tot"] / a["calls"], 1),
                    "MinNs": a["min"], "MaxNs": a["max"], "TotalDurationNs": a["tot"],
                    "LDS": a["lds"], "VGPR": a["vgpr"], "AGPR": a["agpr"], "SGPR": a["sgpr"],
                    "Scratch": a["scratch"]})
    if args.csv:
        with open(args.csv, "w", newline="") as fh:
            w = csv.DictWriter(fh, fieldnames=list(out[0].keys()))
            w.writeheader()
            w.writerows(out)
    for o in out[:40]:
        print(f"{o['AverageNs'] / 1e3:9.2f} us x{o['Calls']:6d}  grid {o['Grid']:>14s} wg {o['Workgroup']:4d} "
              f"v{o['VGPR']}/a{o['AGPR']} lds {o['LDS']:6d} scr {o['Scratch']}  {o['Name'][:110]}")


if __name__ == "__main__":
    sys.exit(main())
