"""Per-process phases of a rocprofv3 kernel trace (`--kernel-trace --output-format csv`): for each
trace file, the runs of step kernels grouped by kind (W-only vs full-Bayes backward instances, the
64-chain launches), with the median kernel duration and the median gap between consecutive
dispatches of the phase.  Used for the two-ranks-on-one-GPU rehearsal.

  python scripts/kt_phases.py gpurun_out/kt_b2
"""
import csv
import glob
import os
import statistics
import sys


def phase_of(name, grid_z):
    if "k_step_bwd<" in name:
        fb = name.split("k_step_bwd<")[1].split(">")[0].split(",")[4].strip() == "true"
        return ("fb" if fb else "w") + ("64" if grid_z > 1 else "")
    if "k_step_fwd<" in name or "k_step_update<" in name:
        return "step" + ("64" if grid_z > 1 else "")
    return None


def main(d):
    for f in sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)):
        rows = list(csv.DictReader(open(f)))
        by_tid = {}
        for r in rows:
            by_tid.setdefault(r["Thread_Id"], []).append(r)
        print(f)
        for tid, rs in by_tid.items():
            rs.sort(key=lambda r: int(r["Start_Timestamp"]))
            # phases of consecutive backward kernels of one kind; fwd / update join the current one
            cur, runs = None, []
            for r in rs:
                p = phase_of(r["Kernel_Name"], int(r["Grid_Size_Z"]))
                if p is None:
                    continue
                if p.startswith("step"):
                    if cur is not None:
                        runs[-1][1].append(r)
                    continue
                if p != cur:
                    runs.append((p, []))
                    cur = p
                runs[-1][1].append(r)
            for p, rr in runs:
                if len(rr) < 50:
                    continue
                dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rr]
                gap = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3
                       for a, b in zip(rr[:-1], rr[1:])]
                span = (int(rr[-1]["End_Timestamp"]) - int(rr[0]["Start_Timestamp"])) / 1e3
                print(f"  thread {tid} phase {p:5s} kernels {len(rr):6d}  median dur {statistics.median(dur):7.2f} us"
                      f"  median gap {statistics.median(gap):7.2f} us  p90 gap {sorted(gap)[int(0.9 * len(gap))]:8.2f}"
                      f"  span {span / 1e3:8.2f} ms")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/kt_b2")
