"""Summarise rocprofv3 --pmc CSVs: mean counter value per dispatch for each kernel.

  python scripts/pmc_summary.py OUT.csv DIR [DIR ...]
Every *counter_collection.csv under the DIRs is read; rows are (kernel, counter, value, dispatch).
"""
import csv
import re
import glob
import os
import sys
from collections import defaultdict


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    acc = defaultdict(float)
    disp = defaultdict(set)
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f, newline="") as fh:
                for row in csv.DictReader(fh):
                    k = row.get("Kernel_Name") or row.get("Kernel-Name") or row.get("KernelName")
                    c = row.get("Counter_Name") or row.get("Counter-Name")
                    v = row.get("Counter_Value") or row.get("Counter-Value")
                    i = row.get("Dispatch_Id") or row.get("Dispatch-Id") or row.get("Correlation_Id")
                    if not (k and c and v):
                        continue
                    short = k.replace("void ", "").replace("(anonymous namespace)::", "")
                    short = re.sub(r"\w+::", "", short.split("(")[0])
                    acc[(short, c)] += float(v)
                    disp[(short, c)].add(i)
    with open(out, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["kernel", "counter", "mean_per_dispatch", "dispatches"])
        for (k, c) in sorted(acc):
            n = max(len(disp[(k, c)]), 1)
            w.writerow([k, c, f"{acc[(k, c)] / n:.6g}", n])
    print(open(out).read())


if __name__ == "__main__":
    main()
