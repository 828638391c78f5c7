"""profiles/<tag>/pmc_traffic_summary.csv -> pmc_traffic.json (bytes per dispatch, FETCH_SIZE doubled
per MI355X_MICROARCH.md §HBM) for bench.py's roofline `traffic`.

  python scripts/pmc_traffic_json.py profiles/r01b
"""
import csv
import json
import os
import sys

d = sys.argv[1]
rows = list(csv.DictReader(open(os.path.join(d, "pmc_traffic_summary.csv"))))
out = {"source": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes) over "
                 "`bench.py --steps 100 --warmup 20 --pred-samples 3` (scripts/gpu_profile_round.sh); "
                 "FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM (gfx950 tallies 128-B requests at "
                 "64 B); both counters include Infinity-Cache hits",
       "unit": "bytes per dispatch", "kernels": {}}
for r in rows:
    k = r["kernel"]
    if not k.startswith(("k_step", "k_forward", "k_gather")):
        continue
    e = out["kernels"].setdefault(k, {})
    v = float(r["mean_per_dispatch"]) * 1024.0  # rocprofv3 reports KB
    e["dispatches"] = int(r["dispatches"])
    if r["counter"] == "FETCH_SIZE":
        e["fetch_raw"] = v
        e["fetch_corrected"] = 2 * v
    else:
        e["write"] = v
for e in out["kernels"].values():
    e["traffic"] = e.get("fetch_corrected", 0) + e.get("write", 0)
json.dump(out, open(os.path.join(d, "pmc_traffic.json"), "w"), indent=1)
print(json.dumps({k: round(v["traffic"]) for k, v in out["kernels"].items()}, indent=1))
