"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks (stdin): one line per kernel with
VGPRs, spills, LDS and occupancy.  Build-time diagnostic only."""
import re
import subprocess
import sys

cur, rows = None, []
for line in sys.stdin:
    m = re.search(r"remark: \s*(\w[\w \[\]/]*?): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2)
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True,
                       text=True).stdout.split("\n")
for r, n in zip(rows, names):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "").replace("dgprf_sk::", "")
    if n.endswith(")"):  # drop the parameter list (match the closing parenthesis)
        depth = 0
        for i in range(len(n) - 1, -1, -1):
            depth += {")": 1, "(": -1}.get(n[i], 0)
            if depth == 0:
                n = n[:i]
                break
    print(f"v{r.get('VGPRs', '?'):>4} a{r.get('AGPRs', '?'):>3} spill {r.get('VGPRs Spill', '?'):>4} "
          f"lds {r.get('LDS Size [bytes/block]', '?'):>6} occ {r.get('Occupancy [waves/SIMD]', '?'):>2}  {n}")
