"""Per-kernel sums of one tools/pmc_pass.sh pass (dev tool): python tools/pmc_report.py NAME"""
import glob
import re
import sqlite3
import sys

name = sys.argv[1]
db = sqlite3.connect(glob.glob(f"gpurun_out/pmc_{name}/**/*.db", recursive=True)[0])
res, calls = {}, {}
for n, c, v in db.execute("select kernel_name, counter_name, value from counters_collection"):
    m = re.match(r"(?:void )?([\w:]+(?:<[^>]*>)?)", n)
    n = m.group(1) if m else n
    res.setdefault(n, {}).setdefault(c, 0)
    res[n][c] += v
for n, d in sorted(res.items()):
    if "k_" not in n:
        continue
    print(n[:32], " ".join(f"{c}={v:.4g}" for c, v in sorted(d.items())))
