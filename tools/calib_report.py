"""Summarise a tools/calib.sh run (gpurun_out/calib) into profiles/<tag>/calib.json (dev tool).

For each table size: the HIP-event rate of tools/gather_calib's three kernels (run_<MB>.txt) and
the raw rocprofv3 FETCH_SIZE / WRITE_SIZE per launch (KB, summed over the dispatch's counter
instances, divided by the kernel's dispatch count: k_stream runs twice, warm-up + timed), turned
into reported bytes per access.  The reference point is k_stream: a coalesced 16-B-per-lane read
of T bytes, whose FETCH_SIZE is T/2 on gfx950 (MI355X_MICROARCH.md, HBM section).

    python tools/calib_report.py [gpurun_out/calib] [profiles/r03_calib]
"""
import glob
import json
import os
import re
import sqlite3
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/calib"
dst = sys.argv[2] if len(sys.argv) > 2 else "profiles/r03_calib"


def pmc(d):
    db = sqlite3.connect(glob.glob(os.path.join(d, "**", "*.db"), recursive=True)[0])
    tot, disp = {}, {}
    for n, c, v, did in db.execute("select kernel_name, counter_name, value, dispatch_id from counters_collection"):
        m = re.search(r"k_(gather|scatter|stream|build)", n)
        if not m:
            continue
        k = m.group(0)
        tot[k] = tot.get(k, 0.0) + v
        disp.setdefault(k, set()).add(did)
    return {k: tot[k] / len(disp[k]) for k in tot}


out = {"tool": "tools/gather_calib.hip", "script": "tools/calib.sh", "unit_pmc": "KB per launch (raw)", "tables": []}
for run in sorted(glob.glob(os.path.join(src, "run_*.txt")), key=lambda p: int(re.search(r"(\d+)", p).group(1))):
    mb = int(re.search(r"run_(\d+)", run).group(1))
    rates = {}
    for line in open(run):
        m = re.match(r"(k_\w+)\s+table \d+ MB\s+\w+ (\d+)\s+([\d.]+) ms\s+([\d.]+)", line)
        if m:
            rates[m.group(1)] = {"accesses": int(m.group(2)), "ms": float(m.group(3)), "rate": float(m.group(4))}
    f, w = pmc(os.path.join(src, f"f_{mb}")), pmc(os.path.join(src, f"w_{mb}"))
    n = rates["k_gather"]["accesses"]
    tb = mb << 20
    out["tables"].append({
        "table_MB": mb,
        "gather_4B_loads_per_s": rates["k_gather"]["rate"] * 1e9,
        "scatter_4B_stores_per_s": rates["k_scatter"]["rate"] * 1e9,
        "stream_GB_per_s": rates["k_stream"]["rate"],
        "stream_fetch_over_bytes": f["k_stream"] * 1024 / tb,
        "gather_fetch_B_per_load_raw": f["k_gather"] * 1024 / n,
        "scatter_write_B_per_store": w["k_scatter"] * 1024 / rates["k_scatter"]["accesses"],
        "gather_fetch_KB": f["k_gather"], "scatter_write_KB": w["k_scatter"], "stream_fetch_KB": f["k_stream"],
    })
# tools/calib2.sh: the read-hash build pattern (k_build) with a per-wave table of 4 / 32 / 128 KB
src2 = src.rstrip("/") + "2"
out["build_pattern"] = []
for run in sorted(glob.glob(os.path.join(src2, "run_*.txt")), key=lambda p: int(re.search(r"run_(\d+)", p).group(1))):
    kb = int(re.search(r"run_(\d+)", run).group(1))
    for line in open(run):
        m = re.match(r"k_build\s+own (\d+) KB per wave\s+updates (\d+)\s+([\d.]+) ms\s+([\d.]+)", line)
        if m:
            n = int(m.group(2))
            f, w = pmc(os.path.join(src2, f"f_{kb}")), pmc(os.path.join(src2, f"w_{kb}"))
            out["build_pattern"].append({"own_KB_per_wave": kb, "updates_per_s": float(m.group(4)) * 1e9,
                                         "fetch_B_per_update_raw": f["k_build"] * 1024 / n,
                                         "write_B_per_update": w["k_build"] * 1024 / n})
os.makedirs(dst, exist_ok=True)
with open(os.path.join(dst, "calib.json"), "w") as fh:
    json.dump(out, fh, indent=1)
for t in out["tables"]:
    print(f"{t['table_MB']:5d} MB  gather {t['gather_4B_loads_per_s']/1e9:5.1f} G/s  {t['gather_fetch_B_per_load_raw']:5.1f} B/load raw"
          f"  scatter {t['scatter_4B_stores_per_s']/1e9:5.1f} G/s  {t['scatter_write_B_per_store']:5.1f} B/store"
          f"  stream {t['stream_GB_per_s']:6.0f} GB/s  fetch/bytes {t['stream_fetch_over_bytes']:.3f}")
for b in out["build_pattern"]:
    print(f"build {b['own_KB_per_wave']:4d} KB/wave  {b['updates_per_s']/1e9:6.1f} G updates/s  fetch {b['fetch_B_per_update_raw']:5.1f} B"
          f"  write {b['write_B_per_update']:5.1f} B per update")
