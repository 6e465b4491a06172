"""Condense rocprofv3 results (tools/profile.sh) into committed summaries under profiles/.

  python tools/prof_summary.py <round-tag> [workload] [reads]

Writes profiles/<tag>/kernel_stats.csv (per-kernel calls / total / average duration, the
--kernel-trace --stats pass), profiles/<tag>/pmc.csv (per-kernel average FETCH_SIZE and
WRITE_SIZE per dispatch, separate passes) and profiles/traffic.json (HBM bytes per launch of
the dominant kernel: 2 x FETCH_SIZE + WRITE_SIZE, the gfx950 correction of
/opt/skills/guides/MI355X_MICROARCH.md §HBM, which bench.py reports as roofline.traffic; and
FETCH_SIZE + WRITE_SIZE, the reading tools/gather_calib.hip calibrates for random 4-B accesses,
reported as roofline.traffic_calibrated).
"""
import csv
import json
import os
import re
import sqlite3
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")


def short(name):
    m = re.match(r"(?:void )?([\w:]+(?:<[^>]*>)?)", name)
    return m.group(1).replace(", false", "").replace(", true", "*") if m else name[:60]


def db(d):
    for f in os.listdir(os.path.join(OUT, d)):
        if f.endswith(".db"):
            return sqlite3.connect(os.path.join(OUT, d, f))
    raise FileNotFoundError(d)


def main():
    tag = sys.argv[1]
    workload = sys.argv[2] if len(sys.argv) > 2 else "C1-proxy-56Mbp"
    reads = int(sys.argv[3]) if len(sys.argv) > 3 else 100000
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    kt = db("prof_kt")
    rows = kt.execute("select name, count(*), sum(duration), avg(duration) from kernels group by name "
                      "order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows)
    rows = [(n, c, t, a, 100.0 * t / tot) for n, c, t, a in rows]
    with open(os.path.join(dst, "kernel_stats.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_ns", "avg_ns", "percent"])
        for n, c, t, a, p in rows:
            w.writerow([short(n), c, int(t), int(a), round(p, 3)])
    pmc = {}
    for d, cn in (("prof_fetch", "FETCH_SIZE"), ("prof_write", "WRITE_SIZE")):
        for n, v in db(d).execute("select kernel_name, value from counters_collection where counter_name = ?", (cn,)):
            pmc.setdefault(short(n), {}).setdefault(cn, []).append(v)
    with open(os.path.join(dst, "pmc.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "dispatches", "avg_FETCH_SIZE_KB", "avg_WRITE_SIZE_KB", "hbm_bytes_per_launch_corrected"])
        for k, v in sorted(pmc.items()):
            fs = sum(v.get("FETCH_SIZE", [0])) / max(1, len(v.get("FETCH_SIZE", [])))
            ws = sum(v.get("WRITE_SIZE", [0])) / max(1, len(v.get("WRITE_SIZE", [])))
            w.writerow([k, len(v.get("FETCH_SIZE", [])), round(fs, 1), round(ws, 1), int((2 * fs + ws) * 1024)])
    top = short(rows[0][0])
    v = pmc.get(top, {})
    fs = sum(v.get("FETCH_SIZE", [0])) / max(1, len(v.get("FETCH_SIZE", [])))
    ws = sum(v.get("WRITE_SIZE", [0])) / max(1, len(v.get("WRITE_SIZE", [])))
    tj = {"workload": workload, "reads": reads, "kernel": top, "tag": tag,
          "avg_duration_ns": int(rows[0][3]),
          "fetch_size_kb_per_launch": round(fs, 1), "write_size_kb_per_launch": round(ws, 1),
          "hbm_bytes_per_launch": int((2 * fs + ws) * 1024),
          "correction": "2 x FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE counts half of 128-B requests)",
          # random 4-B gathers report one 64-B unit each (profiles/r03_calib: 49-56 G loads/s would
          # be 6.3-7.2 TB/s at 128 B, above the 5.8 TB/s streaming rate), scattered stores 32 B
          "hbm_bytes_per_launch_calibrated": int((fs + ws) * 1024),
          "calibration": "FETCH_SIZE + WRITE_SIZE: the random-access reading of profiles/r03_calib/calib.json"}
    with open(os.path.join(ROOT, "profiles", "traffic.json"), "w") as f:
        json.dump(tj, f, indent=1)
    print(json.dumps(tj, indent=1))
    for r in rows[:12]:
        print(f"{short(r[0]):28s} calls={r[1]:4d} avg={r[3] / 1e6:9.3f} ms  {r[4]:5.1f}%")


if __name__ == "__main__":
    main()
