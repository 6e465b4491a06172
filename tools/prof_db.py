#!/usr/bin/env python3
"""Summaries of a rocprofv3 kernel-trace database (rocpd SQLite, ROCm 7):

    python tools/prof_db.py DB [--min-grid N] [--csv OUT]

Per kernel: calls, total and average duration over every dispatch, and over the "main" dispatches
(grid >= N workgroups: one launch per phase per chunk; the overflow re-runs of a few reads are
small launches that would dilute the average the bench's roofline compares with).  Also the idle
time of the GPU between consecutive dispatches (host work between chunks), per gap size.
"""
import argparse
import csv
import re
import sqlite3


def short(name):
    m = re.match(r"(?:void )?([\w:]+(?:<[^>]*>)?)", name)
    return m.group(1) if m else name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--min-grid", type=int, default=1000)
    ap.add_argument("--csv", default=None)
    a = ap.parse_args()
    db = sqlite3.connect(a.db)
    rows = list(db.execute("select name, start, end, duration, grid_x, workgroup_x from kernels order by start"))
    per = {}
    for name, s, e, d, gx, wx in rows:
        k = short(name)
        p = per.setdefault(k, {"calls": 0, "total_ns": 0, "main_calls": 0, "main_ns": 0})
        p["calls"] += 1
        p["total_ns"] += d
        if gx // max(1, wx) >= a.min_grid:
            p["main_calls"] += 1
            p["main_ns"] += d
    tot = sum(p["total_ns"] for p in per.values())
    out = []
    for k, p in sorted(per.items(), key=lambda kv: -kv[1]["total_ns"]):
        out.append({"kernel": k, "calls": p["calls"], "total_ms": round(p["total_ns"] / 1e6, 3),
                    "avg_ms": round(p["total_ns"] / p["calls"] / 1e6, 4), "pct": round(100 * p["total_ns"] / tot, 2),
                    "main_calls": p["main_calls"],
                    "main_avg_ms": round(p["main_ns"] / p["main_calls"] / 1e6, 4) if p["main_calls"] else None})
    for r in out:
        print(f"{r['kernel'][:34]:34s} calls {r['calls']:5d} total {r['total_ms']:10.2f} ms avg {r['avg_ms']:9.4f} "
              f"({r['pct']:5.2f}%)  main: {r['main_calls']} x {r['main_avg_ms']} ms")
    # idle gaps between dispatches (serial stream: end of one to the start of the next)
    gaps = []
    last_end = None
    for name, s, e, d, gx, wx in rows:
        if last_end is not None and s > last_end:
            gaps.append((s - last_end, short(name)))
        last_end = e if last_end is None else max(last_end, e)
    if gaps:
        span = rows[-1][2] - rows[0][1]
        big = [g for g in gaps if g[0] > 100_000]
        print(f"span {span / 1e6:.1f} ms, busy {tot / 1e6:.1f} ms (kernels may overlap), idle gaps {sum(g[0] for g in gaps) / 1e6:.1f} ms "
              f"in {len(gaps)} gaps; {len(big)} gaps > 0.1 ms sum {sum(g[0] for g in big) / 1e6:.1f} ms")
        by = {}
        for g, k in big:
            by.setdefault(k, [0, 0.0])
            by[k][0] += 1
            by[k][1] += g / 1e6
        for k, (n, ms) in sorted(by.items(), key=lambda kv: -kv[1][1])[:8]:
            print(f"  before {k[:34]:34s} {n:4d} gaps {ms:8.1f} ms")
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(out[0].keys()))
            w.writeheader()
            w.writerows(out)


if __name__ == "__main__":
    main()
