#!/usr/bin/env python3
"""Reports over the profiling output of tools/gpu_session.sh (dev tool; runs anywhere).

  python tools/prof_report.py kernels DB [--min-grid N] [--csv OUT]
        per kernel of a rocprofv3 --kernel-trace database: calls, total / average duration over
        every dispatch and over the "main" dispatches (grid >= N workgroups: one launch per phase
        per chunk; an overflow re-run of a few reads is a small launch that would dilute the
        average the bench's roofline compares with); the GPU's idle gaps between dispatches
  python tools/prof_report.py pmc DIR
        per-kernel sums of every counter of one rocprofv3 --pmc pass (gpu_session.sh pmc / sq steps)
  python tools/prof_report.py sq DIR
        VALU lane utilisation, issue and wait fractions per kernel from the SQ counters of the
        gpu_session.sh sq step (SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU), ...)
  python tools/prof_report.py wave BENCH_JSON
        the wave-clock split of the scoring and seeding phases (work_counters t_* of bench.py's
        stats runs: read-hash build / matching / list walks / windows / DP scans; seeding map batches)
  python tools/prof_report.py timeline FILE [READS_FQ]
        the per-read phase timeline a DSB_TL build writes with DSB_WAVE_DBG=4096 DSB_TIMELINE=FILE:
        per phase the active reads, span, duration distribution, the slowest reads, running waves
"""
import argparse
import csv
import glob
import gzip
import json
import re
import sqlite3


def short(name):
    m = re.match(r"(?:void )?([\w:]+(?:<[^>]*>)?)", name)
    return m.group(1) if m else name


def _db(path):
    dbs = [path] if path.endswith(".db") else glob.glob(f"{path}/**/*.db", recursive=True)
    if not dbs:
        raise SystemExit(f"no rocprofv3 database at {path}")
    return sqlite3.connect(dbs[0])


def cmd_kernels(a):
    db = _db(a.db)
    rows = list(db.execute("select name, start, end, duration, grid_x, workgroup_x from kernels order by start"))
    per = {}
    for name, s, e, d, gx, wx in rows:
        p = per.setdefault(short(name), {"calls": 0, "total_ns": 0, "main_calls": 0, "main_ns": 0})
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
    gaps, last_end = [], None
    for name, s, e, d, gx, wx in rows:
        if last_end is not None and s > last_end:
            gaps.append((s - last_end, short(name)))
        last_end = e if last_end is None else max(last_end, e)
    if gaps:
        span = rows[-1][2] - rows[0][1]
        big = [g for g in gaps if g[0] > 100_000]
        print(f"span {span / 1e6:.1f} ms, busy {tot / 1e6:.1f} ms (kernels may overlap), idle gaps "
              f"{sum(g[0] for g in gaps) / 1e6:.1f} ms in {len(gaps)} gaps; {len(big)} gaps > 0.1 ms sum "
              f"{sum(g[0] for g in big) / 1e6:.1f} ms")
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(out[0].keys()))
            w.writeheader()
            w.writerows(out)


def _counters(path):
    res = {}
    for n, c, v in _db(path).execute("select kernel_name, counter_name, value from counters_collection"):
        res.setdefault(short(n), {}).setdefault(c, 0)
        res[short(n)][c] += v
    return res


def cmd_pmc(a):
    for n, d in sorted(_counters(a.dir).items()):
        if "k_" in n:
            print(n[:32], " ".join(f"{c}={v:.4g}" for c, v in sorted(d.items())))


def cmd_sq(a):
    for n, d in _counters(a.dir).items():
        if "k_" not in n:
            continue
        util = d["SQ_THREAD_CYCLES_VALU"] / max(1, d["SQ_ACTIVE_INST_VALU"] * 64)
        print(f"{n[:24]:24s} valu_util={util:.3f} insts_valu={d['SQ_INSTS_VALU']:.3g} "
              f"vmem_rd={d['SQ_INSTS_VMEM_RD']:.3g} issue={d['SQ_ACTIVE_INST_ANY'] / max(1, d['SQ_WAVE_CYCLES']):.3f} "
              f"wait={d['SQ_WAIT_INST_ANY'] / max(1, d['SQ_WAVE_CYCLES']):.3f}")


def cmd_wave(a):
    d = json.load(open(a.bench_json))
    print(d["value"], d["phase_ms_classA"])
    ph = d["work_counters"]["phases"]
    n = max(1, d["config"].get("reads_per_rank", 100000))
    c = ph["delA"]
    tot = c["t_all"] or 1
    print("delA clocks", {k: round(c[k] / tot, 3) for k in ("t_build", "t_match", "t_mprobe", "t_mwalk", "t_win",
                                                             "t_dpm", "t_dps", "t_fill", "t_comb")})
    for p in ("fast0", "slow0"):
        c = ph[p]
        tot = c["t_mem"] or 1
        print(p, "map batches %.3f of the state machine's clocks (map prefix/suffix %.3f, REF_POS items %.3f)"
              % (c["t_map"] / tot, c["t_build"] / tot, c["t_match"] / tot))
    c = ph["fast0"]
    print("fast0 trips/read %.1f  map trips/read %.1f  lanes per map trip %.1f  REF_POS per read %.1f" % (
        c["t_dpm"] / n, c["t_dps"] / n, c["t_fill"] / max(1, c["t_dps"]), c["ref_pos"] / n))


def cmd_timeline(a):
    import numpy as np
    names = ["island", "fast0", "fast1", "resolve_f", "slow0", "resolve_s0", "slow1", "resolve_s1", "delA"]
    stride = 1 << 17
    raw = (gzip.open(a.file) if a.file.endswith(".gz") else open(a.file, "rb")).read()
    tl = np.frombuffer(raw, dtype=np.uint64).reshape(len(names), stride, 4)
    L = None
    if a.reads and a.reads.endswith(".npy"):  # tools/first_call.py DSB_SAVE_LENS
        L = np.load(a.reads)
    elif a.reads:
        with open(a.reads, "rb") as f:
            L = np.array([len(line) - 1 for i, line in enumerate(f) if i % 4 == 1])
    t0 = min(int(tl[p][tl[p][:, 0] > 0][:, 0].min()) for p in range(len(names)) if (tl[p][:, 0] > 0).any())
    for p, nm in enumerate(names):
        e = tl[p][tl[p][:, 0] > 0]
        if not len(e):
            continue
        act = ((e[:, 2] >> np.uint64(40)) & np.uint64(1)).astype(bool)
        s = (e[:, 0].astype(np.int64) - t0) / 100.0  # us (s_memrealtime: 100 MHz)
        d = (e[:, 1].astype(np.int64) - e[:, 0].astype(np.int64)) / 100.0
        da = d[act] if act.any() else np.zeros(1)
        print(f"{nm:10s} waves {len(e):6d} active {act.sum():6d}  start {s.min() / 1e3:8.2f} ms  end "
              f"{(s + d).max() / 1e3:8.2f} ms  active dur us: mean {da.mean():8.1f} p50 {np.percentile(da, 50):8.1f} "
              f"p99 {np.percentile(da, 99):8.1f} max {da.max():8.1f}")
        if nm in ("fast0", "slow0", "resolve_s0", "delA", "resolve_f") and act.any():
            rd = (e[:, 2] & np.uint64(0xffffffff)).astype(np.int64)
            print("   slowest:", ", ".join(f"r{rd[i]}" + (f"(L{L[rd[i]]})" if L is not None else "") +
                                        f" {d[i] / 1e3:.1f}ms@{s[i] / 1e3:.1f}" for i in np.argsort(-d)[:8]))
            end = s + d
            pts = np.linspace(s.min(), end.max(), 11)
            print("   running waves:", " ".join(str(int(((s <= x) & (end > x)).sum())) for x in pts))


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    p = sub.add_parser("kernels")
    p.add_argument("db")
    p.add_argument("--min-grid", type=int, default=1000)
    p.add_argument("--csv", default=None)
    p.set_defaults(fn=cmd_kernels)
    for name, fn in (("pmc", cmd_pmc), ("sq", cmd_sq)):
        p = sub.add_parser(name)
        p.add_argument("dir")
        p.set_defaults(fn=fn)
    p = sub.add_parser("wave")
    p.add_argument("bench_json")
    p.set_defaults(fn=cmd_wave)
    p = sub.add_parser("timeline")
    p.add_argument("file")
    p.add_argument("reads", nargs="?")
    p.set_defaults(fn=cmd_timeline)
    a = ap.parse_args()
    a.fn(a)


if __name__ == "__main__":
    main()
