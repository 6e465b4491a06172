"""Per-read phase timeline (dev tool): the file written with DSB_WAVE_DBG=4096 DSB_TIMELINE=path.

  python tools/timeline.py tl.bin[.gz] [reads.fq]

Each record is {start, end, read | phase << 32 | active << 40, HW_ID | XCC_ID << 32} in
s_memrealtime ticks (100 MHz), slot t of phase ph at [ph * 2^17 + t] (dsb_gpu.h).  Prints per
phase: reads, active reads, span, the duration distribution of active reads, the slowest reads
(with their lengths when the FASTQ is given) and how many waves are still running over time.
"""
import gzip
import sys

import numpy as np

PH = ["island", "fast0", "fast1", "resolve_f", "slow0", "resolve_s0", "slow1", "resolve_s1", "delA"]
STRIDE = 1 << 17


def load(p):
    raw = (gzip.open(p) if p.endswith(".gz") else open(p, "rb")).read()
    return np.frombuffer(raw, dtype=np.uint64).reshape(len(PH), STRIDE, 4)


def lengths(fq):
    out = []
    with open(fq, "rb") as f:
        for i, line in enumerate(f):
            if i % 4 == 1:
                out.append(len(line) - 1)
    return np.array(out)


def main():
    tl = load(sys.argv[1])
    L = lengths(sys.argv[2]) if len(sys.argv) > 2 else None
    t0 = min(int(tl[p][tl[p][:, 0] > 0][:, 0].min()) for p in range(len(PH)) if (tl[p][:, 0] > 0).any())
    for p, nm in enumerate(PH):
        e = tl[p][tl[p][:, 0] > 0]
        if not len(e):
            continue
        act = ((e[:, 2] >> np.uint64(40)) & np.uint64(1)).astype(bool)
        s = (e[:, 0].astype(np.int64) - t0) / 100.0  # us
        d = (e[:, 1].astype(np.int64) - e[:, 0].astype(np.int64)) / 100.0
        print(f"{nm:10s} waves {len(e):6d} active {act.sum():6d}  start {s.min() / 1e3:8.2f} ms  end "
              f"{(s + d).max() / 1e3:8.2f} ms  active dur us: mean {d[act].mean() if act.any() else 0:8.1f} "
              f"p50 {np.percentile(d[act], 50) if act.any() else 0:8.1f} p99 {np.percentile(d[act], 99) if act.any() else 0:8.1f} "
              f"max {d[act].max() if act.any() else 0:8.1f}")
        if nm in ("fast0", "slow0", "delA", "resolve_f") and act.any():
            idx = np.argsort(-d)[:8]
            rd = (e[:, 2] & np.uint64(0xffffffff)).astype(np.int64)
            print("   slowest:", ", ".join(f"r{rd[i]}" + (f"(L{L[rd[i]]})" if L is not None else "") +
                                        f" {d[i] / 1e3:.1f}ms@{s[i] / 1e3:.1f}" for i in idx))
            end = s + d
            span0, span1 = s.min(), end.max()
            pts = np.linspace(span0, span1, 11)
            print("   running waves:", " ".join(str(int(((s <= x) & (end > x)).sum())) for x in pts))


if __name__ == "__main__":
    main()
