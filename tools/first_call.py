"""Dev tool (GPU box): one process, one index, a few classify calls on fresh synthetic reads.

  python tools/first_call.py [n_reads] [workload] [mode]

  mode "dropin" (default): wall time of the first read_classify calls of a fresh process
      (workspace allocation on first use), 4 calls.
  mode "reads:I,J,...": reads I, J, ... of the same synthetic set, each alone in a batch, with the
      work counters (stats 1) and the wave clocks (stats 2) of every phase: what a slow read does.
  mode "batch+slow": "batch", then "reads:" on the 6 reads the timeline shows slowest in delA.
  mode "batch": one Batch.run (resident reads, the bench's path) with the per-phase timing; with a
      DSB_TL=1 library (tools/variant.sh tl "-DDSB_TL=1" 0 1 2 3 4 5 6 7 8, DSB_LIB=...var_tl.so)
      and DSB_WAVE_DBG=4096 DSB_TIMELINE=FILE it leaves the per-read phase timeline in FILE
      (tools/prof_report.py timeline FILE); keep n_reads within one chunk and 2^17 waves.
workload: bench.py's WORKLOADS key (c1, c2, c2l18, c2xl, ...; c2* proxies are built when absent).
"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "desamba-so_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import bench  # noqa: E402  (index unpacking and read simulation, before any GPU use)

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
workload = sys.argv[2] if len(sys.argv) > 2 else "c1"
mode = sys.argv[3] if len(sys.argv) > 3 else "dropin"
d, name = bench.unpack_index(0, workload)
fq = bench.make_reads(d, n, 77, 8000)
if os.environ.get("DSB_SAVE_LENS"):  # read lengths (.npy) for tools/prof_report.py timeline
    import numpy as np
    np.save(os.environ["DSB_SAVE_LENS"], np.array([len(x) for x in fq.split(b"\n")[1::4]], dtype=np.uint32))
import pydesamba  # noqa: E402

t = time.perf_counter()
idx = pydesamba.Index(d)
print(f"{name}: load_index {time.perf_counter() - t:.2f} s", flush=True)


def slow_reads(k=6):
    """the k reads with the longest delA wave in the DSB_TIMELINE file (tools/prof_report.py layout)"""
    import shutil
    import numpy as np
    shutil.copy(os.environ["DSB_TIMELINE"], os.environ["DSB_TIMELINE"] + ".batch")  # the per-read runs rewrite it
    tl = np.fromfile(os.environ["DSB_TIMELINE"], dtype=np.uint64).reshape(9, 1 << 17, 4)[8]
    e = tl[tl[:, 0] > 0]
    d = e[:, 1].astype(np.int64) - e[:, 0].astype(np.int64)
    return [int(e[i, 2] & np.uint64(0xffffffff)) for i in np.argsort(-d)[:k]]


def per_read(ids):
    recs = fq.split(b"\n")
    for i in ids:
        one = b"\n".join(recs[4 * i:4 * i + 4]) + b"\n"
        if os.environ.get("DSB_SAVE_FQ"):
            with open(os.environ["DSB_SAVE_FQ"], "ab") as f:
                f.write(one)
        for st in (1, 2):
            b = idx.batch(one)
            t = time.perf_counter()
            tm = b.run(max_read_l=1 << 20, stats=st)  # 1: work counters, 2: wave clocks
            ms = (time.perf_counter() - t) * 1e3
            sam = b.format(pydesamba.FMT_SAM)
            b.close()
            nz = {ph: {k: v for k, v in d.items() if v} for ph, d in tm["stats_phase"].items()}
            print(json.dumps({"read": i, "len": len(recs[4 * i + 1]), "stats": st, "wall_ms": round(ms, 2),
                              "ms_phase": {k: round(v, 3) for k, v in tm["ms_phase"].items()},
                              "sam_lines": sam.count(b"\n"), "phases": nz}), flush=True)


if mode.startswith("reads:"):
    per_read(map(int, mode[6:].split(",")))
elif mode.startswith("batch"):
    b = idx.batch(fq)
    t = time.perf_counter()
    tm = b.run(max_read_l=0)
    print(f"batch run {time.perf_counter() - t:.3f} s", flush=True)
    keep = ("n_reads", "n_chunks", "n_retry", "n_ws_shrink", "ms_classA", "ms_classB", "ms_phase")
    print(json.dumps({k: tm[k] for k in keep if k in tm}), flush=True)
    b.close()
    if mode == "batch+slow":
        ids = slow_reads()
        print("slowest delA reads:", ids, flush=True)
        per_read(ids)
else:
    out, m = C.c_void_p(), C.c_uint64(0)
    for k in range(4):
        t = time.perf_counter()
        idx.L.read_classify(idx.h, fq, len(fq), C.byref(out), C.byref(m), 100 + k, 1)
        print(f"read_classify {k}: {time.perf_counter() - t:.3f} s, {m.value / 1e9:.2f} GB out", flush=True)
        idx.L.dsb_free(out)
idx.close()
