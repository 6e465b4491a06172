"""Dev tool (GPU box): wall time of the first read_classify calls of a fresh process (workspace
allocation on first use), C1 proxy, 100k reads.  python tools/first_call.py [n_reads]"""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "desamba-so_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import bench  # noqa: E402  (index unpacking and read simulation, before any GPU use)

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
d, name = bench.unpack_index(0, "c1")
fq = bench.make_reads(d, n, 77, 8000)
import pydesamba  # noqa: E402

t = time.perf_counter()
idx = pydesamba.Index(d)
print(f"load_index {time.perf_counter() - t:.2f} s", flush=True)
out, m = C.c_void_p(), C.c_uint64(0)
for k in range(4):
    t = time.perf_counter()
    idx.L.read_classify(idx.h, fq, len(fq), C.byref(out), C.byref(m), 100 + k, 1)
    print(f"read_classify {k}: {time.perf_counter() - t:.3f} s, {m.value / 1e9:.2f} GB out", flush=True)
    idx.L.dsb_free(out)
