"""Dev tool (GPU box): read_classify end to end on the bench workload for a few pipeline settings.

  python tools/dropin_sweep.py [reads] [contexts...]

For each setting (device contexts per GPU x reads per batch): one untimed call (buffers grow on
first use), then 3 timed read_classify calls; prints the median reads/s of the C call timed from
Python, and the pipeline's stage times from a dsb_classify_text call of the same setting."""
import ctypes as C
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "desamba-so_amd"))
import bench  # noqa: E402
import pydesamba as P  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
ctxs = sys.argv[2:] or ["1", "2"]
idx_dir, _ = bench.unpack_index(0, "c1")
fq = bench.make_reads(idx_dir, n, 1000, 8000)
os.environ["DSB_PIPE_MBP"] = "100000"


def rc(idx):
    out, m = C.c_void_p(), C.c_uint64(0)
    t = time.perf_counter()
    idx.L.read_classify(idx.h, fq, len(fq), C.byref(out), C.byref(m), 5, 1)
    s = time.perf_counter() - t
    idx.L.dsb_free(out)
    return s


for ctx in ctxs:
    os.environ["DSB_GPU_CONTEXTS"] = ctx
    idx = P.Index(idx_dir)
    for reads in os.environ.get("SWEEP_READS", "20000 25000 34000 50000").split():
        os.environ["DSB_PIPE_READS"] = reads
        rc(idx)
        secs = statistics.median(rc(idx) for _ in range(3))
        _, tm, _ = idx.classify(fq, fmt=P.FMT_SAM_FULL)
        print(f"contexts {ctx} reads/batch {reads:>6}: {n / secs:9.0f} reads/s (read_classify, median of 3)  "
              f"pipeline: total {tm['ms_total']:.0f} ms parse {tm['ms_parse']:.0f} gather {tm['ms_gather']:.0f} "
              f"format {tm['ms_format']:.0f} wait_gpu {tm['ms_wait_gpu']:.0f} kernels(A) {tm['ms_classA']:.0f} "
              f"seed {tm['ms_seed']:.0f} batches {tm['n_batches']}", flush=True)
    idx.close()
