"""ctypes binding of lib/libdesamba.so for tests and bench.py.

Mirrors the reference's three ABI calls (include/desamba.h) plus the extension entry
points of include/desamba_mi355x.h.  The library is built in-tree by `make -C
desamba-so_amd`; there is no Python or CPU fallback for classification.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libdesamba.so")

FMT_SAM, FMT_SAM_FULL, FMT_DES, FMT_DES_FULL = 1, 2, 3, 4
PHASES = ["island", "fast0", "fast1", "resolve_f", "slow0", "resolve_s0", "slow1", "resolve_s1", "delA"]
# ms_phase slots: the phases (each with a work-counter block), then the scoring's read-hash build in
# LDS (k_hash_lds, DSB_HASH_LDS builds; its counters are in the delA block, hash_b)
MS_PHASES = PHASES + ["hash", "heavy"]
ST_NAMES = ["occ", "occ_nib", "mem_search", "sa", "uni", "ref_pos", "getref_b", "anchor", "chain", "ek1", "ek2",
            "hash_b", "lookup", "node", "t_mem", "t_map", "t_build", "t_match", "t_win", "t_all", "t_dpm", "t_dps",
            "t_fill", "pass2", "replay", "t_mprobe", "t_mwalk", "t_comb", "nwin", "nbatch", "ncand", "nsms"]
ST_STRIDE = 32


class Timing(C.Structure):
    _fields_ = [("stats_on", C.c_int), ("n_launch_phase", C.c_int), ("ms_total", C.c_double), ("ms_h2d", C.c_double),
                ("ms_d2h", C.c_double), ("ms_encode", C.c_double), ("ms_seed", C.c_double),
                ("ms_classA", C.c_double), ("ms_classB", C.c_double), ("ms_phase", C.c_double * 12),
                ("n_reads", C.c_uint64),
                ("n_bases", C.c_uint64), ("n_retry", C.c_uint64), ("n_chunks", C.c_uint64),
                ("seed_positions", C.c_uint64), ("n_launch_dela", C.c_uint64),
                ("stats", C.c_uint64 * 320),
                ("ms_parse", C.c_double), ("ms_gather", C.c_double), ("ms_format", C.c_double),
                ("ms_wait_gpu", C.c_double), ("n_batches", C.c_uint64), ("n_devices", C.c_uint64),
                ("n_view_records", C.c_uint64), ("n_copied_records", C.c_uint64),
                ("n_ws_shrink", C.c_uint64), ("n_heavy", C.c_uint64), ("n_defer_heavy", C.c_uint64)]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_ if k not in ("stats", "ms_phase")}
        d["ms_phase"] = {n: float(self.ms_phase[i]) for i, n in enumerate(MS_PHASES)}
        d["stats_phase"] = {ph: {n: int(self.stats[ST_STRIDE * p + i]) for i, n in enumerate(ST_NAMES)}
                            for p, ph in enumerate(PHASES)}
        d["stats"] = {n: sum(v[n] for v in d["stats_phase"].values()) for n in ST_NAMES}
        d["stats_B"] = {n: int(self.stats[ST_STRIDE * 9 + i]) for i, n in enumerate(ST_NAMES)}
        return d


_lib = None


def lib(path: str | None = None):
    """Load the shared library (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    p = path or os.environ.get("DSB_LIB", LIB_PATH)
    if not os.path.exists(p):
        raise RuntimeError(f"{p} not built: run `make -C desamba-so_amd` (hipcc, gfx950)")
    L = C.CDLL(p, mode=C.RTLD_GLOBAL)
    vp, pp, u64, u64p = C.c_void_p, C.POINTER(C.c_char_p), C.c_uint64, C.POINTER(C.c_uint64)
    L.load_index.argtypes = [C.POINTER(vp), C.c_char_p]
    L.load_index.restype = None
    L.read_classify.argtypes = [vp, C.c_char_p, u64, C.POINTER(C.c_void_p), u64p, C.c_int, C.c_int]
    L.read_classify.restype = None
    L.meta_analysis.argtypes = [vp, C.c_char_p, u64, C.POINTER(C.c_void_p), u64p, C.c_int, C.c_int, u64,
                                C.POINTER(C.c_void_p), u64p]
    L.meta_analysis.restype = None
    L.dsb_classify_text.argtypes = [vp, C.c_char_p, u64, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_void_p), u64p,
                                    C.POINTER(Timing)]
    L.dsb_classify_text.restype = C.c_int
    L.dsb_batch_create.argtypes = [vp, C.c_char_p, u64, C.POINTER(Timing)]
    L.dsb_batch_create.restype = vp
    L.dsb_batch_run.argtypes = [vp, vp, C.POINTER(C.c_int), C.POINTER(Timing)]
    L.dsb_batch_run.restype = C.c_int
    L.dsb_batch_format.argtypes = [vp, vp, C.c_int, C.POINTER(C.c_void_p), u64p]
    L.dsb_batch_format.restype = C.c_int
    L.dsb_batch_format_range.argtypes = [vp, vp, C.c_int, u64, u64, C.POINTER(C.c_void_p), u64p]
    L.dsb_batch_format_range.restype = C.c_int
    L.dsb_batch_carry.argtypes = [vp, C.c_void_p]
    L.dsb_batch_carry.restype = C.c_int
    L.dsb_batch_taxa.argtypes = [vp, vp, C.c_int, C.c_void_p, C.c_void_p]
    L.dsb_batch_taxa.restype = C.c_int
    L.dsb_batch_taxon_counts.argtypes = [vp, vp, C.c_int, C.c_void_p, u64]
    L.dsb_batch_taxon_counts.restype = C.c_int
    L.dsb_batch_reads.argtypes = [vp]
    L.dsb_batch_reads.restype = u64
    L.dsb_batch_bases.argtypes = [vp]
    L.dsb_batch_bases.restype = u64
    L.dsb_batch_free.argtypes = [vp, vp]
    L.dsb_max_tid.argtypes = [vp]
    L.dsb_max_tid.restype = u64
    L.dsb_index_devices.argtypes = [vp, C.c_void_p, C.c_int]
    L.dsb_index_devices.restype = C.c_int
    L.dsb_parse_dump.argtypes = [C.c_char_p, u64, C.c_int, u64, C.POINTER(C.c_void_p), u64p]
    L.dsb_parse_dump.restype = C.c_int
    L.dsb_version.restype = C.c_char_p
    L.dsb_timing_size.restype = C.c_uint64
    if L.dsb_timing_size() != C.sizeof(Timing):  # the binding mirrors include/desamba_mi355x.h
        raise RuntimeError(f"{p}: dsb_timing_t is {L.dsb_timing_size()} bytes, this binding's Timing "
                           f"{C.sizeof(Timing)}: rebuild the library or update pydesamba.Timing")
    L.dsb_device_count.restype = C.c_int
    L.dsb_free.argtypes = [vp]
    L.dsb_unload_index.argtypes = [vp]
    _lib = L
    return L


def view(ptr: int, n: int) -> memoryview:
    """The n bytes at ptr, without a copy (ctypes.string_at takes an int size: outputs of 2 GB and
    more, e.g. SAM_FULL of 1M 8-kb reads, need this)."""
    return memoryview((C.c_char * n).from_address(ptr)).cast("B") if n else memoryview(b"")


def _take(L, p: C.c_void_p, n: int) -> bytes:
    if not p.value:
        return b""
    b = bytes(view(p.value, n))
    L.dsb_free(p)
    return b


class Index:
    """An index resident in the HBM of one GPU (reference load_index)."""

    def __init__(self, dirpath: str):
        self.L = lib()
        h = C.c_void_p()
        self.L.load_index(C.byref(h), dirpath.encode())
        self.h = h

    def read_classify(self, data: bytes | str, thread_id: int = 0, thread_num: int = 1) -> bytes:
        """data: FASTQ/FASTA bytes, or a path (str) -> input_n = (uint64_t)-1."""
        out, n = C.c_void_p(), C.c_uint64(0)
        if isinstance(data, str):
            self.L.read_classify(self.h, data.encode(), C.c_uint64(0xFFFFFFFFFFFFFFFF), C.byref(out), C.byref(n),
                                 thread_id, thread_num)
        else:
            self.L.read_classify(self.h, data, len(data), C.byref(out), C.byref(n), thread_id, thread_num)
        return _take(self.L, out, n.value)

    def classify(self, data: bytes, fmt: int = FMT_SAM_FULL, max_read_l: int = 0, stats: bool = False):
        """-> (output bytes, timing dict, carried max_read_l)"""
        out, n = C.c_void_p(), C.c_uint64(0)
        mrl = C.c_int(max_read_l)
        t = Timing()
        t.stats_on = int(stats)  # 1: work counters, 2: wave clocks (DSB_ST_T_*)
        rc = self.L.dsb_classify_text(self.h, data, len(data), fmt, C.byref(mrl), C.byref(out), C.byref(n),
                                      C.byref(t))
        if rc != 0:
            raise RuntimeError("dsb_classify_text failed")
        return _take(self.L, out, n.value), t.as_dict(), mrl.value

    def batch(self, data: bytes) -> "Batch":
        """Parse + upload reads once; they stay resident in HBM for repeated runs."""
        return Batch(self, data)

    def max_tid(self) -> int:
        return int(self.L.dsb_max_tid(self.h))

    def devices(self) -> list[int]:
        """HIP device ids the index is replicated on (read_classify uses all of them)."""
        ids = (C.c_int * 16)()
        n = self.L.dsb_index_devices(self.h, ids, 16)
        return [ids[k] for k in range(min(n, 16))]

    def meta_analysis(self, sam: bytes, flag: int = 0, max_snapshot_len: int = 65536, thread_id: int = 0):
        out, n = C.c_void_p(), C.c_uint64(0)
        snap, sn = C.c_void_p(), C.c_uint64(0)
        self.L.meta_analysis(self.h, sam, len(sam), C.byref(out), C.byref(n), thread_id, flag, max_snapshot_len,
                             C.byref(snap), C.byref(sn))
        return _take(self.L, out, n.value), _take(self.L, snap, sn.value)

    def close(self):
        if self.h:
            self.L.dsb_unload_index(self.h)
            self.h = None


def parse_dump(data: bytes, slow: bool = False, batch_reads: int = 0) -> bytes:
    """Records the library's FASTQ/FASTA parser yields (host only, no GPU): one
    "name\tseq_l\tseq\tqual\n" line per record."""
    L = lib()
    out, n = C.c_void_p(), C.c_uint64(0)
    L.dsb_parse_dump(data, len(data), int(slow), batch_reads, C.byref(out), C.byref(n))
    return _take(L, out, n.value)


class Batch:
    """Reads resident in HBM (include/desamba_mi355x.h dsb_batch_*)."""

    def __init__(self, index: Index, data: bytes):
        self.ix, self.L = index, index.L
        t = Timing()
        self.h = self.L.dsb_batch_create(index.h, data, len(data), C.byref(t))
        if not self.h:
            raise RuntimeError("dsb_batch_create failed")
        self.upload = t.as_dict()
        self.n_reads = int(self.L.dsb_batch_reads(self.h))
        self.n_bases = int(self.L.dsb_batch_bases(self.h))
        self.max_read_l = 0

    def run(self, max_read_l: int | None = None, stats: bool = False) -> dict:
        """Classify every read of the batch; returns the timing dict."""
        mrl = C.c_int(self.max_read_l if max_read_l is None else max_read_l)
        t = Timing()
        t.stats_on = int(stats)  # 1: work counters, 2: wave clocks (DSB_ST_T_*)
        if self.L.dsb_batch_run(self.ix.h, self.h, C.byref(mrl), C.byref(t)) != 0:
            raise RuntimeError("dsb_batch_run failed")
        self.max_read_l = mrl.value
        return t.as_dict()

    def format(self, fmt: int = FMT_SAM) -> bytes:
        out, n = C.c_void_p(), C.c_uint64(0)
        self.L.dsb_batch_format(self.ix.h, self.h, fmt, C.byref(out), C.byref(n))
        return _take(self.L, out, n.value)

    def format_range(self, lo: int, hi: int, fmt: int = FMT_SAM) -> bytes:
        """Records of reads [lo, hi) only."""
        out, n = C.c_void_p(), C.c_uint64(0)
        self.L.dsb_batch_format_range(self.ix.h, self.h, fmt, lo, hi, C.byref(out), C.byref(n))
        return _take(self.L, out, n.value)

    def format_range_hash(self, lo: int, hi: int, fmt: int, fn) -> str:
        """fn(memoryview) of format_range(lo, hi, fmt), hashed in place (multi-GB outputs)."""
        out, n = C.c_void_p(), C.c_uint64(0)
        self.L.dsb_batch_format_range(self.ix.h, self.h, fmt, lo, hi, C.byref(out), C.byref(n))
        h = fn(view(out.value, n.value) if out.value else b"")
        if out.value:
            self.L.dsb_free(out)
        return h

    def carry(self):
        """-> int32[n]: the max_read_l each read's length filter used in the last run."""
        import numpy as np
        c = np.zeros(self.n_reads, dtype=np.int32)
        self.L.dsb_batch_carry(self.h, c.ctypes.data)
        return c

    def taxa(self, flag: int = 0):
        """-> (tid uint32[n], weight uint64[n]) as meta_analysis assigns them."""
        import numpy as np
        tid = np.zeros(self.n_reads, dtype=np.uint32)
        w = np.zeros(self.n_reads, dtype=np.uint64)
        self.L.dsb_batch_taxa(self.ix.h, self.h, flag, tid.ctypes.data, w.ctypes.data)
        return tid, w

    def taxon_counts(self, counts, flag: int = 0):
        """Per-taxon weights of the last run into `counts` (a torch int64 tensor on this GPU of
        >= max_tid + 1 entries), reduced on the device (dsb_batch_taxon_counts)."""
        import torch
        assert counts.is_cuda and counts.dtype == torch.int64 and counts.is_contiguous()
        dev = self.ix.devices()[0]
        if counts.device.index != dev:
            raise ValueError(f"counts is on cuda:{counts.device.index}, the batch is on GPU {dev}")
        torch.cuda.current_stream().synchronize()  # the library works on its own stream
        if self.L.dsb_batch_taxon_counts(self.ix.h, self.h, flag, counts.data_ptr(), counts.numel()) != 0:
            raise RuntimeError("dsb_batch_taxon_counts failed")
        return counts

    def close(self):
        if self.h:
            self.L.dsb_batch_free(self.ix.h, self.h)
            self.h = None
