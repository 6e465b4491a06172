#!/usr/bin/env python3
"""Throughput of the MI355X classify path (BASELINE.json metric, config C2 at N = 1, C3 beyond).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--reads R] [--workload c2l18|c2|c2xl|c1|fixture]
                  [--mix ont|c4] [--index DIR]

--gpus N without a torch.distributed launcher starts N rank processes itself (one per GPU,
before this process touches any GPU); under torchrun (WORLD_SIZE set) each rank is one process.

A step = classify one batch of R synthetic ONT reads (lognormal, mean 8 kb, 5-15 % error)
already resident in HBM (dsb_batch_run: seed + occ/rank + chaining + scoring on the GPU,
results back on the host), then assign one taxon per read exactly as meta_analysis does
(reference src/cly_mt.c:902-961) and reduce the per-taxon counts across ranks with RCCL
(all_reduce over torch.distributed "nccl" when N > 1).  Reads shard across ranks (weak
scaling: every rank classifies its own R reads); the index is replicated in each GPU's HBM.

Workload c2l18 (the default since round 6; BASELINE configs[2], and per rank configs[3]): a proxy of
the RefSeq index at the reference's own index scale (tools/simulate.py preset c2l18: 1.86 Gbp,
1.06 G distinct 31-mers, so the builder picks l_ek 18 / MASK_33 / 1 GB e-kmer tables, 1.94 G BWT
rows, a 7.0 GB index; RefSeq itself is not available offline), built in this run by
tools/proxy_build.py (simulate.py + this repository's desamba_index, ~2 min on the GPU box's 16
cores, cached under $TMPDIR), + R = 1M reads per rank, simulated by forked workers before the process
touches a GPU.  --workload c2: the smaller C2 proxy of rounds 3-5 (495 Mbp, l_ek 17, 2.3 GB);
c2xl: 5 Gbp, BWT past 2^32 rows, 16.6 GB (an 8-minute build); c1: the 55.8 Mbp proxy of BASELINE
configs[1] (data/c1_index.txz, made by the reference's own builder), usually with --reads 100000.

The JSON line carries:
  roofline     the dominant kernel (the phase of classify part A with the largest HIP-event
               time over the timed steps, on the library's stream): algorithmic bytes per
               launch from the work counters of one untimed stats run
               / its average launch time;
               traffic = HBM bytes per launch from the committed PMC profile of this
               workload (profiles/), or null.
  cpu_baseline the reference classifier (oracle/_ref/deSAMBA, built from the reference
               sources by oracle/Makefile) on the host cores, on a bounded sample of the
               same reads, at -t <usable CPUs> (the cgroup quota) and at -t nproc, the faster
               being the value, and at -t 1, plus the reference's own read_classify through
               dlopen (oracle/_ref/abi_time); the GPU's primary taxids for the sample are
               compared with the reference's records (taxid_mismatch), and the GPU's records of
               the first reads with the hermetic reference's (oracle/_ref/herm_classify,
               t3_mismatch); rank 0 at N = 1 only.
  dropin       the drop-in path end to end: one read_classify(idx, fastq, n, ...) call over
               the first --dropin-reads reads of the batch (text in host memory -> SAM_FULL
               text in host memory: parse, H2D, kernels, D2H, formatting), index preloaded,
               checked against the batch path's records; rank 0 at N = 1 only.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import re
import subprocess
import sys
import tarfile
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "desamba-so_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

METRIC = "long reads classified/sec + Gbases/sec at 1/2/4/8 MI355X; bit-exact taxid match"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md
# random 64-B line rate measured on this hardware (profiles/r03_calib/calib.json: dependent 4-B
# gathers over a 1 GB table, 55.92 G loads/s, one 64-B line each): the ceiling of the classify
# kernels' access pattern, which is random lines, not streams
RANDOM_LINE_PEAK_GBS = 55.92 * 64
# the phase kernels of classify part A (kernels.hip launch_phase)
KERNEL_OF = {"island": "k_island_g<16>", "fast0": "k_wave_phase<1>", "fast1": "k_wave_phase<2>",
             "resolve_f": "k_wave_phase<3>", "slow0": "k_wave_phase<4>", "resolve_s0": "k_wave_phase<5>",
             "slow1": "k_wave_phase<6>", "resolve_s1": "k_wave_phase<7>", "delA": "k_wave_phase<8>",
             "hash": "k_hash_lds<0>"}


def phase_bytes(c):
    """Algorithmic HBM bytes of one phase from its work counters:
    occ checkpoint + nibble bytes, 16 B per MEM-search interval, 8 B per SA sample / unitig /
    ref_pos entry, 2 bits per reference base unpacked, 56 B per anchor / chain written, the
    read-hash build bytes, 4 B per hash lookup and 8 B per hash-list node visited."""
    return (c["occ_nib"] + 16 * c["mem_search"] + 8 * (c["sa"] + c["uni"] + c["ref_pos"]) + c["getref_b"]
            + 56 * (c["anchor"] + c["chain"]) + c["hash_b"] + 4 * c["lookup"] + 8 * c["node"])


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


# ----------------------------------------------------------------------------- inputs
def _tmp():
    return os.environ.get("TMPDIR", "/tmp")


# synthetic proxy indexes: shipped packed (data/, tests/golden/) or, for C2, built in the run
WORKLOADS = {
    "c1": ("C1-proxy-56Mbp", os.path.join(ROOT, "data", "c1_index.txz")),
    "c2": ("C2-proxy-495Mbp-lek17", os.path.join(ROOT, "data", "c2_index.txz")),
    # larger proxies, always built in the run (tools/proxy_build.py): the next e-kmer size classes
    "c2l18": ("C2-proxy-1.86Gbp-lek18", None),
    "c2xl": ("C2-proxy-5Gbp-lek18-bwt-past-2^32", None),
    "fixture": ("C0-fixture-1Mbp", os.path.join(ROOT, "tests", "golden", "fixture_index.txz")),
}


def unpack_index(rank: int, workload: str = "c2") -> tuple[str, str]:
    """-> (index dir, workload name).  Rank 0 unpacks (or builds the C2 proxy), the others wait."""
    name, src = WORKLOADS[workload]
    if workload.startswith("c2") and (src is None or not os.path.exists(src)):
        import proxy_build
        d = proxy_build.ensure_proxy(workload, build=(rank == 0))
        return d, name
    if not os.path.exists(src):
        if workload != "c1":
            raise SystemExit(f"{src} missing")
        name, src = WORKLOADS["fixture"]
    st = os.stat(src)
    key = hashlib.sha1(f"{src}:{st.st_size}:{int(st.st_mtime)}".encode()).hexdigest()[:12]
    d = os.path.join(_tmp(), f"dsb_index_{key}")
    done = os.path.join(d, ".done")
    if rank == 0 and not os.path.exists(done):
        tmpd = tempfile.mkdtemp(dir=_tmp(), prefix="dsb_index_part_")
        t = time.time()
        with tarfile.open(src) as tf:
            tf.extractall(tmpd)
        sub = [e for e in os.listdir(tmpd) if os.path.isdir(os.path.join(tmpd, e))]
        inner = os.path.join(tmpd, sub[0]) if len(sub) == 1 and not os.path.exists(
            os.path.join(tmpd, "deSAMBA.bwt")) else tmpd
        if os.path.exists(d):
            subprocess.run(["rm", "-rf", d], check=True)
        os.rename(inner, d)
        open(done, "w").close()
        log(f"unpacked {os.path.basename(src)} in {time.time() - t:.1f}s -> {d}")
    t0 = time.time()
    while not os.path.exists(done):
        if time.time() - t0 > 900:
            raise RuntimeError("timed out waiting for rank 0 to unpack the index")
        time.sleep(1)
    return d, name


def make_reads(index_dir: str, n: int, seed: int, mean_len: int, mix: str = "ont", world: int = 1) -> bytes:
    """Synthetic reads sampled from the index's own reference (tools/simulate.py): ONT-like
    (lognormal mean `mean_len`), or BASELINE C4's mix (150 bp + 20 kb ONT, 1:1, interleaved),
    made in 10k-read chunks by forked workers (simulate_fastq_parallel; the text does not depend
    on the worker count).  Cached under $TMPDIR when the disk has room.  Must run before this
    process touches a GPU."""
    path = os.path.join(_tmp(), f"dsb_reads_{os.path.basename(index_dir)}_{n}_{seed}_{mean_len}_{mix}_c10k.fq")
    if os.path.exists(path):
        with open(path, "rb") as f:
            return f.read()
    import proxy_build
    import simulate
    t = time.time()
    genomes = simulate.read_fasta_genomes_from_index(index_dir)
    workers = max(1, min(32, proxy_build.usable_cpus() // max(1, world)))
    fq = simulate.simulate_fastq_parallel(genomes, n, seed, mix, mean_len, workers=workers)
    del genomes
    log(f"simulated {n} reads (seed {seed}, {len(fq) / 1e9:.2f} GB of FASTQ) on {workers} workers in {time.time() - t:.1f}s")
    try:
        import shutil
        if shutil.disk_usage(_tmp()).free > 3 * len(fq) + (8 << 30):
            part = path + f".part{os.getpid()}"
            with open(part, "wb") as f:
                f.write(fq)
            os.rename(part, path)
    except OSError:
        pass
    return fq


def index_info(index_dir: str) -> dict:
    """Size and e-kmer parameters of the index (set_ekmer_par, reference src/idx.c:966-982), plus how
    it was made (tools/proxy_build.py's build.json when built in this run)."""
    info = {}
    try:
        info["bytes"] = sum(os.path.getsize(os.path.join(index_dir, f)) for f in os.listdir(index_dir)
                            if f.startswith("deSAMBA."))
        with open(os.path.join(index_dir, "deSAMBA.exki"), "rb") as f:
            ek = int.from_bytes(f.read(8), "little")
        info["e_kmer_table_bytes"] = ek
        info["l_ek"] = {1 << 27: 16, 1 << 28: 17, 1 << 29: 17, 1 << 30: 18, 1 << 31: 18, 1 << 32: 19,
                        1 << 33: 19}.get(ek, 20)
        bj = os.path.join(index_dir, "build.json")
        if os.path.exists(bj):
            with open(bj) as f:
                info["built_in_run"] = json.load(f)
    except OSError:
        pass
    return info


def fastq_head(fq: bytes, n: int) -> bytes:
    pos = 0
    for _ in range(4 * n):
        pos = fq.find(b"\n", pos) + 1
        if pos == 0:
            return fq
    return fq[:pos]


# ----------------------------------------------------------------------------- baseline
def host_cpus() -> dict:
    """nproc, the CPUs this process may run on, the cgroup CPU quota and the model name."""
    info = {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)), "cgroup_quota": None,
            "model": None}
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            info["cgroup_quota"] = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                info["model"] = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return info


def _ref_classify(index_dir: str, sample: bytes, threads: int, sam_out: str | None):
    """The reference CLI on `sample`: (reads, seconds) from its own 'N sequences processed in
    T s' timer (starts after the index load, reference src/cly_mt.c:527,557)."""
    exe = os.path.join(ROOT, "oracle", "_ref", "deSAMBA")
    with tempfile.TemporaryDirectory(dir=_tmp()) as d:
        p = os.path.join(d, "sample.fq")
        with open(p, "wb") as f:
            f.write(sample)
        r = subprocess.run([exe, "classify", "-t", str(threads), "-o", sam_out or os.path.join(d, "o.sam"),
                            index_dir, p], capture_output=True, text=True, timeout=900)
    m = re.search(r"(\d+) sequences processed in ([0-9.]+)s", r.stdout + r.stderr)
    if r.returncode != 0 or not m:
        log("reference CPU run failed:", r.returncode, (r.stdout + r.stderr)[-400:])
        return None
    return int(m.group(1)), float(m.group(2))


def _ref_dropin(index_dir: str, sample: bytes, threads: int):
    """The reference's read_classify(thread_num) through dlopen (oracle/_ref/abi_time), index
    preloaded by its load_index, one call over the sample held in memory."""
    exe = os.path.join(ROOT, "oracle", "_ref", "abi_time")
    lib = os.path.join(ROOT, "oracle", "_ref", "libdesamba.so")
    if not (os.path.exists(exe) and os.path.exists(lib)):
        return None
    with tempfile.TemporaryDirectory(dir=_tmp()) as d:
        p = os.path.join(d, "sample.fq")
        with open(p, "wb") as f:
            f.write(sample)
        r = subprocess.run([exe, lib, index_dir, p, str(threads)], capture_output=True, text=True, timeout=900)
    if r.returncode != 0:
        log("reference read_classify run failed:", r.returncode, r.stderr[-400:])
        return None
    return json.loads(r.stdout.strip().splitlines()[-1])


def n_bases(fq: bytes) -> int:
    return sum(len(l) for i, l in enumerate(fq.split(b"\n")) if i % 4 == 1)


def t3_check(index_dir: str, sample: bytes, gpu_sam: bytes) -> dict | None:
    """The hermetic reference (oracle/_ref/herm_classify: the reference's objects, fresh buffer
    pools per read) on `sample`, every SAM record compared byte for byte with the
    GPU's records of the same reads from the timed batch (T3)."""
    exe = os.path.join(ROOT, "oracle", "_ref", "herm_classify")
    if not os.path.exists(exe):
        return None
    with tempfile.TemporaryDirectory(dir=_tmp()) as d:
        p = os.path.join(d, "t3.fq")
        with open(p, "wb") as f:
            f.write(sample)
        t = time.time()
        r = subprocess.run([exe, "--sam", index_dir, p], capture_output=True, timeout=900)
    if r.returncode != 0:
        log("herm_classify failed:", r.returncode, r.stderr[-400:])
        return None
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from samutil import compare
    c = compare(r.stdout, gpu_sam)
    return {"reads": c["reads"], "t3_mismatch": c["full_mismatch"], "taxid_mismatch": c["taxid_mismatch"],
            "mapped_mismatch": c["mapped_mismatch"], "secs": round(time.time() - t, 1),
            "oracle": "oracle/_ref/herm_classify --sam (hermetic reference build), first reads of the timed batch"}


def cpu_baseline(index_dir: str, fq: bytes, n_sample: int, n_sample_t1: int, gpu_sam_sample: bytes | None):
    """The reference (oracle/_ref, gcc -O3 build of the reference sources) on this box's host
    cores over the first reads of rank 0's batch: `deSAMBA classify -t T` at T = the usable CPUs
    (cgroup quota) and T = nproc, the faster being the value; -t 1 on a smaller sample; and
    read_classify(thread_num = the faster T) through dlopen.  The value run's primary taxids are
    compared with the GPU's records for the same reads."""
    if not os.path.exists(os.path.join(ROOT, "oracle", "_ref", "deSAMBA")):
        return None
    import proxy_build
    cpus = host_cpus()
    nproc = cpus["nproc"]
    eff = proxy_build.usable_cpus()
    cpus["usable"] = eff
    sample = fastq_head(fq, n_sample)
    nb = n_bases(sample)
    runs, sams = {}, {}
    with tempfile.TemporaryDirectory(dir=_tmp()) as d:
        for th in sorted({eff, nproc}):
            sam = os.path.join(d, f"o{th}.sam")
            t = time.time()
            r = _ref_classify(index_dir, sample, th, sam)
            if r is None:
                continue
            runs[th] = {"reads": r[0], "secs": r[1], "wall_s": round(time.time() - t, 1),
                        "value": round(r[0] / r[1], 1)}
            sams[th] = sam
        if not runs:
            return None
        best = min(runs, key=lambda th: runs[th]["secs"])
        n, secs = runs[best]["reads"], runs[best]["secs"]
        mism = None
        if gpu_sam_sample is not None:
            sys.path.insert(0, os.path.join(ROOT, "tests"))
            from samutil import compare
            with open(sams[best], "rb") as f:
                c = compare(f.read(), gpu_sam_sample)
            mism = {"reads": c["reads"], "taxid_mismatch": c["taxid_mismatch"], "mapped_mismatch": c["mapped_mismatch"],
                    "full_record_mismatch": c["full_mismatch"],
                    "note": "against the reference's -tN records (buffer pools shared across reads, SURVEY H1/H2): "
                            "full records may differ, taxids may not"}
    out = {"value": round(n / secs, 1), "unit": "reads/s", "cores": best, "cores_effective": eff, "nproc": nproc,
           "kind": "reference", "gbases_per_s": round(nb / secs / 1e9, 5), "host": cpus,
           "threads_tried": {str(th): v for th, v in runs.items()},
           "sample": f"first {n} reads ({nb / 1e6:.1f} Mbp) of rank 0's batch, `deSAMBA classify -t {best}` "
                     f"(gcc -O3 build of the reference sources; the faster of -t {eff} (usable CPUs) and -t {nproc} "
                     f"(nproc)), own timer {secs:.2f}s",
           "taxid_check_vs_gpu": mism}
    s1 = fastq_head(fq, n_sample_t1)
    r1 = _ref_classify(index_dir, s1, 1, None)
    if r1:
        out["t1"] = {"value": round(r1[0] / r1[1], 1), "reads": r1[0], "secs": r1[1],
                     "gbases_per_s": round(n_bases(s1) / r1[1] / 1e9, 5)}
    dj = _ref_dropin(index_dir, sample, best)
    if dj:
        out["read_classify"] = {"value": round(n / dj["secs"], 1), "secs": dj["secs"], "thread_num": best,
                                "reads": n, "output_bytes": dj["output_bytes"]}
    return out


def digest(buf) -> str:
    """Content hash for the drop-in identity check: xxh3-128 (GB/s, the 1M-read SAM_FULL is ~16 GB)
    when the xxhash module is importable, else sha256."""
    try:
        import xxhash
        return "xxh3_128:" + xxhash.xxh3_128(buf).hexdigest()
    except ImportError:
        return "sha256:" + hashlib.sha256(buf).hexdigest()


def dropin_leg(idx, fq: bytes, n_reads: int, nb: int, batch_digest: str | None, calls: int = 3):
    """read_classify over the given reads (reference desamba.h:23): FASTQ text in host memory ->
    SAM_FULL text in host memory, the index preloaded; the output is checked against the batch
    path's records for the same reads (content hash, in place)."""
    import ctypes as C
    import pydesamba as P
    L = idx.L
    out, n = C.c_void_p(), C.c_uint64(0)
    # one untimed call first: the library's pinned staging, device batch buffers and host pool are
    # allocated on first use and kept with the index (a service's steady state)
    L.read_classify(idx.h, fq, len(fq), C.byref(out), C.byref(n), 6, 1)
    L.dsb_free(out)
    # timed calls (fresh thread_ids, so each carries its own max_read_l from 0): a single 0.2-0.3 s
    # call of 100k reads varies by +-10% from run to run; the median is reported, every time kept
    times, got = [], None
    for k in range(calls):
        t = time.perf_counter()
        L.read_classify(idx.h, fq, len(fq), C.byref(out), C.byref(n), 7 + k, 1)
        times.append(time.perf_counter() - t)
        if k == 0:
            got = digest(P.view(out.value, n.value) if out.value else b"")
        L.dsb_free(out)
    secs = sorted(times)[len(times) // 2]
    same = None
    if batch_digest is not None:
        same = got == batch_digest
    # the same call through dsb_classify_text, for the pipeline's stage times (host wall times)
    t = P.Timing()
    mrl = C.c_int(0)
    if L.dsb_classify_text(idx.h, fq, len(fq), P.FMT_SAM_FULL, C.byref(mrl), C.byref(out), C.byref(n), C.byref(t)) == 0:
        L.dsb_free(out)
    tm = t.as_dict()
    stages = {k: round(tm[k], 2) for k in ("ms_total", "ms_parse", "ms_gather", "ms_format", "ms_wait_gpu", "ms_classA",
                                           "ms_seed", "ms_h2d", "ms_d2h")}
    stages.update({k: int(tm[k]) for k in ("n_batches", "n_devices", "n_view_records", "n_copied_records")})
    return {"value": round(n_reads / secs, 1), "unit": "reads/s", "secs": round(secs, 4),
            "secs_all": [round(x, 4) for x in times], "value_of": f"median of {calls} calls",
            "gbases_per_s": round(nb / secs / 1e9, 4), "reads": n_reads, "input_bytes": len(fq),
            "output_bytes": n.value, "identical_to_batch_records": same, "check": got.split(":")[0] if got else None,
            "pipeline": stages, "host_threads": int(os.environ.get("DSB_HOST_THREADS", "0")) or None,
            "what": "read_classify(idx, fastq_text, n, &out, &out_n, 7, 1): parse + H2D + kernels + D2H + "
                    "SAM_FULL formatting, index preloaded"}


def spawn_ranks(n: int) -> int:
    """--gpus N without a launcher: start N rank processes (RANK/LOCAL_RANK/WORLD_SIZE, rendezvous
    on 127.0.0.1) before this process touches any GPU, forward their exit status.  Rank 0 prints
    the JSON line."""
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c
                log(f"rank pid {p.pid} exited with {c}; stopping the other ranks")
                for q in live:
                    q.kill()
        time.sleep(0.2)
    return rc


# ----------------------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--reads", type=int, default=1000000, help="reads per rank")
    ap.add_argument("--mean-len", type=int, default=8000)
    ap.add_argument("--workload", default="c2l18", choices=sorted(WORKLOADS),
                    help="proxy index: c2l18 (default, 7.0 GB, built in the run), c2 (2.3 GB, built in the run unless "
                         "data/c2_index.txz exists), c2xl (16.6 GB), c1 (data/c1_index.txz)")
    ap.add_argument("--mix", default="ont", choices=["ont", "c4"], help="ONT reads, or C4's 150 bp + 20 kb 1:1 mix")
    ap.add_argument("--index", default=None, help="index directory (overrides --workload)")
    ap.add_argument("--name", default=None, help="workload name for --index")
    ap.add_argument("--cpu-sample", type=int, default=16000, help="reads in the CPU baseline sample (-t nproc)")
    ap.add_argument("--cpu-sample-t1", type=int, default=2000, help="reads in the -t 1 CPU sample")
    ap.add_argument("--t3-reads", type=int, default=2000, help="reads of the timed batch checked against herm_classify")
    ap.add_argument("--dropin-reads", type=int, default=100000, help="reads in the end-to-end read_classify leg")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-dropin", action="store_true", help="skip the end-to-end read_classify leg")
    ap.add_argument("--dropin-all", type=int, default=1,
                    help="1: also time one read_classify call over every read of the batch (rank 0, N = 1)")
    ap.add_argument("--no-stats", action="store_true", help="skip the work-counter run (roofline)")
    a = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(spawn_ranks(a.gpus))

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # inputs first: the index (unpacked, or the C2 proxy built) and the reads (forked workers),
    # before this process touches a GPU
    if a.index:
        index_dir, workload = a.index, a.name or os.path.basename(os.path.normpath(a.index))
    else:
        index_dir, workload = unpack_index(rank, a.workload)
    if a.mix == "c4":
        workload += "+C4-mix-150bp-20kb"
    fq = make_reads(index_dir, a.reads, 1000 + rank, a.mean_len, a.mix, world)
    import torch
    assert torch.cuda.is_available(), "bench.py needs an MI355X"
    # one process per GPU; more ranks than GPUs (a rehearsal on a 1-GPU box) share devices
    local = local % max(1, torch.cuda.device_count())
    os.environ["DSB_DEVICE"] = str(local)
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = os.environ.get("DSB_DIST_BACKEND", "nccl")  # nccl == RCCL on ROCm
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    import pydesamba
    import shard

    if dist:
        dist.barrier()
    t = time.time()
    idx = pydesamba.Index(index_dir)
    log(f"rank {rank}: index resident on cuda:{local} in {time.time() - t:.1f}s")
    t = time.time()
    batch = idx.batch(fq)
    log(f"rank {rank}: {batch.n_reads} reads / {batch.n_bases / 1e6:.1f} Mbp resident in HBM "
        f"(parse+upload {batch.upload['ms_h2d']:.0f} ms, {time.time() - t:.1f}s)")
    # the batch holds its own copy of the text: keep only the head the CPU legs use
    if not (a.dropin_all and rank == 0 and world == 1 and not a.no_dropin):
        fq = fastq_head(fq, max(a.cpu_sample, a.cpu_sample_t1, a.t3_reads, a.dropin_reads))
    n_tax = idx.max_tid() + 1
    cdev = "cuda" if (dist is None or dist.get_backend() == "nccl") else "cpu"
    counts = torch.zeros(n_tax, dtype=torch.int64, device=cdev)

    dev_counts = torch.zeros(n_tax, dtype=torch.int64, device="cuda")

    def step():
        tm = batch.run(max_read_l=0)
        # per-read taxa (computed by the classify kernels) reduced to per-taxon counts on the GPU
        batch.taxon_counts(dev_counts, 0)
        counts.copy_(shard.reduce_counts(dev_counts if cdev == "cuda" else dev_counts.cpu(), cdev))
        return tm

    for _ in range(a.warmup):
        step()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tms = [step() for _ in range(a.steps)]
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    el = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
    if dist:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    reads_total = batch.n_reads * world * a.steps
    bases_total = batch.n_bases * world * a.steps
    classified = int(counts[1:].sum().item())

    # ---- roofline of the dominant kernel: algorithmic bytes (work counters of one untimed
    # stats run) per launch / its average HIP-event launch time
    phase_ms = {k: sum(t["ms_phase"][k] for t in tms) / a.steps for k in tms[0]["ms_phase"]}
    dom = max(phase_ms, key=phase_ms.get)
    launches = tms[0]["n_chunks"]
    roof = None
    stats = None
    if not a.no_stats:
        ts = batch.run(max_read_l=0, stats=1)
        tt = batch.run(max_read_l=0, stats=2)  # wave clocks: a run of its own (no counter traffic)
        for ph, c in ts["stats_phase"].items():
            for k in c:
                if k.startswith("t_") and k not in ("t_dpm", "t_dps", "t_fill") or (ph == "delA" and k.startswith("t_")):
                    c[k] = tt["stats_phase"][ph][k]
        per_phase = {}
        hash_lds = phase_ms.get("hash", 0) > 0  # the read hash built in LDS by k_hash_lds before the scoring
        for ph, c in ts["stats_phase"].items():
            b = phase_bytes(c) + (batch.n_bases if ph in ("fast0", "slow0") else 0)
            if ph == "delA" and hash_lds:  # its hash_b counter is k_hash_lds's work
                b -= c["hash_b"]
            # the scoring kernel runs twice per chunk when part A is split (slow reads / the rest)
            nl = (tms[0].get("n_launch_dela") or launches) if ph == "delA" else (tms[0].get("n_launch_phase") or launches)
            ms = phase_ms[ph] / nl
            per_phase[ph] = {"algorithmic_bytes_per_launch": int(b / nl), "avg_launch_ms": round(ms, 3),
                             "launches_per_step": nl,
                             "achieved_GBs": round(b / nl / (ms / 1e3) / 1e9, 3) if ms > 0 else None}
        if hash_lds:
            nl = tms[0].get("n_launch_dela") or launches
            hb = ts["stats_phase"]["delA"]["hash_b"]
            ms = phase_ms["hash"] / nl
            per_phase["hash"] = {"algorithmic_bytes_per_launch": int(hb / nl), "avg_launch_ms": round(ms, 3),
                                 "launches_per_step": nl, "achieved_GBs": round(hb / nl / (ms / 1e3) / 1e9, 3) if ms > 0 else None,
                                 "note": "k_hash_lds: the scoring's read 9-mer hash, head table at the reference's key length "
                                         "+ 12 B per position (node write, head read / write)"}
        # the Bloom probes (1 B per first / second probe, what one 1-byte gather costs
        # is a 64-B sector) ride in the island block: made by k_island_g itself (the default), or
        # by k_seed over every position before a two-lane island scan of its exist bits.  The stats
        # run covers the whole batch (every chunk): per launch = / launches per step.
        isl = ts["stats_phase"]["island"]
        nl_i = tms[0].get("n_launch_phase") or launches
        probes = (isl["ek1"] + isl["ek2"]) / nl_i
        ms_seed = sum(t["ms_seed"] for t in tms) / a.steps / nl_i
        probe_info = {"probes_per_launch": int(probes), "first_probes_per_launch": int(isl["ek1"] / nl_i),
                      "second_probes_per_launch": int(isl["ek2"] / nl_i), "sector_bytes_per_launch": int(64 * probes)}
        if ms_seed > 0:
            sb = probes + (2 * batch.n_bases + ts["seed_positions"] // 8) / nl_i  # probes + both strands' bases + exist bits
            per_phase["seed"] = dict({"algorithmic_bytes_per_launch": int(sb), "avg_launch_ms": round(ms_seed, 3),
                                      "launches_per_step": nl_i,
                                      "achieved_GBs": round(sb / (ms_seed / 1e3) / 1e9, 3),
                                      "sector_GBs": round(64 * probes / (ms_seed / 1e3) / 1e9, 1),
                                      "note": "k_seed: one 1-byte Bloom probe costs a 64-B sector; sector_GBs is that rate"},
                                     **probe_info)
            ib = ts["seed_positions"] // 8 / nl_i  # the exist bits the scan reads
        else:
            ib = probes + 2 * batch.n_bases / nl_i  # the probes + both strands' bases
            per_phase["island"].update(probe_info)
        per_phase["island"]["algorithmic_bytes_per_launch"] = int(ib)
        ms_i = per_phase["island"]["avg_launch_ms"]
        per_phase["island"]["achieved_GBs"] = round(ib / (ms_i / 1e3) / 1e9, 3) if ms_i > 0 else None
        if ms_seed <= 0 and ms_i > 0:
            per_phase["island"]["sector_GBs"] = round(64 * probes / (ms_i / 1e3) / 1e9, 1)
            per_phase["island"]["probes_per_s"] = round(probes / (ms_i / 1e3))
            per_phase["island"]["sector_frac_of_random_line_peak"] = round(
                64 * probes / (ms_i / 1e3) / 1e9 / RANDOM_LINE_PEAK_GBS, 4)
        # no phase can beat the chip: an achieved rate above its peak is an accounting error — recorded
        # in the line (roofline.accounting_error) and on stderr, without losing the run's measurements
        accounting_error = []
        for ph, v in per_phase.items():
            for key in ("achieved_GBs", "sector_GBs"):
                if v.get(key) is not None and v[key] > HBM_PEAK_GBS:
                    accounting_error.append(f"{ph} {key} {v[key]} > {HBM_PEAK_GBS} GB/s")
                    print(f"[bench] roofline accounting error: {accounting_error[-1]}", file=sys.stderr)
        tj = None
        tf = os.path.join(ROOT, "profiles", "traffic.json")
        if os.path.exists(tf):
            with open(tf) as f:
                tj = json.load(f)
            if not (tj.get("workload") == workload and tj.get("reads") == a.reads):
                tj = None

        def traffic_of(ph):
            """PMC HBM bytes per launch of phase ph's kernel (profiles/traffic.json): (guide-corrected,
            random-access calibrated), or (None, None)"""
            for ent in (tj or {}).get("kernels") or []:
                # rocprof names carry the stats template argument ("k_wave_phase<8, 0>"): compare without it
                tk = re.sub(r"<(\d+)(?:, \d+)*>", r"<\1>", ent.get("kernel") or "")
                if tk == KERNEL_OF.get(ph):
                    return ent.get("hbm_bytes_per_launch"), ent.get("hbm_bytes_per_launch_calibrated")
            return None, None

        def roof_of(ph):
            d = per_phase[ph]
            traffic, traffic_cal = traffic_of(ph)
            rand = None
            if traffic_cal and d["avg_launch_ms"] > 0:
                ra = traffic_cal / (d["avg_launch_ms"] / 1e3) / 1e9
                rand = {"achieved": round(ra, 1), "peak": round(RANDOM_LINE_PEAK_GBS, 1), "unit": "GB/s",
                        "frac": round(ra / RANDOM_LINE_PEAK_GBS, 4),
                        "note": "PMC HBM bytes per launch (FETCH_SIZE + WRITE_SIZE, the random-access calibration) "
                                "over the measured random 64-B line rate; the kernel's time is set by dependent "
                                "random transactions, not by streamed bytes (DESIGN.md section 6)"}
            ab = d["algorithmic_bytes_per_launch"]
            return {"bound": "hbm", "achieved": d["achieved_GBs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(d["achieved_GBs"] / HBM_PEAK_GBS, 6), "traffic": traffic,
                    "traffic_calibrated": traffic_cal,
                    "traffic_ratio": round(traffic / ab, 2) if traffic and ab else None,
                    "traffic_calibrated_ratio": round(traffic_cal / ab, 2) if traffic_cal and ab else None,
                    "random_access": rand, "kernel": KERNEL_OF[ph], "phase": ph, "algorithmic_bytes_per_launch": ab,
                    "launches_per_step": d["launches_per_step"], "avg_launch_ms": d["avg_launch_ms"],
                    "ms_per_step": round(phase_ms[ph], 2)}

        roof = roof_of(dom)
        # the kernels whose step time is within 10% of the dominant one's (fast seeding and scoring
        # trade places from run to run on the C2 proxy): each with its own roofline
        roof["near_tied"] = [roof_of(ph) for ph in sorted(phase_ms, key=phase_ms.get, reverse=True)
                             if ph != dom and ph in per_phase and phase_ms[ph] >= 0.9 * phase_ms[dom]]
        # the whole step: every kernel's algorithmic bytes over the step's wall time
        step_bytes = sum(v["algorithmic_bytes_per_launch"] * v["launches_per_step"] for k, v in per_phase.items()
                         if k != "seed" or ms_seed > 0)
        step_s = elapsed / a.steps
        roof["step"] = {"algorithmic_bytes_per_step": int(step_bytes), "ms_per_step": round(step_s * 1e3, 2),
                        "achieved": round(step_bytes / step_s / 1e9, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(step_bytes / step_s / 1e9 / HBM_PEAK_GBS, 4)}
        roof["phases"] = per_phase
        roof["traffic_profile"] = (tj or {}).get("tag")
        if accounting_error:
            roof["accounting_error"] = accounting_error
        stats = {"phases": ts["stats_phase"], "classB": ts["stats_B"]}

    cpu = dropin = t3 = None
    n_d = min(a.dropin_reads, batch.n_reads)
    fq_d = fastq_head(fq, n_d)
    if rank == 0 and world == 1:
        import pydesamba as P
        n_s = min(a.cpu_sample, batch.n_reads)
        if not a.no_cpu:
            n_t3 = min(a.t3_reads, batch.n_reads)
            t3 = t3_check(index_dir, fastq_head(fq, n_t3), batch.format_range(0, n_t3, P.FMT_SAM))
            cpu = cpu_baseline(index_dir, fq, n_s, min(a.cpu_sample_t1, batch.n_reads),
                               batch.format_range(0, n_s, P.FMT_SAM))
        if not a.no_dropin:
            dropin = dropin_leg(idx, fq_d, n_d, n_bases(fq_d), batch.format_range_hash(0, n_d, P.FMT_SAM_FULL, digest))
            if a.dropin_all and batch.n_reads > n_d:
                # the whole batch in one call (the consumer-facing rate at the config's size)
                dropin["all_reads"] = dropin_leg(idx, fq, batch.n_reads, batch.n_bases,
                                                 batch.format_range_hash(0, batch.n_reads, P.FMT_SAM_FULL, digest),
                                                 calls=2)
    elif world > 1 and not a.no_dropin:
        # every rank: one read_classify over its own reads at the same time (after a barrier);
        # aggregate = all ranks' reads / the slowest rank's call
        import pydesamba as P
        full = batch.format_range_hash(0, n_d, P.FMT_SAM_FULL, digest)
        dist.barrier()
        mine = dropin_leg(idx, fq_d, n_d, n_bases(fq_d), full)
        t_s = torch.tensor([mine["secs"]], dtype=torch.float64, device=cdev)
        t_ok = torch.tensor([float(mine["identical_to_batch_records"] is True)], dtype=torch.float64, device=cdev)
        dist.all_reduce(t_s, op=dist.ReduceOp.MAX)
        dist.all_reduce(t_ok, op=dist.ReduceOp.MIN)
        secs, same = float(t_s.item()), bool(t_ok.item())
        if rank == 0:
            dropin = {"value": round(n_d * world / secs, 1), "unit": "reads/s", "secs": round(secs, 4),
                      "reads": n_d * world, "ranks": world, "identical_to_batch_records": same,
                      "rank0": mine,
                      "what": f"every rank: read_classify over the first {n_d} of its reads at once; slowest rank's time"}

    if rank == 0:
        value = reads_total / elapsed
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "reads/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": ("synthetic ONT reads (tools/simulate.py, lognormal mean 8 kb, 5-15% error)" if a.mix == "ont" else
                     "synthetic C4 mix (tools/simulate.py: 150 bp 1% error + ONT lognormal mean 20 kb, 1:1 interleaved)")
                    + " from a synthetic reference",
            "config": {"workload": workload, "index": index_info(index_dir), "reads_per_rank": batch.n_reads, "mbases_per_rank": round(batch.n_bases / 1e6, 2),
                       "mean_len": round(batch.n_bases / max(1, batch.n_reads)), "read_mix": a.mix, "parallelism": f"reads sharded over {world} GPU(s), index replicated",
                       "taxon_reduce": f"all_reduce({dist.get_backend()})" if world > 1 else "none"},
            "gbases_per_s": round(bases_total / elapsed / 1e9, 4),
            "classified_reads": classified,
            "chunks": tms[0]["n_chunks"], "retried_reads": tms[0]["n_retry"], "heavy_first_reads": tms[0]["n_heavy"],
            "phase_ms": {k: round(sum(t[k] for t in tms) / a.steps, 2)
                         for k in ("ms_encode", "ms_seed", "ms_classA", "ms_classB", "ms_d2h", "ms_total")},
            "phase_ms_classA": {k: round(v, 2) for k, v in phase_ms.items()},
            "roofline": roof,
            "cpu_baseline": cpu,
            "dropin": dropin,
        }
        if t3:
            line["t3_mismatch"] = t3["t3_mismatch"]
            line["t3_check"] = t3
        if cpu:
            line["vs_cpu_baseline"] = round(value / cpu["value"], 2)
            if cpu.get("taxid_check_vs_gpu"):
                line["taxid_mismatch"] = cpu["taxid_check_vs_gpu"]["taxid_mismatch"]
            if dropin and cpu.get("read_classify"):
                line["dropin_vs_reference_read_classify"] = round(dropin["value"] / cpu["read_classify"]["value"], 2)
        if stats:
            line["work_counters"] = stats
        print(json.dumps(line), flush=True)
    batch.close()
    idx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
