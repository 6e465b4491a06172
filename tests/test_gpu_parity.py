"""GPU parity: the HIP classify path (through the C-ABI) against the reference oracle.

Goldens were produced by the reference itself (tools/make_goldens.sh):
  *.herm.*  hermetic reference build (fresh buffer pools, MALLOC_PERTURB 165, clang pattern
            stack init, -t1 max_read_l carry) — the T3 contract: byte-identical records.
  *.t1.*    `deSAMBA classify -t 1` — the T1 contract: identical primary taxid and mapped
            flag for 100 % of reads; full records identical except reads whose reference
            output depends on uninitialised memory.
"""
import gzip
import os
import subprocess
import sys

import pytest

from conftest import GOLDEN, ROOT, golden
from samutil import ana_get_tid, compare, groups, read_parents

pytestmark = pytest.mark.gpu

SETS = ["mixed", "ont", "ont_long", "illumina"]


def test_read_classify_sam_full_is_byte_identical_to_hermetic_reference(gpu_index):
    out = gpu_index.read_classify(golden("mixed.fq"), thread_id=0, thread_num=1)
    assert out == golden("mixed.herm.sam_full")


@pytest.mark.parametrize("name", SETS)
def test_sam_records_identical_to_hermetic_reference(gpu_index, pyd, name):
    out, timing, _ = gpu_index.classify(golden(name + ".fq"), fmt=pyd.FMT_SAM)
    ref = golden(name + ".herm.sam")
    r = compare(ref, out)
    assert r["full_mismatch"] == 0, r
    assert out == ref
    assert timing["n_reads"] > 0


@pytest.mark.parametrize("name", SETS)
def test_taxid_and_mapping_identical_to_reference_t1(gpu_index, pyd, name):
    """T1: primary taxid + mapped flag identical to `deSAMBA classify -t 1` for every read."""
    out, _, _ = gpu_index.classify(golden(name + ".fq"), fmt=pyd.FMT_SAM)
    r = compare(golden(name + ".t1.sam"), out)
    assert r["taxid_mismatch"] == 0, r
    assert r["mapped_mismatch"] == 0, r


@pytest.mark.parametrize("name", SETS)
def test_full_records_identical_to_reference_t1_on_stable_reads(gpu_index, pyd, name):
    """T2: every read whose -t1 record set equals the hermetic reference's (i.e. does not
    depend on uninitialised memory) is byte-identical to -t1."""
    out, _, _ = gpu_index.classify(golden(name + ".fq"), fmt=pyd.FMT_SAM)
    t1, herm, got = groups(golden(name + ".t1.sam")), groups(golden(name + ".herm.sam")), groups(out)
    assert len(t1) == len(herm) == len(got)
    stable = [i for i in range(len(t1)) if t1[i] == herm[i]]
    assert len(stable) >= 0.9 * len(t1)
    bad = [i for i in stable if got[i] != t1[i]]
    assert not bad, bad[:10]


@pytest.mark.parametrize("name", ["mixed", "ont"])
@pytest.mark.parametrize("fmt", ["des", "des_full"])
def test_des_formats_byte_identical_to_hermetic_reference(gpu_index, pyd, name, fmt):
    """DES / DES_FULL records (output_one_result_des / _full, reference src/cly_mt.c:144-227)
    against the hermetic reference's own writers (oracle harness --des / --des-full)."""
    code = pyd.FMT_DES if fmt == "des" else pyd.FMT_DES_FULL
    out, _, _ = gpu_index.classify(golden(name + ".fq"), fmt=code)
    assert out == golden(f"{name}.herm.{fmt}")


def test_des_format_matches_reference_t1(gpu_index, pyd):
    out, _, _ = gpu_index.classify(golden("mixed.fq"), fmt=pyd.FMT_DES)
    ref = golden("mixed.t1.des").split(b"\n\n")
    got = out.split(b"\n\n")
    assert len(ref) == len(got)
    same = sum(a == b for a, b in zip(ref, got))
    assert same >= 0.95 * len(ref)


def test_trailing_nul_input_like_main_test_2(gpu_index, fixture_index, tmp_path):
    """The reference's in-memory consumer passes input_n = fsize + 1, i.e. the text plus its
    terminating NUL (reference main_test_2.c:73).  With a final newline the NUL is skipped by
    kseq's header scan; without one it joins the last quality line, whose length then differs
    from the sequence's and kseq drops that record (utils.c:939-977).  Both against the
    hermetic reference run on this box over files holding the same bytes."""
    herm = os.path.join(ROOT, "oracle", "_ref", "herm_classify")
    if not os.path.exists(herm):
        pytest.skip("oracle/_ref not built")
    fq = golden("ont.fq")[:400000]
    fq = fq[: fq.rindex(b"\n@") + 1]  # whole records
    for data in (fq + b"\0", fq[:-1] + b"\0"):
        p = tmp_path / "nul.fq"
        p.write_bytes(data)
        ref = subprocess.run([herm, fixture_index, str(p)], capture_output=True, check=True, timeout=300).stdout
        got = gpu_index.read_classify(data, thread_id=31, thread_num=4)
        assert got == ref
    assert gpu_index.read_classify(fq + b"\0", thread_id=32) == gpu_index.read_classify(fq, thread_id=33)


def test_concurrent_read_classify_distinct_thread_ids(gpu_index):
    """Concurrent read_classify calls with distinct thread_ids are part of the contract
    (reference cly_mt.c:1279-1307, desamba.h:20-21): four host threads at once, each output equal
    to the serial call's (ctypes releases the GIL, so the calls overlap in the library)."""
    import threading
    inputs = [golden(n + ".fq") for n in ("mixed", "ont", "illumina", "ont_long")]
    serial = [gpu_index.read_classify(d, thread_id=40 + k, thread_num=1) for k, d in enumerate(inputs)]
    got = [None] * len(inputs)
    errs = []

    def work(k):
        try:
            for it in range(2):  # fresh thread_ids: a thread_id carries max_read_l across calls
                got[k] = gpu_index.read_classify(inputs[k], thread_id=50 + 10 * it + k, thread_num=1)
        except Exception as e:  # pragma: no cover
            errs.append(e)

    th = [threading.Thread(target=work, args=(k,)) for k in range(len(inputs))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    assert not errs
    for k in range(len(inputs)):
        assert got[k] == serial[k], k
    assert serial[0] == golden("mixed.herm.sam_full")


def test_concurrent_multi_batch_calls_share_contexts_without_deadlock(gpu_index):
    """Concurrent calls that each span many GPU batches on both device contexts (DSB_PIPE_READS
    41): every batch holds its context's run lock while it waits for the carried max_read_l of
    the batch before, so without the in-order lock hand-out (pipeline.c lock_wait) two calls could
    each hold the lock the other's earlier batch needs.  All calls must finish and equal the
    serial calls."""
    import threading
    inputs = [golden(n + ".fq") for n in ("mixed", "ont", "illumina", "mixed")]
    os.environ["DSB_PIPE_READS"] = "41"
    try:
        serial = [gpu_index.read_classify(d, thread_id=70 + k, thread_num=1) for k, d in enumerate(inputs)]
        got = [None] * len(inputs)
        errs = []

        def work(k):
            try:
                for it in range(3):
                    got[k] = gpu_index.read_classify(inputs[k], thread_id=80 + 10 * it + k, thread_num=1)
            except Exception as e:  # pragma: no cover
                errs.append(e)

        th = [threading.Thread(target=work, args=(k,), daemon=True) for k in range(len(inputs))]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=100)
        assert not any(t.is_alive() for t in th), "concurrent read_classify calls did not finish (deadlock)"
    finally:
        os.environ.pop("DSB_PIPE_READS", None)
    assert not errs
    for k in range(len(inputs)):
        assert got[k] == serial[k], k
    assert serial[0] == golden("mixed.herm.sam_full")


def test_two_calls_carry_pool_state_like_one_call(gpu_index, pyd):
    """max_read_l persists per thread_id across read_classify calls (src/cly.c:2953)."""
    fq = golden("mixed.fq")
    recs = fq.split(b"\n@")
    cut = len(b"\n@".join(recs[:400])) + 1  # a record boundary after the edge-case reads
    one = gpu_index.read_classify(fq, thread_id=11, thread_num=1)
    a = gpu_index.read_classify(fq[:cut], thread_id=12, thread_num=1)
    b = gpu_index.read_classify(fq[cut:], thread_id=12, thread_num=1)
    assert a + b == one


def test_path_mode_and_gzip_input(gpu_index, tmp_path):
    fq = golden("illumina.fq")
    p = tmp_path / "reads.fq.gz"
    with gzip.open(p, "wb") as f:
        f.write(fq)
    via_path = gpu_index.read_classify(str(p), thread_id=21)
    via_gz_bytes = gpu_index.read_classify(p.read_bytes(), thread_id=22)
    via_plain = gpu_index.read_classify(fq, thread_id=23)
    assert via_path == via_plain == via_gz_bytes


def test_empty_input_leaves_output_untouched(gpu_index, pyd):
    import ctypes as C
    L = pyd.lib()
    out, n = C.c_void_p(1234), C.c_uint64(99)
    L.read_classify(gpu_index.h, b"", 0, C.byref(out), C.byref(n), 0, 1)
    assert n.value == 0 and out.value == 1234


def test_meta_analysis_matches_reference(gpu_index):
    sam = golden("mixed.herm.sam_full")
    for flag, gname in [(0, "mixed.meta_reads"), (1, "mixed.meta_bases")]:
        out, snap = gpu_index.meta_analysis(sam, flag=flag, max_snapshot_len=65536, thread_id=0)
        ref_lines = golden(gname).decode().splitlines()
        ref_report = "\n".join(l for l in ref_lines if not l.startswith("#")) + "\n"
        assert out.decode() == ref_report
        meta = dict(l[1:].split("\t", 1) for l in ref_lines if l.startswith("#"))
        assert len(snap) == int(meta["snapshot_n"])
        assert snap[:60].decode() == meta["snapshot_head"]


def test_live_reference_on_fresh_random_reads(gpu_index, fixture_index, tmp_path):
    """Fresh reads (new seed) classified by the compiled reference on this box vs the GPU."""
    herm = os.path.join(ROOT, "oracle", "_ref", "herm_classify")
    if not os.path.exists(herm):
        pytest.skip("oracle/_ref not built")
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import simulate
    genomes = simulate.read_fasta_genomes_from_index(fixture_index)
    seed = int.from_bytes(os.urandom(2), "little")
    fq = tmp_path / "fresh.fq"
    reads = list(simulate.simulate_reads(genomes, 300, seed, "ont", 6000))
    simulate.write_fastq(reads, str(fq))
    ref = subprocess.run([herm, "--sam", fixture_index, str(fq)], capture_output=True, check=True).stdout
    out, _, _ = gpu_index.classify(fq.read_bytes(), fmt=1)
    r = compare(ref, out)
    assert r["full_mismatch"] == 0, (seed, r)


def test_batch_api_matches_one_shot_classify(gpu_index, pyd):
    """dsb_batch_* (reads resident in HBM, repeated runs) == dsb_classify_text."""
    fq = golden("ont.fq")
    b = gpu_index.batch(fq)
    try:
        assert b.n_reads == 2000
        for _ in range(2):
            b.run(max_read_l=0)
            assert b.format(pyd.FMT_SAM) == golden("ont.herm.sam")
    finally:
        b.close()


def test_batch_taxa_match_meta_analysis_rule(gpu_index, fixture_index, pyd):
    parent = read_parents(os.path.join(fixture_index, "nodes.dmp"))
    b = gpu_index.batch(golden("mixed.fq"))
    try:
        b.run(max_read_l=0)
        tid, w = b.taxa(0)
        want = [ana_get_tid(r, parent, gpu_index.max_tid()) for _, r in groups(golden("mixed.herm.sam"))]
        assert list(tid) == want
        assert (w == 1).all()
    finally:
        b.close()


@pytest.mark.parametrize("name", ["mixed", "ont"])
def test_device_taxon_counts_equal_the_meta_analysis_rule(gpu_index, fixture_index, pyd, name):
    """dsb_batch_taxon_counts (per-read taxa from the classB kernel, counted on the GPU) against
    the reference rule applied to the hermetic reference's records, for weights 1 and the read
    length (meta_analysis flag & 1)."""
    import numpy as np
    import torch
    parent = read_parents(os.path.join(fixture_index, "nodes.dmp"))
    n_tax = gpu_index.max_tid() + 1
    b = gpu_index.batch(golden(name + ".fq"))
    try:
        b.run(max_read_l=0)
        want_tid = [ana_get_tid(r, parent, gpu_index.max_tid()) for _, r in groups(golden(name + ".herm.sam"))]
        tid, wl = b.taxa(1)
        assert list(tid) == want_tid
        for flag, w in ((0, None), (1, wl)):
            want = np.bincount(np.array(want_tid, dtype=np.int64), weights=w, minlength=n_tax).astype(np.int64)
            got = b.taxon_counts(torch.full((n_tax,), -7, dtype=torch.int64, device="cuda"), flag).cpu().numpy()
            assert (got == want).all()
    finally:
        b.close()


def test_dlopen_consumer_example(fixture_index, tmp_path):
    """examples/consumer.c (a reference-style dlopen consumer) against the hermetic goldens."""
    exe = tmp_path / "consumer"
    subprocess.run(["gcc", "-O2", "-o", str(exe), os.path.join(ROOT, "examples", "consumer.c"), "-ldl"], check=True)
    fq = tmp_path / "mixed.fq"
    fq.write_bytes(golden("mixed.fq"))
    lib = os.path.join(ROOT, "desamba-so_amd", "lib", "libdesamba.so")
    r = subprocess.run([str(exe), lib, fixture_index, str(fq)], capture_output=True, check=True, timeout=300)
    assert r.stdout == golden("mixed.herm.sam_full")
    ref_lines = golden("mixed.meta_reads").decode().splitlines()
    assert r.stderr.decode().endswith("\n".join(l for l in ref_lines if not l.startswith("#")) + "\n")


def _chimeras(n):
    """Reads that match both strands about equally (a forward half + the reverse complement of
    another read's half), so that classify_seq takes the both_direction branch (FAST1, SLOW1)."""
    comp = bytes.maketrans(b"ACGTN", b"TGCAN")
    lines = golden("ont.fq").split(b"\n")
    seqs = [lines[i + 1] for i in range(0, len(lines) - 3, 4)]
    out = []
    for k in range(n):
        a, b = seqs[(2 * k) % len(seqs)], seqs[(2 * k + 1) % len(seqs)]
        h = min(len(a), len(b)) // 2
        s = a[:h] + b[:h].translate(comp)[::-1]
        out.append(b"@chim%d\n%s\n+\n%s\n" % (k, s, b"I" * len(s)))
    return b"".join(out)


@pytest.mark.parametrize("budget_mb", ["48", "4"])
def test_many_chunks_and_second_strand_passes_byte_identical(gpu_index, fixture_index, pyd, budget_mb, tmp_path):
    """A small workspace budget splits the reads into many chunks that reuse the same workspace
    bytes (the seeding sp_set tables are never cleared: only per-launch slot tags keep them
    exact), and reads matching both strands run FAST1/SLOW1 over the tables FAST0/SLOW0 just
    used.  Goldens: the committed hermetic outputs, and the hermetic reference run on this box
    for the chimeric reads."""
    herm = os.path.join(ROOT, "oracle", "_ref", "herm_classify")
    if not os.path.exists(herm):
        pytest.skip("oracle/_ref not built")
    chim = _chimeras(400)
    fq = tmp_path / "chim.fq"
    fq.write_bytes(chim)
    chim_ref = subprocess.run([herm, "--sam", fixture_index, str(fq)], capture_output=True, check=True,
                              timeout=300).stdout
    os.environ["DSB_WS_BUDGET_MB"] = budget_mb
    try:
        fast1 = slow1 = 0
        for name, data, ref in [("mixed", golden("mixed.fq"), golden("mixed.herm.sam")),
                                ("ont_long", golden("ont_long.fq"), golden("ont_long.herm.sam")),
                                ("chimeras", chim, chim_ref)]:
            out, t, _ = gpu_index.classify(data, fmt=pyd.FMT_SAM, stats=True)
            assert t["n_chunks"] >= 3, (name, t["n_chunks"])
            r = compare(ref, out)
            assert r["full_mismatch"] == 0, (name, r)
            assert out == ref, name
            fast1 += t["stats_phase"]["fast1"]["mem_search"]
            slow1 += t["stats_phase"]["slow1"]["mem_search"]
        assert fast1 > 0
        print(f"FAST1 MEM searches {fast1}, SLOW1 MEM searches {slow1}")
    finally:
        os.environ.pop("DSB_WS_BUDGET_MB", None)


@pytest.mark.parametrize("reads_per_batch,depth", [("37", "2"), ("500", "3"), ("1", "8")])
def test_streaming_batches_byte_identical(gpu_index, pyd, reads_per_batch, depth):
    """read_classify / dsb_classify_text stream the input through GPU batches of at most
    DSB_PIPE_READS reads (pipeline.c); the carried max_read_l crosses every batch boundary
    (reference cly.c:2953, one pool per call) and the records come back in input order.  Tiny
    batches + a shallow or deep pipeline against the hermetic goldens."""
    os.environ["DSB_PIPE_READS"] = reads_per_batch
    os.environ["DSB_PIPE_DEPTH"] = depth
    try:
        for name in ("mixed", "ont_long", "illumina"):
            out, t, _ = gpu_index.classify(golden(name + ".fq"), fmt=pyd.FMT_SAM)
            assert out == golden(name + ".herm.sam"), name
            rpb = int(reads_per_batch)
            first = min(t["n_reads"], -(-rpb // 4))  # the first batch is a quarter size
            assert t["n_batches"] == 1 + -(-(t["n_reads"] - first) // rpb)
            assert t["n_view_records"] + t["n_copied_records"] == t["n_reads"]
        assert gpu_index.read_classify(golden("mixed.fq"), thread_id=61) == golden("mixed.herm.sam_full")
    finally:
        os.environ.pop("DSB_PIPE_READS", None)
        os.environ.pop("DSB_PIPE_DEPTH", None)


def test_single_line_fastq_records_are_views(gpu_index, pyd):
    """Plain single-line FASTQ is classified in place: no record is copied by the parser."""
    _, t, _ = gpu_index.classify(golden("ont.fq"), fmt=pyd.FMT_SAM)
    assert t["n_view_records"] == 2000 and t["n_copied_records"] == 0
