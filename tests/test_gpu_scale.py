"""GPU parity beyond the fixture: the larger-index parameters of BASELINE configs C2-C4, C4's
read mix, and one read_classify call spread over several GPU contexts.

* The C2 proxy itself (tools/simulate.py preset c2: 495 Mbp, 286 M distinct 31-mers, so the
  builder picks l_ek 17 / MASK_31; ~0.5 G BWT rows over 30 occ superblocks), built on the box by
  tools/proxy_build.py (simulate.py + this repo's desamba_index, byte-identical to the reference
  builder on this preset) unless DSB_C2_DIR points at one; the reference classifier
  (oracle/_ref/herm_classify) is the oracle on it.
* Every e-kmer table size of the reference's range (set_ekmer_par / get_EXIST_kmer, reference
  src/idx.c:966-996; utils.h:88-95): the builder switches to larger tables as the distinct 31-mer
  count grows (0.5 GB at >= 477 M, 1 GB at >= 954 M, 4 GB at >= 3.8 G, 16 GB at >= 15.3 G, i.e.
  RefSeq- to nt-scale indexes).  Indexes that large cannot be built here, so the box rebuilds the
  C1 proxy's tables at each size with oracle/_ref/ekmer_tables, this repo's restatement of the
  builder's get_EXIST_kmer, which is byte-identical to the builder's own l_ek-16 tables (fixture,
  C1) and l_ek-17 tables (C2 proxy: tests/test_oracle_pinned.py, profiles/r03_c2/ekmer_check.txt).
  The reference classifier loads such an index exactly as it would a builder-made one (it reads
  e_kmer_size from .exki and calls set_ekmer_par, idx.c:1108-1120), and is the oracle on it.
* BASELINE C4's read mix: 150 bp Illumina-like + ONT-like reads of mean 20 kb, interleaved in a
  fixed order, after a run of short reads: the carried max_read_l (src/cly.c:2953-2963) switches
  from the Illumina rules to the long-read rule inside the input, and 20 kb+ reads take the
  2^15-2^17-bucket read 9-mer hashes (src/cly.c:2160-2219).
* DSB_DEVICES=0,0: the index loaded twice on one GPU, so read_classify's batches alternate
  between two device contexts and the carry chain crosses them, as on an 8-GPU node.
"""
import os
import shutil
import subprocess
import sys
import tarfile

import pytest

from conftest import ROOT, golden
from samutil import compare, groups

pytestmark = pytest.mark.gpu

HERM = os.path.join(ROOT, "oracle", "_ref", "herm_classify")
GCC = os.path.join(ROOT, "oracle", "_ref", "ref_classify")
EKTAB = os.path.join(ROOT, "oracle", "_ref", "ekmer_tables")
C1 = os.path.join(ROOT, "data", "c1_index.txz")


def _need(*paths):
    for p in paths:
        if not os.path.exists(p):
            pytest.skip(f"{os.path.relpath(p, ROOT)} absent")


@pytest.fixture(scope="module")
def c1_dir(tmp_path_factory):
    _need(C1)
    d = tmp_path_factory.mktemp("c1s")
    with tarfile.open(C1) as t:
        t.extractall(d)
    return str(d)


def _host_bytes_available():
    """Host memory this process may still use: MemAvailable, capped by the cgroup limit."""
    avail = None
    with open("/proc/meminfo") as f:
        for line in f:
            if line.startswith("MemAvailable:"):
                avail = int(line.split()[1]) * 1024
    try:
        with open("/sys/fs/cgroup/memory.max") as f:
            v = f.read().strip()
        if v != "max":
            with open("/sys/fs/cgroup/memory.current") as f:
                cur = int(f.read())
            avail = min(avail, int(v) - cur) if avail is not None else int(v) - cur
    except (OSError, ValueError):
        pass
    return avail


def _ek_index(c1_dir, tmp_path_factory, size, l_ek):
    """The C1 proxy with e-kmer tables of `size` bytes per table (oracle/_ref/ekmer_tables)."""
    _need(EKTAB)
    need = 5 * size + (8 << 30)  # both tables written, then read by two reference runs and load_index
    avail = _host_bytes_available()
    if avail is not None and avail < need:
        pytest.skip(f"host memory short for 2 x {size >> 20} MB e-kmer tables: {avail >> 30} GiB available, "
                    f"{need >> 30} GiB needed")
    free_disk = shutil.disk_usage(str(tmp_path_factory.getbasetemp())).free
    if free_disk < 2 * size + (4 << 30):
        pytest.skip(f"disk short for 2 x {size >> 20} MB e-kmer tables: {free_disk >> 30} GiB free")
    d = tmp_path_factory.mktemp(f"c1_ek{size >> 20}M")
    for f in os.listdir(c1_dir):
        if not f.startswith("deSAMBA.exk"):
            os.symlink(os.path.join(c1_dir, f), os.path.join(d, f))
    r = subprocess.run([EKTAB, c1_dir, str(size), str(d)], capture_output=True, text=True, check=True, timeout=600)
    assert f"l_ek {l_ek}," in r.stdout, r.stdout
    with open(os.path.join(d, "deSAMBA.exki"), "rb") as f:
        assert int.from_bytes(f.read(8), "little") == size
    return d


@pytest.fixture(scope="module")
def lek17_dir(c1_dir, tmp_path_factory):
    """The C1 proxy with the quarter-GB l_ek-17 / MASK_31 e-kmer tables."""
    d = _ek_index(c1_dir, tmp_path_factory, 1 << 28, 17)
    yield str(d)
    shutil.rmtree(d, ignore_errors=True)


def _sim(index_dir, tmp_path, n, seed, mix):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import simulate
    genomes = simulate.read_fasta_genomes_from_index(index_dir)
    if mix == "c4":
        lead = list(simulate.simulate_reads(genomes, 20, seed + 7, "illumina"))  # short reads first
        reads = lead + list(simulate.simulate_c4_mix(genomes, n, seed))
    else:
        reads = list(simulate.simulate_reads(genomes, n, seed, "ont", 8000))
    fq = tmp_path / f"{mix}_{seed}.fq"
    simulate.write_fastq(reads, str(fq))
    return fq


def _check_vs_reference(pyd, index_dir, fq, seed, tag):
    """T1 on every read, T2 on every read two reference builds agree on, T3 bounded (the
    uninitialised-memory reads of SURVEY Appendix A H1) — as tests/test_gpu_c1.py."""
    _need(HERM, GCC)
    # both reference builds run while the GPU classifies (each loads the index itself)
    ph = subprocess.Popen([HERM, "--sam", index_dir, str(fq)], stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    pg = subprocess.Popen([GCC, "--sam", "--fresh", index_dir, str(fq)], stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    try:
        idx = pyd.Index(index_dir)
        try:
            out, t, _ = idx.classify(fq.read_bytes(), fmt=1, stats=True)
        finally:
            idx.close()
        herm, eh = ph.communicate(timeout=900)
        t1, eg = pg.communicate(timeout=900)
    finally:
        for p in (ph, pg):
            if p.poll() is None:
                p.kill()
                p.wait()
    assert ph.returncode == 0, eh[-400:]
    assert pg.returncode == 0, eg[-400:]
    r = compare(herm, out)
    assert r["taxid_mismatch"] == 0 and r["mapped_mismatch"] == 0, (tag, seed, r)
    gh, gt, go = groups(herm), groups(t1), groups(out)
    stable = [i for i in range(len(gh)) if gh[i] == gt[i]]
    assert len(stable) >= 0.9 * len(gh), (tag, seed, len(stable))
    bad = [gh[i][0] for i in stable if go[i] != gh[i]]
    assert not bad, (tag, seed, bad[:5])
    unstable = [gh[i][0] for i in range(len(gh)) if go[i] != gh[i]]
    assert len(unstable) <= 0.005 * len(gh), (tag, seed, unstable[:5])
    print(f"{tag} seed {seed}: {len(gh)} reads, {len(stable)} stable, T3 mismatches {len(unstable)}")
    return t


def test_lek17_mask31_index_matches_reference(pyd, lek17_dir, tmp_path):
    seed = int(os.environ.get("DSB_TEST_SEED", 5151 + int.from_bytes(os.urandom(2), "little")))
    fq = _sim(lek17_dir, tmp_path, 2000, seed, "ont")
    t = _check_vs_reference(pyd, lek17_dir, fq, seed, "C1-lek17")
    assert t["seed_positions"] > 0


# the reference's larger table sizes (src/idx.c:966-982): (bytes per table, l_ek, hash mask bits)
EK_SIZES = [(1 << 29, 17, 32), (1 << 30, 18, 33), (1 << 32, 19, 35), (1 << 34, 20, 37)]


@pytest.mark.parametrize("size,l_ek,mask_bits", EK_SIZES, ids=[f"lek{l}_mask{m}_{s >> 20}MB" for s, l, m in EK_SIZES])
def test_ekmer_table_sizes_match_reference(pyd, c1_dir, tmp_path_factory, tmp_path, size, l_ek, mask_bits):
    """l_ek 17-20 with 0.5-16 GB Bloom tables: probe offsets up to 2^37 bits (hash64_1/2 & MASK_37,
    byte offset h >> 3 up to 2^34) against the reference classifier on the same index, T1/T2 on
    every read and T3 bounded, on 1000 fresh reads."""
    assert size * 8 == 1 << mask_bits
    d = _ek_index(c1_dir, tmp_path_factory, size, l_ek)
    try:
        seed = int(os.environ.get("DSB_TEST_SEED", 8181 + l_ek + int.from_bytes(os.urandom(2), "little")))
        fq = _sim(str(d), tmp_path, 1000, seed, "ont")
        t = _check_vs_reference(pyd, str(d), fq, seed, f"C1-lek{l_ek}-mask{mask_bits}")
        assert t["seed_positions"] > 0 or t["stats"]["ek1"] > 0
    finally:
        shutil.rmtree(d, ignore_errors=True)


def test_reads_over_65kb_match_reference(pyd, c1_dir, tmp_path):
    """Reads of 66-100 kb (C4's ONT tail): the reference's read buffer
    realloc(NULL, 2L + 20) (BUFF_REALLOC, src/lib/utils.h:117-122) is then above glibc's 128 KB
    mmap threshold, so the 8 bytes in front of the forward read are an mmapped chunk's header, not
    the heap chunk header dsb_chunk_header models; they matter only to a backward extension that
    runs past the read's first base into them.  These reads also take the 2^17-2^18-key read hashes
    of the reference (and the LDS build's 2^13 keys here).  T1 / T2 on every read, T3 bounded,
    against the hermetic reference, with the long reads interleaved among 8 kb ones."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import simulate
    seed = int(os.environ.get("DSB_TEST_SEED", 9191 + int.from_bytes(os.urandom(2), "little")))
    genomes = simulate.read_fasta_genomes_from_index(c1_dir)
    longs = list(simulate.simulate_reads(genomes, 40, seed, "ont", 80000, min_len=66000, max_len=100000))
    shorts = list(simulate.simulate_reads(genomes, 200, seed + 1, "ont", 8000))
    reads = []
    for i, r in enumerate(shorts):
        reads.append(r)
        if i % 5 == 4 and longs:
            reads.append(longs.pop())
    reads.extend(longs)
    lens = [len(r[1]) for r in reads]
    assert sum(L >= 65526 for L in lens) >= 30, sorted(lens)[-5:]  # 2L + 20 >= 128 KB
    fq = tmp_path / f"long_{seed}.fq"
    simulate.write_fastq(reads, str(fq))
    _check_vs_reference(pyd, c1_dir, fq, seed, "C1-reads-over-65kb")


def test_c4_mix_150bp_20kb_interleaved_matches_reference(pyd, c1_dir, tmp_path):
    seed = int(os.environ.get("DSB_TEST_SEED", 6161 + int.from_bytes(os.urandom(2), "little")))
    fq = _sim(c1_dir, tmp_path, 1000, seed, "c4")
    lens = [len(l) for i, l in enumerate(fq.read_bytes().split(b"\n")) if i % 4 == 1]
    assert min(lens) == 150 and max(lens) >= 32768  # 2^16+ bucket read hashes
    _check_vs_reference(pyd, c1_dir, fq, seed, "C4-mix")


def test_read_classify_over_two_device_contexts(pyd, fixture_index):
    """DSB_DEVICES=0,0: batches of one read_classify call alternate between two contexts holding
    the index; records and the carried max_read_l equal the single-context call."""
    os.environ["DSB_DEVICES"] = "0,0"
    os.environ["DSB_GPU_CONTEXTS"] = "1"
    os.environ["DSB_PIPE_READS"] = "41"
    try:
        idx = pyd.Index(fixture_index)
        try:
            assert idx.devices() == [0, 0]
            assert idx.read_classify(golden("mixed.fq"), thread_id=3) == golden("mixed.herm.sam_full")
            for name in ("mixed", "ont_long"):
                out, t, _ = idx.classify(golden(name + ".fq"), fmt=pyd.FMT_SAM)
                assert out == golden(name + ".herm.sam"), name
                assert t["n_devices"] == 2 and t["n_batches"] >= 2
        finally:
            idx.close()
    finally:
        os.environ.pop("DSB_DEVICES", None)
        os.environ.pop("DSB_GPU_CONTEXTS", None)
        os.environ.pop("DSB_PIPE_READS", None)


def test_default_two_contexts_share_one_index_copy(gpu_index, pyd):
    """load_index's default: two contexts on the GPU sharing one copy of the index tables
    (DSB_GPU_CONTEXTS=2), batches of one call alternating between them."""
    devs = gpu_index.devices()
    assert len(devs) == 2 and devs[0] == devs[1]
    os.environ["DSB_PIPE_READS"] = "64"
    try:
        out, t, _ = gpu_index.classify(golden("ont.fq"), fmt=pyd.FMT_SAM)
        assert out == golden("ont.herm.sam")
        assert t["n_devices"] == 2 and t["n_batches"] >= 30
    finally:
        os.environ.pop("DSB_PIPE_READS", None)


@pytest.fixture(scope="module")
def c2_dir():
    """The C2 proxy index: DSB_C2_DIR when set, else built here by tools/proxy_build.py
    (simulate.py preset c2 + desamba-so_amd/bin/desamba_index, ~60 s on the GPU box's host,
    cached under $TMPDIR for the rest of the call)."""
    d = os.environ.get("DSB_C2_DIR")
    if d and os.path.exists(os.path.join(d, "deSAMBA.bwt")):
        return d
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import proxy_build
    _need(proxy_build.BUILDER)
    return proxy_build.ensure_proxy("c2")


def test_c2_proxy_matches_reference(pyd, c2_dir, tmp_path):
    """The C2-direction proxy (tools/simulate.py preset c2: 495 Mbp, 286 M distinct 31-mers ->
    l_ek 17, MASK_31, 256 MB e-kmer tables, ~0.5 G BWT rows over 30 occ superblocks): T1/T2 on
    every read, T3 bounded, against the reference classifier on 2000 fresh ONT reads and 600
    reads of C4's mix."""
    d = c2_dir
    with open(os.path.join(d, "deSAMBA.exki"), "rb") as f:
        assert int.from_bytes(f.read(8), "little") == 1 << 28  # the builder chose l_ek 17 / MASK_31
    seed = int(os.environ.get("DSB_TEST_SEED", 7171 + int.from_bytes(os.urandom(2), "little")))
    fq = _sim(d, tmp_path, 2000, seed, "ont")
    _check_vs_reference(pyd, d, fq, seed, "C2-proxy")
    fq4 = _sim(d, tmp_path, 600, seed + 1, "c4")
    _check_vs_reference(pyd, d, fq4, seed + 1, "C2-proxy-C4-mix")


def test_c2_lek18_proxy_matches_reference(pyd, tmp_path):
    """The next size class of the reference's builder: tools/simulate.py preset c2l18 (1.86 Gbp,
    ~1.06 G distinct 31-mers >= 2^33 / 9), built on the box by this repo's desamba_index, so the
    builder itself picks 1 GB e-kmer tables, l_ek 18 and MASK_33 (reference src/idx.c:966-996) over a
    1.94 G-row BWT (116 occ superblocks) — a real index of that class, not C1's BWT with rebuilt
    tables.  T1/T2 on every read, T3 bounded, against the reference classifier on 1000 fresh ONT
    reads."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import proxy_build
    _need(proxy_build.BUILDER)
    avail = _host_bytes_available()
    if avail is not None and avail < (96 << 30):
        pytest.skip(f"host memory short for the c2l18 build: {avail >> 30} GiB available")
    d = os.environ.get("DSB_C2L18_DIR") or proxy_build.ensure_proxy("c2l18")
    with open(os.path.join(d, "deSAMBA.exki"), "rb") as f:
        assert int.from_bytes(f.read(8), "little") == 1 << 30  # the builder chose l_ek 18 / MASK_33
    with open(os.path.join(d, "deSAMBA.bwt"), "rb") as f:
        rows = int.from_bytes(f.read(8), "little") // 168 * 256
    assert rows >= 954_000_000, rows
    seed = int(os.environ.get("DSB_TEST_SEED", 7272 + int.from_bytes(os.urandom(2), "little")))
    fq = _sim(d, tmp_path, 1000, seed, "ont")
    _check_vs_reference(pyd, d, fq, seed, "C2-lek18-proxy")


def test_c2_lek18_qbuff_byte_read_set(pyd, tmp_path):
    """Round 5's one stable-read divergence, now modelled: read rd0_9305_487078_+_5 of the c2l18 read
    set with seed 49921.  One seed maps at the read start (q 2) to the four copies of family 269;
    the left get_new_ed window is one base (read C, reference A), so lv_extd's result depends on the
    byte before q_buff (src/cly.c:589, 635).  In the hermetic reference that byte is 0xAA for the
    first REF_POS item and 0x00 after the first push that grew the anchor vector (glibc realloc's
    frame): edit distance 1, then 0, 0, 0.  The GPU follows it (dsb_left_lv,
    dsb_map_seed; the wave seeding replays such seeds in order) and the whole set is T1/T2/T3-exact."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import proxy_build
    _need(proxy_build.BUILDER)
    avail = _host_bytes_available()
    if avail is not None and avail < (96 << 30):
        pytest.skip(f"host memory short for the c2l18 build: {avail >> 30} GiB available")
    d = os.environ.get("DSB_C2L18_DIR") or proxy_build.ensure_proxy("c2l18")
    fq = _sim(d, tmp_path, 1000, 49921, "ont")
    _check_vs_reference(pyd, d, fq, 49921, "C2-lek18-divergence")


def test_c2_lek18_qbuff_byte_with_dirty_workspace(tmp_path):
    """The same read set with every read's workspace filled with 0x5A before the kernels run
    (DSB_TEST_WS_FILL, test library), alone and with every seed group replayed in order
    (DSB_WAVE_DBG=32, so every map_seed is the sequential one, which reads the per-read anchor-vector
    high-water mark).  Round 6 found that field left uninitialised by the island kernel: fresh
    workspaces read 0 and passed, but in a 1M-read c2l18 batch the re-run reads met an earlier read's
    bytes there and four of them ended in M3's NULL case (status 8).  Byte-identical to the clean run
    and to the hermetic reference."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import proxy_build
    from test_gpu_hooks import run_worker
    _need(proxy_build.BUILDER)
    avail = _host_bytes_available()
    if avail is not None and avail < (96 << 30):
        pytest.skip(f"host memory short for the c2l18 build: {avail >> 30} GiB available")
    d = os.environ.get("DSB_C2L18_DIR") or proxy_build.ensure_proxy("c2l18")
    fq = _sim(d, tmp_path, 1000, 49921, "ont")
    _need(HERM)
    herm = subprocess.run([HERM, "--sam", d, str(fq)], capture_output=True, check=True, timeout=900).stdout
    for env in ({"DSB_TEST_WS_FILL": "0x5A"}, {"DSB_TEST_WS_FILL": "0x5A", "DSB_WAVE_DBG": "32"}):
        outs, _ = run_worker(tmp_path, "fill" + env.get("DSB_WAVE_DBG", ""), d, [fq], env)
        bad = [a[0] for a, b in zip(groups(herm), groups(outs[0])) if a != b]
        assert not bad, (env, bad[:5])


@pytest.mark.timeout(900)  # the build takes ~4 min on the box's 16 cores (8 before round 6's builder changes)
def test_c2xl_proxy_past_2_32_rows_matches_reference(pyd, tmp_path):
    """The C2 scale: tools/simulate.py preset c2xl (~5 Gbp, ~2.8 G distinct 31-mers, 2 GB e-kmer
    tables, l_ek 18) built on the box by desamba_index, whose BWT passes 2^32 rows (~17 GB index):
    occ superblocks, SA samples, LF steps and the relayout's chain checks past the u32 range, in a
    real index classified end to end.  T1/T2 on every read, T3 bounded, against the reference
    classifier on 1000 fresh ONT reads.  Part of the default GPU suite since round 6 (the builder's
    unitig walks, SA walk and merges got faster); needs ~120 GB of host memory (skipped below that);
    DSB_C2XL_DIR names a prebuilt index, DSB_SKIP_C2XL=1 skips it."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import proxy_build
    _need(proxy_build.BUILDER)
    d = os.environ.get("DSB_C2XL_DIR")
    if not d:
        avail = _host_bytes_available()
        if avail is not None and avail < (150 << 30):
            pytest.skip(f"host memory short for the c2xl build: {avail >> 30} GiB available")
        if os.environ.get("DSB_SKIP_C2XL"):
            pytest.skip("DSB_SKIP_C2XL set")
        d = proxy_build.ensure_proxy("c2xl")
    with open(os.path.join(d, "deSAMBA.bwt"), "rb") as f:
        rows = int.from_bytes(f.read(8), "little") // 168 * 256
    assert rows > 1 << 32, rows
    seed = int(os.environ.get("DSB_TEST_SEED", 9191 + int.from_bytes(os.urandom(2), "little")))
    fq = _sim(d, tmp_path, 1000, seed, "ont")
    _check_vs_reference(pyd, d, fq, seed, "C2-xl-proxy")
