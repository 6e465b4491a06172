"""The index builder (desamba-so_amd/bin/desamba_index) against the reference's.

desamba_index restates `deSAMBA index` (reference src/idx.c:884-1101, 1163-1282; src/bwt.c:106-277)
from the same two inputs (sorted 31-mers, reference FASTA).  Host only.  Pinned here:
  * the committed fixture index (tests/golden/fixture_index.txz, made by the reference builder
    from tools/simulate.py's fixture preset) is rebuilt byte for byte from the regenerated
    inputs — no reference binary needed;
  * on references built to hit the builder's edge cases (N runs, lowercase, ACGT runs of exactly
    30 / 31 / 32 bases, single-k-mer and short unitigs, several sequences, a name with a comment,
    IUPAC codes) the compiled reference builder (oracle/_ref/deSAMBA) and desamba_index write
    the same files (tools/idx_compare.py: bytes the reference leaves undefined excepted);
  * the serial LF walk (the reference's) and the parallel per-unitig walks give the same files.
"""
import os
import random
import struct
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

IDX = os.path.join(ROOT, "desamba-so_amd", "bin", "desamba_index")
REF = os.path.join(ROOT, "oracle", "_ref", "deSAMBA")
CMP = os.path.join(ROOT, "tools", "idx_compare.py")
SIM = os.path.join(ROOT, "tools", "simulate.py")


@pytest.fixture(scope="module")
def builder():
    if not os.path.exists(IDX):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "desamba-so_amd"), "bin/desamba_index"], check=True,
                       timeout=600)
    return IDX


def _build(exe, kmer, fa, out, env=None):
    r = subprocess.run([exe, str(kmer), str(fa), str(out)], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, **(env or {})))
    assert r.returncode == 0, r.stderr[-2000:]
    return r


def _compare(a, b):
    r = subprocess.run([sys.executable, CMP, str(a), str(b)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout
    return r.stdout


def test_fixture_index_rebuilt_byte_identical(builder, fixture_index, tmp_path):
    subprocess.run([sys.executable, SIM, "reference", "--preset", "fixture", "--out", str(tmp_path)], check=True,
                   capture_output=True, timeout=600)
    _build(builder, tmp_path / "kmer.srt", tmp_path / "ref.fa", tmp_path / "idx")
    out = _compare(fixture_index, tmp_path / "idx")
    assert "IDENTICAL" in out


def _edge_reference(seed):
    """FASTA text + the sorted distinct forward 31-mers of its ACGT runs (either case)."""
    rng = random.Random(seed)
    core = "".join(rng.choice("ACGT") for _ in range(3000))
    seqs = []
    # repeats of the core (shared unitigs, branching), N runs, lowercase, IUPAC, exact-length runs
    seqs.append(("seqA comment text", core[:1800] + "N" * 5 + core[1700:2600].lower() + "R" + core[:40]))
    seqs.append(("seqB", core[500:2200] + "NN" + core[100:131] + "N" + core[200:232] + "N" + core[300:330]))
    mutated = list(core[:2500])
    for p in rng.sample(range(2500), 12):
        mutated[p] = rng.choice("ACGT")
    seqs.append(("seqC\tdesc", "".join(mutated) + "ACGTYK" + "".join(rng.choice("ACGT") for _ in range(400))))
    seqs.append(("seqD", "".join(rng.choice("ACGT") for _ in range(rng.randint(200, 900)))))
    fa = "".join(f">{n}\n" + "\n".join(s[i:i + 70] for i in range(0, len(s), 70)) + "\n" for n, s in seqs)
    lut = {c: i for i, c in enumerate("ACGT")}
    lut.update({c: i for i, c in enumerate("acgt")})
    kms = set()
    for _, s in seqs:
        run = []
        for ch in s + "N":
            if ch in lut:
                run.append(lut[ch])
                continue
            for j in range(len(run) - 30):
                v = 0
                for b in run[j:j + 31]:
                    v = (v << 2) | b
                kms.add(v)
            run = []
    k = np.array(sorted(kms), dtype="<u8")
    return fa.encode(), struct.pack("<Q", len(k)) + k.tobytes()


@pytest.mark.parametrize("seed", [1, 2])
def test_edge_references_match_reference_builder(builder, tmp_path, seed):
    if not os.path.exists(REF):
        pytest.skip("oracle/_ref/deSAMBA not built (oracle/Makefile needs the reference sources)")
    fa, srt = _edge_reference(seed)
    (tmp_path / "ref.fa").write_bytes(fa)
    (tmp_path / "kmer.srt").write_bytes(srt)
    r = subprocess.run([REF, "index", str(tmp_path / "kmer.srt"), str(tmp_path / "ref.fa"), str(tmp_path / "ref_idx")],
                       capture_output=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    _build(builder, tmp_path / "kmer.srt", tmp_path / "ref.fa", tmp_path / "mine")
    assert "IDENTICAL" in _compare(tmp_path / "ref_idx", tmp_path / "mine")
    _build(builder, tmp_path / "kmer.srt", tmp_path / "ref.fa", tmp_path / "serial", {"DSB_INDEX_SERIAL_SA": "1"})
    assert "IDENTICAL" in _compare(tmp_path / "mine", tmp_path / "serial")


def test_missing_kmer_fails_loudly(builder, tmp_path):
    fa, srt = _edge_reference(4)
    (tmp_path / "ref.fa").write_bytes(fa)
    n = struct.unpack_from("<Q", srt)[0]
    short = struct.pack("<Q", n - 1) + srt[16:]  # drop the first k-mer
    (tmp_path / "kmer.srt").write_bytes(short)
    r = subprocess.run([builder, str(tmp_path / "kmer.srt"), str(tmp_path / "ref.fa"), str(tmp_path / "o")],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode != 0 and "missing from the sorted k-mer file" in r.stderr


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_kmer_list_from_the_reference(builder, tmp_path, seed):
    """SortedKmer "-": the builder computes the distinct forward 31-mers of the reference's ACGT runs
    itself (parallel, index_build.cpp kmers_from_reference) — the same index as from the k-mer
    file (lowercase, N / IUPAC breaks and exact 31-base runs included)."""
    fa, srt = _edge_reference(seed)
    (tmp_path / "ref.fa").write_bytes(fa)
    (tmp_path / "kmer.srt").write_bytes(srt)
    _build(builder, tmp_path / "kmer.srt", tmp_path / "ref.fa", tmp_path / "from_file")
    r = _build(builder, "-", tmp_path / "ref.fa", tmp_path / "from_ref", {"DSB_HOST_THREADS": "3"})
    assert "k-mers from the reference" in r.stderr
    assert "IDENTICAL" in _compare(tmp_path / "from_file", tmp_path / "from_ref")


def test_fixture_index_from_reference_kmers(builder, fixture_index, tmp_path):
    subprocess.run([sys.executable, SIM, "reference", "--preset", "fixture", "--out", str(tmp_path)], check=True,
                   capture_output=True, timeout=600)
    _build(builder, "-", tmp_path / "ref.fa", tmp_path / "idx")
    assert "IDENTICAL" in _compare(fixture_index, tmp_path / "idx")


def test_rank_superblocks(builder, fixture_index, tmp_path):
    """The builder's rank structure counts per 2^32-row superblock (index_build.cpp Rank: BWTs past
    2^32 rows).  bin/desamba_index_sb16 is the same builder with 2^16-row superblocks: the fixture
    index (~17 superblocks then) rebuilt byte for byte with both SA walks."""
    exe = os.path.join(ROOT, "desamba-so_amd", "bin", "desamba_index_sb16")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "desamba-so_amd"), "bin/desamba_index_sb16"],
                       check=True, timeout=600)
    subprocess.run([sys.executable, SIM, "reference", "--preset", "fixture", "--out", str(tmp_path)], check=True,
                   capture_output=True, timeout=600)
    with open(os.path.join(fixture_index, "deSAMBA.bwt"), "rb") as f:
        rows = int.from_bytes(f.read(8), "little") // 168 * 256
    assert rows > 4 << 16, rows
    for ser in ("0", "1"):
        _build(exe, tmp_path / "kmer.srt", tmp_path / "ref.fa", tmp_path / f"idx{ser}", {"DSB_INDEX_SERIAL_SA": ser})
        assert "IDENTICAL" in _compare(fixture_index, tmp_path / f"idx{ser}")
