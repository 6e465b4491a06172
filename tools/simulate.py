#!/usr/bin/env python3
"""Deterministic synthetic inputs for the deSAMBA classify path.

Nothing here comes from the reference; it generates:

* a family-structured reference collection (decoy first, then genome families made
  of a random core plus mutated copies, unique flanks, shared segments and
  interspersed repeat elements), FASTA headers ``>tid|<taxid>|ref|<acc>``
  (the convention of reference ``build-index:22-23``);
* a matching NCBI-style ``nodes.dmp`` / ``names.dmp`` taxonomy (parsed by reference
  ``src/cly_mt.c:590-670``);
* ``kmer.srt`` for the reference index builder: ``[u64 n][n sorted distinct forward
  31-mers]``, 2-bit A0 C1 G2 T3, first base in the high bits — what
  ``src/idx_sort.c:101-204`` writes from a non-canonical jellyfish count and what
  ``build_deb`` (``src/idx.c:143-235``) consumes (probe P2);
* ONT-like / Illumina-like FASTQ reads with a recorded seed.

The reference index builder itself (``deSAMBA index``) is run by tools/make_index.sh
in the development container only; the GPU box never runs it.
"""
from __future__ import annotations

import argparse
import json
import os
import struct
import sys

import numpy as np

BASES = np.frombuffer(b"ACGT", dtype=np.uint8)
COMP = np.array([3, 2, 1, 0], dtype=np.uint8)


# ----------------------------------------------------------------------------- reference
def _mutate(rng, seq, rate):
    """Substitutions only (keeps coordinates), at `rate`."""
    if rate <= 0:
        return seq.copy()
    out = seq.copy()
    m = rng.random(len(seq)) < rate
    out[m] = (out[m] + rng.integers(1, 4, size=int(m.sum()), dtype=np.uint8)) & 3
    return out


def make_reference(seed, n_families, copies, core_len, flank_len, decoy_len=5000,
                   n_shared=4, shared_len=3000, repeat_specs=((300, 60, 0.01), (150, 1200, 0.005)),
                   human_like=True):
    """Return list of dict(name, taxid, seq uint8[0..3]) and the taxonomy edges.

    taxonomy: 1 (root) -> 131567 -> 2 (Bacteria) -> family 3000+f -> genus 4000+f ->
    species 5000+f*16+c (one per copy); optional human-like genome tid 9606 under
    9605 -> 33208 (Metazoa) -> 2759 -> 131567.
    """
    rng = np.random.default_rng(seed)
    genomes = []
    nodes = {1: (1, "no rank", "root"), 131567: (1, "no rank", "cellular organisms"),
             2: (131567, "superkingdom", "Bacteria"), 2759: (131567, "superkingdom", "Eukaryota"),
             33208: (2759, "kingdom", "Metazoa"), 9605: (33208, "genus", "Homo"),
             9606: (9605, "species", "Homo sapiens")}
    decoy = rng.integers(0, 4, size=decoy_len, dtype=np.uint8)
    nodes[7] = (1, "no rank", "synthetic decoy")
    genomes.append(dict(name="tid|7|ref|DECOY_0000", taxid=7, seq=decoy, decoy=True))
    shared = [rng.integers(0, 4, size=shared_len, dtype=np.uint8) for _ in range(n_shared)]
    repeats = [(rng.integers(0, 4, size=L, dtype=np.uint8), n, r) for (L, n, r) in repeat_specs]
    fam_seqs = []
    for f in range(n_families):
        fam, genus = 3000 + f, 4000 + f
        nodes[fam] = (2, "family", f"Synthfamilia{f}")
        nodes[genus] = (fam, "genus", f"Synthgenus{f}")
        core = rng.integers(0, 4, size=core_len, dtype=np.uint8)
        for c in range(copies):
            tid = 5000 + f * 16 + c
            nodes[tid] = (genus, "species", f"Synthgenus{f} species{c}")
            rate = 0.0 if c == 0 else rng.uniform(0.003, 0.024)
            body = _mutate(rng, core, rate)
            parts = [rng.integers(0, 4, size=flank_len, dtype=np.uint8), body,
                     rng.integers(0, 4, size=flank_len, dtype=np.uint8)]
            if n_shared:
                sh = shared[(f + c) % n_shared]
                parts.insert(2, _mutate(rng, sh, 0.002))
            seq = np.concatenate(parts)
            fam_seqs.append(dict(name=f"tid|{tid}|ref|SYN_{f:03d}_{c:02d}", taxid=tid, seq=seq))
    if human_like:
        hs = rng.integers(0, 4, size=max(core_len // 2, 2000), dtype=np.uint8)
        fam_seqs.append(dict(name="tid|9606|ref|SYN_HUMAN_00", taxid=9606, seq=hs))
    # interspersed repeats: copy each element n times at random positions across genomes
    for elem, n, rate in repeats:
        for _ in range(n):
            g = fam_seqs[int(rng.integers(0, len(fam_seqs)))]
            s = g["seq"]
            if len(s) <= len(elem) + 10:
                continue
            p = int(rng.integers(0, len(s) - len(elem)))
            s[p:p + len(elem)] = _mutate(rng, elem, rate)
    genomes.extend(fam_seqs)
    return genomes, nodes


def write_fasta(genomes, path, width=80):
    with open(path, "wb") as f:
        for g in genomes:
            f.write(b">" + g["name"].encode() + b"\n")
            s = BASES[g["seq"]].tobytes()
            for i in range(0, len(s), width):
                f.write(s[i:i + width] + b"\n")


def write_taxonomy(nodes, dirpath):
    # the reference takes max_tid from the LAST line of nodes.dmp (cly_mt.c:601-613): keep
    # the largest tid last.
    tids = sorted(nodes)
    with open(os.path.join(dirpath, "nodes.dmp"), "w") as f:
        for t in tids:
            p, rank, _ = nodes[t]
            f.write(f"{t}\t|\t{p}\t|\t{rank}\t|\t\t|\n")
    with open(os.path.join(dirpath, "names.dmp"), "w") as f:
        for t in tids:
            f.write(f"{t}\t|\t{nodes[t][2]}\t|\t\t|\tscientific name\t|\n")


def kmers31(seq):
    """Forward 31-mer values of one ACGT-only sequence (first base high bits)."""
    n = len(seq) - 30
    if n <= 0:
        return np.zeros(0, dtype=np.uint64)
    s = seq.astype(np.uint64)
    v = np.zeros(n, dtype=np.uint64)
    for j in range(31):
        v = (v << np.uint64(2)) | s[j:j + n]
    return v


def write_kmer_srt(genomes, path):
    allk = np.unique(np.concatenate([kmers31(g["seq"]) for g in genomes]))
    with open(path, "wb") as f:
        f.write(struct.pack("<Q", len(allk)))
        allk.astype("<u8").tofile(f)
    return len(allk)


# ----------------------------------------------------------------------------- reads
def apply_errors(rng, tmpl, err):
    """ONT-like error model: per base, with prob err an event: sub 50%, del 25%, ins 25%."""
    n = len(tmpl)
    u = rng.random(n)
    ev = np.zeros(n, dtype=np.uint8)  # 0 match, 1 sub, 2 del, 3 ins
    hit = u < err
    kind = rng.random(n)
    ev[hit & (kind < 0.5)] = 1
    ev[hit & (kind >= 0.5) & (kind < 0.75)] = 2
    ev[hit & (kind >= 0.75)] = 3
    base = tmpl.copy()
    sub = ev == 1
    base[sub] = (base[sub] + rng.integers(1, 4, size=int(sub.sum()), dtype=np.uint8)) & 3
    counts = np.where(ev == 2, 0, np.where(ev == 3, 2, 1))
    idx = np.repeat(np.arange(n), counts)
    out = base[idx]
    # inserted copies: the second copy of an ins position becomes a random base
    ins_pos = np.flatnonzero(ev == 3)
    if len(ins_pos):
        start = np.cumsum(counts) - counts  # first output slot of each template base
        out[start[ins_pos] + 1] = rng.integers(0, 4, size=len(ins_pos), dtype=np.uint8)
    return out


def simulate_reads(genomes, n_reads, seed, kind="ont", mean_len=8000, sigma=0.5,
                   err_choices=(0.05, 0.10, 0.15), random_frac=0.03, min_len=40, max_len=100000):
    """Yield (name, seq_bytes, qual_bytes). Reads never start inside the decoy."""
    rng = np.random.default_rng(seed)
    src = [g for g in genomes if not g.get("decoy")]
    lens = np.array([len(g["seq"]) for g in src], dtype=np.float64)
    w = lens / lens.sum()
    mu = np.log(mean_len) - sigma * sigma / 2
    for i in range(n_reads):
        if kind == "illumina":
            L = 150
        else:
            L = int(min(max(rng.lognormal(mu, sigma), min_len), max_len))
        if rng.random() < random_frac:
            seq = rng.integers(0, 4, size=L, dtype=np.uint8)
            name = f"rd{i}_random"
        else:
            gi = int(rng.choice(len(src), p=w))
            g = src[gi]["seq"]
            L = min(L, len(g))
            p = int(rng.integers(0, len(g) - L + 1))
            tmpl = g[p:p + L]
            err = 0.01 if kind == "illumina" else float(rng.choice(err_choices))
            if kind == "illumina":
                seq = tmpl.copy()
                m = rng.random(L) < err
                seq[m] = (seq[m] + rng.integers(1, 4, size=int(m.sum()), dtype=np.uint8)) & 3
            else:
                seq = apply_errors(rng, tmpl, err)
            strand = "+"
            if rng.random() < 0.5:
                seq = COMP[seq[::-1]]
                strand = "-"
            name = f"rd{i}_{src[gi]['taxid']}_{p}_{strand}_{int(err * 100)}"
        s = BASES[seq].tobytes()
        # low-entropy qualities (one symbol per read) keep committed fixtures small
        q = bytes([33 + 10 + (i % 30)]) * len(s)
        yield name, s, q


def simulate_c4_mix(genomes, n_reads, seed, long_mean=20000):
    """BASELINE config C4's read mix: 150 bp Illumina-like and ONT-like reads (lognormal mean
    `long_mean`) 1:1 by count, interleaved in a fixed order (even = long, odd = short), since
    the carried max_read_l makes results order-dependent (reference cly.c:2953)."""
    ont = simulate_reads(genomes, (n_reads + 1) // 2, seed, "ont", long_mean)
    ill = simulate_reads(genomes, n_reads // 2, seed + 1, "illumina")
    for i in range(n_reads):
        name, s, q = next(ont) if i % 2 == 0 else next(ill)
        yield f"m{i}_{name}", s, q


def fastq_bytes(reads) -> bytes:
    return b"".join(b"@" + name.encode() + b"\n" + s + b"\n+\n" + q + b"\n" for name, s, q in reads)


_PAR = {}  # the genomes, inherited by forked workers


def _chunk_fastq(args):
    c, n, seed, mix, mean_len = args
    g = _PAR["genomes"]
    s = seed if c == 0 else seed + 7919 * c
    gen = simulate_c4_mix(g, n, s) if mix == "c4" else simulate_reads(g, n, s, "ont", mean_len)
    if c:
        gen = ((f"c{c}_{name}", sq, q) for name, sq, q in gen)
    return fastq_bytes(gen)


def simulate_fastq_parallel(genomes, n_reads, seed, mix="ont", mean_len=8000, workers=8, chunk=10000) -> bytes:
    """FASTQ text of n_reads reads made in chunks of `chunk` reads over forked workers: chunk 0 is
    simulate_reads(seed) (or simulate_c4_mix) itself, chunk c > 0 the same generator seeded
    seed + 7919 c with names prefixed `c<c>_`, so the text depends on (n_reads, seed, mix,
    mean_len, chunk) only, never on the worker count.  Call it before the process touches a GPU
    (the workers are forked)."""
    import multiprocessing as mp
    jobs = [(c, min(chunk, n_reads - c * chunk), seed, mix, mean_len) for c in range((n_reads + chunk - 1) // chunk)]
    _PAR["genomes"] = genomes
    try:
        if workers <= 1 or len(jobs) <= 1:
            parts = [_chunk_fastq(j) for j in jobs]
        else:
            with mp.get_context("fork").Pool(min(workers, len(jobs))) as pool:
                parts = pool.map(_chunk_fastq, jobs, chunksize=1)
    finally:
        _PAR.clear()
    out = b"".join(parts)
    del parts
    return out


def write_fastq(reads, path):
    with open(path, "wb") as f:
        for name, s, q in reads:
            f.write(b"@" + name.encode() + b"\n" + s + b"\n+\n" + q + b"\n")


def edge_case_reads(rng):
    """Reads the reference treats specially (src/cly.c:3058,3084; CLY_Bit non-ACGT->C)."""
    out = []
    out.append(("edge_len39", BASES[rng.integers(0, 4, 39, dtype=np.uint8)].tobytes()))
    out.append(("edge_len40", BASES[rng.integers(0, 4, 40, dtype=np.uint8)].tobytes()))
    out.append(("edge_empty", b""))
    out.append(("edge_allA", b"A" * 500))
    out.append(("edge_lower", BASES[rng.integers(0, 4, 300, dtype=np.uint8)].tobytes().lower()))
    s = bytearray(BASES[rng.integers(0, 4, 400, dtype=np.uint8)].tobytes())
    for p in rng.integers(0, 400, 20):
        s[p] = ord("N")
    out.append(("edge_withN", bytes(s)))
    return [(n, s, b"I" * len(s)) for n, s in out]


# ----------------------------------------------------------------------------- CLI
PRESETS = {
    # C0: committed fixture (~1 Mbp), mirrors SURVEY P4/P8
    "fixture": dict(seed=20240601, n_families=4, copies=3, core_len=60000, flank_len=8000,
                    decoy_len=5000, n_shared=3, shared_len=2500,
                    repeat_specs=((300, 40, 0.01), (150, 200, 0.005))),
    # C1 proxy: >= 50 Mbp family-structured reference
    "c1": dict(seed=20240602, n_families=25, copies=5, core_len=400000, flank_len=20000,
               decoy_len=5000, n_shared=6, shared_len=5000,
               repeat_specs=((300, 400, 0.01), (150, 3000, 0.005))),
    # C2-direction proxy: >= 238.6M distinct 31-mers, so the reference builder picks the
    # quarter-GB e-kmer tables, l_ek 17 and MASK_31 (reference idx.c:966-996), and the BWT
    # passes 2^28 symbols (many 2^24-symbol occ superblocks)
    "c2": dict(seed=20240603, n_families=80, copies=4, core_len=1300000, flank_len=120000,
               decoy_len=5000, n_shared=8, shared_len=5000,
               repeat_specs=((300, 2000, 0.01), (150, 12000, 0.005))),
    # the next e-kmer size class: >= 954.4M distinct 31-mers (2^33 / 9), so the builder picks 1 GB
    # tables, l_ek 18 and MASK_33 (reference idx.c:966-996); the c2 preset's families x 3.75
    # (1.86 Gbp, ~1.07 G 31-mers, ~1.1 G BWT rows)
    "c2l18": dict(seed=20240604, n_families=300, copies=4, core_len=1300000, flank_len=120000,
                  decoy_len=5000, n_shared=8, shared_len=5000,
                  repeat_specs=((300, 7500, 0.01), (150, 45000, 0.005))),
    # a BWT past 2^32 rows (C2's RefSeq-scale index): the c2l18 preset's families x 2.67 (~5 Gbp,
    # ~2.8 G distinct 31-mers >= 2^34 / 9, so 2 GB e-kmer tables, l_ek 18, MASK_34; ~75 M unitigs;
    # BWT rows = unitigs x 31 + 31-mers ~ 5.1 G), an index of ~17 GB
    "c2xl": dict(seed=20240605, n_families=800, copies=4, core_len=1300000, flank_len=120000,
                 decoy_len=5000, n_shared=8, shared_len=5000,
                 repeat_specs=((300, 20000, 0.01), (150, 120000, 0.005))),
}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("reference")
    r.add_argument("--preset", choices=sorted(PRESETS), required=True)
    r.add_argument("--out", required=True, help="output directory")
    r.add_argument("--no-kmers", action="store_true",
                   help="skip kmer.srt (desamba_index computes the k-mer list itself when given '-')")
    q = sub.add_parser("reads")
    q.add_argument("--fasta", required=True)
    q.add_argument("--out", required=True)
    q.add_argument("-n", type=int, required=True)
    q.add_argument("--seed", type=int, default=7)
    q.add_argument("--kind", choices=["ont", "illumina", "mixed"], default="ont")
    q.add_argument("--mean-len", type=int, default=8000)
    q.add_argument("--edge", action="store_true", help="prepend edge-case reads")
    a = ap.parse_args(argv)

    if a.cmd == "reference":
        os.makedirs(a.out, exist_ok=True)
        p = PRESETS[a.preset]
        genomes, nodes = make_reference(**p)
        write_fasta(genomes, os.path.join(a.out, "ref.fa"))
        write_taxonomy(nodes, a.out)
        nk = None if a.no_kmers else write_kmer_srt(genomes, os.path.join(a.out, "kmer.srt"))
        meta = dict(preset=a.preset, params={k: (list(v) if isinstance(v, tuple) else v) for k, v in p.items()},
                    n_genomes=len(genomes), total_bp=int(sum(len(g["seq"]) for g in genomes)), n_kmer31=nk)
        with open(os.path.join(a.out, "manifest.json"), "w") as f:
            json.dump(meta, f, indent=1, default=str)
        print(json.dumps(meta, default=str))
    else:
        genomes = read_fasta_genomes(a.fasta)
        rng = np.random.default_rng(a.seed + 999)
        reads = []
        if a.edge:
            reads.extend(edge_case_reads(rng))
        if a.kind == "mixed":
            # interleaved in a fixed order: max_read_l semantics depend on order
            ont = list(simulate_reads(genomes, a.n - a.n // 4, a.seed, "ont", a.mean_len))
            ill = list(simulate_reads(genomes, a.n // 4, a.seed + 1, "illumina"))
            k = 0
            for i, x in enumerate(ont):
                reads.append(x)
                if i % 3 == 2 and k < len(ill):
                    reads.append(ill[k]); k += 1
            reads.extend(ill[k:])
        else:
            reads.extend(simulate_reads(genomes, a.n, a.seed, a.kind, a.mean_len))
        write_fastq(reads, a.out)


def read_fasta_genomes(path):
    lut = np.full(256, 0, dtype=np.uint8)
    for i, c in enumerate(b"ACGT"):
        lut[c] = i
        lut[c + 32] = i
    genomes, name, buf = [], None, []
    with open(path, "rb") as f:
        for line in f:
            line = line.rstrip(b"\n")
            if line.startswith(b">"):
                if name is not None:
                    genomes.append(_mk(name, buf, lut))
                name, buf = line[1:].decode(), []
            else:
                buf.append(line)
    if name is not None:
        genomes.append(_mk(name, buf, lut))
    return genomes


def read_fasta_genomes_from_index(idx_dir):
    """Genomes decoded from an index's packed reference (deSAMBA.ref_b / .ref_i, idx.c:1141-1152),
    so reads can be simulated where only the index exists (e.g. the GPU box)."""
    import numpy as np
    with open(os.path.join(idx_dir, "deSAMBA.ref_i"), "rb") as f:
        n = struct.unpack("<Q", f.read(8))[0]
        infos = []
        for _ in range(n):
            rec = f.read(144)
            name = rec[:128].split(b"\0", 1)[0].decode()
            seq_l, seq_off = struct.unpack("<QQ", rec[128:144])
            infos.append((name, seq_l, seq_off))
    packed = np.fromfile(os.path.join(idx_dir, "deSAMBA.ref_b"), dtype=np.uint8, offset=8)
    bases = np.empty(len(packed) * 4, dtype=np.uint8)
    for k in range(4):
        bases[k::4] = (packed >> (6 - 2 * k)) & 3
    out = []
    for name, seq_l, seq_off in infos:
        taxid = int(name.split("|")[1]) if name.startswith("tid|") else 0
        out.append(dict(name=name, taxid=taxid, seq=bases[seq_off:seq_off + seq_l].copy(), decoy="DECOY" in name))
    return out


def _mk(name, buf, lut):
    seq = lut[np.frombuffer(b"".join(buf), dtype=np.uint8)]
    taxid = int(name.split("|")[1]) if name.startswith("tid|") else 0
    return dict(name=name, taxid=taxid, seq=seq, decoy="DECOY" in name)


if __name__ == "__main__":
    main()
