"""Dev tool: how many Bloom probes and batch round trips a sub-group-per-strand island scan
needs, against the exact bits the scan reads (search_exist_kmer_M2, reference src/cly.c:1066-1155).

  python tools/island_sim.py INDEX_DIR [n_reads]

Exist bits of simulated C1 reads are computed with numpy from the index's Bloom tables
(get_exist_kmer, src/cly.c:951-967); the scan is then replayed with batches of G positions
(grid batches i, i+3, ..; run batches h-2, h-1, h+1, ..) and the probes / batches are counted.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import simulate  # noqa: E402

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def h1(k):
    k = k.astype(np.uint64)
    with np.errstate(over="ignore"):
        k = (~k) + (k << np.uint64(21))
        k = k ^ (k >> np.uint64(24))
        k = (k + (k << np.uint64(3))) + (k << np.uint64(8))
        k = k ^ (k >> np.uint64(14))
        k = (k + (k << np.uint64(2))) + (k << np.uint64(4))
        k = k ^ (k >> np.uint64(28))
        k = k + (k << np.uint64(31))
    return k


def h2(k):
    k = k.astype(np.uint64)
    with np.errstate(over="ignore"):
        k = k + ~(k << np.uint64(32))
        k = k ^ (k >> np.uint64(22))
        k = k + ~(k << np.uint64(13))
        k = k ^ (k >> np.uint64(8))
        k = k + (k << np.uint64(3))
        k = k ^ (k >> np.uint64(15))
        k = k + ~(k << np.uint64(27))
        k = k ^ (k >> np.uint64(31))
    return k


def exist_bits(codes, l, sbm, ek0, ek1, mask):
    n = len(codes) - l + 1
    if n <= 0:
        return np.zeros(0, np.uint8)
    v = np.zeros(n, np.uint64)
    cnt = np.zeros((4, n), np.int32)
    for i in range(l):
        c = codes[i:i + n].astype(np.uint64)
        v = (v << np.uint64(2)) | c
        for b in range(4):
            cnt[b] += codes[i:i + n] == b
    bad = (cnt >= sbm).any(axis=0)
    v[bad] = 0
    a = h1(v) & np.uint64(mask)
    b1 = (ek0[(a >> np.uint64(3)).astype(np.int64)] >> (7 - (a & np.uint64(7))).astype(np.uint8)) & 1
    b = h2(v) & np.uint64(mask)
    b2 = (ek1[(b >> np.uint64(3)).astype(np.int64)] >> (7 - (b & np.uint64(7))).astype(np.uint8)) & 1
    return ((v != 0) & (b1 == 1) & (b2 == 1)).astype(np.uint8)


def scan_fwd(bits, G, GR=None):
    """forward scan with G-position grid batches and GR-position run batches; returns
    (probes, batches, needed, seeds)"""
    GR = GR or G
    n = len(bits)
    probes = batches = 0
    need = set()
    seeds = []
    i = 2
    while i < n:
        # grid batches
        h = -1
        while i < n:
            pos = [i + 3 * g for g in range(G) if i + 3 * g < n]
            probes += len(pos)
            batches += 1
            hit = [p for p in pos if bits[p]]
            if hit:
                h = hit[0]
                need.update(range(i, h + 1, 3))
                break
            need.update(pos)
            i += 3 * G
        if h < 0:
            break
        off, ln = h, 1
        # first run batch: h-1, h-2, h+1 .. h+G-2
        back = [h - 1, h - 2]
        fwd0 = h + 1
        nf = GR - 2
        probes += 2
        batches += 1
        for p in back:
            need.add(p)
            if bits[p]:
                off -= 1
                ln += 1
            else:
                break
        p = fwd0
        stop = False
        while not stop:
            end = min(p + nf, n)
            probes += max(0, end - p)
            for q in range(p, end):
                need.add(q)
                if bits[q]:
                    ln += 1
                    if ln > 60:
                        stop = True
                        break
                else:
                    stop = True
                    break
            if not stop:
                if end >= n:
                    stop = True
                else:
                    p = end
                    nf = GR
                    batches += 1
        seeds.append((off, ln))
        i = off + ln + 3
    return probes, batches, len(need), seeds


def main():
    d = sys.argv[1]
    nr = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    ek0 = np.fromfile(os.path.join(d, "deSAMBA.exk0"), np.uint8)
    ek1 = np.fromfile(os.path.join(d, "deSAMBA.exk1"), np.uint8)
    sizes = {0x8000000: (0x3FFFFFFF, 16), 0x10000000: (0x7FFFFFFF, 17), 0x20000000: (0xFFFFFFFF, 17)}
    mask, l = sizes[len(ek0)]
    sbm = int(0.8 * l)
    genomes = simulate.read_fasta_genomes_from_index(d)
    reads = list(simulate.simulate_reads(genomes, nr, 1000, "ont", 8000))
    lut = np.full(256, 1, np.uint8)
    for c, v in zip(b"ACGTacgt", [0, 1, 2, 3, 0, 1, 2, 3]):
        lut[c] = v
    allbits = []
    tot_pos = 0
    for r in reads:
        seq = r[1] if isinstance(r, tuple) else r
        if isinstance(seq, str):
            seq = seq.encode()
        c = lut[np.frombuffer(seq, np.uint8)]
        tot_pos += 2 * max(0, len(c) - l + 1)
        allbits.append(exist_bits(c, l, sbm, ek0, ek1, mask))
        allbits.append(exist_bits((3 - c)[::-1].copy(), l, sbm, ek0, ek1, mask))
    print(f"{nr} reads, {tot_pos} k-mer positions, exist rate {sum(b.sum() for b in allbits) / tot_pos:.3f}")
    for G, GR in ((4, 4), (8, 8), (16, 16), (32, 32), (8, 16), (12, 16), (16, 8), (6, 16), (16, 32), (8, 32)):
        P = B = N = 0
        maxb = 0
        for b in allbits:
            p, bt, nd, _ = scan_fwd(b, G, GR)
            P += p
            B += bt
            N += nd
            maxb = max(maxb, bt)
        print(f"grid {G:2d} run {GR:2d}: probes {P / tot_pos:.3f} of all positions, needed {N / tot_pos:.3f}, "
              f"batches/strand {B / len(allbits):.0f} (max {maxb})")


if __name__ == "__main__":
    main()
