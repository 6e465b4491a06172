#!/usr/bin/env python3
"""CPU-only parity sweep: the CPU emulation of the kernels (build/emu/emu_classify, which reproduces
the GPU's records exactly) against the hermetic reference (oracle/_ref/herm_classify) and the gcc
reference (oracle/_ref/ref_classify --fresh) on freshly simulated reads.

    python tools/emu_vs_herm.py <index_dir> -n 20000 --seed 1 [--jobs 4] [--kind ont]

The reads are cut into chunks classified by parallel processes (ONT reads are all longer than the
reference's 510-bp carry threshold, so chunking does not change the carried max_read_l).  Prints
one JSON line: reads, T3 mismatches (emulator vs hermetic), stable reads (hermetic == gcc) and the
stable reads whose emulated records differ (T2 violations), with their names.  Test tooling only.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

HERM = os.path.join(ROOT, "oracle", "_ref", "herm_classify")
GCC = os.path.join(ROOT, "oracle", "_ref", "ref_classify")
EMU = os.path.join(ROOT, "build", "emu", "emu_classify")


def _run(cmd, env=None):
    return subprocess.run(cmd, capture_output=True, check=True, env=env).stdout


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("index")
    ap.add_argument("-n", type=int, default=2000)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--kind", default="ont")
    ap.add_argument("--mean-len", type=int, default=8000)
    ap.add_argument("--jobs", type=int, default=4)
    ap.add_argument("--chunk", type=int, default=500)
    ap.add_argument("--no-gcc", action="store_true")
    ap.add_argument("--wave", action="store_true", help="run the wave-cooperative code paths (EMU_WAVE=1)")
    ap.add_argument("--fq", help="classify this FASTQ instead of simulating")
    a = ap.parse_args(argv)
    import simulate
    from samutil import groups

    tmp = tempfile.mkdtemp(prefix="evh_")
    if a.fq:
        recs = open(a.fq, "rb").read().split(b"\n")
        recs = [b"\n".join(recs[i:i + 4]) + b"\n" for i in range(0, len(recs) - 3, 4)]
    else:
        genomes = simulate.read_fasta_genomes_from_index(a.index)
        fq = os.path.join(tmp, "all.fq")
        simulate.write_fastq(list(simulate.simulate_reads(genomes, a.n, a.seed, a.kind, a.mean_len)), fq)
        recs = open(fq, "rb").read().split(b"\n")
        recs = [b"\n".join(recs[i:i + 4]) + b"\n" for i in range(0, len(recs) - 3, 4)]
    chunks = []
    for c in range(0, len(recs), a.chunk):
        p = os.path.join(tmp, f"c{c // a.chunk:05d}.fq")
        with open(p, "wb") as f:
            f.write(b"".join(recs[c:c + a.chunk]))
        chunks.append(p)

    def one(p):
        h = _run([HERM, "--sam", a.index, p])
        g = b"" if a.no_gcc else _run([GCC, "--sam", "--fresh", a.index, p])
        e = _run([EMU, "--sam", a.index, p], env=dict(os.environ, EMU_WAVE="1") if a.wave else None)
        return h, g, e

    t3, t2, stable, n = [], [], 0, 0
    with cf.ThreadPoolExecutor(a.jobs) as ex:
        for h, g, e in ex.map(one, chunks):
            gh, ge = groups(h), groups(e)
            gg = groups(g) if not a.no_gcc else gh
            assert len(gh) == len(ge) == len(gg)
            for i in range(len(gh)):
                n += 1
                st = gh[i] == gg[i]
                stable += st
                if ge[i] != gh[i]:
                    name = gh[i][0].decode() if isinstance(gh[i][0], bytes) else str(gh[i][0])
                    t3.append(name)
                    if st:
                        t2.append(name)
    print(json.dumps({"index": a.index, "reads": n, "seed": a.seed, "wave": a.wave, "t3_mismatch": len(t3), "stable": stable,
                      "t2_violations": len(t2), "t3_reads": t3[:50], "t2_reads": t2[:50]}))


if __name__ == "__main__":
    main()
