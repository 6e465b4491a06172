"""Classify a golden read set several times on the GPU; report reads that differ from the
hermetic reference per run (determinism / parity triage)."""
import os
import sys
import tarfile
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "desamba-so_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import pydesamba  # noqa: E402
from conftest import golden  # noqa: E402
from samutil import groups  # noqa: E402

names = (sys.argv[1] if len(sys.argv) > 1 else "mixed").split(",")
runs = int(sys.argv[2]) if len(sys.argv) > 2 else 1
with tempfile.TemporaryDirectory() as d:
    with tarfile.open(os.path.join(ROOT, "tests", "golden", "fixture_index.txz")) as t:
        t.extractall(d)
    idx = pydesamba.Index(d)
    for r, name in [(r, n) for r in range(runs) for n in names]:
        ref = groups(golden(name + ".herm.sam"))
        fq = golden(name + ".fq")
        out, tm, _ = idx.classify(fq, fmt=pydesamba.FMT_SAM)
        got = groups(out)
        bad = [i for i in range(len(ref)) if i >= len(got) or got[i] != ref[i]]
        print(f"run {r} {name}: n_retry {tm['n_retry']} chunks {tm['n_chunks']}: {len(bad)} reads differ {bad[:20]}", flush=True)
        for i in bad[:3]:
            print("  want:", b"".join(ref[i][1])[:600])
            print("  got: ", b"".join(got[i][1])[:600] if i < len(got) else None)
    idx.close()
