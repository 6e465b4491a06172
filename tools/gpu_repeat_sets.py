"""Dev tool (GPU box): classify committed read sets N times (SAM and DES) and report the reads
whose records differ from the hermetic reference, with the differing records (non-determinism
hunt).  python tools/gpu_repeat_sets.py N [sets...]"""
import lzma, os, sys, tarfile, tempfile
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "desamba-so_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import pydesamba
from samutil import groups
g = os.path.join(ROOT, "tests", "golden")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
sets = sys.argv[2:] or ["ont", "mixed", "ont_long", "illumina"]
tot_bad = 0
with tempfile.TemporaryDirectory() as d:
    with tarfile.open(os.path.join(g, "fixture_index.txz")) as t:
        t.extractall(d)
    idx = pydesamba.Index(d)
    for rep in range(n):
        for name in sets:
            fq = lzma.open(os.path.join(g, name + ".fq.xz")).read()
            ref = groups(lzma.open(os.path.join(g, name + ".herm.sam.xz")).read())
            out, tm, _ = idx.classify(fq, fmt=pydesamba.FMT_SAM)
            got = groups(out)
            bad = [i for i in range(len(ref)) if got[i] != ref[i]]
            tot_bad += len(bad)
            print(name, rep, "sam mismatch", len(bad), bad[:8], flush=True)
            for i in bad[:3]:
                print("  ref", ref[i][1], "\n  got", got[i][1], flush=True)
            if name in ("mixed", "ont"):
                out, _, _ = idx.classify(fq, fmt=pydesamba.FMT_DES)
                want = lzma.open(os.path.join(g, name + ".herm.des.xz")).read()
                a, b = out.split(b"\n\n"), want.split(b"\n\n")
                dbad = [i for i in range(min(len(a), len(b))) if a[i] != b[i]]
                tot_bad += len(dbad) + (len(a) != len(b))
                print(name, rep, "des mismatch", len(dbad), dbad[:8], len(a), len(b), flush=True)
                for i in dbad[:2]:
                    print("  ref", b[i][:600], "\n  got", a[i][:600], flush=True)
    idx.close()
print("TOTAL_BAD", tot_bad)
