"""Quick GPU timing on the committed fixture (dev tool): classify a golden read set twice."""
import lzma, os, sys, tarfile, tempfile, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "desamba-so_amd"))
import pydesamba
g = os.path.join(ROOT, "tests", "golden")
name = sys.argv[1] if len(sys.argv) > 1 else "ont"
with tempfile.TemporaryDirectory() as d:
    with tarfile.open(os.path.join(g, "fixture_index.txz")) as t:
        t.extractall(d)
    t0 = time.time(); idx = pydesamba.Index(d); print("load_index s", time.time() - t0, flush=True)
    fq = lzma.open(os.path.join(g, name + ".fq.xz")).read()
    for rep in range(3):
        out, tm, _ = idx.classify(fq, fmt=pydesamba.FMT_SAM, stats=(rep == 2))
        print(json.dumps(tm), flush=True)
    ref = lzma.open(os.path.join(g, name + ".herm.sam.xz")).read()
    print("identical_to_hermetic_reference", out == ref)
    idx.close()
