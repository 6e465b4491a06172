"""Dev tool: classify golden sets on the GPU and save outputs under gpurun_out/ for offline diffing."""
import lzma, os, sys, tarfile, tempfile
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "desamba-so_amd"))
import pydesamba
g = os.path.join(ROOT, "tests", "golden")
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
with tempfile.TemporaryDirectory() as d:
    with tarfile.open(os.path.join(g, "fixture_index.txz")) as t:
        t.extractall(d)
    idx = pydesamba.Index(d)
    for name in sys.argv[1:]:
        fq = lzma.open(os.path.join(g, name + ".fq.xz")).read()
        out, tm, _ = idx.classify(fq, fmt=pydesamba.FMT_SAM_FULL)
        open(os.path.join(ROOT, "gpurun_out", name + ".gpu.sam_full"), "wb").write(out)
        print(name, tm["ms_classA"], flush=True)
    idx.close()
