"""Runs one classify scenario in a process of its own, with the library named by DSB_LIB (the
test build lib/libdesamba_test.so for the test-hook scenarios of tests/test_gpu_hooks.py) and the
DSB_* switches of the spec in its environment before the library is loaded.

    python tests/hook_worker.py spec.json

spec: {"index": dir, "inputs": [fastq paths], "fmt": int, "mode": "text" | "batch",
       "out": prefix, "max_read_l": int (batch mode: the carry the run starts from, default 0)}
For every input k the records go to <out>.<k> and a JSON summary (timings of each call) is
printed on stdout.  "batch" classifies through dsb_batch_create / run / format (the API bench.py
times), "text" through dsb_classify_text (the read_classify pipeline).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "desamba-so_amd"))


def main():
    spec = json.load(open(sys.argv[1]))
    import pydesamba as P
    P.lib()
    idx = P.Index(spec["index"])
    summary = {"lib": os.environ.get("DSB_LIB"), "devices": idx.devices(), "calls": []}
    try:
        for k, path in enumerate(spec["inputs"]):
            data = open(path, "rb").read()
            if spec.get("mode", "text") == "batch":
                b = idx.batch(data)
                try:
                    tm = b.run(max_read_l=spec.get("max_read_l", 0))
                    out = b.format(spec.get("fmt", P.FMT_SAM))
                finally:
                    b.close()
            else:
                out, tm, _ = idx.classify(data, fmt=spec.get("fmt", P.FMT_SAM))
            with open(f"{spec['out']}.{k}", "wb") as f:
                f.write(out)
            summary["calls"].append({k2: tm[k2] for k2 in ("n_retry", "n_chunks", "n_batches", "n_devices", "n_heavy")
                                     if k2 in tm})
    finally:
        idx.close()
    print(json.dumps(summary), flush=True)


if __name__ == "__main__":
    main()
