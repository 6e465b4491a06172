"""HBM-exhaustion scenarios of tests/test_gpu_hbm.py, one per process (the process may end in the
library's fatal exit, like the reference's err_fatal, which is what some scenarios check).

    python tests/hbm_worker.py SCENARIO INDEX_DIR READS_FQ GOLDEN_SAM

Another user of the GPU is modelled by torch allocations that leave `leave` MB of HBM free.
  load_full    fill the HBM, then load_index: must end the process with a clear error, quickly
  second_index load + classify one index, fill the HBM, classify again (its workspace is held),
               then load a second index: must end the process with a clear error, quickly
  shrink       load the index, leave less HBM than the batch's workspace at the default chunk
               size, classify: the chunks must shrink until they fit, records identical
Prints "STEP <name> <seconds>" lines as it goes and "RESULT ok" at a normal end.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "desamba-so_amd"))


def fill(leave_mb):
    import torch
    hold = []
    while True:
        free, _ = torch.cuda.mem_get_info()
        extra = free - (leave_mb << 20)
        if extra <= (64 << 20):
            break
        n = min(extra, 8 << 30)
        hold.append(torch.empty(n, dtype=torch.uint8, device="cuda"))
    free, _ = torch.cuda.mem_get_info()
    print(f"STEP fill free_mb {free >> 20}", flush=True)
    return hold


def main():
    scen, index_dir, fq_path, sam_path = sys.argv[1:5]
    import torch
    torch.cuda.set_device(0)
    import pydesamba as P
    fq = open(fq_path, "rb").read()
    want = open(sam_path, "rb").read()
    t = time.time()

    def step(name):
        print(f"STEP {name} {time.time() - t:.2f}", flush=True)

    if scen == "load_full":
        hold = fill(int(os.environ.get("LEAVE_MB", "256")))
        step("filled")
        P.Index(index_dir)  # the library's fatal path ends the process here
        step("loaded")  # not reached
    elif scen == "second_index":
        a = P.Index(index_dir)
        out, _, _ = a.classify(fq, fmt=P.FMT_SAM)
        assert out == want
        step("classified_a")
        hold = fill(int(os.environ.get("LEAVE_MB", "256")))
        out, _, _ = a.classify(fq, fmt=P.FMT_SAM)
        assert out == want
        step("classified_a_again")
        P.Index(index_dir)  # fatal: no room for a second copy of the index
        step("loaded_b")  # not reached
    elif scen == "shrink":
        a = P.Index(index_dir)
        step("loaded")
        hold = fill(int(os.environ.get("LEAVE_MB", "1024")))
        out, tm, _ = a.classify(fq, fmt=P.FMT_SAM)
        step(f"classified chunks {tm['n_chunks']} shrinks {tm['n_ws_shrink']}")
        assert out == want, "records differ after the workspace shrank"
        a.close()
    del hold
    print("RESULT ok", flush=True)


if __name__ == "__main__":
    main()
