"""HBM exhaustion ends in bounded time: a clean error (the reference's err_fatal: message +
exit(1)) or a run in smaller chunks, never a wait.  Each scenario runs in a process of its own
(tests/hbm_worker.py) under a time limit; another user of the GPU is modelled by torch allocations
that leave little HBM free.  Round 4's suite once stopped in the test that loaded a 32 GB-table
index beside an index whose contexts held most of the HBM ("HBM exhaustion")."""
import os
import subprocess
import sys
import time

import pytest

from conftest import ROOT, golden

pytestmark = pytest.mark.gpu

WORKER = os.path.join(ROOT, "tests", "hbm_worker.py")


def run(scen, fixture_index, tmp_path, env=None, limit=120):
    fq = tmp_path / "ont.fq"
    fq.write_bytes(golden("ont.fq"))
    sam = tmp_path / "ont.sam"
    sam.write_bytes(golden("ont.herm.sam"))
    e = {k: v for k, v in os.environ.items() if not k.startswith("DSB_")}
    e["DSB_DEVICE"] = "0"
    e.update(env or {})
    t = time.time()
    r = subprocess.run([sys.executable, "-u", WORKER, scen, fixture_index, str(fq), str(sam)], capture_output=True,
                       env=e, timeout=limit)
    out, err = r.stdout.decode(), r.stderr.decode(errors="replace")
    print(out, err[-1500:])
    return r.returncode, out, err, time.time() - t


def test_load_index_on_a_full_gpu_fails_cleanly(fixture_index, tmp_path):
    rc, out, err, secs = run("load_full", fixture_index, tmp_path)
    assert rc == 1, (rc, err[-800:])
    assert "STEP filled" in out and "STEP loaded" not in out
    assert "[load_index]" in err and "HBM" in err, err[-800:]


def test_second_index_beside_a_held_workspace_fails_cleanly(fixture_index, tmp_path):
    rc, out, err, secs = run("second_index", fixture_index, tmp_path)
    assert "STEP classified_a_again" in out, (rc, out, err[-800:])
    assert rc == 1 and "STEP loaded_b" not in out, (rc, err[-800:])
    assert "[load_index]" in err and "HBM" in err, err[-800:]


def test_workspace_shrinks_to_the_free_hbm(fixture_index, tmp_path):
    """2000 ONT reads need ~2 GB of workspace in one chunk; with a budget of 8 GB
    (DSB_WS_BUDGET_MB) and 1 GB free the allocation fails, and the chunks shrink until they fit."""
    rc, out, err, secs = run("shrink", fixture_index, tmp_path, {"LEAVE_MB": "1024", "DSB_WS_BUDGET_MB": "8192"})
    assert rc == 0 and "RESULT ok" in out, (rc, out, err[-800:])
    chunks = int(out.split("classified chunks ")[1].split()[0])
    shrinks = int(out.split("shrinks ")[1].split()[0])
    assert chunks >= 2 and shrinks >= 1, out
