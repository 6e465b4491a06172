"""The HBM occ layout past 2^32 BWT rows (reference rows are uint64_t, src/bwt.h:45; C4's
nt-scale index has more than 2^32 BWT rows).  A synthetic BWT string of 2^32 + 2^20 + 37 symbols
is written in the reference's 168-B block format by the reference's own builder functions
(oracle/_ref/bigbwt gen: bwt_cal_check_point, bwt_str2bwt_occ, bwt_cal_AGCTCounter, write_bwt), then
loaded through this library's occ_relayout (index_load.c, which verifies every checkpoint on the
way) and queried on the GPU (dsb_gpu_selftest_occ: dsb_occ for c = 0..4 and the LF symbol read)
at ~1M rows — random rows, rows past 2^32, line / block / superblock edges, the '$' row — each
compared with the reference's own occ on the same file (oracle/_ref/bigbwt occ, load_bwt + occ,
src/bwt.c:43-104)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

BIGBWT = os.path.join(ROOT, "oracle", "_ref", "bigbwt")
NSYM = (1 << 32) + (1 << 20) + 37
DOLLOR_POS = 123456789  # what occ returns at the '$' row (the unitig count - 2 in a real index)


def rows_to_check(n, dollar, seed=7):
    rng = np.random.default_rng(seed)
    r = [rng.integers(0, n, 700_000, dtype=np.uint64),
         rng.integers(1 << 32, n, 200_000, dtype=np.uint64)]  # past 2^32
    base = rng.integers(0, n >> 7, 20_000, dtype=np.uint64) << np.uint64(7)
    for d in (0, 1, 63, 64, 127, 128, 255, 256):  # 64-B line (128 symbols) and 168-B block (256) edges
        r.append(base + np.uint64(d))
    sb = np.arange(0, n, 1 << 24, dtype=np.uint64)  # every 2^24-symbol superblock start
    for d in (0, 1, 127, 128):
        r.append(sb + np.uint64(d))
        r.append(sb[1:] - np.uint64(d + 1))
    fixed = [0, 1, 2, 255, 256, (1 << 31) - 1, 1 << 31, (1 << 32) - 129, (1 << 32) - 128, (1 << 32) - 1, 1 << 32,
             (1 << 32) + 1, (1 << 32) + 127, (1 << 32) + 128, n - 2, n - 1]
    fixed += [dollar + d for d in range(-130, 131)]
    r.append(np.array(fixed, dtype=np.uint64))
    out = np.concatenate(r)
    return out[out < n]


@pytest.fixture(scope="module")
def big_bwt(tmp_path_factory):
    if not os.path.exists(BIGBWT):
        pytest.skip("oracle/_ref not built")
    d = tmp_path_factory.mktemp("bigbwt")
    g = subprocess.run([BIGBWT, "gen", str(d), str(NSYM), "11"], capture_output=True, text=True, timeout=900)
    assert g.returncode == 0, g.stderr[-800:]
    dollar = int(g.stdout.split("dollar_row")[1].split()[0])
    yield str(d), dollar


def test_occ_past_2_32_rows_matches_reference(big_bwt, tmp_path):
    d, dollar = big_bwt
    rows = rows_to_check(NSYM, dollar)
    assert (rows >= (1 << 32)).sum() > 200_000
    rp = tmp_path / "rows.bin"
    rows.tofile(rp)
    op = tmp_path / "ref_occ.bin"
    r = subprocess.run([BIGBWT, "occ", d, str(DOLLOR_POS), str(rp), str(op)], capture_output=True, text=True,
                       timeout=900)
    assert r.returncode == 0, r.stderr[-800:]
    want = np.fromfile(op, dtype=np.uint64).reshape(-1, 7)
    # the device occ self-test is in the test build only: run in a process of its own
    gp = tmp_path / "gpu_occ.bin"
    w = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "selftest_worker.py"), "occ", d, str(DOLLOR_POS),
                        str(rp), str(gp)], capture_output=True, text=True, timeout=900)
    assert w.returncode == 0, w.stderr[-800:]
    st = json.loads(w.stdout.strip().splitlines()[-1])
    assert st["rc"] == 0, st["err"]
    got = np.fromfile(gp, dtype=np.uint64).reshape(-1, 7)
    bad = np.nonzero((got != want).any(axis=1))[0]
    assert len(bad) == 0, [(int(rows[i]), got[i].tolist(), want[i].tolist()) for i in bad[:5]]
    assert int(got[np.nonzero(rows == dollar)[0][0], 6]) == 5  # the '$' row
    # occ of every symbol before r sums to r (the '$' row is not counted by any c): past 2^32 too
    tot = want[:, :5].sum(axis=1) + (rows > dollar).astype(np.uint64)
    assert (tot == rows).all()
    print(f"{len(rows)} rows ({(rows >= (1 << 32)).sum()} past 2^32) x 6 occ: identical to the reference")
