"""Device self-tests of building blocks whose exact behaviour the parity depends on.  They live in
the test build of the library (lib/libdesamba_test.so, include/desamba_mi355x_test.h), which runs in
a process of its own (tests/selftest_worker.py)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

WHICH = [0, 1, 2, 3, 4]
NS = [2, 3, 7, 64, 400]
WORKER = os.path.join(ROOT, "tests", "selftest_worker.py")


@pytest.fixture(scope="module")
def sort_results():
    cases = [[n, 512, w, 1000 + n] for w in WHICH for n in NS]
    r = subprocess.run([sys.executable, WORKER, "sort", json.dumps(cases)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-800:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    return {(c[2], c[0]): v for c, v in zip(cases, res)}


@pytest.mark.parametrize("which", WHICH,
                         ids=["chain_cmp_by_pos", "chain_cmp_by_MEM_score", "chain_cmp_by_score",
                              "Anchor_cmp_by_chr_ID_and_pos", "MEM_rst_cmp_by_match_len"])
@pytest.mark.parametrize("n", NS)
def test_glibc_msort_restatement_same_on_device_and_host(sort_results, which, n):
    """dsb_msort (glibc 2.35 msort_with_tmp restated) gives the host permutation on gfx950.
    which=0 pins the hipcc mis-scheduling of the early-return comparator form."""
    assert sort_results[(which, n)] == 0
