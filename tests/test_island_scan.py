"""The island scan in batches of G positions (k_island_g's logic: dsb_isl_* + dsb_top_push in
desamba-so_amd/csrc/gpu/dsb_classify.h) equals the one-bit-at-a-time scan + top-seed pass (the
reference's search_exist_kmer_M2 / get_seed_vector_M2, src/cly.c:1066-1229) on the same exist
bits — seeds, counts, total score and every stale top-byte write (tests/emu/isl_check.cpp)."""
import os
import subprocess

import pytest

from conftest import ROOT

EXE = os.path.join(ROOT, "build", "emu", "isl_check")


@pytest.mark.parametrize("seed", [5, 77])
def test_batched_island_scan_equals_bitwise_scan(seed):
    if not os.path.exists(EXE):
        pytest.skip("tests/emu not built")
    r = subprocess.run([EXE, str(seed), "20000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and " 0 mismatches" in r.stdout, r.stdout + r.stderr
