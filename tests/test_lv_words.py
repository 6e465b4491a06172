"""The GPU path's register-word lv_extd (dsb_lv_extd_w) agrees with the byte-buffer form and with
the oracle restatement of the reference's lv_extd (tests/emu/lv_check.cpp, CPU build of the
device header) on seeded random windows: substitutions, indels, ragged lengths, guard bytes."""
import os
import subprocess

import pytest

from conftest import ROOT

EXE = os.path.join(ROOT, "build", "emu", "lv_check")


@pytest.mark.parametrize("seed", [3, 99])
def test_word_lv_matches_byte_lv_and_oracle(seed):
    if not os.path.exists(EXE):
        pytest.skip("tests/emu not built")
    r = subprocess.run([EXE, str(seed), "1000000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 mismatches" in r.stdout


@pytest.mark.parametrize("words", [1, 2, 4])
def test_word_mem_search_matches_byte_loop(words):
    """dsb_MEM_search reading 8 x DSB_MEM_WORDS bytes per step == the reference's byte loop
    (src/cly.c:1805-1813) in both directions for every max (tests/emu/mem_check.cpp)."""
    exe = os.path.join(ROOT, "build", "emu", f"mem_check{words}")
    if not os.path.exists(exe):
        pytest.skip("tests/emu not built")
    r = subprocess.run([exe, "11", "300000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and " 0 mismatches" in r.stdout, r.stdout
