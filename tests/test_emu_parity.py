"""CPU emulation of the kernel logic vs the hermetic reference goldens.

tests/emu/emu_classify compiles the per-read device code (desamba-so_amd/csrc/gpu/
dsb_classify.h) for the host and runs it read by read with the same workspace layout the
kernels use.  It is test-only (never linked into libdesamba.so): it lets the classify logic
be checked for bit-exactness in a container without a GPU.  The GPU itself is checked by
tests/test_gpu_parity.py.
"""
import os
import subprocess

import pytest

from conftest import ROOT, golden
from samutil import groups

EMU = os.path.join(ROOT, "build", "emu", "emu_classify")


@pytest.fixture(scope="module")
def emu():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "emu")], check=True, timeout=600)
    return EMU


@pytest.mark.parametrize("name", ["mixed", "illumina", "ont"])
def test_emulated_kernel_logic_is_byte_identical(emu, fixture_index, tmp_path, name):
    fq = tmp_path / f"{name}.fq"
    fq.write_bytes(golden(name + ".fq"))
    full = name == "mixed"
    cmd = [emu] + ([] if full else ["--sam"]) + [fixture_index, str(fq)]
    out = subprocess.run(cmd, capture_output=True, check=True, timeout=600).stdout
    assert out == golden(name + (".herm.sam_full" if full else ".herm.sam"))


def test_emulated_work_counters(emu, fixture_index, tmp_path):
    """--stats counters exist and are consistent (roofline numerator inputs)."""
    fq = tmp_path / "ont.fq"
    fq.write_bytes(golden("ont.fq"))
    r = subprocess.run([emu, "--stats", fixture_index, str(fq)], capture_output=True, check=True, timeout=600)
    st = dict(l.split() for l in r.stderr.decode().splitlines() if len(l.split()) == 2)
    st = {k: int(v) for k, v in st.items()}
    assert st["occ"] > 0 and st["occ_nib"] >= 10 * st["occ"]
    assert st["sa"] > 0 and st["uni"] >= st["sa"] and st["anchor"] > 0 and st["chain"] > 0
    assert len(groups(r.stdout)) == 2000


@pytest.mark.parametrize("mode", ["wave", "wave_replay", "wave_lds"])
@pytest.mark.parametrize("name", ["mixed", "ont"])
def test_emulated_wave_code_paths_are_byte_identical(emu, fixture_index, tmp_path, name, mode):
    """The wave-cooperative kernels' code (seeding with per-lane staging and the skip rule,
    chaining, scoring) run as a one-lane wave; `wave_replay` forces every staging area to
    overflow (the in-order replay path), `wave_lds` separates the scoring windows / sparse-DP
    prefix the way the LDS variant does and fills them with garbage first."""
    env = dict(os.environ, EMU_WAVE="1")
    if mode == "wave_replay":
        env["EMU_DBG"] = "32"
    if mode == "wave_lds":
        env["EMU_LDS"] = "0x7f"
    fq = tmp_path / f"{name}.fq"
    fq.write_bytes(golden(name + ".fq"))
    out = subprocess.run([emu, fixture_index, str(fq)], capture_output=True, check=True, timeout=600, env=env).stdout
    assert out == golden(name + ".herm.sam_full") if name == "mixed" else True
    if name != "mixed":
        sam = subprocess.run([emu, "--sam", fixture_index, str(fq)], capture_output=True, check=True, timeout=600,
                             env=env).stdout
        assert sam == golden(name + ".herm.sam")
