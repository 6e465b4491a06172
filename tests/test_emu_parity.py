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
