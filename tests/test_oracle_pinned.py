"""The oracle, pinned: the committed goldens are reproduced by the reference itself.

oracle/_ref holds the reference classifier compiled from the reference sources
(oracle/Makefile: `deSAMBA` gcc -O3 = the reference's own build flags, and `herm_classify`,
the hermetic harness = reference objects built with clang -ftrivial-auto-var-init=pattern,
fresh buffer pools per read, MALLOC_PERTURB 165).  These tests re-run them on the committed
inputs and require byte-identical output to the committed fixtures, so the fixtures the GPU
tests compare against are exactly what the reference produces.
"""
import hashlib
import json
import os
import subprocess

import pytest

from conftest import GOLDEN, ROOT, golden

REF = os.path.join(ROOT, "oracle", "_ref")


def _need(exe):
    p = os.path.join(REF, exe)
    if not os.path.exists(p):
        pytest.skip(f"{p} not built (oracle/Makefile needs the reference sources)")
    return p


def test_golden_manifest_checksums():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        man = json.load(f)
    for name, meta in man["files"].items():
        with open(os.path.join(GOLDEN, name), "rb") as f:
            assert hashlib.sha256(f.read()).hexdigest() == meta["sha256_packed"], name
        if "sha256" in meta:
            assert hashlib.sha256(golden(name[:-3])).hexdigest() == meta["sha256"], name


@pytest.mark.parametrize("name", ["mixed", "illumina", "ont"])
def test_hermetic_reference_reproduces_goldens(fixture_index, tmp_path, name):
    exe = _need("herm_classify")
    fq = tmp_path / f"{name}.fq"
    fq.write_bytes(golden(name + ".fq"))
    out = subprocess.run([exe, "--sam", fixture_index, str(fq)], capture_output=True, check=True,
                         timeout=300).stdout
    assert out == golden(name + ".herm.sam")


def test_hermetic_reference_sam_full(fixture_index, tmp_path):
    exe = _need("herm_classify")
    fq = tmp_path / "mixed.fq"
    fq.write_bytes(golden("mixed.fq"))
    out = subprocess.run([exe, fixture_index, str(fq)], capture_output=True, check=True, timeout=300).stdout
    assert out == golden("mixed.herm.sam_full")


def test_reference_cli_t1_reproduces_goldens(fixture_index, tmp_path):
    """`deSAMBA classify -t 1` (the reference CLI) == the committed t1 fixture."""
    exe = _need("deSAMBA")
    fq = tmp_path / "mixed.fq"
    fq.write_bytes(golden("mixed.fq"))
    o = tmp_path / "o.sam"
    subprocess.run([exe, "classify", "-t", "1", "-f", "SAM_FULL", "-o", str(o), fixture_index, str(fq)],
                   capture_output=True, check=True, timeout=300)
    assert o.read_bytes() == golden("mixed.t1.sam_full")


def test_shared_pool_harness_equals_cli_t1(fixture_index, tmp_path):
    """The harness in --shared mode is the CLI's -t 1 path (pins the harness's pipeline emulation)."""
    exe = _need("ref_classify")
    fq = tmp_path / "mixed.fq"
    fq.write_bytes(golden("mixed.fq"))
    out = subprocess.run([exe, "--shared", "--no-perturb", fixture_index, str(fq)], capture_output=True, check=True,
                         timeout=300).stdout
    assert out == golden("mixed.t1.sam_full")
