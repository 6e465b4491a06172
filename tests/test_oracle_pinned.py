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


@pytest.mark.parametrize("name", ["mixed", "ont"])
@pytest.mark.parametrize("fmt", ["des", "des_full"])
def test_hermetic_reference_reproduces_des_goldens(fixture_index, tmp_path, name, fmt):
    """DES / DES_FULL goldens = the reference's own writers (cly_mt.c:144-227) via the harness."""
    exe = _need("herm_classify")
    fq = tmp_path / f"{name}.fq"
    fq.write_bytes(golden(name + ".fq"))
    out = subprocess.run([exe, "--" + fmt.replace("_", "-"), fixture_index, str(fq)], capture_output=True,
                         check=True, timeout=300).stdout
    assert out == golden(f"{name}.herm.{fmt}")


def test_ekmer_table_restatement_equals_builder_tables(fixture_index):
    """oracle/ekmer_tables (get_EXIST_kmer restated, idx.c:986-1027) rebuilds the fixture index's
    128 MB l_ek-16 tables byte for byte from its unitigs (the GPU box uses it to make the l_ek-17
    variant of the C1 proxy, tests/test_gpu_scale.py)."""
    exe = _need("ekmer_tables")
    r = subprocess.run([exe, fixture_index, str(1 << 27), "/nonexistent", "--check"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("identical"), r.stdout


@pytest.mark.parametrize("preset,size", [("c1", 1 << 27), ("c2", 1 << 28)])
def test_ekmer_tables_equal_builder_on_proxy_indexes(preset, size):
    """The same on the C1 proxy (l_ek 16) and, where it was built (development container,
    tools/make_proxy_index.sh c2), the 495 Mbp / 286 M 31-mer C2 proxy, whose builder-made
    tables are the quarter-GB l_ek-17 / MASK_31 ones (idx.c:966-996)."""
    exe = _need("ekmer_tables")
    d = os.path.join(ROOT, "build", preset, "idx")
    if not os.path.exists(os.path.join(d, "deSAMBA.exk0")):
        pytest.skip(f"{d} not built here")
    r = subprocess.run([exe, d, str(size), "/nonexistent", "--check"], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0 and r.stdout.startswith("identical"), r.stdout
