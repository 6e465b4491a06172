"""The drop-in boundary: libdesamba.so loads without a GPU and exports exactly the C-ABI
declared in include/*.h (desamba.h = the reference's three entry points)."""
import os
import re
import subprocess
import sys

import pytest

from conftest import ROOT

LIB = os.path.join(ROOT, "desamba-so_amd", "lib", "libdesamba.so")


def _declared(headers=("desamba.h", "desamba_mi355x.h")):
    names = set()
    for h in headers:
        with open(os.path.join(ROOT, "include", h)) as f:
            text = re.sub(r"/\*.*?\*/", "", f.read(), flags=re.S)
        text = re.sub(r"//[^\n]*", "", text)
        for m in re.finditer(r"^[A-Za-z_][\w \t\*]*?\b([A-Za-z_]\w*)\s*\([^;{]*\)\s*;", text, re.M):
            if not m.group(0).lstrip().startswith(("typedef", "#")):
                names.add(m.group(1))
    return names


@pytest.fixture(scope="module")
def exported():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "desamba-so_amd")], check=True, timeout=900)
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    return {l.split()[-1] for l in out.splitlines() if " T " in l}


def test_reference_entry_points_exported(exported):
    assert {"load_index", "read_classify", "meta_analysis"} <= exported


def test_every_declared_function_is_exported(exported):
    decl = _declared()
    assert {"load_index", "read_classify", "meta_analysis", "dsb_batch_run", "dsb_classify_text"} <= decl
    assert decl <= exported, decl - exported


def test_no_undeclared_exports(exported):
    extra = exported - _declared()
    assert not extra, extra


def test_library_loads_without_gpu(pyd):
    L = pyd.lib()
    assert L.dsb_version().decode().startswith("desamba-mi355x")
    assert L.dsb_device_count() >= 0


def test_load_index_fails_loudly_without_gpu(pyd, fixture_index):
    """No CPU fallback: with no GPU, load_index aborts like the reference's err_fatal."""
    if pyd.lib().dsb_device_count() > 0:
        pytest.skip("a GPU is present")
    code = ("import sys; sys.path.insert(0, %r); import pydesamba; pydesamba.Index(%r); print('LOADED')"
            % (os.path.join(ROOT, "desamba-so_amd"), fixture_index))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "LOADED" not in r.stdout
    assert "load_index" in r.stderr


TEST_LIB = os.path.join(ROOT, "desamba-so_amd", "lib", "libdesamba_test.so")
HOOK_ENV = ("DSB_TEST_SCALE0", "DSB_TEST_ROUND_ROBIN", "DSB_WAVE_PHASES", "DSB_TEST_FORCE_RERUN", "DSB_TEST_POOL_FENCED",
            "DSB_TEST_RETRY_GROUP_MB", "DSB_TEST_WS_FILL",
            "DSB_TEST_RELEASE_WS")


def _strings(path):
    with open(path, "rb") as f:
        return set(re.findall(rb"[\x20-\x7e]{6,}", f.read()))


def test_test_hooks_only_in_the_test_build():
    """The env-reachable test hooks (forced overflows, lane-per-read phases, batch-to-context
    order) are compiled into lib/libdesamba_test.so only; the production library does not even
    read those variables (kernels.hip / pipeline.c DSB_TEST_HOOKS)."""
    if not os.path.exists(TEST_LIB):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "desamba-so_amd")], check=True, timeout=900)
    prod, test = _strings(LIB), _strings(TEST_LIB)
    for name in HOOK_ENV:
        assert name.encode() not in prod, name
        assert name.encode() in test, name
    out = subprocess.run(["nm", "-D", "--defined-only", TEST_LIB], capture_output=True, text=True, check=True).stdout
    test_exports = {l.split()[-1] for l in out.splitlines() if " T " in l}
    test_only = _declared(("desamba_mi355x_test.h",))
    assert {"dsb_gpu_selftest_sort", "dsb_gpu_selftest_occ"} <= test_only
    assert test_exports == _declared() | test_only, test_exports ^ (_declared() | test_only)
    # the device self-tests are not in the production library at all
    assert not (test_only & {l.split()[-1] for l in subprocess.run(
        ["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout.splitlines() if " T " in l})
