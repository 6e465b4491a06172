"""Shared fixtures.  `-m gpu` tests need a MI355X; everything else runs on CPU."""
import hashlib
import importlib.util
import json
import lzma
import os
import subprocess
import tarfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X (gfx950) GPU")


def golden(name: str) -> bytes:
    """Unpacked content of tests/golden/<name>.xz"""
    with lzma.open(os.path.join(GOLDEN, name + ".xz")) as f:
        return f.read()


@pytest.fixture(scope="session")
def fixture_index(tmp_path_factory):
    """The committed fixture index (built by the reference builder), unpacked."""
    d = tmp_path_factory.mktemp("fixture_index")
    with tarfile.open(os.path.join(GOLDEN, "fixture_index.txz")) as t:
        t.extractall(d)
    return str(d)


def load_pydesamba():
    spec = importlib.util.spec_from_file_location("pydesamba", os.path.join(ROOT, "desamba-so_amd", "pydesamba.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.fixture(scope="session")
def pyd():
    return load_pydesamba()


@pytest.fixture(scope="session")
def gpu_index(fixture_index, pyd):
    idx = pyd.Index(fixture_index)
    yield idx
    idx.close()
