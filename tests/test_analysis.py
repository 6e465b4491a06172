"""The evaluation commands (`deSAMBA analysis`) against the reference.

desamba-so_amd/bin/desamba_analysis restates the reference's documented analysis commands
(reference src/analysis.c:2684-2689: ana_meta, ana_meta_base, count_base, split_fastq,
fastq_to_fasta, and the trailing print_list switch).  Each case runs the compiled reference
(oracle/_ref/deSAMBA analysis ...) and the restatement on the same committed files and requires
byte-identical stdout and stderr.  Host only (no GPU).
"""
import gzip
import os
import subprocess

import pytest

from conftest import ROOT, golden

REF = os.path.join(ROOT, "oracle", "_ref", "deSAMBA")
ANA = os.path.join(ROOT, "desamba-so_amd", "bin", "desamba_analysis")

CASES = [
    ("ana_meta", "mixed.herm.sam_full"),
    ("ana_meta", "ont.herm.sam"),
    ("ana_meta", "illumina.herm.sam"),
    ("ana_meta_base", "mixed.herm.sam_full"),
    ("ana_meta_base", "ont_long.herm.sam"),
    ("ana_meta_base", "illumina.herm.sam"),
    ("ana_meta", "ont.t1.sam"),
]


@pytest.fixture(scope="module")
def tools():
    if not os.path.exists(ANA):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "desamba-so_amd"), "bin/desamba_analysis"], check=True,
                       timeout=600)
    if not os.path.exists(REF):
        pytest.skip("oracle/_ref/deSAMBA not built (oracle/Makefile needs the reference sources)")
    return REF, ANA


def _both(tools, args, cwd):
    ref, ana = tools
    r = subprocess.run([ref, "analysis"] + args, capture_output=True, cwd=cwd, timeout=300)
    m = subprocess.run([ana] + args, capture_output=True, cwd=cwd, timeout=300)
    return r, m


@pytest.mark.parametrize("cmd,sam", CASES)
@pytest.mark.parametrize("print_list", [False, True])
def test_ana_meta_reports_identical(tools, fixture_index, tmp_path, cmd, sam, print_list):
    (tmp_path / "in.sam").write_bytes(golden(sam))
    args = [cmd, "in.sam", os.path.join(fixture_index, "nodes.dmp")] + (["print_list"] if print_list else [])
    r, m = _both(tools, args, tmp_path)
    assert r.returncode == 0
    assert m.stdout == r.stdout
    assert m.stderr == r.stderr
    assert b"TID:1 " in m.stdout or print_list


@pytest.mark.parametrize("name", ["ont", "illumina", "mixed", "ont_long"])
def test_fastq_utilities_identical(tools, tmp_path, name):
    data = golden(name + ".fq")
    (tmp_path / "r.fq").write_bytes(data)
    with gzip.open(tmp_path / "r.fq.gz", "wb") as f:
        f.write(data)
    for args in (["count_base", "r.fq"], ["count_base", "r.fq.gz"], ["split_fastq", "r.fq", "3", "7"],
                 ["split_fastq", "r.fq.gz", "0", "1"], ["fastq_to_fasta", "r.fq"]):
        r, m = _both(tools, args, tmp_path)
        assert (m.stdout, m.stderr) == (r.stdout, r.stderr), args
