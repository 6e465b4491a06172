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


TAX_CASES = [
    ("ana_species", "5034", None),
    ("ana_genus", "4002", None),
    ("ana_sam", "2", "null"),
    ("ana_sam", "3002", "family"),
    ("ana_sam", "5032", "null"),
    ("ana_sam", "1", "null"),
    ("ana_sam", "2", "superkingdom"),
]


@pytest.mark.parametrize("sam", ["ont.herm.sam", "mixed.herm.sam_full", "illumina.t1.sam"])
@pytest.mark.parametrize("cmd,tid,rank", TAX_CASES)
def test_ana_tax_accuracy_identical(tools, fixture_index, tmp_path, sam, cmd, tid, rank):
    """ana_species / ana_genus / ana_sam (reference src/analysis.c:1073-1234, 2014-2025): the
    per-read UM / PRI / SEC verdicts against one true taxon (stdout) and the totals and rates
    (stderr), byte-identical."""
    (tmp_path / "in.sam").write_bytes(golden(sam))
    args = [cmd, "in.sam", tid, os.path.join(fixture_index, "nodes.dmp")] + ([rank] if rank else [])
    r, m = _both(tools, args, tmp_path)
    assert r.returncode == 0
    assert (m.stdout, m.stderr) == (r.stdout, r.stderr)
    assert m.stderr.startswith(b"in.sam.temp\t")


def test_ana_species_per_simulated_source_taxon(tools, fixture_index, tmp_path):
    """Scoring against simulated truth: tools/simulate.py names each read rd<i>_<taxid>_...; the
    records of the reads of each source taxon are scored with ana_species against that taxon,
    by both tools, on the hermetic reference's records of the ONT set."""
    groups = {}
    for line in golden("ont.herm.sam").splitlines(keepends=True):
        name = line.split(b"\t", 1)[0]
        parts = name.split(b"_")
        if len(parts) >= 3 and parts[1].isdigit():
            groups.setdefault(parts[1].decode(), []).append(line)
    assert len(groups) >= 3
    for tid, lines in sorted(groups.items()):
        (tmp_path / "t.sam").write_bytes(b"".join(lines))
        r, m = _both(tools, ["ana_species", "t.sam", tid, os.path.join(fixture_index, "nodes.dmp")], tmp_path)
        assert (m.stdout, m.stderr) == (r.stdout, r.stderr), tid


def test_ana_tax_empty_sam_identical(tools, fixture_index, tmp_path):
    (tmp_path / "e.sam").write_bytes(b"")
    """The reference aborts in skip_sam_head on a SAM file without records (analysis.c:343)."""
    (tmp_path / "h.sam").write_bytes(b"@HD\tVN:1.0\n")
    for f in ("e.sam", "h.sam"):
        for cmd in (["ana_genus", f, "4002"], ["ana_meta", f]):
            r, m = _both(tools, cmd[:2] + cmd[2:] + [os.path.join(fixture_index, "nodes.dmp")], tmp_path)
            assert r.returncode == m.returncode != 0
            assert (m.stdout, m.stderr) == (r.stdout, r.stderr)
