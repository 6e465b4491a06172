"""The C restatement of the hot-path primitives (oracle/restate.c), pinned against the
reference's own compiled functions by oracle/_ref/restate_check (oracle/Makefile `restate`):
occ, hash64_1/2, store_kmers, get_exist_kmer, get_ref, get_uni, lv_extd, bwt_MEM_search
(fast and slow parameters, with the sp_set) and glibc qsort vs the msort restatement, on the
committed fixture index and seeded random / simulated inputs."""
import os
import subprocess

import pytest

from conftest import ROOT

EXE = os.path.join(ROOT, "oracle", "_ref", "restate_check")


@pytest.mark.parametrize("seed", [1, 20261016])
def test_restatement_matches_reference_primitives(fixture_index, seed):
    if not os.path.exists(EXE):
        pytest.skip("oracle/_ref/restate_check not built (needs the reference sources)")
    r = subprocess.run([EXE, fixture_index, str(seed)], capture_output=True, text=True, timeout=600)
    lines = [l for l in r.stdout.splitlines() if l.startswith("restate_check")]
    assert r.returncode == 0, r.stdout + r.stderr[-2000:]
    checked = {l.split()[1] for l in lines if "mismatches" in l}
    assert {"occ", "hash64", "store_kmers", "exist_kmer", "get_ref", "get_uni", "lv_extd", "mem_search",
            "msort"} <= checked
    for l in lines:
        if "mismatches" in l:
            f = l.split()
            assert int(f[2]) > 0 and int(f[4]) == 0, l
