"""GPU tests that need the library's test hooks (forced staging overflows, capacities below the
defaults, stale sp_set pool generations, a fixed batch-to-context order).  The hooks exist only in
the test build of the library (lib/libdesamba_test.so, -DDSB_TEST_HOOKS=1; kernels.hip and
pipeline.c); the production library ignores the same environment variables, which
test_production_library_ignores_test_hooks checks.  Each scenario runs in a process of its own
(tests/hook_worker.py) so that the library and its environment are chosen before it loads.
"""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT, golden
from samutil import groups

pytestmark = pytest.mark.gpu

TEST_LIB = os.path.join(ROOT, "desamba-so_amd", "lib", "libdesamba_test.so")
PROD_LIB = os.path.join(ROOT, "desamba-so_amd", "lib", "libdesamba.so")
WORKER = os.path.join(ROOT, "tests", "hook_worker.py")


def run_worker(tmp_path, tag, index, inputs, env, lib=TEST_LIB, mode="text", fmt=1, max_read_l=0):
    """-> (list of output bytes per input, summary dict) of one hook_worker process."""
    if not os.path.exists(lib):
        pytest.fail(f"{lib} not built (make -C desamba-so_amd)")
    spec = {"index": index, "inputs": [str(p) for p in inputs], "fmt": fmt, "mode": mode,
            "out": str(tmp_path / f"{tag}.out"), "max_read_l": max_read_l}
    sp = tmp_path / f"{tag}.json"
    sp.write_text(json.dumps(spec))
    e = {k: v for k, v in os.environ.items() if not k.startswith("DSB_")}
    e.update({"DSB_LIB": lib, "DSB_DEVICE": os.environ.get("DSB_DEVICE", "0")})
    e.update(env)
    r = subprocess.run([sys.executable, "-u", WORKER, str(sp)], capture_output=True, env=e, timeout=300)
    assert r.returncode == 0, (tag, r.returncode, r.stderr.decode()[-2000:])
    summary = json.loads(r.stdout.decode().strip().splitlines()[-1])
    summary["stderr"] = r.stderr.decode(errors="replace")
    outs = [open(f"{spec['out']}.{k}", "rb").read() for k in range(len(inputs))]
    return outs, summary


def _golden_files(tmp_path, names):
    out = []
    for n in names:
        p = tmp_path / f"{n}.fq"
        p.write_bytes(golden(n + ".fq"))
        out.append(p)
    return out


def test_staging_overflow_replay_is_byte_identical(fixture_index, tmp_path):
    """DSB_WAVE_DBG=32: two anchors of staging per lane, so every seed group of fast and slow
    seeding takes the in-order replay path: still byte-identical to the hermetic goldens."""
    names = ("mixed", "ont", "ont_long")
    outs, _ = run_worker(tmp_path, "dbg32", fixture_index, _golden_files(tmp_path, names), {"DSB_WAVE_DBG": "32"})
    for name, out in zip(names, outs):
        assert out == golden(name + ".herm.sam"), name


def test_overflow_reruns_byte_identical(fixture_index, tmp_path):
    """Every read starts at 1/8 of the default workspace capacities (DSB_TEST_SCALE0=1), so many
    overflow and are re-run with larger capacities in the retry buffer (several rounds, and with
    a small budget several chunks): still byte-identical to the hermetic reference."""
    names = ("mixed", "ont", "ont_long")
    files = _golden_files(tmp_path, names)
    for budget in (None, "8"):
        env = {"DSB_TEST_SCALE0": "1"}
        if budget:
            env["DSB_WS_BUDGET_MB"] = budget
        outs, summ = run_worker(tmp_path, f"scale0_{budget}", fixture_index, files, env)
        for name, out in zip(names, outs):
            assert out == golden(name + ".herm.sam"), (name, budget)
        assert sum(c["n_retry"] for c in summ["calls"]) > 0


def test_deferred_reruns_beyond_the_largest_chunk(fixture_index, tmp_path):
    """Overflow re-runs deferred to the end of a batch (kernels.hip batch_run) from many small
    chunks: far more deferred reads than any chunk holds, so the re-run's order / carry arrays must
    be sized for all of them (round-4 advisor finding: they were sized per chunk).  Batch API; every
    2nd read takes the re-run path (DSB_TEST_FORCE_RERUN) and every one is deferrable (the run
    starts from a carry above every read length); byte-identical to the production library's run of
    the same batch, with deferral on and off."""
    fq = tmp_path / "ont_x3.fq"
    fq.write_bytes(golden("ont.fq") * 3)  # 6000 reads
    carry = 1 << 20
    want, _ = run_worker(tmp_path, "prod", fixture_index, [fq], {}, lib=PROD_LIB, mode="batch", max_read_l=carry)
    for defer in ("1", "0"):
        env = {"DSB_TEST_FORCE_RERUN": "2", "DSB_WS_BUDGET_MB": "64", "DSB_DEFER_RETRY": defer}
        got, s = run_worker(tmp_path, f"defer{defer}", fixture_index, [fq], env, mode="batch", max_read_l=carry)
        c = s["calls"][0]
        print(f"defer {defer}: {c['n_retry']} re-runs over {c['n_chunks']} chunks")
        assert c["n_retry"] >= 3000 and c["n_chunks"] > 20, c
        assert got[0] == want[0], defer


def test_deferred_reruns_in_groups(fixture_index, tmp_path):
    """The deferred re-runs of one call go in groups whose re-run workspace fits the HBM the chunk
    workspace leaves (kernels.hip batch_run; round 5: a repeat-rich proxy overflowed thousands of
    reads of a 1M-read call and the single re-run buffer did not fit beside a 220-GB chunk
    workspace).  Groups of at most 4 MB (DSB_TEST_RETRY_GROUP_MB): hundreds of groups, each with its
    own part B and hit gather, records byte-identical to the production library's."""
    fq = tmp_path / "ont_x2.fq"
    fq.write_bytes(golden("ont.fq") * 2)
    carry = 1 << 20
    want, _ = run_worker(tmp_path, "prod", fixture_index, [fq], {}, lib=PROD_LIB, mode="batch", max_read_l=carry)
    env = {"DSB_TEST_FORCE_RERUN": "3", "DSB_WS_BUDGET_MB": "64", "DSB_DEFER_RETRY": "1",
           "DSB_TEST_RETRY_GROUP_MB": "4"}
    got, s = run_worker(tmp_path, "groups", fixture_index, [fq], env, mode="batch", max_read_l=carry)
    c = s["calls"][0]
    assert c["n_retry"] >= 1300, c
    assert got[0] == want[0]


def test_deferred_reruns_after_the_chunk_workspace_is_released(fixture_index, tmp_path):
    """The deferred re-runs when the chunk workspace has been released for them (kernels.hip
    batch_run: a 220-GB chunk workspace leaves too little HBM for a large group; forced here with
    DSB_TEST_RELEASE_WS).  Round 6: the re-run kernels were then given a null workspace base with
    absolute offsets, and four reads of a 1M-read c2l18 batch lost a replayed seed's anchors (M3's
    NULL case, status 8, "overflows every workspace size"); the retry buffer is now allocated
    first and is the base.  Every 2nd read re-runs (DSB_TEST_FORCE_RERUN), tiny staging makes the
    seeding replay seeds in order (DSB_WAVE_DBG=32), workspace bytes are pre-filled
    (DSB_TEST_WS_FILL): records byte-identical to the production library's run."""
    fq = tmp_path / "ont_x2.fq"
    fq.write_bytes(golden("ont.fq") * 2)
    carry = 1 << 20
    want, _ = run_worker(tmp_path, "prod", fixture_index, [fq], {}, lib=PROD_LIB, mode="batch", max_read_l=carry)
    env = {"DSB_TEST_FORCE_RERUN": "2", "DSB_DEFER_RETRY": "1", "DSB_TEST_RELEASE_WS": "1", "DSB_WAVE_DBG": "32",
           "DSB_TEST_WS_FILL": "0x5A", "DSB_HOST_TIMING": "1"}
    got, s = run_worker(tmp_path, "released", fixture_index, [fq], env, mode="batch", max_read_l=carry)
    assert s["calls"][0]["n_retry"] >= 2000, s["calls"][0]
    assert "deferred re-runs" in s["stderr"]
    assert got[0] == want[0]


@pytest.mark.parametrize("cost", ["1", "300000"])
def test_heavy_reads_scored_over_waves_byte_identical(fixture_index, tmp_path, cost):
    """The heavy reads' scoring (dsb_kern.h k_heavy_prep / k_heavy_spec / k_heavy_fin): every chain
    of a read scored speculatively on its own wave, then accepted in chain order or scored again.
    DSB_HEAVY_COST=1 sends every read with a chain that way (300000: the longer / many-chain
    ones); records byte-identical to the one-wave-per-read scoring (DSB_HEAVY_SPEC=0), batch and
    text paths."""
    fq = tmp_path / "ont_x2.fq"
    fq.write_bytes(golden("ont.fq") * 2)
    for mode in ("batch", "text"):
        want, _ = run_worker(tmp_path, f"one_{mode}", fixture_index, [fq], {"DSB_HEAVY_SPEC": "0"}, lib=PROD_LIB,
                             mode=mode)
        got, s = run_worker(tmp_path, f"heavy_{mode}_{cost}", fixture_index, [fq], {"DSB_HEAVY_COST": cost, "DSB_HEAVY_SPEC": "1"},
                            lib=PROD_LIB, mode=mode)
        nh = sum(c.get("n_heavy", 0) for c in s["calls"])
        print(f"{mode} cost {cost}: {nh} heavy reads")
        assert nh > 0, s["calls"]
        assert got[0] == want[0], (mode, cost)


@pytest.mark.parametrize("cost", ["1", "300000"])
def test_rerun_heavy_reads_scored_over_waves_byte_identical(fixture_index, tmp_path, cost):
    """DSB_RETRY_SPEC=1 (kernels.hip retry_score): an overflow re-run scores its heavy reads over
    DSB_HEAVY_W waves each beside the one-wave scoring of the rest; unlike the chunk's split, the
    re-run's list also takes reads that went through slow seeding.  Every 2nd read re-runs
    (DSB_TEST_FORCE_RERUN), deferred to the end of the batch and chunk by chunk;
    DSB_RETRY_HEAVY_COST=1 (the default) sends every re-run read with a chain that way.  Records byte-identical to the production
    library's run; the text path against the hermetic goldens with capacities below the defaults."""
    fq = tmp_path / "ont_x2.fq"
    fq.write_bytes(golden("ont.fq") * 2)
    carry = 1 << 20
    want, _ = run_worker(tmp_path, "prod", fixture_index, [fq], {}, lib=PROD_LIB, mode="batch", max_read_l=carry)
    for defer in ("1", "0"):
        env = {"DSB_TEST_FORCE_RERUN": "2", "DSB_DEFER_RETRY": defer, "DSB_RETRY_SPEC": "1", "DSB_RETRY_HEAVY_COST": cost,
               "DSB_HOST_TIMING": "1"}
        got, s = run_worker(tmp_path, f"rspec{defer}_{cost}", fixture_index, [fq], env, mode="batch", max_read_l=carry)
        assert s["calls"][0]["n_retry"] >= 2000, s["calls"][0]
        nh = [int(l.split()[2]) for l in s["stderr"].splitlines() if "re-run reads scored over" in l]
        print(f"defer {defer} cost {cost}: {sum(nh)} re-run reads over waves in {len(nh)} re-runs")
        assert sum(nh) > 0
        assert got[0] == want[0], (defer, cost)
    names = ("mixed", "ont", "ont_long")
    outs, summ = run_worker(tmp_path, f"rspec_scale0_{cost}", fixture_index, _golden_files(tmp_path, names),
                            {"DSB_TEST_SCALE0": "1", "DSB_RETRY_SPEC": "1", "DSB_RETRY_HEAVY_COST": cost})
    assert sum(c["n_retry"] for c in summ["calls"]) > 0
    for name, out in zip(names, outs):
        assert out == golden(name + ".herm.sam"), (name, cost)


def test_sp_set_pool_sets_never_match_stale_slots(fixture_index, tmp_path):
    """Regression test for round 3's lost-anchor race, in its round-4 form: the seeding sp_set
    slots are never cleared; they live in a per-GPU pool of wave-sized sets that seeding waves take
    and hand back (dsb_kern.h dsb_hpool_acquire / dsb_hpool_release), and a slot matches only the
    generations of its current holder because every holder moves the set's generation base past the
    generations it used.  Deterministic form: the same reads X run again and again (X X X X X over
    two batches, DSB_PIPE_READS = 4 |X|, two contexts sharing one GPU's pool with
    DSB_GPU_CONTEXTS=2, DSB_TEST_ROUND_ROBIN for the batch-to-context order), so the same reads'
    seeding waves take sets that waves with the same nodes held before.  Every copy of X must give
    X's records.  With the base kept in place and sets picked by read length (DSB_WAVE_DBG bit 13,
    DSB_DBG_POOL_NOGEN), a later copy of a read takes the set an earlier copy filled, meets its
    slots as live and drops anchors, which this test detects."""
    lines = golden("ont.fq").split(b"\n")
    x = b"\n".join(lines[:800]) + b"\n"  # the first 200 four-line records
    assert x.count(b"\n+\n") == 200
    fq = tmp_path / "x5.fq"
    fq.write_bytes(x * 5)
    env = {"DSB_DEVICES": "0", "DSB_GPU_CONTEXTS": "2", "DSB_PIPE_READS": "800", "DSB_TEST_ROUND_ROBIN": "1"}
    (out,), s = run_worker(tmp_path, "pool", fixture_index, [fq], env)
    assert s["devices"] == [0, 0]
    assert s["calls"][0]["n_batches"] == 2 and s["calls"][0]["n_devices"] == 2
    g = groups(out)
    assert len(g) == 1000
    first = g[:200]
    for c in range(1, 5):
        assert g[200 * c:200 * (c + 1)] == first, f"copy {c} of the reads differs"
    assert first == groups(golden("ont.herm.sam"))[:200]
    (bad,), _ = run_worker(tmp_path, "pool_nogen", fixture_index, [fq], dict(env, DSB_WAVE_DBG=str(1 << 13)))
    assert groups(bad) != g, "pool sets handed back without moving their generation base should drop rows: " \
        "the test would not detect stale slots"


def test_production_library_ignores_test_hooks(fixture_index, tmp_path):
    """The same switches given to the production library change nothing: no forced re-runs, no
    stale pool generations, the hermetic records."""
    files = _golden_files(tmp_path, ("ont",))
    (plain,), s0 = run_worker(tmp_path, "prod_plain", fixture_index, files, {}, lib=PROD_LIB)
    env = {"DSB_TEST_SCALE0": "1", "DSB_WAVE_DBG": str((1 << 13) | 32), "DSB_WAVE_PHASES": "0"}
    (out,), s = run_worker(tmp_path, "prod_hooks", fixture_index, files, env, lib=PROD_LIB)
    assert s["calls"][0]["n_retry"] == s0["calls"][0]["n_retry"]
    assert out == plain == golden("ont.herm.sam")


def test_fenced_pool_hand_over_byte_identical(fixture_index, tmp_path):
    """The fallback dev_init takes when the XCC ids the device's waves report are not exactly
    0..n-1 (or the XCC count is unknown): one sp_set pool partition, every hand-over an agent-scope
    release / acquire.  Forced here (DSB_TEST_POOL_FENCED), two contexts sharing the pool."""
    names = ("mixed", "ont")
    env = {"DSB_TEST_POOL_FENCED": "1", "DSB_DEVICES": "0", "DSB_GPU_CONTEXTS": "2", "DSB_PIPE_READS": "300"}
    outs, s = run_worker(tmp_path, "fenced", fixture_index, _golden_files(tmp_path, names), env)
    assert "sp_set pool hand-over fenced" in s["stderr"]
    for name, out in zip(names, outs):
        assert out == golden(name + ".herm.sam"), name


def test_production_pool_is_not_fenced_on_mi355x(fixture_index, tmp_path):
    """On the MI355X (8 XCDs, ids 0..7) the load-time check passes and the pool runs unfenced."""
    _, s = run_worker(tmp_path, "unfenced", fixture_index, _golden_files(tmp_path, ("illumina",)), {}, lib=PROD_LIB)
    assert "hand-over fenced" not in s["stderr"], s["stderr"][-500:]
