#!/usr/bin/env python3
"""profiles/traffic.json from two rocprofv3 --pmc passes of tools/gpu_session.sh (FETCH_SIZE in one,
WRITE_SIZE in the other; they cannot share a pass on gfx950) over the same bench.py workload:

    python tools/traffic_json.py gpurun_out/TAG WORKLOAD READS KERNEL_PREFIX[,PREFIX...] PROFILE_TAG

Per launch of each kernel (KERNEL_PREFIX, e.g. "k_wave_phase<8"; the bench's dominant kernel can be
either of two whose step times are close, so several may be given: "kernels" lists them all, and the
first one's figures also sit at the top level): FETCH_SIZE and WRITE_SIZE (KB)
summed over its dispatches of >= 1000 workgroups (the chunk launches the bench's HIP events time;
an overflow re-run of a few reads is a small launch) / the number of those dispatches; hbm_bytes_per_launch = 2 x FETCH + WRITE
(MI355X_MICROARCH.md: gfx950's FETCH_SIZE counts half of a streaming read's bytes), and the
random-access reading FETCH + WRITE (profiles/r03_calib: a random 4-B load is one 64-B unit and
FETCH_SIZE counts it whole) as hbm_bytes_per_launch_calibrated.
"""
import glob
import json
import re
import sqlite3
import sys


def per_launch(pass_dir, counter, prefix, min_grid=1000):
    dbs = glob.glob(f"{pass_dir}/**/*.db", recursive=True)
    if not dbs:
        raise SystemExit(f"no rocprofv3 database under {pass_dir}")
    db = sqlite3.connect(dbs[0])
    cols = [r[1] for r in db.execute("pragma table_info(counters_collection)")]
    did = "dispatch_id" if "dispatch_id" in cols else None
    tot, disp, name = 0.0, set(), None
    q = (f"select kernel_name, counter_name, value, grid_size, workgroup_size{', ' + did if did else ''} "
         "from counters_collection")
    n_rows = 0
    for row in db.execute(q):
        k, c, v = row[0], row[1], row[2]
        if row[3] // max(1, row[4]) < min_grid:  # an overflow re-run of a few reads, not a chunk launch
            continue
        m = re.match(r"(?:void )?([\w:]+(?:<[^>]*>)?)", k)
        k = m.group(1) if m else k
        if not k.startswith(prefix) or c != counter:
            continue
        name = k
        tot += v
        n_rows += 1
        if did:
            disp.add(row[5])
    n = len(disp) if did else n_rows
    return name, tot / max(1, n), n


def main():
    d, workload, reads, prefix, tag = sys.argv[1:6]
    fdir = wdir = None
    for cf in glob.glob(f"{d}/pmc_*/counters.txt"):
        ctr = open(cf).read().strip()
        if "FETCH_SIZE" in ctr:
            fdir = cf.rsplit("/", 1)[0]
        if "WRITE_SIZE" in ctr:
            wdir = cf.rsplit("/", 1)[0]
    ents = []
    for pf in prefix.split(","):
        kname, fetch_kb, nf = per_launch(fdir, "FETCH_SIZE", pf)
        _, write_kb, nw = per_launch(wdir, "WRITE_SIZE", pf)
        ents.append({"kernel": kname, "launches": [nf, nw],
                     "fetch_size_kb_per_launch": round(fetch_kb, 1), "write_size_kb_per_launch": round(write_kb, 1),
                     "hbm_bytes_per_launch": int(1024 * (2 * fetch_kb + write_kb)),
                     "hbm_bytes_per_launch_calibrated": int(1024 * (fetch_kb + write_kb))})
    out = dict({"workload": workload, "reads": int(reads), "tag": tag}, **ents[0])
    out.update({"correction": "2 x FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE counts half of 128-B requests)",
                "calibration": "FETCH_SIZE + WRITE_SIZE: the random-access reading of profiles/r03_calib/calib.json",
                "kernels": ents})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
