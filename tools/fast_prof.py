"""Seeding-phase clock split from a bench.py JSON line with work counters (dev tool)."""
import json, sys
d = json.load(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/bench.json"))
print(d["value"], d["phase_ms_classA"])
for ph in ("fast0", "slow0"):
    c = d["work_counters"]["phases"][ph]
    tot = c["t_mem"] or 1
    print(ph, "map batch %.3f  (map prefix/suffix %.3f, REF_POS items %.3f)" % (c["t_map"] / tot, c["t_build"] / tot,
                                                                        c["t_match"] / tot))
c = d["work_counters"]["phases"]["fast0"]
print("fast0 trips/read %.1f  map trips/read %.1f  lanes per map trip %.1f  REF_POS per read %.1f" % (
    c["t_dpm"] / 1e5, c["t_dps"] / 1e5, c["t_fill"] / max(1, c["t_dps"]), c["ref_pos"] / 1e5))
c = d["work_counters"]["phases"]["delA"]
tot = c["t_all"] or 1
print("delA", {k: round(c[k] / tot, 3) for k in ("t_build", "t_match", "t_win", "t_dpm", "t_dps", "t_fill")})
