"""Print the scoring / seeding phase clock breakdown from a bench.py JSON line (dev tool)."""
import json, sys
d = json.load(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/bench.json"))
print(d["value"], d["phase_ms_classA"])
c = d["work_counters"]["phases"]["delA"]
tot = c["t_all"] or 1
print("delA", {k: round(c[k] / tot, 3) for k in ("t_build", "t_match", "t_mprobe", "t_mwalk", "t_win", "t_dpm", "t_dps", "t_fill", "t_comb")})
c = d["work_counters"]["phases"]["fast0"]
print("fast0 t_mem/t_map", c["t_mem"], c["t_map"])
