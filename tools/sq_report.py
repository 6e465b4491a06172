"""Summarise tools/sq_util.sh output (dev tool)."""
import glob, re, sqlite3
db = sqlite3.connect(glob.glob('gpurun_out/prof_sq/*.db')[0])
res = {}
for n, c, v in db.execute("select kernel_name, counter_name, value from counters_collection"):
    m = re.match(r"(?:void )?([\w:]+(?:<[^>]*>)?)", n)
    n = m.group(1) if m else n
    res.setdefault(n, {}).setdefault(c, 0)
    res[n][c] += v
for n, d in res.items():
    if 'k_' not in n:
        continue
    util = d['SQ_THREAD_CYCLES_VALU'] / max(1, d['SQ_ACTIVE_INST_VALU'] * 64)
    print(f"{n[:24]:24s} valu_util={util:.3f} insts_valu={d['SQ_INSTS_VALU']:.3g} vmem_rd={d['SQ_INSTS_VMEM_RD']:.3g} "
          f"issue={d['SQ_ACTIVE_INST_ANY'] / max(1, d['SQ_WAVE_CYCLES']):.3f} wait={d['SQ_WAIT_INST_ANY'] / max(1, d['SQ_WAVE_CYCLES']):.3f}")
