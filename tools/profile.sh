#!/bin/bash
# tools/profile.sh — rocprofv3 evidence for the bench workload (GPU box):
#   pass 1: kernel trace + stats (per-kernel average durations)
#   pass 2: FETCH_SIZE, pass 3: WRITE_SIZE (separate passes: TCC slots; no tracing domains)
# Results land in gpurun_out/prof_*; tools/prof_summary.py condenses them into profiles/.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out
export TMPDIR=/tmp
cd /tmp
B="$R/bench.py --steps ${STEPS:-2} --warmup 1 --no-cpu --no-stats --no-dropin"
[ -z "${ONLY_EXTRA:-}" ] && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/prof_kt" -o kt -- python3 $B > "$OUT/prof_kt.json" 2> "$OUT/prof_kt.err"
[ -z "${ONLY_EXTRA:-}" ] && timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE -d "$OUT/prof_fetch" -o pf -- python3 $B > "$OUT/prof_fetch.json" 2> "$OUT/prof_fetch.err"
[ -z "${ONLY_EXTRA:-}" ] && timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE -d "$OUT/prof_write" -o pw -- python3 $B > "$OUT/prof_write.json" 2> "$OUT/prof_write.err"
if [ -n "${SQ:-}" ]; then
  timeout -k 10 500 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM -d "$OUT/prof_sq" -o psq -- python3 $B > "$OUT/prof_sq.json" 2> "$OUT/prof_sq.err"
fi
if [ -n "${INSTS:-}" ]; then
  timeout -k 10 500 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_FLAT SQ_INSTS_BRANCH -d "$OUT/prof_insts" -o pin -- python3 $B > "$OUT/prof_insts.json" 2> "$OUT/prof_insts.err"
fi
