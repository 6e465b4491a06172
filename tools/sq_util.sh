#!/bin/bash
# tools/sq_util.sh — per-kernel VALU lane utilisation / issue / wait fractions (one rocprofv3 PMC pass; GPU box)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -s KILL 240 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD -d gpurun_out/prof_sq -o sq -- python3 bench.py --no-cpu --no-stats --steps 1 --warmup 0 > gpurun_out/sq.json 2> gpurun_out/sq.err
