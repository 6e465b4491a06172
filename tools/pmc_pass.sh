#!/bin/bash
# tools/pmc_pass.sh NAME COUNTERS... — one rocprofv3 PMC pass over a 1-step bench run (GPU box);
# results in gpurun_out/pmc_NAME (summarise with tools/pmc_report.py NAME)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
N=$1; shift
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc "$@" -d "$R/gpurun_out/pmc_$N" -o p -- python3 "$R/bench.py" --no-cpu --no-stats --no-dropin --steps 1 --warmup 0 ${BENCH_ARGS:-} > "$R/gpurun_out/pmc_$N.json" 2> "$R/gpurun_out/pmc_$N.err"
