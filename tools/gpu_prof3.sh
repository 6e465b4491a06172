# profiles of the current tree (C1 bench workload): drop-in sweep, bench (stats + CPU + drop-in),
# rocprofv3 kernel trace + FETCH / WRITE passes.  Outputs under gpurun_out/.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/p3
timeout -k 10 500 python -u tools/dropin_sweep.py > gpurun_out/p3/dropin_sweep.txt 2> gpurun_out/p3/dropin_sweep.err || { echo SWEEPFAIL; tail -20 gpurun_out/p3/dropin_sweep.err; exit 1; }
cat gpurun_out/p3/dropin_sweep.txt
if [ -z "${SWEEP_ONLY:-}" ]; then
timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 > gpurun_out/p3/bench.json 2> gpurun_out/p3/bench.err || { echo BENCHFAIL; tail -30 gpurun_out/p3/bench.err; exit 1; }
STEPS=2 bash tools/profile.sh || { echo PROFFAIL; exit 1; }
fi
echo PROFOK
