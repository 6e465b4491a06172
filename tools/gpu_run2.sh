# GPU suite + smoke + bench with the drop-in leg (round 3 pipeline)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/t2.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/t2.log; exit 1; }
tail -5 gpurun_out/t2.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --no-stats > gpurun_out/b3.json 2> gpurun_out/b3.err || { echo BENCHFAIL; tail -30 gpurun_out/b3.err; exit 1; }
tail -c 1500 gpurun_out/b3.json
echo ALLOK
