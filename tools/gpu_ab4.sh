# drop-in sweep + MEM_search width A/B (dev)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/p4
timeout -k 10 500 python -u tools/dropin_sweep.py > gpurun_out/p4/dropin_sweep.txt 2> gpurun_out/p4/dropin_sweep.err || { echo SWEEPFAIL; tail -20 gpurun_out/p4/dropin_sweep.err; exit 1; }
cat gpurun_out/p4/dropin_sweep.txt
timeout -k 10 700 bash tools/ab.sh mw2 mw4 || { echo ABFAIL; exit 1; }
timeout -k 10 300 bash tools/ab.sh base || true
echo AB4OK
