# tools/gpu_nd.sh — GPU box: repeat the committed read sets (SAM + DES) REPS times with the
# default library (non-determinism check), the parity file, then an A/B over VARS
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/nd
timeout -k 10 400 python -u tools/gpu_repeat_sets.py ${REPS:-12} > gpurun_out/nd/default.txt 2>&1 || { tail -20 gpurun_out/nd/default.txt; exit 1; }
echo "default $(grep TOTAL_BAD gpurun_out/nd/default.txt)"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q --timeout 200 --timeout-method thread > gpurun_out/nd/parity.log 2>&1
tail -3 gpurun_out/nd/parity.log | grep -E "passed|failed"
[ -n "${VARS:-}" ] && { bash tools/ab.sh $VARS > gpurun_out/ab.txt 2>&1; cat gpurun_out/ab.txt; }
echo NDDONE
