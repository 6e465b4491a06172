# tools/gpu_nd2.sh — GPU box: the parity file twice with the default library and twice with var_bf0
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/nd2
for k in 1 2; do
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q --timeout 200 --timeout-method thread > gpurun_out/nd2/def_$k.log 2>&1
tail -3 gpurun_out/nd2/def_$k.log | grep -E "passed|failed"
DSB_LIB=desamba-so_amd/lib/var_bf0.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q --timeout 200 --timeout-method thread > gpurun_out/nd2/bf0_$k.log 2>&1
tail -3 gpurun_out/nd2/bf0_$k.log | grep -E "passed|failed"
done
grep -h FAILED gpurun_out/nd2/*.log
echo ND2DONE
