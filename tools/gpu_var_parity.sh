# tools/gpu_var_parity.sh VAR — GPU box: the parity files on lib/var_VAR.so, then an A/B against
# the default library
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/vp
DSB_LIB=desamba-so_amd/lib/var_$1.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c1.py -x -q --timeout 300 --timeout-method thread > gpurun_out/vp/pytest_$1.log 2>&1
rc=$?
tail -3 gpurun_out/vp/pytest_$1.log
[ $rc -ne 0 ] && { tail -40 gpurun_out/vp/pytest_$1.log; exit 1; }
bash tools/ab.sh $1 > gpurun_out/ab.txt 2>&1; cat gpurun_out/ab.txt
