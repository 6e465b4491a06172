set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "des or nul or concurrent or carry" > gpurun_out/t1.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/t1.log; exit 1; }
tail -15 gpurun_out/t1.log
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 > gpurun_out/b1.json 2> gpurun_out/b1.err || { echo BENCHFAIL; tail -30 gpurun_out/b1.err; exit 1; }
DSB_DIST_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 --steps 2 --warmup 1 --no-stats --reads 20000 > gpurun_out/b2.json 2> gpurun_out/b2.err || { echo BENCH2FAIL; tail -30 gpurun_out/b2.err; exit 1; }
echo ALLOK
