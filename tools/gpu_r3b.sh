# tools/gpu_r3b.sh — GPU box: read-hash build calibration, then bench.py --gpus 2 rehearsed on one
# GPU (two ranks, gloo) for the per-rank drop-in leg.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r3b
mkdir -p $O
bash tools/calib2.sh > $O/calib2.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
DSB_DIST_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 --steps 1 --warmup 1 > $O/bench2.log 2>&1 || exit 1
tail -c 3000 $O/bench2.log
cd $GRAFT_REPO_ROOT
DSB_LIB=desamba-so_amd/lib/var_qr.so timeout -k 10 400 python -u bench.py --steps 1 --warmup 0 --no-cpu --no-dropin > $O/bench_qr.json 2> $O/bench_qr.err || exit 1
echo R3BOK
