# tools/gpu_qr.sh — GPU box (dev): window read-range statistics of the scoring phase (lib/var_qr.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/qr
mkdir -p $O
DSB_LIB=desamba-so_amd/lib/var_qr.so timeout -k 10 400 python -u bench.py --steps 1 --warmup 0 --no-cpu --no-dropin > $O/bench_qr.json 2> $O/bench_qr.err || exit 1
echo QROK
