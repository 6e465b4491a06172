# tools/gpu_lazy.sh — GPU box: A/B of the on-demand Bloom probing island scan (DSB_LAZY_EXIST) at
# batch sizes 4/8/16, the needed-bit counters, and the parity suite on the K=8 variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/lazy
mkdir -p $O
bash tools/ab.sh lazy4 lazy8 lazy16 > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
DSB_LIB=desamba-so_amd/lib/var_need.so timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu --no-dropin > $O/need.json 2> $O/need.err || { tail $O/need.err; exit 1; }
DSB_LIB=desamba-so_amd/lib/var_lazy8.so timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu --no-dropin > $O/lazy8_stats.json 2> $O/lazy8_stats.err || { tail $O/lazy8_stats.err; exit 1; }
DSB_LIB=desamba-so_amd/lib/var_lazy8.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c1.py -x -q --timeout 300 --timeout-method thread > $O/pytest_lazy8.log 2>&1 || { tail -30 $O/pytest_lazy8.log; exit 1; }
tail -2 $O/pytest_lazy8.log
echo LAZYOK
