# tools/gpu_isl.sh — GPU box: parity of the k_island_g default, then A/B against the k_seed +
# two-lane island path (var_g0) and other batch sizes, and one stats run for the probe counts.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/isl
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c1.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/ab.sh ${VARS:-g0 g4 g16} > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu --no-dropin > $O/stats.json 2> $O/stats.err || { tail $O/stats.err; exit 1; }
echo ISLOK
