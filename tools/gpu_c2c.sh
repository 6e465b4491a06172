# tools/gpu_c2c.sh — GPU box: the C2-direction proxy index built by desamba_index (as
# tools/gpu_c2b.sh, without the reference builder's file comparison), the C2 parity test and a C2
# bench line.  Outputs under gpurun_out/c2c/.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/c2c
mkdir -p $O
W=${TMPDIR:-/tmp}/dsb_c2c
rm -rf $W; mkdir -p $W
t0=$(date +%s)
python3 tools/simulate.py reference --preset c2 --out $W > $O/manifest.json || exit 1
desamba-so_amd/bin/desamba_index $W/kmer.srt $W/ref.fa $W/mine > $O/build_mine.log 2>&1 || { echo MINEFAIL; tail -5 $O/build_mine.log; exit 1; }
echo "simulate + desamba_index $(( $(date +%s) - t0 ))s"
rm -f $W/kmer.srt
cp $W/nodes.dmp $W/names.dmp $W/mine/
DSB_C2_DIR=$W/mine timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -k c2 -x -v -s --timeout 580 --timeout-method thread > $O/test.log 2>&1 || { echo C2TESTFAIL; tail -30 $O/test.log; exit 1; }
tail -3 $O/test.log
timeout -k 10 400 python -u bench.py --index $W/mine --name C2-proxy-495Mbp-lek17 --steps 3 --warmup 1 --no-dropin > $O/bench.json 2> $O/bench.err || { echo C2BENCHFAIL; tail -20 $O/bench.err; exit 1; }
tail -c 400 $O/bench.json
echo C2COK
