# tools/gpu_c2b.sh — GPU box: the C2-direction proxy index built by this repo's builder
# (desamba-so_amd/bin/desamba_index) and by the reference builder (oracle/_ref/deSAMBA index) from
# the same inputs, compared file by file (tools/idx_compare.py); then the C2 parity test and a C2
# bench line on the index this repo built.  Outputs under gpurun_out/c2b/.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/c2b
mkdir -p $O
W=${TMPDIR:-/tmp}/dsb_c2b
rm -rf $W; mkdir -p $W
t0=$(date +%s)
python3 tools/simulate.py reference --preset c2 --out $W > $O/manifest.json || exit 1
echo "simulate $(( $(date +%s) - t0 ))s" > $O/build_times.txt
t1=$(date +%s)
desamba-so_amd/bin/desamba_index $W/kmer.srt $W/ref.fa $W/mine > $O/build_mine.log 2>&1 || { echo MINEFAIL; tail -5 $O/build_mine.log; exit 1; }
echo "desamba_index $(( $(date +%s) - t1 ))s" >> $O/build_times.txt
t2=$(date +%s)
oracle/_ref/deSAMBA index $W/kmer.srt $W/ref.fa $W/ref > $O/build_ref.log 2>&1 || { echo REFFAIL; tail -5 $O/build_ref.log; exit 1; }
echo "reference deSAMBA index $(( $(date +%s) - t2 ))s" >> $O/build_times.txt
rm -f $W/kmer.srt
python3 tools/idx_compare.py $W/ref $W/mine > $O/compare.txt 2>&1; echo "compare rc $?" >> $O/compare.txt
cat $O/build_times.txt $O/compare.txt
rm -rf $W/ref
cp $W/nodes.dmp $W/names.dmp $W/mine/
DSB_C2_DIR=$W/mine timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -k c2 -x -v -s --timeout 580 --timeout-method thread > $O/test.log 2>&1 || { echo C2TESTFAIL; tail -30 $O/test.log; exit 1; }
tail -3 $O/test.log
timeout -k 10 400 python -u bench.py --index $W/mine --name C2-proxy-495Mbp-lek17 --steps 3 --warmup 1 --no-dropin > $O/bench.json 2> $O/bench.err || { echo C2BENCHFAIL; tail -20 $O/bench.err; exit 1; }
tail -c 400 $O/bench.json
echo C2BOK
