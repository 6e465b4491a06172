# tools/gpu_c2.sh — GPU box: build the genuine C2-direction proxy index with the reference builder
# (CPU, ~10 min; it does not fit the 512 MiB upload) while the GPU runs the C1 work given in
# $C1_WORK, then the C2 parity test and a C2 bench line.  Outputs under gpurun_out/c2/.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/c2
mkdir -p $O
W=${TMPDIR:-/tmp}/dsb_c2w
rm -rf $W; mkdir -p $W
(
  set -e
  t0=$(date +%s)
  python3 tools/simulate.py reference --preset c2 --out $W > $O/manifest.json
  echo "simulate $(( $(date +%s) - t0 ))s" > $O/build_times.txt
  ( time oracle/_ref/deSAMBA index $W/kmer.srt $W/ref.fa $W/idx ) > $O/build.log 2>&1
  cp $W/nodes.dmp $W/names.dmp $W/idx/
  rm -f $W/kmer.srt
  echo "total $(( $(date +%s) - t0 ))s" >> $O/build_times.txt
  touch $W/DONE
) &
BPID=$!
if [ -n "${C1_WORK:-}" ]; then
  bash -c "$C1_WORK" || { echo C1WORKFAIL; kill $BPID; exit 1; }
fi
while [ ! -e $W/DONE ]; do
  if ! kill -0 $BPID 2>/dev/null; then echo C2BUILDFAIL; tail -c 2000 $O/build.log; exit 1; fi
  sleep 10; echo "waiting for the C2 build $(date +%T)" >> $O/wait.log
done
ls -la $W/idx > $O/index_files.txt
DSB_C2_DIR=$W/idx timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -k c2 -x -v -s --timeout 580 --timeout-method thread > $O/test.log 2>&1 || { echo C2TESTFAIL; tail -30 $O/test.log; exit 1; }
tail -3 $O/test.log
timeout -k 10 600 python -u bench.py --index $W/idx --name C2-proxy-495Mbp-lek17 --steps 3 --warmup 1 --no-dropin > $O/bench.json 2> $O/bench.err || { echo C2BENCHFAIL; tail -20 $O/bench.err; exit 1; }
tail -c 600 $O/bench.json
echo C2OK
