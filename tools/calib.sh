# tools/calib.sh — GPU box: FETCH_SIZE / WRITE_SIZE per random 4-B gather / scattered store / streamed byte
# (tools/gather_calib), for tables below, near and beyond the 256 MB Infinity Cache.  gpurun_out/calib/
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/calib
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for mb in 64 1024 8192; do
  timeout -k 10 120 $GRAFT_REPO_ROOT/tools/gather_calib $mb 256 > $O/run_$mb.txt 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/kt_$mb -o kt -- $GRAFT_REPO_ROOT/tools/gather_calib $mb 256 > /dev/null 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/f_$mb -o f -- $GRAFT_REPO_ROOT/tools/gather_calib $mb 256 > /dev/null 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/w_$mb -o w -- $GRAFT_REPO_ROOT/tools/gather_calib $mb 256 > /dev/null 2>&1 || exit 1
done
cat $O/run_*.txt
echo CALIBOK
