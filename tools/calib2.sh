# tools/calib2.sh — GPU box: the read-hash build pattern (tools/gather_calib k_build: per-wave own
# table, load + store per update) at 4 / 32 / 128 KB per wave: rate and WRITE_SIZE / FETCH_SIZE per
# update, beside the random gather / scatter of a 2 GB table.  gpurun_out/calib2/
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/calib2
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for kb in 4 32 128; do
  timeout -k 10 120 $GRAFT_REPO_ROOT/tools/gather_calib 2048 256 $kb > $O/run_$kb.txt 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/f_$kb -o f -- $GRAFT_REPO_ROOT/tools/gather_calib 2048 256 $kb > /dev/null 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/w_$kb -o w -- $GRAFT_REPO_ROOT/tools/gather_calib 2048 256 $kb > /dev/null 2>&1 || exit 1
done
cat $O/run_*.txt
echo CALIBOK
