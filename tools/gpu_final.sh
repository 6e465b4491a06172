# tools/gpu_final.sh OUTNAME — GPU box: the GPU suite, smoke(), the default bench line and the
# rocprofv3 kernel-stats + FETCH/WRITE passes of the same tree, into gpurun_out/OUTNAME.
set -o pipefail
cd $GRAFT_REPO_ROOT
N=${1:-final}
O=$GRAFT_REPO_ROOT/gpurun_out/$N
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo TESTFAIL; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 $O/smoke.log; exit 1; }
timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { echo BENCHFAIL; tail -30 $O/bench.err; exit 1; }
python3 -c "
import json
d = json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'], 'dropin', d.get('dropin', {}).get('value'))"
[ -n "${NOPROF:-}" ] && { echo FINALOK; exit 0; }
bash tools/profile.sh || { echo PROFFAIL; exit 1; }
echo FINALOK
