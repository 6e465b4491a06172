# GPU suite + smoke + bench on the current tree (r3 pipeline defaults)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo TESTFAIL; tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 $O/smoke.log; exit 1; }
timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 > $O/bench.json 2> $O/bench.err || { echo BENCHFAIL; tail -30 $O/bench.err; exit 1; }
python3 -c "
import json
d = json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'dropin', d['dropin']['value'], d['dropin']['pipeline'])"
SWEEP_READS="12500 25000 50000" timeout -k 10 500 python -u tools/dropin_sweep.py 100000 2 1 > $O/dropin_sweep.txt 2> $O/dropin_sweep.err || { echo SWEEPFAIL; exit 1; }
cat $O/dropin_sweep.txt
echo RUN5OK
