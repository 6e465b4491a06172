# C1 GPU work of one box call: the GPU suite, smoke(), the default bench (stats + CPU baselines +
# drop-in leg).  Logs under gpurun_out/r3/.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo TESTFAIL; tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 $O/smoke.log; exit 1; }
timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 > $O/bench.json 2> $O/bench.err || { echo BENCHFAIL; tail -30 $O/bench.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r3/bench.json").read().strip().splitlines()[-1])
print("value", d["value"], "dropin", (d.get("dropin") or {}).get("value"), "cpu", (d.get("cpu_baseline") or {}).get("value"),
      "taxid_mismatch", d.get("taxid_mismatch"))
PY
