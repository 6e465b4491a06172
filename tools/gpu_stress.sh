# tools/gpu_stress.sh — GPU box: the GPU suite twice more and the committed read sets repeated
# (SAM + DES, tools/gpu_repeat_sets.py) — the determinism evidence of the final tree
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/stress
mkdir -p $O
for k in 1 2; do
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu_$k.log 2>&1
  echo "suite run $k rc=$?: $(tail -1 $O/pytest_gpu_$k.log)"
done
timeout -k 10 600 python -u tools/gpu_repeat_sets.py 10 > $O/repeat_sets.txt 2>&1 || { tail -5 $O/repeat_sets.txt; exit 1; }
grep TOTAL_BAD $O/repeat_sets.txt
