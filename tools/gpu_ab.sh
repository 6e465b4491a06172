# tools/gpu_ab.sh VAR... — GPU box: tools/ab.sh over the given variants into gpurun_out/ab.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab.sh "$@" > gpurun_out/ab.txt 2>&1 || { cat gpurun_out/ab.txt; exit 1; }
cat gpurun_out/ab.txt
