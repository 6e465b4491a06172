#!/bin/bash
# tools/sweep.sh — bench each library variant given on the command line (GPU box)
for v in "$@"; do
  echo "== $v" >> gpurun_out/sweep.log
  DSB_LIB=$PWD/desamba-so_amd/lib/$v timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu --no-stats 2>>gpurun_out/sweep.err | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["phase_ms_classA"])' >> gpurun_out/sweep.log || exit 1
done
