#!/bin/bash
# tools/ab_env.sh NAME "ENV=V ..." — bench the default library with extra environment (dev tool)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
env $2 timeout -k 10 240 python bench.py --no-cpu --no-stats --steps 3 > gpurun_out/ab_$1.json 2> gpurun_out/ab_$1.err || exit 1
python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_$1.json')); print('$1', d['value'], {k: round(x,1) for k,x in d['phase_ms_classA'].items()})"
