#!/bin/bash
# tools/ab.sh VAR... — bench the default library and each lib/var_VAR.so on the GPU box (dev tool)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in base "$@"; do
	if [ "$v" = base ]; then unset DSB_LIB; else export DSB_LIB="desamba-so_amd/lib/var_$v.so"; fi
	timeout -k 10 240 python bench.py --no-cpu --no-stats --steps 3 > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || exit 1
	python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_$v.json')); print('$v', d['value'], {k: round(x,1) for k,x in d['phase_ms_classA'].items()}, 'dropin', (d.get('dropin') or {}).get('value'))"
done
