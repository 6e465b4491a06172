#!/bin/bash
# tools/gpu_session.sh TAG STEP... — one GPU call made of named steps, each under its own time
# limit, outputs under gpurun_out/TAG/; the call stops at the first failing step.
#
#   bench[:ARGS]      python bench.py ARGS (default: the driver's defaults, 5 steps)   -> bench.json
#   ab:VARS:ARGS      bench.py --no-cpu --no-stats --no-dropin ARGS for the default library and
#                     each variant (VARS comma-separated): desamba-so_amd/lib/var_VAR.so, or
#                     env.KEY.VALUE[+KEY.VALUE] = the default library with KEY=VALUE (DROPIN= keeps the
#                     drop-in leg)                                                     -> ab_*.json
#   parity:VAR        tests/test_gpu_parity.py + test_gpu_c1.py with lib/var_VAR.so     -> parity_VAR.log
#   scale[:K]         tests/test_gpu_scale.py -k K (C2 proxy, e-kmer table sizes)       -> scale.log
#   suite             the whole -m gpu suite                                            -> suite.log
#   prof[:ARGS]       rocprofv3 --kernel-trace --stats over bench.py ARGS               -> prof/
#   pmc:COUNTERS:ARGS one rocprofv3 --pmc pass over bench.py ARGS                        -> pmc_N/
#                     (tools/traffic_json.py turns a FETCH_SIZE and a WRITE_SIZE pass into
#                     profiles/traffic.json; tools/prof_report.py pmc DIR prints any pass)
#   sq[:ARGS]         SQ counters of a 1-step bench.py ARGS (VALU lane utilisation, issue, wait;
#                     tools/prof_report.py sq)                                          -> sq/
#   calib[:MB,...]    the random-access calibration (tools/gather_calib.hip: dependent 4-B gathers,
#                     scattered stores, streams, the read-hash build pattern) with kernel-trace,
#                     FETCH_SIZE and WRITE_SIZE passes per table size; tools/calib_report.py
#                                                                                       -> calib/
#   selftest          the device msort restatement against the host (tools/gpu_selftest.py)
#   stress[:N]        the committed read sets N times over two contexts, SAM + DES
#                     (tools/gpu_repeat_sets.py): determinism evidence                   -> stress.txt
#
# Usage: gpurun -- 'bash tools/gpu_session.sh r4a bench ab:qcopy,memo:--reads=300000 scale'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=${TMPDIR:-/tmp}
{ date; df -h /tmp "$TMPDIR" /dev/shm; free -g; cat /sys/fs/cgroup/memory.max /sys/fs/cgroup/cpu.max; nproc; } > "$O/env.txt" 2>&1
PY="python -u"
npmc=0
for step in "$@"; do
	name=${step%%:*}
	rest=${step#*:}; [ "$rest" = "$step" ] && rest=""
	echo "[gpu_session] $(date +%T) $step" | tee -a "$O/steps.txt"
	case $name in
	bench)
		rest=${rest//=/ }
		timeout -k 10 ${BENCH_TIMEOUT:-560} $PY bench.py ${rest:---steps 5 --warmup 1} > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
		tail -c 600 "$O/bench.json" ;;
	ab|abd) # abd: with the drop-in leg
		[ "$name" = abd ] && DROPIN="" || unset DROPIN
		vars=${rest%%:*}; args=${rest#*:}; [ "$args" = "$rest" ] && args=""
		args=${args//=/ }
		for v in base ${vars//,/ }; do
			# a variant is lib/var_V.so, or env.KEY.VALUE (the default library with KEY=VALUE)
			envs=()
			if [ "$v" = base ]; then unset DSB_LIB
			elif [[ $v == env.* ]]; then unset DSB_LIB; envs=(); IFS=+ read -ra kvs <<< "${v#env.}"
				for kv in "${kvs[@]}"; do envs+=("${kv%%.*}=${kv#*.}"); done
			else export DSB_LIB=desamba-so_amd/lib/var_$v.so; fi
			vn=${v//\//_} # a file name
			env "${envs[@]}" timeout -k 10 300 $PY bench.py --no-cpu --no-stats ${DROPIN---no-dropin} $args > "$O/${name}_$vn.json" 2> "$O/${name}_$vn.err" || { tail -20 "$O/${name}_$vn.err"; exit 1; }
			python3 -c "import json; d=json.load(open('$O/${name}_$vn.json')); print('$vn', d['value'], d['ms_per_step'], 'chunks', d['chunks'], 'retry', d['retried_reads'], {k: round(x, 1) for k, x in d['phase_ms_classA'].items()}, 'dropin', (d.get('dropin') or {}).get('value'), (d.get('dropin') or {}).get('identical_to_batch_records'))" | tee -a "$O/$name.txt"
		done
		unset DSB_LIB ;;
	parity)
		DSB_LIB=desamba-so_amd/lib/var_$rest.so timeout -k 10 400 $PY -m pytest tests/test_gpu_parity.py tests/test_gpu_c1.py -x -q --timeout 300 --timeout-method thread > "$O/parity_$rest.log" 2>&1 || { tail -30 "$O/parity_$rest.log"; exit 1; }
		tail -2 "$O/parity_$rest.log" ;;
	scale)
		timeout -k 10 900 $PY -m pytest tests/test_gpu_scale.py -x -v -s ${rest:+-k "$rest"} --timeout 600 --timeout-method thread > "$O/scale.log" 2>&1 || { tail -40 "$O/scale.log"; exit 1; }
		grep -E "PASSED|FAILED|SKIPPED|T3 mismatches" "$O/scale.log" | tail -20 ;;
	tests) # tests:FILE,FILE  (paths under tests/)
		timeout -k 10 1000 $PY -u -m pytest ${rest//,/ } -x -v -s --timeout 600 --timeout-method thread > "$O/tests.log" 2>&1 || { tail -40 "$O/tests.log"; exit 1; }
		grep -E "PASSED|FAILED|SKIPPED|ERROR" "$O/tests.log" | tail -30 ;;
	suite)
		timeout -k 10 1100 $PY -u -m pytest tests -m gpu -x -v -s --timeout 600 --timeout-method thread > "$O/suite.log" 2>&1 || { tail -40 "$O/suite.log"; exit 1; }
		tail -3 "$O/suite.log" ;;
	prof)
		rest=${rest//=/ }
		rm -rf "$O/prof"
		timeout -k 10 ${PROF_TIMEOUT:-500} rocprofv3 --kernel-trace --stats -d "$O/prof" -o run -- python3 bench.py ${rest:---steps 3 --warmup 1 --no-cpu --no-dropin} > "$O/prof_bench.json" 2> "$O/prof.err" || { tail -20 "$O/prof.err"; exit 1; }
		find "$O/prof" -name "*kernel_stats.csv" | head -1 | xargs -r head -12 ;;
	pmc)
		ctr=${rest%%:*}; args=${rest#*:}; [ "$args" = "$rest" ] && args=""
		args=${args//=/ }
		npmc=$((npmc + 1))
		rm -rf "$O/pmc_$npmc"
		timeout -s KILL 400 rocprofv3 --pmc ${ctr//,/ } -d "$O/pmc_$npmc" -o run -- python3 bench.py ${args:---steps 1 --warmup 0 --no-cpu --no-dropin --no-stats} > "$O/pmc_$npmc.json" 2> "$O/pmc_$npmc.err" || { tail -20 "$O/pmc_$npmc.err"; exit 1; }
		echo "$ctr" > "$O/pmc_$npmc/counters.txt" ;;
	sq)
		rest=${rest//=/ }
		rm -rf "$O/sq"
		timeout -s KILL 300 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD -d "$O/sq" -o sq -- python3 bench.py ${rest:---steps 1 --warmup 0 --no-cpu --no-dropin --no-stats} > "$O/sq.json" 2> "$O/sq.err" || { tail -20 "$O/sq.err"; exit 1; }
		python3 tools/prof_report.py sq "$O/sq" | tee "$O/sq_util.txt" ;;
	calib)
		[ -x tools/gather_calib ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o tools/gather_calib tools/gather_calib.hip || exit 1
		for mb in ${rest//,/ }; do
			[ -z "$rest" ] && break
			timeout -k 10 120 tools/gather_calib $mb 256 > "$O/calib_run_$mb.txt" 2>&1 || exit 1
			timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$O/calib_kt_$mb" -o kt -- tools/gather_calib $mb 256 > /dev/null 2>&1 || exit 1
			timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$O/calib_f_$mb" -o f -- tools/gather_calib $mb 256 > /dev/null 2>&1 || exit 1
			timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$O/calib_w_$mb" -o w -- tools/gather_calib $mb 256 > /dev/null 2>&1 || exit 1
		done
		cat "$O"/calib_run_*.txt ;;
	selftest)
		timeout -k 10 300 $PY tools/gpu_selftest.py > "$O/selftest.txt" 2>&1 || { tail -20 "$O/selftest.txt"; exit 1; }
		tail -3 "$O/selftest.txt" ;;
	stress)
		timeout -k 10 900 $PY tools/gpu_repeat_sets.py ${rest:-10} > "$O/stress.txt" 2>&1 || { tail -5 "$O/stress.txt"; exit 1; }
		grep TOTAL_BAD "$O/stress.txt" ;;
	*)
		echo "unknown step $step"; exit 2 ;;
	esac
done
for d in "$TMPDIR"/dsb_*_proxy_*/; do # the proxy indexes built in this call: how long, how much memory
	[ -f "$d/build.json" ] && { b=$(basename "$d"); cp "$d/build.json" "$O/$b.build.json"; cp "$d/build.log" "$O/$b.build.log" 2>/dev/null; }
done
echo "[gpu_session] $(date +%T) done" | tee -a "$O/steps.txt"
