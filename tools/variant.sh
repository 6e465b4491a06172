#!/bin/bash
# tools/variant.sh NAME "HIPCC FLAGS" [phases...] — build desamba-so_amd/lib/var_NAME.so: the given
# phase translation units recompiled with extra flags, linked with the current objects (dev tool
# for A/B runs; KERNELS=1 also recompiles kernels.hip on the GPU box: DSB_LIB=desamba-so_amd/lib/var_NAME.so python bench.py ...).
set -euo pipefail
D=$(cd "$(dirname "$0")/../desamba-so_amd" && pwd)
NAME=$1; FLAGS=$2; shift 2
PH=${*:-1 2 4 6}
B=$D/build; V=$B/var_$NAME; mkdir -p $V
HIPFLAGS="--offload-arch=gfx950 -O3 -g -std=c++17 -fPIC -Wno-sign-compare -Wno-unused-result -Wno-unused-value -fno-strict-aliasing -DDSB_HDN_INLINE=1"
OBJS=""
for p in 0 1 2 3 4 5 6 7 8; do
	if [[ " $PH " == *" $p "* ]]; then
		/opt/rocm/bin/hipcc $HIPFLAGS $FLAGS -DDSB_PH=$p -c $D/csrc/gpu/phase.hip -o $V/phase$p.o &
		OBJS="$OBJS $V/phase$p.o"
	else
		OBJS="$OBJS $B/phase$p.o"
	fi
done
KOBJ=$B/kernels.o
if [ -n "${KERNELS:-}" ]; then # also recompile kernels.hip (k_encode / k_seed / k_classB) with FLAGS
	/opt/rocm/bin/hipcc $HIPFLAGS $FLAGS -c $D/csrc/gpu/kernels.hip -o $V/kernels.o &
	KOBJ=$V/kernels.o
fi
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/lib/var_$NAME.so $B/index_load.o $B/fastq.o $B/sam_out.o $B/pool.o $B/pipeline.o \
	$B/meta.o $B/abi.o $KOBJ $OBJS -Wl,--version-script=$D/exports.map -lz -lm -lpthread
echo "built $D/lib/var_$NAME.so"
