#!/bin/bash
# tools/kres.sh — register / scratch usage of the phase kernels (from the built objects)
B=$(cd "$(dirname "$0")/.." && pwd)/desamba-so_amd/build
T=$(mktemp -d)
for o in "$B"/phase*.o "$B"/kernels.o; do
	/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section=.hip_fatbin=$T/f.bin "$o" 2>/dev/null || continue
	/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$T/f.bin \
		--targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/k.co 2>/dev/null || continue
	/opt/rocm/lib/llvm/bin/llvm-readelf --notes $T/k.co | python3 -c '
import re,sys
t=sys.stdin.read()
for blk in t.split("  - .agpr_count")[1:]:
    g=lambda k:(re.search(r"\.%s:\s+(\S+)"%k,blk) or [0,"?"])[1]
    n=g("name")
    if "Lb1E" in n: continue
    print("%-28s vgpr %4s sgpr %4s vspill %4s scratch %5s lds %6s" % (re.sub(r"^_Z\d+","",n)[:28], g("vgpr_count"), g("sgpr_count"), g("vgpr_spill_count"), g("private_segment_fixed_size"), g("group_segment_fixed_size")))
'
done
rm -rf $T
