#!/bin/bash
# tools/kres.sh — per-kernel VGPR / scratch / occupancy of kernels.hip for gfx950
cd "$(dirname "$0")/../desamba-so_amd"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-sign-compare -Wno-unused-result -Wno-unused-value -fno-strict-aliasing -DDSB_HDN_INLINE=1 $KRES_FLAGS \
  -c csrc/gpu/kernels.hip -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import re, sys
cur = None
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m: cur = m.group(1); print(); print(cur[:60], end="")
    for k in ("VGPRs", "AGPRs", "ScratchSize \[bytes/lane\]", "Occupancy \[waves/SIMD\]", "LDS Size \[bytes/block\]"):
        m = re.search(k + r": (\d+)", line)
        if m: print(f"  {k.split()[0]}={m.group(1)}", end="")
print()'
