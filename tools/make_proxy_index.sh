#!/bin/bash
# tools/make_proxy_index.sh PRESET — build a synthetic proxy index (data/<preset>_index.txz).
#
# PRESET is a tools/simulate.py reference preset: c1 (55.8 Mbp, 28.2 M 31-mers, l_ek 16) or
# c2 (the C2-direction proxy: >= 238.6 M 31-mers, so l_ek 17 / MASK_31 / quarter-GB e-kmer
# tables, reference idx.c:966-996).  The index is made by the REFERENCE's own builder
# (`deSAMBA index`, oracle/_ref, compiled from the reference sources by oracle/Makefile), so it
# runs in the development container only.  data/ is git-ignored but travels to the GPU box.
set -euo pipefail
P=${1:?preset}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=${W:-$ROOT/build/$P}
mkdir -p "$W" "$ROOT/data"
make -s -C "$ROOT/oracle" ref
python3 "$ROOT/tools/simulate.py" reference --preset "$P" --out "$W" > "$W/manifest.json"
rm -rf "$W/idx"
( time "$ROOT/oracle/_ref/deSAMBA" index "$W/kmer.srt" "$W/ref.fa" "$W/idx" ) > "$W/build.log" 2>&1
cp "$W/nodes.dmp" "$W/names.dmp" "$W/idx/"
tar -C "$W/idx" -cf - . | xz -T8 -${XZ_LEVEL:-3} > "$ROOT/data/${P}_index.txz"
ls -la "$ROOT/data/${P}_index.txz"
