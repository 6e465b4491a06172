#!/bin/bash
# tools/make_c1_index.sh — build the C1 proxy index used by bench.py (data/c1_index.txz).
#
# The demo human index of BASELINE config C1 is not available offline, so C1 uses a
# >= 50 Mbp synthetic family-structured reference (tools/simulate.py preset "c1": 127
# genomes, 55.83 Mbp, 28.2 M distinct 31-mers) indexed by the REFERENCE's own builder
# (`deSAMBA index`, oracle/_ref, built from the reference sources by oracle/Makefile).
# Runs in the development container only (needs /root/reference).  data/ is git-ignored
# but travels to the GPU box with the repository snapshot.
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=${W:-$ROOT/build/c1}
mkdir -p "$W" "$ROOT/data"
make -s -C "$ROOT/oracle" ref
python3 "$ROOT/tools/simulate.py" reference --preset c1 --out "$W" > "$W/manifest.json"
rm -rf "$W/idx"
( time "$ROOT/oracle/_ref/deSAMBA" index "$W/kmer.srt" "$W/ref.fa" "$W/idx" ) > "$W/build.log" 2>&1
cp "$W/nodes.dmp" "$W/names.dmp" "$W/idx/"
tar -C "$W/idx" -cf - . | xz -T8 -3 > "$ROOT/data/c1_index.txz"
ls -la "$ROOT/data/c1_index.txz"
