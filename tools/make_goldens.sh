#!/bin/bash
# tools/make_goldens.sh — (re)generate the committed parity fixtures under tests/golden/.
#
# Runs ONLY in the development container (needs /root/reference to build the oracle):
#   1. builds the reference classifier + hermetic harness (oracle/Makefile)
#   2. generates the synthetic fixture reference (tools/simulate.py, seeded)
#   3. builds its index with the REFERENCE builder (`deSAMBA index`)
#   4. simulates read sets and classifies them with the reference:
#        *.herm.sam  hermetic oracle (fresh pools, MALLOC_PERTURB 165, clang pattern init)
#        *.t1.sam    `deSAMBA classify -t 1`
#   5. packs inputs + outputs (xz) and writes tests/golden/manifest.json
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=${W:-$ROOT/build/golden_work}
G=$ROOT/tests/golden
REF=$ROOT/oracle/_ref
mkdir -p "$W" "$G"
make -s -C "$ROOT/oracle" ref harness herm
python3 "$ROOT/tools/simulate.py" reference --preset fixture --out "$W" > "$W/ref_manifest.json"
rm -rf "$W/idx"
"$REF/deSAMBA" index "$W/kmer.srt" "$W/ref.fa" "$W/idx" > "$W/index.log" 2>&1
cp "$W/nodes.dmp" "$W/names.dmp" "$W/idx/"
S="python3 $ROOT/tools/simulate.py reads --fasta $W/ref.fa"
$S --out "$W/mixed.fq" -n 600 --seed 11 --kind mixed --edge
$S --out "$W/ont.fq" -n 2000 --seed 21 --kind ont
$S --out "$W/ont_long.fq" -n 200 --seed 23 --kind ont --mean-len 16000
$S --out "$W/illumina.fq" -n 3000 --seed 22 --kind illumina
for s in mixed ont ont_long illumina; do
	"$REF/herm_classify" "$W/idx" "$W/$s.fq" > "$W/$s.herm.sam_full" 2>/dev/null
	"$REF/herm_classify" --sam "$W/idx" "$W/$s.fq" > "$W/$s.herm.sam" 2>/dev/null
	"$REF/deSAMBA" classify -t 1 -f SAM "$W/idx" "$W/$s.fq" > "$W/$s.t1.sam" 2>/dev/null || echo "reference -t1 failed on $s (exit $?)"
done
"$REF/deSAMBA" classify -t 1 -f SAM_FULL "$W/idx" "$W/mixed.fq" > "$W/mixed.t1.sam_full" 2>/dev/null
"$REF/deSAMBA" classify -t 1 -f DES "$W/idx" "$W/mixed.fq" > "$W/mixed.t1.des" 2>/dev/null
# hermetic DES / DES_FULL (the reference's own output_one_result_des / _full, cly_mt.c:144-227)
for s in mixed ont; do
	"$REF/herm_classify" --des "$W/idx" "$W/$s.fq" > "$W/$s.herm.des" 2>/dev/null
	"$REF/herm_classify" --des-full "$W/idx" "$W/$s.fq" > "$W/$s.herm.des_full" 2>/dev/null
done
# reference meta_analysis over the hermetic SAM_FULL of the mixed set (via its own .so)
gcc -O1 -o "$W/ref_meta" "$ROOT/tools/ref_meta.c" -ldl
"$W/ref_meta" "$REF/libdesamba.so" "$W/idx" "$W/mixed.herm.sam_full" 0 > "$W/mixed.meta_reads" 2>/dev/null
"$W/ref_meta" "$REF/libdesamba.so" "$W/idx" "$W/mixed.herm.sam_full" 1 > "$W/mixed.meta_bases" 2>/dev/null
tar -C "$W/idx" -cf - . | xz -T8 -6 > "$G/fixture_index.txz"
for f in mixed.fq ont.fq ont_long.fq illumina.fq mixed.herm.sam_full mixed.t1.sam_full mixed.t1.des \
	 mixed.herm.sam ont.herm.sam ont_long.herm.sam illumina.herm.sam \
	 mixed.t1.sam ont.t1.sam ont_long.t1.sam illumina.t1.sam mixed.meta_reads mixed.meta_bases \
	 mixed.herm.des mixed.herm.des_full ont.herm.des ont.herm.des_full; do
	xz -T4 -9 -c "$W/$f" > "$G/$f.xz"
done
cp "$W/ref_manifest.json" "$G/fixture_reference.json"
python3 - "$G" "$W" <<'EOF'
import hashlib, json, os, sys
g, w = sys.argv[1], sys.argv[2]
m = {"generator": "tools/make_goldens.sh", "files": {}}
for f in sorted(os.listdir(g)):
    if f.endswith(".xz") or f.endswith(".txz"):
        raw = os.path.join(w, f[:-3]) if f.endswith(".xz") else None
        e = {"sha256_packed": hashlib.sha256(open(os.path.join(g, f), "rb").read()).hexdigest()}
        if raw and os.path.exists(raw):
            e["sha256"] = hashlib.sha256(open(raw, "rb").read()).hexdigest()
        m["files"][f] = e
json.dump(m, open(os.path.join(g, "manifest.json"), "w"), indent=1)
EOF
du -sh "$G"
