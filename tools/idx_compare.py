"""Compare two deSAMBA index directories file by file (tests/test_index_build.py, dev use).

    python tools/idx_compare.py <reference_index_dir> <built_index_dir>

Byte equality for every file, except the bytes the reference builder leaves undefined:
  * deSAMBA.ref_i: REF_INFO.ref_name bytes after the terminating NUL (strcpy into realloc'd
    memory, reference src/idx.c:587-590) — compared up to and including the NUL;
  * deSAMBA.bwt: the unused tail of the last 128-byte BWT block when the BWT has at most 256
    blocks (a reused, never-written buffer, reference src/bwt.c:213-238).
Prints one line per file and "IDENTICAL" / "DIFFERENT" at the end; exit status 0 / 1.
"""
import os
import struct
import sys

FILES = [".bwt", ".sa", ".acg", ".exk0", ".exk1", ".exki", ".unv", ".ref_b", ".ref_i", ".ref_p"]


def read(d, suf):
    with open(os.path.join(d, "deSAMBA" + suf), "rb") as f:
        return f.read()


def mask_ref_i(b):
    n = struct.unpack_from("<Q", b, 0)[0]
    out = bytearray(b)
    for i in range(n):
        o = 8 + 144 * i
        z = out.index(0, o, o + 128) if 0 in out[o:o + 128] else o + 127
        out[z + 1:o + 128] = bytes(o + 128 - z - 1)
    return bytes(out)


def mask_bwt(b, sa_size):
    """Zero the never-written tail of the last BWT block (<= 256 blocks only).  The symbol count
    L is not stored; deSAMBA.sa holds ceil(L / 8) samples, so L >= 8 (sa_size - 1) + 1 and the
    bytes from there on are masked (at most 4 real bytes more than the undefined ones)."""
    byte_len = struct.unpack_from("<Q", b, 0)[0]
    nb = byte_len // 168
    if nb == 0 or nb > 256:
        return b
    l_min = 8 * (sa_size - 1) + 1
    copied = (l_min + 1) // 2 - (nb - 1) * 128
    last = 8 + (nb - 1) * 168
    out = bytearray(b)
    s = last + 40 + max(0, copied)
    out[s:last + 168] = bytes(last + 168 - s)
    return bytes(out)


def main():
    ref, mine = sys.argv[1], sys.argv[2]
    ok = True
    for suf in FILES:
        a, b = read(ref, suf), read(mine, suf)
        if suf == ".ref_i":
            a, b = mask_ref_i(a), mask_ref_i(b)
        if suf == ".bwt":
            n_sa = struct.unpack_from("<Q", read(ref, ".sa"), 0)[0]
            a, b = mask_bwt(a, n_sa), mask_bwt(b, n_sa)
        same = a == b
        if not same:
            first = next((i for i in range(min(len(a), len(b))) if a[i] != b[i]), min(len(a), len(b)))
            print(f"{suf:7s} DIFFERENT  sizes {len(a)} / {len(b)}  first difference at byte {first}")
            ok = False
        else:
            print(f"{suf:7s} identical  {len(a)} bytes")
    print("IDENTICAL" if ok else "DIFFERENT")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
