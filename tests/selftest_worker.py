"""Runs the device self-tests of the TEST build (lib/libdesamba_test.so, include/desamba_mi355x_test.h)
in a process of their own: the production library does not export them.

    python tests/selftest_worker.py sort CASES_JSON          -> one JSON list of results on stdout
    python tests/selftest_worker.py occ DIR DOLLOR ROWS OUT  -> OUT: 7 x u64 per row; rc on stdout
"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TEST_LIB = os.path.join(ROOT, "desamba-so_amd", "lib", "libdesamba_test.so")


def main():
    L = C.CDLL(os.environ.get("DSB_TEST_LIB", TEST_LIB))
    if sys.argv[1] == "sort":
        f = L.dsb_gpu_selftest_sort
        f.argtypes = [C.c_uint32, C.c_uint32, C.c_int, C.c_uint32]
        f.restype = C.c_int
        print(json.dumps([f(n, na, which, seed) for n, na, which, seed in json.loads(sys.argv[2])]), flush=True)
    elif sys.argv[1] == "occ":
        import numpy as np
        d, dollar, rows_p, out_p = sys.argv[2], int(sys.argv[3]), sys.argv[4], sys.argv[5]
        rows = np.fromfile(rows_p, dtype=np.uint64)
        f = L.dsb_gpu_selftest_occ
        f.argtypes = [C.c_char_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p, C.c_char_p, C.c_size_t]
        f.restype = C.c_int
        got = np.zeros((len(rows), 7), dtype=np.uint64)
        err = C.create_string_buffer(512)
        rc = f(d.encode(), dollar, rows.ctypes.data, len(rows), got.ctypes.data, err, 512)
        got.tofile(out_p)
        print(json.dumps({"rc": rc, "err": err.value.decode()}), flush=True)


if __name__ == "__main__":
    main()
