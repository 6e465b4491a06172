import ctypes as C, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = C.CDLL(os.path.join(ROOT, "desamba-so_amd", "lib", "libdesamba_test.so"))  # self-tests: the test build only
f = L.dsb_gpu_selftest_sort
f.argtypes = [C.c_uint32, C.c_uint32, C.c_int, C.c_uint32]
for n in [2, 3, 5, 7, 8, 13, 64, 200, 400]:
    print(n, [f(n, 256, w, 1234 + n) for w in (0, 1, 2, 3, 4)], flush=True)
