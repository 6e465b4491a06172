/* desamba_mi355x_test.h — entry points of the TEST build only (desamba-so_amd/lib/libdesamba_test.so,
 * exports_test.map): device self-tests the GPU tests call.  The production library
 * (lib/libdesamba.so) does not contain them (tests/test_abi.py). */
#ifndef DESAMBA_MI355X_TEST_H
#define DESAMBA_MI355X_TEST_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* Self-tests of device code against host code (tests/): the glibc-2.35 msort restatement on the
 * device vs the host (returns the arrays whose permutation differs), and the HBM occ layout of
 * any index's .bwt (rows up to its length, past 2^32 included): out[7 i + c] = occ(rows[i], c) for
 * c = 0..4, out[7 i + 5] = occ(rows[i], 0xff) and out[7 i + 6] the symbol it read (0-4, or 5 for
 * the '$' row, which returns dollor_pos) — reference bwt.c:43-65.  Returns 0, or -1 with err. */
int dsb_gpu_selftest_sort(uint32_t n, uint32_t n_arrays, int which, uint32_t seed);
int dsb_gpu_selftest_occ(const char *dir, uint64_t dollor_pos, const uint64_t *rows, uint64_t n, uint64_t *out,
			 char *err, size_t errn);

#ifdef __cplusplus
}
#endif
#endif
