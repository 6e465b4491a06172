// tests/emu/lv_check.cpp — TEST ONLY: the register-word lv_extd of the GPU path (dsb_lv_extd_w,
// desamba-so_amd/csrc/gpu/dsb_core.h) against the byte-buffer form (dsb_lv_extd) and against the
// oracle's restatement (oracle/restate.c rs_lv_extd, pinned to the reference's lv_extd) on seeded
// random windows of the shape every caller uses (32-byte buffers, string at +8, stack-pattern
// guards, lengths 0..12, substitutions / indels, ragged lengths).  Exit status 0 iff all agree.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "../../desamba-so_amd/csrc/gpu/dsb_core.h"
extern "C" {
#include "../../oracle/restate.h"
}
int main(int argc, char **argv)
{
	uint64_t st = argc > 1 ? strtoull(argv[1], 0, 10) | 1 : 1;
	auto rnd = [&]() { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; };
	long n = argc > 2 ? atol(argv[2]) : 2000000, bad = 0;
	for (long t = 0; t < n; t++) {
		uint8_t r[32], q[32];
		uint8_t fill = (rnd() & 7) == 0 ? (uint8_t)(rnd() & 3) : 0xAA;
		memset(r, fill, 32);
		memset(q, 0xAA, 32);
		int len = (int)(rnd() % 13);
		for (int k = 0; k < 24; k++) {
			r[8 + k] = (k < len + 4 || (rnd() & 1)) ? (uint8_t)(rnd() & 3) : r[8 + k];
			q[8 + k] = (rnd() % 100 < 15) ? (uint8_t)(rnd() & 3) : r[8 + k];
		}
		if (rnd() % 3 == 0 && len > 1) { int p = (int)(rnd() % len); memmove(q + 8 + p + 1, q + 8 + p, 23 - p); }
		if (rnd() % 3 == 0 && len > 1) { int p = (int)(rnd() % len); memmove(q + 8 + p, q + 8 + p + 1, 23 - p); }
		if (rnd() % 5 == 0) { q[7] = (uint8_t)(rnd() & 3); r[3 + (rnd() % 5)] = (uint8_t)(rnd() & 3); }
		int rl = len, ql = (rnd() % 6 == 0) ? (int)(rnd() % 13) : len;
		uint8_t r1[32], q1[32], r2[32], q2[32];
		memcpy(r1, r, 32); memcpy(q1, q, 32); memcpy(r2, r, 32); memcpy(q2, q, 32);
		int32_t a = dsb_lv_extd_w(r + 8, rl, q + 8, ql);
		int32_t b = dsb_lv_extd(r1 + 8, rl, q1 + 8, ql);
		int32_t c = rs_lv_extd(r2 + 8, rl, q2 + 8, ql);
		if (a != b || b != c || memcmp(r, r1, 32) || memcmp(q, q1, 32)) {
			if (bad < 5) fprintf(stderr, "mismatch rl=%d ql=%d: words %d bytes %d oracle %d\n", rl, ql, a, b, c);
			bad++;
		}
	}
	printf("lv_check %ld compared %ld mismatches\n", n, bad);
	return bad != 0;
}
