// tests/emu/mem_check.cpp — TEST ONLY: the GPU path's word-wise MEM_search (dsb_MEM_search,
// desamba-so_amd/csrc/gpu/dsb_classify.h; built here with DSB_MEM_WORDS = 1, 2 or 4) against the
// reference's byte loop (src/cly.c:1805-1813: `len < max && *q++ == *t++`, or `*q-- == *t--`) on
// seeded random strings with planted runs of matches, both directions, max from -3 to 300.
// Exit status 0 iff all agree.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "../../desamba-so_amd/csrc/gpu/dsb_classify.h"

static int byte_loop(const uint8_t *q, const uint8_t *t, int forward, int max)
{
	int len = 0;
	if (forward)
		while (len < max && *q++ == *t++) len++;
	else
		while (len < max && *q-- == *t--) len++;
	return len;
}

int main(int argc, char **argv)
{
	uint64_t st = argc > 1 ? strtoull(argv[1], 0, 10) | 1 : 1;
	auto rnd = [&]() { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; };
	long n = argc > 2 ? atol(argv[2]) : 1000000, bad = 0;
	static uint8_t q[2048], t[2048];
	for (long it = 0; it < n; it++) {
		for (int k = 0; k < 2048; k++) q[k] = (uint8_t)(rnd() & 3);
		memcpy(t, q, sizeof(t));
		int run = (int)(rnd() % 260);
		int qo = 700 + (int)(rnd() % 300), to = 700 + (int)(rnd() % 300);
		for (int k = -400; k < 400; k++) t[to + k] = q[qo + k]; /* aligned copy around the start */
		int fw = (int)(rnd() & 1);
		int cut = fw ? qo + run : qo - run; /* first mismatch */
		t[to + (cut - qo)] ^= 1 + (uint8_t)(rnd() % 3);
		int max = (int)(rnd() % 304) - 3;
		int a = dsb_MEM_search(q + qo, t + to, fw, max);
		int b = byte_loop(q + qo, t + to, fw, max);
		if (b < 0) b = 0;
		if (a != b) {
			if (bad < 10) printf("mismatch: fw %d max %d run %d -> %d vs %d\n", fw, max, run, a, b);
			bad++;
		}
	}
	printf("%ld trials, %ld mismatches\n", n, bad);
	return bad != 0;
}
