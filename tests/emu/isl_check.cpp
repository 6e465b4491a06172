// tests/emu/isl_check.cpp — TEST ONLY: the island scan in batches of G positions (dsb_isl_* +
// dsb_top_push, desamba-so_amd/csrc/gpu/dsb_classify.h, the logic of k_island_g) against the
// one-bit-at-a-time scan dsb_search_exist + the top-seed pass of dsb_seed_vector (the reference's
// search_exist_kmer_M2 / get_seed_vector_M2, src/cly.c:1066-1229) over the same exist bits:
// seeded random bit vectors of many densities, long runs (the len > 60 cut), lengths 0..3000,
// both directions, grid / run batches of 4..32 positions, first run batches of 4..8.  The seed buffers start with the same
// garbage, so the stale top-byte writes must match too.  Exit status 0 iff everything agrees.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "../../desamba-so_amd/csrc/gpu/dsb_classify.h"

static uint64_t st = 1;
static uint64_t rnd() { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; }

/* the reference form: dsb_search_exist + dsb_seed_vector's top pass (one strand) */
static uint32_t ref_scan(const uint64_t *ex, uint32_t nk, dsb_seed_t *seed_v, uint32_t dir, uint32_t *total)
{
	uint32_t l = dsb_search_exist(ex, nk, seed_v, dir);
	uint32_t tot = 0, max_length = 0, index_end = 100;
	int max_index = 0;
	for (uint32_t m = 0; m < l; m++) {
		seed_v[m].top = 0;
		uint32_t key = dir == DSB_FORWARD ? seed_v[m].offset : nk - seed_v[m].offset - seed_v[m].len;
		if (key < index_end) {
			if (max_length < seed_v[m].len) { max_length = seed_v[m].len; max_index = m; }
			seed_v[max_index].top = 0;
		} else {
			seed_v[max_index].top = 1;
			index_end += 100;
			tot += max_length;
			max_index = m;
			max_length = seed_v[m].len;
		}
	}
	seed_v[max_index].top = 1;
	*total = tot + max_length;
	return l;
}

/* the batched form, lanes emulated: the stores k_island_g's group lane 0 makes */
template <int GG, int GR, int GR1>
static uint32_t batch_scan(const uint64_t *ex, uint32_t nk, dsb_seed_t *seed_v, uint32_t dir, uint32_t *total,
			   uint64_t *probes)
{
	dsb_isl_t s;
	dsb_isl_init(&s, (int)nk, dir == DSB_FORWARD, 1);
	dsb_topst_t top;
	dsb_top_init(&top);
	while (s.mode != DSB_ISL_DONE) {
		uint32_t mb = 0;
		for (int g = 0; g < 32; g++) {
			int q = dsb_isl_pos<GG, GR, GR1>(&s, g);
			if (q >= 0) {
				(*probes)++;
				if ((ex[q >> 6] >> (q & 63)) & 1) mb |= 1u << g;
			}
		}
		uint32_t so = 0, sl = 0;
		if (dsb_isl_step<GG, GR, GR1>(&s, mb, &so, &sl)) {
			uint32_t m = top.n, ti;
			seed_v[m].offset = so;
			seed_v[m].len = sl;
			seed_v[m].top = 0;
			uint8_t tv = dsb_top_push(&top, dir == DSB_FORWARD ? so : nk - so - sl, sl, &ti);
			seed_v[ti].top = tv;
		}
	}
	seed_v[top.max_index].top = 1;
	*total = top.total + top.max_length;
	return top.n;
}

template <int GG, int GR, int GR1 = GR>
static long check(long trials, uint64_t *probes, uint64_t *positions)
{
	long bad = 0;
	for (long t = 0; t < trials; t++) {
		uint32_t nk = (uint32_t)(rnd() % 3001);
		if (rnd() % 10 == 0) nk = (uint32_t)(rnd() % 8);
		std::vector<uint64_t> ex((nk + 63) / 64 + 1, 0);
		/* runs of set bits: density and run length vary per trial (long runs hit the 60 cut) */
		int p_on = (int)(rnd() % 60), p_stay = (int)(rnd() % 100);
		int on = 0;
		for (uint32_t q = 0; q < nk; q++) {
			on = on ? (int)(rnd() % 100) < p_stay : (int)(rnd() % 100) < p_on;
			if (on) ex[q >> 6] |= 1ull << (q & 63);
		}
		for (uint32_t dir : {(uint32_t)DSB_FORWARD, (uint32_t)DSB_REVERSE}) {
			size_t cap = nk / 2 + 8;
			std::vector<dsb_seed_t> a(cap), b(cap);
			for (size_t k = 0; k < cap; k++) { /* the same garbage in both */
				uint64_t g1 = rnd(), g2 = rnd();
				memcpy(&a[k], &g1, 8);
				memcpy((char *)&a[k] + 8, &g2, sizeof(dsb_seed_t) - 8);
			}
			b = a;
			uint32_t ta = 0, tb = 0;
			uint32_t la = ref_scan(ex.data(), nk, a.data(), dir, &ta);
			uint32_t lb = batch_scan<GG, GR, GR1>(ex.data(), nk, b.data(), dir, &tb, probes);
			*positions += nk;
			if (la != lb || ta != tb || memcmp(a.data(), b.data(), cap * sizeof(dsb_seed_t))) {
				if (bad < 5)
					fprintf(stderr, "GG=%d GR=%d GR1=%d nk=%u dir=%u: seeds %u vs %u, total %u vs %u\n", GG, GR, GR1, nk, dir, la, lb, ta, tb);
				bad++;
			}
		}
	}
	return bad;
}

int main(int argc, char **argv)
{
	st = argc > 1 ? strtoull(argv[1], 0, 10) | 1 : 1;
	long n = argc > 2 ? atol(argv[2]) : 20000, bad = 0;
	uint64_t pr[10] = {0}, pos[10] = {0};
	bad += check<4, 4>(n, &pr[0], &pos[0]);
	bad += check<8, 8>(n, &pr[1], &pos[1]);
	bad += check<16, 16>(n, &pr[2], &pos[2]);
	bad += check<32, 32>(n, &pr[3], &pos[3]);
	bad += check<16, 8>(n, &pr[4], &pos[4]);
	bad += check<8, 16>(n, &pr[5], &pos[5]);
	bad += check<12, 16>(n, &pr[6], &pos[6]);
	/* a narrower first run batch (RUN1: 2 back neighbours + GR1 - 2 after the hit) */
	bad += check<8, 16, 8>(n, &pr[7], &pos[7]);
	bad += check<8, 12, 4>(n, &pr[8], &pos[8]);
	bad += check<4, 32, 6>(n, &pr[9], &pos[9]);
	printf("grid/run/run1 4/4/4 8/8/8 16/16/16 32/32/32 16/8/8 8/16/16 12/16/16 8/16/8 8/12/4 4/32/6 probes per position:");
	for (int k = 0; k < 10; k++) printf(" %.3f", (double)pr[k] / pos[k]);
	printf("\nisl_check: %ld trials x 2 directions x 10 batch shapes, %ld mismatches\n", n, bad);
	return bad != 0;
}
