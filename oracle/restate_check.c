/*
 * oracle/restate_check.c — TEST INFRASTRUCTURE ONLY: pins this repository's C restatement
 * (oracle/restate.c) against the reference's own compiled functions.
 *
 * Linked with the reference objects built from /root/reference/src by oracle/Makefile; the
 * reference's cly.c is compiled with -Dstatic= (a compile flag, the sources are untouched) so
 * that its file-local primitives (get_exist_kmer, bwt_MEM_search, get_ref, get_uni, lv_extd)
 * can be called directly.  Every comparison runs on the committed fixture index (loaded with
 * the reference's own load_index) and on seeded random or simulated inputs.
 *
 * usage: restate_check <index_dir> [seed]      exit 0 iff no mismatch
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include <stdbool.h>
#include "cly.h"
#include "idx.h"
#include "lib/utils.h"
#include "restate.h"

/* the reference's primitives (cly.c, bwt.c, lib/utils.c) */
typedef struct { uint64_t *set; int l, m; } REF_SP_SET;            /* cly.c:1275-1279 */
typedef struct { int match_len; uint64_t sp, sa_sp; int sa_sp_l, kmer_index, read_offset; } REF_MEM; /* cly.c:614-622 */
void load_index(void **idx, const char *dirPath);
uint64_t occ(bwt *bt, uint64_t r, uint8_t *c);
int get_exist_kmer(uint8_t *e1, uint8_t *e2, uint64_t kmer, uint64_t mask);
void store_kmers(uint8_t *bin_read, uint32_t kmer_len, uint8_t l_e_kmer, int single_base_max, uint64_t *kmer_buff);
void get_ref(uint8_t *unitig_str, uint8_t *ref_str, uint64_t uni_offset, uint32_t length, bool isForward);
UNITIG *get_uni(DA_IDX *idx, uint64_t bwt_pos, int search_l, uint64_t *global_offset, uint32_t *uni_offset_);
int32_t lv_extd(uint8_t *ref, int32_t ref_length, uint8_t *query, int32_t query_length);
int bwt_MEM_search(bwt *bt, uint8_t *string, uint64_t pre_v, int max_rst, int l_min_mth, int l_max_mth,
		   REF_SP_SET *sp_set, REF_MEM *mem_rst);

static uint64_t g_state;
static uint64_t rnd(void)
{
	g_state ^= g_state << 13;
	g_state ^= g_state >> 7;
	g_state ^= g_state << 17;
	return g_state;
}

static int g_bad_total = 0;
static void report(const char *what, uint64_t n, uint64_t bad)
{
	printf("restate_check %-14s %9lu compared %6lu mismatches\n", what, (unsigned long)n, (unsigned long)bad);
	if (bad)
		g_bad_total = 1;
}

/* a read of length L copied from the packed reference at a random position, with substitutions */
static void sim_read(DA_IDX *idx, uint8_t *bin, uint32_t L, int err_pct)
{
	uint64_t n_bases = idx->ref_bin.n * 4;
	uint64_t st = 64 + rnd() % (n_bases - L - 128);
	rs_get_ref(idx->ref_bin.a, bin, st, L, 1);
	for (uint32_t k = 0; k < L; k++)
		if ((int)(rnd() % 100) < err_pct)
			bin[k] = (uint8_t)(rnd() & 3);
}

static int cmp01(const void *a, const void *b) /* Anchor_cmp_by_chr_ID_and_pos style: 0/1 only */
{
	const uint32_t *x = a, *y = b;
	return (x[0] != y[0]) ? (x[0] > y[0]) : (x[1] > y[1]);
}
static int cmp_mod2(const void *a, const void *b) /* chain_cmp_by_MEM_score style: ties -> a % 2 */
{
	const uint32_t *x = a, *y = b;
	int sa = (int)(x[0] << 5), sb = (int)(y[0] << 5);
	if (sa < sb) return 1;
	if (sa > sb) return -1;
	return (int)(x[0] % 2);
}

int main(int argc, char **argv)
{
	if (argc < 2) {
		fprintf(stderr, "usage: %s <index_dir> [seed]\n", argv[0]);
		return 2;
	}
	g_state = argc > 2 ? strtoull(argv[2], NULL, 10) | 1 : 88172645463325252ull;
	DA_IDX *idx = NULL;
	load_index((void **)&idx, argv[1]);
	bwt *bt = &idx->bt;
	rs_fm_t fm;
	fm.bwt_occ = bt->bwt_occ;
	memcpy(fm.rank, bt->rank, sizeof(fm.rank));
	fm.hash_index = bt->hash_index;
	fm.dollor_pos = bt->DOLLOR_POS;
	uint64_t n_rows = bt->hash_index[1ull << (2 * 13)];

	/* 1. occ with a given symbol and with the symbol read at r */
	uint64_t n = 0, bad = 0;
	for (int t = 0; t < 400000; t++) {
		uint64_t r = rnd() % n_rows;
		uint8_t c = (t % 5 == 4) ? 0xff : (uint8_t)(t % 5), c2 = c;
		uint64_t a = occ(bt, r, &c), b = rs_occ(&fm, r, &c2);
		n++;
		bad += (a != b || c != c2);
	}
	report("occ", n, bad);

	/* 2. hash64_1 / hash64_2 */
	n = bad = 0;
	for (int t = 0; t < 1000000; t++) {
		uint64_t k = rnd() >> (rnd() & 31);
		n++;
		bad += hash64_1(k) != rs_hash64_1(k) || hash64_2(k) != rs_hash64_2(k);
	}
	report("hash64", n, bad);

	/* 3. store_kmers + get_exist_kmer on simulated reads (both strands) */
	E_KMER *ek = &idx->ek;
	uint64_t nk = 0, badk = 0, ne = 0, bade = 0, hits = 0;
	for (int t = 0; t < 400; t++) {
		uint32_t L = 40 + (uint32_t)(rnd() % 3000);
		uint8_t *bin = malloc(2 * L + 64);
		sim_read(idx, bin, L, (int)(rnd() % 16));
		for (uint32_t k = 0; k < L; k++)
			bin[L + L - 1 - k] = 3 - bin[k];
		uint32_t nkm = L - ek->len_e_kmer + 1;
		uint64_t *ka = malloc(8 * nkm), *kb = malloc(8 * nkm);
		for (int s = 0; s < 2; s++) {
			store_kmers(bin + s * L, nkm, ek->len_e_kmer, ek->single_base_max, ka);
			rs_store_kmers(bin + s * L, nkm, ek->len_e_kmer, ek->single_base_max, kb);
			nk += nkm;
			for (uint32_t k = 0; k < nkm; k++) {
				badk += ka[k] != kb[k];
				int x = get_exist_kmer(ek->e_kmer0, ek->e_kmer1, ka[k], ek->e_kmer_hash_mask);
				int y = rs_exist_kmer(ek->e_kmer0, ek->e_kmer1, ka[k], ek->e_kmer_hash_mask);
				ne++;
				hits += x;
				bade += x != y;
			}
		}
		free(ka); free(kb); free(bin);
	}
	report("store_kmers", nk, badk);
	report("exist_kmer", ne, bade);
	printf("restate_check exist_kmer hits %lu of %lu\n", (unsigned long)hits, (unsigned long)ne);

	/* 4. get_ref, both directions */
	n = bad = 0;
	uint64_t n_bases = idx->ref_bin.n * 4;
	for (int t = 0; t < 200000; t++) {
		uint32_t len = (uint32_t)(rnd() % 80);
		uint64_t off = 100 + rnd() % (n_bases - 200);
		int fwd = (int)(rnd() & 1);
		uint8_t a[96], b[96];
		memset(a, 0xAA, sizeof(a));
		memset(b, 0xAA, sizeof(b));
		get_ref(idx->ref_bin.a, a, off, len, fwd);
		rs_get_ref(idx->ref_bin.a, b, off, len, fwd);
		n++;
		bad += memcmp(a, b, sizeof(a)) != 0;
	}
	report("get_ref", n, bad);

	/* 5. get_uni at SA-sampled rows, search_l 0..8 */
	n = bad = 0;
	for (int t = 0; t < 200000; t++) {
		uint64_t r = (rnd() % n_rows) & ~7ull;
		int sl = (int)(rnd() % 17) - 8; /* map_seed passes sa_sp_l <= 0 or an LF-walk length >= 0 */
		uint64_t ga, gb;
		uint32_t ua, ub;
		{ /* skip walks that run past the last unitig (a reference out-of-bounds read) */
			uint32_t uu = bt->sa_taxon[r >> 3].unitig_ID, off = bt->sa_taxon[r >> 3].offset + sl + 1;
			int ok = 1;
			if (sl > 0)
				while (ok && off >= idx->unitig_v.a[uu].length) {
					off -= idx->unitig_v.a[uu].length + 1;
					if (++uu >= idx->unitig_v.n) ok = 0;
				}
			if (!ok)
				continue;
		}
		UNITIG *u = get_uni(idx, r, sl, &ga, &ua);
		uint32_t ui = rs_get_uni((const rs_sa_t *)bt->sa_taxon, (const rs_uni_t *)idx->unitig_v.a,
					 (const uint64_t *)idx->r_p_v.a, r, sl, &gb, &ub);
		n++;
		bad += (ui != (uint32_t)(u - idx->unitig_v.a)) || ga != gb || ua != ub;
	}
	report("get_uni", n, bad);

	/* 6. lv_extd on <= 12-base windows (the map_seed / get_new_ed use) with stack-pattern guards */
	n = bad = 0;
	for (int t = 0; t < 400000; t++) {
		uint8_t r1[48], q1[48], r2[48], q2[48];
		memset(r1, 0xAA, sizeof(r1));
		memset(q1, 0xAA, sizeof(q1));
		int len = (int)(rnd() % 13);
		for (int k = 0; k < len + 8; k++) {
			r1[16 + k] = (uint8_t)(rnd() & 3);
			q1[16 + k] = (rnd() % 100 < 20) ? (uint8_t)(rnd() & 3) : r1[16 + k];
		}
		if (rnd() % 4 == 0 && len > 2) { /* an indel */
			int p = (int)(rnd() % len);
			memmove(q1 + 16 + p + 1, q1 + 16 + p, 20);
		}
		memcpy(r2, r1, 48);
		memcpy(q2, q1, 48);
		int rl = len, ql = (rnd() % 8 == 0) ? (int)(rnd() % 13) : len;
		int32_t a = lv_extd(r1 + 16, rl, q1 + 16, ql);
		int32_t b = rs_lv_extd(r2 + 16, rl, q2 + 16, ql);
		n++;
		bad += a != b || memcmp(r1, r2, 48) || memcmp(q1, q2, 48);
	}
	report("lv_extd", n, bad);

	/* 7. bwt_MEM_search (fast-mode parameters and slow-mode parameters) along simulated reads */
	uint64_t ns = 0, bads = 0, found = 0;
	uint64_t *set_a = malloc(8 * 500), *set_b = malloc(8 * 500);
	for (int t = 0; t < 300; t++) {
		uint32_t L = 200 + (uint32_t)(rnd() % 2000);
		uint8_t *bin = malloc(L + 64);
		memset(bin, 0, 32);
		sim_read(idx, bin + 32, L, (int)(rnd() % 12));
		uint8_t *rd = bin + 32;
		REF_SP_SET sa = {set_a, 0, 500};
		rs_spset_t sb = {set_b, 0, 500};
		for (uint32_t end = 20; end < L; end += 1 + (uint32_t)(rnd() % 7)) {
			uint64_t pre_v = 0;
			for (int k = 12; k >= 0; k--)
				pre_v = (pre_v << 2) | rd[end - k];
			int slow = (int)(rnd() & 1);
			int max_rst = slow ? 8 : 2, l_min = slow ? 19 : 20, l_max = (int)end;
			REF_MEM ma[16];
			rs_mem_t mb[16];
			memset(ma, 0, sizeof(ma));
			memset(mb, 0, sizeof(mb));
			if (rnd() % 16 == 0) { sa.l = 0; sb.l = 0; }
			int x = bwt_MEM_search(bt, rd + end, pre_v, max_rst, l_min, l_max, &sa, ma);
			int y = rs_mem_search(&fm, rd + end, pre_v, max_rst, l_min, l_max, &sb, mb);
			ns++;
			found += x;
			int diff = x != y || sa.l != sb.l || memcmp(set_a, set_b, 8 * (size_t)sa.l);
			for (int k = 0; k < x && k < y && !diff; k++)
				diff = ma[k].match_len != mb[k].match_len || ma[k].sp != mb[k].sp || ma[k].sa_sp != mb[k].sa_sp ||
				       ma[k].sa_sp_l != mb[k].sa_sp_l;
			bads += diff;
		}
		free(bin);
	}
	free(set_a); free(set_b);
	report("mem_search", ns, bads);
	printf("restate_check mem_search hits %lu\n", (unsigned long)found);

	/* 8. glibc qsort vs the msort restatement, with the reference's partial comparators */
	n = bad = 0;
	for (int t = 0; t < 3000; t++) {
		size_t m = (size_t)(rnd() % 700);
		uint32_t *a = malloc(8 * m + 8), *b = malloc(8 * m + 8);
		for (size_t k = 0; k < m; k++) {
			a[2 * k] = (uint32_t)(rnd() % 6);
			a[2 * k + 1] = (uint32_t)(rnd() % 9);
		}
		memcpy(b, a, 8 * m);
		int which = t & 1;
		qsort(a, m, 8, which ? cmp_mod2 : cmp01);
		rs_msort(b, m, 8, which ? cmp_mod2 : cmp01);
		n++;
		bad += memcmp(a, b, 8 * m) != 0;
		free(a); free(b);
	}
	report("msort", n, bad);
	return g_bad_total;
}
