/*
 * oracle/restate.c — TEST INFRASTRUCTURE ONLY (see restate.h): a plain-C restatement of the
 * classify hot-path primitives of the reference, each function citing the reference lines it
 * follows (paths relative to /root/reference/src).  Written for clarity, one symbol at a
 * time, with none of the GPU path's data-layout or word-level tricks, so that agreement
 * between this file, the reference's compiled functions and the GPU kernels is evidence
 * about the algorithm rather than about shared code.
 *
 * Pinned by oracle/restate_check.c (tests/test_oracle_restate.py): every function here is
 * compared with the reference's own compiled function on the committed fixture index and on
 * random inputs.
 */
#include <stdlib.h>
#include <string.h>
#include "restate.h"

#define RS_L_PRE_IDX 13   /* idx.h:58 */
#define RS_SA_MASK 7      /* bwt.h:7 */
#define RS_SA_OFF 3       /* bwt.h:8 */
#define RS_LV_ERROR 4     /* cly.c:493 */
#define RS_MIN(a, b) ((a) < (b) ? (a) : (b))
#define RS_MAX(a, b) ((a) > (b) ? (a) : (b))

/* cly.c:16-34 — the table maps A/a -> 0, C/c -> 1, G/g -> 2, T/t -> 3 and every other byte
 * of 0..127 to 1.  (Bytes >= 128 index the table with a negative int8 in the reference:
 * unpinned, 1 here.) */
uint8_t rs_cly_bit(uint8_t c)
{
	if (c == 'A' || c == 'a') return 0;
	if (c == 'G' || c == 'g') return 2;
	if (c == 'T' || c == 't') return 3;
	return 1;
}

/* cly.c:1245-1254 */
void rs_encode_read(const char *seq, uint32_t L, uint8_t *bin)
{
	for (uint32_t k = 0; k < L; k++)
		bin[k] = rs_cly_bit((uint8_t)seq[k]);
	for (uint32_t k = 0; k < L; k++)
		bin[L + (L - k - 1)] = (uint8_t)(3 - bin[k]);
}

/* cly.c:359-397 with bit2_nextKmer_init / bit2_nextKmerMASK (lib/utils.h:164,173) and
 * kmerMask[l] = low 2l bits (lib/utils.c:1000) */
void rs_store_kmers(const uint8_t *bin, uint32_t n, int l, int single_base_max, uint64_t *out)
{
	uint64_t mask = (l >= 32) ? ~0ull : ((1ull << (2 * l)) - 1);
	int cnt[4] = {0, 0, 0, 0};
	uint64_t kmer = 0;
	for (int i = 0; i < l; i++)
		cnt[bin[i]]++;
	for (int i = 0; i < l - 1; i++) /* binchar2Kmer(s, l) >> 2: the first l-1 bases */
		kmer = (kmer << 2) | bin[i];
	for (uint32_t i = 0; i < n; i++) {
		if (i > 0) {
			cnt[bin[i - 1]]--;
			cnt[bin[i + l - 1]]++;
		}
		kmer = ((kmer << 2) | bin[i + l - 1]) & mask;
		int low = cnt[0] >= single_base_max || cnt[1] >= single_base_max || cnt[2] >= single_base_max ||
			  cnt[3] >= single_base_max;
		out[i] = low ? 0 : kmer;
	}
}

/* lib/utils.c:1067-1077 (Thomas Wang's 64-bit mix) */
uint64_t rs_hash64_1(uint64_t key)
{
	key = (~key) + (key << 21);
	key = key ^ (key >> 24);
	key = (key + (key << 3)) + (key << 8);
	key = key ^ (key >> 14);
	key = (key + (key << 2)) + (key << 4);
	key = key ^ (key >> 28);
	key = key + (key << 31);
	return key;
}

/* lib/utils.c:1080-1091 */
uint64_t rs_hash64_2(uint64_t key)
{
	key += ~(key << 32);
	key ^= (key >> 22);
	key += ~(key << 13);
	key ^= (key >> 8);
	key += (key << 3);
	key ^= (key >> 15);
	key += ~(key << 27);
	key ^= (key >> 31);
	return key;
}

/* cly.c:951-967: bit 7-(h&7) of byte h>>3 in each table; table 2 only after a hit */
int rs_exist_kmer(const uint8_t *ek0, const uint8_t *ek1, uint64_t kmer, uint64_t hash_mask)
{
	if (kmer == 0)
		return 0;
	uint64_t h1 = rs_hash64_1(kmer) & hash_mask;
	if (((ek0[h1 >> 3] >> (7 - (h1 & 7))) & 1) == 0)
		return 0;
	uint64_t h2 = rs_hash64_2(kmer) & hash_mask;
	return (ek1[h2 >> 3] >> (7 - (h2 & 7))) & 1;
}

/* bwt.c:43-65: block r>>8 of 168 bytes, checkpoint count[c] + the symbols equal to c among
 * positions [r & ~255, r) of the block.  Symbol k of a block is nibble k of its 128 bytes,
 * little-endian nibble order within each u16 group (bwt.c:32-42). */
static uint8_t rs_sym(const uint8_t *blk, uint32_t k)
{
	uint8_t b = blk[40 + (k >> 1)];
	return (k & 1) ? (uint8_t)(b >> 4) : (uint8_t)(b & 0xf);
}
uint64_t rs_occ(const rs_fm_t *fm, uint64_t r, uint8_t *c)
{
	const uint8_t *blk = fm->bwt_occ + (r >> 8) * 168;
	uint32_t within = (uint32_t)(r & 0xff);
	if (*c == 0xff) {
		*c = rs_sym(blk, within);
		if (*c == 5)
			return fm->dollor_pos;
	}
	uint64_t base;
	memcpy(&base, blk + 8 * (*c), 8);
	uint64_t count = 0;
	for (uint32_t k = 0; k < within; k++)
		count += rs_sym(blk, k) == *c;
	return base + count;
}

/* cly.c:1281-1293: a 500-slot array that forgets everything when full */
int rs_spset_insert(uint64_t node, rs_spset_t *s)
{
	if (s->l == s->m)
		s->l = 0;
	for (int i = 0; i < s->l; i++)
		if (s->set[i] == node)
			return 0;
	s->set[s->l++] = node;
	return 1;
}

/* cly.c:1339-1378 */
void rs_single_search(const rs_fm_t *fm, uint64_t sp, const uint8_t *string, int max_match_len, rs_spset_t *set,
		      rs_mem_t *out)
{
	uint64_t sa_sp = ~0ull;
	int match_len = 0, sa_sp_l = 0;
	for (;;) {
		if (match_len >= max_match_len)
			break;
		if ((sp & RS_SA_MASK) == 0) {
			sa_sp = sp;
			sa_sp_l = 0;
		} else
			sa_sp_l--;
		uint8_t c = 0xff;
		uint64_t new_sp = rs_occ(fm, sp, &c) + fm->rank[c];
		if (c != *string)
			break;
		match_len++;
		string--;
		if (!rs_spset_insert(new_sp, set)) {
			out->match_len = -1000;
			return;
		}
		sp = new_sp;
	}
	out->sp = sp;
	out->match_len = match_len;
	out->sa_sp = sa_sp;
	out->sa_sp_l = sa_sp_l;
}

/* cly.c:1383-1442: backward search from the 13-mer prefix interval until at most max_rst
 * rows remain (once the match reaches l_min - 1), then single-row extension of each row */
int rs_mem_search(const rs_fm_t *fm, const uint8_t *string, uint64_t pre_v, int max_rst, int l_min, int l_max,
		  rs_spset_t *set, rs_mem_t *out)
{
	int n = 0;
	uint64_t sp = fm->hash_index[pre_v], ep = fm->hash_index[pre_v + 1], nsp, nep;
	string -= RS_L_PRE_IDX;
	int match_len = RS_L_PRE_IDX;
	for (;;) {
		uint8_t c = *string, c2;
		string--;
		c2 = c;
		nsp = fm->rank[c] + rs_occ(fm, sp, &c);
		nep = fm->rank[c2] + rs_occ(fm, ep, &c2);
		if (match_len >= l_min - 1) {
			if (nsp + (uint64_t)max_rst >= nep)
				break;
			if (match_len >= l_max)
				return 0;
		}
		if (nsp + 1 >= nep)
			break;
		match_len++;
		sp = nsp;
		ep = nep;
	}
	if (nsp >= nep)
		return 0;
	for (uint64_t row = nsp; row < nep; row++) { /* one row: the reference's first branch */
		if (!rs_spset_insert(row, set)) {
			if (nsp + 1 == nep)
				return 0;
			continue;
		}
		rs_single_search(fm, row, string, RS_MAX(0, l_max - match_len), set, out + n);
		out[n].match_len += match_len + 1;
		if (out[n].match_len >= l_min)
			n++;
	}
	return n;
}

/* cly.c:434-461: MSB-first 2-bit unpacking, forwards or backwards from uni_offset */
void rs_get_ref(const uint8_t *ref_bin, uint8_t *out, uint64_t uni_offset, uint32_t length, int forward)
{
	for (uint32_t k = 0; k < length; k++) {
		uint64_t pos = forward ? uni_offset + k : uni_offset - k;
		out[k] = (uint8_t)((ref_bin[pos >> 2] >> (6 - 2 * (pos & 3))) & 3);
	}
}

/* cly.c:466-491 (uni_offset is a uint32, so the search_l <= 0 loop never runs) */
uint32_t rs_get_uni(const rs_sa_t *sa, const rs_uni_t *uni, const uint64_t *r_p, uint64_t bwt_pos, int search_l,
		    uint64_t *global_offset, uint32_t *uni_offset)
{
	uint32_t u = sa[bwt_pos >> RS_SA_OFF].unitig_ID;
	uint32_t off = sa[bwt_pos >> RS_SA_OFF].offset + search_l + 1;
	if (search_l > 0)
		while (off >= uni[u].length) {
			off -= uni[u].length + 1;
			u++;
		}
	*global_offset = (r_p[uni[u].ref_list] & 0xFFFFFFFFFFull) + off;
	*uni_offset = off;
	return u;
}

/* cly.c:505-604: semi-global banded Landau-Vishkin, diagonals -4..4, at most 4 errors.
 * mn[d] / ed[d]: furthest match and edit count on diagonal d. */
int32_t rs_lv_extd(uint8_t *ref, int32_t ref_length, uint8_t *query, int32_t query_length)
{
	if (ref_length < query_length) {
		uint8_t *tp = ref; ref = query; query = tp;
		int32_t tl = ref_length; ref_length = query_length; query_length = tl;
	}
	int32_t mn_store[2 * RS_LV_ERROR + 5], ed_store[2 * RS_LV_ERROR + 5];
	int32_t *mn = mn_store + RS_LV_ERROR + 1, *ed = ed_store + RS_LV_ERROR + 1;
	for (int d = -RS_LV_ERROR - 1; d <= RS_LV_ERROR + 1; d++) {
		mn[d] = -1;
		ed[d] = d > 0 ? d : -d;
	}
	mn[RS_LV_ERROR + 2] = -1; /* read after the last diagonal, never used */
	ed[RS_LV_ERROR + 2] = RS_LV_ERROR + 2;
	uint8_t keep_r = ref[ref_length], keep_q = query[query_length];
	ref[ref_length] = '#';
	query[query_length] = '$';
	int32_t best = query_length;
	for (int e = 0; e <= RS_LV_ERROR; e++) {
		int32_t p_mn = -1, c_mn = e - 1, n_mn = mn[-e + 1];
		int32_t p_ed = e + 1, c_ed = e, n_ed = ed[-e + 1];
		for (int d = -e; d <= RS_LV_ERROR; d++) {
			int32_t m, x;
			if (c_mn + d < ref_length - 1) { /* extend along, or take the insertion / deletion */
				int32_t key = c_mn + 1 - c_ed;
				m = c_mn + 1;
				x = c_ed + 1;
				if (key < n_mn + 1 - n_ed) {
					m = n_mn + 1;
					x = n_ed + 1;
					key = n_mn - n_ed;
				}
				if (key < p_mn - p_ed) {
					m = p_mn + 1;
					x = p_ed + 1;
				}
			} else { /* at the end of the reference */
				int32_t key = c_mn - c_ed;
				m = c_mn;
				x = c_ed + 1;
				if (key < p_mn - p_ed) {
					m = p_mn;
					x = p_ed + 1;
					key = p_mn - p_ed;
				}
				if (key < n_mn + 1 - n_ed) {
					m = n_mn + 1;
					x = n_ed + 1;
				}
			}
			int32_t j = RS_MIN(m, query_length);
			j = RS_MIN(j, ref_length - d);
			while (ref[j + d] == query[j])
				j++;
			mn[d] = j;
			ed[d] = x;
			if (query[j] == '$' || ref[j + d] == '#') {
				best = RS_MIN(x - 1, best);
				if (d <= e + 1) {
					ref[ref_length] = keep_r;
					query[query_length] = keep_q;
					return best;
				}
			}
			p_mn = c_mn; c_mn = n_mn; n_mn = mn[d + 2];
			p_ed = c_ed; c_ed = n_ed; n_ed = ed[d + 2];
		}
	}
	ref[ref_length] = keep_r;
	query[query_length] = keep_q;
	return best;
}

/* glibc 2.35 stdlib/msort.c msort_with_tmp: recursive top-down merge sort, n1 = n / 2, the
 * left element is taken when cmp(left, right) <= 0 (elements copied by value here; glibc's
 * indirect sorting of large elements performs the same comparisons). */
static void rs_msort_rec(char *b, size_t n, size_t s, int (*cmp)(const void *, const void *), char *tmp)
{
	if (n <= 1)
		return;
	size_t n1 = n / 2, n2 = n - n1;
	char *b1 = b, *b2 = b + n1 * s;
	rs_msort_rec(b1, n1, s, cmp, tmp);
	rs_msort_rec(b2, n2, s, cmp, tmp);
	char *t = tmp;
	while (n1 > 0 && n2 > 0) {
		if (cmp(b1, b2) <= 0) {
			memcpy(t, b1, s);
			b1 += s;
			n1--;
		} else {
			memcpy(t, b2, s);
			b2 += s;
			n2--;
		}
		t += s;
	}
	if (n1 > 0)
		memcpy(t, b1, n1 * s);
	memcpy(b, tmp, (n - n2) * s);
}
void rs_msort(void *base, size_t n, size_t size, int (*cmp)(const void *, const void *))
{
	char *tmp = malloc(n * size + 1);
	rs_msort_rec(base, n, size, cmp, tmp);
	free(tmp);
}
