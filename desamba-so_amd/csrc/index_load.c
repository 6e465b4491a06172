/*
 * index_load.c — read a deSAMBA index directory into host memory.
 *
 * File formats as read by the reference loader:
 *   load_bwt  (src/bwt.c:68-104)   .bwt .sa (.acg is not needed: occ counts nibbles with
 *                                  bit operations instead of the AGCTCounter tables)
 *   load_idx  (src/idx.c:1103-1160) .exki .exk0 .exk1 .unv .ref_b .ref_i .ref_p
 *   set_ekmer_par (src/idx.c:966-982)
 *   calculate_MAPQ_TABLE (src/cly_mt.c:396-420)
 *   taxonTree_rank (src/cly_mt.c:590-670)
 */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <pthread.h>
#include "dsb_host.h"

#define REF_BIN_PAD 65536 /* zero bytes after the packed reference (over-reads read 'A') */

static FILE *open_ix(const char *dir, const char *postfix, char *err, size_t errn)
{
	size_t n = strlen(dir);
	char *p = malloc(n + 64);
	strcpy(p, dir);
	if (n == 0 || p[n - 1] != '/')
		strcat(p, "/");
	strcat(p, "deSAMBA");
	strcat(p, postfix);
	FILE *f = fopen(p, "rb");
	if (!f)
		snprintf(err, errn, "cannot open index file %s", p);
	free(p);
	return f;
}

static int rd(FILE *f, void *dst, size_t sz, size_t cnt, const char *what, char *err, size_t errn)
{
	if (cnt == 0)
		return 0;
	if (fread(dst, sz, cnt, f) != cnt) {
		snprintf(err, errn, "[xREAD] Wrong in read file, data not enough (%s)", what);
		return -1;
	}
	return 0;
}

static void *xm(size_t n)
{
	void *p = malloc(n ? n : 1);
	if (!p) {
		fprintf(stderr, "[dsb] out of memory (%zu bytes)\n", n);
		abort();
	}
	return p;
}

/* set_ekmer_par, src/idx.c:966-982 */
static void set_ekmer_par(dsb_index *ix)
{
	uint64_t mask = 0x1fffffffffull; /* MASK_37 */
	int l = 20;
	switch (ix->ek_size) {
	case 0x8000000ull:   mask = 0x3fffffffull;  l = 16; break;
	case 0x10000000ull:  mask = 0x7fffffffull;  l = 17; break;
	case 0x20000000ull:  mask = 0xffffffffull;  l = 17; break;
	case 0x40000000ull:  mask = 0x1ffffffffull; l = 18; break;
	case 0x80000000ull:  mask = 0x3ffffffffull; l = 18; break;
	case 0x100000000ull: mask = 0x7ffffffffull; l = 19; break;
	case 0x200000000ull: mask = 0xfffffffffull; l = 19; break;
	case 0x400000000ull: mask = 0x1fffffffffull; l = 20; break;
	}
	ix->ek_mask = mask;
	ix->l_ek = l;
	ix->single_base_max = (int)(0.8 * l); /* SINGLE_BASE_MAX_RATIO_THEADHOLD * len_e_kmer */
}

/*
 * occ table re-layout: the reference's 168-B blocks (bwt.c:32-42: u64 count of
 * A,C,G,T,'#' before the block + 256 4-bit symbols) -> one 64-B line per 128 symbols + a u64
 * count table per 2^24-symbol superblock.  Runs in parallel over block ranges: a line's counts come
 * from its block's checkpoint in the file plus the symbols before it in the block, a superblock's
 * from the checkpoint of the block it starts at.  The file is verified on the way: every block's
 * A/C/G/T checkpoints must equal the previous block's plus its symbols, and the '$' count the
 * '#' checkpoint implies (block start - A - C - G - T - '#') must grow by the '$' symbols of the
 * block, so the re-layout is lossless on every index it loads (rows are u64 throughout: BWTs past
 * 2^32 symbols, reference bwt.h:45; tests/test_gpu_bigbwt.py).
 */
typedef struct {
	dsb_index *ix;
	uint64_t b0, b1, nb;          /* blocks [b0, b1) of nb */
	uint64_t dollar[DSB_MAX_DOLLAR];
	int n_dollar, bad;
	char msg[256];
} relayout_part;

static void *relayout_range(void *arg)
{
	relayout_part *P = arg;
	dsb_index *ix = P->ix;
	for (uint64_t b = P->b0; b < P->b1 && !P->bad; b++) {
		const uint8_t *src = ix->bwt_occ + b * 168;
		uint64_t cnt[5], run[4];
		memcpy(cnt, src, 40);
		memcpy(run, cnt, 32);
		uint64_t dol_before = (b << 8) - cnt[0] - cnt[1] - cnt[2] - cnt[3] - cnt[4], dol = 0;
		if (b == 0 && (cnt[0] | cnt[1] | cnt[2] | cnt[3] | cnt[4])) {
			snprintf(P->msg, sizeof(P->msg), "deSAMBA.bwt: block 0 has non-zero checkpoints");
			P->bad = 1;
			break;
		}
		for (uint32_t k = 0; k < 256; k++) {
			uint64_t line = (b << 8 | k) / DSB_OCC_LINE_SYM;
			uint32_t kk = k % DSB_OCC_LINE_SYM;
			uint64_t *ln = ix->occ + line * DSB_OCC_LINE_U64;
			if (kk == 0) { /* line start: counts relative to its superblock (which starts at a block) */
				uint64_t sb_line = line & ~((1ull << DSB_OCC_SUPER_SHIFT) - 1);
				const uint8_t *sb_src = ix->bwt_occ + (sb_line * DSB_OCC_LINE_SYM / 256) * 168;
				uint64_t sp[4];
				memcpy(sp, sb_src, 32);
				if (line == sb_line)
					memcpy(ix->occ_super + (line >> DSB_OCC_SUPER_SHIFT) * 4, sp, 32);
				uint32_t rel[4];
				for (int c = 0; c < 4; c++)
					rel[c] = (uint32_t)(run[c] - sp[c]);
				memcpy(ln, rel, 16);
			}
			uint32_t nib = (uint32_t)((src[40 + (k >> 1)] >> ((k & 1) << 2)) & 0xf);
			if (nib < 4) {
				ln[2 + (kk >> 5)] |= (uint64_t)nib << (2 * (kk & 31));
				run[nib]++;
			} else {
				ln[6 + (kk >> 6)] |= 1ull << (kk & 63);
				if (nib == 5) {
					if (P->n_dollar >= DSB_MAX_DOLLAR) {
						snprintf(P->msg, sizeof(P->msg), "deSAMBA.bwt: more than %d '$' symbols (unsupported)", DSB_MAX_DOLLAR);
						P->bad = 1;
						break;
					}
					P->dollar[P->n_dollar++] = (b << 8) + k;
					dol++;
				}
			}
		}
		if (b + 1 < P->nb) { /* the next block's checkpoints continue this one's */
			uint64_t nx[5];
			memcpy(nx, ix->bwt_occ + (b + 1) * 168, 40);
			for (int c = 0; c < 4; c++)
				if (nx[c] != run[c]) {
					snprintf(P->msg, sizeof(P->msg), "deSAMBA.bwt: block %lu: checkpoint of symbol %d is %lu, %lu counted",
						 (unsigned long)(b + 1), c, (unsigned long)nx[c], (unsigned long)run[c]);
					P->bad = 1;
				}
			uint64_t nd = ((b + 1) << 8) - nx[0] - nx[1] - nx[2] - nx[3] - nx[4];
			if (!P->bad && nd != dol_before + dol) {
				snprintf(P->msg, sizeof(P->msg), "deSAMBA.bwt: block %lu: '#' checkpoint %lu implies %lu '$' before it, %lu counted",
					 (unsigned long)(b + 1), (unsigned long)nx[4], (unsigned long)nd, (unsigned long)(dol_before + dol));
				P->bad = 1;
			}
		} else { /* the line past the end (occ at r == n) */
			uint64_t nl = P->nb * (256 / DSB_OCC_LINE_SYM);
			uint64_t *ln = ix->occ + nl * DSB_OCC_LINE_U64;
			uint64_t sb_line = nl & ~((1ull << DSB_OCC_SUPER_SHIFT) - 1);
			uint64_t *sp = ix->occ_super + (nl >> DSB_OCC_SUPER_SHIFT) * 4;
			if (nl == sb_line)
				memcpy(sp, run, 32);
			uint32_t rel[4];
			for (int c = 0; c < 4; c++)
				rel[c] = (uint32_t)(run[c] - sp[c]);
			memcpy(ln, rel, 16);
		}
	}
	return NULL;
}

static int occ_relayout(dsb_index *ix, char *err, size_t errn)
{
	if (ix->byteLen % 168) {
		snprintf(err, errn, "deSAMBA.bwt: occ section of %lu bytes is not a whole number of 168-B blocks",
			 (unsigned long)ix->byteLen);
		return -1;
	}
	uint64_t nb = ix->byteLen / 168;          /* file blocks of 256 symbols */
	uint64_t nl = nb * (256 / DSB_OCC_LINE_SYM); /* HBM lines */
	ix->n_occ_line = nl;
	ix->occ = calloc((nl + 1) * DSB_OCC_LINE_U64, 8); /* + one line past the end (occ at r == n) */
	ix->n_occ_super = ((nl + 1) >> DSB_OCC_SUPER_SHIFT) + 1;
	ix->occ_super = calloc(ix->n_occ_super * 4, 8);
	if (!ix->occ || !ix->occ_super) {
		snprintf(err, errn, "deSAMBA.bwt: out of host memory for the occ re-layout");
		return -1;
	}
	ix->n_dollar = 0;
	if (nb == 0)
		return 0;
	/* whole superblocks per thread (2^16 blocks): the threads write disjoint lines */
	const uint64_t sb_blocks = (1ull << DSB_OCC_SUPER_SHIFT) * DSB_OCC_LINE_SYM / 256;
	uint64_t n_sb = (nb + sb_blocks - 1) / sb_blocks;
	int nt = dsb_host_threads();
	if (nt > 64) nt = 64;
	if ((uint64_t)nt > n_sb) nt = (int)n_sb;
	if (nt < 1) nt = 1;
	relayout_part *P = calloc(nt, sizeof(relayout_part));
	pthread_t *th = calloc(nt, sizeof(pthread_t));
	for (int t = 0; t < nt; t++) {
		P[t].ix = ix;
		P[t].nb = nb;
		P[t].b0 = n_sb * t / nt * sb_blocks;
		P[t].b1 = n_sb * (t + 1) / nt * sb_blocks;
		if (P[t].b1 > nb) P[t].b1 = nb;
	}
	int started[64] = {0};
	for (int t = 1; t < nt; t++)
		started[t] = pthread_create(&th[t], NULL, relayout_range, &P[t]) == 0;
	relayout_range(&P[0]);
	for (int t = 1; t < nt; t++) {
		if (started[t])
			pthread_join(th[t], NULL);
		else
			relayout_range(&P[t]);
	}
	int rc = 0;
	for (int t = 0; t < nt && !rc; t++)
		if (P[t].bad) {
			snprintf(err, errn, "%s", P[t].msg);
			rc = -1;
		}
	for (int t = 0; t < nt && !rc; t++)
		for (int d = 0; d < P[t].n_dollar; d++) {
			if (ix->n_dollar >= DSB_MAX_DOLLAR) {
				snprintf(err, errn, "deSAMBA.bwt: more than %d '$' symbols (unsupported)", DSB_MAX_DOLLAR);
				rc = -1;
				break;
			}
			ix->dollar_row[ix->n_dollar++] = P[t].dollar[d];
		}
	free(P);
	free(th);
	return rc;
}

/* .bwt: u64 byteLen | occ blocks | u64 rank[5] | u64 hash_index[2^26+1] (reference load_bwt,
 * src/bwt.c:68-85), the occ blocks re-laid out for HBM; with_hash 0 skips the 13-mer table */
int dsb_index_load_bwt(dsb_index *ix, const char *dir, int with_hash, char *err, size_t errn)
{
	FILE *f;
	if (!(f = open_ix(dir, ".bwt", err, errn))) return -1;
	if (rd(f, &ix->byteLen, 8, 1, "bwt len", err, errn)) goto fail;
	if (ix->byteLen / 168 >= (1ull << 32)) { /* 256 rows per 168-B block: rows < 2^40 (the seeding's packed sp_set slots) */
		snprintf(err, errn, "BWT of %llu bytes: more than 2^40 rows", (unsigned long long)ix->byteLen);
		goto fail;
	}
	ix->bwt_occ = xm(ix->byteLen + 256); /* slack: occ may touch the u16 after a block */
	memset(ix->bwt_occ + ix->byteLen, 0xFF, 256);
	if (rd(f, ix->bwt_occ, 1, ix->byteLen, "bwt occ", err, errn)) goto fail;
	if (rd(f, ix->rank, 8, 5, "rank", err, errn)) goto fail;
	ix->rank[5] = ix->rank[0] - 1;
	if (occ_relayout(ix, err, errn)) goto fail;
	free(ix->bwt_occ);
	ix->bwt_occ = NULL;
	if (with_hash) {
		uint64_t n = (1ull << (DSB_L_PRE_IDX << 1)) + 1;
		ix->hash_index = xm(n * 8);
		if (rd(f, ix->hash_index, 8, n, "hash_index", err, errn)) goto fail;
	}
	fclose(f);
	return 0;
fail:
	fclose(f);
	return -1;
}

int dsb_index_load_files(dsb_index *ix, const char *dir, char *err, size_t errn)
{
	FILE *f;
	if (dsb_index_load_bwt(ix, dir, 1, err, errn)) return -1;
	/* ---- .sa: u64 n | SA_taxon[n] */
	if (!(f = open_ix(dir, ".sa", err, errn))) return -1;
	if (rd(f, &ix->sa_size, 8, 1, "sa n", err, errn)) goto fail;
	ix->sa = xm(ix->sa_size * sizeof(dsb_sa_t));
	if (rd(f, ix->sa, sizeof(dsb_sa_t), ix->sa_size, "sa", err, errn)) goto fail;
	fclose(f);
	/* ---- e-kmer tables */
	if (!(f = open_ix(dir, ".exki", err, errn))) return -1;
	if (rd(f, &ix->ek_size, 8, 1, "exki", err, errn)) goto fail;
	fclose(f);
	set_ekmer_par(ix);
	if (!(f = open_ix(dir, ".exk0", err, errn))) return -1;
	ix->ek0 = xm(ix->ek_size);
	if (rd(f, ix->ek0, 1, ix->ek_size, "exk0", err, errn)) goto fail;
	fclose(f);
	if (!(f = open_ix(dir, ".exk1", err, errn))) return -1;
	ix->ek1 = xm(ix->ek_size);
	if (rd(f, ix->ek1, 1, ix->ek_size, "exk1", err, errn)) goto fail;
	fclose(f);
	/* ---- unitigs + sentinel (idx.c:1123-1129).  The reference sets only the sentinel's
	 * ref_list; its length is uninitialised heap (MALLOC_PERTURB: 0x5A5A5A5A) and the entry
	 * after it is the next heap chunk's header.  A backward LF walk that wraps through '$'
	 * lands on the last unitig and get_uni walks forward onto the sentinel (src/cly.c:476-480):
	 * the hermetic reference then maps nothing there, the -t1 build (zeroed heap) walks off the
	 * array and crashes.  Modelled as {formula, 0x5A5A5A5A}, {0, 0} (unpinned). */
	if (!(f = open_ix(dir, ".unv", err, errn))) return -1;
	if (rd(f, &ix->n_uni, 8, 1, "unv n", err, errn)) goto fail;
	ix->uni = xm((ix->n_uni + 2) * sizeof(dsb_unitig_t));
	if (rd(f, ix->uni, sizeof(dsb_unitig_t), ix->n_uni, "unv", err, errn)) goto fail;
	if (ix->n_uni > 0)
		ix->uni[ix->n_uni].ref_list = ix->uni[ix->n_uni - 1].ref_list + 1 + ix->uni[ix->n_uni - 1].length;
	else
		ix->uni[0].ref_list = 0;
	ix->uni[ix->n_uni].length = 0x5A5A5A5Au;
	ix->uni[ix->n_uni + 1].ref_list = 0;
	ix->uni[ix->n_uni + 1].length = 0;
	ix->dollor_pos = ix->n_uni - 1 - 1;
	fclose(f);
	/* ---- packed reference */
	if (!(f = open_ix(dir, ".ref_b", err, errn))) return -1;
	if (rd(f, &ix->ref_bin_n, 8, 1, "ref_b n", err, errn)) goto fail;
	ix->ref_bin_padded = ix->ref_bin_n + REF_BIN_PAD;
	ix->ref_bin = xm(ix->ref_bin_padded);
	memset(ix->ref_bin + ix->ref_bin_n, 0, REF_BIN_PAD);
	if (rd(f, ix->ref_bin, 1, ix->ref_bin_n, "ref_b", err, errn)) goto fail;
	fclose(f);
	/* ---- REF_INFO {char name[128]; u64 seq_l; u64 seq_offset} */
	if (!(f = open_ix(dir, ".ref_i", err, errn))) return -1;
	if (rd(f, &ix->n_ref, 8, 1, "ref_i n", err, errn)) goto fail;
	ix->ref_name = xm(ix->n_ref * 128);
	ix->ref_seq_l = xm(ix->n_ref * 8);
	ix->ref_seq_offset = xm(ix->n_ref * 8);
	for (uint64_t i = 0; i < ix->n_ref; i++) {
		struct { char name[128]; uint64_t l, off; } r;
		if (rd(f, &r, sizeof(r), 1, "ref_i", err, errn)) goto fail;
		memcpy(ix->ref_name[i], r.name, 128);
		ix->ref_seq_l[i] = r.l;
		ix->ref_seq_offset[i] = r.off;
	}
	fclose(f);
	/* ---- REF_POS */
	if (!(f = open_ix(dir, ".ref_p", err, errn))) return -1;
	if (rd(f, &ix->n_rp, 8, 1, "ref_p n", err, errn)) goto fail;
	ix->r_p = xm((ix->n_rp + 64) * 8); /* zero tail: reads one or two past the end (sentinel unitig) */
	if (rd(f, ix->r_p, 8, ix->n_rp, "ref_p", err, errn)) goto fail;
	memset(ix->r_p + ix->n_rp, 0, 64 * 8);
	fclose(f);
	return 0;
fail:
	fclose(f);
	return -1;
}

/* calculate_MAPQ_TABLE, src/cly_mt.c:396-420 — the only floating point on the path,
 * evaluated once on the host exactly as the reference does (double, truncation). */
void dsb_mapq_tables(dsb_index *ix, double P_E, uint64_t L_REF)
{
	double REF_SIZE_PUNALTY = -10 * log(L_REF) / log(10);
	double MATCH_SCORE = -10 * log(0.25 / (1 - P_E)) / log(10);
	double MISMATCH_PUNALTY = -10 * log(0.75 / (P_E)) / log(10);
	if (!ix->Q_MEM)
		ix->Q_MEM = xm(sizeof(int) * DSB_Q_MEM_PAD);
	for (int i = 0; i < DSB_Q_MEM_MAX; i++)
		ix->Q_MEM[i] = REF_SIZE_PUNALTY + i * MATCH_SCORE + 0.5;
	/* Entries past Q_MEM_MAX are an out-of-bounds heap read in the reference (match
	 * length >= 2000); they are unpinned — extend the linear formula. */
	for (int i = DSB_Q_MEM_MAX; i < DSB_Q_MEM_PAD; i++)
		ix->Q_MEM[i] = REF_SIZE_PUNALTY + i * MATCH_SCORE + 0.5;
	for (int j = 0; j < DSB_LV_DIM; j++)
		for (int i = 0; i < DSB_LV_DIM; i++) {
			int v = (j - i) * MATCH_SCORE + i * MISMATCH_PUNALTY + 0.5;
			if (j < 5)
				v += 15;
			if (v < -8)
				v = -8;
			ix->Q_LV[i * DSB_LV_DIM + j] = v;
		}
}

/* taxonTree_rank, src/cly_mt.c:590-670 */
int dsb_taxonomy_load(dsb_index *ix, const char *dir, char *err, size_t errn)
{
	char buf[4096];
	snprintf(buf, sizeof(buf), "%s/nodes.dmp", dir);
	FILE *fp = fopen(buf, "r");
	if (!fp) { snprintf(err, errn, "cannot open %s", buf); return -1; }
	char *line = NULL;
	size_t max_l = 0;
	uint32_t max_tid = 0;
	while (getline(&line, &max_l, fp) > 0) {
		char *tok = strtok(line, "\t|");
		max_tid = strtoul(tok, NULL, 10);
	}
	rewind(fp);
	max_tid += 1000000;
	ix->max_tid = max_tid;
	ix->tax = malloc(sizeof(dsb_taxon_t) * ((uint64_t)max_tid + 1));
	if (!ix->tax) { fclose(fp); snprintf(err, errn, "taxonomy: out of memory"); return -1; }
	for (uint64_t i = 0; i <= max_tid; i++) {
		ix->tax[i].p_tid = 0xffffffffu;
		ix->tax[i].name[0] = '\0';
		ix->tax[i].rank[0] = '\0';
	}
	while (getline(&line, &max_l, fp) > 0) {
		char *tok = strtok(line, "\t|");
		uint32_t tid = strtoul(tok, NULL, 10);
		tok = strtok(NULL, "\t|");
		if (tid <= max_tid) {
			ix->tax[tid].p_tid = strtoul(tok, NULL, 10);
			tok = strtok(NULL, "\t|");
			if (tok) {
				strncpy(ix->tax[tid].rank, tok, sizeof(ix->tax[tid].rank) - 1);
				ix->tax[tid].rank[sizeof(ix->tax[tid].rank) - 1] = 0;
			}
		}
	}
	fclose(fp);
	ix->tax[1].p_tid = 0xffffffffu;
	ix->tax[0].p_tid = 0xffffffffu;
	strcpy(ix->tax[0].rank, "no rank");
	strcpy(ix->tax[0].name, "CLY_FAIL");
	snprintf(buf, sizeof(buf), "%s/names.dmp", dir);
	fp = fopen(buf, "r");
	if (!fp) { free(line); snprintf(err, errn, "cannot open %s", buf); return -1; }
	while (getline(&line, &max_l, fp) > 0) {
		char *tok = strtok(line, "|\t");
		uint32_t tid = strtoul(tok, NULL, 10);
		char *name = strtok(NULL, "\t|");
		tok = strtok(NULL, "|");
		tok = strtok(NULL, "|");
		if (tok && strncmp("\tscien", tok, 6) == 0 && tid <= max_tid && name) {
			strncpy(ix->tax[tid].name, name, 200);
			ix->tax[tid].name[200] = 0;
		}
	}
	fclose(fp);
	free(line);
	return 0;
}

void dsb_index_free_host_tables(dsb_index *ix)
{
	free(ix->bwt_occ); ix->bwt_occ = NULL;
	free(ix->occ); ix->occ = NULL;
	free(ix->occ_super); ix->occ_super = NULL;
	free(ix->hash_index); ix->hash_index = NULL;
	free(ix->sa); ix->sa = NULL;
	free(ix->ek0); ix->ek0 = NULL;
	free(ix->ek1); ix->ek1 = NULL;
	free(ix->uni); ix->uni = NULL;
	free(ix->ref_bin); ix->ref_bin = NULL;
	free(ix->r_p); ix->r_p = NULL;
}

void dsb_index_host_view(const dsb_index *ix, dsb_dindex_t *d)
{
	memset(d, 0, sizeof(*d));
	d->occ = ix->occ; d->n_occ_line = ix->n_occ_line;
	d->occ_super = ix->occ_super;
	memcpy(d->dollar_row, ix->dollar_row, sizeof(d->dollar_row)); d->n_dollar = ix->n_dollar;
	memcpy(d->rank, ix->rank, sizeof(d->rank));
	d->hash_index = ix->hash_index;
	d->sa = ix->sa; d->sa_size = ix->sa_size; d->dollor_pos = ix->dollor_pos;
	d->ek0 = ix->ek0; d->ek1 = ix->ek1; d->ek_size = ix->ek_size; d->ek_mask = ix->ek_mask;
	d->l_ek = ix->l_ek; d->single_base_max = ix->single_base_max;
	d->uni = ix->uni; d->n_uni = ix->n_uni;
	d->ref_bin = ix->ref_bin; d->ref_bin_n = ix->ref_bin_n; d->ref_bin_padded = ix->ref_bin_padded;
	d->ref_seq_offset = ix->ref_seq_offset; d->ref_seq_l = ix->ref_seq_l; d->n_ref = ix->n_ref;
	d->r_p = ix->r_p; d->n_rp = ix->n_rp;
	d->Q_MEM = ix->Q_MEM; d->Q_LV = ix->Q_LV;
	d->filter_min_length = ix->filter_min_length;
	d->filter_min_score = ix->filter_min_score;
	d->filter_min_score_LV3 = ix->filter_min_score_LV3;
	d->ref_tid = ix->ref_tid; d->p_tid = ix->p_tid; d->max_tid = ix->max_tid;
}
