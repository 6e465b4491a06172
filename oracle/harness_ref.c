/*
 * oracle/harness_ref.c — TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * A driver around the *reference's own compiled objects* (built from
 * /root/reference/src by oracle/Makefile).  It re-expresses the control flow of
 * classify_seq (reference src/cly.c:3059-3127) by calling the reference's exported
 * stage functions, so that per-stage intermediate results can be dumped, and
 * prints SAM_FULL records with the reference's own output_one_result_sam
 * (src/cly_mt.c:229-327).
 *
 * Modes
 *   default      one shared buffer pool for all reads, in input order
 *                == `deSAMBA classify -t 1 -f SAM_FULL` (byte-identical)
 *   --fresh      a fresh Classify_buff_pool + fresh cly_r per read (the "hermetic"
 *                oracle of SURVEY §8c T3) with buff->max_read_l carried read to read
 *                exactly as the -t1 pool carries it (src/cly.c:2953 only updates it
 *                for reads that reach delete_small_score_rst with hits).
 *   --perturb    mallopt(M_PERTURB, 165): fresh heap bytes read as 0x5A
 *                (default on in the herm_classify build).
 *   --dump F     per-read stage dump (seeds, anchors, chains) to file F.
 *   --max-read-l N  initial max_read_l carried into the first read.
 *   --sam        SAM instead of SAM_FULL (SEQ and QUAL printed as '*').
 *   --des        DES records (the reference's output_one_result_des, src/cly_mt.c:144-185).
 *   --des-full   DES_FULL records (output_one_result_full, src/cly_mt.c:187-227).
 *
 * usage: ref_classify [opts] <index_dir> <reads.fq>
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include <malloc.h>
#include <zlib.h>
#include "cly.h"
#include "idx.h"
#include "lib/utils.h"

#ifndef HERMETIC_DEFAULT
#define HERMETIC_DEFAULT 0
#endif

/* Same layout as the file-local SEARCH_DIR of src/cly.c:941-949. */
typedef struct {
	CLY_seed *seed_v_f;
	uint32_t l_seed_v_f;
	uint8_t *bin_read;
	uint64_t *kmer;
	uint32_t direction;
	uint32_t total_score;
} H_SEARCH_DIR;

/* reference stage entry points (non-static in src/cly.c / src/cly_mt.c) */
void getIsland(kseq_t *read, Classify_buff_pool *buff, E_KMER *ek, H_SEARCH_DIR *search_dir);
int fast_classify(DA_IDX *idx, H_SEARCH_DIR *s_d, uint32_t read_len, cly_r *results);
void slow_classify(DA_IDX *idx, H_SEARCH_DIR *search_dir, uint32_t read_len, cly_r *results);
void resolve_tree(cly_r *results);
void delete_small_score_rst(DA_IDX *idx, cly_r *results, H_SEARCH_DIR *search_dir, Classify_buff_pool *buff);
void detect_primary(chain_item *hit, uint32_t n_hit, uint32_t read_len);
void calculate_MAPQ_TABLE(int *Q_MEM, int (*Q_LV)[MAX_LV_R_LEN], double P_E, uint64_t L_REF);
void output_one_result_sam(DA_IDX *idx, cly_r *p_rst, int output_seq, MAP_opt *o);
void output_one_result_des(DA_IDX *idx, cly_r *p_rst, MAP_opt *o);
void output_one_result_full(DA_IDX *idx, cly_r *p_rst, MAP_opt *o);

/* 0: SAM / SAM_FULL (with_seq), 1: DES, 2: DES_FULL */
static int g_des = 0;
static void output_one(DA_IDX *idx, cly_r *r, int with_seq, MAP_opt *o)
{
	if (g_des == 1)
		output_one_result_des(idx, r, o);
	else if (g_des == 2)
		output_one_result_full(idx, r, o);
	else
		output_one_result_sam(idx, r, with_seq, o);
}

static FILE *g_dump = NULL;

static void dump_seeds(H_SEARCH_DIR *sd)
{
	for (int s = 0; s < 2; s++) {
		fprintf(g_dump, "S %d %u %u %u\n", s, sd[s].direction, sd[s].l_seed_v_f, sd[s].total_score);
		for (uint32_t i = 0; i < sd[s].l_seed_v_f; i++)
			fprintf(g_dump, "s %u %u %u\n", sd[s].seed_v_f[i].offset, sd[s].seed_v_f[i].len,
				(unsigned)sd[s].seed_v_f[i].top);
	}
}

static void dump_anchors(const char *tag, cly_r *r)
{
	fprintf(g_dump, "A %s %lu\n", tag, (unsigned long)r->anchor_v.n);
	for (uint64_t i = 0; i < r->anchor_v.n; i++) {
		Anchor *a = r->anchor_v.a + i;
		fprintf(g_dump, "a %u %u %u %u %lu %u %d %u %u %u %u %u %u %u\n",
			(unsigned)a->direction, a->ref_ID, a->ref_offset, a->index_in_read,
			(unsigned long)a->global_offset, (unsigned)a->a_m.mtch_len, (int)a->a_m.score,
			(unsigned)a->a_m.left_len, (unsigned)a->a_m.left_ED, (unsigned)a->a_m.rigt_len,
			(unsigned)a->a_m.rigt_ED, (unsigned)a->seed_ID, (unsigned)a->anchor_useless,
			(unsigned)a->duplicate);
	}
}

static void dump_hits(const char *tag, cly_r *r, int with_primary)
{
	fprintf(g_dump, "H %s %lu\n", tag, (unsigned long)r->hit.n);
	for (uint64_t i = 0; i < r->hit.n; i++) {
		chain_item *c = r->hit.a + i;
		fprintf(g_dump, "h %u %u %d %u %u %u %u %u %u %u %u",
			c->ref_ID, (unsigned)c->direction, c->q_t_dis, c->sum_score, c->anchor_number,
			(unsigned)c->with_top_anchor, c->t_st, c->t_ed, c->q_st, c->q_ed, c->indel);
		if (with_primary)
			fprintf(g_dump, " %u %u", (unsigned)c->primary, (unsigned)c->pri_index);
		fputc('\n', g_dump);
	}
}

/* Re-expression of classify_seq (src/cly.c:3059-3127) with stage dumps. */
#define H_MIN_READ_LEN 40 /* src/cly.c:3058 */
static void classify_one(kseq_t *read, DA_IDX *idx, cly_r *results, Classify_buff_pool *buff)
{
	H_SEARCH_DIR search_dir[2];
	uint32_t read_len = read->seq.l;
	results->anchor_v.n = 0;
	results->read = read;
	results->fast_classify = true;
	results->hit.n = 0;
	if (read_len < H_MIN_READ_LEN)
		return;
	getIsland(read, buff, &(idx->ek), search_dir);
	if (g_dump) dump_seeds(search_dir);
	int both_direction = ((search_dir[0].total_score - search_dir[1].total_score) <= (search_dir[0].total_score >> 3));
	int super_repeat = fast_classify(idx, search_dir, read_len, results);
	if (both_direction)
		super_repeat += fast_classify(idx, search_dir + 1, read_len, results);
	if (g_dump) dump_anchors("fast", results);
	resolve_tree(results);
	if (g_dump) dump_hits("fast", results, 0);
	int run_slow_mode = 0;
	if (results->hit.n <= 0)
		run_slow_mode = 1;
	else if (results->hit.a[0].anchor_number < 5 && super_repeat < 3) {
		run_slow_mode = 1;
		if (read_len <= 300 && results->hit.a[0].sum_score > 200)
			run_slow_mode = 0;
	}
	if (run_slow_mode) {
		results->anchor_v.n = 0;
		slow_classify(idx, search_dir, read_len, results);
		if (g_dump) dump_anchors("slow1", results);
		resolve_tree(results);
		if (g_dump) dump_hits("slow1", results, 0);
		if (both_direction || results->hit.n <= 0 || (results->hit.a[0].anchor_number < 5 && super_repeat < 3)) {
			slow_classify(idx, search_dir + 1, read_len, results);
			if (g_dump) dump_anchors("slow2", results);
			resolve_tree(results);
			if (g_dump) dump_hits("slow2", results, 0);
		}
	}
	delete_small_score_rst(idx, results, search_dir, buff);
	detect_primary(results->hit.a, results->hit.n, read_len);
	if (g_dump) dump_hits("final", results, 1);
}

static void pool_init(Classify_buff_pool *b)
{
	memset(b, 0, sizeof(*b));
	b->sa_hash[0] = malloc(sizeof(sparse_align_HASH) * 0x100000); /* src/cly_mt.c:537-538 */
	b->sa_hash[1] = malloc(sizeof(sparse_align_HASH) * 0x100000);
}

static void pool_free(Classify_buff_pool *b)
{
	free(b->bin_read); free(b->kmer_buff); free(b->seed_v); free(b->sp_table);
	free(b->sp_hash); free(b->sa_hash[0]); free(b->sa_hash[1]); free(b->sc_hash);
	free(b->sms.a);
}

int main(int argc, char **argv)
{
	int fresh = HERMETIC_DEFAULT, perturb = HERMETIC_DEFAULT;
	int max_read_l = 0, with_seq = 1;
	const char *dump_path = NULL;
	int ai = 1;
	for (; ai < argc && argv[ai][0] == '-' && argv[ai][1] == '-'; ai++) {
		if (!strcmp(argv[ai], "--fresh")) fresh = 1;
		else if (!strcmp(argv[ai], "--shared")) fresh = 0;
		else if (!strcmp(argv[ai], "--perturb")) perturb = 1;
		else if (!strcmp(argv[ai], "--no-perturb")) perturb = 0;
		else if (!strcmp(argv[ai], "--dump") && ai + 1 < argc) dump_path = argv[++ai];
		else if (!strcmp(argv[ai], "--max-read-l") && ai + 1 < argc) max_read_l = atoi(argv[++ai]);
		else if (!strcmp(argv[ai], "--sam")) with_seq = 0; /* SAM: SEQ/QUAL printed as '*' */
		else if (!strcmp(argv[ai], "--des")) g_des = 1;
		else if (!strcmp(argv[ai], "--des-full")) g_des = 2;
		else { fprintf(stderr, "unknown option %s\n", argv[ai]); return 2; }
	}
	if (ai + 2 > argc) {
		fprintf(stderr, "usage: %s [--fresh|--shared] [--perturb] [--dump F] [--max-read-l N] <index_dir> <reads>\n", argv[0]);
		return 2;
	}
	if (perturb)
		mallopt(M_PERTURB, 165);
	if (dump_path) {
		g_dump = fopen(dump_path, "w");
		if (!g_dump) { perror(dump_path); return 1; }
	}
	DA_IDX *idx = calloc(1, sizeof(DA_IDX));
	load_idx(idx, argv[ai]);
	/* fixed .so parameters, src/cly_mt.c:1257-1262 */
	idx->filter_min_length = 170;
	idx->filter_min_score = 64;
	idx->filter_min_score_LV3 = 64 + 10;
	idx->mapQ.Q_MEM = malloc(sizeof(int) * Q_MEM_MAX);
	idx->mapQ.Q_LV = (int(*)[MAX_LV_R_LEN])malloc(MAX_LV_WRONG * MAX_LV_R_LEN * sizeof(int));
	calculate_MAPQ_TABLE(idx->mapQ.Q_MEM, idx->mapQ.Q_LV, 0.15, idx->ref_bin.n * 4);

	MAP_opt o = {170, 1, 5, 2 /*SAM_FULL*/, 0, stdout, 64};
	gzFile fp = gzopen(argv[ai + 1], "r");
	if (!fp) { perror(argv[ai + 1]); return 1; }
	kstream_t *ks = ks_init(fp);
	/* The CLI/.so read batches through kt_pipeline (src/cly_mt.c:361-381, src/lib/kthread.c:
	 * 114-197): batch k is parsed by pipeline worker (k mod 3) into that worker's own array of
	 * N_NEEDED kseq_t slots (src/cly_mt.c:29-43, 544); each slot keeps its own last_char, a
	 * batch ends after 5000 reads, once 10 Mbp are read, or at the first kseq_read() < 0, and a
	 * worker whose batch is empty leaves the pipeline.  Reproduced here so that the harness
	 * sees exactly the reads the CLI sees. */
	enum { NW = 3, NSLOT = 5000 };
	const long MAXSZ = 10000000;
	kseq_t *slots[NW];
	for (int w = 0; w < NW; w++) slots[w] = calloc(NSLOT, sizeof(kseq_t));
	int64_t widx[NW] = {0, 1, 2};
	int alive[NW] = {1, 1, 1};
	int64_t next_index = NW;
	Classify_buff_pool shared;
	pool_init(&shared);
	cly_r shared_r[NSLOT];
	memset(shared_r, 0, sizeof(shared_r));
	shared.max_read_l = max_read_l;
	uint64_t n = 0;
	for (;;) {
		int w = -1;
		for (int k = 0; k < NW; k++)
			if (alive[k] && (w < 0 || widx[k] < widx[w])) w = k;
		if (w < 0) break;
		long nb = 0, total = 0;
		for (; nb < NSLOT && total < MAXSZ; nb++) {
			slots[w][nb].f = ks;
			if (kseq_read(slots[w] + nb) < 0) break;
			total += slots[w][nb].seq.l;
		}
		if (nb == 0) { alive[w] = 0; continue; }
		for (long i = 0; i < nb; i++) {
			kseq_t *seq = slots[w] + i;
			if (g_dump) fprintf(g_dump, "R %lu %s %lu\n", (unsigned long)n, seq->name.s, (unsigned long)seq->seq.l);
			if (fresh) {
				Classify_buff_pool b;
				cly_r r;
				pool_init(&b);
				memset(&r, 0, sizeof(r));
				b.max_read_l = max_read_l;
				classify_one(seq, idx, &r, &b);
				max_read_l = b.max_read_l;
				output_one(idx, &r, with_seq, &o);
				free(r.hit.a); free(r.anchor_v.a);
				pool_free(&b);
			} else {
				classify_one(seq, idx, shared_r + i, &shared);
				output_one(idx, shared_r + i, with_seq, &o);
			}
			n++;
		}
		widx[w] = next_index++;
	}
	if (g_dump) { fprintf(g_dump, "max_read_l %d\n", fresh ? max_read_l : shared.max_read_l); fclose(g_dump); }
	fflush(stdout);
	return 0;
}
