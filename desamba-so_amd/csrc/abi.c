/*
 * abi.c — the drop-in C-ABI of desamba.h (reference /root/reference/desamba.h:10,23,45),
 * backed by the MI355X classify kernels.
 *
 *   load_index     reference src/cly_mt.c:1238-1274
 *   read_classify  reference src/cly_mt.c:1309-1316 (+ read_classify_core :1041-1081)
 *   meta_analysis  reference src/cly_mt.c:1329-1414
 *
 * Semantics kept from the reference: fixed filters 170/64/74, P_E 0.15, L_REF = 4*ref_b.n,
 * SAM_FULL records with no header, malloc'd zero-filled output of out_n+1 bytes that the
 * caller frees with free(), input_n == (uint64_t)-1 meaning "input is a path", input_n == 0
 * leaving *output untouched, per-thread_id state (the carried max_read_l, reset when the
 * thread_num of a thread_id changes, :1287-1295).  Fatal errors print and exit(1) like
 * the reference's err_fatal (src/lib/utils.c:144-177).  Results are those of a single
 * buffer pool in input order (the reference's -t 1 order).
 */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include "dsb_host.h"
#include "gpu/dsb_gpu.h"
#include "../../include/desamba.h"
#include "../../include/desamba_mi355x.h"
_Static_assert(sizeof(((dsb_timing_t *)0)->stats) == sizeof(((dsb_gpu_timing *)0)->stats), "ABI timing.stats mirrors dsb_gpu_timing.stats");

struct dsb_thread_state {
	int thread_id;
	int thread_num;
	int max_read_l;
	struct dsb_thread_state *next;
};

static void fatal(const char *func, const char *msg)
{
	fprintf(stderr, "[%s] %s Abort!\n", func, msg);
	exit(1);
}

/* taxid of "tid|<taxid>|..." reference names (getOneSAM, src/cly_mt.c:778-786) */
static uint32_t name_taxid(const char *name)
{
	const char *p = strchr(name, '|');
	return p ? (uint32_t)strtoul(p + 1, NULL, 10) : 0;
}

void load_index(void **idx, const char *dirPath)
{
	char err[1024];
	dsb_index *ix = calloc(1, sizeof(dsb_index));
	if (!ix) fatal("load_index", "out of memory");
	if (dsb_index_load_files(ix, dirPath, err, sizeof(err))) fatal("load_index", err);
	ix->filter_min_length = 170;
	ix->filter_min_score = 64;
	ix->filter_min_score_LV3 = 64 + 10;
	dsb_mapq_tables(ix, 0.15, ix->ref_bin_n * 4);
	if (dsb_taxonomy_load(ix, dirPath, err, sizeof(err))) fatal("load_index", err);
	ix->ref_tid = malloc(sizeof(uint32_t) * (ix->n_ref + 1));
	for (uint64_t r = 0; r < ix->n_ref; r++)
		ix->ref_tid[r] = name_taxid(ix->ref_name[r]);
	ix->p_tid = malloc(sizeof(uint32_t) * (ix->max_tid + 1));
	for (uint64_t t = 0; t <= ix->max_tid; t++)
		ix->p_tid[t] = ix->tax[t].p_tid;
	if (dsb_gpu_init(ix, -1, err, sizeof(err))) fatal("load_index", err);
	if (!getenv("DSB_KEEP_HOST_TABLES"))
		dsb_index_free_host_tables(ix);
	pthread_mutex_init(&ix->state_mutex, NULL);
	ix->states = NULL;
	*idx = ix;
}

static struct dsb_thread_state *thread_state(dsb_index *ix, int thread_id, int thread_num)
{
	pthread_mutex_lock(&ix->state_mutex);
	struct dsb_thread_state *s = ix->states;
	for (; s; s = s->next)
		if (s->thread_id == thread_id) break;
	if (s && thread_num != -1 && s->thread_num != thread_num) {
		s->thread_num = thread_num; /* the reference frees and re-creates the pools */
		s->max_read_l = 0;
	}
	if (!s) {
		s = calloc(1, sizeof(*s));
		s->thread_id = thread_id;
		s->thread_num = thread_num;
		s->max_read_l = 0;
		s->next = ix->states;
		ix->states = s;
	}
	pthread_mutex_unlock(&ix->state_mutex);
	return s;
}

int dsb_classify_text(void *idx, const char *text, uint64_t text_n, int format, int *max_read_l, char **output,
		      uint64_t *output_n, dsb_timing_t *timing)
{
	dsb_index *ix = idx;
	char err[1024];
	dsb_reads_t reads;
	memset(&reads, 0, sizeof(reads));
	dsb_parse_reads(text, text_n, &reads);
	dsb_read_out_t *ro = calloc(reads.n + 1, sizeof(dsb_read_out_t));
	dsb_hit_out_t *hits = NULL;
	uint64_t n_hits = 0;
	dsb_gpu_timing gt;
	memset(&gt, 0, sizeof(gt));
	if (dsb_gpu_classify(ix, &reads, max_read_l, ro, &hits, &n_hits, timing ? timing->stats_on : 0, &gt, err,
			     sizeof(err))) {
		fprintf(stderr, "[read_classify] %s\n", err);
		free(ro);
		free(hits);
		dsb_reads_free(&reads);
		return -1;
	}
	dsb_str out = {0, 0, 0};
	for (uint64_t i = 0; i < reads.n; i++)
		dsb_format_read(&out, ix, &reads, i, ro + i, hits + ro[i].hit_off, format, 5);
	*output_n = out.l;
	*output = malloc(out.l + 1);
	memset(*output, 0, out.l + 1);
	if (out.l) memcpy(*output, out.s, out.l);
	free(out.s);
	if (timing) {
		int st = timing->stats_on;
		memset(timing, 0, sizeof(*timing));
		timing->stats_on = st;
		timing->ms_total = gt.ms_total;
		timing->ms_h2d = gt.ms_h2d;
		timing->ms_d2h = gt.ms_d2h;
		timing->ms_encode = gt.ms_encode;
		timing->ms_seed = gt.ms_seed;
		timing->ms_classA = gt.ms_classA;
		timing->ms_classB = gt.ms_classB;
		for (int k = 0; k < 12; k++) timing->ms_phase[k] = gt.ms_phase[k];
		timing->n_reads = gt.n_reads;
		timing->n_bases = gt.n_bases;
		timing->n_retry = gt.n_retry;
		timing->n_chunks = gt.n_chunks;
		timing->seed_positions = gt.seed_positions;
		timing->n_launch_dela = gt.n_launch_dela;
		timing->n_launch_phase = (int)gt.n_launch_phase;
		for (int k = 0; k < DSB_N_STATS; k++) timing->stats[k] = gt.stats[k];
	}
	free(ro);
	free(hits);
	dsb_reads_free(&reads);
	return 0;
}

void read_classify(void *idx, char *input, uint64_t input_n, char **output, uint64_t *output_n, int thread_id,
		   int thread_num)
{
	if (input_n == 0) {
		*output_n = 0;
		return;
	}
	dsb_index *ix = idx;
	struct dsb_thread_state *st = thread_state(ix, thread_id, thread_num);
	char *buf = NULL;
	uint64_t len = 0;
	int owned = 0;
	if (input_n == (uint64_t)-1) {
		if (dsb_slurp_path(input, &buf, &len)) {
			char msg[4200];
			snprintf(msg, sizeof(msg), "fail to open file '%s' : No such file or directory", input);
			fatal("read_classify", msg);
		}
		owned = 1;
	} else if (dsb_inflate_if_gzip(input, input_n, &buf, &len, &owned)) {
		fatal("read_classify", "cannot decompress input");
	}
	int mrl = st->max_read_l;
	if (dsb_classify_text(ix, buf, len, DSB_OUT_SAM_FULL, &mrl, output, output_n, NULL))
		fatal("read_classify", "GPU classify failed");
	st->max_read_l = mrl;
	if (owned) free(buf);
}

void meta_analysis(void *idx, char *input, uint64_t input_n, char **output, uint64_t *output_n, int thread_id,
		   int flag, uint64_t max_snapshot_len, char **human_snapshot, uint64_t *human_snapshot_n)
{
	if (input_n == 0) {
		*output_n = 0;
		*human_snapshot_n = 0;
		return;
	}
	dsb_index *ix = idx;
	thread_state(ix, thread_id, -1);
	dsb_meta_analysis(ix, input, input_n, output, output_n, flag, max_snapshot_len, human_snapshot, human_snapshot_n);
}

/* ------------------------------------------------------------------ batch API */
struct dsb_batch {
	dsb_reads_t reads;
	dsb_gpu_batch *g;
};

static void copy_timing(dsb_timing_t *t, const dsb_gpu_timing *gt)
{
	int st = t->stats_on;
	memset(t, 0, sizeof(*t));
	t->stats_on = st;
	t->ms_total = gt->ms_total;
	t->ms_h2d = gt->ms_h2d;
	t->ms_d2h = gt->ms_d2h;
	t->ms_encode = gt->ms_encode;
	t->ms_seed = gt->ms_seed;
	t->ms_classA = gt->ms_classA;
	t->ms_classB = gt->ms_classB;
	for (int k = 0; k < 12; k++) t->ms_phase[k] = gt->ms_phase[k];
	t->n_reads = gt->n_reads;
	t->n_bases = gt->n_bases;
	t->n_retry = gt->n_retry;
	t->n_chunks = gt->n_chunks;
	t->seed_positions = gt->seed_positions;
	t->n_launch_dela = gt->n_launch_dela;
	t->n_launch_phase = (int)gt->n_launch_phase;
	for (int k = 0; k < DSB_N_STATS; k++) t->stats[k] = gt->stats[k];
}

dsb_batch *dsb_batch_create(void *idx, const char *text, uint64_t text_n, dsb_timing_t *timing)
{
	char err[1024];
	dsb_batch *b = calloc(1, sizeof(*b));
	dsb_parse_reads(text, text_n, &b->reads);
	dsb_gpu_timing gt;
	memset(&gt, 0, sizeof(gt));
	if (dsb_gpu_batch_upload(idx, &b->reads, &b->g, &gt, err, sizeof(err))) {
		fprintf(stderr, "[dsb_batch_create] %s\n", err);
		dsb_reads_free(&b->reads);
		free(b);
		return NULL;
	}
	if (timing) copy_timing(timing, &gt);
	return b;
}

int dsb_batch_run(void *idx, dsb_batch *b, int *max_read_l, dsb_timing_t *timing)
{
	char err[1024];
	dsb_gpu_timing gt;
	memset(&gt, 0, sizeof(gt));
	int rc = dsb_gpu_batch_run(idx, b->g, max_read_l, timing ? timing->stats_on : 0, &gt, err, sizeof(err));
	if (rc) fprintf(stderr, "[dsb_batch_run] %s\n", err);
	if (timing) copy_timing(timing, &gt);
	return rc;
}

int dsb_batch_format(void *idx, dsb_batch *b, int format, char **output, uint64_t *output_n)
{
	return dsb_batch_format_range(idx, b, format, 0, b->reads.n, output, output_n);
}

int dsb_batch_format_range(void *idx, dsb_batch *b, int format, uint64_t lo, uint64_t hi, char **output,
			   uint64_t *output_n)
{
	const dsb_read_out_t *ro = dsb_gpu_batch_ro(b->g);
	const dsb_hit_out_t *hits = dsb_gpu_batch_hits(b->g);
	dsb_str out = {0, 0, 0};
	if (hi > b->reads.n) hi = b->reads.n;
	for (uint64_t i = lo; i < hi; i++)
		dsb_format_read(&out, idx, &b->reads, i, ro + i, hits + ro[i].hit_off, format, 5);
	*output_n = out.l;
	*output = calloc(out.l + 1, 1);
	if (out.l) memcpy(*output, out.s, out.l);
	free(out.s);
	return 0;
}

int dsb_batch_taxa(void *idx, dsb_batch *b, int flag, uint32_t *tid_out, uint64_t *weight_out)
{
	dsb_index *ix = idx;
	const dsb_read_out_t *ro = dsb_gpu_batch_ro(b->g);
	const dsb_hit_out_t *hits = dsb_gpu_batch_hits(b->g);
	for (uint64_t i = 0; i < b->reads.n; i++) {
		const dsb_rec_t *rec = b->reads.rec + i;
		/* the SAM text meta_analysis parses prints SEQ with %s: its length is strlen */
		weight_out[i] = (flag & 1) ? (uint64_t)strlen(b->reads.arena + rec->seq_off) : 1;
		tid_out[i] = dsb_read_taxon(hits + ro[i].hit_off, ro[i].n_hit, ix->ref_tid, ix->p_tid, ix->max_tid);
	}
	return 0;
}

int dsb_batch_taxon_counts(void *idx, dsb_batch *b, int flag, uint64_t *dev_counts, uint64_t n_counts)
{
	dsb_index *ix = idx;
	char err[512];
	if (n_counts < ix->max_tid + 1)
		return -1;
	uint32_t *w = NULL;
	if (flag & 1) { /* strlen of each SEQ, as meta_analysis' parse of the SAM text sees it */
		w = malloc(sizeof(uint32_t) * (b->reads.n + 1));
		for (uint64_t i = 0; i < b->reads.n; i++)
			w[i] = (uint32_t)strlen(b->reads.arena + b->reads.rec[i].seq_off);
	}
	int rc = dsb_gpu_batch_counts(ix, b->g, w, dev_counts, n_counts, err, sizeof(err));
	free(w);
	if (rc)
		fprintf(stderr, "[dsb] dsb_batch_taxon_counts: %s\n", err);
	return rc;
}

int dsb_batch_carry(dsb_batch *b, int32_t *carry_out)
{
	const int32_t *c = dsb_gpu_batch_carry(b->g);
	for (uint64_t i = 0; i < b->reads.n; i++)
		carry_out[i] = c ? c[i] : 0;
	return 0;
}

uint64_t dsb_batch_reads(dsb_batch *b) { return b->reads.n; }
uint64_t dsb_batch_bases(dsb_batch *b) { return dsb_gpu_batch_bases(b->g); }
uint64_t dsb_max_tid(void *idx) { return ((dsb_index *)idx)->max_tid; }

void dsb_batch_free(void *idx, dsb_batch *b)
{
	if (!b) return;
	dsb_gpu_batch_free(idx, b->g);
	dsb_reads_free(&b->reads);
	free(b);
}

/* ------------------------------------------------------------------ extensions */
const char *dsb_version(void)
{
	return "desamba-mi355x 0.1 (gfx950)";
}

int dsb_device_count(void)
{
	return dsb_gpu_device_count();
}

void dsb_free(void *p)
{
	free(p);
}

void dsb_unload_index(void *idx)
{
	dsb_index *ix = idx;
	if (!ix) return;
	dsb_gpu_free(ix);
	dsb_index_free_host_tables(ix);
	free(ix->Q_MEM); free(ix->ref_name); free(ix->ref_tid); free(ix->p_tid); free(ix->ref_seq_l); free(ix->ref_seq_offset); free(ix->tax);
	struct dsb_thread_state *s = ix->states;
	while (s) { struct dsb_thread_state *n = s->next; free(s); s = n; }
	pthread_mutex_destroy(&ix->state_mutex);
	free(ix);
}
