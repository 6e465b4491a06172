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
#include <time.h>
#include <pthread.h>
#include <sys/mman.h>
#include "dsb_host.h"
#include "pipeline.h"
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
	ix->pool = dsb_pool_new(dsb_host_threads() - 1);
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

static void copy_gpu_timing(dsb_timing_t *t, const dsb_gpu_timing *gt)
{
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
	t->n_ws_shrink = gt->n_ws_shrink;
	t->n_heavy = gt->n_heavy;
	t->n_defer_heavy = gt->n_defer_heavy;
	t->n_chunks = gt->n_chunks;
	t->seed_positions = gt->seed_positions;
	t->n_launch_dela = gt->n_launch_dela;
	t->n_launch_phase = (int)gt->n_launch_phase;
	for (int k = 0; k < DSB_N_STATS; k++) t->stats[k] = gt->stats[k];
}

/* text (plain FASTQ/FASTA, resident for the call) -> records through the streaming pipeline */
static int classify_resident(dsb_index *ix, const char *text, uint64_t text_n, int format, int *max_read_l,
			     char **output, uint64_t *output_n, dsb_timing_t *timing)
{
	char err[1024];
	dsb_pipe_timing pt;
	int st = timing ? timing->stats_on : 0;
	int rc = dsb_pipeline_classify(ix, (dsb_pool *)ix->pool, text, text_n, format, 5, max_read_l, st, output,
				       output_n, &pt, err, sizeof(err));
	if (rc) {
		fprintf(stderr, "[read_classify] %s\n", err);
		return -1;
	}
	if (timing) {
		memset(timing, 0, sizeof(*timing));
		timing->stats_on = st;
		copy_gpu_timing(timing, &pt.gpu);
		timing->ms_total = pt.ms_total;
		timing->ms_parse = pt.ms_parse;
		timing->ms_gather = pt.ms_gather;
		timing->ms_format = pt.ms_format;
		timing->ms_wait_gpu = pt.ms_wait_gpu;
		timing->n_batches = pt.n_batches;
		timing->n_devices = pt.n_devices;
		timing->n_view_records = pt.n_view_records;
		timing->n_copied_records = pt.n_copied_records;
	}
	return 0;
}

int dsb_classify_text(void *idx, const char *text, uint64_t text_n, int format, int *max_read_l, char **output,
		      uint64_t *output_n, dsb_timing_t *timing)
{
	dsb_index *ix = idx;
	char *buf = NULL;
	uint64_t len = 0;
	int owned = 0;
	if (dsb_inflate_if_gzip(text, text_n, &buf, &len, &owned)) {
		fprintf(stderr, "[dsb_classify_text] cannot decompress input\n");
		return -1;
	}
	int rc = classify_resident(ix, buf, len, format, max_read_l, output, output_n, timing);
	if (owned) free(buf);
	return rc;
}

/* reference read_classify (cly_mt.c:1309-1316, read_classify_core :1041-1081): the input text is
 * classified where it lies (a path is mapped, gzip is inflated), batch by batch over every GPU
 * holding the index, and the SAM_FULL records come back in one malloc'd buffer */
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
	uint64_t len = 0, unmap = 0;
	int owned = 0;
	if (input_n == (uint64_t)-1) {
		if (dsb_open_path(input, &buf, &len, &unmap)) {
			char msg[4200];
			snprintf(msg, sizeof(msg), "fail to open file '%s' : No such file or directory", input);
			fatal("read_classify", msg);
		}
		owned = unmap == 0;
	} else if (dsb_inflate_if_gzip(input, input_n, &buf, &len, &owned)) {
		fatal("read_classify", "cannot decompress input");
	}
	int mrl = st->max_read_l;
	struct timespec c0, c1, c2;
	clock_gettime(CLOCK_MONOTONIC, &c0);
	dsb_timing_t tm;
	memset(&tm, 0, sizeof(tm));
	if (classify_resident(ix, buf, len, DSB_OUT_SAM_FULL, &mrl, output, output_n, &tm))
		fatal("read_classify", "GPU classify failed");
	clock_gettime(CLOCK_MONOTONIC, &c1);
	st->max_read_l = mrl;
	if (unmap)
		munmap(buf, unmap);
	else if (owned)
		free(buf);
	clock_gettime(CLOCK_MONOTONIC, &c2);
	if (getenv("DSB_HOST_TIMING")) /* dev: where a call's wall time goes beyond the pipeline's */
		fprintf(stderr, "[dsb call] pipeline %.1f ms (parse %.1f, wait_gpu %.1f, format %.1f), classify_resident %.1f ms, after %.1f ms\n",
			tm.ms_total, tm.ms_parse, tm.ms_wait_gpu, tm.ms_format,
			(c1.tv_sec - c0.tv_sec) * 1e3 + (c1.tv_nsec - c0.tv_nsec) / 1e6,
			(c2.tv_sec - c1.tv_sec) * 1e3 + (c2.tv_nsec - c1.tv_nsec) / 1e6);
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
	t->n_ws_shrink = gt->n_ws_shrink;
	t->n_heavy = gt->n_heavy;
	t->n_defer_heavy = gt->n_defer_heavy;
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
	/* the batch outlives the caller's text: its records view a copy */
	char *own = malloc(text_n + 1);
	if (text_n) memcpy(own, text, text_n);
	own[text_n] = 0;
	dsb_parse_reads(own, text_n, &b->reads);
	b->reads.text_owner = own;
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
		weight_out[i] = (flag & 1) ? dsb_cstr_len(rec->seq, rec->seq_l) : 1;
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
			w[i] = (uint32_t)dsb_cstr_len(b->reads.rec[i].seq, b->reads.rec[i].seq_l);
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
int dsb_index_devices(void *idx, int *device_ids, int max_ids)
{
	dsb_index *ix = idx;
	int n = dsb_gpu_n_devices(ix);
	for (int k = 0; k < n && k < max_ids; k++)
		device_ids[k] = dsb_gpu_device_id(ix, k);
	return n;
}

void dsb_batch_free(void *idx, dsb_batch *b)
{
	if (!b) return;
	dsb_gpu_batch_free(idx, b->g);
	dsb_reads_free(&b->reads);
	free(b);
}

/* ------------------------------------------------------------------ extensions */
/* The records the parser yields for `text` (kseq + kt_pipeline semantics), one line each:
 * name, seq, qual (or "(null)") as printf("%s") prints them, '\t'-separated; slow != 0 turns
 * the zero-copy FASTQ fast path off, batch_reads > 0 parses in batches of that many reads
 * (the streaming parser).  Host only: lets the CPU tests pin the parser. */
int dsb_parse_dump(const char *text, uint64_t text_n, int slow, uint64_t batch_reads, char **output,
		   uint64_t *output_n)
{
	dsb_parser *p = dsb_parser_new(text, text_n);
	if (slow) /* a parser field, not the process environment other library threads read */
		dsb_parser_set_fast(p, 0);
	dsb_reads_t r;
	memset(&r, 0, sizeof(r));
	dsb_str out = {0, 0, 0};
	for (;;) {
		r.n = 0;
		if (!dsb_parser_next(p, &r, batch_reads ? batch_reads : UINT64_MAX, UINT64_MAX))
			break;
		for (uint64_t i = 0; i < r.n; i++) {
			const dsb_rec_t *c = r.rec + i;
			dsb_str_put(&out, c->name, dsb_cstr_len(c->name, c->name_l));
			dsb_str_printf(&out, "\t%u\t", c->seq_l);
			dsb_str_put(&out, c->seq, dsb_cstr_len(c->seq, c->seq_l));
			dsb_str_put(&out, "\t", 1);
			if (c->qual)
				dsb_str_put(&out, c->qual, dsb_cstr_len(c->qual, c->qual_l));
			else
				dsb_str_put(&out, "(null)", 6);
			dsb_str_put(&out, "\n", 1);
		}
	}
	free(r.rec);
	dsb_parser_free(p);
	*output_n = out.l;
	*output = out.s ? out.s : calloc(1, 1);
	return 0;
}

uint64_t dsb_timing_size(void)
{
	return sizeof(dsb_timing_t);
}

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
	dsb_pool_free((dsb_pool *)ix->pool);
	dsb_index_free_host_tables(ix);
	free(ix->Q_MEM); free(ix->ref_name); free(ix->ref_tid); free(ix->p_tid); free(ix->ref_seq_l); free(ix->ref_seq_offset); free(ix->tax);
	struct dsb_thread_state *s = ix->states;
	while (s) { struct dsb_thread_state *n = s->next; free(s); s = n; }
	pthread_mutex_destroy(&ix->state_mutex);
	free(ix);
}
