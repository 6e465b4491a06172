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
		timing->n_reads = gt.n_reads;
		timing->n_bases = gt.n_bases;
		timing->n_retry = gt.n_retry;
		timing->n_chunks = gt.n_chunks;
		timing->seed_positions = gt.seed_positions;
		for (int k = 0; k < 16; k++) timing->stats[k] = gt.stats[k];
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
	free(ix->Q_MEM); free(ix->ref_name); free(ix->ref_seq_l); free(ix->ref_seq_offset); free(ix->tax);
	struct dsb_thread_state *s = ix->states;
	while (s) { struct dsb_thread_state *n = s->next; free(s); s = n; }
	pthread_mutex_destroy(&ix->state_mutex);
	free(ix);
}
