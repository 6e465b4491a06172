/*
 * pipeline.c — read_classify as a stream of batches over the GPUs holding the index.
 *
 * The reference runs one read_classify call as a 3-step kt_pipeline (src/cly_mt.c:361-381,
 * src/lib/kthread.c:114-197): read <= 5000 reads / 10 Mbp, classify them with kt_for over
 * thread_num pthreads, write the records in input order.  Here the steps are:
 *
 *   parse    (one thread)      kt_pipeline batches of the resident text, as record views
 *                              (fastq.c), grouped into GPU batches of up to DSB_PIPE_READS
 *                              reads / DSB_PIPE_MBP Mbp
 *   stage    (one thread/GPU)  bases gathered into pinned staging by the host pool, copied on
 *                              the GPU's copy stream while the batch before is classified
 *   classify (one thread/GPU)  the kernels (kernels.hip batch_run); the carried max_read_l
 *                              (cly.c:2953) passes from batch to batch, across GPUs, between
 *                              part A and part B of each batch
 *   format   (calling thread)  SAM / SAM_FULL / DES / DES_FULL records of each batch in input
 *                              order, formatted in parallel by the host pool into one growing
 *                              output buffer
 *
 * At most DSB_PIPE_DEPTH batches are alive at once, so host and device memory are bounded by
 * the batch size, not by the input (the output buffer itself is the call's result).
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <sys/mman.h>
#include "dsb_host.h"
#include "pipeline.h"
#ifndef DSB_TEST_HOOKS
#define DSB_TEST_HOOKS 0 /* lib/libdesamba_test.so: -DDSB_TEST_HOOKS=1 */
#endif
#include "gpu/dsb_gpu.h"

typedef struct pbatch {
	uint64_t seq;         /* batch number, input order */
	dsb_reads_t reads;    /* views into the text / the parser's arena */
	dsb_gpu_batch *g;
	int slot;             /* GPU */
	int classified;
	struct pbatch *next;  /* queue link */
} pbatch;

typedef struct {
	dsb_index *ix;
	dsb_pool *pool;
	int format, max_sec_N, stats_on, n_dev, round_robin;
	pthread_mutex_t mu;
	pthread_cond_t cv;
	pbatch *parsed_head, *parsed_tail;       /* parsed, not yet staged */
	pbatch *runq_head[DSB_MAX_GPUS], *runq_tail[DSB_MAX_GPUS];
	int runq_n[DSB_MAX_GPUS];
	pbatch **by_seq; uint64_t by_seq_cap;     /* classified batches for the formatter */
	uint64_t n_parsed, n_formatted;
	int parse_done, failed, stagers_done;
	char err[512];
	/* carry chain */
	uint64_t n_locked;  /* batches that have taken their GPU run lock (they do so in input order) */
	int carry0;
	int *carry; uint8_t *carry_ready; uint64_t carry_cap;
	/* output */
	char *out; uint64_t out_n, out_m;
	/* formatter per-task buffers; SAM_FULL: per read the offset in its task buffer where SEQ\tQUAL
	 * go (composed straight into the output by the copy pass), per task the output bytes */
	dsb_str *tbuf; uint64_t n_tbuf;
	uint64_t *hole, hole_cap, *tsize;
	/* accounting */
	dsb_gpu_timing gt;
	double ms_parse, ms_gather, ms_format, ms_wait_gpu;
	uint64_t n_batches;
	/* parser thread */
	dsb_parser *ps;
	uint64_t max_reads, max_bases, depth;
	uint64_t first_div, tail_div; /* batch sizing (parser_main) */
} pipe_t;

typedef struct {
	pipe_t *p;
	uint64_t seq;
} chain_ctx;

static double now_ms(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec * 1e3 + ts.tv_nsec / 1e6;
}

static uint64_t env_u64(const char *name, uint64_t dflt)
{
	const char *e = getenv(name);
	return e && *e ? strtoull(e, NULL, 10) : dflt;
}

static void fail(pipe_t *p, const char *msg)
{
	pthread_mutex_lock(&p->mu);
	if (!p->failed) {
		p->failed = 1;
		snprintf(p->err, sizeof(p->err), "%s", msg);
	}
	pthread_cond_broadcast(&p->cv);
	pthread_mutex_unlock(&p->mu);
}

/* ---------------------------------------------------------------- carry chain */
static void carry_reserve(pipe_t *p, uint64_t seq) /* mu held */
{
	if (seq < p->carry_cap)
		return;
	uint64_t c = p->carry_cap ? p->carry_cap : 64;
	while (c <= seq)
		c *= 2;
	p->carry = realloc(p->carry, c * sizeof(int));
	p->carry_ready = realloc(p->carry_ready, c);
	memset(p->carry_ready + p->carry_cap, 0, c - p->carry_cap);
	p->carry_cap = c;
}

static int carry_in(void *ctx)
{
	chain_ctx *c = ctx;
	pipe_t *p = c->p;
	if (c->seq == 0)
		return p->carry0;
	pthread_mutex_lock(&p->mu);
	carry_reserve(p, c->seq);
	while (!p->carry_ready[c->seq - 1] && !p->failed)
		pthread_cond_wait(&p->cv, &p->mu);
	/* a failed pipeline discards every result: hand back a defined value */
	int v = p->carry_ready[c->seq - 1] ? p->carry[c->seq - 1] : p->carry0;
	pthread_mutex_unlock(&p->mu);
	return v;
}

/* Run locks in input order.  A batch holds its context's run lock while it waits in carry_in for
 * the batch before; if that batch could still be queued for a lock held by another call's waiting
 * batch, two concurrent read_classify calls could each hold the lock the other needs.  With every
 * call's batches taking their locks in input order, a lock holder only ever waits for an earlier
 * batch of its own call that already holds (or has released) a lock, so the waits cannot close a
 * cycle. */
static void lock_wait(void *ctx)
{
	chain_ctx *c = ctx;
	pipe_t *p = c->p;
	pthread_mutex_lock(&p->mu);
	while (p->n_locked < c->seq && !p->failed)
		pthread_cond_wait(&p->cv, &p->mu);
	pthread_mutex_unlock(&p->mu);
}

static void locked(void *ctx)
{
	chain_ctx *c = ctx;
	pipe_t *p = c->p;
	pthread_mutex_lock(&p->mu);
	if (p->n_locked < c->seq + 1)
		p->n_locked = c->seq + 1;
	pthread_cond_broadcast(&p->cv);
	pthread_mutex_unlock(&p->mu);
}

static void carry_out(void *ctx, int v)
{
	chain_ctx *c = ctx;
	pipe_t *p = c->p;
	pthread_mutex_lock(&p->mu);
	carry_reserve(p, c->seq);
	p->carry[c->seq] = v;
	p->carry_ready[c->seq] = 1;
	pthread_cond_broadcast(&p->cv);
	pthread_mutex_unlock(&p->mu);
}

/* ---------------------------------------------------------------- GPU threads */
typedef struct {
	pipe_t *p;
	int slot;
} dev_arg;

static void acc_timing(dsb_gpu_timing *a, const dsb_gpu_timing *b)
{
	a->ms_h2d += b->ms_h2d;
	a->ms_d2h += b->ms_d2h;
	a->ms_encode += b->ms_encode;
	a->ms_seed += b->ms_seed;
	a->ms_classA += b->ms_classA;
	a->ms_classB += b->ms_classB;
	for (int k = 0; k < 12; k++)
		a->ms_phase[k] += b->ms_phase[k];
	a->n_reads += b->n_reads;
	a->n_bases += b->n_bases;
	a->n_retry += b->n_retry;
	a->n_ws_shrink += b->n_ws_shrink;
	a->n_heavy += b->n_heavy;
	a->n_defer_heavy += b->n_defer_heavy;
	a->n_chunks += b->n_chunks;
	a->seed_positions += b->seed_positions;
	a->n_launch_dela += b->n_launch_dela;
	a->n_launch_phase += b->n_launch_phase;
	for (int k = 0; k < DSB_N_STATS; k++)
		a->stats[k] += b->stats[k];
}

/* stager of GPU `slot`: takes parsed batches in input order, uploads them, queues them for
 * the classify thread of the same GPU (at most one staged ahead) */
static void *stager(void *arg)
{
	dev_arg *a = arg;
	pipe_t *p = a->p;
	int slot = a->slot;
	char err[512];
	for (;;) {
		pthread_mutex_lock(&p->mu);
		/* at most two batches per GPU between staging and classified: one classifying, one staged;
		 * DSB_TEST_ROUND_ROBIN (test build of the library): batch k goes to GPU context k mod n */
		while (!p->failed && (p->runq_n[slot] >= 2 || (!p->parsed_head && !p->parse_done) ||
				      (p->round_robin && p->parsed_head && p->parsed_head->seq % (uint64_t)p->n_dev != (uint64_t)slot)))
			pthread_cond_wait(&p->cv, &p->mu);
		if (p->failed || !p->parsed_head) {
			p->stagers_done++;
			pthread_cond_broadcast(&p->cv);
			pthread_mutex_unlock(&p->mu);
			return NULL;
		}
		pbatch *b = p->parsed_head;
		p->parsed_head = b->next;
		if (!p->parsed_head)
			p->parsed_tail = NULL;
		b->next = NULL;
		p->runq_n[slot]++;
		pthread_mutex_unlock(&p->mu);
		double ms_g = 0;
		b->slot = slot;
		if (dsb_gpu_batch_stage(p->ix, slot, &b->reads, p->pool, &b->g, &ms_g, err, sizeof(err))) {
			fail(p, err);
			return NULL;
		}
		pthread_mutex_lock(&p->mu);
		p->ms_gather += ms_g;
		if (p->runq_tail[slot])
			p->runq_tail[slot]->next = b;
		else
			p->runq_head[slot] = b;
		p->runq_tail[slot] = b;
		pthread_cond_broadcast(&p->cv);
		pthread_mutex_unlock(&p->mu);
	}
}

static void *runner(void *arg)
{
	dev_arg *a = arg;
	pipe_t *p = a->p;
	int slot = a->slot;
	char err[512];
	for (;;) {
		pthread_mutex_lock(&p->mu);
		while (!p->failed && !p->runq_head[slot] && p->stagers_done < p->n_dev)
			pthread_cond_wait(&p->cv, &p->mu);
		pbatch *b = p->runq_head[slot];
		if (p->failed || !b) {
			pthread_mutex_unlock(&p->mu);
			return NULL;
		}
		p->runq_head[slot] = b->next;
		if (!p->runq_head[slot])
			p->runq_tail[slot] = NULL;
		pthread_mutex_unlock(&p->mu);
		chain_ctx cc = {p, b->seq};
		dsb_carry_hooks h = {carry_in, carry_out, &cc, lock_wait, locked};
		dsb_gpu_timing t;
		memset(&t, 0, sizeof(t));
		if (dsb_gpu_batch_run_chain(p->ix, b->g, p->stats_on, &h, &t, err, sizeof(err))) {
			fail(p, err);
			return NULL;
		}
		pthread_mutex_lock(&p->mu);
		acc_timing(&p->gt, &t);
		b->classified = 1;
		p->runq_n[slot]--;
		pthread_cond_broadcast(&p->cv);
		pthread_mutex_unlock(&p->mu);
	}
}

/* ---------------------------------------------------------------- format */
/* The output is written once by many threads: ask for transparent huge pages on it, so that
 * its first touch faults 2 MB at a time instead of 4 KB (a hint; ignored where THP is off). */
static void out_hugepages(char *p, uint64_t n)
{
	uintptr_t a = ((uintptr_t)p + 4095) & ~(uintptr_t)4095, e = ((uintptr_t)p + n) & ~(uintptr_t)4095;
	if (e > a + (2u << 20))
		madvise((void *)a, e - a, MADV_HUGEPAGE);
}

typedef struct {
	pipe_t *p;
	pbatch *b;
	uint64_t per_task;
	const uint64_t *off; /* output offsets of the task buffers (copy pass) */
} fmt_ctx;

static void format_task(void *c_, uint64_t t, int worker)
{
	(void)worker;
	fmt_ctx *c = c_;
	pipe_t *p = c->p;
	dsb_str *s = p->tbuf + t;
	s->l = 0;
	uint64_t lo = t * c->per_task, hi = lo + c->per_task;
	if (hi > c->b->reads.n)
		hi = c->b->reads.n;
	const dsb_read_out_t *ro = dsb_gpu_batch_ro(c->b->g);
	const dsb_hit_out_t *hits = dsb_gpu_batch_hits(c->b->g);
	uint64_t extra = 0;
	for (uint64_t i = lo; i < hi; i++) {
		uint64_t hn = 0;
		dsb_format_read_hole(s, p->ix, &c->b->reads, i, ro + i, hits + ro[i].hit_off, p->format, p->max_sec_N,
				     p->hole + i, &hn);
		if (p->hole[i] != UINT64_MAX)
			extra += hn;
	}
	p->tsize[t] = s->l + extra;
}

/* the task's records into the output: its buffer, with each read's SEQ\tQUAL copied from the
 * record views into the holes (SAM_FULL) */
static void copy_task(void *c_, uint64_t t, int worker)
{
	(void)worker;
	fmt_ctx *c = c_;
	pipe_t *p = c->p;
	const dsb_str *s = p->tbuf + t;
	char *d = p->out + c->off[t];
	uint64_t lo = t * c->per_task, hi = lo + c->per_task, pos = 0;
	if (hi > c->b->reads.n)
		hi = c->b->reads.n;
	for (uint64_t i = lo; i < hi; i++) {
		uint64_t h = p->hole[i];
		if (h == UINT64_MAX)
			continue;
		memcpy(d, s->s + pos, h - pos);
		d += h - pos;
		pos = h;
		const char *sq, *ql;
		uint64_t sn, qn;
		dsb_sam_seq_qual(c->b->reads.rec + i, &sq, &sn, &ql, &qn);
		memcpy(d, sq, sn);
		d += sn;
		*d++ = '\t';
		memcpy(d, ql, qn);
		d += qn;
	}
	if (s->l > pos)
		memcpy(d, s->s + pos, s->l - pos);
}

static int format_batch(pipe_t *p, pbatch *b)
{
	uint64_t n = b->reads.n;
	uint64_t n_tasks = (uint64_t)dsb_pool_size(p->pool) * 4;
	if (n_tasks > n)
		n_tasks = n ? n : 1;
	fmt_ctx c = {p, b, n / n_tasks + (n % n_tasks != 0), NULL};
	if (c.per_task == 0)
		c.per_task = 1;
	n_tasks = n ? (n + c.per_task - 1) / c.per_task : 0;
	if (n_tasks > p->n_tbuf) {
		p->tbuf = realloc(p->tbuf, n_tasks * sizeof(dsb_str));
		memset(p->tbuf + p->n_tbuf, 0, (n_tasks - p->n_tbuf) * sizeof(dsb_str));
		p->tsize = realloc(p->tsize, n_tasks * sizeof(uint64_t));
		p->n_tbuf = n_tasks;
	}
	if (n > p->hole_cap) {
		p->hole = realloc(p->hole, n * sizeof(uint64_t));
		p->hole_cap = n;
	}
	dsb_pool_run(p->pool, n_tasks, format_task, &c);
	uint64_t *off = malloc((n_tasks + 1) * sizeof(uint64_t));
	uint64_t tot = p->out_n;
	for (uint64_t t = 0; t < n_tasks; t++) {
		off[t] = tot;
		tot += p->tsize[t];
	}
	if (tot + 1 > p->out_m) { /* large chunks are mmap'd: realloc moves pages, not bytes */
		uint64_t m = p->out_m ? p->out_m : (1u << 20);
		while (m < tot + 1)
			m += m / 2;
		char *q = realloc(p->out, m);
		if (!q) {
			free(off);
			return -1;
		}
		p->out = q;
		p->out_m = m;
		out_hugepages(p->out, p->out_m);
	}
	c.off = off;
	dsb_pool_run(p->pool, n_tasks, copy_task, &c);
	p->out_n = tot;
	free(off);
	return 0;
}

/* ---------------------------------------------------------------- parse */
/* parser thread: GPU batches of the text in input order while fewer than `depth` batches are
 * alive, so that parsing batch k+1 overlaps formatting batch k on the calling thread */
static void *parser_main(void *arg)
{
	pipe_t *p = arg;
	uint64_t seq = 0;
	for (;;) {
		pthread_mutex_lock(&p->mu);
		while (!p->failed && p->n_parsed - p->n_formatted >= p->depth)
			pthread_cond_wait(&p->cv, &p->mu);
		if (p->failed)
			break; /* mu held */
		pthread_mutex_unlock(&p->mu);
		double tp = now_ms();
		pbatch *b = calloc(1, sizeof(pbatch));
		/* batch sizes: the first batch is 1/first_div of a full one, so the GPU starts sooner;
		 * when what is left of the input makes at most 1.5 full batches, it is cut into a large
		 * batch and a last one of 1/tail_div of it, so that little formatting follows the last
		 * GPU batch (FASTQ text: ~2 bytes per base) */
		uint64_t mr = p->max_reads, mb = p->max_bases;
		if (seq == 0) {
			mr = (mr + p->first_div - 1) / p->first_div;
			mb = (mb + p->first_div - 1) / p->first_div;
		} else if (p->tail_div > 1) {
			uint64_t left = dsb_parser_left(p->ps) / 2;
			if (left <= mb + mb / 2 && left > mb / p->tail_div)
				mb = left - left / p->tail_div;
		}
		uint64_t got = b ? dsb_parser_next(p->ps, &b->reads, mr, mb) : 0;
		double dt = now_ms() - tp;
		pthread_mutex_lock(&p->mu);
		p->ms_parse += dt;
		if (!got) {
			if (b) {
				free(b->reads.rec);
				free(b);
			}
			break; /* parse_done below */
		}
		b->seq = seq++;
		if (b->seq >= p->by_seq_cap) {
			uint64_t c = p->by_seq_cap ? p->by_seq_cap * 2 : 64;
			pbatch **q = realloc(p->by_seq, c * sizeof(pbatch *));
			if (!q) {
				pthread_mutex_unlock(&p->mu);
				free(b->reads.rec);
				free(b);
				fail(p, "out of memory parsing the input");
				pthread_mutex_lock(&p->mu);
				break;
			}
			p->by_seq = q;
			memset(p->by_seq + p->by_seq_cap, 0, (c - p->by_seq_cap) * sizeof(pbatch *));
			p->by_seq_cap = c;
		}
		p->by_seq[b->seq] = b;
		if (p->parsed_tail)
			p->parsed_tail->next = b;
		else
			p->parsed_head = b;
		p->parsed_tail = b;
		p->n_parsed++;
		pthread_cond_broadcast(&p->cv);
		pthread_mutex_unlock(&p->mu);
	}
	/* mu held */
	p->parse_done = 1;
	pthread_cond_broadcast(&p->cv);
	pthread_mutex_unlock(&p->mu);
	return NULL;
}

/* ---------------------------------------------------------------- driver */
int dsb_pipeline_classify(dsb_index *ix, dsb_pool *pool, const char *text, uint64_t text_n, int format, int max_sec_N,
			  int *max_read_l, int stats_on, char **output, uint64_t *output_n, dsb_pipe_timing *pt,
			  char *err, size_t errn)
{
	double t0 = now_ms();
	int n_dev = dsb_gpu_n_devices(ix);
	if (n_dev <= 0) {
		snprintf(err, errn, "index not resident on a GPU");
		return -1;
	}
	pipe_t P;
	memset(&P, 0, sizeof(P));
	pipe_t *p = &P;
	p->ix = ix;
	p->pool = pool;
	p->format = format;
	p->max_sec_N = max_sec_N;
	p->stats_on = stats_on;
	p->n_dev = n_dev;
	p->carry0 = *max_read_l;
	pthread_mutex_init(&p->mu, NULL);
	pthread_cond_init(&p->cv, NULL);
	p->round_robin = DSB_TEST_HOOKS && env_u64("DSB_TEST_ROUND_ROBIN", 0) != 0; /* test build only */
	p->max_reads = env_u64("DSB_PIPE_READS", 100000); /* measured (C2 proxy, 100k reads): 25k / 50k / 100k -> 278k / 292k / 317k reads/s */
	p->max_bases = env_u64("DSB_PIPE_MBP", 400) * 1000000ull;
	p->first_div = env_u64("DSB_PIPE_FIRST", 4);
	p->tail_div = env_u64("DSB_PIPE_TAIL", 0);
	if (p->first_div == 0) p->first_div = 1;
	if (p->max_reads == 0) p->max_reads = 1;
	if (dsb_gpu_fit_contexts(ix, p->max_reads, err, errn))
		return -1;
	p->depth = env_u64("DSB_PIPE_DEPTH", 2 + 2 * (uint64_t)n_dev);
	if (p->max_reads == 0) p->max_reads = 1;
	if (p->depth < 2) p->depth = 2;
	/* SAM_FULL output is about the input's size */
	p->out_m = text_n + text_n / 8 + (1u << 20);
	p->out = malloc(p->out_m);
	if (!p->out) {
		snprintf(err, errn, "out of memory for the output (%lu bytes)", (unsigned long)p->out_m);
		return -1;
	}
	out_hugepages(p->out, p->out_m);
	p->ps = dsb_parser_new(text, text_n);
	pthread_t th[2 * DSB_MAX_GPUS], pth;
	dev_arg args[DSB_MAX_GPUS];
	for (int d = 0; d < n_dev; d++) {
		args[d].p = p;
		args[d].slot = d;
		pthread_create(th + 2 * d, NULL, stager, args + d);
		pthread_create(th + 2 * d + 1, NULL, runner, args + d);
	}
	pthread_create(&pth, NULL, parser_main, p);
	/* format each batch in input order once it is classified */
	for (;;) {
		double tw = now_ms();
		pbatch *b = NULL;
		pthread_mutex_lock(&p->mu);
		while (!p->failed) {
			b = p->n_formatted < p->n_parsed ? p->by_seq[p->n_formatted] : NULL;
			if (b && b->classified)
				break;
			b = NULL;
			if (p->parse_done && p->n_formatted == p->n_parsed)
				break;
			pthread_cond_wait(&p->cv, &p->mu);
		}
		p->ms_wait_gpu += now_ms() - tw;
		pthread_mutex_unlock(&p->mu);
		if (!b)
			break; /* failed, or everything formatted */
		double tf = now_ms();
		if (format_batch(p, b)) {
			fail(p, "out of memory formatting the output");
			break;
		}
		dsb_gpu_batch_recycle(ix, b->g);
		free(b->reads.rec);
		pthread_mutex_lock(&p->mu);
		p->ms_format += now_ms() - tf;
		p->by_seq[b->seq] = NULL;
		p->n_formatted++;
		p->n_batches++;
		pthread_cond_broadcast(&p->cv);
		pthread_mutex_unlock(&p->mu);
		free(b);
	}
	pthread_join(pth, NULL);
	uint64_t seq = p->n_parsed;
	pthread_mutex_lock(&p->mu);
	p->parse_done = 1;
	pthread_cond_broadcast(&p->cv);
	pthread_mutex_unlock(&p->mu);
	for (int d = 0; d < 2 * n_dev; d++)
		pthread_join(th[d], NULL);
	int rc = 0;
	if (p->failed) {
		snprintf(err, errn, "%s", p->err);
		rc = -1;
		/* batches left in flight: give their GPU buffers back */
		for (uint64_t k = p->n_formatted; k < p->n_parsed; k++)
			if (p->by_seq[k]) {
				if (p->by_seq[k]->g)
					dsb_gpu_batch_recycle(ix, p->by_seq[k]->g);
				free(p->by_seq[k]->reads.rec);
				free(p->by_seq[k]);
			}
		free(p->out);
		*output = NULL;
		*output_n = 0;
	} else {
		if (seq > 0 && p->carry_cap > seq - 1 && p->carry_ready[seq - 1])
			*max_read_l = p->carry[seq - 1];
		char *q = realloc(p->out, p->out_n + 1); /* shrink to out_n + 1 */
		if (q)
			p->out = q;
		p->out[p->out_n] = 0;
		*output = p->out;
		*output_n = p->out_n;
	}
	if (pt) {
		memset(pt, 0, sizeof(*pt));
		pt->gpu = p->gt;
		pt->ms_total = now_ms() - t0;
		pt->ms_parse = p->ms_parse;
		pt->ms_gather = p->ms_gather;
		pt->ms_format = p->ms_format;
		pt->ms_wait_gpu = p->ms_wait_gpu;
		pt->n_batches = p->n_batches;
		pt->n_devices = (uint64_t)n_dev;
		uint64_t nf = 0, ns = 0;
		dsb_parser_stats(p->ps, &nf, &ns);
		pt->n_view_records = nf;
		pt->n_copied_records = ns;
	}
	dsb_parser_free(p->ps);
	for (uint64_t t = 0; t < p->n_tbuf; t++)
		free(p->tbuf[t].s);
	free(p->tbuf);
	free(p->tsize);
	free(p->hole);
	free(p->by_seq);
	free(p->carry);
	free(p->carry_ready);
	pthread_cond_destroy(&p->cv);
	pthread_mutex_destroy(&p->mu);
	return rc;
}
