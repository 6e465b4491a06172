/*
 * pool.c — a small persistent host thread pool for the host stages of the read_classify
 * pipeline (FASTQ views -> pinned staging gather, SAM/DES formatting, output assembly).
 *
 * The reference spreads one read_classify call over `thread_num` pthreads with kt_for
 * (src/lib/kthread.c:32-86); here the GPU does the classification and the host threads only
 * move bytes, so one pool serves every stage.  Jobs are lists of independent tasks; several
 * threads may submit jobs at once (the gather of batch k+1 runs while batch k is formatted),
 * and a submitting thread works on its own job until it is done.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#include "dsb_host.h"

typedef struct job {
	void (*fn)(void *, uint64_t, int);
	void *ctx;
	uint64_t n, next, done;
	struct job *nxt;
	pthread_cond_t finished;
} job;

struct dsb_pool {
	pthread_mutex_t mu;
	pthread_cond_t work;
	job *head; /* jobs with tasks left to hand out */
	int n_threads, stop, next_id;
	pthread_t *th;
};

/* take one task of the first job that has any left (mu held); NULL when none */
static job *take(dsb_pool *p, uint64_t *task)
{
	while (p->head && p->head->next >= p->head->n)
		p->head = p->head->nxt;
	job *j = p->head;
	if (j)
		*task = j->next++;
	return j;
}

static void finish(dsb_pool *p, job *j)
{
	if (++j->done == j->n)
		pthread_cond_broadcast(&j->finished);
	(void)p;
}

static void *worker(void *arg)
{
	dsb_pool *p = arg;
	pthread_mutex_lock(&p->mu);
	int id = ++p->next_id; /* 1..n_threads; the submitting thread is 0 */
	for (;;) {
		uint64_t t;
		job *j;
		while (!p->stop && !(j = take(p, &t)))
			pthread_cond_wait(&p->work, &p->mu);
		if (p->stop)
			break;
		pthread_mutex_unlock(&p->mu);
		j->fn(j->ctx, t, id);
		pthread_mutex_lock(&p->mu);
		finish(p, j);
	}
	pthread_mutex_unlock(&p->mu);
	return NULL;
}

/* host threads for the byte-moving stages: DSB_HOST_THREADS, else half the CPUs this process
 * may use (affinity mask, capped by a cgroup CPU quota), at most 32: the other half stays free
 * for the pipeline's own threads and the HIP runtime, so that a CPU quota never throttles the
 * thread that launches the kernels (measured: 16 busy threads on a 16-CPU quota stretched the
 * GPU waits of a read_classify call from 120 to 360 ms) */
int dsb_host_threads(void)
{
	const char *e = getenv("DSB_HOST_THREADS");
	if (e && atoi(e) > 0)
		return atoi(e);
	cpu_set_t cs;
	int n = 0;
	if (sched_getaffinity(0, sizeof(cs), &cs) == 0)
		n = CPU_COUNT(&cs);
	if (n <= 0)
		n = (int)sysconf(_SC_NPROCESSORS_ONLN);
	FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r");
	if (f) {
		char q[64] = {0};
		long per = 0;
		if (fscanf(f, "%63s %ld", q, &per) == 2 && strcmp(q, "max") != 0 && per > 0) {
			long quota = atol(q) / per;
			if (quota >= 1 && quota < n)
				n = (int)quota;
		}
		fclose(f);
	}
	n /= 2;
	if (n < 1) n = 1;
	if (n > 32) n = 32;
	return n;
}

dsb_pool *dsb_pool_new(int n_threads)
{
	dsb_pool *p = calloc(1, sizeof(*p));
	pthread_mutex_init(&p->mu, NULL);
	pthread_cond_init(&p->work, NULL);
	p->n_threads = n_threads > 0 ? n_threads : 0;
	p->th = calloc((size_t)p->n_threads + 1, sizeof(pthread_t));
	for (int i = 0; i < p->n_threads; i++)
		pthread_create(p->th + i, NULL, worker, p);
	return p;
}

int dsb_pool_size(const dsb_pool *p)
{
	return p ? p->n_threads + 1 : 1;
}

void dsb_pool_run(dsb_pool *p, uint64_t n_tasks, void (*fn)(void *ctx, uint64_t task, int worker), void *ctx)
{
	if (n_tasks == 0)
		return;
	if (!p || p->n_threads == 0 || n_tasks == 1) {
		for (uint64_t t = 0; t < n_tasks; t++)
			fn(ctx, t, 0);
		return;
	}
	job j;
	memset(&j, 0, sizeof(j));
	j.fn = fn;
	j.ctx = ctx;
	j.n = n_tasks;
	pthread_cond_init(&j.finished, NULL);
	pthread_mutex_lock(&p->mu);
	job **tail = &p->head;
	while (*tail)
		tail = &(*tail)->nxt;
	*tail = &j;
	pthread_cond_broadcast(&p->work);
	/* the caller works on its own job (worker id 0) */
	while (j.next < j.n) {
		uint64_t t = j.next++;
		pthread_mutex_unlock(&p->mu);
		fn(ctx, t, 0);
		pthread_mutex_lock(&p->mu);
		finish(p, &j);
	}
	while (j.done < j.n)
		pthread_cond_wait(&j.finished, &p->mu);
	/* unlink (take() skips exhausted jobs, but this one's memory goes away now) */
	for (job **q = &p->head; *q; q = &(*q)->nxt)
		if (*q == &j) {
			*q = j.nxt;
			break;
		}
	pthread_mutex_unlock(&p->mu);
	pthread_cond_destroy(&j.finished);
}

void dsb_pool_free(dsb_pool *p)
{
	if (!p)
		return;
	pthread_mutex_lock(&p->mu);
	p->stop = 1;
	pthread_cond_broadcast(&p->work);
	pthread_mutex_unlock(&p->mu);
	for (int i = 0; i < p->n_threads; i++)
		pthread_join(p->th[i], NULL);
	free(p->th);
	pthread_cond_destroy(&p->work);
	pthread_mutex_destroy(&p->mu);
	free(p);
}
