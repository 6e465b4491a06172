/*
 * oracle/abi_time.c — TEST / MEASUREMENT INFRASTRUCTURE ONLY (never linked into the product).
 *
 * Times the drop-in call the way an existing consumer makes it: dlopen a libdesamba.so
 * (the reference's, oracle/_ref/libdesamba.so, or this repository's), bind the reference
 * ABI with dlsym (reference main_test.c:29-32), load_index once, then time ONE
 * read_classify(idx, text, n, &out, &out_n, thread_id 0, thread_num) over the whole FASTQ
 * held in memory (reference desamba.h:23, cly_mt.c:1309-1316).  The index load is outside
 * the timed region, as in the reference's own "sequences processed" timer (cly_mt.c:527).
 *
 *   abi_time <libdesamba.so> <index_dir> <reads.fq> <thread_num> [out.sam]
 *
 * prints one JSON line: {"secs": ..., "input_bytes": ..., "output_bytes": ..., "records": ...}
 */
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

typedef void (*load_index_f)(void **, const char *);
typedef void (*read_classify_f)(void *, char *, uint64_t, char **, uint64_t *, int, int);

static double now_s(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}

int main(int argc, char **argv)
{
	if (argc < 5) {
		fprintf(stderr, "usage: %s <libdesamba.so> <index_dir> <reads.fq> <thread_num> [out.sam]\n", argv[0]);
		return 2;
	}
	void *h = dlopen(argv[1], RTLD_NOW);
	if (!h) {
		fprintf(stderr, "%s\n", dlerror());
		return 1;
	}
	load_index_f li = (load_index_f)dlsym(h, "load_index");
	read_classify_f rc = (read_classify_f)dlsym(h, "read_classify");
	if (!li || !rc) {
		fprintf(stderr, "missing ABI symbols\n");
		return 1;
	}
	FILE *f = fopen(argv[3], "rb");
	if (!f) {
		perror(argv[3]);
		return 1;
	}
	fseek(f, 0, SEEK_END);
	long n = ftell(f);
	rewind(f);
	char *buf = malloc((size_t)n + 1);
	if (fread(buf, 1, (size_t)n, f) != (size_t)n) {
		fprintf(stderr, "short read\n");
		return 1;
	}
	buf[n] = 0;
	fclose(f);
	int threads = atoi(argv[4]);
	void *idx = NULL;
	li(&idx, argv[2]);
	char *out = NULL;
	uint64_t out_n = 0;
	double t0 = now_s();
	rc(idx, buf, (uint64_t)n, &out, &out_n, 0, threads);
	double secs = now_s() - t0;
	uint64_t recs = 0;
	for (uint64_t i = 0; i < out_n; i++)
		recs += out[i] == '\n';
	if (argc > 5) {
		FILE *o = fopen(argv[5], "wb");
		if (!o || fwrite(out, 1, out_n, o) != out_n) {
			perror(argv[5]);
			return 1;
		}
		fclose(o);
	}
	printf("{\"secs\": %.6f, \"input_bytes\": %ld, \"output_bytes\": %lu, \"records\": %lu, \"thread_num\": %d}\n",
	       secs, n, (unsigned long)out_n, (unsigned long)recs, threads);
	fflush(stdout);
	free(out);
	free(buf);
	/* the reference never frees an index (desamba.h); exit without unloading */
	_exit(0);
}
