/*
 * examples/consumer.c — an existing libdesamba.so consumer, unchanged except for the .so path.
 *
 * Binds the three reference entry points with dlsym (the pattern of the reference's own
 * consumer, main_test.c:30-32), classifies a FASTQ given by path, writes the SAM_FULL text to
 * stdout and the meta_analysis report to stderr.
 *
 *   cc -O2 -o consumer examples/consumer.c -ldl
 *   ./consumer desamba-so_amd/lib/libdesamba.so <index_dir> <reads.fq[.gz]>
 */
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include "../include/desamba.h"

typedef void (*load_index_f)(void **, const char *);
typedef void (*read_classify_f)(void *, char *, uint64_t, char **, uint64_t *, int, int);
typedef void (*meta_analysis_f)(void *, char *, uint64_t, char **, uint64_t *, int, int, uint64_t, char **,
				 uint64_t *);

int main(int argc, char **argv)
{
	if (argc < 4) {
		fprintf(stderr, "usage: %s <libdesamba.so> <index_dir> <reads.fq>\n", argv[0]);
		return 2;
	}
	void *h = dlopen(argv[1], RTLD_NOW);
	if (!h) {
		fprintf(stderr, "%s\n", dlerror());
		return 1;
	}
	load_index_f load_index_p = (load_index_f)dlsym(h, "load_index");
	read_classify_f read_classify_p = (read_classify_f)dlsym(h, "read_classify");
	meta_analysis_f meta_analysis_p = (meta_analysis_f)dlsym(h, "meta_analysis");
	if (!load_index_p || !read_classify_p || !meta_analysis_p) {
		fprintf(stderr, "missing symbol\n");
		return 1;
	}
	void *idx = NULL;
	load_index_p(&idx, argv[2]);
	char *sam = NULL, *report = NULL, *snapshot = NULL;
	uint64_t sam_n = 0, report_n = 0, snapshot_n = 0;
	read_classify_p(idx, argv[3], (uint64_t)-1, &sam, &sam_n, 0, 1);
	fwrite(sam, 1, sam_n, stdout);
	meta_analysis_p(idx, sam, sam_n, &report, &report_n, 0, META_USE_READ_NUM, 65536, &snapshot, &snapshot_n);
	fwrite(report, 1, report_n, stderr);
	free(sam);
	free(report);
	free(snapshot);
	return 0;
}
