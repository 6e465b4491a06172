/* tools/ref_meta.c — dev-container tool: run the REFERENCE libdesamba.so's meta_analysis
 * (reference desamba.h:45) on a SAM file to produce a golden report.  dlopen consumer in
 * the style of reference main_test.c.  usage: ref_meta <libdesamba.so> <index_dir> <sam> <flag> */
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
int main(int argc, char **argv)
{
	if (argc < 5) return 2;
	void *h = dlopen(argv[1], RTLD_NOW);
	if (!h) { fprintf(stderr, "%s\n", dlerror()); return 1; }
	void (*li)(void **, const char *) = dlsym(h, "load_index");
	void (*ma)(void *, char *, uint64_t, char **, uint64_t *, int, int, uint64_t, char **, uint64_t *) =
		dlsym(h, "meta_analysis");
	FILE *f = fopen(argv[3], "rb");
	if (!f) return 1;
	fseek(f, 0, SEEK_END);
	long n = ftell(f);
	rewind(f);
	char *buf = malloc(n + 1);
	if (fread(buf, 1, n, f) != (size_t)n) return 1;
	buf[n] = 0;
	void (*rc)(void *, char *, uint64_t, char **, uint64_t *, int, int) = dlsym(h, "read_classify");
	void *idx = NULL;
	li(&idx, argv[2]);
	/* the reference's meta_analysis needs the thread_id's buffers to exist already
	 * (find_and_init_buff_for_thread_mutex with thread_num -1 aborts, cly_mt.c:1338) */
	{
		char fq[] = "@warmup\nACGTACGTACGTACGTACGTACGTACGTACGTACGTACGTACGTACGT\n+\nIIIIIIIIIIIIIIIIIIIIIIIIIIIIIIIIIIIIIIIIIIIIIIII\n";
		char *o = NULL;
		uint64_t on = 0;
		rc(idx, fq, sizeof(fq) - 1, &o, &on, 0, 1);
		free(o);
	}
	char *out = NULL, *snap = NULL;
	uint64_t out_n = 0, snap_n = 0;
	ma(idx, buf, (uint64_t)n, &out, &out_n, 0, atoi(argv[4]), 65536, &snap, &snap_n);
	fwrite(out, 1, out_n, stdout);
	printf("#snapshot_n\t%lu\n", (unsigned long)snap_n);
	if (snap) printf("#snapshot_head\t%.60s\n", snap);
	return 0;
}
