/*
 * pipeline.h — the streaming classify of one read_classify call (pipeline.c).
 */
#ifndef DSB_PIPELINE_H
#define DSB_PIPELINE_H
#include "dsb_host.h"
#include "gpu/dsb_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
	dsb_gpu_timing gpu;     /* kernel / transfer times and work counters summed over the batches */
	double ms_total;        /* wall time of the call */
	double ms_parse, ms_gather, ms_format; /* host stages (parse on the calling thread) */
	double ms_wait_gpu;     /* time the formatter waited for classified batches */
	uint64_t n_batches, n_devices;
	uint64_t n_view_records, n_copied_records; /* records viewed in place / assembled by the kseq emulation */
} dsb_pipe_timing;

/* Classify the FASTQ/FASTA text (resident for the whole call) on every GPU holding the index and
 * write `format` records (DSB_OUT_*) in input order into *output (malloc'd, out_n + 1 bytes,
 * NUL-terminated).  *max_read_l: the carried pool state, in/out.  Returns 0, or -1 (err). */
int dsb_pipeline_classify(dsb_index *ix, dsb_pool *pool, const char *text, uint64_t text_n, int format, int max_sec_N,
			  int *max_read_l, int stats_on, char **output, uint64_t *output_n, dsb_pipe_timing *pt,
			  char *err, size_t errn);

#ifdef __cplusplus
}
#endif
#endif
