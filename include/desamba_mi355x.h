/*
 * desamba_mi355x.h — extensions exported next to the drop-in ABI (desamba.h).
 * Used by the tests and bench.py; not part of the reference interface.
 */
#ifndef DESAMBA_MI355X_H
#define DESAMBA_MI355X_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
	int stats_on;          /* in: collect algorithmic-work counters (slower kernel variant) */
	int pad;
	double ms_total;       /* host wall time of the GPU classify call */
	double ms_h2d, ms_d2h; /* read upload / result download (host-measured) */
	double ms_encode, ms_seed, ms_classA, ms_classB; /* per-kernel HIP-event times */
	uint64_t n_reads, n_bases, n_retry, n_chunks;
	uint64_t seed_positions; /* k-mer positions probed by k_seed (both strands) */
	uint64_t stats[16];    /* DSB_ST_* counters (occ, MEM searches, SA lookups, ...) */
} dsb_timing_t;

/* Classify FASTQ/FASTA text.  format: 1 SAM, 2 SAM_FULL, 3 DES, 4 DES_FULL.
 * *max_read_l: carried buffer-pool state (in/out), 0 for a fresh caller.
 * *output is malloc'd (free with free()/dsb_free).  timing may be NULL.  Returns 0. */
int dsb_classify_text(void *idx, const char *text, uint64_t text_n, int format, int *max_read_l, char **output,
		      uint64_t *output_n, dsb_timing_t *timing);

const char *dsb_version(void);
int dsb_device_count(void);
void dsb_free(void *p);
void dsb_unload_index(void *idx);

#ifdef __cplusplus
}
#endif
#endif
