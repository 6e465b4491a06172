/*
 * desamba_mi355x.h — extensions exported next to the drop-in ABI (desamba.h).
 * Used by the tests and bench.py; not part of the reference interface.
 */
#ifndef DESAMBA_MI355X_H
#define DESAMBA_MI355X_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
	int stats_on;          /* in: 1 collect algorithmic-work counters, 2 wave clocks per code region (slower kernel variants) */
	int n_launch_phase;   /* out: launches of each part-A phase kernel (chunks x pipelined halves) */
	double ms_total;       /* host wall time of the GPU classify call */
	double ms_h2d, ms_d2h; /* read upload / result download (host-measured) */
	double ms_encode, ms_seed, ms_classA, ms_classB; /* per-kernel HIP-event times */
	double ms_phase[12];   /* classify part A per phase (island, fast0/1, resolve, slow0/1, ...) */
	uint64_t n_reads, n_bases, n_retry, n_chunks;
	uint64_t seed_positions; /* k-mer positions probed by k_seed (both strands) */
	uint64_t n_launch_dela;  /* launches of the scoring kernel k_wave_phase<8> (2 per chunk when split) */
	uint64_t stats[320];   /* work counters: [32*ph, +32) phase ph of part A, [288,320) k_classB */
	/* the streaming pipeline of dsb_classify_text / read_classify (host stages, wall times) */
	double ms_parse, ms_gather, ms_format, ms_wait_gpu;
	uint64_t n_batches, n_devices, n_view_records, n_copied_records;
	uint64_t n_ws_shrink;  /* chunks re-partitioned smaller: their workspace did not fit in the free HBM */
	uint64_t n_heavy;      /* scoring reads launched first (many chains of a long read) */
	uint64_t n_defer_heavy; /* heavy reads classified with the batch's deferred re-runs (DSB_HEAVY_DEFER) */
} dsb_timing_t;

/* Classify FASTQ/FASTA text.  format: 1 SAM, 2 SAM_FULL, 3 DES, 4 DES_FULL.
 * *max_read_l: carried buffer-pool state (in/out), 0 for a fresh caller.
 * *output is malloc'd (free with free()/dsb_free).  timing may be NULL.  Returns 0. */
int dsb_classify_text(void *idx, const char *text, uint64_t text_n, int format, int *max_read_l, char **output,
		      uint64_t *output_n, dsb_timing_t *timing);

/* Batch API: parse + upload once (reads resident in HBM), classify any number of times,
 * format or reduce the results.  Used by bench.py to time the path with inputs in HBM. */
typedef struct dsb_batch dsb_batch;
dsb_batch *dsb_batch_create(void *idx, const char *text, uint64_t text_n, dsb_timing_t *timing);
int dsb_batch_run(void *idx, dsb_batch *b, int *max_read_l, dsb_timing_t *timing);
int dsb_batch_format(void *idx, dsb_batch *b, int format, char **output, uint64_t *output_n);
/* the records of reads [lo, hi) only (input order), as dsb_batch_format writes them */
int dsb_batch_format_range(void *idx, dsb_batch *b, int format, uint64_t lo, uint64_t hi, char **output,
			   uint64_t *output_n);
/* carry_out[i] = the max_read_l read i's length filter used in the last run (the carried
 * Classify_buff_pool.max_read_l, reference src/cly.c:2953-2963); monotone over the batch */
int dsb_batch_carry(dsb_batch *b, int32_t *carry_out);
/* Per-read taxon as meta_analysis assigns it (ana_get_tid, reference src/cly_mt.c:902-961):
 * tid_out[i] (0 = unclassified); weight_out[i] = 1 or the read length (flag & 1). */
int dsb_batch_taxa(void *idx, dsb_batch *b, int flag, uint32_t *tid_out, uint64_t *weight_out);
/* The same taxa reduced on the GPU: dev_counts[t] = the summed weights (1, or the read length
 * when flag & 1) of the last run's reads assigned taxon t (meta_analysis node_count, reference
 * src/cly_mt.c:1352-1362).  dev_counts: device memory of the index's GPU, n_counts >=
 * dsb_max_tid(idx) + 1 u64 entries, overwritten; the per-read taxa are computed by the classify
 * kernels, so nothing but the table crosses PCIe.  Returns 0, or -1 (message on stderr). */
int dsb_batch_taxon_counts(void *idx, dsb_batch *b, int flag, uint64_t *dev_counts, uint64_t n_counts);
uint64_t dsb_batch_reads(dsb_batch *b);
uint64_t dsb_batch_bases(dsb_batch *b);
void dsb_batch_free(void *idx, dsb_batch *b);
/* largest taxid of the loaded taxonomy (+1e6, reference src/cly_mt.c:613) */
uint64_t dsb_max_tid(void *idx);
/* the GPUs the index is replicated on (load_index: DSB_DEVICES "all" / "0,1,..", else DSB_DEVICE,
 * else the current device): writes up to max_ids HIP device ids, returns their number.
 * read_classify spreads its batches over all of them; the batch API uses the first. */
int dsb_index_devices(void *idx, int *device_ids, int max_ids);

/* Diagnostics (host only): the records the FASTQ/FASTA parser yields, one "name\tseq_l\tseq\tqual\n"
 * line each (strings as printf %s prints them); slow: byte-level kseq emulation only;
 * batch_reads > 0: parse as the streaming pipeline does, in batches. */
int dsb_parse_dump(const char *text, uint64_t text_n, int slow, uint64_t batch_reads, char **output,
		   uint64_t *output_n);

const char *dsb_version(void);

/* sizeof(dsb_timing_t) as this library fills it: a caller built against another version of this
 * header checks it before passing a timing struct (the struct has grown between versions) */
uint64_t dsb_timing_size(void);
int dsb_device_count(void);
void dsb_free(void *p);
void dsb_unload_index(void *idx);

#ifdef __cplusplus
}
#endif
#endif
