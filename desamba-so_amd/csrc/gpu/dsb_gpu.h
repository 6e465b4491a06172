/*
 * dsb_gpu.h — the thin C-ABI between the C host code and the HIP kernels.
 * Plain pointers and sizes only; implemented in kernels.hip.
 */
#ifndef DSB_GPU_H
#define DSB_GPU_H
#include <stdint.h>
#include <stddef.h>
#include "../dsb_host.h"

#ifdef __cplusplus
extern "C" {
#endif

#define DSB_MAX_HITS 400 /* delete_small_score_rst keeps at most 400 chains (src/cly.c:2892) */

#define DSB_ST_STRIDE 32 /* counters per phase */
/* DSB_WAVE_DBG bit: per-read wall-clock timeline of the wave phases (dev tool: a DSB_TL=1 build,
 * DSB_TIMELINE=path):
 * record {start, end, read | phase << 32, hw_id} of slot t of phase ph at
 * stats[DSB_N_STATS + 4 * (ph * DSB_TL_STRIDE + t)] (s_memrealtime, 100 MHz) */
#define DSB_DBG_TIMELINE (1u << 12)
#define DSB_TL_STRIDE (1u << 17)
/* DSB_WAVE_DBG bit (tests): seeding waves hand their sp_set pool set back without moving its
 * generation base on, so later holders meet slots that still match (dsb_hpool_release) */
#define DSB_DBG_POOL_NOGEN (1u << 13)
#define DSB_N_STATS 320 /* 32 counters x (9 phases of part A + k_classB) */
#define DSB_STATS_B 288
#define DSB_STATS_SEED 0 /* k_seed's Bloom-probe counters (ek1, ek2): the island phase's block (island itself probes nothing) */

typedef struct {
	double ms_total;      /* wall time of dsb_gpu_classify, host-measured */
	double ms_h2d, ms_d2h;
	double ms_encode, ms_seed, ms_classA, ms_classB; /* HIP-event kernel times, summed over chunks */
	double ms_phase[12];  /* k_phase<ph> times (ms_classA = their sum) */
	uint64_t n_reads, n_bases, n_retry, n_chunks;
	uint64_t seed_positions; /* k-mer positions probed by the seed kernel (both strands) */
	uint64_t n_launch_dela;  /* launches of the scoring kernel (2 per chunk when part A was split) */
	uint64_t n_launch_phase; /* launches of each part-A phase kernel (1 per chunk, 2 when the halves are pipelined) */
	uint64_t stats[DSB_N_STATS]; /* work counters DSB_ST_*: [32*ph, 32*ph+32) phase ph, [288,320) k_classB */
	uint64_t n_ws_shrink;    /* chunks re-partitioned smaller because their workspace did not fit in the free HBM */
	uint64_t n_heavy;        /* scoring reads launched first as heavy (chains x length, kernels.hip k_split) */
	uint64_t n_defer_heavy;  /* heavy reads whose scoring went to the batch's re-run group (DSB_HEAVY_DEFER) */
} dsb_gpu_timing;

/* Upload the index to `device`; -1: the DSB_DEVICES list ("all" or "0,1,..."), else the
 * DSB_DEVICE env var, else the current HIP device.  Returns 0; on failure fills err. */
int dsb_gpu_init(dsb_index *ix, int device, char *err, size_t errn);
void dsb_gpu_free(dsb_index *ix);

/* Classify reads[0..n).  *max_read_l is the carried Classify_buff_pool.max_read_l (in/out).
 * ro[n] receives the per-read results; *hits (malloc'd, caller frees) the compact hit records,
 * read i owning hits[ro[i].hit_off .. + ro[i].n_hit).  stats_on: collect work counters. */
int dsb_gpu_classify(dsb_index *ix, const dsb_reads_t *reads, int *max_read_l, dsb_read_out_t *ro,
		     dsb_hit_out_t **hits, uint64_t *n_hits, int stats_on, dsb_gpu_timing *timing, char *err,
		     size_t errn);

/* Batches: reads resident in HBM, classified by one or more runs. */
typedef struct dsb_gpu_batch dsb_gpu_batch;
int dsb_gpu_batch_upload(dsb_index *ix, const dsb_reads_t *reads, dsb_gpu_batch **b, dsb_gpu_timing *timing,
			 char *err, size_t errn);
int dsb_gpu_batch_run(dsb_index *ix, dsb_gpu_batch *b, int *max_read_l, int stats_on, dsb_gpu_timing *timing,
		      char *err, size_t errn);
const dsb_read_out_t *dsb_gpu_batch_ro(const dsb_gpu_batch *b);
const dsb_hit_out_t *dsb_gpu_batch_hits(const dsb_gpu_batch *b);
const int32_t *dsb_gpu_batch_carry(const dsb_gpu_batch *b);
uint64_t dsb_gpu_batch_n(const dsb_gpu_batch *b);
uint64_t dsb_gpu_batch_bases(const dsb_gpu_batch *b);
void dsb_gpu_batch_free(dsb_index *ix, dsb_gpu_batch *b);
/* per-taxon weights of the last run into dev_counts[0, n_counts) on the index's GPU (zeroed
 * first): the per-read taxa come from classB (dsb_read_taxon); weights[i] (host, NULL = 1) */
int dsb_gpu_batch_counts(dsb_index *ix, dsb_gpu_batch *b, const uint32_t *weights, uint64_t *dev_counts,
			 uint64_t n_counts, char *err, size_t errn);

/* The carried max_read_l of a stream of batches (the reference's one buffer pool per
 * read_classify thread, cly.c:2953): carry_in blocks until the batch before has published its
 * carry-out; carry_out publishes this batch's (called after its part A, before its part B).
 * A batch holds its GPU context's run lock while it waits for the carry, so the batches of one
 * stream must take their run locks in stream order, or two streams sharing the contexts can each
 * hold the lock the other's earlier batch needs: lock_wait (before the run lock, may block until
 * the batch before has taken its own) and locked (right after) keep that order.  Any of the
 * hooks may be NULL. */
typedef struct {
	int (*carry_in)(void *ctx);
	void (*carry_out)(void *ctx, int carry);
	void *ctx;
	void (*lock_wait)(void *ctx);
	void (*locked)(void *ctx);
} dsb_carry_hooks;
int dsb_gpu_batch_run_chain(dsb_index *ix, dsb_gpu_batch *b, int stats_on, const dsb_carry_hooks *hooks,
			    dsb_gpu_timing *timing, char *err, size_t errn);
/* Upload reads to GPU `slot` of the index (0 .. n_devices-1) through pinned staging on the
 * device's copy stream, without its run lock (overlaps the batch before).  The records' bases
 * are gathered by `pool`; *ms_gather += the gather time.  Recycle the batch when done. */
int dsb_gpu_batch_stage(dsb_index *ix, int slot, const dsb_reads_t *reads, dsb_pool *pool, dsb_gpu_batch **b,
			double *ms_gather, char *err, size_t errn);
void dsb_gpu_batch_recycle(dsb_index *ix, dsb_gpu_batch *b);
int dsb_gpu_batch_device(const dsb_index *ix, const dsb_gpu_batch *b);
int dsb_gpu_n_devices(const dsb_index *ix);
/* before a streamed call of batches of up to max_reads reads: split each GPU's workspace HBM
 * between its contexts and size their buffers for such batches (kernels.hip) */
int dsb_gpu_fit_contexts(dsb_index *ix, uint64_t max_reads, char *err, size_t errn);
int dsb_gpu_device_id(const dsb_index *ix, int slot);

/* Number of visible devices (0 if HIP has none). */
int dsb_gpu_device_count(void);

#ifdef __cplusplus
}
#endif
#endif
