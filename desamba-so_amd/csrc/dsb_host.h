/*
 * dsb_host.h — host-side (C) part of the MI355X deSAMBA classify library.
 *
 * The host owns everything the reference does outside classify_seq: index files,
 * FASTQ/FASTA parsing with the reference's kseq + kt_pipeline batch semantics,
 * SAM formatting, the taxonomy and meta_analysis.  The classify path itself runs in
 * HIP kernels behind dsb_gpu.h.
 */
#ifndef DSB_HOST_H
#define DSB_HOST_H
#include <stdint.h>
#include <stddef.h>
#include <pthread.h>
#include <string.h>
#include "dsb_types.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ index */
#define DSB_MAX_GPUS 16
typedef struct {
	uint32_t p_tid;
	char rank[20];
	char name[201];
} dsb_taxon_t; /* TAXONOMY_rank (idx.h:11-15) */

typedef struct dsb_index {
	/* host copies (big tables are released after the device upload unless kept) */
	uint8_t *bwt_occ; uint64_t byteLen;  /* the file's 168-B blocks (freed after the re-layout) */
	uint64_t *occ; uint64_t n_occ_line; /* HBM layout, dsb_types.h */
	uint64_t *occ_super; uint64_t n_occ_super;
	uint64_t dollar_row[DSB_MAX_DOLLAR]; int n_dollar;
	uint64_t rank[6];
	uint64_t *hash_index;
	dsb_sa_t *sa; uint64_t sa_size;
	uint64_t dollor_pos;
	uint8_t *ek0, *ek1; uint64_t ek_size, ek_mask; int l_ek, single_base_max;
	dsb_unitig_t *uni; uint64_t n_uni;
	uint8_t *ref_bin; uint64_t ref_bin_n, ref_bin_padded;
	uint64_t n_ref;
	char (*ref_name)[128];
	uint32_t *ref_tid;        /* taxid of each reference name ("tid|<taxid>|...", cly_mt.c:778-786) */
	uint32_t *p_tid;          /* parent taxid per taxid (tax[].p_tid), max_tid + 1 entries */
	uint64_t *ref_seq_l, *ref_seq_offset;
	uint64_t *r_p; uint64_t n_rp;
	int *Q_MEM;               /* DSB_Q_MEM_PAD */
	int Q_LV[DSB_LV_DIM * DSB_LV_DIM];
	int filter_min_length, filter_min_score, filter_min_score_LV3;
	/* taxonomy (cly_mt.c:590-670) */
	dsb_taxon_t *tax; uint64_t max_tid;
	/* device side (gpu/kernels.hip): the index replicated on n_gpu GPUs; gpu == gpus[0] */
	void *gpu;
	void *gpus[DSB_MAX_GPUS];
	int n_gpu;
	void *pool;               /* host thread pool of the read_classify pipeline (pool.c) */
	/* per-thread_id state (cly_mt.c:1279-1307) */
	pthread_mutex_t state_mutex;
	struct dsb_thread_state *states;
} dsb_index;

/* Load deSAMBA.{bwt,sa,exk0,exk1,exki,unv,ref_b,ref_i,ref_p} (idx.c:1103-1160, bwt.c:68-104).
 * Returns 0 on success; on failure writes a message to err. */
int dsb_index_load_files(dsb_index *ix, const char *dir, char *err, size_t errn);
/* only the .bwt (occ re-laid out for HBM, rank, and the 13-mer hash index when with_hash) */
int dsb_index_load_bwt(dsb_index *ix, const char *dir, int with_hash, char *err, size_t errn);
/* MAPQ tables (cly_mt.c:396-420), P_E 0.15, L_REF = 4 * ref_bin.n */
void dsb_mapq_tables(dsb_index *ix, double P_E, uint64_t L_REF);
/* Taxonomy (cly_mt.c:590-670). Returns 0 on success. */
int dsb_taxonomy_load(dsb_index *ix, const char *dir, char *err, size_t errn);
void dsb_index_free_host_tables(dsb_index *ix);
/* Fill a dsb_dindex_t with the host pointers (CPU emulation / tests only) */
void dsb_index_host_view(const dsb_index *ix, dsb_dindex_t *d);

/* ------------------------------------------------------------------ reads */
/* One read as kseq_read leaves it (utils.c:939-977).  The strings are views into the resident
 * input text, or into the parser's arena (records kseq assembles from several lines); they are
 * not NUL-terminated in general, and the SAM writer prints them like printf's %s does (up to
 * the first NUL within the length).  qual == NULL: qual.s was never set ("(null)"); a FASTA
 * record's qual is its slot's stale quality string (cly_mt.c:229-327 prints qual.s). */
typedef struct {
	const char *name, *seq, *qual;
	uint32_t name_l, seq_l, qual_l;
	uint32_t pad;
} dsb_rec_t;

typedef struct {
	dsb_rec_t *rec; uint64_t n, m;
	void *arena_owner; /* arena chunks these records point into (dsb_parse_reads), freed with them */
	char *text_owner;  /* an owned copy of the input text the records view (dsb_batch_create) */
} dsb_reads_t;

/* Parse `len` bytes of FASTQ/FASTA text with the semantics of read_reads + kseq_read +
 * kt_pipeline (cly_mt.c:29-43,361-381; utils.c:841-977; kthread.c:114-197).  The records view
 * `buf`, which must outlive them. */
int dsb_parse_reads(const char *buf, uint64_t len, dsb_reads_t *out);
/* The same as a stream of batches over resident text: each call appends whole kt_pipeline
 * batches until >= max_reads records or >= max_bases bases were added; returns the number of
 * records appended (0: end of input).  Records stay valid until dsb_parser_free. */
typedef struct dsb_parser dsb_parser;
dsb_parser *dsb_parser_new(const char *buf, uint64_t len);
void dsb_parser_set_fast(dsb_parser *p, int fast);
uint64_t dsb_parser_next(dsb_parser *p, dsb_reads_t *out, uint64_t max_reads, uint64_t max_bases);
void dsb_parser_stats(const dsb_parser *p, uint64_t *n_fast, uint64_t *n_slow);
uint64_t dsb_parser_left(const dsb_parser *p); /* input bytes not yet read (estimate) */
void dsb_parser_free(dsb_parser *p);
/* One kseq_t over resident text (the evaluation tools): kseq_read's return value; the accessors
 * return its buffers (NULL if never set; stale content kept as the reference keeps it). */
typedef struct dsb_kseq1 dsb_kseq1;
dsb_kseq1 *dsb_kseq1_open(const char *buf, uint64_t len);
int64_t dsb_kseq1_read(dsb_kseq1 *k);
const char *dsb_kseq1_name(const dsb_kseq1 *k);
const char *dsb_kseq1_comment(const dsb_kseq1 *k);
const char *dsb_kseq1_seq(const dsb_kseq1 *k);
const char *dsb_kseq1_qual(const dsb_kseq1 *k);
uint64_t dsb_kseq1_seq_l(const dsb_kseq1 *k);
void dsb_kseq1_close(dsb_kseq1 *k);
/* read a whole (optionally gzip) file or memory buffer (gzip auto-detected) */
int dsb_slurp_path(const char *path, char **buf, uint64_t *len);
int dsb_open_path(const char *path, char **buf, uint64_t *len, uint64_t *unmap_len);
int dsb_inflate_if_gzip(const char *in, uint64_t in_n, char **buf, uint64_t *len, int *owned);
void dsb_reads_free(dsb_reads_t *r);

/* ------------------------------------------------------------------ host thread pool */
/* fn(ctx, task, worker) for every task in [0, n_tasks), spread over the pool's threads and the
 * calling thread; returns when all are done.  Several threads may run jobs at once. */
typedef struct dsb_pool dsb_pool;
dsb_pool *dsb_pool_new(int n_threads);
int dsb_pool_size(const dsb_pool *p);
void dsb_pool_run(dsb_pool *p, uint64_t n_tasks, void (*fn)(void *ctx, uint64_t task, int worker), void *ctx);
void dsb_pool_free(dsb_pool *p);
int dsb_host_threads(void);

/* ------------------------------------------------------------------ output */
typedef struct { char *s; uint64_t l, m; } dsb_str;
void dsb_str_put(dsb_str *s, const char *p, uint64_t n);
void dsb_str_printf(dsb_str *s, const char *fmt, ...);

enum { DSB_OUT_SAM = 1, DSB_OUT_SAM_FULL = 2, DSB_OUT_DES = 3, DSB_OUT_DES_FULL = 4 };
void dsb_format_read(dsb_str *out, const dsb_index *ix, const dsb_reads_t *r, uint64_t i,
		     const dsb_read_out_t *ro, const dsb_hit_out_t *hits, int format, int max_sec_N);
void dsb_sam_seq_qual(const dsb_rec_t *rec, const char **seq, uint64_t *seq_n, const char **qual, uint64_t *qual_n);
/* the same records; SAM_FULL with hole != NULL leaves out "SEQ\tQUAL" (*hole_n bytes) and sets
 * *hole to the offset in out where they go (*hole = UINT64_MAX: no hole) */
void dsb_format_read_hole(dsb_str *out, const dsb_index *ix, const dsb_reads_t *r, uint64_t i, const dsb_read_out_t *ro,
			  const dsb_hit_out_t *hits, int format, int max_sec_N, uint64_t *hole, uint64_t *hole_n);
/* printed length of a %s argument held as (p, n): up to the first NUL */
static inline uint64_t dsb_cstr_len(const char *p, uint64_t n) { return p ? strnlen(p, n) : 0; }

/* ------------------------------------------------------------------ meta analysis */
int dsb_meta_analysis(dsb_index *ix, const char *input, uint64_t input_n, char **output, uint64_t *output_n,
		      int flag, uint64_t max_snapshot_len, char **human_snapshot, uint64_t *human_snapshot_n);

#ifdef __cplusplus
}
#endif
#endif
