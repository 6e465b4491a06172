/*
 * dsb_types.h — plain-old-data types shared by the C host code and the HIP kernels.
 *
 * Everything on the classify path is integer arithmetic; widths mirror the reference
 * exactly because the reference relies on uint32 wrap-around in several places
 * (SURVEY Appendix A, H11).  Reference citations are to /root/reference/src.
 */
#ifndef DSB_TYPES_H
#define DSB_TYPES_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* SA sample, one per 8 BWT rows (bwt.h:6-13) */
typedef struct { uint32_t unitig_ID, offset; } dsb_sa_t;
/* UNITIG (idx.h:28-32); the loader appends a sentinel (idx.c:1127) */
typedef struct { uint32_t ref_list, length; } dsb_unitig_t;

/* REF_POS (idx.h:42-48): u64 bitfield {global_offset:40, ref_ID:23, direction:1} */
#define DSB_RP_OFF(x) ((x) & 0xFFFFFFFFFFull)
#define DSB_RP_REF(x) ((uint32_t)(((x) >> 40) & 0x7FFFFF))

/* Constants of the classify path (src/idx.h, src/cly.c) */
#define DSB_L_PRE_IDX 13
#define DSB_PRE_IDX_MASK 0x3FFFFFFull
#define DSB_Q_MEM_MAX 2000
#define DSB_Q_MEM_PAD 4096  /* device copy padded; see DESIGN.md "unpinned corners" */
#define DSB_LV_DIM 20
#define DSB_MIN_UNI_L 35
#define DSB_MIN_READ_LEN 40
#define DSB_MAX_DOLLAR 4     /* '$' symbols in the BWT the HBM occ layout supports (one in practice) */
#define DSB_OCC_LINE_U64 8   /* u64 words per occ line (64 B) */
#define DSB_OCC_LINE_SYM 128 /* BWT symbols per occ line */
#define DSB_OCC_SUPER_SHIFT 17 /* lines per superblock: 2^17 (2^24 symbols; line counts are relative to it) */

/*
 * Device-visible index: raw pointers into HBM (or host memory for the
 * kernel-logic CPU emulation used only by tests).
 */
typedef struct {
	/* occ/rank table re-laid out for HBM: one 64-B line per 128 BWT symbols,
	 * u32 cnt[4] (occ of A,C,G,T at the line start, relative to its superblock) | u64 sym[4]
	 * (2-bit symbols, 32 per word, '#'/'$' stored as 0) | u64 spc[2] (1 = '#' or '$', 64 per
	 * word); occ_super: u64 cnt[4] at the start of every 2^DSB_OCC_SUPER_SHIFT lines.  Replaces
	 * the reference's 168-B blocks (bwt.c:32-42) losslessly: '$' rows are listed below and the
	 * '#' count is line start - A - C - G - T - '$' before it. */
	const uint64_t *occ;
	const uint64_t *occ_super;
	uint64_t n_occ_line;
	uint64_t dollar_row[DSB_MAX_DOLLAR];
	int n_dollar;
	uint64_t rank[6];            /* rank[5] = rank[0]-1 (bwt.c:81) */
	const uint64_t *hash_index;  /* (2^26+1) u64, 13-mer prefix -> SA interval (bwt.c:83-85) */
	const dsb_sa_t *sa;
	uint64_t sa_size;
	uint64_t dollor_pos;         /* unitig_v.n - 2 (idx.c:1128) */
	const uint8_t *ek0, *ek1;    /* e-kmer Bloom tables (idx.c:1108-1121) */
	uint64_t ek_size, ek_mask;
	int l_ek, single_base_max;   /* set_ekmer_par (idx.c:966-982) */
	const dsb_unitig_t *uni;     /* n_uni + 1 entries (sentinel) */
	uint64_t n_uni;
	const uint8_t *ref_bin;      /* 2-bit MSB-first packed reference, zero padded */
	uint64_t ref_bin_n;          /* bytes in the file (padding not counted) */
	uint64_t ref_bin_padded;     /* bytes readable */
	const uint64_t *ref_seq_offset, *ref_seq_l; /* REF_INFO (idx.h:22-26) minus the name */
	uint64_t n_ref;
	const uint64_t *r_p;         /* REF_POS raw */
	uint64_t n_rp;
	const int *Q_MEM;            /* DSB_Q_MEM_PAD ints */
	const int *Q_LV;             /* [20][20] row-major: Q_LV[ed*20 + len] */
	int filter_min_length, filter_min_score, filter_min_score_LV3;
	/* taxonomy for the per-read taxon (meta_analysis' ana_get_tid): taxid of each reference and
	 * parent taxid of every taxid <= max_tid (0xffffffff: none) */
	const uint32_t *ref_tid;
	const uint32_t *p_tid;
	uint64_t max_tid;
	/* seeding sp_set pool (GPU build, dsb_classify.h DSB_HSET_POOL): hpool_nx partitions (one per
	 * XCD) of hpool_part wave-sized sets (DSB_HSET_WAVE_U64 words each), an owner flag and a
	 * generation base per set; hpool_part is a power of two >= the waves an XCD can hold at once,
	 * so an acquiring wave always finds one in its XCD's partition (dsb_kern.h).  hpool_fenced:
	 * the XCC ids the device's waves report were not exactly 0..hpool_nx-1 at load (or the XCC
	 * count was unknown), so one partition is used and every hand-over is an agent-scope
	 * release / acquire (kernels.hip dev_init). */
	uint64_t *hpool;
	uint32_t *hpool_own;
	uint64_t *hpool_gen;
	uint32_t hpool_part, hpool_nx, hpool_fenced;
} dsb_dindex_t;

/* Output record per hit (what output_one_result_sam needs, cly_mt.c:229-327) */
typedef struct {
	uint32_t ref_ID;
	uint32_t sum_score;
	uint32_t t_st, t_ed, q_st, q_ed;
	uint32_t indel;
	uint8_t direction, primary, pri_index, pad;
} dsb_hit_out_t;

/*
 * The taxon meta_analysis assigns a read from its records (ana_get_tid, reference
 * src/cly_mt.c:902-961), taken from the hits in the order output_one_result_sam prints them
 * (src/cly_mt.c:229-327: primary, supplementaries (pri_index 0), secondaries (pri_index 1..5)):
 * the first record's taxid, replaced by a later record of equal score whose taxid descends from
 * the current one.  0 = unclassified.  Shared by the host (dsb_batch_taxa) and the classB kernel.
 */
#if defined(__HIPCC__)
#define DSB_TAX_HD __host__ __device__ static inline
#else
#define DSB_TAX_HD static inline
#endif
DSB_TAX_HD uint32_t dsb_read_taxon(const dsb_hit_out_t *h, uint32_t nh, const uint32_t *ref_tid, const uint32_t *p_tid,
				   uint64_t max_tid)
{
	if (nh == 0)
		return 0;
	uint32_t tid = 0, score = 0;
	uint32_t t0 = ref_tid[h[0].ref_ID];
	if (t0 <= max_tid) {
		tid = t0;
		score = h[0].sum_score;
	}
	for (int loop = 0; loop <= 1 && score != 0; loop++)
		for (uint32_t k = 1; k < nh && score != 0; k++) {
			int printed = loop == 0 ? h[k].pri_index == 0 : (h[k].pri_index > 0 && h[k].pri_index <= 5);
			if (!printed || h[k].sum_score != score)
				continue;
			uint32_t rt = ref_tid[h[k].ref_ID];
			if (rt > max_tid)
				continue;
			for (uint32_t pt = rt;; pt = p_tid[pt]) {
				if (pt == tid) {
					tid = rt;
					break;
				}
				if (pt < 1 || pt == 4294967295u || pt > max_tid)
					break;
			}
		}
	return tid;
}

/* Per-read result summary */
typedef struct {
	uint32_t n_hit;        /* hits written to the read's output slot */
	uint32_t n_anchor;     /* anchor_v.n at the end (DES output) */
	uint32_t fast;         /* results->fast_classify */
	uint32_t status;       /* 0 ok; bit0 overflow (re-run with larger workspace) */
	uint32_t reached_update; /* read reached the max_read_l update (cly.c:2953) */
	uint32_t pad;
	uint64_t hit_off;      /* index of the read's first hit in the compact hit array */
} dsb_read_out_t;

#ifdef __cplusplus
}
#endif
#endif
