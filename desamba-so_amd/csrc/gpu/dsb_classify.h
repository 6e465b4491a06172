/*
 * dsb_classify.h — the per-read classify path (reference classify_seq, src/cly.c:3059-3127)
 * restated for one GPU lane per read, over a per-read workspace carved from HBM.
 *
 * Pointers of the reference (chain_anchor_pre, chain_anchor_cur, SEARCH_DIR members) are
 * indices here; dynamic vectors (kvec) are fixed-capacity arrays whose overflow marks the
 * read for a second pass with a larger workspace (never a CPU fallback).
 */
#ifndef DSB_CLASSIFY_H
#define DSB_CLASSIFY_H
#include "dsb_core.h"
#include "dsb_wave.h"

/* Sequential variants of the wave loops (w->dbg bits 1, 2, 4, 8, 64) exist for the host
 * emulation and diagnostics builds only; device builds compile them out (-DDSB_WAVE_DIAG=1
 * keeps them). */
#ifndef DSB_WAVE_DIAG
#if defined(__HIP_DEVICE_COMPILE__)
#define DSB_WAVE_DIAG 0
#else
#define DSB_WAVE_DIAG 1
#endif
#endif
#define DSB_SEQ(w, bit) (DSB_WAVE_DIAG && ((w)->dbg & (bit)))

/* ------------------------------------------------------------------ per-read types */
typedef struct { uint32_t offset, len; uint8_t top, p0, p1, p2; } dsb_seed_t; /* CLY_seed, cly.h:27-32 */

typedef struct { /* Anchor, cly.h:44-61 (pointers -> indices) */
	uint64_t global_offset;
	uint32_t ref_ID, ref_offset, index_in_read;
	int32_t pre;            /* chain_anchor_pre, -1 = NULL */
	uint16_t mtch_len;      /* Anchor_map (cly.h:34-42) */
	int16_t score;
	uint8_t left_len, left_ED, rigt_len, rigt_ED;
	uint16_t seed_ID, chain_id;
	uint8_t direction, anchor_useless, duplicate, pad;
} dsb_anchor_t;

typedef struct { /* chain_item, cly.h:69-89 */
	uint32_t ref_ID;
	int32_t q_t_dis;
	uint32_t sum_score, anchor_number;
	uint8_t direction, with_top_anchor, primary, pri_index;
	uint32_t t_st, t_ed, q_st, q_ed, indel, chain_id;
	int32_t cur;            /* chain_anchor_cur */
} dsb_chain_t;

typedef struct { uint32_t t_pos, q_pos, len, score; } dsb_spd_t; /* spd_match, cly.h:127-133 */

typedef struct { /* MEM_rst, src/cly.c:614-622 */
	int match_len;
	uint64_t sp, sa_sp;
	int sa_sp_l, kmer_index, read_offset;
} dsb_mem_t;

#define DSB_WIN_MID 64
#define DSB_WIN_RL (64 + 2064 + 64)
#define DSB_WIN_BYTES (DSB_WIN_RL + 1064 + 64)
typedef struct { uint16_t next; uint16_t seed_ID_s_or_e; } dsb_sch_t; /* seed_con_hash, cly.h:120-125 */

typedef struct { /* SEARCH_DIR, src/cly.c:941-949 */
	uint32_t seed_off;      /* index of seed_v_f in the seed buffer */
	uint32_t l_seed_v_f;
	uint32_t strand;        /* 0: forward buffer half, 1: reverse half */
	uint32_t direction;
	uint32_t total_score;
} dsb_sdir_t;

/* Anchor_cmp_by_chr_ID_and_pos, src/cly.c:225-234: returns only 0/1 ("a > b"), which under
 * glibc's merge sort is a stable ascending sort by (ref_ID, direction, ref_offset). */
DSB_HD int dsb_anchor_cmp(const dsb_anchor_t *a, const dsb_anchor_t *b)
{
	int r = (a->ref_ID > b->ref_ID);
	int d = (a->direction > b->direction);
	int o = (a->ref_offset > b->ref_offset);
	return (a->ref_ID != b->ref_ID) ? r : ((a->direction != b->direction) ? d : o);
}

/* MEM_rst_cmp_by_match_len, src/cly.c:1325-1328 */
DSB_HD int dsb_mem_cmp(const dsb_mem_t *a, const dsb_mem_t *b)
{
	return b->match_len - a->match_len;
}

/* workspace capacities (elements) */
typedef struct {
	uint32_t anc, hit, sms;
} dsb_caps_t;

/* Per-read workspace (all pointers into the read's arena) */
typedef struct {
	const dsb_dindex_t *ix;
	uint32_t L;             /* read length */
	uint8_t *bin;           /* F at bin[0..L), R at bin[L..2L); guard before/after */
	const uint64_t *exF, *exR; /* exist bits per k-mer position (K_seed output) */
	const uint32_t *pre;    /* k-mer & 0x3FFFFFF per position (K_seed output): F at [0, L), R at [L, 2L) */
	dsb_seed_t *seeds;      /* (L>>1)+20 (+spill) entries; R seeds at L>>2 (src/cly.c:1238,1252) */
	dsb_anchor_t *anc; uint32_t n_anc;
	uint32_t anc_hw;        /* the most anchors the reference's anchor_v held so far in this read (its capacity
	                         * is 10 * 2^k above it: the realloc points of kv_pushp_2, dsb_map_seed) */
	dsb_anchor_t *anc_tmp;
	dsb_anchor_t *anc_tmp2; /* the seeding state machine's second staging pool (cap.anc entries) */
	uint32_t *sidx, *stmp;  /* msort permutation scratch (max(anc, hit) entries) */
	dsb_chain_t *hit; uint32_t n_hit;
	dsb_chain_t *hit_tmp;
	dsb_spd_t *sms; uint32_t n_sms;
	dsb_spd_t *sms_lds;     /* wave scoring: the first DSB_SMS_LDS sms entries live in LDS */
	uint64_t *lds_key;      /* wave chaining: anchor sort keys / ids in LDS (lds_n entries each), or 0 */
	uint32_t *lds_id;
	uint32_t lds_n;         /* entries of lds_key / lds_id: DSB_SORT_LDS, DSB_SORT_LDS_SLOW for the slow resolves */
	uint16_t *lds_cand;     /* wave scoring: 64 candidate slots of the register k-mer match (DSB_MATCH_BF), or 0 */
	uint8_t *lds_q;         /* wave scoring: DSB_QCOPY_BYTES of LDS for a window's read range (DSB_QCOPY), or 0 */
	uint8_t *lds_hb;        /* wave read-hash build: DSB_HB_LDS lane-id bytes in LDS (key groups of a chunk), or 0 */
	uint32_t *hh[2], *hn[2]; /* read 9-mer hash per strand: list heads per key, one node per position */
	dsb_sch_t *sch;         /* 256 + 2*400 */
	dsb_chain_t *spec_ch;   /* speculative scoring of one chain (heavy reads, dsb_kern.h k_heavy_spec): its private */
	uint64_t *spec_bits;    /* copy, and the bitset of the chains it merged (left live in w->hit); else 0 */
	uint16_t *sc_off;       /* the seed_con_hash lists as arrays (wave combine_chain): per key [off, off + 1) */
	uint16_t *sc_flat;      /* into sc_flat, list order; sc_off[256 + k] the tails while the lists are built */
	uint8_t *win;           /* DSB_WIN_BYTES: sdp_middle ref[2000] and sdp_right/left ref[1000] windows */
	dsb_mem_t *mem;         /* 16 MEM results per lane (slow mode) */
	uint64_t *spset;        /* 500 */
	dsb_caps_t cap;
	uint32_t overflow;
	uint32_t fast_classify;
	dsb_sdir_t sd[2];
	int max_read_l;         /* Classify_buff_pool.max_read_l, supplied (H2) */
	uint32_t reached_update;
	/* optional counters for algorithmic-byte accounting (bench) */
	uint64_t *stats;
	uint32_t dbg;           /* diagnostics: force sequential variants of the wave loops */
	uint64_t launch_tag;    /* unique per kernel launch (host counter, never 0, < 2^40): seeding sp_set slot tags */
	uint64_t *tmr;          /* timer kernels: wave clocks per DSB_ST_T_* slot (LDS, lane 0), or 0 */
} dsb_read_ws;

enum { DSB_ST_OCC = 0, DSB_ST_OCC_NIB, DSB_ST_MEMSEARCH, DSB_ST_SA, DSB_ST_UNI, DSB_ST_REFPOS,
       DSB_ST_GETREF_B, DSB_ST_ANCHOR, DSB_ST_CHAIN, DSB_ST_EK1, DSB_ST_EK2,
       DSB_ST_HASH_B,   /* read 9-mer hash: bytes written/read while building it */
       DSB_ST_LOOKUP,   /* reference-window k-mer lookups into that hash (4 B head each) */
       DSB_ST_NODE,     /* hash-list nodes visited by those lookups (8 B each) */
       DSB_ST_T_MEM,    /* seeding: wave clocks of the seed state machine (stats kernels, lane 0) */
       DSB_ST_T_MAP,    /* seeding: wave clocks of its batched map_seed steps (stats kernels, lane 0) */
       /* scoring phase clocks (stats kernels, lane 0) */
       DSB_ST_T_BUILD,  /* build_hash_table_M2 */
       DSB_ST_T_MATCH,  /* sdp_match */
       DSB_ST_T_WIN,    /* reference windows: get_ref */
       DSB_ST_T_ALL,    /* get_score_M2 as a whole */
       DSB_ST_T_DPM,    /* sdp_middle predecessor scans */
       DSB_ST_T_DPS,    /* sdp_right / sdp_left predecessor scans */
       DSB_ST_T_FILL,   /* stack-pattern fills of the windows */
       DSB_ST_PASS2,    /* seeding: seeds run again in the state machine's second pass */
       DSB_ST_REPLAY,   /* seeding: seeds replayed serially by the whole wave (both passes overflowed) */
       DSB_ST_T_MPROBE, /* sdp_match: window probe k-mers + list heads */
       DSB_ST_T_MWALK,  /* sdp_match: list walks + MEM_search extensions */
       DSB_ST_T_COMB,   /* sdp_right / sdp_left: combine_chain */
       DSB_ST_NWIN,     /* sdp_match calls (reference windows matched) */
       DSB_ST_NBATCH,   /* sdp_match: 64-probe batches */
       DSB_ST_NCAND,    /* sdp_match: list entries whose 9-mer and read range match (extended) */
       DSB_ST_NSMS,     /* sdp_right / sdp_left: sparse-DP nodes processed */
       DSB_ST_N };
/* wave clocks of a code region (timer kernels only: lane 0 accumulates into LDS, so that the
 * timing run pays no private-memory traffic for its counters) */
#define DSB_T0() ((w->tmr && dsb_lane() == 0) ? dsb_clock() : 0)
#define DSB_T1(slot, t0) do { if (w->tmr && dsb_lane() == 0) w->tmr[slot] += dsb_clock() - (t0); } while (0)

DSB_HD uint64_t dsb_clock(void)
{
#if defined(__HIP_DEVICE_COMPILE__)
	return __builtin_amdgcn_s_memtime();
#else
	return 0;
#endif
}

/*
 * Work accounting (stats kernels only; w->stats == 0 otherwise).  The byte figures are the
 * algorithmic bytes of DESIGN.md §Roofline: 8 B checkpoint + the nibble bytes up to r in
 * the 256-symbol occ block, 8 B per SA sample / unitig entry / ref_pos entry, 2 bits per
 * reference base unpacked.
 */
DSB_HD void dsb_stat_occ(dsb_read_ws *w, uint64_t r)
{
	if (w->stats) {
		w->stats[DSB_ST_OCC]++;
		w->stats[DSB_ST_OCC_NIB] += 8 + 2 * (((r & 255) >> 2) + 1);
	}
}
DSB_HD uint64_t dsb_lf_w(dsb_read_ws *w, uint64_t r, uint8_t *c)
{
	dsb_stat_occ(w, r);
	return dsb_lf(w->ix, r, c);
}
DSB_HD uint64_t dsb_occ_w(dsb_read_ws *w, uint64_t r, uint8_t *c)
{
	dsb_stat_occ(w, r);
	return dsb_occ(w->ix, r, c);
}
DSB_HD void dsb_get_ref_w(dsb_read_ws *w, uint8_t *ref_str, uint64_t uni_offset, uint32_t length, int isForward)
{
	if (w->stats) w->stats[DSB_ST_GETREF_B] += (length + 3) / 4;
	dsb_get_ref(w->ix, ref_str, uni_offset, length, isForward);
}

DSB_HD int dsb_exist_bit(const uint64_t *ex, uint32_t k)
{
	return (int)((ex[k >> 6] >> (k & 63)) & 1);
}

/* diagnostics (dbg 256): is [p+lo, p+hi) inside the read's window buffer? */
DSB_HD int dsb_win_ok(const dsb_read_ws *w, const uint8_t *p, int64_t lo, int64_t hi, int tag)
{
#if defined(__HIP_DEVICE_COMPILE__) && DSB_WAVE_DIAG
	if (w->dbg & 256) {
		int64_t a = (int64_t)(p - w->win) + lo, b = (int64_t)(p - w->win) + hi;
		if (a < 0 || b > DSB_WIN_BYTES) {
			printf("[dsb] window access [%ld,%ld) outside [0,%d) tag %d lane %u\n", (long)a, (long)b, DSB_WIN_BYTES,
			       tag, dsb_lane());
			return 0;
		}
	}
#endif
	(void)w; (void)p; (void)lo; (void)hi; (void)tag;
	return 1;
}

/* ------------------------------------------------------------------ seeding */
/* search_exist_kmer_M2, src/cly.c:1066-1155, on precomputed exist bits */
/* exist-bit reader keeping the last 64-bit word in a register (the scan revisits it ~20x) */
typedef struct { const uint64_t *ex; uint32_t wi; uint64_t word; } dsb_bitrd_t;
DSB_HD int dsb_bit(dsb_bitrd_t *b, uint32_t i)
{
	uint32_t wi = i >> 6;
	if (wi != b->wi) {
		b->wi = wi;
		b->word = b->ex[wi];
	}
	return (int)((b->word >> (i & 63)) & 1);
}

/* positions p with p % 3 == rho inside a 64-bit word (64 % 3 == 1) */
DSB_HD uint64_t dsb_mask3(uint32_t rho)
{
	const uint64_t M0 = 0x9249249249249249ull; /* bits 0, 3, ..., 63 */
	return rho == 0 ? M0 : (rho == 1 ? (M0 << 1) : (M0 << 2));
}
/* smallest p >= i with p == i (mod 3), p < n and exist bit p set; n if none */
DSB_HD uint32_t dsb_next_set3(const uint64_t *ex, uint32_t i, uint32_t n)
{
	uint32_t r3 = i % 3;
	while (i < n) {
		uint32_t w = i >> 6, b = i & 63;
		uint64_t bits = ex[w] & dsb_mask3((r3 + 3 - (w << 6) % 3) % 3) & (~0ull << b);
		if (bits) {
			uint32_t p = (w << 6) + (uint32_t)__builtin_ctzll(bits);
			return p < n ? p : n;
		}
		uint32_t nx = (w + 1) << 6;
		i = nx + (r3 + 3 - nx % 3) % 3;
	}
	return n;
}
/* largest p <= i with p == i (mod 3) and exist bit p set; -1 if none */
DSB_HD int dsb_prev_set3(const uint64_t *ex, int i)
{
	uint32_t r3 = (uint32_t)i % 3;
	while (i >= 0) {
		uint32_t w = (uint32_t)i >> 6, b = (uint32_t)i & 63;
		uint64_t upto = (b == 63) ? ~0ull : ((2ull << b) - 1);
		uint64_t bits = ex[w] & dsb_mask3((r3 + 3 - (w << 6) % 3) % 3) & upto;
		if (bits)
			return (int)((w << 6) + 63 - (uint32_t)__builtin_clzll(bits));
		if (w == 0)
			return -1;
		int last = (int)(w << 6) - 1;
		i = last - (int)(((uint32_t)last % 3 + 3 - r3) % 3);
	}
	return -1;
}

#ifndef DSB_NEED_STATS
#define DSB_NEED_STATS 0 /* dev: count the exist bits the scan reads (dsb_search_exist's *need) */
#endif
DSB_HD uint32_t dsb_search_exist(const uint64_t *ex_, uint32_t l_kmer_v, dsb_seed_t *seed_v, uint32_t direction,
				 uint64_t *need = nullptr)
{
	uint32_t l_seed_v = 0;
	uint64_t nd = 0;
	dsb_bitrd_t br = {ex_, 0xffffffffu, 0};
	dsb_bitrd_t *ex = &br;
	const uint32_t STEP_EK = 3;
	/* the candidate positions (every 3rd k-mer, restarting after each seed) are found a word
	 * at a time (dsb_next_set3 / dsb_prev_set3) instead of bit by bit */
	if (direction == DSB_FORWARD) {
		for (uint32_t i = STEP_EK - 1; i < l_kmer_v; i += STEP_EK) {
			uint32_t i0 = i;
			i = dsb_next_set3(ex_, i, l_kmer_v);
			if (DSB_NEED_STATS) nd += (DSB_MIN(i, l_kmer_v - 1) - i0) / 3 + 1;
			if (i >= l_kmer_v)
				break;
			uint32_t offset = i, len = 1;
			for (int j = 1; j < (int)STEP_EK; ++j) {
				if (DSB_NEED_STATS) nd++;
				if (dsb_bit(ex, i - j)) { offset--; len++; }
				else break;
			}
			for (int j = 1; i + j < l_kmer_v; ++j) {
				if (DSB_NEED_STATS) nd++;
				if (dsb_bit(ex, i + j)) {
					len++;
					if (len > 60) break; /* the i += 50 is overwritten below */
				} else break;
			}
			seed_v[l_seed_v].offset = offset;
			seed_v[l_seed_v].len = len;
			l_seed_v++;
			i = offset + len;
		}
	} else {
		for (int i = (int)l_kmer_v - (int)STEP_EK; i >= 0; i -= STEP_EK) {
			int i0 = i;
			i = dsb_prev_set3(ex_, i);
			if (DSB_NEED_STATS) nd += (uint64_t)((i0 - DSB_MAX(i, 0)) / 3 + 1);
			if (i < 0)
				break;
			uint32_t offset = i, len = 1;
			for (int j = 1; j < (int)STEP_EK; ++j) {
				if (DSB_NEED_STATS) nd++;
				if (dsb_bit(ex, (uint32_t)(i + j))) { offset++; len++; }
				else break;
			}
			for (int j = 1; j <= i; ++j) {
				if (DSB_NEED_STATS) nd++;
				if (dsb_bit(ex, (uint32_t)(i - j))) {
					len++;
					if (len > 60) break;
				} else break;
			}
			seed_v[l_seed_v].offset = offset - len + 1;
			seed_v[l_seed_v].len = len;
			l_seed_v++;
			i = (int)(offset - len);
		}
	}
	if (need)
		*need += nd;
	return l_seed_v;
}

/* search_exist_kmer_M2 (src/cly.c:1066-1155) in batches of G positions (k_island_g).
 *
 * The scan reads the exist bit of only part of the k-mer positions (every 3rd one between
 * seeds, the two neighbours behind a hit, the run of hits after it: 42% of them on C1), so the
 * island kernel probes the Bloom tables itself instead of k_seed probing every position of both
 * strands up front.  G lanes scan one strand together: a GRID batch is the next G positions of
 * the scan's stride-3 grid (i, i+3, ...; backwards i, i-3, ... for the reverse scan), the first
 * set bit among them is the hit the reference's loop stops at; a RUN1 batch is the hit's two
 * back neighbours + the first G-2 positions of the run after it; RUN batches continue the run
 * G positions at a time.  Every batch's bits are probed together (one round trip), the state
 * update below is the reference loop's over those bits, so the seeds equal dsb_search_exist's
 * for any batch sizes >= 4 (tests/emu/isl_check.cpp replays both over the same bits). */
#ifndef DSB_ISLAND_G
#define DSB_ISLAND_G 16 /* lanes per strand (k_island_g); 0: k_seed's exist bits + the two-lane k_island */
#endif
enum { DSB_ISL_GRID = 0, DSB_ISL_RUN1, DSB_ISL_RUN, DSB_ISL_DONE };
typedef struct {
	int32_t mode, i, h, off, ln, p, nk, fwd;
} dsb_isl_t;

DSB_HD void dsb_isl_init(dsb_isl_t *s, int nk, int fwd, int live)
{
	s->nk = nk;
	s->fwd = fwd;
	s->i = fwd ? 2 : nk - 3; /* for (i = STEP_EK - 1; ...) / for (i = l_kmer_v - STEP_EK; ...) */
	s->h = s->off = s->ln = s->p = 0;
	s->mode = (live && (fwd ? s->i < nk : s->i >= 0)) ? DSB_ISL_GRID : DSB_ISL_DONE;
}

/* Batch shapes: a grid batch is GG positions of the stride-3 grid; the first run batch after a
 * hit (RUN1) is its two back neighbours + GR1 - 2 positions after it (most runs are short: on
 * the ONT fixture half of the seeds are <= 10 long); the later run batches are GR positions, and
 * never more than the run can still read: the scan stops at the position that makes the seed 61
 * long (len > 60), so a run at length ln reads at most 61 - ln. */
template <int GR>
DSB_HD int dsb_isl_rw(const dsb_isl_t *s) { return DSB_MIN(GR, 61 - s->ln); }

/* the position lane gl of the strand's lanes probes in this batch (GG positions per grid
 * batch, GR per run batch); -1: none */
template <int GG, int GR, int GR1 = GR>
DSB_HD int dsb_isl_pos(const dsb_isl_t *s, int gl)
{
	int d = s->fwd ? 1 : -1, q;
	switch (s->mode) {
	case DSB_ISL_GRID: if (gl >= GG) return -1; q = s->i + 3 * d * gl; break;
	case DSB_ISL_RUN1: if (gl >= GR1) return -1; q = gl < 2 ? s->h - d * (gl + 1) : s->h + d * (gl - 1); break;
	case DSB_ISL_RUN: if (gl >= dsb_isl_rw<GR>(s)) return -1; q = s->p + d * gl; break;
	default: return -1;
	}
	return (q >= 0 && q < s->nk) ? q : -1;
}

/* the lowest and highest position the batch probes (lo > hi: none) */
template <int GG, int GR, int GR1 = GR>
DSB_HD void dsb_isl_span(const dsb_isl_t *s, int *lo, int *hi)
{
	int a = 0, b = -1, rw = dsb_isl_rw<GR>(s);
	if (s->fwd) {
		switch (s->mode) {
		case DSB_ISL_GRID: a = s->i; b = s->i + 3 * DSB_MIN(GG - 1, (s->nk - 1 - s->i) / 3); break;
		case DSB_ISL_RUN1: a = s->h - 2; b = DSB_MIN(s->h + GR1 - 2, s->nk - 1); break;
		case DSB_ISL_RUN: a = s->p; b = DSB_MIN(s->p + rw - 1, s->nk - 1); break;
		}
	} else {
		switch (s->mode) {
		case DSB_ISL_GRID: b = s->i; a = s->i - 3 * DSB_MIN(GG - 1, s->i / 3); break;
		case DSB_ISL_RUN1: b = s->h + 2; a = DSB_MAX(s->h - (GR1 - 2), 0); break;
		case DSB_ISL_RUN: b = s->p; a = DSB_MAX(s->p - (rw - 1), 0); break;
		}
	}
	*lo = a;
	*hi = b;
}

/* one batch: bit g of mb = exist bit of dsb_isl_pos(s, g).  Returns 1 when a seed closes
 * (*so, *sl = CLY_seed offset / len as search_exist_kmer_M2 stores them). */
template <int GG, int GR, int GR1 = GR>
DSB_HD int dsb_isl_step(dsb_isl_t *s, uint32_t mb, uint32_t *so, uint32_t *sl)
{
	int d = s->fwd ? 1 : -1;
	if (s->mode == DSB_ISL_GRID) {
		if (mb) { /* the first set grid position: a seed starts there */
			s->h = s->i + 3 * d * (int)__builtin_ctz(mb);
			s->off = s->h;
			s->ln = 1;
			s->mode = DSB_ISL_RUN1;
		} else {
			s->i += 3 * d * GG;
			if (s->fwd ? s->i >= s->nk : s->i < 0)
				s->mode = DSB_ISL_DONE;
		}
		return 0;
	}
	if (s->mode != DSB_ISL_RUN1 && s->mode != DSB_ISL_RUN)
		return 0;
	int g = 0, cur = s->p, stop = 0, gr = s->mode == DSB_ISL_RUN ? dsb_isl_rw<GR>(s) : GR1;
	if (s->mode == DSB_ISL_RUN1) { /* for (j = 1; j < STEP_EK; ++j) behind the hit */
		if (mb & 1) {
			s->off -= d;
			s->ln++;
			if (mb & 2) {
				s->off -= d;
				s->ln++;
			}
		}
		g = 2;
		cur = s->h + d;
	}
	for (; g < gr; g++, cur += d) { /* the run: i + j < l_kmer_v / j <= i, len > 60 ends it */
		if (s->fwd ? cur >= s->nk : cur < 0) { stop = 1; break; }
		if (!((mb >> g) & 1)) { stop = 1; break; }
		if (++s->ln > 60) { stop = 1; break; }
	}
	if (!stop) {
		s->p = cur;
		s->mode = DSB_ISL_RUN;
		return 0;
	}
	if (s->fwd) {
		*so = (uint32_t)s->off;
		*sl = (uint32_t)s->ln;
		s->i = s->off + s->ln + 3;
	} else {
		*so = (uint32_t)(s->off - s->ln + 1);
		*sl = (uint32_t)s->ln;
		s->i = s->off - s->ln - 3;
	}
	s->mode = (s->fwd ? s->i < s->nk : s->i >= 0) ? DSB_ISL_GRID : DSB_ISL_DONE;
	return 1;
}

/* get_seed_vector_M2's top-seed pass (src/cly.c:1190-1225) over seeds as they are produced: after
 * seed m is stored with top = 0, the reference writes one more top byte per seed (0 to the
 * current maximum of the group, or 1 to the maximum of the group seed m closes), and one at the
 * end; the same writes in the same order leave the same bytes */
typedef struct { uint32_t n, max_index, max_length, index_end, total; } dsb_topst_t;
DSB_HD void dsb_top_init(dsb_topst_t *t) { t->n = 0; t->max_index = 0; t->max_length = 0; t->index_end = 100; t->total = 0; }
/* seed m = t->n with key `key` and length l: *idx gets the seed whose top byte is written, the
 * return value the byte */
DSB_HD uint8_t dsb_top_push(dsb_topst_t *t, uint32_t key, uint32_t l, uint32_t *idx)
{
	uint32_t m = t->n++;
	if (key < t->index_end) {
		if (t->max_length < l) {
			t->max_length = l;
			t->max_index = m;
		}
		*idx = t->max_index;
		return 0;
	}
	*idx = t->max_index;
	t->index_end += 100;
	t->total += t->max_length;
	t->max_index = m;
	t->max_length = l;
	return 1;
}

/* get_seed_vector_M2, src/cly.c:1157-1229 */
DSB_HD void dsb_seed_vector(dsb_read_ws *w, uint32_t strand, uint32_t seed_off, uint32_t direction, dsb_sdir_t *sd)
{
	uint32_t l_kmer_buff = w->L - w->ix->l_ek + 1;
	dsb_seed_t *seed_v = w->seeds + seed_off;
	uint32_t l_seed_v = dsb_search_exist(strand ? w->exR : w->exF, l_kmer_buff, seed_v, direction,
					     (DSB_NEED_STATS && w->stats) ? w->stats + DSB_ST_OCC : nullptr);
	uint32_t total_score = 0;
	int max_index = 0;
	uint32_t max_length = 0, index_end = 100; /* SEED_RANGE */
	for (uint32_t m = 0; m < l_seed_v; m++) {
		seed_v[m].top = 0;
		uint32_t key = (direction == DSB_FORWARD) ? seed_v[m].offset
						       : l_kmer_buff - seed_v[m].offset - seed_v[m].len;
		if (key < index_end) {
			if (max_length < seed_v[m].len) {
				max_length = seed_v[m].len;
				max_index = m;
			}
			seed_v[max_index].top = 0;
		} else {
			seed_v[max_index].top = 1;
			index_end += 100;
			total_score += max_length;
			max_index = m;
			max_length = seed_v[m].len;
		}
	}
	seed_v[max_index].top = 1; /* also when l_seed_v == 0 (writes a stale slot, as the reference) */
	total_score += max_length;
	sd->seed_off = seed_off;
	sd->l_seed_v_f = l_seed_v;
	sd->strand = strand;
	sd->direction = direction;
	sd->total_score = total_score;
}

/* getIsland, src/cly.c:1231-1263: forward seeds at seed_v[0..), reverse at seed_v[L>>2..) */
DSB_HD void dsb_get_island(dsb_read_ws *w)
{
	dsb_seed_vector(w, 0, 0, DSB_FORWARD, &w->sd[0]);
	dsb_seed_vector(w, 1, w->L >> 2, DSB_REVERSE, &w->sd[1]);
	if (w->sd[0].total_score < w->sd[1].total_score) {
		dsb_sdir_t t = w->sd[0];
		w->sd[0] = w->sd[1];
		w->sd[1] = t;
	}
}

/* ------------------------------------------------------------------ FM search */
typedef struct { uint64_t *set; int l, m; } dsb_spset_t;

/* sp_set_insert, src/cly.c:1281-1293 */
DSB_HD int dsb_spset_insert(uint64_t node, dsb_spset_t *s)
{
	if (s->l == s->m)
		s->l = 0;
	int i = 0;
	for (; i < s->l; i++)
		if (s->set[i] == node)
			return 0;
	s->set[i] = node;
	s->l++;
	return 1;
}

DSB_HD void dsb_set_reset(dsb_spset_t *s) { s->l = 0; }
DSB_HD int dsb_set_insert(uint64_t node, dsb_spset_t *s) { return dsb_spset_insert(node, s); }

/*
 * The same set as an open-addressing hash (one per lane of the wave-cooperative seeding):
 * membership == "inserted since the last reset or since the last wrap of the reference's
 * 500-entry array" (a wrap is `l == m -> l = 0`, i.e. the array forgets everything), so a
 * generation counter replaces clearing.  A slot is {node, gen64}: gen64 = the set's tag + the
 * lane's generation (24 bits: a lane starts far fewer generations in one launch).  The tag is the
 * generation base of the pool set the wave holds (DSB_HSET_POOL, below), or without the pool the
 * launch tag << 24, as follows.  Launch
 * tags come from one 64-bit counter for the whole process (every context of every GPU) and never
 * repeat below 2^40, so slots written by earlier launches — of any context whose workspace bytes
 * these are — never compare equal and read as empty: the table is never cleared.  Within one
 * launch a lane's generation holds at most 500 entries (the reference's wrap), so a probe always
 * finds a slot of another generation among the 512.
 */
#ifndef DSB_HSET_LOG2
#define DSB_HSET_LOG2 9
#endif
#define DSB_HSET_SLOTS (1u << DSB_HSET_LOG2) /* > 500: the reference's set never holds more */
#define DSB_HSET_SLOT_U64 2
#define DSB_HSET_GEN_BITS 24
/* the tables of one 64-lane wave: 512 KB (64, not DSB_WV: host code sizes the pool and the
 * workspaces, and DSB_WV is 1 outside the device pass) */
#define DSB_HSET_WAVE_U64 ((uint64_t)DSB_HSET_SLOT_U64 * DSB_HSET_SLOTS * 64)
/* DSB_HSET_POOL (the GPU build): the tables live in a per-GPU pool of wave-sized sets that a
 * seeding wave holds only while it seeds (dsb_hpool_acquire, dsb_kern.h), not in every read's
 * workspace — 512 KB less per read, i.e. more reads per chunk.  A pool set carries its own
 * generation base, advanced past every generation a holder used, so its slots are never cleared
 * either.  The CPU emulator (tests/emu) mirrors one pool set, used by every read in turn. */
#ifndef DSB_HSET_POOL
#if defined(__HIPCC__)
#define DSB_HSET_POOL 1
#else
#define DSB_HSET_POOL 0
#endif
#endif
/* The first DSB_HSET_L1_MAX entries of a generation go to a small per-lane table in LDS
 * (DSB_HSET_L1 slots of 8 bytes, (generation & 0xffffff) << 40 | node; BWT rows are < 2^40,
 * checked at index load), and only the entries after them to the pool set.  A lookup probes the
 * LDS table first, so membership is unchanged.  Measured with the emulator on C2-proxy ONT reads
 * (tests/emu emu_prof, INSHIST): 81% of all inserts happen while the set holds fewer than 24
 * entries, 91% below 32 — those never touch HBM, where each insert was a dependent 16-B probe and a
 * scattered store (the fast seeding's WRITE_SIZE).  lt == 0: no first level (the host paths). */
#ifndef DSB_HSET_L1_LOG2
#define DSB_HSET_L1_LOG2 5
#endif
#define DSB_HSET_L1 (1u << DSB_HSET_L1_LOG2)
#ifndef DSB_HSET_L1_MAX
#define DSB_HSET_L1_MAX 24 /* < DSB_HSET_L1: a probe always meets a free slot */
#endif
static_assert(DSB_HSET_L1_MAX < DSB_HSET_L1, "first-level sp_set table");
#define DSB_HSET_NODE_BITS 40
typedef struct { uint64_t *tab; uint32_t stride, gen; int l, m; uint64_t tag; uint64_t *lt; } dsb_hset_t;
/* slot tag without the pool: the launch's tag (a host counter bumped for every phase launch, so
 * two launches — FAST0/FAST1, SLOW0/SLOW1, later chunks reusing the same workspace bytes, overflow
 * re-runs — never share one) in the high word, the lane's generation in the low word */
DSB_HD uint64_t dsb_hset_tag(const dsb_read_ws *w)
{
	return w->launch_tag << DSB_HSET_GEN_BITS;
}
/* the set of this lane: `hset` holds the wave's DSB_WV interleaved tables; slot tags are `tag` +
 * the lane's generation (generation 0 is never used: every seed resets the set first).  `lt`: the
 * wave's first-level LDS tables (DSB_HSET_L1 x DSB_WV u64, lane-interleaved) or 0; this lane's
 * slots are cleared to generation 0 here (LDS starts undefined in every workgroup). */
DSB_HD dsb_hset_t dsb_hset_make(uint64_t *hset, uint64_t tag, uint64_t *lt)
{
	dsb_hset_t hs = {hset + DSB_HSET_SLOT_U64 * dsb_lane(), DSB_HSET_SLOT_U64 * DSB_WV, 0, 0, 500, tag, lt ? lt + dsb_lane() : 0};
	if (hs.lt)
		for (int k = 0; k < DSB_HSET_L1; k++)
			hs.lt[(uint32_t)k * DSB_WV] = 0;
	return hs;
}
DSB_HD void dsb_set_reset(dsb_hset_t *s)
{
	s->l = 0;
	s->gen++;
}
DSB_HD int dsb_set_insert(uint64_t node, dsb_hset_t *s)
{
#ifdef DSB_EXP_NO_HSET
	return 1; /* timing experiment only: no duplicate detection */
#endif
	if (s->l == s->m) {
		s->l = 0;
		s->gen++;
	}
#ifdef DSB_EMU_PROF
	dsb_emu_prof_insert(s->l);
#endif
	if (s->lt) { /* first level: the generation's first DSB_HSET_L1_MAX entries */
		uint64_t g24 = (uint64_t)(s->gen & ((1u << DSB_HSET_GEN_BITS) - 1));
		uint64_t want = (g24 << DSB_HSET_NODE_BITS) | node;
		uint32_t h = (uint32_t)((node * 0x9E3779B97F4A7C15ull) >> (64 - DSB_HSET_L1_LOG2));
		for (;;) {
			uint64_t e = s->lt[h * DSB_WV];
			if (e == want)
				return 0;
			if ((e >> DSB_HSET_NODE_BITS) != g24)
				break; /* a free slot: the node is not in the first level */
			h = (h + 1) & (DSB_HSET_L1 - 1);
		}
		if (s->l < DSB_HSET_L1_MAX) {
			s->lt[h * DSB_WV] = want;
			s->l++;
			return 1;
		}
	}
	uint32_t h = (uint32_t)((node * 0x9E3779B97F4A7C15ull) >> (64 - DSB_HSET_LOG2));
	uint64_t g = s->tag + (s->gen & ((1u << DSB_HSET_GEN_BITS) - 1));
	for (;;) {
		uint64_t *slot = s->tab + (uint64_t)h * s->stride;
		uint64_t sn = slot[0], sg = slot[1];
		if (sg == g && sn == node)
			return 0;
		if (sg != g) {
			slot[0] = node;
			slot[1] = g;
			s->l++;
			return 1;
		}
		h = (h + 1) & (DSB_HSET_SLOTS - 1);
	}
}

/* bwt_single_search, src/cly.c:1339-1378; `string` indexes the read buffer, read backwards */
template <typename SET>
DSB_HD void dsb_single_search(dsb_read_ws *w, uint64_t sp, const uint8_t *string, int max_match_len,
			       SET *sp_set, dsb_mem_t *mem_rst)
{
	const dsb_dindex_t *ix = w->ix;
	uint64_t new_sp, sa_sp = ~0ull;
	int match_len = 0, sa_sp_l = 0;
	while (1) {
		if (match_len >= max_match_len)
			break;
		if ((sp & 7) == 0) {
			sa_sp = sp;
			sa_sp_l = 0;
		} else
			sa_sp_l--;
		uint8_t c;
		new_sp = dsb_lf_w(w, sp, &c);
		if (c != *string)
			break;
		match_len++;
		string--;
		if (dsb_set_insert(new_sp, sp_set) == 0) {
			mem_rst->match_len = -1000;
			return;
		}
		sp = new_sp;
	}
	mem_rst->sp = sp;
	mem_rst->match_len = match_len;
	mem_rst->sa_sp = sa_sp;
	mem_rst->sa_sp_l = sa_sp_l;
}

/* bwt_MEM_search, src/cly.c:1383-1442 */
template <typename SET>
DSB_HD int dsb_mem_search(dsb_read_ws *w, const uint8_t *string, uint64_t pre_v, int max_rst, int l_min_mth,
			   int l_max_mth, SET *sp_set, dsb_mem_t *mem_rst)
{
	const dsb_dindex_t *ix = w->ix;
	int n_rst = 0;
	uint64_t sp = dsb_gld(ix->hash_index + pre_v), ep = dsb_gld(ix->hash_index + pre_v + 1), new_sp, new_ep;
	if (w->stats) w->stats[DSB_ST_MEMSEARCH]++;
	string -= DSB_L_PRE_IDX;
	int match_len = DSB_L_PRE_IDX;
	uint8_t c;
	while (1) {
		c = *string;
		string--;
		uint8_t c2 = c;
		new_sp = ix->rank[c] + dsb_occ_w(w, sp, &c);
		new_ep = ix->rank[c2] + dsb_occ_w(w, ep, &c2);
		if (match_len >= l_min_mth - 1) {
			if (new_sp + max_rst >= new_ep)
				break;
			if (match_len >= l_max_mth)
				return 0;
		}
		if (new_sp + 1 >= new_ep)
			break;
		match_len++;
		sp = new_sp;
		ep = new_ep;
	}
	if (new_sp >= new_ep)
		return 0;
	if (new_sp + 1 == new_ep) {
		if (dsb_set_insert(new_sp, sp_set) == 0)
			return 0;
		dsb_single_search(w, new_sp, string, DSB_MAX(0, l_max_mth - match_len), sp_set, mem_rst + n_rst);
		mem_rst[n_rst].match_len += match_len + 1;
		if (mem_rst[n_rst].match_len >= l_min_mth)
			n_rst++;
	} else {
		for (uint64_t c_sp = new_sp; c_sp < new_ep; c_sp++) {
			if (dsb_set_insert(c_sp, sp_set) == 0)
				continue;
			dsb_single_search(w, c_sp, string, DSB_MAX(0, l_max_mth - match_len), sp_set, mem_rst + n_rst);
			mem_rst[n_rst].match_len += match_len + 1;
			if (mem_rst[n_rst].match_len >= l_min_mth)
				n_rst++;
		}
	}
	return n_rst;
}

/* ------------------------------------------------------------------ seed mapping */
/* get_uni, src/cly.c:466-491 (the `uni_offset < 0` loop never runs: uint32) */
DSB_HD uint32_t dsb_get_uni(const dsb_dindex_t *ix, uint64_t bwt_pos, int search_l, uint64_t *global_offset,
			     uint32_t *uni_offset_)
{
	dsb_sa_t s = dsb_gld(ix->sa + (bwt_pos >> 3));
	uint32_t u = s.unitig_ID;
	uint32_t uni_offset = s.offset + search_l + 1;
	if (search_l > 0)
		for (; uni_offset >= dsb_gld(ix->uni + u).length && u < ix->n_uni;) { /* sentinel stops the walk */
			uni_offset -= (dsb_gld(ix->uni + u).length + 1);
			u++;
		}
	uint64_t rp = dsb_gld(ix->r_p + dsb_gld(ix->uni + u).ref_list);
	*global_offset = DSB_RP_OFF(rp) + uni_offset;
	*uni_offset_ = uni_offset;
	return u;
}
DSB_HD uint32_t dsb_get_uni_w(dsb_read_ws *w, uint64_t bwt_pos, int search_l, uint64_t *global_offset,
			       uint32_t *uni_offset_)
{
	uint32_t u = dsb_get_uni(w->ix, bwt_pos, search_l, global_offset, uni_offset_);
	if (w->stats) {
		w->stats[DSB_ST_SA]++;
		w->stats[DSB_ST_UNI] += 1 + (u - w->ix->sa[bwt_pos >> 3].unitig_ID);
		w->stats[DSB_ST_REFPOS]++;
	}
	return u;
}

/* bytes k = 0..15 of lo | hi = end[-k] (two word loads; the read buffer has guards) */
DSB_HD void dsb_rev16(const uint8_t *end, uint64_t *lo, uint64_t *hi)
{
	*lo = __builtin_bswap64(dsb_ld8u(end - 7));
	*hi = __builtin_bswap64(dsb_ld8u(end - 15));
}

/* get_ref of <= 16 bases into string bytes [0, length) of a register window */
DSB_HD void dsb_get_ref_r(dsb_read_ws *w, dsb_w32 &T, uint64_t uni_offset, uint32_t length, int isForward)
{
	if (w->stats) w->stats[DSB_ST_GETREF_B] += (length + 3) / 4;
	uint64_t lo, hi;
	dsb_get_ref16(w->ix, uni_offset, length, isForward, &lo, &hi);
	dsb_w32_put(T, length, lo, hi);
}

/*
 * The byte before get_new_ed's q_buff (H1).  lv_extd reads query[-1] on windows of 1-4 bases, and
 * only that byte of the stale ones can change its result (every other read below the strings is
 * masked by the '#'/'$' terminators).  In the hermetic build (clang -O2, pattern init) get_new_ed
 * is an out-of-line function called from map_seed's REF_POS loop; its frame holds t_buff at
 * rsp+0x08 and q_buff at rsp+0x18, both pattern-initialised, and the 3 padding bytes between them
 * are not, so q_buff[-1] keeps what the last callee of map_seed at that depth left there:
 *   - lv_extd (map_seed's prefix / suffix extensions, src/cly.c:767,820) pattern-initialises its
 *     match_num_data[99], which covers that byte: 0xAA when the REF_POS loop starts;
 *   - kv_pushp_2's realloc (src/cly.c:921) of the anchor vector when a push finds n == m: glibc
 *     2.35's realloc stores the old chunk size (8 bytes, < 2^40) across it: 0x00;
 *   - get_new_ed itself never writes it.
 * So q_buff[-1] is 0xAA until the first kept REF_POS item of the call whose push grew the vector,
 * 0x00 after it (dsb_map_seed).  Derived from the objects oracle/Makefile builds
 * (llvm-objdump / llvm-dwarfdump of _ref/obj_herm/cly.o) and pinned by tools/emu_vs_herm.py.
 * A realloc(NULL) served from the tcache leaves the byte alone (the first push of a read);
 * DSB_QB_FIRST_PUSH is what the first push leaves.
 */
#define DSB_QB_M1_LOOP 0xAA /* q_buff[-1] before any push of the call grew the anchor vector */
#ifndef DSB_QB_M1_GROWN /* (tools: -DDSB_QB_M1_GROWN=0xAA builds the model without the realloc byte) */
#define DSB_QB_M1_GROWN 0x00 /* after one did */
#endif
#ifndef DSB_QB_FIRST_PUSH
#define DSB_QB_FIRST_PUSH DSB_QB_M1_GROWN
#endif
/* map_seed's prefix window q_pre sits at rsp+0x78 of its frame in the hermetic build, right above
 * the spilled s_i pointer (a stack address, top byte 0): q_pre[-1] reads 0x00 */
#define DSB_QPRE_M1 0x00

/* lv_extd of get_new_ed's left window with q_buff[-1] = qm1; *amb set when the other value of
 * that byte would give another edit distance (windows of 1-4 bases only) */
DSB_HD uint32_t dsb_left_lv(const dsb_w32 &T, uint32_t len, dsb_w32 Q, uint32_t qm1, int *amb)
{
	dsb_w32_set_byte(Q, -1, qm1);
	uint32_t ed = (uint32_t)dsb_lv_extd_r(T, (int32_t)len, Q, (int32_t)len);
	if (amb && len >= 1 && len <= 4) {
		dsb_w32_set_byte(Q, -1, qm1 == DSB_QB_M1_LOOP ? DSB_QB_M1_GROWN : DSB_QB_M1_LOOP);
		if ((uint32_t)dsb_lv_extd_r(T, (int32_t)len, Q, (int32_t)len) != ed)
			*amb = 1;
	}
	return ed;
}

/* get_new_ed, src/cly.c:624-689.  q_buff / t_buff (32-byte stack buffers, pattern-initialised)
 * are register windows; the query of the reverse direction is read in place (two word loads
 * per step), as the reference compares against the read buffer itself.  qm1: q_buff[-1] of the
 * forward (left) call, amb: see dsb_left_lv. */
DSB_HD void dsb_get_new_ed(dsb_read_ws *w, uint8_t *q_b, uint32_t *e_d, uint32_t *len_, uint32_t *l_mem_ext,
			    int32_t q_off, uint64_t t_off, uint32_t l_read, int is_FWD, uint32_t qm1 = DSB_QB_M1_LOOP,
			    int *amb = 0)
{
	dsb_w32 Q = dsb_w32_splat(DSB_STACK_PATTERN), T = Q;
	const uint8_t *q = q_b;
	uint32_t len, max_len;
	uint64_t lo, hi, ql, qh;
	if (is_FWD) {
		if (q_off < 0)
			q_off = 0;
		max_len = q_off;
		len = DSB_MIN(12u, max_len);
		dsb_rev16(q_b + q_off, &lo, &hi);
		dsb_w32_put(Q, len, lo, hi);
		ql = Q.b;
		qh = Q.c;
	} else {
		max_len = l_read - q_off;
		len = DSB_MIN(12u, max_len);
		q = q_b + q_off;
		ql = dsb_ld8u(q);
		qh = dsb_ld8u(q + 8);
	}
	dsb_get_ref_r(w, T, t_off, len, !is_FWD);
	if (len > 0 && (T.b & 0xff) == (ql & 0xff)) {
		uint32_t mtc;
		do {
			mtc = dsb_w32_mismatch(T, ql, qh, len); /* for (mtc = 0; mtc < len; mtc++) if (t[mtc] != q[mtc]) break; */
			if (mtc > 0) {
				*l_mem_ext += mtc;
				max_len -= mtc;
				len = DSB_MIN(12u, max_len);
				if (is_FWD) {
					q_off -= mtc;
					t_off -= mtc;
					dsb_rev16(q_b + q_off, &lo, &hi);
					dsb_w32_put(Q, len, lo, hi);
					ql = Q.b;
					qh = Q.c;
				} else {
					t_off += mtc;
					q += mtc;
					ql = dsb_ld8u(q);
					qh = dsb_ld8u(q + 8);
				}
				dsb_get_ref_r(w, T, t_off, len, !is_FWD);
			}
		} while (mtc > 0);
	}
	if (is_FWD)
		*e_d = dsb_left_lv(T, len, Q, qm1, amb);
	else /* lv_extd terminates a copy of the read's bytes (q - 8 .. q + 24) */
		*e_d = (uint32_t)dsb_lv_extd_r(T, (int32_t)len, dsb_w32_load(q - 8), (int32_t)len);
	*len_ = len;
}

/* get_new_ed split into steps (dsb_ned_*), so that a caller can advance two independent
 * extensions in one loop and have both chains' loads in flight together (dsb_map_item: the
 * left and right extension of a REF_POS entry).  Same bytes, compares and result as
 * dsb_get_new_ed. */
typedef struct {
	dsb_w32 T, Q;           /* get_new_ed's t_buff / q_buff: bytes past len keep earlier values */
	uint64_t ql, qh, t_off;
	const uint8_t *q;
	int32_t q_off;
	uint32_t len, max_len, ext;
	int fwd, go;
} dsb_ned_t;

DSB_HD void dsb_ned_load(dsb_read_ws *w, dsb_ned_t *e, const uint8_t *q_b)
{
	if (e->fwd) {
		uint64_t lo, hi;
		dsb_rev16(q_b + e->q_off, &lo, &hi);
		dsb_w32_put(e->Q, e->len, lo, hi);
		e->ql = e->Q.b;
		e->qh = e->Q.c;
	} else {
		e->ql = dsb_ld8u(e->q);
		e->qh = dsb_ld8u(e->q + 8);
	}
	dsb_get_ref_r(w, e->T, e->t_off, e->len, !e->fwd);
}

DSB_HD void dsb_ned_start(dsb_read_ws *w, dsb_ned_t *e, const uint8_t *q_b, int32_t q_off, uint64_t t_off, uint32_t l_read,
			  int is_FWD)
{
	e->fwd = is_FWD;
	e->ext = 0;
	e->T = dsb_w32_splat(DSB_STACK_PATTERN);
	e->Q = e->T;
	e->t_off = t_off;
	if (is_FWD) {
		if (q_off < 0)
			q_off = 0;
		e->max_len = (uint32_t)q_off;
		e->q = q_b;
	} else {
		e->max_len = l_read - (uint32_t)q_off;
		e->q = q_b + q_off;
	}
	e->q_off = q_off;
	e->len = DSB_MIN(12u, e->max_len);
	dsb_ned_load(w, e, q_b);
	e->go = e->len > 0 && (e->T.b & 0xff) == (e->ql & 0xff);
}

/* one trip of get_new_ed's do-while: extend over the matching prefix and reload */
DSB_HD void dsb_ned_step(dsb_read_ws *w, dsb_ned_t *e, const uint8_t *q_b)
{
	uint32_t mtc = dsb_w32_mismatch(e->T, e->ql, e->qh, e->len);
	if (mtc == 0) {
		e->go = 0;
		return;
	}
	e->ext += mtc;
	e->max_len -= mtc;
	e->len = DSB_MIN(12u, e->max_len);
	if (e->fwd) {
		e->q_off -= (int32_t)mtc;
		e->t_off -= mtc;
	} else {
		e->t_off += mtc;
		e->q += mtc;
	}
	dsb_ned_load(w, e, q_b);
}

DSB_HD uint32_t dsb_ned_finish(const dsb_ned_t *e, uint32_t qm1 = DSB_QB_M1_LOOP, int *amb = 0)
{
	if (e->fwd)
		return dsb_left_lv(e->T, e->len, e->Q, qm1, amb);
	/* !fwd: lv_extd terminates a copy of the read's bytes (q - 8 .. q + 24) */
	return (uint32_t)dsb_lv_extd_r(e->T, (int32_t)e->len, dsb_w32_load(e->q - 8), (int32_t)e->len);
}

typedef struct { uint8_t *bin_read; uint32_t read_L; uint16_t seed_ID; uint32_t direction; } dsb_seedinfo_t;

/* Q_MEM[l]: the reference reads past its 2000 entries for exact matches >= 2000 bp
 * (unpinned); the device table is padded and the index clamped. */
DSB_HD int dsb_qmem(const dsb_dindex_t *ix, uint32_t l)
{
	return dsb_gld(ix->Q_MEM + (l < DSB_Q_MEM_PAD ? l : DSB_Q_MEM_PAD - 1));
}

DSB_HD dsb_anchor_t *dsb_push_anchor(dsb_read_ws *w)
{
	if (w->n_anc >= w->cap.anc) {
		w->overflow |= 1;
		return 0;
	}
	return w->anc + w->n_anc++;
}

#define DSB_LV_L 12
#define DSB_MIN_S_1 12
#define DSB_MIN_S_2 20
#ifndef DSB_MAP_SUF_EARLY
#define DSB_MAP_SUF_EARLY 0
#endif
/* map_seed, src/cly.c:701-934, in two parts: dsb_map_seed_pre (locate the hit, extend and
 * score its prefix / suffix: src/cly.c:701-884) leaves the REF_POS list of the hit's unitig in
 * a context; dsb_map_item scores one REF_POS entry of it into an Anchor (src/cly.c:886-931).
 * dsb_map_seed runs both in sequence; the wave seeding spreads the items over its lanes. */
typedef struct {
	uint64_t rp_s;          /* first REF_POS entry of the unitig */
	uint32_t n_items;       /* REF_POS entries to score (0: none) */
	int32_t ret;            /* map_seed's value when n_items == 0 */
	int32_t q_off;
	uint32_t l_m, u_off;
	uint16_t am_mtch;
	int16_t am_score;
	uint8_t am_ll, am_le, am_rl, am_re, ref_l, ref_r;
} dsb_mapctx_t;

DSB_HD void dsb_map_seed_pre(dsb_read_ws *w, dsb_mem_t *m_r, dsb_seedinfo_t *s_i, dsb_mapctx_t *cx)
{
	const dsb_dindex_t *ix = w->ix;
	const int *Q_LV = ix->Q_LV;
	uint64_t b_p = m_r->sp;
	int32_t q_off = m_r->read_offset;
	uint32_t l_m = m_r->match_len;
	uint8_t *q_b = s_i->bin_read;
	int32_t uni = -1;
	uint32_t u_off = 0;
	uint64_t t_off = 0;
	uint32_t l_pre = 0, l_suf = 0;
	uint32_t d_pre = 0, d_suf = 0;
	int32_t s = 0, max_s = 0;
	/* stack windows q_pre / t_pre / t_suf[LV_L + 1] (src/cly.c:705-707), in registers */
	dsb_w32 QP = dsb_w32_splat(DSB_STACK_PATTERN), TP = QP, TS = QP;
	dsb_w32_set_byte(QP, -1, DSB_QPRE_M1);
	uint64_t lo, hi;
	do {
		const uint8_t *q_suf;
		l_pre = DSB_MIN(q_off + 1, DSB_LV_L);
		dsb_rev16(q_b + q_off, &lo, &hi);
		dsb_w32_put(QP, l_pre, lo, hi);
		int s_l = 0;
		if (m_r->sa_sp != ~0ull) {
			uni = (int32_t)dsb_get_uni_w(w, m_r->sa_sp, m_r->sa_sp_l, &t_off, &u_off);
		} else {
			uint8_t c;
			uint64_t new_sp;
			while (1) {
				if ((b_p & 7) == 0)
					break;
				new_sp = dsb_lf_w(w, b_p, &c);
				if (c == 4)
					break;
				dsb_w32_set_byte(TP, s_l++, c);
				b_p = new_sp;
				if ((uint32_t)s_l >= l_pre)
					break;
			}
			if ((b_p & 7) == 0) {
				uni = (int32_t)dsb_get_uni_w(w, b_p, s_l, &t_off, &u_off);
			} else
				l_pre = s_l;
		}
		int ts_pre = 0; /* the suffix window is loaded already */
		if (uni >= 0) {
			if (dsb_gld(ix->uni + uni).length < DSB_MIN_UNI_L)
				break;
			l_pre = DSB_MIN(l_pre, u_off);
			dsb_get_ref_r(w, TP, t_off - 1, l_pre, 0);
#if DSB_MAP_SUF_EARLY
			/* the suffix's first window depends on t_off and l_m only: its load goes out with
			 * the prefix window's instead of after the prefix extension (one round trip less) */
			{
				uint32_t lms = DSB_MIN(dsb_gld(ix->uni + uni).length - u_off - l_m, s_i->read_L - (q_off + l_m + 1));
				if (lms != 0) {
					dsb_get_ref_r(w, TS, t_off + l_m, DSB_MIN(lms, (uint32_t)DSB_LV_L), 1);
					ts_pre = 1;
				}
			}
#endif
		}
		d_pre = dsb_lv_extd_r(TP, l_pre, QP, l_pre);
		s = dsb_qmem(ix, l_m) + dsb_gld(Q_LV + (d_pre * DSB_LV_DIM + l_pre));
		if (s < DSB_MIN_S_1 && l_pre == DSB_LV_L && uni < 0) {
			s = 0;
			break;
		}
		if (uni < 0) {
			while (b_p & 7) {
				uint8_t c;
				b_p = dsb_lf_w(w, b_p, &c);
				s_l++;
			}
			uni = (int32_t)dsb_get_uni_w(w, b_p, s_l, &t_off, &u_off);
			if (dsb_gld(ix->uni + uni).length < DSB_MIN_UNI_L) {
				s = 0;
				break;
			}
		}
		int32_t q_off_r = q_off + l_m + 1;
		uint32_t l_max_suf = DSB_MIN(dsb_gld(ix->uni + uni).length - u_off - l_m, s_i->read_L - q_off_r);
		if (l_max_suf != 0) {
			l_suf = DSB_MIN(l_max_suf, (uint32_t)DSB_LV_L);
			q_suf = q_b + q_off_r;
			uint64_t ql = dsb_ld8u(q_suf), qh = dsb_ld8u(q_suf + 8);
			if (!ts_pre)
				dsb_get_ref_r(w, TS, t_off + l_m, l_suf, 1);
			if ((TS.b & 0xff) == (ql & 0xff)) {
				uint32_t mtc;
				do {
					mtc = dsb_w32_mismatch(TS, ql, qh, l_suf);
					if (mtc > 0) {
						l_m += mtc;
						s = dsb_qmem(ix, l_m) + dsb_gld(Q_LV + (d_pre * DSB_LV_DIM + l_pre));
						l_max_suf -= mtc;
						l_suf = DSB_MIN(l_max_suf, (uint32_t)DSB_LV_L);
						q_suf += mtc;
						ql = dsb_ld8u(q_suf);
						qh = dsb_ld8u(q_suf + 8);
						dsb_get_ref_r(w, TS, t_off + l_m, l_suf, 1);
					}
				} while (mtc > 0);
			}
			/* lv_extd terminates a copy of the read's bytes (q_suf - 8 .. q_suf + 24) */
			d_suf = dsb_lv_extd_r(TS, l_suf, dsb_w32_load(q_suf - 8), l_suf);
			s += dsb_gld(Q_LV + (d_suf * DSB_LV_DIM + l_suf));
		} else
			l_suf = d_suf = 0;
		if (s <= DSB_MIN_S_2 && l_suf == DSB_LV_L) {
			s = 0;
			break;
		}
	} while (0);

	cx->n_items = 0;
	cx->ret = 0;
	cx->q_off = q_off;
	cx->l_m = l_m;
	cx->u_off = u_off;
	if (s > 0) {
		/* Anchor_map a_m = {l_m, s, l_pre, d_pre, l_suf, d_suf} (uint16/int16/uint8 fields) */
		cx->am_mtch = (uint16_t)l_m;
		cx->am_score = (int16_t)s;
		cx->am_ll = (uint8_t)l_pre; cx->am_le = (uint8_t)d_pre; cx->am_rl = (uint8_t)l_suf; cx->am_re = (uint8_t)d_suf;
		uint64_t rp_s = dsb_gld(ix->uni + uni).ref_list, rp_e = dsb_gld(ix->uni + uni + 1).ref_list;
		cx->ref_l = (uint8_t)(l_pre < DSB_LV_L || d_pre == 0);
		cx->ref_r = (uint8_t)(l_suf < DSB_LV_L || d_suf == 0);
		if (rp_e - rp_s > 50 && !(rp_e - rp_s < 1000)) {
			cx->ret = 50;
			return;
		}
		cx->rp_s = rp_s;
		cx->n_items = (uint32_t)(rp_e - rp_s);
	}
}

/* REF_POS entry rp_s + item of a hit: 1 and the Anchor in *a when the reference pushes one.
 * qm1: get_new_ed's q_buff[-1] for this item; amb: see dsb_left_lv. */
DSB_HD int dsb_map_item(dsb_read_ws *w, const dsb_mapctx_t *cx, uint32_t item, const dsb_seedinfo_t *s_i, dsb_anchor_t *a,
			uint32_t qm1 = DSB_QB_M1_LOOP, int *amb = 0)
{
	const dsb_dindex_t *ix = w->ix;
	const int *Q_LV = ix->Q_LV;
	uint64_t rp = dsb_gld(ix->r_p + cx->rp_s + item);
	if (w->stats) w->stats[DSB_ST_REFPOS]++;
	uint16_t am_mtch = cx->am_mtch;
	int16_t am_score = cx->am_score;
	uint8_t am_ll = cx->am_ll, am_le = cx->am_le, am_rl = cx->am_rl, am_re = cx->am_re;
	uint32_t l_m_ext_l = 0;
	uint32_t ref_id = DSB_RP_REF(rp);
	uint64_t seq_off = dsb_gld(ix->ref_seq_offset + ref_id); /* issued with the extensions' loads */
	if (cx->ref_l || cx->ref_r) {
#ifndef DSB_NED_PAIR
#define DSB_NED_PAIR 0 /* measured: fast seeding 44.9 -> 45.8 ms with the pair (registers at the 256 cap): off */
#endif
		if (DSB_NED_PAIR) {
			/* the left and right extensions are independent: both chains advance in one loop */
			dsb_ned_t L, R;
			L.go = R.go = 0;
			if (cx->ref_l)
				dsb_ned_start(w, &L, s_i->bin_read, cx->q_off, DSB_RP_OFF(rp) + cx->u_off - 1, s_i->read_L, 1);
			if (cx->ref_r)
				dsb_ned_start(w, &R, s_i->bin_read, cx->q_off + cx->l_m + 1, DSB_RP_OFF(rp) + cx->u_off + cx->l_m,
					      s_i->read_L, 0);
			while (L.go || R.go) {
				if (L.go) dsb_ned_step(w, &L, s_i->bin_read);
				if (R.go) dsb_ned_step(w, &R, s_i->bin_read);
			}
			if (cx->ref_l) {
				am_le = (uint8_t)dsb_ned_finish(&L, qm1, amb);
				am_ll = (uint8_t)L.len;
				l_m_ext_l = L.ext;
			}
			am_mtch = (uint16_t)(cx->l_m + l_m_ext_l);
			if (cx->ref_r) {
				am_re = (uint8_t)dsb_ned_finish(&R);
				am_rl = (uint8_t)R.len;
				am_mtch = (uint16_t)(am_mtch + R.ext);
			}
		} else {
			uint32_t ed_l, ed_r, len_l, len_r, l_m_ext_r;
			if (cx->ref_l) {
				dsb_get_new_ed(w, s_i->bin_read, &ed_l, &len_l, &l_m_ext_l, cx->q_off, DSB_RP_OFF(rp) + cx->u_off - 1,
					       s_i->read_L, 1, qm1, amb);
				am_ll = (uint8_t)len_l;
				am_le = (uint8_t)ed_l;
			}
			am_mtch = (uint16_t)(cx->l_m + l_m_ext_l);
			if (cx->ref_r) {
				l_m_ext_r = 0;
				dsb_get_new_ed(w, s_i->bin_read, &ed_r, &len_r, &l_m_ext_r, cx->q_off + cx->l_m + 1,
					       DSB_RP_OFF(rp) + cx->u_off + cx->l_m, s_i->read_L, 0);
				am_rl = (uint8_t)len_r;
				am_re = (uint8_t)ed_r;
				am_mtch = (uint16_t)(am_mtch + l_m_ext_r);
			}
		}
		am_score = (int16_t)(dsb_qmem(ix, am_mtch) + dsb_gld(Q_LV + (am_le * DSB_LV_DIM + am_ll)) + dsb_gld(Q_LV + (am_re * DSB_LV_DIM + am_rl)));
		if (am_score < DSB_MIN_S_2)
			return 0;
	}
	a->direction = (uint8_t)s_i->direction;
	a->index_in_read = cx->q_off + 1 - l_m_ext_l;
	a->global_offset = DSB_RP_OFF(rp) + cx->u_off - l_m_ext_l;
	a->ref_ID = ref_id;
	a->ref_offset = (uint32_t)(a->global_offset - seq_off);
	a->mtch_len = am_mtch;
	a->score = am_score;
	a->left_len = am_ll; a->left_ED = am_le; a->rigt_len = am_rl; a->rigt_ED = am_re;
	a->seed_ID = s_i->seed_ID;
	a->duplicate = 0;
	a->pre = -1;
	a->chain_id = 0;
	a->anchor_useless = 0;
	return 1;
}

/* kv_pushp_2 (src/lib/kvec.h:103-109) grows the vector when n reaches m: m = 0, 10, 20, 40, ... */
DSB_HD int dsb_anc_grows(uint32_t n)
{
	if (n == 0)
		return 1;
	if (n % 10)
		return 0;
	n /= 10;
	return (n & (n - 1)) == 0;
}

DSB_HDN int32_t dsb_map_seed(dsb_read_ws *w, dsb_mem_t *m_r, dsb_seedinfo_t *s_i)
{
	dsb_mapctx_t cx;
	dsb_map_seed_pre(w, m_r, s_i, &cx);
	if (cx.n_items == 0)
		return cx.ret;
	int32_t max_s = 0;
	/* the reference's anchor_v: n = w->n_anc, capacity m = 0, 10, 20, 40 ... the least one >= every n
	 * it held; kv_pushp_2 reallocs when a push finds n == m, and from then on get_new_ed's
	 * q_buff[-1] reads what realloc left (dsb_left_lv) */
	uint32_t hw = DSB_MAX(w->anc_hw, w->n_anc), qm1 = DSB_QB_M1_LOOP;
	for (uint32_t it = 0; it < cx.n_items; it++) {
		dsb_anchor_t an;
		if (!dsb_map_item(w, &cx, it, s_i, &an, qm1))
			continue;
		max_s = DSB_MAX(max_s, (int32_t)an.score);
		if (w->n_anc == hw && dsb_anc_grows(hw))
			qm1 = hw == 0 ? DSB_QB_FIRST_PUSH : DSB_QB_M1_GROWN;
		dsb_anchor_t *a = dsb_push_anchor(w);
		hw = DSB_MAX(hw, w->n_anc);
		if (!a)
			return max_s;
		if (w->stats) w->stats[DSB_ST_ANCHOR]++;
		*a = an;
	}
	return max_s;
}

/* ------------------------------------------------------------------ fast / slow */
#define DSB_MEM_SEARCH_FAST 2
#define DSB_MIN_MEM_LEN_FAST 21
/* One seed of fast_classify (src/cly.c:1483-1538): FM searches along the seed, map_seed of
 * the hits (anchors pushed at w->n_anc), then the seed's anchors below its top score are
 * marked useless.  Returns 1 when the reference skips the next seed (`ci++`). */
template <typename SET>
DSB_HD int dsb_fast_seed(dsb_read_ws *w, const dsb_sdir_t *s_d, uint32_t ci, SET *sp_set)
{
	const dsb_dindex_t *ix = w->ix;
	uint8_t l_ek = (uint8_t)ix->l_ek;
	int min_index = DSB_MIN_MEM_LEN_FAST - l_ek;
	uint8_t *bin_read = w->bin + (s_d->strand ? w->L : 0);
	dsb_mem_t m_r[DSB_MEM_SEARCH_FAST];
	dsb_seed_t *c_sv = w->seeds + s_d->seed_off + ci;
	dsb_seedinfo_t s_i = {bin_read, w->L, (uint16_t)ci, s_d->direction};
	dsb_set_reset(sp_set);
	uint32_t a_b_idx = w->n_anc;
	int skip = 0;
	for (int j = (int)c_sv->len - 1; j >= min_index;) {
		int kmer_index = (int)c_sv->offset + j;
		uint64_t kmer = dsb_kmer_at(bin_read + kmer_index, l_ek, ix->single_base_max);
		uint64_t prefixValue = kmer & DSB_PRE_IDX_MASK;
		int string_index = kmer_index + l_ek - 1;
		uint64_t t0 = w->tmr ? dsb_clock() : 0;
		int n_m = dsb_mem_search(w, bin_read + string_index, prefixValue, DSB_MEM_SEARCH_FAST,
					 DSB_MIN_MEM_LEN_FAST - 1, string_index, sp_set, m_r);
		if (w->tmr) w->tmr[DSB_ST_T_MEM] += dsb_clock() - t0;
		if (n_m == 0) {
			j -= 2;
			continue;
		}
		j -= 3;
		int max_score = 0;
		for (int k = 0; k < n_m; k++) {
			m_r[k].read_offset = string_index - m_r[k].match_len;
			uint64_t t1 = w->tmr ? dsb_clock() : 0;
			int c_score = dsb_map_seed(w, m_r + k, &s_i);
			if (w->tmr) w->tmr[DSB_ST_T_MAP] += dsb_clock() - t1;
			max_score = DSB_MAX(c_score, max_score);
		}
		if (w->overflow)
			return 0;
		if (max_score > 35)
			j -= 7;
		if (max_score > 256) {
			if (max_score > 512)
				skip = 1;
			break;
		}
	}
	int top_score = 35;
	for (uint32_t k = a_b_idx; k < w->n_anc; k++)
		top_score = DSB_MAX(top_score, (int)w->anc[k].score);
	for (uint32_t k = a_b_idx; k < w->n_anc; k++)
		w->anc[k].anchor_useless = (w->anc[k].score < top_score) ? 1 : 0;
	return skip;
}

/* fast_classify, src/cly.c:1473-1541 */
DSB_HDN void dsb_fast_classify(dsb_read_ws *w, const dsb_sdir_t *s_d)
{
	dsb_spset_t sp_set = {w->spset, 0, 500};
	uint32_t n_sv = s_d->l_seed_v_f;
	for (uint32_t ci = 0; ci < n_sv; ci++) {
		if (w->seeds[s_d->seed_off + ci].top == 0)
			continue;
		int skip = dsb_fast_seed(w, s_d, ci, &sp_set);
		if (w->overflow)
			return;
		if (skip)
			ci++;
	}
}

/*
 * fast_classify as a per-lane state machine (one wavefront per read).
 *
 * A lane-per-seed form (one seed per lane, each lane running the reference's nested loops in
 * its own control flow) leaves the lanes of a wave diverged and the wave serialises them
 * (measured VALU lane utilisation ~8 %).  Here every lane
 * advances its seed by one step per trip of a single wave-wide loop, so lanes doing the same
 * kind of step run together:
 *   J    start the next FM search at position j of the seed (k-mer, 13-mer prefix interval)
 *   EXT  one backward-extension step of bwt_MEM_search (two occ)        src/cly.c:1396-1413
 *   ROW  next SA row of the final interval: sp_set insert               src/cly.c:1416-1440
 *   SS   one step of bwt_single_search (one LF)                         src/cly.c:1349-1372
 *   MAP  map_seed of one MEM hit                                        src/cly.c:1505-1513
 *   FIN  the seed's anchors below its top score become useless; next seed src/cly.c:1530-1537
 * EXT and SS share one occ evaluation per trip.  MAP is the long step: lanes reaching it wait
 * until at least DSB_SM_MAP_BATCH lanes (or every lane still working) are there, then run it
 * together.  Seeds are handed out in top-seed order as lanes become free; each seed's anchors
 * are staged in its lane's area and described by a record (lane, offset, count, trigger,
 * overflow), after which the reference's skip rule and the ordered compaction run over the
 * records: a top seed is skipped iff the previously processed seed triggered the reference's
 * `ci++` (src/cly.c:1526, score > 512) and sits immediately before it; kept anchors are
 * compacted in seed order (prefix sum); a group holding an overflowed seed is replayed seed by
 * seed in order.  SLOW (slow_classify, src/cly.c:1545-1606): every seed the reference takes,
 * every 2nd k-mer, up to 8 rows per FM hit, the seed's stable top-8 hits mapped at its end.
 */
/* DSB_SEED_PRE 1: k_seed stores every position's 13-mer prefix value (u32, 6.4 GB at C1) for
 * the J step; 0: the J step recomputes it from the read (three word loads).  Measured on
 * C1: k_seed -1.3 ms, fast seeding +1.6 ms: kept at 1 */
#ifndef DSB_SEED_PRE
#define DSB_SEED_PRE 1
#endif
#ifndef DSB_SM_LPT
#define DSB_SM_LPT 1 /* pass 0 hands seeds out longest first */
#endif
#ifndef DSB_SM_LPT_CH
#define DSB_SM_LPT_CH 2 /* top-seed lengths held in registers for the hand-out sort (x 64 seeds) */
#endif
#ifndef DSB_SM_MAP_BATCH
#define DSB_SM_MAP_BATCH 64
#endif
enum { DSB_SM_J = 0, DSB_SM_EXT, DSB_SM_ROW, DSB_SM_SS, DSB_SM_MAP, DSB_SM_FIN, DSB_SM_DONE };

#define DSB_MEM_SEARCH_SLOW 8
#define DSB_MIN_MEM_LEN_SLOW 20
/* One seed of slow_classify (src/cly.c:1556-1603): MEM searches every other position of the
 * seed, the hits ordered by match length (stable msort, MEM_rst_cmp_by_match_len) and the
 * first 8 mapped.  Only those 8 are ever used, so they are kept as a stable top-8 while the
 * hits stream in (tmp: 16 entries).  The seed's anchors below its top score become useless. */
template <typename SET>
DSB_HD void dsb_slow_seed(dsb_read_ws *w, const dsb_sdir_t *sd, uint32_t i, SET *sp_set, dsb_mem_t *tmp)
{
	const dsb_dindex_t *ix = w->ix;
	int l_ek = ix->l_ek;
	uint8_t *bin_read = w->bin + (sd->strand ? w->L : 0);
	dsb_seed_t *sv = w->seeds + sd->seed_off + i;
	int min_match_len = DSB_MIN(DSB_MIN_MEM_LEN_SLOW - 1, l_ek + 1);
	dsb_set_reset(sp_set);
	dsb_mem_t *top = tmp, *cur = tmp + DSB_MEM_SEARCH_SLOW;
	int n_top = 0, total = 0;
	for (int j = (int)sv->len - 1; j >= 1; j -= 2) {
		int k_idx = (int)sv->offset + j;
		uint64_t kmer = dsb_kmer_at(bin_read + k_idx, l_ek, ix->single_base_max);
		uint64_t pre_v = kmer & DSB_PRE_IDX_MASK;
		int s_idx = k_idx + l_ek - 1;
		int c = dsb_mem_search(w, bin_read + s_idx, pre_v, DSB_MEM_SEARCH_SLOW, min_match_len, s_idx, sp_set, cur);
		for (int k = 0; k < c; k++) {
			cur[k].read_offset = k_idx + l_ek - 1 - cur[k].match_len;
			int p = 0; /* stable, match_len descending: after every kept hit at least as long */
			while (p < n_top && top[p].match_len >= cur[k].match_len)
				p++;
			if (p >= DSB_MEM_SEARCH_SLOW)
				continue;
			for (int q = DSB_MIN(n_top, DSB_MEM_SEARCH_SLOW - 1); q > p; q--)
				top[q] = top[q - 1];
			top[p] = cur[k];
			n_top = DSB_MIN(n_top + 1, DSB_MEM_SEARCH_SLOW);
		}
		total += c;
	}
	if (total == 0)
		return;
	dsb_seedinfo_t seed_info = {bin_read, w->L, (uint16_t)i, sd->direction};
	uint32_t a_b_idx = w->n_anc;
	for (int k = 0; k < n_top; k++)
		dsb_map_seed(w, top + k, &seed_info);
	if (w->overflow)
		return;
	int top_score = 35;
	for (uint32_t k = a_b_idx; k < w->n_anc; k++)
		top_score = DSB_MAX(top_score, (int)w->anc[k].score);
	for (uint32_t k = a_b_idx; k < w->n_anc; k++)
		w->anc[k].anchor_useless = (w->anc[k].score < top_score) ? 1 : 0;
}

/* src/cly.c:1563: the guard reads seed 0's `top`, not seed i's (H10) */
DSB_HD int dsb_slow_takes(const dsb_read_ws *w, const dsb_sdir_t *sd, uint32_t i)
{
	const dsb_seed_t *sv_f = w->seeds + sd->seed_off;
	return !((int)(sv_f[i].len) < 3 && sv_f->top == 0);
}

/* slow_classify, src/cly.c:1545-1606 */
DSB_HDN void dsb_slow_classify(dsb_read_ws *w, const dsb_sdir_t *sd)
{
	dsb_spset_t sp_set = {w->spset, 0, 500};
	for (uint32_t i = 0; i < sd->l_seed_v_f; i++) {
		if (!dsb_slow_takes(w, sd, i))
			continue;
		dsb_slow_seed(w, sd, i, &sp_set, w->mem);
		if (w->overflow)
			return;
	}
	w->fast_classify = 0;
}

template <bool SLOW, int G>
DSB_HDN void dsb_seed_sm(dsb_read_ws *w, const dsb_sdir_t *s_d, dsb_hset_t *hsp, dsb_mem_t *memtmp, int32_t *lds)
{
	const dsb_dindex_t *ix = w->ix;
	/* G lanes per read (DSB_SM_G): the read's seeds run on a group of G lanes of the wave; `lane`
	 * is the lane's index in its group, and every ballot, scan and broadcast is the group's */
	constexpr uint32_t GW = (uint32_t)G < (uint32_t)DSB_WV ? (uint32_t)G : (uint32_t)DSB_WV;
	uint32_t lane = dsb_glane<GW>();
	uint32_t n_sv = s_d->l_seed_v_f;
	uint32_t S = (w->dbg & 32) ? 2 : w->cap.anc / GW; /* dbg 32: tiny staging (tests the replay) */
	dsb_hset_t &hs = *hsp; /* the caller reads the generations used back (the pool's base) */
	uint8_t l_ek = (uint8_t)ix->l_ek;
	int min_index = DSB_MIN_MEM_LEN_FAST - l_ek;
	/* bwt_MEM_search parameters: fast src/cly.c:1500-1501, slow src/cly.c:1568-1570 */
	const int MAX_RST = SLOW ? DSB_MEM_SEARCH_SLOW : DSB_MEM_SEARCH_FAST;
	const int L_MIN = SLOW ? DSB_MIN(DSB_MIN_MEM_LEN_SLOW - 1, (int)l_ek + 1) : DSB_MIN_MEM_LEN_FAST - 1;
	dsb_mem_t *top = memtmp + (uint64_t)lane * (2 * DSB_MEM_SEARCH_SLOW); /* slow: stable top-8 hits */
	int n_top = 0, total = 0;
	uint8_t *bin_read = w->bin + (s_d->strand ? w->L : 0);
	/* ---- top seeds, in order (tix) */
	/* the read-hash region is free while seeding (>= 8 L + 8 KB bytes; n_sv <= L/3 + 1): 5 words per seed
	 * — 2 record words, the pass-1 list, the top-seed list and the pass-0 hand-out order */
	uint32_t *rec = w->hh[0], *klist = rec + 2 * (uint64_t)n_sv, *tix = rec + 3 * (uint64_t)n_sv;
	uint32_t *hand = rec + 4 * (uint64_t)n_sv; /* pass-0 hand-out order (DSB_SM_LPT) */
	uint32_t m = 0;
	for (uint32_t gb = 0; gb < n_sv; gb += GW) {
		uint32_t ci = gb + lane;
		int t = ci < n_sv && (SLOW ? dsb_slow_takes(w, s_d, ci) : w->seeds[s_d->seed_off + ci].top != 0);
		uint64_t bm = dsb_gballot<GW>(t);
		uint64_t below = (lane == 0) ? 0 : (bm & (~0ull >> (64 - lane)));
		if (t)
			tix[m + (uint32_t)__builtin_popcountll(below)] = ci;
		m += (uint32_t)__builtin_popcountll(bm);
	}
	dsb_wsync();
	if (m == 0) {
		if (SLOW)
			w->fast_classify = 0;
		return;
	}
	/* Pass 0 hands the top seeds out longest first (a seed's FM / map work grows with its
	 * length), so that the long ones do not start in the last lanes to free up; ties in seed
	 * order.  The output does not depend on the hand-out order: every seed's anchors and skip
	 * trigger are recorded per seed and compacted in seed order below. */
	if (DSB_SM_LPT) {
		auto seed_len = [&](uint32_t q) -> uint32_t {
			return q < m ? DSB_MIN(w->seeds[s_d->seed_off + tix[q]].len, 63u) : 64u;
		};
		uint32_t slen[DSB_SM_LPT_CH];
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
		for (int c = 0; c < DSB_SM_LPT_CH; c++)
			slen[c] = seed_len((uint32_t)c * GW + lane);
		uint32_t pos = 0;
		auto place = [&](uint32_t q, int t) {
			uint64_t bm = dsb_gballot<GW>(t);
			if (t) {
				uint64_t below = lane == 0 ? 0 : (bm & (~0ull >> (64 - lane)));
				hand[pos + (uint32_t)__builtin_popcountll(below)] = q;
			}
			pos += (uint32_t)__builtin_popcountll(bm);
		};
		for (uint32_t b = 64; b-- > 0;) {
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
			for (int c = 0; c < DSB_SM_LPT_CH; c++)
				if ((uint32_t)c * GW < m)
					place((uint32_t)c * GW + lane, slen[c] == b);
			for (uint32_t gb = DSB_SM_LPT_CH * GW; gb < m; gb += GW)
				place(gb + lane, seed_len(gb + lane) == b);
		}
		dsb_wsync();
	}
	dsb_anchor_t *anc0 = w->anc;
	uint32_t n0 = w->n_anc, cap0 = w->cap.anc, of0 = w->overflow;
	/* ---- per-lane seed state; every record starts as "overflowed" (replayed if never written) */
	for (uint32_t q = lane; q < m; q += GW) {
		rec[2 * q] = 0;
		rec[2 * q + 1] = 1u << 30;
	}
	dsb_wsync();
	/* Two passes.  Pass 0 hands every top seed out; a lane's anchors go to its 1/64 slice of the
	 * staging pool (anc_tmp) and a lane whose slice fills retires, leaving its seed (and the seeds
	 * never handed out) flagged overflowed.  Pass 1 runs those seeds again with a second pool
	 * (anc_tmp2) split over only as many lanes as there are such seeds, so one seed of a repeat
	 * region with hundreds of anchors still runs on the state machine instead of the serial
	 * replay of the compaction below (which stays for what overflows both). */
	uint32_t n_ovf = 0, S2 = S;
	for (uint32_t pr = 0; pr < 2; pr++) {
	uint32_t mp = pr ? n_ovf : m;
	if (mp == 0)
		break;
	uint32_t Sp = pr ? S2 : S;
	dsb_anchor_t *pool = pr ? w->anc_tmp2 : w->anc_tmp;
	/* ---- the lane's anchor vector is its staging area while seeds run */
	dsb_anchor_t *stg = pool + (uint64_t)lane * Sp;
	w->anc = stg;
	w->n_anc = 0;
	w->cap.anc = Sp;
	w->overflow = 0;
	uint32_t next_k = DSB_MIN((uint32_t)GW, mp); /* next seed of the pass to hand out (uniform) */
	uint32_t k = lane;                                 /* my top-seed index */
	int st = DSB_SM_DONE;
	uint32_t ci = 0, a_b = 0, seed_off = 0;
	int j = 0, skip = 0, n_m = 0, k_map = 0, max_score = 0, string_index = 0, match_len = 0, row_single = 0;
	int seed_amb = 0; /* an item of the seed read q_buff[-1] where it matters: replayed in order (dsb_map_seed) */
	uint64_t sp = 0, ep = 0, row = 0, row_end = 0, ss_sp = 0, sa_sp = 0;
	int ss_len = 0, ss_max = 0, sa_sp_l = 0, l_max = 0;
	const uint8_t *str = bin_read, *ss_str = bin_read;
	dsb_mem_t m_r[DSB_MEM_SEARCH_FAST];
	for (int q = 0; q < DSB_MEM_SEARCH_FAST; q++) {
		m_r[q].match_len = 0; m_r[q].sp = 0; m_r[q].sa_sp = 0; m_r[q].sa_sp_l = 0; m_r[q].kmer_index = 0; m_r[q].read_offset = 0;
	}
#define DSB_SM_START_SEED(K)                                                   \
	do {                                                                   \
		k = pr ? klist[K] : (DSB_SM_LPT ? hand[K] : (K));              \
		ci = tix[k];                                                   \
		const dsb_seed_t *c_sv_ = w->seeds + s_d->seed_off + ci;       \
		seed_off = c_sv_->offset;                                      \
		j = (int)c_sv_->len - 1;                                       \
		skip = 0;                                                      \
		seed_amb = 0;                                                  \
		n_top = 0;                                                     \
		total = 0;                                                     \
		a_b = w->n_anc;                                                \
		dsb_set_reset(&hs);                                            \
		st = DSB_SM_J;                                                 \
		DSB_EMU_PROF_START();                                          \
	} while (0)
	/* a finished single search: fast keeps hits >= L_MIN in m_r (src/cly.c:1424-1426); slow keeps a
	 * stable top 8 by match length of all hits of the seed (the qsort of src/cly.c:1590) */
#define DSB_SM_KEEP(R)                                                                         \
	do {                                                                                   \
		if ((R).match_len >= L_MIN) {                                                  \
			if (!SLOW) {                                                           \
				m_r[n_m] = (R);                                                \
				n_m++;                                                         \
			} else {                                                               \
				(R).read_offset = string_index - (R).match_len;                \
				total++;                                                       \
				int p_ = 0;                                                    \
				while (p_ < n_top && top[p_].match_len >= (R).match_len)       \
					p_++;                                                  \
				if (p_ < DSB_MEM_SEARCH_SLOW) {                                \
					for (int q_ = DSB_MIN(n_top, DSB_MEM_SEARCH_SLOW - 1); q_ > p_; q_--) \
						top[q_] = top[q_ - 1];                         \
					top[p_] = (R);                                         \
					n_top = DSB_MIN(n_top + 1, DSB_MEM_SEARCH_SLOW);       \
				}                                                              \
			}                                                                      \
		}                                                                              \
	} while (0)
#ifdef DSB_EMU_PROF /* test-only emulator profile (tests/emu): trips of the state machine per seed */
	uint64_t prof_trips = 0, prof_maps = 0;
#define DSB_EMU_PROF_START() (prof_trips = 0, prof_maps = 0)
#else
#define DSB_EMU_PROF_START() ((void)0)
#endif
	if (lane < mp)
		DSB_SM_START_SEED(lane);
	uint64_t t_sm = DSB_T0();
	for (;;) {
		uint64_t act = dsb_gballot<GW>(st != DSB_SM_DONE);
		if (!act)
			break;
#ifdef DSB_EMU_PROF
		prof_trips++;
#endif
		uint64_t mapm = dsb_gballot<GW>(st == DSB_SM_MAP);
		int do_map = mapm != 0 && ((uint32_t)__builtin_popcountll(mapm) >= DSB_MIN((uint32_t)DSB_SM_MAP_BATCH, GW) || mapm == act);
		if (w->stats && lane == 0) { /* trip counters (stats kernels): trips, map trips, lanes mapping */
			w->stats[DSB_ST_T_DPM]++;
			if (do_map) {
				w->stats[DSB_ST_T_DPS]++;
				w->stats[DSB_ST_T_FILL] += (uint64_t)__builtin_popcountll(mapm);
			}
		}
		/* ---- MAP: map_seed of hit k_map, batched; its REF_POS entries are spread over the wave.
		 * Items are numbered owner by owner (lane order), REF_POS order inside an owner; a kept
		 * Anchor goes to its owner's staging at the owner's count + the number of kept items of
		 * that owner before it, i.e. the order of the reference's loop (src/cly.c:886-931). */
		if (do_map) {
			uint64_t t1 = DSB_T0();
			int inmap = st == DSB_SM_MAP;
			dsb_mapctx_t cx;
			cx.n_items = 0;
			cx.ret = 0;
			dsb_seedinfo_t s_i = {bin_read, w->L, (uint16_t)ci, s_d->direction};
			uint64_t tp0 = DSB_T0();
			if (inmap) {
				dsb_mem_t *mq = SLOW ? top + k_map : m_r + k_map;
				if (!SLOW)
					mq->read_offset = string_index - mq->match_len;
#ifndef DSB_EXP_NO_PRE
				dsb_map_seed_pre(w, mq, &s_i, &cx);
#endif
			}
			DSB_T1(DSB_ST_T_BUILD, tp0); /* lane 0: wave clocks in map_seed's prefix / suffix part */
#ifdef DSB_EXP_NO_ITEMS
			cx.n_items = 0; /* timing experiment only */
#endif
			uint32_t cnt = inmap ? cx.n_items : 0;
			uint32_t tot, pfx = dsb_gscan<GW>(cnt, &tot);
			uint32_t n_before = w->n_anc;
			int32_t *own = lds + 2 * dsb_gbase<GW>(), *omax = own + GW; /* LDS: owner lane of each item of a chunk; kept max per owner (the group's part) */
			omax[lane] = 0;
			for (uint32_t cb = 0; cb < tot; cb += GW) {
				uint32_t it = cb + lane;
				if (inmap) /* owners label their items of this chunk */
					for (uint32_t q = DSB_MAX(pfx, cb); q < pfx + cnt && q < cb + GW; q++)
						own[q - cb] = (int32_t)lane;
				dsb_wsync();
				int o = it < tot ? own[lane] : 0;
				dsb_wsync();
				dsb_mapctx_t oc;
				uint32_t opfx = (uint32_t)dsb_gshfl_any<GW>((int)pfx, o);
				oc.rp_s = ((uint64_t)(uint32_t)dsb_gshfl_any<GW>((int)(uint32_t)(cx.rp_s >> 32), o) << 32) |
					  (uint32_t)dsb_gshfl_any<GW>((int)(uint32_t)cx.rp_s, o);
				oc.q_off = dsb_gshfl_any<GW>(cx.q_off, o);
				oc.l_m = (uint32_t)dsb_gshfl_any<GW>((int)cx.l_m, o);
				oc.u_off = (uint32_t)dsb_gshfl_any<GW>((int)cx.u_off, o);
				uint32_t pk1 = (uint32_t)cx.am_mtch | ((uint32_t)(uint16_t)cx.am_score << 16);
				uint32_t pk2 = (uint32_t)cx.am_ll | ((uint32_t)cx.am_le << 8) | ((uint32_t)cx.am_rl << 16) |
					       ((uint32_t)cx.am_re << 24);
				uint32_t pk3 = (uint32_t)cx.ref_l | ((uint32_t)cx.ref_r << 1) | ((ci & 0xffffu) << 16);
				pk1 = (uint32_t)dsb_gshfl_any<GW>((int)pk1, o);
				pk2 = (uint32_t)dsb_gshfl_any<GW>((int)pk2, o);
				pk3 = (uint32_t)dsb_gshfl_any<GW>((int)pk3, o);
				uint32_t o_n = (uint32_t)dsb_gshfl_any<GW>((int)n_before, o);
				oc.am_mtch = (uint16_t)pk1;
				oc.am_score = (int16_t)(pk1 >> 16);
				oc.am_ll = (uint8_t)pk2; oc.am_le = (uint8_t)(pk2 >> 8); oc.am_rl = (uint8_t)(pk2 >> 16);
				oc.am_re = (uint8_t)(pk2 >> 24);
				oc.ref_l = (uint8_t)(pk3 & 1);
				oc.ref_r = (uint8_t)((pk3 >> 1) & 1);
				dsb_seedinfo_t os = {bin_read, w->L, (uint16_t)(pk3 >> 16), s_d->direction};
				dsb_anchor_t an;
				uint64_t ti0 = DSB_T0();
				/* q_buff[-1] is the loop's 0xAA until a push of this call grows the reference's anchor
				 * vector, which depends on the anchors of every seed before this one: an item after
				 * the first whose result would change with it sends its seed to the in-order replay */
				int amb = 0;
				int pass = it < tot ? dsb_map_item(w, &oc, it - opfx, &os, &an, DSB_QB_M1_LOOP, it > opfx ? &amb : 0) : 0;
				DSB_T1(DSB_ST_T_MATCH, ti0); /* lane 0: wave clocks in the REF_POS items themselves */
				uint64_t pm = dsb_gballot<GW>(pass);
				uint64_t ambm = dsb_gballot<GW>(amb);
				uint32_t start = opfx > cb ? opfx - cb : 0; /* the owner's first item in this chunk */
				uint64_t before = (lane == 0 ? 0 : (~0ull >> (64 - lane))) & ~(start == 0 ? 0 : (~0ull >> (64 - start)));
				uint32_t dest = o_n + (uint32_t)__builtin_popcountll(pm & before);
				if (pass && dest < Sp) {
					pool[(uint64_t)o * Sp + dest] = an;
					if (w->stats) w->stats[DSB_ST_ANCHOR]++;
				}
				if (pass)
					dsb_lds_max(omax + o, (int32_t)an.score);
				/* owners: count their kept items of this chunk */
				if (inmap) {
					uint32_t lo = pfx > cb ? pfx - cb : 0, hi = DSB_MIN(pfx + cnt, cb + GW) - cb;
					if (pfx + cnt > cb && lo < hi) {
						uint64_t mine = (hi >= 64 ? ~0ull : ((1ull << hi) - 1)) & ~(lo == 0 ? 0ull : ((1ull << lo) - 1));
						n_before += (uint32_t)__builtin_popcountll(pm & mine);
						if (ambm & mine)
							seed_amb = 1;
					}
				}
			}
			dsb_wsync();
			if (inmap) {
				int c_score = cx.ret;
				if (cx.n_items) { /* max over the kept anchors (the reference's max_s) */
					if (n_before > Sp) {
						w->overflow |= 1;
						n_before = Sp;
					}
					c_score = omax[lane];
					w->n_anc = n_before;
				}
				max_score = DSB_MAX(c_score, max_score);
				k_map++;
#ifdef DSB_EMU_PROF
				prof_maps++;
#endif
			}
			DSB_T1(DSB_ST_T_MAP, t1); /* lane 0: wave clocks in the batched map steps */
		}
		if (st == DSB_SM_MAP && do_map) {
			if (k_map == n_m) {
				if (SLOW || w->overflow) {
					st = DSB_SM_FIN;
				} else {
					if (max_score > 35)
						j -= 7;
					if (max_score > 256) {
						if (max_score > 512)
							skip = 1;
						st = DSB_SM_FIN;
					} else
						st = DSB_SM_J;
				}
			}
		}
		/* ---- EXT / SS: one occ evaluation shared by both kinds of step */
		if (st == DSB_SM_EXT || st == DSB_SM_SS) {
			int ext = st == DSB_SM_EXT;
			uint8_t c1 = ext ? *str : (uint8_t)0xff;
			uint64_t o1 = dsb_occ_w(w, ext ? sp : ss_sp, &c1);
			if (ext) {
				uint8_t c2 = *str;
				uint64_t o2 = dsb_occ_w(w, ep, &c2);
				str--;
				uint64_t new_sp = ix->rank[c1] + o1, new_ep = ix->rank[c2] + o2;
				int done = 0, none = 0;
				if (match_len >= L_MIN - 1) {
					if (new_sp + (uint64_t)MAX_RST >= new_ep)
						done = 1;
					else if (match_len >= l_max)
						none = 1;
				}
				if (!done && !none && new_sp + 1 >= new_ep)
					done = 1;
				if (none || (done && new_sp >= new_ep)) { /* no hit at this position */
					n_m = 0;
					j -= 2;
					st = DSB_SM_J;
				} else if (done) {
					row = new_sp;
					row_end = new_ep;
					row_single = (new_sp + 1 == new_ep);
					n_m = 0;
					st = DSB_SM_ROW;
				} else {
					match_len++;
					sp = new_sp;
					ep = new_ep;
				}
			} else {
				/* bwt_single_search: the symbol at ss_sp is c1, LF = o1 + rank */
				uint64_t new_sp = o1 + ix->rank[c1];
				int end = 0, dup = 0;
				if (c1 != *ss_str) {
					end = 1;
				} else {
					ss_len++;
					ss_str--;
					if (dsb_set_insert(new_sp, &hs) == 0)
						dup = 1;
					else
						ss_sp = new_sp;
				}
				if (!end && !dup && ss_len >= ss_max)
					end = 1;
				if (!end && !dup) { /* SA-sample bookkeeping at the top of the next step */
					if ((ss_sp & 7) == 0) {
						sa_sp = ss_sp;
						sa_sp_l = 0;
					} else
						sa_sp_l--;
				} else {
					dsb_mem_t r;
					r.kmer_index = 0;
					r.read_offset = 0;
					r.sp = ss_sp;
					r.match_len = dup ? -1000 : ss_len;
					r.sa_sp = sa_sp;
					r.sa_sp_l = sa_sp_l;
					r.match_len += match_len + 1;
					DSB_SM_KEEP(r);
					row++;
					st = DSB_SM_ROW;
				}
			}
		}
		/* ---- ROW: rows of the final interval (sp_set), start single searches */
		if (st == DSB_SM_ROW) {
			for (;;) {
				if (row >= row_end) {
					if (SLOW || n_m == 0) {
						j -= 2;
						st = DSB_SM_J;
					} else {
						j -= 3;
						k_map = 0;
						max_score = 0;
						st = DSB_SM_MAP;
					}
					break;
				}
				if (dsb_set_insert(row, &hs) == 0) {
					row = row_single ? row_end : row + 1;
					continue;
				}
				ss_sp = row;
				ss_str = str;
				ss_max = DSB_MAX(0, l_max - match_len);
				ss_len = 0;
				sa_sp = ~0ull;
				sa_sp_l = 0;
				if (ss_max <= 0) { /* the single search ends before its first step */
					dsb_mem_t r;
					r.kmer_index = 0;
					r.read_offset = 0;
					r.sp = ss_sp;
					r.match_len = match_len + 1;
					r.sa_sp = sa_sp;
					r.sa_sp_l = sa_sp_l;
					DSB_SM_KEEP(r);
					row++;
					continue;
				}
				if ((ss_sp & 7) == 0) {
					sa_sp = ss_sp;
					sa_sp_l = 0;
				} else
					sa_sp_l--;
				st = DSB_SM_SS;
				break;
			}
		}
		/* ---- FIN: close the seed (anchors below its top score are useless) and record it */
		if (st == DSB_SM_FIN) {
			if (!w->overflow) {
				int top_score = 35;
				for (uint32_t a = a_b; a < w->n_anc; a++)
					top_score = DSB_MAX(top_score, (int)stg[a].score);
				for (uint32_t a = a_b; a < w->n_anc; a++)
					stg[a].anchor_useless = (stg[a].score < top_score) ? 1 : 0;
			}
#ifdef DSB_EMU_PROF
			dsb_emu_prof_seed(SLOW, k, prof_trips, prof_maps);
#endif
			rec[2 * k] = (pr << 31) | (lane << 24) | a_b;
			rec[2 * k + 1] = ((uint32_t)(!SLOW && skip && !w->overflow) << 31) | ((uint32_t)(w->overflow != 0) << 30) |
					 ((uint32_t)(seed_amb != 0) << 29) | (w->overflow ? 0u : (w->n_anc - a_b));
		}
		/* ---- hand the next top seeds to the lanes that finished one, in lane order */
		uint64_t finm = dsb_gballot<GW>(st == DSB_SM_FIN);
		if (finm) {
			uint64_t below = (lane == 0) ? 0 : (finm & (~0ull >> (64 - lane)));
			uint32_t mine = next_k + (uint32_t)__builtin_popcountll(below);
			next_k += (uint32_t)__builtin_popcountll(finm);
			if (st == DSB_SM_FIN) {
				if (w->overflow || mine >= mp)
					st = DSB_SM_DONE; /* an overflowed lane's staging is full: it retires */
				else
					DSB_SM_START_SEED(mine);
			}
		}
		/* ---- J: start the FM search at position j of the seed */
		if (st == DSB_SM_J) {
			if (SLOW ? j < 1 : j < min_index) {
				if (SLOW && total > 0) { /* map the kept top hits (src/cly.c:1590-1597) */
					n_m = n_top;
					k_map = 0;
					st = DSB_SM_MAP;
				} else
					st = DSB_SM_FIN;
			} else {
				int kmer_index = (int)seed_off + j;
				/* (kmer_at(...) & DSB_PRE_IDX_MASK), computed once per position by k_seed */
				uint64_t pre_v = DSB_SEED_PRE ? w->pre[(s_d->strand ? w->L : 0) + (uint32_t)kmer_index]
							      : (dsb_kmer_at(bin_read + kmer_index, l_ek, ix->single_base_max) & DSB_PRE_IDX_MASK);
				string_index = kmer_index + l_ek - 1;
				if (w->stats) w->stats[DSB_ST_MEMSEARCH]++;
				sp = dsb_gld(ix->hash_index + pre_v);
				ep = dsb_gld(ix->hash_index + pre_v + 1);
				str = bin_read + string_index - DSB_L_PRE_IDX;
				match_len = DSB_L_PRE_IDX;
				l_max = string_index;
				n_m = 0;
				st = DSB_SM_EXT;
			}
		}
	}
	DSB_T1(DSB_ST_T_MEM, t_sm); /* lane 0: wave clocks in the whole state machine */
#undef DSB_SM_START_SEED
#undef DSB_SM_KEEP
#undef DSB_EMU_PROF_START
	dsb_wsync();
	if (pr == 0) { /* the seeds pass 1 runs again: records still flagged overflowed, in order */
		for (uint32_t gb = 0; gb < m; gb += GW) {
			uint32_t kk = gb + lane;
			int o = kk < m && ((rec[2 * kk + 1] >> 30) & 1);
			uint64_t bm = dsb_gballot<GW>(o);
			uint64_t below = (lane == 0) ? 0 : (bm & (~0ull >> (64 - lane)));
			if (o)
				klist[n_ovf + (uint32_t)__builtin_popcountll(below)] = kk;
			n_ovf += (uint32_t)__builtin_popcountll(bm);
		}
		dsb_wsync();
		if (n_ovf && w->stats && lane == 0)
			w->stats[DSB_ST_PASS2] += n_ovf;
		S2 = (w->dbg & 32) ? 2 : cap0 / DSB_MIN((uint32_t)GW, DSB_MAX(n_ovf, 1u));
	}
	} /* passes */
	w->anc = anc0;
	w->n_anc = n0;
	w->cap.anc = cap0;
	w->overflow = of0;
	/* ---- skip rule + ordered compaction over the seed records */
	int last_trig = 0;
	uint32_t last_ci = 0;
	for (uint32_t gb = 0; gb < m; gb += GW) {
		uint32_t kk = gb + lane;
		uint32_t gn = DSB_MIN((uint32_t)GW, m - gb);
		int act = kk < m;
		uint32_t cix = act ? tix[kk] : 0;
		uint32_t r0 = act ? rec[2 * kk] : 0, r1 = act ? rec[2 * kk + 1] : 0;
		int trig = (int)(r1 >> 31), ovf = (int)((r1 >> 29) & 3) != 0; /* overflowed, or replayed for q_buff[-1] */
		uint32_t cnt = r1 & 0x1fffffffu, src_lane = (r0 >> 24) & 0x7fu, src_off = r0 & 0xffffffu, pool_ = r0 >> 31;
		uint64_t tm = dsb_gballot<GW>(act && trig);
		uint64_t om = dsb_gballot<GW>(act && ovf);
		uint64_t skipm = 0;
		int lt = last_trig;
		uint32_t lc = last_ci;
		int unknown = 0;
		for (uint32_t q = 0; q < gn; q++) {
			uint32_t cq = (uint32_t)dsb_gshfl<GW>((int)cix, (int)q);
			if (lt && cq == lc + 1) {
				skipm |= 1ull << q;
				lt = 0;
				continue;
			}
			if ((om >> q) & 1)
				unknown = 1;
			lt = (int)((tm >> q) & 1);
			lc = cq;
		}
		if (!unknown) {
			last_trig = lt;
			last_ci = lc;
			if ((skipm >> lane) & 1)
				cnt = 0;
			uint32_t tot, off = dsb_gscan<GW>(cnt, &tot);
			if (w->n_anc + tot > w->cap.anc) {
				w->overflow |= 1;
				dsb_wsync();
				return;
			}
			const dsb_anchor_t *src = (pool_ ? w->anc_tmp2 + (uint64_t)src_lane * S2 : w->anc_tmp + (uint64_t)src_lane * S) + src_off;
			for (uint32_t e = 0; e < cnt; e++)
				w->anc[w->n_anc + off + e] = src[e];
			w->n_anc += tot;
		} else { /* seed by seed, in order, deciding the skips as the reference does */
			for (uint32_t q = 0; q < gn; q++) {
				uint32_t cq = (uint32_t)dsb_gshfl<GW>((int)cix, (int)q);
				if (last_trig && cq == last_ci + 1) {
					last_trig = 0;
					continue;
				}
				if ((om >> q) & 1) { /* replay on every lane, straight into the anchor vector */
					if (w->stats && lane == 0)
						w->stats[DSB_ST_REPLAY]++;
					if (SLOW) {
						dsb_slow_seed(w, s_d, cq, &hs, top);
						last_trig = 0;
					} else
						last_trig = dsb_fast_seed(w, s_d, cq, &hs);
					if (w->overflow) {
						dsb_wsync();
						return;
					}
				} else {
					last_trig = (int)((tm >> q) & 1);
					uint32_t kc = (uint32_t)dsb_gshfl<GW>((int)cnt, (int)q);
					uint32_t sl = (uint32_t)dsb_gshfl<GW>((int)src_lane, (int)q), so = (uint32_t)dsb_gshfl<GW>((int)src_off, (int)q);
					if (w->n_anc + kc > w->cap.anc) {
						w->overflow |= 1;
						dsb_wsync();
						return;
					}
					uint32_t sp_ = (uint32_t)dsb_gshfl<GW>((int)pool_, (int)q);
					const dsb_anchor_t *src = (sp_ ? w->anc_tmp2 + (uint64_t)sl * S2 : w->anc_tmp + (uint64_t)sl * S) + so;
					for (uint32_t e = lane; e < kc; e += GW)
						w->anc[w->n_anc + e] = src[e];
					w->n_anc += kc;
				}
				last_ci = cq;
				dsb_wsync();
			}
		}
		dsb_wsync();
	}
	if (SLOW)
		w->fast_classify = 0;
}

/* fast_classify / slow_classify with one wavefront per read: the per-lane state machine */
/* lds: 2 x DSB_WV int32 of workgroup-local memory; hset: the wave's sp_set tables, slot tags from
 * `tag` on (dsb_hset_make).  Returns the lane's last generation: the wave's maximum + 1 is the
 * next free tag offset of these tables. */
template <int G = 64>
DSB_HDN uint32_t dsb_fast_classify_sm(dsb_read_ws *w, const dsb_sdir_t *s_d, uint64_t *hset, uint64_t tag, int32_t *lds,
				      uint64_t *lt = 0)
{
	dsb_hset_t hs = dsb_hset_make(hset, tag, lt);
	dsb_seed_sm<false, G>(w, s_d, &hs, w->mem, lds);
	return hs.gen;
}
template <int G = 64>
DSB_HDN uint32_t dsb_slow_classify_sm(dsb_read_ws *w, const dsb_sdir_t *sd, uint64_t *hset, uint64_t tag, dsb_mem_t *memtmp,
				      int32_t *lds, uint64_t *lt = 0)
{
	dsb_hset_t hs = dsb_hset_make(hset, tag, lt);
	dsb_seed_sm<true, G>(w, sd, &hs, memtmp, lds);
	return hs.gen;
}

/* ------------------------------------------------------------------ chaining */
DSB_HD dsb_chain_t *dsb_push_chain(dsb_read_ws *w)
{
	if (w->n_hit >= w->cap.hit) {
		w->overflow |= 4;
		return 0;
	}
	if (w->stats) w->stats[DSB_ST_CHAIN]++;
	return w->hit + w->n_hit++;
}

/* chain_insert_meta, src/cly.c:71-111 */
DSB_HD void dsb_chain_insert_meta(dsb_read_ws *w, uint32_t ai, dsb_chain_t *c, int new_chain, int dis_minus)
{
	dsb_anchor_t *anchor = w->anc + ai;
	uint32_t ref_l = anchor->ref_offset;
	uint32_t ref_r = ref_l + anchor->mtch_len;
	uint32_t read_l = anchor->index_in_read;
	uint32_t read_r = read_l + anchor->mtch_len;
	if (new_chain) {
		anchor->chain_id = (uint16_t)c->chain_id;
		anchor->pre = -1;
		c->ref_ID = anchor->ref_ID;
		c->direction = anchor->direction;
		c->q_t_dis = (int32_t)(anchor->ref_offset - anchor->index_in_read);
		c->t_st = ref_l;
		c->t_ed = ref_r;
		c->q_st = read_l;
		c->q_ed = read_r;
		c->with_top_anchor = !anchor->anchor_useless;
		c->anchor_number = 1;
		c->sum_score = anchor->duplicate ? 1 : (uint32_t)(int32_t)anchor->score;
		c->indel = 0;
		c->cur = (int32_t)ai;
	} else {
		anchor->chain_id = (uint16_t)c->chain_id;
		c->with_top_anchor |= (!anchor->anchor_useless);
		if (c->q_ed >= read_r)
			return;
		c->t_ed = DSB_MAX(ref_r, c->t_ed);
		c->q_ed = read_r;
		anchor->pre = c->cur;
		c->cur = (int32_t)ai;
		c->q_t_dis = (int32_t)(anchor->ref_offset - anchor->index_in_read);
		c->indel += dis_minus;
		c->anchor_number++;
		c->sum_score += anchor->duplicate ? 1 : (uint32_t)(int32_t)anchor->score;
	}
}

/* chain_insert_M2, src/cly.c:200-223 */
DSB_HD void dsb_chain_insert_M2(dsb_read_ws *w, uint32_t ai)
{
	dsb_anchor_t *anchor = w->anc + ai;
	uint8_t direction = anchor->direction;
	uint32_t ref_ID = anchor->ref_ID;
	int32_t dis = (int32_t)(anchor->ref_offset - anchor->index_in_read);
	int dis_minus = 0;
	for (uint32_t k = 0; k < w->n_hit; k++) {
		dsb_chain_t *c_s = w->hit + k;
		if (c_s->direction == direction && c_s->ref_ID == ref_ID &&
		    (dis_minus = DSB_ABS(dis - c_s->q_t_dis)) < 30 &&
		    DSB_ABS_U(c_s->t_ed, anchor->ref_offset) < 400) {
			dsb_chain_insert_meta(w, ai, c_s, 0, dis_minus);
			return;
		}
	}
	dsb_chain_t *nc = dsb_push_chain(w);
	if (!nc)
		return;
	nc->chain_id = w->n_hit - 1;
	dsb_chain_insert_meta(w, ai, nc, 1, dis_minus);
}

/* chain_insert_M3, src/cly.c:237-322 (anchors sorted in place first, src/cly.c:242) */
/* Anchor_cmp_by_chr_ID_and_pos under glibc msort == stable ascending sort by
 * (ref_ID, direction, ref_offset).  WAVE: bitonic sort of (key, index) pairs (a total order,
 * so the same permutation as any stable sort), keys/indices staged in hit_tmp. */
#define DSB_SORT_LDS 512
/* the slow-mode resolves' LDS sorts (RESOLVE_S0/S1: ~2% of the reads, a few with thousands of
 * anchors).  4096 entries (48 KB: sorts of up to 4096 anchors and M3 segments of up to the
 * reference's 1024 anchors in LDS) took one read's 64-85 ms per chunk out of HBM, but a 48-KB
 * workgroup waits for a CU with that much LDS free beside the scoring grid of the split: on the C2
 * proxy resolve_s0 + resolve_s1 231 + 50 ms per step at 4096 vs 175 + 2 at 512 (r05_u, 5 steps) */
#ifndef DSB_SORT_LDS_SLOW
#define DSB_SORT_LDS_SLOW 512
#endif
template <bool WAVE>
DSB_HD void dsb_sort_anchors(dsb_read_ws *w)
{
	uint32_t n = w->n_anc;
	dsb_anchor_t *A = w->anc;
	if (!WAVE || DSB_SEQ(w, 64)) {
		uint32_t *idx = w->sidx, *tmp = w->stmp;
		for (uint32_t k = 0; k < n; k++) idx[k] = k;
		dsb_msort(idx, tmp, n, [A](uint32_t ia, uint32_t ib) -> int { return dsb_anchor_cmp(A + ia, A + ib); });
		for (uint32_t k = 0; k < n; k++) w->anc_tmp[k] = A[idx[k]];
		for (uint32_t k = 0; k < n; k++) A[k] = w->anc_tmp[k];
		return;
	}
	uint32_t lane = dsb_lane();
	uint32_t N = 1;
	while (N < n) N <<= 1;
	uint64_t *key = (uint64_t *)w->hit_tmp;
	uint32_t *id = (uint32_t *)(key + N);
	if (w->lds_key && N <= w->lds_n) { /* small sorts run in LDS */
		key = w->lds_key;
		id = w->lds_id;
	}
	for (uint32_t k = lane; k < N; k += DSB_WV) {
		if (k < n) {
			key[k] = ((uint64_t)A[k].ref_ID << 33) | ((uint64_t)(A[k].direction != 0) << 32) | A[k].ref_offset;
			id[k] = k;
		} else {
			key[k] = ~0ull;
			id[k] = 0xffffffffu;
		}
	}
	dsb_wsync();
	for (uint32_t size = 2; size <= N; size <<= 1) {
		for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
			for (uint32_t t = lane; t < N / 2; t += DSB_WV) {
				uint32_t lo = ((t / stride) * stride << 1) + (t % stride);
				uint32_t hi = lo + stride;
				int asc = ((lo & size) == 0);
				uint64_t ka = key[lo], kb = key[hi];
				uint32_t ia = id[lo], ib = id[hi];
				int gt = (ka > kb) || (ka == kb && ia > ib);
				if (gt == asc) {
					key[lo] = kb; key[hi] = ka;
					id[lo] = ib; id[hi] = ia;
				}
			}
			dsb_wsync();
		}
	}
	for (uint32_t k = lane; k < n; k += DSB_WV)
		w->anc_tmp[k] = A[id[k]];
	dsb_wsync();
	for (uint32_t k = lane; k < n; k += DSB_WV)
		A[k] = w->anc_tmp[k];
	dsb_wsync();
}

/* chain_insert_M3's DP on LDS copies of a segment of up to lds_n / 2 anchors (wave kernels): four
 * u32 arrays in the sort keys' 8 * lds_n bytes, two in the ids' 4 * lds_n */
template <bool WAVE>
DSB_HDN void dsb_chain_insert_M3(dsb_read_ws *w)
{
	uint32_t n = w->n_anc;
	dsb_anchor_t *A = w->anc;
	dsb_sort_anchors<WAVE>(w);
	int *score_v = (int *)w->stmp; /* 1024 ints; stmp is free again */
	for (uint32_t chr_st = 0; chr_st < n;) {
		uint32_t chr_ed = chr_st + 1;
		uint32_t ref_ID = A[chr_st].ref_ID;
		uint32_t direction = A[chr_st].direction;
		if (!WAVE || DSB_SEQ(w, 64)) {
			for (; chr_ed < n && A[chr_ed].ref_ID == ref_ID && A[chr_ed].direction == direction &&
			       A[chr_ed].ref_offset - A[chr_ed - 1].ref_offset < 2000;
			     chr_ed++);
		} else { /* the first anchor that ends the segment, 64 at a time (only the first 1025 matter) */
			uint32_t lane = dsb_lane();
			uint32_t kb = chr_st + 1;
			for (; kb < n && kb <= chr_st + 1024; kb += DSB_WV) {
				uint32_t k = kb + lane;
				int fail = k < n && !(A[k].ref_ID == ref_ID && A[k].direction == direction &&
						      A[k].ref_offset - A[k - 1].ref_offset < 2000);
				uint64_t bm = dsb_wballot(fail);
				if (bm) {
					kb += (uint32_t)__builtin_ctzll(bm);
					break;
				}
			}
			chr_ed = DSB_MIN(kb, n);
		}
		if (chr_ed - chr_st > 1024)
			chr_ed = chr_st + 1024;
		int32_t max_anchor = -1;
		int max_score = 0, anchor_max_score;
		uint32_t seg = chr_ed - chr_st;
		const uint32_t M3N = w->lds_n / 2;
		if (WAVE && !DSB_SEQ(w, 64) && w->lds_key && seg <= M3N) {
			/* the segment's DP fields staged in LDS (the sort's key/id arrays are free again):
			 * read offset, reference offset, mtch_len | score << 16, score_v, pre, flags */
			uint32_t lane = dsb_lane();
			uint32_t *Lq = (uint32_t *)w->lds_key, *Lt = Lq + M3N, *Lms = Lt + M3N;
			int32_t *Lsv = (int32_t *)(Lms + M3N);
			int32_t *Lpre = (int32_t *)w->lds_id;
			uint32_t *Lfl = (uint32_t *)w->lds_id + M3N;
			for (uint32_t k = lane; k < seg; k += DSB_WV) {
				const dsb_anchor_t *a = A + chr_st + k;
				Lq[k] = a->index_in_read;
				Lt[k] = a->ref_offset;
				Lms[k] = (uint32_t)a->mtch_len | ((uint32_t)(uint16_t)a->score << 16);
				Lfl[k] = (uint32_t)(a->duplicate != 0) | ((uint32_t)(a->anchor_useless != 0) << 1);
			}
			dsb_wsync();
			for (uint32_t ci = 0; ci < seg; ci++) {
				uint32_t ms = Lms[ci];
				uint32_t c_mtch = ms & 0xffffu;
				anchor_max_score = (int)(int16_t)(ms >> 16);
				int32_t c_pre = -1;
				uint32_t max_t = Lt[ci] + 3;
				uint32_t max_q = Lq[ci] + 3;
				uint64_t best = 0;
				for (int64_t pb = (int64_t)ci - 1; pb >= 0; pb -= DSB_WV) {
					int64_t pi = pb - (int64_t)lane;
					uint64_t cand = 0;
					int brk = 0;
					if (pi >= 0) {
						uint32_t pq = Lq[pi], pt = Lt[pi], pm = Lms[pi] & 0xffffu;
						if (!(pq + pm > max_q) && !(pt + pm > max_t)) {
							if (pq + 1000 < max_q || pt + 1000 < max_t)
								brk = 1;
							else {
								int indel = (int)(pq - pt - (max_q - max_t));
								int ABS_indel = DSB_ABS(indel);
								if (ABS_indel <= 200) {
									int new_score = (int)((uint32_t)(Lsv[pi] + (int)c_mtch - (ABS_indel >> 4)) -
											      ((max_q - pq) >> 8));
									cand = ((uint64_t)((uint32_t)new_score ^ 0x80000000u) << 32) | (uint32_t)(pi + 1);
								}
							}
						}
					}
					uint64_t bm = dsb_wballot(brk);
					if (bm && lane >= (uint32_t)__builtin_ctzll(bm))
						cand = 0;
					best = DSB_MAX(best, cand);
					if (bm)
						break;
				}
				best = dsb_wmax64(best);
				if (best) {
					int bs = (int)((uint32_t)(best >> 32) ^ 0x80000000u);
					if (bs > anchor_max_score) {
						anchor_max_score = bs;
						c_pre = (int32_t)((uint32_t)best - 1);
					}
				}
				if (lane == 0) {
					Lsv[ci] = anchor_max_score;
					Lpre[ci] = c_pre;
				}
				dsb_wsync();
				if (max_score < anchor_max_score) {
					max_score = anchor_max_score;
					max_anchor = (int32_t)ci;
				}
			}
			for (uint32_t k = lane; k < seg; k += DSB_WV)
				A[chr_st + k].pre = Lpre[k] < 0 ? -1 : (int32_t)chr_st + Lpre[k];
			if (max_anchor < 0) { /* NULL dereference in the reference (all scores <= 0): unreachable */
				dsb_wsync();
				w->overflow |= 8;
				return;
			}
			int sum_INDEL = 0, anchor_number = 1;
			int32_t pre = max_anchor;
			uint32_t fl = Lfl[max_anchor];
			int sum_score = (fl & 1) ? 1 : (int)(int16_t)(Lms[max_anchor] >> 16);
			int with_top = !(fl & 2);
			for (; Lpre[pre] != -1; anchor_number++) {
				int32_t pre_ = Lpre[pre];
				sum_INDEL += (int)((Lq[pre] - Lq[pre_]) - (Lt[pre] - Lt[pre_]));
				fl = Lfl[pre];
				with_top |= !(fl & 2);
				sum_score += (fl & 1) ? 1 : (int)(int16_t)(Lms[pre] >> 16);
				pre = pre_;
			}
			uint32_t m_q = Lq[max_anchor], m_t = Lt[max_anchor], m_m = Lms[max_anchor] & 0xffffu;
			uint32_t p_q = Lq[pre], p_t = Lt[pre];
			dsb_wsync();
			dsb_chain_t *nc = dsb_push_chain(w);
			if (!nc)
				return;
			nc->chain_id = w->n_hit - 1;
			nc->ref_ID = ref_ID;
			nc->direction = (uint8_t)direction;
			nc->q_t_dis = (int32_t)(m_t - m_q);
			nc->t_st = p_t;
			nc->t_ed = m_t + m_m;
			nc->q_st = p_q;
			nc->q_ed = m_q + m_m;
			nc->with_top_anchor = (uint8_t)with_top;
			nc->anchor_number = anchor_number;
			nc->sum_score = sum_score;
			nc->indel = sum_INDEL;
			nc->cur = (int32_t)chr_st + max_anchor;
			chr_st = chr_ed;
			continue;
		}
		for (uint32_t ca = chr_st; ca < chr_ed; ca++) {
			dsb_anchor_t *c_a = A + ca;
			c_a->pre = -1;
			anchor_max_score = c_a->score;
			uint32_t max_t = c_a->ref_offset + 3;
			uint32_t max_q = c_a->index_in_read + 3;
			if (!WAVE || DSB_SEQ(w, 64)) {
				for (int64_t pi = (int64_t)ca - 1; pi >= (int64_t)chr_st; pi--) {
					dsb_anchor_t *pre = A + pi;
					if (pre->index_in_read + pre->mtch_len > max_q) continue;
					if (pre->ref_offset + pre->mtch_len > max_t) continue;
					if (pre->index_in_read + 1000 < max_q) break;
					if (pre->ref_offset + 1000 < max_t) break;
					int indel = (int)(pre->index_in_read - pre->ref_offset - (max_q - max_t));
					int ABS_indel = DSB_ABS(indel);
					if (ABS_indel > 200) continue;
					int new_score = (int)((uint32_t)(score_v[pi - chr_st] + c_a->mtch_len - (ABS_indel >> 4)) -
							      ((max_q - pre->index_in_read) >> 8));
					if (new_score > anchor_max_score) {
						anchor_max_score = new_score;
						c_a->pre = (int32_t)pi;
					}
				}
			} else { /* best (score, highest index) over the scan, stopped at the first break */
				uint32_t lane = dsb_lane();
				uint64_t best = 0;
				for (int64_t pb = (int64_t)ca - 1; pb >= (int64_t)chr_st; pb -= DSB_WV) {
					int64_t pi = pb - (int64_t)lane;
					uint64_t cand = 0;
					int brk = 0;
					if (pi >= (int64_t)chr_st) {
						dsb_anchor_t *pre = A + pi;
						if (!(pre->index_in_read + pre->mtch_len > max_q) && !(pre->ref_offset + pre->mtch_len > max_t)) {
							if (pre->index_in_read + 1000 < max_q || pre->ref_offset + 1000 < max_t)
								brk = 1;
							else {
								int indel = (int)(pre->index_in_read - pre->ref_offset - (max_q - max_t));
								int ABS_indel = DSB_ABS(indel);
								if (ABS_indel <= 200) {
									int new_score = (int)((uint32_t)(score_v[pi - chr_st] + c_a->mtch_len -
												 (ABS_indel >> 4)) -
											      ((max_q - pre->index_in_read) >> 8));
									cand = ((uint64_t)((uint32_t)new_score ^ 0x80000000u) << 32) |
									       (uint32_t)(pi + 1);
								}
							}
						}
					}
					uint64_t bm = dsb_wballot(brk);
					if (bm && lane >= (uint32_t)__builtin_ctzll(bm))
						cand = 0;
					best = DSB_MAX(best, cand);
					if (bm)
						break;
				}
				best = dsb_wmax64(best);
				if (best) {
					int bs = (int)((uint32_t)(best >> 32) ^ 0x80000000u);
					if (bs > anchor_max_score) {
						anchor_max_score = bs;
						c_a->pre = (int32_t)((uint32_t)best - 1);
					}
				}
			}
			score_v[ca - chr_st] = anchor_max_score;
			if (max_score < anchor_max_score) {
				max_score = anchor_max_score;
				max_anchor = (int32_t)ca;
			}
		}
		if (max_anchor < 0) { /* NULL dereference in the reference (all scores <= 0): unreachable */
			w->overflow |= 8;
			return;
		}
		int sum_INDEL = 0, anchor_number = 1;
		int32_t pre = max_anchor;
		int sum_score = A[max_anchor].duplicate ? 1 : A[max_anchor].score;
		int with_top = !A[max_anchor].anchor_useless;
		for (; A[pre].pre != -1; anchor_number++) {
			int32_t pre_ = A[pre].pre;
			sum_INDEL += (int)((A[pre].index_in_read - A[pre_].index_in_read) - (A[pre].ref_offset - A[pre_].ref_offset));
			with_top |= !A[pre].anchor_useless;
			sum_score += A[pre].duplicate ? 1 : A[pre].score;
			pre = pre_;
		}
		dsb_chain_t *nc = dsb_push_chain(w);
		if (!nc)
			return;
		nc->chain_id = w->n_hit - 1;
		nc->ref_ID = ref_ID;
		nc->direction = (uint8_t)direction;
		nc->q_t_dis = (int32_t)(A[max_anchor].ref_offset - A[max_anchor].index_in_read);
		nc->t_st = A[pre].ref_offset;
		nc->t_ed = A[max_anchor].ref_offset + A[max_anchor].mtch_len;
		nc->q_st = A[pre].index_in_read;
		nc->q_ed = A[max_anchor].index_in_read + A[max_anchor].mtch_len;
		nc->with_top_anchor = (uint8_t)with_top;
		nc->anchor_number = anchor_number;
		nc->sum_score = sum_score;
		nc->indel = sum_INDEL;
		nc->cur = max_anchor;
		chr_st = chr_ed;
	}
}

/* chain_cmp_by_score, src/cly.c:37-51 */
DSB_HD int dsb_chain_cmp_by_score(const dsb_chain_t *a, const dsb_chain_t *b)
{
	if (a->with_top_anchor != b->with_top_anchor)
		return a->with_top_anchor ? -1 : 1;
	int score_a = (int)(a->sum_score + ((a->q_ed - a->q_st) << 1));
	score_a -= (int)(a->indel << 2);
	int score_b = (int)(b->sum_score + ((b->q_ed - b->q_st) << 1));
	score_b -= (int)(b->indel << 2);
	if (score_a < score_b) return 1;
	if (score_a > score_b) return -1;
	return 0;
}

/* sort the chain vector in place with one of the reference comparators */
template <typename Cmp>
DSB_HD void dsb_sort_chains(dsb_read_ws *w, Cmp cmp)
{
	uint32_t n = w->n_hit;
	if (n <= 1)
		return;
	uint32_t *idx = w->sidx, *tmp = w->stmp;
	for (uint32_t k = 0; k < n; k++) idx[k] = k;
	dsb_chain_t *H = w->hit;
	dsb_msort(idx, tmp, n, [H, cmp](uint32_t a, uint32_t b) -> int { return cmp(H + a, H + b); });
	for (uint32_t k = 0; k < n; k++) w->hit_tmp[k] = H[idx[k]];
	for (uint32_t k = 0; k < n; k++) H[k] = w->hit_tmp[k];
}

/*
 * chain_cmp_by_score as a stable sort on a key (the comparator is a total preorder, so glibc's
 * stable merge sort and any stable sort give the same permutation): with_top_anchor first, then
 * score = sum_score + 2 (q_ed - q_st) - 4 indel (int arithmetic of src/cly.c:37-51) descending.
 * WAVE + LDS: bitonic sort of (key, index) pairs over the wave for <= w->lds_n chains.
 */
template <bool WAVE>
DSB_HD void dsb_sort_chains_by_score(dsb_read_ws *w)
{
	uint32_t n = w->n_hit;
	if (n <= 1)
		return;
	uint32_t N = 1;
	while (N < n) N <<= 1;
	if (!WAVE || !w->lds_key || N > w->lds_n) {
		dsb_sort_chains(w, [](const dsb_chain_t *a, const dsb_chain_t *b) -> int { return dsb_chain_cmp_by_score(a, b); });
		return;
	}
	uint32_t lane = dsb_lane();
	uint64_t *key = w->lds_key;
	uint32_t *id = w->lds_id;
	dsb_chain_t *H = w->hit;
	for (uint32_t k = lane; k < N; k += DSB_WV) {
		if (k < n) {
			int sc = (int)(H[k].sum_score + ((H[k].q_ed - H[k].q_st) << 1));
			sc -= (int)(H[k].indel << 2);
			uint64_t k2 = (uint64_t)((int64_t)0x7fffffff - (int64_t)sc);
			key[k] = ((uint64_t)(H[k].with_top_anchor ? 0 : 1) << 33) | k2;
			id[k] = k;
		} else {
			key[k] = ~0ull;
			id[k] = 0xffffffffu;
		}
	}
	dsb_wsync();
	for (uint32_t size = 2; size <= N; size <<= 1) {
		for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
			for (uint32_t t = lane; t < N / 2; t += DSB_WV) {
				uint32_t lo = ((t / stride) * stride << 1) + (t % stride);
				uint32_t hi = lo + stride;
				int asc = ((lo & size) == 0);
				uint64_t ka = key[lo], kb = key[hi];
				uint32_t ia = id[lo], ib = id[hi];
				int gt = (ka > kb) || (ka == kb && ia > ib);
				if (gt == asc) {
					key[lo] = kb; key[hi] = ka;
					id[lo] = ib; id[hi] = ia;
				}
			}
			dsb_wsync();
		}
	}
	for (uint32_t k = lane; k < n; k += DSB_WV)
		w->hit_tmp[k] = H[id[k]];
	dsb_wsync();
	for (uint32_t k = lane; k < n; k += DSB_WV)
		H[k] = w->hit_tmp[k];
	dsb_wsync();
}

/* resolve_tree, src/cly.c:325-348 */
template <bool WAVE>
DSB_HDN void dsb_resolve_tree(dsb_read_ws *w)
{
	w->n_hit = 0;
	if (w->n_anc < 50)
		for (uint32_t k = 0; k < w->n_anc; k++)
			dsb_chain_insert_M2(w, k);
	else
		dsb_chain_insert_M3<WAVE>(w);
	if (w->overflow)
		return;
	if (w->n_hit > 1)
		dsb_sort_chains_by_score<WAVE>(w);
	uint32_t rst_num = DSB_MIN(5u, w->n_hit);
	while (rst_num < w->n_hit && w->hit[rst_num].with_top_anchor == 1)
		rst_num++;
	w->n_hit = rst_num;
}

/* ------------------------------------------------------------------ scoring (M2) */
/* get_ref forward into an SDP window; WAVE: lanes unpack strided bases, then barrier */
template <bool WAVE>
DSB_HD void dsb_get_ref_win(dsb_read_ws *w, uint8_t *ref_str, uint64_t uni_offset, uint32_t length)
{
	uint64_t tw0 = DSB_T0();
	if (!WAVE || DSB_SEQ(w, 8)) {
		dsb_get_ref_w(w, ref_str, uni_offset, length, 1);
	} else {
		uint32_t lane = dsb_lane();
		if (w->stats && lane == 0) w->stats[DSB_ST_GETREF_B] += (length + 3) / 4;
		if (!dsb_win_ok(w, ref_str, 0, length, 1))
			length = 0;
		uint64_t b0 = uni_offset >> 2;
		uint32_t odd = (uint32_t)(uni_offset & 3);
#ifndef DSB_WIN_WORDS
#define DSB_WIN_WORDS 1 /* 8 bases per lane and load (with the windows in LDS: 83 -> 78 ms) */
#endif
		if (DSB_WIN_WORDS && ((uintptr_t)ref_str & 7) == 0) {
			/* 8 bases per lane: one 8-byte window of the packed reference, one 8-byte store
			 * (bytes past `length` are left as they are: they hold earlier window contents) */
			for (uint32_t k0 = lane * 8; k0 < length; k0 += 8 * DSB_WV) {
				uint64_t pos0 = uni_offset + k0;
				uint64_t B = pos0 >> 2;
				uint64_t out = 0;
				if (B + 16 <= w->ix->ref_bin_padded) {
					uint64_t v = __builtin_bswap64(dsb_gld8u(w->ix->ref_bin + B));
					uint32_t sh = (uint32_t)(pos0 & 3);
					for (int j = 0; j < 8; j++)
						out |= ((v >> (62 - 2 * (sh + j))) & 3) << (8 * j);
				} else {
					for (int j = 0; j < 8; j++) {
						uint64_t p = pos0 + j;
						out |= (uint64_t)((dsb_ref_byte(w->ix, p >> 2) >> (6 - 2 * (p & 3))) & 3) << (8 * j);
					}
				}
				if (k0 + 8 <= length)
					*(uint64_t *)(ref_str + k0) = out;
				else
					for (uint32_t j = 0; j < length - k0; j++)
						ref_str[k0 + j] = (uint8_t)(out >> (8 * j));
			}
		} else {
			for (uint32_t k = lane; k < length; k += DSB_WV) {
				uint32_t pos = odd + k;
				uint8_t b = dsb_ref_byte(w->ix, b0 + (pos >> 2));
				ref_str[k] = (b >> (6 - 2 * (pos & 3))) & 0x3;
			}
		}
		dsb_wsync();
	}
	DSB_T1(DSB_ST_T_WIN, tw0);
}

/* fill ref[lo, hi) with the stack pattern */
template <bool WAVE>
DSB_HD void dsb_fill_pattern_impl(uint8_t *ref, int lo, int hi)
{
	if constexpr (!WAVE) {
		for (int k = lo; k < hi; k++) ref[k] = DSB_STACK_PATTERN;
	} else {
		for (int k = lo + (int)dsb_lane(); k < hi; k += DSB_WV) ref[k] = DSB_STACK_PATTERN;
		dsb_wsync();
	}
}
template <bool WAVE>
DSB_HD void dsb_fill_pattern(dsb_read_ws *w, uint8_t *ref, int lo, int hi)
{
	uint64_t t0 = DSB_T0();
	dsb_fill_pattern_impl<WAVE>(ref, lo, hi);
	DSB_T1(DSB_ST_T_FILL, t0);
}

#define DSB_S_A_KMER_L 9
#define DSB_MIN_SCORE_MEM 12
#define DSB_OVER_SEARCH 50
#define DSB_MAX_SMS_OVERLAP 6

/* sc_hash_idx, src/cly.c:1686-1705 */
#define DSB_SC_OFF_U16 (257 + 256 + 256) /* sc_off: list starts, then the tails and the cursors (scratch) */
#define DSB_SC_FLAT_U16 (2 * 400)
DSB_HD void dsb_sc_hash_idx(dsb_read_ws *w)
{
	/* the lists as the reference links them (a key's entries in insertion order, each list ending
	 * in an empty node), appended through a tail per key instead of a walk to the end; and the same
	 * lists as arrays, sc_flat[sc_off[k] .. sc_off[k + 1]), for the wave's combine_chain */
	dsb_sch_t *sc = w->sch;
	uint16_t *off = w->sc_off, *tail = off + 257, *cur = off + 257 + 256, *flat = w->sc_flat;
	for (int k = 0; k < 256; k++) { sc[k].next = 0; sc[k].seed_ID_s_or_e = 0; tail[k] = (uint16_t)k; cur[k] = 0; }
	for (uint32_t h = 0; h < w->n_hit; h++) {
		const dsb_chain_t *c_h = w->hit + h;
		cur[(c_h->t_st - c_h->q_st) & 0xff]++;
		cur[(c_h->t_ed - c_h->q_ed) & 0xff]++;
	}
	uint32_t acc = 0;
	for (int k = 0; k < 256; k++) {
		off[k] = (uint16_t)acc;
		acc += cur[k];
		cur[k] = off[k];
	}
	off[256] = (uint16_t)acc;
	int sc_con_index = 256;
	for (uint32_t h = 0; h < w->n_hit; h++) {
		const dsb_chain_t *c_h = w->hit + h;
		for (int i = 1; i >= 0; i--) {
			uint16_t c_key = (uint16_t)(((i == 1) ? (c_h->t_st - c_h->q_st) : (c_h->t_ed - c_h->q_ed)) & 0xff);
			uint16_t node = tail[c_key];
			/* seed_ID:15 low bits, s_or_e:1 high bit (gcc bitfield order) */
			uint16_t e = (uint16_t)(((h + 1) & 0x7fff) | ((uint32_t)i << 15));
			sc[node].seed_ID_s_or_e = e;
			sc[node].next = (uint16_t)sc_con_index;
			sc[sc_con_index].next = 0;
			tail[c_key] = (uint16_t)sc_con_index++;
			flat[cur[c_key]++] = e;
		}
	}
}

/*
 * Read 9-mer hash (per strand): heads[key] = the entry of the first position with that key,
 * node[p] = the entry of the position after p in p's list (EMPTY = none).  An entry is
 *   key_len < 18:  bits 0-22 the position, bit 23 "a successor follows" (node[position] is
 *                  valid), bits 24-31 the k-mer bits above the key (kmer >> key_len, <= 8 bits)
 *   key_len == 18: the position (the key is the whole 18-bit k-mer; node[] is always read)
 * (positions are < 2^17 whenever key_len < 18).  A probe whose list has a single element thus
 * costs one load; equality with the probe k-mer is (probe >> key_len) == stored high bits, which
 * is also false for the unmasked probes (> 0x3ffff) of the backward scan, as in the
 * reference's 64-bit compare.
 */
#define DSB_HEMPTY 0xffffffffu
#define DSB_HB_LDS 4096 /* LDS bytes of the wave hash build's key-group slots (power of two) */
DSB_HD uint32_t dsb_hentry(uint32_t pos, uint32_t kmer, int has_next, int kl)
{
	return kl >= 18 ? pos : (pos | ((uint32_t)has_next << 23) | ((kmer >> kl) << 24));
}
DSB_HD uint32_t dsb_hpos(uint32_t e, int kl)
{
	return kl >= 18 ? e : (e & 0x7fffffu);
}
DSB_HD uint32_t dsb_hstep(uint32_t e, const uint32_t *node, int kl)
{
	if (kl >= 18)
		return node[e];
	return (e & 0x800000u) ? node[e & 0x7fffffu] : DSB_HEMPTY;
}
DSB_HD int dsb_hmatch(uint32_t e, uint64_t kmer, int kl)
{
	return (kmer >> kl) == (uint64_t)(kl >= 18 ? 0u : (e >> 24));
}

/* the read 9-mer at c: kmer(c) = (OR_k q[c+k] << 2(8-k)) & 0x3ffff, the rolled value */
DSB_HD uint32_t dsb_q9mer(const uint8_t *q)
{
	uint64_t a = dsb_ld8u(q), b = dsb_ld8u(q + 8);
	uint32_t kmer = 0;
	for (int k = 0; k < 8; k++) kmer = (kmer << 2) | (uint32_t)((a >> (8 * k)) & 0xff);
	kmer = (kmer << 2) | (uint32_t)(b & 0xff);
	return kmer & 0x3ffff;
}

/* key bits of the read 9-mer hash: the reference's choice (the smallest of 10..18 with 2^key >= read
 * length, src/cly.c:2179-2182) + DSB_HASH_KL_DELTA, within 10..18.  The key length is not
 * observable: a lookup keeps exactly the entries whose whole 9-mer equals the probe's, in position
 * order, whatever the number of lists. */
#ifndef DSB_HASH_KL_DELTA
#define DSB_HASH_KL_DELTA 1 /* measured (C1): -1 / 0 / +1 -> scoring 60.4 / 57.5 / 56.2 ms */
#endif
DSB_HD int dsb_hash_kl(uint32_t q_len)
{
	int key_len = 10;
	for (; key_len < 18; key_len++)
		if ((int64_t)(1u << key_len) >= (int64_t)q_len)
			break;
	if (q_len >= (1u << 23)) /* entries hold 23-bit positions below key length 18 */
		return 18;
	key_len += DSB_HASH_KL_DELTA;
	return key_len < 10 ? 10 : (key_len > 18 ? 18 : key_len);
}

/* The read hash built in LDS by its own kernel before the scoring (k_hash_lds, DSB_HASH_LDS):
 * a 2^14-entry head table (64 KB of LDS) holds the key of every read up to 2^23 positions; the
 * key length is not observable (above), so reads whose dsb_hash_kl is longer use 14 bits. */
#ifndef DSB_HASH_LDS
#define DSB_HASH_LDS 1 /* measured (C2, 300k reads): 609.8k -> 632.5k reads/s (profiles/r04_i) */
#endif
#ifndef DSB_HASH_LDS_KL
#define DSB_HASH_LDS_KL 13 /* measured (C2, 300k reads): key length 12 / 13 / 14 -> hash build 39 / 52 / 91 ms, scoring 197 / 169 / 157 ms */
#endif
DSB_HD int dsb_hash_lds_read(uint32_t q_len) { return DSB_HASH_LDS && q_len < (1u << 23); }
DSB_HD int dsb_hash_kl_lds(uint32_t q_len)
{
	int kl = dsb_hash_kl(q_len);
	return kl < DSB_HASH_LDS_KL ? kl : DSB_HASH_LDS_KL;
}
/* the reference's key length (src/cly.c:2179-2182): the roofline counts head-table bytes at it */
DSB_HD int dsb_hash_kl_ref(uint32_t q_len)
{
	int key_len = 10;
	for (; key_len < 18; key_len++)
		if ((int64_t)(1u << key_len) >= (int64_t)q_len)
			break;
	return key_len;
}

/* the strands the scoring looks up (get_score_M2 via delete_small_score_rst, src/cly.c:2186-2194):
 * bit 1 forward, bit 0 reverse, over the hits the scoring keeps (dsb_delete_small_A's trim) */
DSB_HD int dsb_hash_dirs(const dsb_read_ws *w)
{
	uint32_t n = w->n_hit;
	if (n > 200) {
		uint32_t rst_num = 200;
		for (; rst_num < n && w->hit[rst_num].sum_score > 50; rst_num++);
		n = rst_num;
	}
	n = DSB_MIN(400u, n);
	int both_dir = 0;
	for (uint32_t i = 0; i < n; i++) {
		both_dir |= (w->hit[i].direction == DSB_FORWARD) ? 0x2 : 0x1;
		if (both_dir == 3)
			break;
	}
	return both_dir;
}

/* One strand of the read hash by one wave (the wave form of build_hash_table_M2's loop): chunks of
 * 64 positions from the end; inside a chunk each lane finds the nearest higher lane with its key
 * (its list successor) and whether a lower lane has it.  heads: 2^key_len entries (HBM in the
 * scoring kernel, LDS in k_hash_lds), initialised here; lds_hb: DSB_HB_LDS bytes of LDS or 0. */
DSB_HDN void dsb_hash_strand_w(const uint8_t *q, int n_pos, uint32_t *heads, uint32_t *node, int key_len, uint8_t *lds_hb,
			       uint64_t *stats)
{
	uint32_t KEY_MASK = (1u << key_len) - 1;
	uint32_t lane = dsb_lane();
	for (uint32_t k = lane; k <= KEY_MASK; k += DSB_WV) heads[k] = DSB_HEMPTY;
	dsb_wsync();
	for (int cb = n_pos > 0 ? ((n_pos - 1) & ~(DSB_WV - 1)) : -1; cb >= 0; cb -= DSB_WV) {
		int c_pos = cb + (int)lane;
		int act = c_pos < n_pos;
		uint32_t kmer = act ? dsb_q9mer(q + c_pos) : 0;
		int key = act ? (int)(kmer & KEY_MASK) : -1 - (int)lane;
		int has_prev = 0, nxt = -1;
		if (lds_hb) {
			/* every lane writes its id to a byte slot of its key's low bits and reads it
			 * back: lanes sharing a key all lost, or lost to the one of them that won, so
			 * walking the (few) losers and their winners finds every group */
			uint8_t *hb = lds_hb + (key & (DSB_HB_LDS - 1));
			if (act) *hb = (uint8_t)lane;
			dsb_wsync();
			int won = act ? (int)*hb : (int)lane;
			uint64_t lost = dsb_wballot(won != (int)lane);
			nxt = DSB_WV;
			while (lost) {
				int o = __builtin_ctzll(lost);
				lost &= lost - 1;
				int w2 = dsb_wshfl(won, o);
				int k2 = dsb_wshfl(key, o), k3 = dsb_wshfl(key, w2);
				if (k2 == key) {
					if (o < (int)lane) has_prev = 1;
					else if (o > (int)lane) nxt = DSB_MIN(nxt, o);
				}
				if (k3 == key) {
					if (w2 < (int)lane) has_prev = 1;
					else if (w2 > (int)lane) nxt = DSB_MIN(nxt, w2);
				}
			}
			if (nxt == DSB_WV) nxt = -1;
		} else {
			for (int o = DSB_WV - 1; o >= 0; o--) {
				int k2 = dsb_wshfl(key, o);
				if (k2 == key) {
					if (o < (int)lane) has_prev = 1;
					else if (o > (int)lane) nxt = o;
				}
			}
		}
		uint32_t old = act ? heads[key] : DSB_HEMPTY;
		uint32_t ent = dsb_hentry((uint32_t)c_pos, kmer, nxt >= 0 || old != DSB_HEMPTY, key_len);
		uint32_t nent = (uint32_t)dsb_wshfl_any((int)ent, nxt >= 0 ? nxt : (int)lane);
		if (act) {
			if (stats) stats[DSB_ST_HASH_B] += 12;
			node[c_pos] = nxt >= 0 ? nent : old;
			if (!has_prev)
				heads[key] = ent;
		}
		dsb_wsync();
	}
}

/* build_hash_table_M2, src/cly.c:2168-2219: chained 9-mer hash of the read, per strand.
 * Lists hold positions in increasing order (the reference appends in position order), built
 * here from the last position backwards so that only the heads array is needed. */
template <bool WAVE>
DSB_HDN int dsb_build_hash_table(dsb_read_ws *w, int q_len)
{
#if defined(__HIP_DEVICE_COMPILE__)
	if (WAVE && dsb_hash_lds_read((uint32_t)q_len))
		return dsb_hash_kl_lds((uint32_t)q_len); /* built by k_hash_lds before this launch */
#endif
	int both_dir = 0;
	if (!WAVE || DSB_SEQ(w, 1)) {
		for (uint32_t i = 0; i < w->n_hit; i++) {
			both_dir |= (w->hit[i].direction == DSB_FORWARD) ? 0x2 : 0x1;
			if (both_dir == 3)
				break;
		}
	} else {
		/* the hits' directions 64 at a time (one round trip per 64 hits, not one per hit) */
		uint32_t lane = dsb_lane();
		for (uint32_t gb = 0; gb < w->n_hit && both_dir != 3; gb += DSB_WV) {
			uint32_t i = gb + lane;
			int d = i < w->n_hit ? (w->hit[i].direction == DSB_FORWARD ? 2 : 1) : 0;
			both_dir |= (dsb_wballot(d == 2) ? 2 : 0) | (dsb_wballot(d == 1) ? 1 : 0);
		}
	}
	int key_len = dsb_hash_kl((uint32_t)q_len);
	uint32_t KEY_MASK = (1u << key_len) - 1;
	for (int c_dir = 2; c_dir >= 1; c_dir--) {
		if ((c_dir & both_dir) == 0)
			continue;
		uint32_t direction = (c_dir == 1) ? DSB_REVERSE : DSB_FORWARD;
		const dsb_sdir_t *csd = (w->sd[0].direction == direction) ? &w->sd[0] : &w->sd[1];
		int h = (c_dir == 2) ? 0 : 1;
		uint32_t *heads = w->hh[h], *node = w->hn[h];
		const uint8_t *q = w->bin + (csd->strand ? w->L : 0);
		int n_pos = q_len - DSB_S_A_KMER_L + 1;
		if (!WAVE || DSB_SEQ(w, 1)) {
			for (uint32_t k = 0; k <= KEY_MASK; k++) heads[k] = DSB_HEMPTY;
			for (int c_pos = n_pos - 1; c_pos >= 0; c_pos--) {
				uint32_t kmer = dsb_q9mer(q + c_pos);
				uint32_t key = kmer & KEY_MASK;
				uint32_t old = heads[key];
				node[c_pos] = old;
				heads[key] = dsb_hentry((uint32_t)c_pos, kmer, old != DSB_HEMPTY, key_len);
			}
		} else {
			/* algorithmic bytes: the head table at the reference's key length (a longer key is an
			 * implementation choice, not work), + 12 B per position */
			if (w->stats && dsb_lane() == 0) w->stats[DSB_ST_HASH_B] += 4ull << dsb_hash_kl_ref((uint32_t)q_len);
			dsb_hash_strand_w(q, n_pos, heads, node, key_len, w->lds_hb, w->stats);
		}
	}
	return key_len;
}

/* sparse-DP node i of the current window (LDS-resident prefix for the wave kernel) */
#define DSB_SMS_LDS 384
#ifndef DSB_SMS_IN_LDS
#define DSB_SMS_IN_LDS 0 /* experimental (DSB_LDS=1 path); off: sms entries stay in the workspace */
#endif
DSB_HD dsb_spd_t *dsb_sms(dsb_read_ws *w, uint64_t i)
{
#if DSB_SMS_IN_LDS
	return (w->sms_lds && i < DSB_SMS_LDS) ? w->sms_lds + i : w->sms + i;
#else
	return w->sms + i;
#endif
}

DSB_HD dsb_spd_t *dsb_push_sms(dsb_read_ws *w)
{
	if (w->n_sms >= w->cap.sms) {
		w->overflow |= 16;
		return 0;
	}
	return dsb_sms(w, w->n_sms++);
}

/* MEM_search, src/cly.c:1805-1813 */
/* MEM_search: the byte loop `len < max && *q++ == *t++` (or `*q-- == *t--`) compared 8 bytes
 * per step: the first differing byte is the lowest (forward) / highest (backward) set byte of
 * the XOR.  Same result as the byte loop for every max >= 0. */
#ifndef DSB_MEM_WORDS
#define DSB_MEM_WORDS 1
#endif
/* W consecutive unaligned u64 at p from W + 1 aligned loads, all issued before any is used */
template <int W>
DSB_HD void dsb_ldwu(const uint8_t *p, uint64_t *out)
{
	uint32_t o = (uint32_t)((uintptr_t)p & 7), sh = o * 8;
	const uint64_t *b = (const uint64_t *)(p - o);
	uint64_t v[W + 1];
	for (int k = 0; k <= W; k++) v[k] = b[k];
	for (int k = 0; k < W; k++) out[k] = sh ? (v[k] >> sh) | (v[k + 1] << (64 - sh)) : v[k];
}

DSB_HD int dsb_MEM_search(const uint8_t *q, const uint8_t *t, int forward, int max)
{
	int len = 0;
	if (DSB_MEM_WORDS > 1 && max > 8) {
		/* long extensions: DSB_MEM_WORDS words of both strings per step, one dependent round
		 * trip per 8 * DSB_MEM_WORDS bytes instead of per 8 (the bytes past `max` are ignored) */
		const int W = DSB_MEM_WORDS, NB = 8 * DSB_MEM_WORDS;
		while (len < max) {
			uint64_t a[DSB_MEM_WORDS], b[DSB_MEM_WORDS];
			if (forward) {
				dsb_ldwu<DSB_MEM_WORDS>(q + len, a);
				dsb_ldwu<DSB_MEM_WORDS>(t + len, b);
				for (int k = 0; k < W; k++) {
					uint64_t x = a[k] ^ b[k];
					if (x) {
						len += 8 * k + (__builtin_ctzll(x) >> 3);
						return DSB_MIN(len, max);
					}
				}
			} else { /* words k = W-1 .. 0 cover the NB bytes ending at q - len; the nearest is k = W-1 */
				dsb_ldwu<DSB_MEM_WORDS>(q - len - NB + 1, a);
				dsb_ldwu<DSB_MEM_WORDS>(t - len - NB + 1, b);
				for (int k = W - 1; k >= 0; k--) {
					uint64_t x = a[k] ^ b[k];
					if (x) {
						len += 8 * (W - 1 - k) + (__builtin_clzll(x) >> 3);
						return DSB_MIN(len, max);
					}
				}
			}
			len += NB;
		}
		return max > 0 ? max : 0;
	}
	if (forward) {
		while (len < max) {
			uint64_t x = dsb_ld8u(q + len) ^ dsb_ld8u(t + len);
			if (x) {
				len += __builtin_ctzll(x) >> 3;
				return DSB_MIN(len, max);
			}
			len += 8;
		}
	} else {
		while (len < max) {
			uint64_t x = dsb_ld8u(q - len - 7) ^ dsb_ld8u(t - len - 7);
			if (x) {
				len += __builtin_clzll(x) >> 3;
				return DSB_MIN(len, max);
			}
			len += 8;
		}
	}
	return max > 0 ? max : 0;
}

/* sdp_match, src/cly.c:2330-2435.  q_str: read buffer; t_str: reference window.
 * WAVE: every 4th window position (the only ones looked up) is one lane; a lane's matches
 * keep the hash-list order, lanes keep position order (prefix-sum compaction). */
template <bool WAVE>
DSB_HDN void dsb_sdp_match_impl(dsb_read_ws *w, uint32_t q_bg, uint32_t q_ed, const uint8_t *q_str, const uint8_t *t_str,
			    uint32_t t_len, int key_len, int hslot, uint32_t t_st, int isForward)
{
	if (!WAVE || DSB_SEQ(w, 2)) {
	uint32_t KEY_MASK = (1u << key_len) - 1;
	uint32_t t_kmer_num = t_len - DSB_S_A_KMER_L + 1;
	const uint32_t *heads = w->hh[hslot], *hnode = w->hn[hslot];
	if (isForward) {
		const uint8_t *c_t_str = t_str + 4;
		uint64_t kmer = 0;
		for (int k = 0; k < DSB_S_A_KMER_L; k++) kmer = (kmer << 2) | c_t_str[k];
		kmer >>= 2;
		for (int i = 4; i < (int)t_kmer_num; i++, c_t_str++) {
			kmer = ((kmer << 2) | c_t_str[DSB_S_A_KMER_L - 1]) & 0x3ffff;
			if ((i & 0x03) != 0)
				continue;
			for (uint32_t e = heads[kmer & KEY_MASK]; e != DSB_HEMPTY; e = dsb_hstep(e, hnode, key_len)) {
				if (!dsb_hmatch(e, kmer, key_len))
					continue;
				uint32_t q_pos = dsb_hpos(e, key_len);
				if (q_pos >= q_bg && q_pos <= q_ed) {
					int back_len = dsb_MEM_search(q_str + q_pos - 1, c_t_str - 1, 0, 4);
					if (back_len < 4 || i == 4) {
						uint32_t max_search = q_ed - q_pos - 1;
						max_search = DSB_MIN(max_search, t_len - i - 1) + DSB_OVER_SEARCH;
						int forward_len = dsb_MEM_search(q_str + q_pos + DSB_S_A_KMER_L, c_t_str + DSB_S_A_KMER_L, 1,
										 (int)max_search);
						int total_len = back_len + forward_len + 1;
						if (total_len >= 4) {
							dsb_spd_t *p = dsb_push_sms(w);
							if (!p) return;
							p->len = total_len;
							p->q_pos = q_pos - back_len;
							p->t_pos = i - back_len + t_st;
						}
					}
				}
			}
		}
	} else {
		const uint8_t *c_t_str = t_str + t_len - DSB_S_A_KMER_L - 4;
		uint64_t kmer = 0;
		for (int k = 0; k < DSB_S_A_KMER_L; k++) kmer = (kmer << 2) | c_t_str[k];
		kmer <<= 2;
		for (int i = 4; i < (int)t_kmer_num; i++, c_t_str--) {
			kmer = (kmer >> 2) | ((uint64_t)c_t_str[0] << 16); /* bit2_preKmerMOVE, no mask */
			if ((i & 0x03) != 0)
				continue;
			for (uint32_t e = heads[kmer & KEY_MASK]; e != DSB_HEMPTY; e = dsb_hstep(e, hnode, key_len)) {
				if (!dsb_hmatch(e, kmer, key_len))
					continue;
				uint32_t q_pos = dsb_hpos(e, key_len);
				if (q_pos >= q_bg && q_pos <= q_ed) {
					int forward_len = dsb_MEM_search(q_str + q_pos + DSB_S_A_KMER_L, c_t_str + DSB_S_A_KMER_L, 1, 4);
					if (forward_len < 4 || i == 4) {
						uint32_t max_search = q_pos;
						max_search = DSB_MIN(max_search, (uint32_t)(c_t_str - t_str)) + DSB_OVER_SEARCH;
						int back_len = dsb_MEM_search(q_str + q_pos - 1, c_t_str - 1, 0, (int)max_search);
						int total_len = back_len + forward_len + 1;
						if (total_len >= 4) {
							dsb_spd_t *p = dsb_push_sms(w);
							if (!p) return;
							p->len = total_len;
							p->q_pos = q_pos - back_len;
							p->t_pos = (uint32_t)(c_t_str - t_str) - back_len + t_st;
						}
					}
				}
			}
		}
	}
	} else {
		uint32_t KEY_MASK = (1u << key_len) - 1;
		uint32_t t_kmer_num = t_len - DSB_S_A_KMER_L + 1;
		int lim = (int)t_kmer_num;
		if (lim <= 4)
			return;
		const uint32_t *heads = w->hh[hslot], *hnode = w->hn[hslot];
		int n_i = (lim - 1) >> 2; /* looked-up positions i = 4m, m = 1..n_i */
		uint32_t lane = dsb_lane();
		if (!dsb_win_ok(w, t_str, isForward ? 0 : -51, (int64_t)t_len + 64, 2))
			return;
#ifndef DSB_MATCH_PF
#define DSB_MATCH_PF 0
#endif
#ifndef DSB_QR_STATS
#define DSB_QR_STATS 0
#endif
		/* the probe 9-mer of position i = 4m and the window byte it starts at */
		auto probe = [&](int m, const uint8_t *&cts) -> uint64_t {
			int i = 4 * m;
			uint64_t kmer = 0;
			if (isForward) { /* ((k << 2) | c) & 0x3ffff rolled: only the 9 bytes at i remain */
				cts = t_str + i;
				kmer = dsb_q9mer(cts);
			} else {
				/* (k >> 2) | (c << 16) rolled without a mask: bytes > 3 (pattern/stale window
				 * bytes, sdp_left's t_offset_global == 0 case) linger for up to 12 steps */
				cts = t_str + ((int)t_len - DSB_S_A_KMER_L - i);
				if (i < 16) {
					const uint8_t *c0 = t_str + ((int)t_len - DSB_S_A_KMER_L - 4);
					uint64_t k0 = 0;
					for (int k = 0; k < DSB_S_A_KMER_L; k++) k0 = (k0 << 2) | c0[k];
					kmer = (k0 << 2) >> (2 * (i - 3));
				}
				/* bytes t_str[t_len - 9 - j], j = i .. i-12, are cts[d], d = i - j: two word loads */
				uint64_t w0 = dsb_ld8u(cts), w1 = dsb_ld8u(cts + 8);
				int dmax = DSB_MIN(12, i - 4);
				for (int d = 0; d <= 12; d++) {
					if (d > dmax)
						break;
					uint64_t b = (d < 8 ? (w0 >> (8 * d)) : (w1 >> (8 * (d - 8)))) & 0xff;
					kmer |= (b << 16) >> (2 * d);
				}
			}
			return kmer;
		};
#ifndef DSB_MATCH_BF
#define DSB_MATCH_BF 0 /* measured: 3 -> scoring 56.7 -> 60.6 ms, 2 -> 59.2 ms (the compare loop and its spills cost more than the head loads): off */
#endif
		/* Forward windows whose read range [q_bg, q_ed] is at most 64 x DSB_MATCH_BF positions
		 * (most sdp_middle windows): the candidates of a probe are the range's positions whose
		 * read 9-mer equals the probe's — exactly the list entries the lookup keeps (key and
		 * high bits equal, position in the range, in increasing position order) — so they are
		 * found by comparing the probes with the range's 9-mers held in registers (3 per lane)
		 * instead of head / node loads from the read hash.  Candidates go to 64 LDS slots in
		 * (probe, position) order and are extended one per lane; accepted matches are appended
		 * in that order, as the reference's loop appends them. */
#if DSB_MATCH_BF
		if (isForward && w->lds_cand && w->L >= DSB_S_A_KMER_L) {
			uint32_t qhi = DSB_MIN(q_ed, w->L - DSB_S_A_KMER_L); /* the hash holds positions < L - 8 */
			uint32_t nr = q_bg <= qhi ? qhi - q_bg + 1 : 0;
			if (nr <= (uint32_t)(DSB_WV * DSB_MATCH_BF)) {
				if (w->stats && lane == 0) { w->stats[DSB_ST_NWIN]++; w->stats[DSB_ST_NBATCH] += (n_i + DSB_WV - 1) / DSB_WV; }
				if (nr == 0)
					return;
				uint32_t rk[DSB_MATCH_BF];
				for (int j = 0; j < DSB_MATCH_BF; j++) {
					uint32_t qq = lane + (uint32_t)(DSB_WV * j);
					rk[j] = qq < nr ? dsb_q9mer(q_str + q_bg + qq) : 0xffffffffu;
				}
				uint16_t *cl = w->lds_cand;
				for (int mb = 0; mb < n_i; mb += DSB_WV) {
					int np = DSB_MIN(DSB_WV, n_i - mb);
					const uint8_t *pc_t = t_str;
					uint32_t pk = (int)lane < np ? (uint32_t)probe(mb + (int)lane + 1, pc_t) : 0xfffffffeu;
					uint32_t nc = 0; /* candidates in the slots (uniform) */
					/* extend the slotted candidates, one per lane, and append the matches in order */
					auto flush = [&]() {
						dsb_wsync();
						uint32_t ok = 0;
						dsb_spd_t e = {0, 0, 0, 0};
						if (lane < nc) {
							uint32_t c = cl[lane];
							int m = mb + (int)(c >> 10) + 1, i = 4 * m;
							uint32_t q_pos = q_bg + (c & 1023u);
							const uint8_t *c_t_str = t_str + i;
							if (w->stats) w->stats[DSB_ST_NCAND]++;
							int back_len = dsb_MEM_search(q_str + q_pos - 1, c_t_str - 1, 0, 4);
							if (back_len < 4 || i == 4) {
								uint32_t max_search = q_ed - q_pos - 1;
								max_search = DSB_MIN(max_search, t_len - i - 1) + DSB_OVER_SEARCH;
								int forward_len = dsb_MEM_search(q_str + q_pos + DSB_S_A_KMER_L, c_t_str + DSB_S_A_KMER_L,
												 1, (int)max_search);
								int total_len = back_len + forward_len + 1;
								if (total_len >= 4) {
									e.len = total_len;
									e.q_pos = q_pos - back_len;
									e.t_pos = i - back_len + t_st;
									ok = 1;
								}
							}
						}
						uint32_t tot, off = dsb_wscan(ok, &tot);
						if (tot) {
							if (w->n_sms + tot > w->cap.sms) {
								w->overflow |= 16;
							} else {
								if (ok) { dsb_spd_t *d = dsb_sms(w, w->n_sms + off); d->len = e.len; d->q_pos = e.q_pos; d->t_pos = e.t_pos; }
								w->n_sms += tot;
							}
						}
						nc = 0;
						dsb_wsync();
					};
					for (int p = 0; p < np; p++) {
						uint32_t pkp = (uint32_t)dsb_wshfl((int)pk, p);
						for (int j = 0; j < DSB_MATCH_BF; j++) {
							uint64_t mk = dsb_wballot(rk[j] == pkp);
							if (!mk)
								continue;
							uint32_t cnt = (uint32_t)__builtin_popcountll(mk);
							if (nc + cnt > (uint32_t)DSB_WV) {
								flush();
								if (w->overflow) return;
							}
							if ((mk >> lane) & 1) {
								uint64_t below = lane == 0 ? 0 : (mk & (~0ull >> (64 - lane)));
								cl[nc + (uint32_t)__builtin_popcountll(below)] = (uint16_t)(((uint32_t)p << 10) | (lane + (uint32_t)(DSB_WV * j)));
							}
							nc += cnt;
						}
					}
					if (nc) {
						flush();
						if (w->overflow) return;
					}
				}
				dsb_wsync();
				return;
			}
		}
#endif
#ifndef DSB_QCOPY
#define DSB_QCOPY 0
#endif
#define DSB_BIN_TAIL_BYTES 256 /* bytes after R in the read buffer (dsb_ws.h DSB_BIN_TAIL) */
#ifndef DSB_QCOPY_BYTES
#define DSB_QCOPY_BYTES 768
#endif
		/* The candidates' extensions (MEM_search over the read bytes) read the window's read
		 * range [q_bg, q_ed] and a few bytes around it.  With DSB_QCOPY, when that range fits, the
		 * wave copies it once into LDS (one coalesced load per lane), and an extension whose bytes
		 * all lie inside the copy reads LDS instead of making its own dependent global round
		 * trips; the others read the read buffer.  Same bytes either way.  The LDS address is
		 * always formed as lds_q + (x - qv_lo) with 0 <= x - qv_lo < DSB_QCOPY_BYTES, never as an
		 * LDS pointer moved outside the array and indexed back in (round 3's version of this
		 * copy did that: an LDS pointer is a 32-bit offset, so lds_q - (qca - q_str) wrapped, and
		 * converted to a flat address then offset by 64-bit arithmetic it pointed outside the
		 * shared aperture - a memory violation on the box). */
		int64_t qv_lo = 1, qv_hi = 0; /* read bytes [qv_lo, qv_hi] are in LDS at lds_q[x - qv_lo] */
#if DSB_QCOPY
		{
			/* the copy stays inside the read buffer (the F | R halves + the tail guard) */
			const uint8_t *qca = (const uint8_t *)((uintptr_t)(q_str + q_bg - 32) & ~(uintptr_t)7);
			if (w->lds_q && q_bg <= q_ed && (int64_t)q_ed - (int64_t)q_bg + 128 <= DSB_QCOPY_BYTES - 16 &&
			    (int64_t)q_bg >= 32 && qca >= w->bin && qca + DSB_QCOPY_BYTES <= w->bin + 2ull * w->L + DSB_BIN_TAIL_BYTES) {
				const uint64_t *src = (const uint64_t *)qca;
				uint64_t *dst = (uint64_t *)w->lds_q;
				for (uint32_t k = lane; k < DSB_QCOPY_BYTES / 8; k += DSB_WV)
					dst[k] = src[k];
				dsb_wsync();
				qv_lo = (int64_t)(qca - q_str);
				qv_hi = qv_lo + DSB_QCOPY_BYTES - 1;
			}
		}
#endif
		/* read byte x of the strand for an access touching bytes [a, b] */
		auto qat = [&](int64_t x, int64_t a, int64_t b) -> const uint8_t * {
			if (DSB_QCOPY && a >= qv_lo && b <= qv_hi)
				return w->lds_q + (x - qv_lo);
			return q_str + x;
		};
		/* software pipeline: the next batch's probe and list head are loaded before this
		 * batch's lists are walked, so that their latency overlaps the walk */
		const uint8_t *n_cts = t_str;
		uint64_t n_kmer = 0;
		uint32_t n_head = DSB_HEMPTY;
		if (DSB_MATCH_PF && (int)lane + 1 <= n_i) {
			n_kmer = probe((int)lane + 1, n_cts);
			n_head = heads[n_kmer & KEY_MASK];
		}
		if (w->stats && lane == 0) w->stats[DSB_ST_NWIN]++;
#if DSB_QR_STATS /* dev: read-range histogram of the windows, in delA slots the phase leaves unused */
		if (w->stats && lane == 0) {
			int64_t hi = DSB_MIN((int64_t)q_ed, (int64_t)w->L - 9), r = hi - (int64_t)q_bg + 1;
			uint64_t *s = w->stats;
			int mid = t_str == w->win + DSB_WIN_MID;
			if (r < 0) r = 0;
			r = DSB_MIN(r, (int64_t)1 << 20);
			if (mid) {
				s[DSB_ST_OCC]++; s[DSB_ST_OCC_NIB] += r; s[DSB_ST_MEMSEARCH] += n_i;
				if (r <= 64) { s[DSB_ST_ANCHOR]++; s[DSB_ST_CHAIN] += n_i; }
				if (r <= 128) { s[DSB_ST_EK1]++; s[DSB_ST_EK2] += n_i; }
				s[DSB_ST_REPLAY] += t_len;
			} else {
				s[DSB_ST_SA]++; s[DSB_ST_UNI] += r; s[DSB_ST_REFPOS] += n_i;
				if (r <= 1024) s[DSB_ST_PASS2]++;
			}
		}
#endif
		for (int mb = 0; mb < n_i; mb += DSB_WV) {
			int m = mb + (int)lane + 1;
			if (w->stats && lane == 0) w->stats[DSB_ST_NBATCH]++;
			uint32_t cnt = 0;
			dsb_spd_t e0 = {0, 0, 0, 0}, e1 = {0, 0, 0, 0};
			const uint8_t *c_t_str = t_str;
			uint64_t kmer = 0;
			uint32_t head = DSB_HEMPTY;
			int i = 4 * m;
			if (DSB_MATCH_PF) {
				c_t_str = n_cts;
				kmer = n_kmer;
				head = n_head;
				n_head = DSB_HEMPTY;
				if (m + DSB_WV <= n_i) {
					n_kmer = probe(m + DSB_WV, n_cts);
					n_head = heads[n_kmer & KEY_MASK];
				}
			} else if (m <= n_i) {
				uint64_t tp0 = DSB_T0();
				kmer = probe(m, c_t_str);
				head = heads[kmer & KEY_MASK];
				DSB_T1(DSB_ST_T_MPROBE, tp0);
			}
			uint64_t tw0 = DSB_T0();
			if (m <= n_i) {
				if (w->stats) w->stats[DSB_ST_LOOKUP]++;
				for (uint32_t he = head; he != DSB_HEMPTY; he = dsb_hstep(he, hnode, key_len)) {
					if (w->stats) w->stats[DSB_ST_NODE]++;
					if (!dsb_hmatch(he, kmer, key_len))
						continue;
					uint32_t q_pos = dsb_hpos(he, key_len);
					if (!(q_pos >= q_bg && q_pos <= q_ed))
						continue;
					if (w->stats) w->stats[DSB_ST_NCAND]++;
					dsb_spd_t e;
					int ok = 0;
					int64_t xb = (int64_t)q_pos - 1, xf = (int64_t)q_pos + DSB_S_A_KMER_L;
					if (isForward) {
						int back_len = dsb_MEM_search(qat(xb, xb - 24, xb + 16), c_t_str - 1, 0, 4);
						if (back_len < 4 || i == 4) {
							uint32_t max_search = q_ed - q_pos - 1;
							max_search = DSB_MIN(max_search, t_len - i - 1) + DSB_OVER_SEARCH;
							int forward_len = dsb_MEM_search(qat(xf, xf - 8, xf + (int64_t)max_search + 16),
											 c_t_str + DSB_S_A_KMER_L, 1, (int)max_search);
							int total_len = back_len + forward_len + 1;
							if (total_len >= 4) {
								e.len = total_len;
								e.q_pos = q_pos - back_len;
								e.t_pos = i - back_len + t_st;
								ok = 1;
							}
						}
					} else {
						int forward_len = dsb_MEM_search(qat(xf, xf - 8, xf + 20), c_t_str + DSB_S_A_KMER_L, 1, 4);
						if (forward_len < 4 || i == 4) {
							uint32_t max_search = q_pos;
							max_search = DSB_MIN(max_search, (uint32_t)(c_t_str - t_str)) + DSB_OVER_SEARCH;
							int back_len = dsb_MEM_search(qat(xb, xb - (int64_t)max_search - 24, xb + 16), c_t_str - 1, 0,
										      (int)max_search);
							int total_len = back_len + forward_len + 1;
							if (total_len >= 4) {
								e.len = total_len;
								e.q_pos = q_pos - back_len;
								e.t_pos = (uint32_t)(c_t_str - t_str) - back_len + t_st;
								ok = 1;
							}
						}
					}
					if (ok) {
						if (cnt == 0) e0 = e;
						else if (cnt == 1) e1 = e;
						cnt++;
					}
				}
			}
			DSB_T1(DSB_ST_T_MWALK, tw0);
			uint32_t tot, off = dsb_wscan(cnt, &tot);
			if (tot == 0)
				continue;
			if (w->n_sms + tot > w->cap.sms) {
				w->overflow |= 16;
				dsb_wsync();
				return;
			}
			uint32_t dst = w->n_sms + off; /* score is left as the buffer holds it */
			if (cnt > 0) { dsb_spd_t *d = dsb_sms(w, dst); d->len = e0.len; d->q_pos = e0.q_pos; d->t_pos = e0.t_pos; }
			if (cnt > 1) { dsb_spd_t *d = dsb_sms(w, dst + 1); d->len = e1.len; d->q_pos = e1.q_pos; d->t_pos = e1.t_pos; }
			if (cnt > 2) { /* rare: more than two matches for one position, walk the list again */
				uint32_t k = 0;
				for (uint32_t e = heads[kmer & KEY_MASK]; e != DSB_HEMPTY; e = dsb_hstep(e, hnode, key_len)) {
					if (!dsb_hmatch(e, kmer, key_len))
						continue;
					uint32_t q_pos = dsb_hpos(e, key_len);
					if (!(q_pos >= q_bg && q_pos <= q_ed))
						continue;
					int ok = 0;
					uint32_t len = 0, qp = 0, tp = 0;
					if (isForward) {
						int back_len = dsb_MEM_search(q_str + q_pos - 1, c_t_str - 1, 0, 4);
						if (back_len < 4 || i == 4) {
							uint32_t max_search = q_ed - q_pos - 1;
							max_search = DSB_MIN(max_search, t_len - i - 1) + DSB_OVER_SEARCH;
							int forward_len = dsb_MEM_search(q_str + q_pos + DSB_S_A_KMER_L, c_t_str + DSB_S_A_KMER_L,
											 1, (int)max_search);
							int total_len = back_len + forward_len + 1;
							if (total_len >= 4) { len = total_len; qp = q_pos - back_len; tp = i - back_len + t_st; ok = 1; }
						}
					} else {
						int forward_len = dsb_MEM_search(q_str + q_pos + DSB_S_A_KMER_L, c_t_str + DSB_S_A_KMER_L, 1, 4);
						if (forward_len < 4 || i == 4) {
							uint32_t max_search = q_pos;
							max_search = DSB_MIN(max_search, (uint32_t)(c_t_str - t_str)) + DSB_OVER_SEARCH;
							int back_len = dsb_MEM_search(q_str + q_pos - 1, c_t_str - 1, 0, (int)max_search);
							int total_len = back_len + forward_len + 1;
							if (total_len >= 4) {
								len = total_len; qp = q_pos - back_len;
								tp = (uint32_t)(c_t_str - t_str) - back_len + t_st; ok = 1;
							}
						}
					}
					if (ok) {
						if (k >= 2) { dsb_spd_t *d = dsb_sms(w, dst + k); d->len = len; d->q_pos = qp; d->t_pos = tp; }
						k++;
					}
				}
			}
			w->n_sms += tot;
		}
		dsb_wsync();
	}
}

template <bool WAVE>
DSB_HD void dsb_sdp_match(dsb_read_ws *w, uint32_t q_bg, uint32_t q_ed, const uint8_t *q_str, const uint8_t *t_str,
			  uint32_t t_len, int key_len, int hslot, uint32_t t_st, int isForward)
{
	uint64_t t0 = DSB_T0();
	dsb_sdp_match_impl<WAVE>(w, q_bg, q_ed, q_str, t_str, t_len, key_len, hslot, t_st, isForward);
	DSB_T1(DSB_ST_T_MATCH, t0);
}

/* sdp_middle_M2, src/cly.c:2439-2525 */
template <bool WAVE>
DSB_HDN int dsb_sdp_middle(dsb_read_ws *w, int32_t c_a_i, const uint8_t *q_str, int hslot, int key_len)
{
	const dsb_dindex_t *ix = w->ix;
	int score = 10000;
	if (c_a_i < 0)
		return score - 10000;
	uint64_t t_offset = dsb_gld(ix->ref_seq_offset + w->anc[c_a_i].ref_ID);
	/* the anchor list is walked one pair ahead: the fields of the next pair's predecessor are
	 * loaded at the top of each window, so that their round trip overlaps the window's work
	 * instead of starting the next window (anchors are read-only in this phase) */
	struct mid_anchor { uint32_t ref_offset, index_in_read, mtch_len; int32_t pre; };
	auto ld_anchor = [&](int32_t i) -> mid_anchor {
		const dsb_anchor_t *a = w->anc + i;
		mid_anchor m;
		m.ref_offset = dsb_gld(&a->ref_offset);
		m.index_in_read = dsb_gld(&a->index_in_read);
		m.pre = dsb_gld(&a->pre);
		m.mtch_len = dsb_gld((const uint32_t *)&a->mtch_len) & 0xffffu; /* u16 mtch_len | i16 score */
		return m;
	};
	mid_anchor ca = ld_anchor(c_a_i), pa;
	pa.pre = -1;
	if (ca.pre >= 0)
		pa = ld_anchor(ca.pre);
	while (c_a_i >= 0) {
		const mid_anchor *c_a = &ca;
		int32_t pre_i = c_a->pre;
		if (pre_i >= 0) {
			const mid_anchor *pre_a = &pa;
			mid_anchor na;
			na.pre = -1;
			if (pa.pre >= 0)
				na = ld_anchor(pa.pre);
			int pre_mch = pre_a->mtch_len;
			int pre_refoffset = (int)(pre_a->ref_offset - 3);
			int total_ref_len = (int)(c_a->ref_offset - (uint32_t)(pre_refoffset + pre_mch) + 3);
			w->n_sms = 0;
			dsb_spd_t *p = dsb_push_sms(w);
			if (!p) return 0;
			p->score = score;
			p->q_pos = pre_a->index_in_read;
			p->t_pos = pre_a->ref_offset;
			p->len = pre_a->mtch_len - DSB_S_A_KMER_L + 1;
			if (total_ref_len > 12) {
				/* uint8_t ref[2000] (src/cly.c:2467), pattern-initialised per entry */
				uint8_t *ref = w->win + DSB_WIN_MID;
				if (total_ref_len >= 2000) { /* xassert(total_ref_len < 2000) exits the reference */
					w->overflow |= 32;
					return 0;
				}
				dsb_get_ref_win<WAVE>(w, ref, (uint64_t)(int64_t)(pre_refoffset + pre_mch) + t_offset, (uint32_t)total_ref_len);
				/* the reference re-initialises the whole ref[2000]; a forward scan of t_len bytes reads
				 * at most ref[t_len + 58] (MEM_search bound t_len - i - 1 + OVER_SEARCH past i + 9) */
				dsb_fill_pattern<WAVE>(w, ref, total_ref_len, DSB_MIN(total_ref_len + 64, 2000 + 64));
				dsb_sdp_match<WAVE>(w, pre_a->index_in_read + pre_mch - 8, c_a->index_in_read - 1, q_str, ref,
					      (uint32_t)total_ref_len, key_len, hslot, (uint32_t)(pre_refoffset + pre_mch), 1);
				if (w->overflow) return 0;
			}
			p = dsb_push_sms(w);
			if (!p) return 0;
			p->q_pos = c_a->index_in_read;
			p->t_pos = c_a->ref_offset;
			p->len = c_a->mtch_len - DSB_S_A_KMER_L + 1;
			uint64_t tdp0 = DSB_T0();
			if (WAVE && !DSB_SEQ(w, 4) && w->n_sms > 1 && w->n_sms <= DSB_WV) {
				/* register-resident DP: lane l holds node l (q, t, len, score); node cs's fields
				 * come by v_readlane, its predecessors are lanes < cs, its score goes back to
				 * lane cs — no memory traffic inside the node loop */
				uint32_t lane = dsb_lane(), n = w->n_sms;
				uint32_t nq = 0, nt = 0, nl = 0, nsc = 0;
				if (lane < n) {
					const dsb_spd_t *me = dsb_sms(w, lane);
					nq = me->q_pos; nt = me->t_pos; nl = me->len; nsc = me->score;
				}
				int pre_q_ed = (int)(nq + nl + DSB_S_A_KMER_L - 1);
				int pre_t_ed = (int)(nt + nl + DSB_S_A_KMER_L - 1);
				for (uint32_t cs = 1; cs < n; cs++) {
					uint32_t cq = (uint32_t)dsb_wshfl((int)nq, (int)cs), ct = (uint32_t)dsb_wshfl((int)nt, (int)cs);
					uint32_t cl = (uint32_t)dsb_wshfl((int)nl, (int)cs);
					int max_score = (int)cl;
					uint32_t max_q = cq + DSB_MAX_SMS_OVERLAP;
					uint32_t max_t = ct + DSB_MAX_SMS_OVERLAP;
					int cand = INT32_MIN;
					if (lane < cs && !((uint32_t)pre_q_ed > max_q) && !((uint32_t)pre_t_ed > max_t)) {
						int indel = (int)(nq - nt - (max_q - max_t));
						int ABS_indel = DSB_ABS(indel);
						if (ABS_indel <= 200) {
							cand = (int)(nsc + cl - (uint32_t)(ABS_indel >> 3));
							if ((uint32_t)pre_q_ed > cq || (uint32_t)pre_t_ed > ct)
								cand -= DSB_MAX(pre_q_ed - (int)cq, pre_t_ed - (int)ct);
						}
					}
					int best = dsb_wmax(cand);
					max_score = DSB_MAX(max_score, best);
					score = DSB_MAX(max_score, score);
					if (lane == cs)
						nsc = (uint32_t)max_score;
				}
				if (lane < n && lane > 0)
					dsb_sms(w, lane)->score = nsc;
				dsb_wsync();
			} else if (w->n_sms > 1) {
				for (uint32_t cs = 1; cs < w->n_sms; cs++) {
					dsb_spd_t *c_spd = dsb_sms(w, cs);
					int max_score = (int)c_spd->len;
					uint32_t max_q = c_spd->q_pos + DSB_MAX_SMS_OVERLAP;
					uint32_t max_t = c_spd->t_pos + DSB_MAX_SMS_OVERLAP;
					int best = INT32_MIN;
					const bool wv = WAVE && !DSB_SEQ(w, 4);
					for (int64_t pb = (int64_t)cs - 1; pb >= 0; pb -= (wv ? DSB_WV : 1)) {
						int64_t ps = pb - (wv ? (int64_t)dsb_lane() : 0);
						for (int64_t pe = (wv && ps >= 0) ? ps : 0; ps >= pe; ps--) { /* WAVE: one node per lane */
							dsb_spd_t *c_pre = dsb_sms(w, ps);
							int pre_q_ed = (int)(c_pre->q_pos + c_pre->len + DSB_S_A_KMER_L - 1);
							int pre_t_ed = (int)(c_pre->t_pos + c_pre->len + DSB_S_A_KMER_L - 1);
							if ((uint32_t)pre_q_ed > max_q) continue; /* int vs uint32 */
							if ((uint32_t)pre_t_ed > max_t) continue;
							int indel = (int)(c_pre->q_pos - c_pre->t_pos - (max_q - max_t));
							int ABS_indel = DSB_ABS(indel);
							if (ABS_indel > 200) continue;
							int new_score = (int)(c_pre->score + c_spd->len - (uint32_t)(ABS_indel >> 3));
							if ((uint32_t)pre_q_ed > c_spd->q_pos || (uint32_t)pre_t_ed > c_spd->t_pos) {
								int overlap_q = pre_q_ed - (int)c_spd->q_pos;
								int overlap_t = pre_t_ed - (int)c_spd->t_pos;
								new_score -= DSB_MAX(overlap_q, overlap_t);
							}
							best = DSB_MAX(best, new_score);
						}
						if (!wv)
							break;
					}
					if (wv)
						best = dsb_wmax(best);
					max_score = DSB_MAX(max_score, best);
					score = DSB_MAX(max_score, score);
					c_spd->score = (uint32_t)max_score;
				}
			}
			DSB_T1(DSB_ST_T_DPM, tdp0);
			ca = pa;
			pa = na;
		} else
			score += c_a->mtch_len - DSB_S_A_KMER_L + 1;
		c_a_i = pre_i;
	}
	return score - 10000;
}

/* combine_chain, src/cly.c:1758-1803: the first entry of the key's list (in list order) whose
 * chain continues chain_ID's at this diagonal is merged into it */
DSB_HD int dsb_comb_ok(const dsb_chain_t *c_h, const dsb_chain_t *c, uint16_t e, int chain_ID, int dis, int isleft,
			int c_q_pos)
{
	int seed_ID = e & 0x7fff;
	int s_or_e = e >> 15;
	int dis_con = isleft ? (int)(c->t_ed - c->q_ed) : (int)(c->t_st - c->q_st);
	int q_pos_con = (!isleft) ? (int)c->q_st : (int)(c->q_ed - DSB_S_A_KMER_L);
	return dis == dis_con && c_h != c && isleft != s_or_e && DSB_ABS_U(c_q_pos, q_pos_con) < 8 &&
	       c_h->ref_ID == c->ref_ID && c_h->direction == c->direction && c->sum_score != 0 && seed_ID - 1 > chain_ID;
}

DSB_HD void dsb_comb_merge(dsb_chain_t *c_h, dsb_chain_t *c)
{
	c_h->sum_score += c->sum_score;
	c_h->anchor_number += c->anchor_number;
	c_h->indel += c->indel;
	c_h->q_st = DSB_MIN(c_h->q_st, c->q_st);
	c_h->t_st = DSB_MIN(c_h->t_st, c->t_st);
	c_h->q_ed = DSB_MAX(c_h->q_ed, c->q_ed);
	c_h->t_ed = DSB_MAX(c_h->t_ed, c->t_ed);
	c->sum_score = 0;
	c->t_st = c->t_ed = c->q_st = c->q_ed = 0;
}

/* the chain being scored: its private copy while scored speculatively (spec_ch), else w->hit */
DSB_HD dsb_chain_t *dsb_ch(dsb_read_ws *w, int chain_ID) { return w->spec_ch ? w->spec_ch : w->hit + chain_ID; }
DSB_HD int dsb_spec_merged(const dsb_read_ws *w, uint32_t c) { return w->spec_bits && ((w->spec_bits[c >> 6] >> (c & 63)) & 1); }

/* a speculative merge: c_h takes c's counts and extent as dsb_comb_merge does, c stays as it is in
 * w->hit (other chains' speculative runs read it) and is only marked merged */
DSB_HD void dsb_comb_merge_spec(dsb_read_ws *w, dsb_chain_t *c_h, uint32_t ci)
{
	const dsb_chain_t *c = w->hit + ci;
	c_h->sum_score += c->sum_score;
	c_h->anchor_number += c->anchor_number;
	c_h->indel += c->indel;
	c_h->q_st = DSB_MIN(c_h->q_st, c->q_st);
	c_h->t_st = DSB_MIN(c_h->t_st, c->t_st);
	c_h->q_ed = DSB_MAX(c_h->q_ed, c->q_ed);
	c_h->t_ed = DSB_MAX(c_h->t_ed, c->t_ed);
	w->spec_bits[ci >> 6] |= 1ull << (ci & 63);
}

/* combine_chain's candidates for one side (right or left) of one chain's scoring, in the wave:
 * the later chains (seed_ID - 1 > chain_ID) on c_h's reference and strand that are still live,
 * lane k holding the k-th in chain order with the diagonal and read position its list entry is
 * compared on.  A later chain's coordinates are those it had when the lists were built until it
 * is merged (then zeroed, and dead here too) or scored itself, so the entries the reference's
 * walk would accept are exactly the cached ones that match, and the first in list order (insertion
 * order: by chain) is the lowest lane.  Built at the side's first call; more than a wave of
 * candidates (n < 0) takes the list scan. */
typedef struct {
	int built, n;
	int32_t dis, qpos, sid;
} dsb_comb_cache;

template <bool WAVE>
DSB_HD int dsb_combine_chain_impl(dsb_read_ws *w, dsb_comb_cache *cc, int chain_ID, int dis, int isleft, int c_q_pos,
				  int32_t *combined)
{
	uint16_t key = (uint16_t)(dis & 0xff);
	dsb_chain_t *c_h = dsb_ch(w, chain_ID);
	if (WAVE && !DSB_SEQ(w, 4) && cc) {
		const uint32_t lane = dsb_lane();
		if (!cc->built) {
			cc->built = 1;
			cc->n = 0;
			cc->dis = cc->qpos = cc->sid = 0;
			const uint32_t ref = c_h->ref_ID, dir = c_h->direction;
			for (uint32_t h0 = (uint32_t)chain_ID + 1; h0 < w->n_hit; h0 += DSB_WV) {
				uint32_t h = h0 + lane;
				int ok = 0;
				int32_t d = 0, q = 0;
				if (h < w->n_hit) {
					const dsb_chain_t *c = w->hit + h;
					/* live: not zeroed, and not merged by this speculative run (k_heavy_spec leaves
					 * its merges in w->hit and only marks them, so the side built second would
					 * otherwise see a chain the first side already took) */
					ok = c->ref_ID == ref && c->direction == dir && c->sum_score != 0 && !dsb_spec_merged(w, h);
					d = isleft ? (int)(c->t_ed - c->q_ed) : (int)(c->t_st - c->q_st);
					q = isleft ? (int)(c->q_ed - DSB_S_A_KMER_L) : (int)c->q_st;
				}
				uint64_t bm = dsb_wballot(ok);
				int cnt = __builtin_popcountll(bm);
				if (cc->n + cnt > DSB_WV) {
					cc->n = -1;
					break;
				}
				if (cnt) {
					int k = (int)lane - cc->n; /* this lane's place among the new candidates */
					int mine = k >= 0 && k < cnt;
					int src = mine ? (int)dsb_select64(bm, (uint32_t)k) : (int)lane;
					int d2 = dsb_wshfl_any(d, src), q2 = dsb_wshfl_any(q, src), s2 = dsb_wshfl_any((int)h + 1, src);
					if (mine) {
						cc->dis = d2;
						cc->qpos = q2;
						cc->sid = s2;
					}
					cc->n += cnt;
				}
			}
		}
		if (cc->n >= 0) {
			int ok = cc->sid != 0 && cc->dis == dis && DSB_ABS_U(c_q_pos, cc->qpos) < 8;
			uint64_t bm = dsb_wballot(ok);
			if (!bm)
				return 0;
			int seed_ID = dsb_wshfl(cc->sid, (int)__builtin_ctzll(bm));
			dsb_wsync();
			if (lane == 0) {
				if (w->spec_bits)
					dsb_comb_merge_spec(w, c_h, (uint32_t)seed_ID - 1);
				else
					dsb_comb_merge(c_h, w->hit + seed_ID - 1);
			}
			dsb_wsync();
			if (cc->sid == seed_ID)
				cc->sid = 0; /* merged: zeroed, never a candidate again */
			*combined = seed_ID - 1;
			return 1;
		}
	}
	if (WAVE && !DSB_SEQ(w, 4)) {
		/* the list as an array: one entry per lane, the lowest matching lane is the first match
		 * in list order */
		const dsb_chain_t hd = *c_h;
		uint32_t b = w->sc_off[key], e = w->sc_off[key + 1];
		for (uint32_t k0 = b; k0 < e; k0 += DSB_WV) {
			uint32_t k = k0 + dsb_lane();
			uint16_t ent = 0;
			int ok = 0;
			if (k < e) {
				ent = w->sc_flat[k];
				const dsb_chain_t *c = w->hit + (ent & 0x7fff) - 1;
				ok = dsb_comb_ok(&hd, c, ent, chain_ID, dis, isleft, c_q_pos) && c != c_h &&
				     !dsb_spec_merged(w, (uint32_t)(ent & 0x7fff) - 1);
			}
			uint64_t bm = dsb_wballot(ok);
			if (bm) {
				int first = (int)__builtin_ctzll(bm);
				int seed_ID = dsb_wshfl((int)ent, first) & 0x7fff;
				dsb_wsync();
				if (dsb_lane() == 0) {
					if (w->spec_bits)
						dsb_comb_merge_spec(w, c_h, (uint32_t)seed_ID - 1);
					else
						dsb_comb_merge(c_h, w->hit + seed_ID - 1);
				}
				dsb_wsync();
				*combined = seed_ID - 1;
				return 1;
			}
		}
		return 0;
	}
	dsb_sch_t *sc = w->sch;
	while (sc[key].next != 0) {
		uint16_t ent = sc[key].seed_ID_s_or_e;
		dsb_chain_t *c = w->hit + (ent & 0x7fff) - 1;
		if (dsb_comb_ok(c_h, c, ent, chain_ID, dis, isleft, c_q_pos)) {
			dsb_comb_merge(c_h, c);
			*combined = (ent & 0x7fff) - 1;
			return 1;
		}
		key = sc[key].next;
	}
	return 0;
}

template <bool WAVE>
DSB_HD int dsb_combine_chain(dsb_read_ws *w, dsb_comb_cache *cc, int chain_ID, int dis, int isleft, int c_q_pos,
			     int32_t *combined)
{
	uint64_t t0 = DSB_T0();
	int r = dsb_combine_chain_impl<WAVE>(w, cc, chain_ID, dis, isleft, c_q_pos, combined);
	DSB_T1(DSB_ST_T_COMB, t0);
	return r;
}

/* sdp_right_M2, src/cly.c:2527-2672 */
template <bool WAVE>
DSB_HDN int dsb_sdp_right(dsb_read_ws *w, const uint8_t *q_str, int hslot, int key_len, int chain_ID,
			   uint32_t l_read, int score_ori)
{
	const dsb_dindex_t *ix = w->ix;
	score_ori += 10000;
	int total_max_score = score_ori;
	int max_sms_id = 0;
	dsb_chain_t *c_h = dsb_ch(w, chain_ID);
	int32_t combined;
	w->n_sms = 0;
	uint8_t *ref = w->win + DSB_WIN_RL; /* uint8_t ref[1000] (src/cly.c:2537) */
	dsb_comb_cache cc = {0, 0, 0, 0, 0};
	dsb_fill_pattern<WAVE>(w, ref, -64, 1000 + 64); /* ref[-1] is read by sdp_left's back extension */
	dsb_spd_t *p = dsb_push_sms(w);
	if (!p) return 0;
	p->score = score_ori;
	p->q_pos = c_h->q_ed;
	p->t_pos = c_h->t_ed;
	p->len = 1 - DSB_S_A_KMER_L;
	uint32_t current_sms = 1;
	uint64_t t_offset_global = dsb_gld(ix->ref_seq_offset + c_h->ref_ID);
	uint64_t t_length = dsb_gld(ix->ref_seq_l + c_h->ref_ID);
	uint32_t c_t_offset = c_h->t_ed - 3;
	int last_search = 0;
	while (1) {
		if (w->n_sms == current_sms) {
			uint32_t next_step = (uint32_t)(t_length - c_t_offset);
			if (next_step < DSB_MIN_SCORE_MEM)
				break;
			uint32_t max_search_ref;
			if (l_read - c_h->q_ed < 600) {
				if (last_search)
					break;
				last_search = 1;
				max_search_ref = l_read - c_h->q_ed + 60;
			} else
				max_search_ref = (uint32_t)(t_length - c_t_offset);
			max_search_ref = DSB_MIN(600u, max_search_ref);
			dsb_get_ref_win<WAVE>(w, ref, c_t_offset + t_offset_global, max_search_ref + DSB_OVER_SEARCH);
			int search_q_ed = (int)dsb_sms(w, max_sms_id)->q_pos + 1000;
			search_q_ed = DSB_MIN(search_q_ed, l_read);                /* int vs uint32: unsigned */
			int search_q_st = DSB_MAX(search_q_ed - 2000, c_h->q_st - 8); /* idem (H11) */
			dsb_sdp_match<WAVE>(w, (uint32_t)search_q_st, (uint32_t)search_q_ed, q_str, ref, max_search_ref, key_len, hslot,
				      c_t_offset, 1);
			if (w->overflow) return 0;
			c_t_offset += max_search_ref - DSB_S_A_KMER_L - 3;
			if (w->n_sms == current_sms)
				break;
			if (dsb_sms(w, current_sms)->t_pos > dsb_sms(w, max_sms_id)->t_pos + 1000)
				break;
		}
		dsb_spd_t *c_sms = dsb_sms(w, current_sms++);
		if (w->stats && dsb_lane() == 0) w->stats[DSB_ST_NSMS]++;
		/* WAVE: the first batch of predecessors (one per lane) is loaded together with the node
		 * itself, one round trip for both */
		dsb_spd_t pre0 = {0, 0, 0, 0};
		const int64_t pfirst = (int64_t)current_sms - 2;
		if (WAVE && !DSB_SEQ(w, 4) && pfirst - (int64_t)dsb_lane() >= 0)
			pre0 = *dsb_sms(w, pfirst - (int64_t)dsb_lane());
		int max_score = (int)c_sms->len;
		uint32_t max_pre_q = c_sms->q_pos + DSB_MAX_SMS_OVERLAP;
		uint32_t max_pre_t = c_sms->t_pos + DSB_MAX_SMS_OVERLAP;
		uint64_t tdp0 = DSB_T0();
		if (!WAVE || DSB_SEQ(w, 4)) {
			for (int64_t ps = (int64_t)current_sms - 2; ps >= 0; ps--) {
				dsb_spd_t *c_pre = dsb_sms(w, ps);
				int pre_q_ed = (int)(c_pre->q_pos + c_pre->len + DSB_S_A_KMER_L - 1);
				int pre_t_ed = (int)(c_pre->t_pos + c_pre->len + DSB_S_A_KMER_L - 1);
				if ((uint32_t)pre_q_ed > max_pre_q) continue; /* int vs uint32 */
				if ((uint32_t)pre_t_ed > max_pre_t) continue;
				if (c_pre->t_pos + 600 < max_pre_t) break;
				int indel = (int)(c_pre->q_pos - c_pre->t_pos - (max_pre_q - max_pre_t));
				int ABS_indel = DSB_ABS(indel);
				if (ABS_indel > 200) continue;
				int new_score = (int)(c_pre->score + c_sms->len - (uint32_t)(ABS_indel >> 3));
				if ((uint32_t)pre_q_ed > c_sms->q_pos || (uint32_t)pre_t_ed > c_sms->t_pos) {
					int overlap_q = pre_q_ed - (int)c_sms->q_pos;
					int overlap_t = pre_t_ed - (int)c_sms->t_pos;
					new_score -= DSB_MAX(overlap_q, overlap_t);
				}
				max_score = DSB_MAX(max_score, new_score);
			}
		} else { /* lanes scan predecessors downwards; the first `break` node ends the scan */
			int best = INT32_MIN;
			uint32_t lane = dsb_lane();
			for (int64_t pb = (int64_t)current_sms - 2; pb >= 0; pb -= DSB_WV) {
				int64_t ps = pb - (int64_t)lane;
				int cand = INT32_MIN, brk = 0;
				if (ps >= 0) {
					const dsb_spd_t cp = (pb == pfirst) ? pre0 : *dsb_sms(w, ps);
					const dsb_spd_t *c_pre = &cp;
					int pre_q_ed = (int)(c_pre->q_pos + c_pre->len + DSB_S_A_KMER_L - 1);
					int pre_t_ed = (int)(c_pre->t_pos + c_pre->len + DSB_S_A_KMER_L - 1);
					if (!((uint32_t)pre_q_ed > max_pre_q) && !((uint32_t)pre_t_ed > max_pre_t)) {
						if (c_pre->t_pos + 600 < max_pre_t)
							brk = 1;
						else {
							int indel = (int)(c_pre->q_pos - c_pre->t_pos - (max_pre_q - max_pre_t));
							int ABS_indel = DSB_ABS(indel);
							if (ABS_indel <= 200) {
								cand = (int)(c_pre->score + c_sms->len - (uint32_t)(ABS_indel >> 3));
								if ((uint32_t)pre_q_ed > c_sms->q_pos || (uint32_t)pre_t_ed > c_sms->t_pos) {
									int overlap_q = pre_q_ed - (int)c_sms->q_pos;
									int overlap_t = pre_t_ed - (int)c_sms->t_pos;
									cand -= DSB_MAX(overlap_q, overlap_t);
								}
							}
						}
					}
				}
				uint64_t bm = dsb_wballot(brk);
				if (bm) {
					uint32_t first = (uint32_t)__builtin_ctzll(bm);
					if (lane >= first)
						cand = INT32_MIN;
				}
				best = DSB_MAX(best, cand);
				if (bm)
					break;
			}
			best = dsb_wmax(best);
			max_score = DSB_MAX(max_score, best);
		}
		DSB_T1(DSB_ST_T_DPS, tdp0);
		c_sms->score = (uint32_t)max_score;
		if (c_sms->len >= 8 &&
		    dsb_combine_chain<WAVE>(w, &cc, chain_ID, (int)(c_sms->t_pos - c_sms->q_pos), 0, (int)c_sms->q_pos, &combined)) {
			total_max_score = DSB_MAX(score_ori, max_score) - (int)c_sms->len +
					  dsb_sdp_middle<WAVE>(w, w->hit[combined].cur, q_str, hslot, key_len);
			if (w->overflow) return 0;
			score_ori = total_max_score;
			max_sms_id = 0;
			w->n_sms = 0;
			p = dsb_push_sms(w);
			if (!p) return 0;
			p->score = total_max_score;
			p->q_pos = c_h->q_ed;
			p->t_pos = c_h->t_ed;
			p->len = (uint32_t)(-DSB_S_A_KMER_L);
			current_sms = 1;
			c_t_offset = c_h->t_ed;
			continue;
		}
		if (total_max_score < max_score) {
			total_max_score = max_score;
			max_sms_id = current_sms - 1;
		}
		if (c_sms->t_pos > dsb_sms(w, max_sms_id)->t_pos + 1000)
			break;
	}
	c_h->q_ed = dsb_sms(w, max_sms_id)->q_pos + dsb_sms(w, max_sms_id)->len + DSB_S_A_KMER_L;
	c_h->t_ed = dsb_sms(w, max_sms_id)->t_pos + dsb_sms(w, max_sms_id)->len + DSB_S_A_KMER_L;
	return total_max_score - 10000;
}

/* sdp_left_M2, src/cly.c:2674-2814 (the first node's len is not written: H6) */
template <bool WAVE>
DSB_HDN int dsb_sdp_left(dsb_read_ws *w, const uint8_t *q_str, int hslot, int key_len, int chain_ID,
			  uint32_t l_read, int score_ori)
{
	const dsb_dindex_t *ix = w->ix;
	(void)l_read;
	score_ori += 10000;
	int total_max_score = score_ori;
	int max_sms_id = 0;
	dsb_chain_t *c_h = dsb_ch(w, chain_ID);
	int32_t combined;
	w->n_sms = 0;
	uint8_t *ref = w->win + DSB_WIN_RL; /* uint8_t ref[1000] (src/cly.c:2683) */
	dsb_comb_cache cc = {0, 0, 0, 0, 0};
	dsb_fill_pattern<WAVE>(w, ref, -64, 1000 + 64); /* ref[-1] is read by sdp_left's back extension */
	dsb_spd_t *p = dsb_push_sms(w);
	if (!p) return 0;
	p->score = score_ori;
	p->q_pos = c_h->q_st;
	p->t_pos = c_h->t_st;
	uint32_t current_sms = 1;
	uint64_t t_offset_global = dsb_gld(ix->ref_seq_offset + c_h->ref_ID);
	uint32_t c_t_offset = c_h->t_st + 3;
	int last_search = 0;
	while (1) {
		if (w->n_sms == current_sms) {
			uint32_t next_step = c_t_offset;
			if (next_step < DSB_MIN_SCORE_MEM)
				break;
			uint32_t max_search_ref;
			if (c_h->q_st < 600) {
				if (last_search)
					break;
				last_search = 1;
				max_search_ref = c_h->q_st + 60;
			} else
				max_search_ref = c_t_offset;
			max_search_ref = DSB_MIN(600u, max_search_ref);
			if (t_offset_global == 0 && c_t_offset < DSB_OVER_SEARCH + max_search_ref)
				dsb_get_ref_win<WAVE>(w, ref, c_t_offset + t_offset_global - max_search_ref, max_search_ref);
			else
				dsb_get_ref_win<WAVE>(w, ref, c_t_offset + t_offset_global - max_search_ref - DSB_OVER_SEARCH,
						      max_search_ref + DSB_OVER_SEARCH);
			int search_q_st = (int)dsb_sms(w, max_sms_id)->q_pos - 1000;
			search_q_st = DSB_MAX(search_q_st, 0);
			int search_q_ed = DSB_MIN(search_q_st + 2000, c_h->q_st - 1); /* int vs uint32: unsigned */
			dsb_sdp_match<WAVE>(w, (uint32_t)search_q_st, (uint32_t)search_q_ed, q_str, ref + DSB_OVER_SEARCH, max_search_ref,
				      key_len, hslot, c_t_offset - max_search_ref, 0);
			if (w->overflow) return 0;
			c_t_offset = c_t_offset - max_search_ref + DSB_S_A_KMER_L + 3;
			if (w->n_sms == current_sms)
				break;
			if (dsb_sms(w, current_sms)->t_pos + 1000 < dsb_sms(w, max_sms_id)->t_pos)
				break;
		}
		dsb_spd_t *c_sms = dsb_sms(w, current_sms++);
		if (w->stats && dsb_lane() == 0) w->stats[DSB_ST_NSMS]++;
		/* WAVE: the first batch of predecessors (one per lane) is loaded together with the node
		 * itself, one round trip for both */
		dsb_spd_t pre0 = {0, 0, 0, 0};
		const int64_t pfirst = (int64_t)current_sms - 2;
		if (WAVE && !DSB_SEQ(w, 4) && pfirst - (int64_t)dsb_lane() >= 0)
			pre0 = *dsb_sms(w, pfirst - (int64_t)dsb_lane());
		int max_score = (int)c_sms->len;
		uint32_t min_pre_q = c_sms->q_pos + c_sms->len - DSB_MAX_SMS_OVERLAP + DSB_S_A_KMER_L - 1;
		uint32_t min_pre_t = c_sms->t_pos + c_sms->len - DSB_MAX_SMS_OVERLAP + DSB_S_A_KMER_L - 1;
		uint64_t tdp0 = DSB_T0();
		if (!WAVE || DSB_SEQ(w, 4)) {
			for (int64_t ps = (int64_t)current_sms - 2; ps >= 0; ps--) {
				dsb_spd_t *c_pre = dsb_sms(w, ps);
				if (c_pre->q_pos < min_pre_q) continue;
				if (c_pre->t_pos < min_pre_t) continue;
				if (min_pre_t + 600 < c_pre->t_pos) break;
				int indel = (int)(c_pre->q_pos - c_pre->t_pos - (min_pre_q - min_pre_t));
				int ABS_indel = DSB_ABS(indel);
				if (ABS_indel > 200) continue;
				int new_score = (int)(c_pre->score + c_sms->len - (uint32_t)(ABS_indel >> 3));
				if (min_pre_q + DSB_MAX_SMS_OVERLAP > c_pre->q_pos || min_pre_t + DSB_MAX_SMS_OVERLAP > c_pre->t_pos) {
					int overlap_q = (int)(min_pre_q + DSB_MAX_SMS_OVERLAP - c_pre->q_pos);
					int overlap_t = (int)(min_pre_t + DSB_MAX_SMS_OVERLAP - c_pre->t_pos);
					new_score -= DSB_MAX(overlap_q, overlap_t);
				}
				max_score = DSB_MAX(max_score, new_score);
			}
		} else {
			int best = INT32_MIN;
			uint32_t lane = dsb_lane();
			for (int64_t pb = (int64_t)current_sms - 2; pb >= 0; pb -= DSB_WV) {
				int64_t ps = pb - (int64_t)lane;
				int cand = INT32_MIN, brk = 0;
				if (ps >= 0) {
					const dsb_spd_t cp = (pb == pfirst) ? pre0 : *dsb_sms(w, ps);
					const dsb_spd_t *c_pre = &cp;
					if (!(c_pre->q_pos < min_pre_q) && !(c_pre->t_pos < min_pre_t)) {
						if (min_pre_t + 600 < c_pre->t_pos)
							brk = 1;
						else {
							int indel = (int)(c_pre->q_pos - c_pre->t_pos - (min_pre_q - min_pre_t));
							int ABS_indel = DSB_ABS(indel);
							if (ABS_indel <= 200) {
								cand = (int)(c_pre->score + c_sms->len - (uint32_t)(ABS_indel >> 3));
								if (min_pre_q + DSB_MAX_SMS_OVERLAP > c_pre->q_pos ||
								    min_pre_t + DSB_MAX_SMS_OVERLAP > c_pre->t_pos) {
									int overlap_q = (int)(min_pre_q + DSB_MAX_SMS_OVERLAP - c_pre->q_pos);
									int overlap_t = (int)(min_pre_t + DSB_MAX_SMS_OVERLAP - c_pre->t_pos);
									cand -= DSB_MAX(overlap_q, overlap_t);
								}
							}
						}
					}
				}
				uint64_t bm = dsb_wballot(brk);
				if (bm) {
					uint32_t first = (uint32_t)__builtin_ctzll(bm);
					if (lane >= first)
						cand = INT32_MIN;
				}
				best = DSB_MAX(best, cand);
				if (bm)
					break;
			}
			best = dsb_wmax(best);
			max_score = DSB_MAX(max_score, best);
		}
		DSB_T1(DSB_ST_T_DPS, tdp0);
		c_sms->score = (uint32_t)max_score;
		if (c_sms->len >= 8 && dsb_combine_chain<WAVE>(w, &cc, chain_ID, (int)(c_sms->t_pos - c_sms->q_pos), 1,
							 (int)(c_sms->q_pos + c_sms->len), &combined)) {
			total_max_score = DSB_MAX(score_ori, max_score) - (int)c_sms->len +
					  dsb_sdp_middle<WAVE>(w, w->hit[combined].cur, q_str, hslot, key_len);
			if (w->overflow) return 0;
			score_ori = total_max_score;
			max_sms_id = 0;
			w->n_sms = 0;
			p = dsb_push_sms(w);
			if (!p) return 0;
			p->score = total_max_score;
			p->q_pos = c_h->q_st;
			p->t_pos = c_h->t_st;
			current_sms = 1;
			c_t_offset = c_h->t_st;
			continue;
		}
		if (total_max_score < max_score) {
			total_max_score = max_score;
			max_sms_id = current_sms - 1;
		}
		if (c_sms->t_pos + 1000 < dsb_sms(w, max_sms_id)->t_pos)
			break;
	}
	c_h->q_st = dsb_sms(w, max_sms_id)->q_pos;
	c_h->t_st = dsb_sms(w, max_sms_id)->t_pos;
	return total_max_score - 10000;
}

/* one iteration of get_score_M2's loop (src/cly.c:2832-2842): chain i's middle, right and left
 * scores; 0 when the read overflowed */
template <bool WAVE>
DSB_HD int dsb_score_chain(dsb_read_ws *w, uint32_t i, uint32_t l_read, int key_len)
{
	dsb_chain_t *ch = dsb_ch(w, (int)i);
	const dsb_sdir_t *csd = (w->sd[0].direction == ch->direction) ? &w->sd[0] : &w->sd[1];
	int hslot = (ch->direction == DSB_FORWARD) ? 0 : 1;
	const uint8_t *q_str = w->bin + (csd->strand ? w->L : 0);
	int score = dsb_sdp_middle<WAVE>(w, ch->cur, q_str, hslot, key_len);
	if (w->overflow) return 0;
	score = dsb_sdp_right<WAVE>(w, q_str, hslot, key_len, (int)i, l_read, score);
	if (w->overflow) return 0;
	score = dsb_sdp_left<WAVE>(w, q_str, hslot, key_len, (int)i, l_read, score);
	if (w->overflow) return 0;
	ch->sum_score = (uint32_t)score;
	return 1;
}

/* get_score_M2, src/cly.c:2816-2844 */
template <bool WAVE>
DSB_HDN void dsb_get_score(dsb_read_ws *w, uint32_t l_read)
{
	uint64_t tb0 = DSB_T0();
#ifdef DSB_EXP_BUILD2 /* timing experiment only: the build's marginal cost (the second build rewrites the same tables) */
	dsb_build_hash_table<WAVE>(w, (int)l_read);
#endif
	int key_len = dsb_build_hash_table<WAVE>(w, (int)l_read);
	DSB_T1(DSB_ST_T_BUILD, tb0);
	for (uint32_t i = 0; i < w->n_hit; i++) {
		if (w->hit[i].sum_score == 0)
			continue;
		if (!dsb_score_chain<WAVE>(w, i, l_read, key_len))
			return;
	}
}

/* chain_cmp_by_pos, src/cly.c:2848-2865.  Written as sign differences: the early-return form
 * of the reference is mis-scheduled by hipcc (ROCm 7.2, gfx950) inside the merge loop of
 * dsb_msort (permutation with duplicates; tests/test_gpu_selftest.py pins it). */
DSB_HD int dsb_chain_cmp_by_pos(const dsb_chain_t *a, const dsb_chain_t *b)
{
	int c = (a->ref_ID > b->ref_ID) - (a->ref_ID < b->ref_ID);
	if (c)
		return c;
	c = (a->t_st > b->t_st) - (a->t_st < b->t_st);
	if (c)
		return c;
	return (a->sum_score < b->sum_score) - (a->sum_score > b->sum_score);
}

/* chain_cmp_by_MEM_score, src/cly.c:53-63 (ties return a->sum_score % 2: H9) */
DSB_HD int dsb_chain_cmp_by_MEM_score(const dsb_chain_t *a, const dsb_chain_t *b)
{
	int score_a = (int)(a->sum_score << 5);
	int score_b = (int)(b->sum_score << 5);
	if (score_a < score_b) return 1;
	if (score_a > score_b) return -1;
	return (int)(a->sum_score % 2);
}

/* delete_small_score_rst, src/cly.c:2878-2952 — part A (up to the max_read_l update), in three
 * steps: the chains kept and their seed_con_hash (dsb_dela_prep; 0: no chains), the scores
 * (dsb_get_score, or the heavy reads' speculative scoring, dsb_kern.h), the merges (dsb_dela_post) */
DSB_HD int dsb_dela_prep(dsb_read_ws *w)
{
	w->reached_update = 0;
	if (w->n_hit == 0)
		return 0;
	if (w->n_hit > 200) {
		uint32_t rst_num = 200;
		for (; rst_num < w->n_hit && w->hit[rst_num].sum_score > 50; rst_num++);
		w->n_hit = rst_num;
	}
	w->n_hit = DSB_MIN(400u, w->n_hit);
	dsb_sc_hash_idx(w);
	return 1;
}

DSB_HDN void dsb_dela_post(dsb_read_ws *w);

template <bool WAVE>
DSB_HDN void dsb_delete_small_A(dsb_read_ws *w)
{
	if (!dsb_dela_prep(w))
		return;
	uint64_t ta0 = DSB_T0();
	dsb_get_score<WAVE>(w, w->L);
	DSB_T1(DSB_ST_T_ALL, ta0);
	if (w->overflow)
		return;
	dsb_dela_post(w);
}

DSB_HDN void dsb_dela_post(dsb_read_ws *w)
{
	uint32_t n = w->n_hit;
	if (n > 1)
		dsb_sort_chains(w, [](const dsb_chain_t *a, const dsb_chain_t *b) -> int { return dsb_chain_cmp_by_pos(a, b); });
	dsb_chain_t *H = w->hit;
	for (uint32_t ci = 0; n > 0 && ci < n - 1; ci++) {
		dsb_chain_t *c_c = H + ci;
		if (c_c->sum_score == 0)
			continue;
		for (uint32_t ni = ci + 1; ni < n; ni++) {
			dsb_chain_t *next_c = H + ni;
			if (c_c->ref_ID == next_c->ref_ID) {
				if (c_c->direction != next_c->direction)
					continue;
				if (next_c->sum_score == 0)
					continue;
				if (next_c->t_st < c_c->t_st + 5 && next_c->q_st < c_c->q_st + 5 &&
				    next_c->sum_score < c_c->sum_score + 5) {
					next_c->sum_score = 0;
					next_c->q_ed = next_c->q_st;
					next_c->t_ed = next_c->t_st;
					continue;
				}
				int dis_t = (int)(next_c->t_st - c_c->t_ed);
				int dis_q = (int)(next_c->q_st - c_c->q_ed);
				int dis_t_q = DSB_ABS(dis_t - dis_q);
				if ((dis_t > -20 && dis_t < 1000 && dis_q > -20 && dis_q < 1000) && dis_t_q < 200) {
					c_c->t_ed = DSB_MAX(c_c->t_ed, next_c->t_ed);
					c_c->q_ed = DSB_MAX(c_c->q_ed, next_c->q_ed);
					c_c->sum_score += next_c->sum_score;
					next_c->sum_score = 0;
					next_c->q_ed = next_c->q_st;
					next_c->t_ed = next_c->t_st;
				}
			} else
				break;
		}
	}
	w->reached_update = 1;
}

/* delete_small_score_rst part B (src/cly.c:2953-2987) + detect_primary (src/cly.c:2990-3053);
 * max_read_l is the carried pool value already including this read (H2). */
DSB_HDN void dsb_delete_small_B(dsb_read_ws *w, int max_read_l)
{
	if (!w->reached_update)
		return;
	const dsb_dindex_t *ix = w->ix;
	uint32_t l_read = w->L;
	dsb_chain_t *H = w->hit;
	uint32_t n = w->n_hit;
	if (max_read_l < 510) {
		for (uint32_t k = 0; k < n; k++) {
			int score = (int)(H[k].sum_score + ((H[k].q_ed - H[k].q_st) >> 5));
			if (score < 26) H[k].sum_score = 0;
		}
	} else if (l_read < 310) {
		for (uint32_t k = 0; k < n; k++) {
			int score = (int)(H[k].sum_score + ((H[k].q_ed - H[k].q_st) >> 5));
			if (score < 30) H[k].sum_score = 0;
		}
	} else {
		for (uint32_t k = 0; k < n; k++) {
			int score = (int)(H[k].sum_score + ((H[k].q_ed - H[k].q_st) >> 5));
			if (score < ix->filter_min_score_LV3 &&
			    ((H[k].q_ed - H[k].q_st) < (uint32_t)ix->filter_min_length || score < ix->filter_min_score))
				H[k].sum_score = 0;
		}
	}
	if (n > 1)
		dsb_sort_chains(w, [](const dsb_chain_t *a, const dsb_chain_t *b) -> int { return dsb_chain_cmp_by_MEM_score(a, b); });
	uint32_t k = 0;
	for (; k < n; k++)
		if (H[k].sum_score == 0)
			break;
	w->n_hit = k;
}

/* detect_primary, src/cly.c:2990-3053 */
DSB_HDN void dsb_detect_primary(dsb_read_ws *w, uint32_t read_len, int *primary_v, uint8_t *primary_v_idx)
{
	dsb_chain_t *hit = w->hit;
	uint32_t n_hit = w->n_hit;
	if (n_hit == 0)
		return;
	int n_primary_v = 1;
	hit->pri_index = primary_v_idx[0] = 0;
	primary_v[0] = 0;
	hit->primary = 1; /* PRIMARY */
	for (uint32_t k = 0; k < n_hit; k++)
		if (hit[k].q_st > 4294960000u)
			hit[k].q_st = 0;
	for (uint32_t ci = 1; ci < n_hit; ci++) {
		dsb_chain_t *c_hit = hit + ci;
		int overlap = 0;
		for (int i = 0; i < n_primary_v; i++) {
			int primary_st, primary_ed;
			if (hit[primary_v[i]].direction == c_hit->direction) {
				primary_st = (int)hit[primary_v[i]].q_st;
				primary_ed = (int)hit[primary_v[i]].q_ed;
			} else {
				primary_st = (int)(read_len - hit[primary_v[i]].q_ed);
				primary_ed = (int)(read_len - hit[primary_v[i]].q_st);
			}
			/* MAX/MIN on uint32 vs int: compared as unsigned */
			uint32_t overlap_st = DSB_MAX(c_hit->q_st, (uint32_t)primary_st);
			uint32_t overlap_ed = DSB_MIN(c_hit->q_ed, (uint32_t)primary_ed);
			if ((overlap_st < overlap_ed) && (((overlap_ed - overlap_st) << 1) >= (c_hit->q_ed - c_hit->q_st)))
				overlap = 1;
			if (overlap) {
				c_hit->primary = 2; /* SECONDARY */
				c_hit->pri_index = ++primary_v_idx[i];
				int max_gap = DSB_MAX((int)(hit[primary_v[i]].sum_score >> 6), 5);
				if (c_hit->sum_score + max_gap > hit[primary_v[i]].sum_score) /* uint32 + int: unsigned */
					c_hit->pri_index = 1;
				if (primary_v_idx[i] == 255)
					primary_v_idx[i] = 254;
				break;
			}
		}
		if (!overlap) {
			c_hit->primary = 3; /* SUPPLYMENTARY */
			c_hit->pri_index = primary_v_idx[n_primary_v] = 0;
			primary_v[n_primary_v++] = (int)ci;
			if (n_primary_v > 750)
				n_primary_v = 750;
		}
	}
}

/*
 * classify_seq, src/cly.c:3059-3127 — part A (everything before the max_read_l update),
 * cut into phases so that each can run as its own launch over all reads of a chunk.
 * dsb_rflags_t carries the control decisions between phases; running the phases in order
 * is exactly the reference's control flow (including the returns on overflow).
 */
enum {
	DSB_PH_ISLAND = 0, /* get_island: seed vectors of both strands */
	DSB_PH_FAST0,      /* fast_classify, forward seed vector */
	DSB_PH_FAST1,      /* fast_classify, reverse seed vector (both_direction) */
	DSB_PH_RESOLVE_F,  /* resolve_tree (chaining + SDP), slow-mode decision */
	DSB_PH_SLOW0,      /* slow_classify, forward */
	DSB_PH_RESOLVE_S0,
	DSB_PH_SLOW1,      /* slow_classify, reverse */
	DSB_PH_RESOLVE_S1,
	DSB_PH_DELA,       /* delete_small_score_rst part A */
	DSB_PH_N
};

typedef struct {
	uint8_t done;      /* read finished early (short read / overflow) */
	uint8_t both;      /* both_direction */
	uint8_t run_slow;
	uint8_t slow1;
} dsb_rflags_t;

/* does phase ph do any work for this read? (lets the host skip empty launches) */
DSB_HD int dsb_phase_active(const dsb_read_ws *w, const dsb_rflags_t *f, int ph)
{
	if (ph == DSB_PH_ISLAND)
		return 1;
	if (f->done || w->overflow)
		return 0;
	switch (ph) {
	case DSB_PH_FAST1: return f->both;
	case DSB_PH_SLOW0: case DSB_PH_RESOLVE_S0: return f->run_slow;
	case DSB_PH_SLOW1: case DSB_PH_RESOLVE_S1: return f->run_slow && f->slow1;
	default: return 1;
	}
}

template <bool WAVE = false>
DSB_HD void dsb_phase(dsb_read_ws *w, dsb_rflags_t *f, int ph)
{
	if (!dsb_phase_active(w, f, ph))
		return;
	const int super_repeat = 0; /* fast_classify returns super_repeat[0], never incremented */
	switch (ph) {
	case DSB_PH_ISLAND:
		w->n_anc = 0;
		w->anc_hw = 0;
		w->fast_classify = 1;
		w->n_hit = 0;
		w->reached_update = 0;
		f->done = f->both = f->run_slow = f->slow1 = 0;
		if (w->L < DSB_MIN_READ_LEN) {
			f->done = 1;
			return;
		}
		dsb_get_island(w);
		f->both = ((w->sd[0].total_score - w->sd[1].total_score) <= (w->sd[0].total_score >> 3));
		return;
	case DSB_PH_FAST0:
		dsb_fast_classify(w, &w->sd[0]);
		return;
	case DSB_PH_FAST1:
		dsb_fast_classify(w, &w->sd[1]);
		return;
	case DSB_PH_RESOLVE_F:
		dsb_resolve_tree<WAVE>(w);
		if (w->overflow)
			return;
		if (w->n_hit <= 0)
			f->run_slow = 1;
		else if (w->hit[0].anchor_number < 5 && super_repeat < 3) {
			f->run_slow = 1;
			if (w->L <= 300 && w->hit[0].sum_score > 200)
				f->run_slow = 0;
		}
		if (f->run_slow) {
			w->anc_hw = DSB_MAX(w->anc_hw, w->n_anc); /* slow_classify starts at n = 0, the capacity stays */
			w->n_anc = 0;
		}
		return;
	case DSB_PH_SLOW0:
		dsb_slow_classify(w, &w->sd[0]);
		return;
	case DSB_PH_RESOLVE_S0:
		dsb_resolve_tree<WAVE>(w);
		if (w->overflow)
			return;
		f->slow1 = (f->both || w->n_hit <= 0 || (w->hit[0].anchor_number < 5 && super_repeat < 3));
		return;
	case DSB_PH_SLOW1:
		dsb_slow_classify(w, &w->sd[1]);
		return;
	case DSB_PH_RESOLVE_S1:
		dsb_resolve_tree<WAVE>(w);
		return;
	case DSB_PH_DELA:
		dsb_delete_small_A<WAVE>(w);
		return;
	}
}

DSB_HDN void dsb_classify_A(dsb_read_ws *w)
{
	dsb_rflags_t f = {0, 0, 0, 0};
	for (int ph = 0; ph < DSB_PH_N; ph++)
		dsb_phase(w, &f, ph);
}

/* Per-read state carried between phase launches (in the read's workspace). */
typedef struct {
	dsb_sdir_t sd[2];
	uint32_t n_anc, n_hit, fast_classify, overflow, reached_update, anc_hw;
	dsb_rflags_t f;
} dsb_rstate_t;

DSB_HD void dsb_state_save(const dsb_read_ws *w, const dsb_rflags_t *f, dsb_rstate_t *s)
{
	s->sd[0] = w->sd[0];
	s->sd[1] = w->sd[1];
	s->n_anc = w->n_anc;
	s->anc_hw = w->anc_hw;
	s->n_hit = w->n_hit;
	s->fast_classify = w->fast_classify;
	s->overflow = w->overflow;
	s->reached_update = w->reached_update;
	s->f = *f;
}

DSB_HD void dsb_state_load(dsb_read_ws *w, dsb_rflags_t *f, const dsb_rstate_t *s)
{
	w->sd[0] = s->sd[0];
	w->sd[1] = s->sd[1];
	w->n_anc = s->n_anc;
	w->anc_hw = s->anc_hw;
	w->n_hit = s->n_hit;
	w->fast_classify = s->fast_classify;
	w->overflow = s->overflow;
	w->reached_update = s->reached_update;
	*f = s->f;
}


/* ------------------------------------------------------------------ finish + output */
/* delete_small_score_rst part B + detect_primary + copy of the hits the SAM writer needs. */
DSB_HD void dsb_classify_B(dsb_read_ws *w, int max_read_l, dsb_read_out_t *ro, dsb_hit_out_t *out, uint32_t out_cap)
{
	if (w->reached_update)
		dsb_delete_small_B(w, max_read_l);
	dsb_detect_primary(w, w->L, (int *)w->stmp, (uint8_t *)w->sidx);
	uint32_t n = DSB_MIN(w->n_hit, out_cap);
	for (uint32_t k = 0; k < n; k++) {
		const dsb_chain_t *c = w->hit + k;
		dsb_hit_out_t *o = out + k;
		o->ref_ID = c->ref_ID;
		o->sum_score = c->sum_score;
		o->t_st = c->t_st; o->t_ed = c->t_ed; o->q_st = c->q_st; o->q_ed = c->q_ed;
		o->indel = c->indel;
		o->direction = c->direction; o->primary = c->primary; o->pri_index = c->pri_index; o->pad = 0;
	}
	ro->n_hit = n;
	ro->n_anchor = w->n_anc;
	ro->fast = w->fast_classify;
	ro->status = w->overflow;
	ro->reached_update = w->reached_update;
}
#endif /* DSB_CLASSIFY_H */
