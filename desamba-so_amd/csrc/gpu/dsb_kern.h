/*
 * dsb_kern.h — the phase kernels of classify part A (templates).  Each phase is compiled in
 * its own translation unit (phase.hip, -DDSB_PH=n) so the phases build in parallel and get
 * their own register allocation; kernels.hip launches them through dsb_phase_kernel_<n>().
 */
#ifndef DSB_KERN_H
#define DSB_KERN_H
#include <hip/hip_runtime.h>
#include "dsb_ws.h"
#include "dsb_gpu.h"

/* minimum waves per SIMD requested from the register allocator (spills beyond) */
/* measured on MI355X (C1 workload, fully inlined phase kernels): fast/slow seeding is fastest
 * at 2 waves/SIMD, the scoring phase at 8, the lane-per-read phases at 2 */
#ifndef DSB_MINW_LANE
#define DSB_MINW_LANE 2
#endif
#ifndef DSB_MINW_FAST
#define DSB_MINW_FAST 2
#endif
#ifndef DSB_MINW_DELA
#define DSB_MINW_DELA 8
#endif
#ifndef DSB_MINW_ISLAND
#define DSB_MINW_ISLAND 6 /* measured (C2, 300k reads): 8 / 6 waves per SIMD -> island 83.0 / 79.3 ms (15 / 2 VGPRs spilled) */
#endif
#ifndef DSB_MINW_RESOLVE
#define DSB_MINW_RESOLVE 4
#endif
/* slow resolves built with 48 KB of LDS per wave (DSB_SORT_LDS_SLOW 4096): at most 3 per CU anyway */
#define DSB_MINW_WAVE(PH) ((PH) == DSB_PH_DELA ? DSB_MINW_DELA : \
			   ((PH) == DSB_PH_FAST0 || (PH) == DSB_PH_FAST1 || (PH) == DSB_PH_SLOW0 || (PH) == DSB_PH_SLOW1) \
			   ? DSB_MINW_FAST : (((PH) == DSB_PH_RESOLVE_S0 || (PH) == DSB_PH_RESOLVE_S1) && DSB_SORT_LDS_SLOW > 1024) ? 1 : DSB_MINW_RESOLVE)
#define DSB_WIN_LDS_BYTES ((DSB_WIN_BYTES + 15) & ~15)
/* The scoring phase's reference windows (sdp_middle ref[2000], sdp_right/left ref[1000]) live in
 * LDS, in the same 4 KB the read-hash build uses for its key-group slots before the first window
 * is loaded (every window byte a scan reads is written in the same call: DESIGN.md §5), so the
 * kernel keeps its 8 waves per SIMD.  DSB_WIN_IN_LDS=0 keeps them in the workspace (HBM). */
#ifndef DSB_WIN_IN_LDS
#define DSB_WIN_IN_LDS 1
#endif
/* DSB_TL=1 (dev builds, tools/variant.sh): the per-read timeline of DSB_DBG_TIMELINE */
#ifndef DSB_TL
#define DSB_TL 0
#endif
#define DSB_DELA_LDS_BYTES (DSB_WIN_LDS_BYTES + 64 > DSB_HB_LDS ? DSB_WIN_LDS_BYTES + 64 : DSB_HB_LDS)
#define DSB_DELA_CAND_OFF 3840 /* 64 u16 candidate slots (dsb_sdp_match_impl, DSB_MATCH_BF) */
static_assert(sizeof(dsb_rstate_t) <= DSB_STATE_BYTES, "per-read phase state must fit its workspace slot");

/* One phase of classify part A (dsb_phase), one lane per read; the read's control state
 * lives in its workspace between launches.  The last phase publishes the read's summary. */
template <int PH, int STATS>
__global__ __launch_bounds__(64, DSB_MINW_LANE) void k_phase(const dsb_dindex_t *__restrict__ ix, const uint32_t *__restrict__ len,
					       const uint64_t *__restrict__ ws_off, const uint32_t *__restrict__ scale,
					       uint8_t *__restrict__ ws, const uint32_t *__restrict__ order, uint32_t n,
					       dsb_read_out_t *__restrict__ ro, uint32_t *__restrict__ n_overflow,
					       unsigned long long *__restrict__ gstats, uint32_t dbg,
									      uint64_t tag)
{
	(void)dbg;
	uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
	if (t >= n)
		return;
	(void)tag;
	uint32_t r = order[t];
	uint32_t L = len[r];
	uint8_t *base = ws + ws_off[r];
	dsb_caps_t cap = dsb_default_caps(L, scale[r]);
	dsb_read_ws w;
	dsb_ws_init(&w, ix, base, L, cap);
	dsb_rstate_t *sp = (dsb_rstate_t *)(base + dsb_layout(L, cap).state);
	dsb_rflags_t f = {0, 0, 0, 0};
	if (PH != DSB_PH_ISLAND)
		dsb_state_load(&w, &f, sp);
	uint64_t st[DSB_ST_N];
	if (STATS == 1) {
		for (int k = 0; k < DSB_ST_N; k++) st[k] = 0;
		w.stats = st;
	}
	dsb_phase(&w, &f, PH);
	dsb_state_save(&w, &f, sp);
	if (PH == DSB_PH_DELA) {
		dsb_read_out_t o;
		o.n_hit = w.n_hit;
		o.n_anchor = w.n_anc;
		o.fast = w.fast_classify;
		o.status = w.overflow;
		o.reached_update = w.reached_update;
		o.pad = 0;
		o.hit_off = 0;
		ro[r] = o;
		if (w.overflow)
			atomicAdd(n_overflow, 1u);
	}
	if (STATS == 1)
		for (int k = 0; k < DSB_ST_N; k++)
			atomicAdd(gstats + DSB_ST_STRIDE * PH + k, (unsigned long long)st[k]);
}

/* The island phase (getIsland, src/cly.c:1231-1263) with two lanes per read: lane 2i scans the
 * forward strand, lane 2i+1 the reverse strand (search_exist_kmer_M2 + get_seed_vector_M2), and
 * the pair exchanges its SEARCH_DIRs.  The reference writes the reverse seeds after the forward
 * ones into one buffer (reverse at L/4, H8): when the forward list runs past L/4 the reverse
 * lane redoes its pass after the forward stores have completed, so its values win there. */
template <int STATS>
__global__ __launch_bounds__(64, DSB_MINW_LANE) void k_island(const dsb_dindex_t *__restrict__ ix, const uint32_t *__restrict__ len,
							   const uint64_t *__restrict__ ws_off, const uint32_t *__restrict__ scale,
							   uint8_t *__restrict__ ws, const uint32_t *__restrict__ order, uint32_t n,
							   dsb_read_out_t *__restrict__ ro, uint32_t *__restrict__ n_overflow,
							   unsigned long long *__restrict__ gstats, uint32_t dbg,
									      uint64_t tag)
{
	(void)dbg; (void)ro; (void)n_overflow; (void)gstats; (void)tag;
	uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
	uint32_t i = t >> 1, strand = t & 1;
	if (i >= n) /* both lanes of a pair leave together */
		return;
	uint32_t r = order[i];
	uint32_t L = len[r];
	uint8_t *base = ws + ws_off[r];
	dsb_caps_t cap = dsb_default_caps(L, scale[r]);
	dsb_read_ws w;
	dsb_ws_init(&w, ix, base, L, cap);
	dsb_rstate_t *sp = (dsb_rstate_t *)(base + dsb_layout(L, cap).state);
	dsb_rflags_t f = {0, 0, 0, 0};
	w.n_anc = 0;
	w.anc_hw = 0;
	w.fast_classify = 1;
	w.n_hit = 0;
	w.reached_update = 0;
	uint64_t st_isl[DSB_ST_N]; /* the scan's own counters: bits read (DSB_NEED_STATS), on-demand probes */
	if (DSB_NEED_STATS && STATS == 1) {
		for (int k = 0; k < DSB_ST_N; k++) st_isl[k] = 0;
		w.stats = st_isl;
	}
	if (L < DSB_MIN_READ_LEN) {
		f.done = 1;
	} else {
		dsb_sdir_t sd;
		if (strand == 0)
			dsb_seed_vector(&w, 0, 0, DSB_FORWARD, &sd);
		else
			dsb_seed_vector(&w, 1, L >> 2, DSB_REVERSE, &sd);
		dsb_sdir_t o;
		o.seed_off = (uint32_t)__shfl_xor((int)sd.seed_off, 1);
		o.l_seed_v_f = (uint32_t)__shfl_xor((int)sd.l_seed_v_f, 1);
		o.strand = (uint32_t)__shfl_xor((int)sd.strand, 1);
		o.direction = (uint32_t)__shfl_xor((int)sd.direction, 1);
		o.total_score = (uint32_t)__shfl_xor((int)sd.total_score, 1);
		uint32_t l_fwd = strand == 0 ? sd.l_seed_v_f : o.l_seed_v_f;
		if (l_fwd > (L >> 2)) { /* forward seeds reach the reverse buffer: the reverse pass goes last */
			__threadfence();
			if (strand == 1)
				dsb_seed_vector(&w, 1, L >> 2, DSB_REVERSE, &sd);
		}
		w.sd[0] = strand == 0 ? sd : o;
		w.sd[1] = strand == 0 ? o : sd;
		if (w.sd[0].total_score < w.sd[1].total_score) {
			dsb_sdir_t x = w.sd[0];
			w.sd[0] = w.sd[1];
			w.sd[1] = x;
		}
		f.both = ((w.sd[0].total_score - w.sd[1].total_score) <= (w.sd[0].total_score >> 3));
	}
	if (strand == 0)
		dsb_state_save(&w, &f, sp);
	if (DSB_NEED_STATS && STATS == 1 && gstats) {
		const int sl[3] = {DSB_ST_OCC, DSB_ST_EK1, DSB_ST_EK2};
		for (int k = 0; k < 3; k++)
			if (st_isl[sl[k]])
				atomicAdd(gstats + DSB_STATS_SEED + sl[k], (unsigned long long)st_isl[sl[k]]);
	}
}

/* The island phase probing the Bloom tables itself (DSB_ISLAND_G lanes per strand, both strands
 * of a read in one wave; dsb_isl_* in dsb_classify.h): search_exist_kmer_M2 + get_seed_vector_M2
 * + getIsland (src/cly.c:1066-1263) without k_seed's exist bits.  Each batch, every lane probes
 * one position (get_exist_kmer, src/cly.c:951-967: the l_ek-mer, table 0, table 1 for a hit),
 * the strand's G bits come from one ballot, and the strand's lanes update the same scan state.
 * The lanes also store the 13-mer prefix value (the seeding J step's) of the positions that can
 * lie inside a seed: every run batch position and each grid hit.  H8: when the forward list runs
 * past L/4 the reverse strand redoes its scan after the forward stores, so its values win
 * there, and the read's prefix values are then filled for every position. */
#ifndef DSB_ISL_WIN
#define DSB_ISL_WIN 1
#endif
#ifndef DSB_ISL_GG
#define DSB_ISL_GG 8 /* positions per grid batch (0: DSB_ISLAND_G); measured grid 16 / 12 / 8: 24.7 / 22.8 / 21.8 ms */
#endif
#ifndef DSB_ISL_GR
#define DSB_ISL_GR 0 /* positions per run batch (0: DSB_ISLAND_G) */
#endif
#ifndef DSB_ISL_SPEC2
#define DSB_ISL_SPEC2 0 /* probe both Bloom tables at once (the second speculatively) */
#endif
#ifndef DSB_ISL_GR1
#define DSB_ISL_GR1 0 /* positions of a run's first batch, 2 back neighbours included (0: as DSB_ISL_GR) */
#endif

template <int G, int STATS>
__global__ __launch_bounds__(64, DSB_MINW_ISLAND) void k_island_g(const dsb_dindex_t *__restrict__ ix, const uint32_t *__restrict__ len,
								   const uint64_t *__restrict__ ws_off, const uint32_t *__restrict__ scale,
								   uint8_t *__restrict__ ws, const uint32_t *__restrict__ order, uint32_t n,
								   dsb_read_out_t *__restrict__ ro, uint32_t *__restrict__ n_overflow,
								   unsigned long long *__restrict__ gstats, uint32_t dbg, uint64_t tag)
{
	static_assert(G >= 4 && G <= 32 && (G & (G - 1)) == 0, "lanes per strand: 4, 8, 16 or 32");
	/* positions per grid / run batch (<= G lanes) */
	constexpr int GG = DSB_ISL_GG > 0 && DSB_ISL_GG < G ? DSB_ISL_GG : G;
	constexpr int GR = DSB_ISL_GR > 0 && DSB_ISL_GR < G ? DSB_ISL_GR : G;
	constexpr int GR1 = DSB_ISL_GR1 >= 4 && DSB_ISL_GR1 < GR ? DSB_ISL_GR1 : GR;
	(void)dbg; (void)ro; (void)n_overflow; (void)tag;
	const uint32_t GM = G == 32 ? 0xffffffffu : ((1u << G) - 1);
	uint32_t lane = threadIdx.x, sg = lane / G, gl = lane % G;
	uint32_t t = blockIdx.x * (64 / (2 * G)) + (sg >> 1), strand = sg & 1;
	int live = t < n;
	uint32_t r = live ? order[t] : 0;
	uint32_t L = live ? len[r] : 0;
	int l_ek = ix->l_ek, sbm = ix->single_base_max;
	uint8_t *base = ws + (live ? ws_off[r] : 0);
	int run = live && L >= DSB_MIN_READ_LEN;
	int nk = run ? (int)L - l_ek + 1 : 0; /* l_kmer_buff */
	/* the read's buffers (dsb_ws_init's carving, without the rest of the per-read state) */
	dsb_ws_layout lay = dsb_layout(L, dsb_default_caps(L, live ? scale[r] : DSB_SCALE_UNIT));
	uint64_t sb = lay.bin + DSB_BIN_GUARD + strand * L; /* the strand's first base */
	uint32_t *pre = (uint32_t *)(base + lay.pre) + strand * L;
	dsb_seed_t *seed_v = (dsb_seed_t *)(base + lay.seeds) + (strand ? L >> 2 : 0);
	dsb_rstate_t *sp = (dsb_rstate_t *)(base + lay.state);
	uint32_t p1 = 0, p2 = 0;
	dsb_topst_t top;
	dsb_top_init(&top);
	uint32_t l_fwd = 0;
#if DSB_ISL_WIN
	/* the strand as aligned 8-byte words: position q is byte (q + bo) of word 0 (the workspace
	 * base is 8-aligned; the window never starts before it) */
	const uint64_t *bw = (const uint64_t *)(base + (sb & ~7ull));
	int bo = (int)(sb & 7);
	int64_t wmin = -(int64_t)(sb >> 3), wb = INT64_MIN / 2;
	uint64_t wv = 0;
#else
	const uint8_t *bin = base + sb;
#endif
	for (int pass = 0; pass < 2; pass++) {
		/* pass 1: only the reverse strands of reads whose forward list reached L/4 */
		int mine = run && (pass == 0 || (strand == 1 && l_fwd > (L >> 2)));
		if (!__ballot(mine))
			break;
		dsb_isl_t s;
		dsb_isl_init(&s, nk, strand == 0, mine);
		if (mine)
			dsb_top_init(&top);
		for (;;) {
			if (!__ballot(s.mode != DSB_ISL_DONE))
				break;
			int q = dsb_isl_pos<GG, GR, GR1>(&s, (int)gl);
			int b = 0;
			uint32_t pv = 0;
#if DSB_ISL_WIN
			/* the bytes of the batch's k-mers as aligned words of the strand: lane gl of the
			 * group holds word wb + gl of a G-word window, reloaded (one coalesced load) only
			 * when the batch leaves it; each k-mer's four words come by lane shuffles */
			int lo, hi;
			dsb_isl_span<GG, GR, GR1>(&s, &lo, &hi);
			int64_t klo = ((int64_t)lo + bo) >> 3, khi = (((int64_t)hi + bo) >> 3) + 3;
			if (s.mode != DSB_ISL_DONE && lo <= hi && (klo < wb || khi >= wb + G)) {
				wb = s.fwd ? klo : DSB_MAX(khi - (G - 1), wmin);
				wv = dsb_gld(bw + wb + gl);
			}
			int src = q >= 0 ? (int)(sg * G) + (int)((((int64_t)q + bo) >> 3) - wb) : (int)lane;
			uint64_t wq[4];
#pragma unroll
			for (int j = 0; j < 4; j++) {
				int sj = q >= 0 ? src + j : (int)lane;
				wq[j] = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(wv >> 32), sj) << 32) |
					(uint32_t)__shfl((int)(uint32_t)wv, sj);
			}
			if (q >= 0) {
				uint32_t sh = (uint32_t)((q + bo) & 7) * 8;
				uint64_t x0 = sh ? (wq[0] >> sh) | (wq[1] << (64 - sh)) : wq[0];
				uint64_t x1 = sh ? (wq[1] >> sh) | (wq[2] << (64 - sh)) : wq[1];
				uint64_t x2 = sh ? (wq[2] >> sh) | (wq[3] << (64 - sh)) : wq[2];
				uint64_t km = dsb_kmer_w(x0, x1, x2, l_ek, sbm);
#else
			if (q >= 0) {
				uint64_t km = dsb_kmer_at(bin + q, l_ek, sbm);
#endif
				pv = (uint32_t)(km & DSB_PRE_IDX_MASK);
				if (km) {
					uint64_t h1 = dsb_hash64_1(km) & ix->ek_mask;
					p1++;
#if DSB_ISL_SPEC2
					/* both tables' bytes in one round trip: the second probe is speculative (the
					 * reference reads table 1 only after a table-0 hit; the bit is the same) */
					uint64_t h2 = dsb_hash64_2(km) & ix->ek_mask;
					uint8_t e0 = dsb_gld(ix->ek0 + (h1 >> 3)), e1 = dsb_gld(ix->ek1 + (h2 >> 3));
					if ((e0 >> (7 - (h1 & 0x7))) & 0x1) {
						p2++;
						b = (e1 >> (7 - (h2 & 0x7))) & 0x1;
					}
#else
					if ((dsb_gld(ix->ek0 + (h1 >> 3)) >> (7 - (h1 & 0x7))) & 0x1) {
						uint64_t h2 = dsb_hash64_2(km) & ix->ek_mask;
						p2++;
						b = (dsb_gld(ix->ek1 + (h2 >> 3)) >> (7 - (h2 & 0x7))) & 0x1;
					}
#endif
				}
			}
			uint32_t mb = (uint32_t)(__ballot(b) >> (sg * G)) & GM;
			if (q >= 0 && (s.mode != DSB_ISL_GRID || (mb && (int)gl == __builtin_ctz(mb))))
				pre[q] = pv;
			uint32_t so = 0, sl = 0;
			if (dsb_isl_step<GG, GR, GR1>(&s, mb, &so, &sl) && gl == 0) {
				uint32_t m = top.n, ti;
				seed_v[m].offset = so;
				seed_v[m].len = sl;
				seed_v[m].top = 0;
				uint8_t tv = dsb_top_push(&top, strand == 0 ? so : (uint32_t)nk - so - sl, sl, &ti);
				seed_v[ti].top = tv;
			}
		}
		if (mine && gl == 0) {
			seed_v[top.max_index].top = 1; /* also when no seed (a stale slot, as the reference) */
			top.total += top.max_length;
		}
		/* the forward lists' lengths, then (pass 1) the reverse pass after the forward stores */
		uint32_t lf = (uint32_t)__shfl((int)top.n, (int)(lane & ~(2u * G - 1)));
		if (pass == 0)
			l_fwd = lf;
		__threadfence_block();
	}
	/* H8: a reverse list rewritten over the forward one moves the seeds the J step starts from:
	 * store the prefix value of every position of both strands of such a read */
	if (__ballot(run && l_fwd > (L >> 2))) {
		if (run && l_fwd > (L >> 2))
			for (int q = (int)gl; q < nk; q += G)
				pre[q] = (uint32_t)(dsb_kmer_at(base + sb + q, l_ek, sbm) & DSB_PRE_IDX_MASK);
	}
	/* getIsland's SEARCH_DIRs + the read's state for the next phases (k_island's, dsb_phase
	 * ISLAND): the forward group's lane 0 takes the reverse group's results */
	uint32_t rn = (uint32_t)__shfl((int)top.n, (int)(lane + G) & 63);
	uint32_t rt = (uint32_t)__shfl((int)top.total, (int)(lane + G) & 63);
	if (live && strand == 0 && gl == 0) {
		dsb_rflags_t f = {0, 0, 0, 0};
		dsb_sdir_t a = {0, top.n, 0, DSB_FORWARD, top.total}, c = {L >> 2, rn, 1, DSB_REVERSE, rt};
		if (L < DSB_MIN_READ_LEN) {
			f.done = 1;
			a = sp->sd[0]; /* untouched, as k_island leaves them */
			c = sp->sd[1];
		} else {
			if (a.total_score < c.total_score) {
				dsb_sdir_t x = a;
				a = c;
				c = x;
			}
			f.both = ((a.total_score - c.total_score) <= (a.total_score >> 3));
		}
		sp->sd[0] = a;
		sp->sd[1] = c;
		sp->n_anc = 0;
		sp->anc_hw = 0; /* the read's anchor-vector high-water mark (dsb_map_seed): the workspace holds an earlier read's */
		sp->n_hit = 0;
		sp->fast_classify = 1;
		sp->overflow = 0;
		sp->reached_update = 0;
		sp->f = f;
	}
	if (STATS == 1 && gstats) {
		for (int o = 32; o >= 1; o >>= 1) {
			p1 += (uint32_t)__shfl_xor((int)p1, o);
			p2 += (uint32_t)__shfl_xor((int)p2, o);
		}
		if (lane == 0) {
			atomicAdd(gstats + DSB_STATS_SEED + DSB_ST_EK1, (unsigned long long)p1);
			atomicAdd(gstats + DSB_STATS_SEED + DSB_ST_EK2, (unsigned long long)p2);
		}
	}
}

/* The read 9-mer hash of the scoring phase (build_hash_table_M2, src/cly.c:2168-2219), built in
 * LDS by a workgroup of 256 lanes per (read, strand) before the scoring launch (DSB_HASH_LDS):
 * the scoring kernel's own build updated its head table in HBM, a scattered 4-B read-modify-
 * write per position (~1 G per 100k reads, 32-B write granules), and building the tables twice
 * there cost ~20 ms per 100k-read chunk on the C2 proxy (profiles/r04_d).  Here the head table
 * (2^14 keys, dsb_hash_kl_lds) lives in LDS while the positions are inserted, and goes to HBM once,
 * coalesced; the node entries are written as before (consecutive positions, coalesced).
 *
 * Positions are inserted from the end in blocks of 256 (one per lane), so every list keeps
 * increasing positions.  Inside a block each lane must find the nearest higher lane with its key
 * (its list successor) and whether a lower lane has it (then that lane, not this one, becomes the
 * head): every lane writes its lane id to a byte slot of its key's low bits and reads it back; two
 * lanes with one key wrote the same slot, so at least one of them lost, and the lost lanes (a few
 * per block) with the lanes they lost to are all the candidates a lane has to compare with (the
 * wave build's argument, dsb_build_hash_table). */
#define DSB_HL_WG 256
static_assert(DSB_HASH_LDS_KL <= 16, "k_hash_lds keeps keys in 16 bits");
#define DSB_HL_SLOTS 4096
template <int STATS>
__global__ __launch_bounds__(DSB_HL_WG, DSB_HASH_LDS_KL <= 13 ? 4 : 2) void k_hash_lds(const dsb_dindex_t *__restrict__ ix, const uint32_t *__restrict__ len,
							 const uint64_t *__restrict__ ws_off, const uint32_t *__restrict__ scale,
							 uint8_t *__restrict__ ws, const uint32_t *__restrict__ order, uint32_t n,
							 unsigned long long *__restrict__ gstats)
{
	__shared__ uint32_t heads[1u << DSB_HASH_LDS_KL];
	__shared__ uint8_t slot[DSB_HL_SLOTS];
	__shared__ uint16_t keyl[DSB_HL_WG]; /* the lanes' keys (< 2^14) */
	__shared__ uint32_t entl[DSB_HL_WG];
	__shared__ uint2 los[DSB_HL_WG]; /* lost lane | winner << 8 | its key << 16, the winner's key */
	__shared__ uint32_t n_los, sh_n, sh_dirs;
	uint32_t t = blockIdx.x >> 1, h = blockIdx.x & 1, tid = threadIdx.x;
	if (t >= n)
		return;
	uint32_t r = order[t];
	uint32_t L = len[r];
	if (!dsb_hash_lds_read(L) || L < DSB_S_A_KMER_L)
		return;
	uint8_t *base = ws + ws_off[r];
	dsb_caps_t cap = dsb_default_caps(L, scale[r]);
	dsb_ws_layout lay = dsb_layout(L, cap);
	dsb_read_ws w;
	dsb_ws_init(&w, ix, base, L, cap);
	dsb_rflags_t f;
	dsb_state_load(&w, &f, (const dsb_rstate_t *)(base + lay.state));
	if (f.done || w.overflow || w.n_hit == 0)
		return; /* dsb_delete_small_A does not reach the build */
	/* dsb_hash_dirs over the workgroup: the hits the scoring keeps (the first one from 200 on
	 * scoring <= 50 ends them, at most 400), then their directions */
	if (tid == 0) {
		sh_n = w.n_hit;
		sh_dirs = 0;
	}
	__syncthreads();
	if (w.n_hit > 200)
		for (uint32_t i = 200 + tid; i < w.n_hit; i += DSB_HL_WG)
			if (w.hit[i].sum_score <= 50)
				atomicMin(&sh_n, i);
	__syncthreads();
	uint32_t nh = DSB_MIN(400u, sh_n);
	for (uint32_t i = tid; i < nh; i += DSB_HL_WG)
		atomicOr(&sh_dirs, w.hit[i].direction == DSB_FORWARD ? 2u : 1u);
	__syncthreads();
	int dirs = (int)sh_dirs;
	int c_dir = h == 0 ? 2 : 1; /* table 0: the forward hits' strand, table 1: the reverse hits' */
	if ((c_dir & dirs) == 0)
		return;
	uint32_t direction = (c_dir == 1) ? DSB_REVERSE : DSB_FORWARD;
	const dsb_sdir_t *csd = (w.sd[0].direction == direction) ? &w.sd[0] : &w.sd[1];
	const uint8_t *q = w.bin + (csd->strand ? L : 0);
	int kl = dsb_hash_kl_lds(L);
	uint32_t KEY_MASK = (1u << kl) - 1;
	uint32_t *g_heads = w.hh[h], *node = w.hn[h];
	int n_pos = (int)L - DSB_S_A_KMER_L + 1;
	for (uint32_t k = tid; k <= KEY_MASK; k += DSB_HL_WG) heads[k] = DSB_HEMPTY;
	if (STATS && tid == 0) {
		unsigned long long *st = gstats + DSB_ST_STRIDE * DSB_PH_DELA;
		/* head table at the reference's key length + per position: the node write, head read and write */
		atomicAdd(st + DSB_ST_HASH_B, (unsigned long long)(4ull * (1ull << dsb_hash_kl_ref(L)) + 12ull * n_pos));
	}
	/* the blocks' k-mers, loaded four blocks ahead (a block's LDS work is shorter than a load) */
	int cb = (n_pos - 1) & ~(DSB_HL_WG - 1);
	auto ld = [&](int b) -> uint32_t { return (b >= 0 && b + (int)tid < n_pos) ? dsb_q9mer(q + b + tid) : 0; };
	uint32_t k0 = ld(cb), k1 = ld(cb - DSB_HL_WG), k2 = ld(cb - 2 * DSB_HL_WG), k3 = ld(cb - 3 * DSB_HL_WG);
	__syncthreads();
	for (; cb >= 0; cb -= DSB_HL_WG) {
		int c_pos = cb + (int)tid;
		int act = c_pos < n_pos;
		uint32_t km = k0;
		k0 = k1;
		k1 = k2;
		k2 = k3;
		k3 = ld(cb - 4 * DSB_HL_WG);
		int key = act ? (int)(km & KEY_MASK) : -1 - (int)tid;
		keyl[tid] = (uint16_t)key; /* read back for active (winning) lanes only */
		if (tid == 0)
			n_los = 0;
		if (act)
			slot[key & (DSB_HL_SLOTS - 1)] = (uint8_t)tid;
		__syncthreads();
		int won = act ? (int)slot[key & (DSB_HL_SLOTS - 1)] : (int)tid;
		if (won != (int)tid) {
			uint32_t k = atomicAdd(&n_los, 1u);
			los[k] = make_uint2(tid | ((uint32_t)won << 8) | ((uint32_t)key << 16), keyl[won]);
		}
		__syncthreads();
		int has_prev = 0, nxt = DSB_HL_WG;
		uint32_t nl = n_los;
		if (act)
			for (uint32_t k = 0; k < nl; k++) {
				uint2 e = los[k]; /* one 8-B LDS read per lost lane, independent of the others */
				int o = (int)(e.x & 0xffu), w2 = (int)((e.x >> 8) & 0xffu);
				if ((int)(e.x >> 16) == key) {
					if (o < (int)tid) has_prev = 1;
					else if (o > (int)tid) nxt = DSB_MIN(nxt, o);
				}
				if ((int)e.y == key) {
					if (w2 < (int)tid) has_prev = 1;
					else if (w2 > (int)tid) nxt = DSB_MIN(nxt, w2);
				}
			}
		uint32_t old = act ? heads[key] : DSB_HEMPTY;
		uint32_t ent = dsb_hentry((uint32_t)c_pos, km, nxt < DSB_HL_WG || old != DSB_HEMPTY, kl);
		entl[tid] = ent;
		__syncthreads();
		if (act) {
			node[c_pos] = nxt < DSB_HL_WG ? entl[nxt] : old;
			if (!has_prev)
				heads[key] = ent;
		}
		/* no barrier here: the next block's first LDS writes (keys, slots, the loser count) touch
		 * nothing this block reads after the barrier above, and its head reads follow its own
		 * first barrier */
	}
	__syncthreads();
	for (uint32_t k = tid; k <= KEY_MASK; k += DSB_HL_WG) g_heads[k] = heads[k];
}

/* The seeding sp_set pool (DSB_HSET_POOL): a wave takes a free set for its seeding call and hands
 * it back with the set's generation base moved past every generation its lanes used.
 *
 * The pool is split by XCD (hpool_nx partitions of hpool_part sets), and a wave takes a set of its
 * own XCD's partition: the sets' slots are written with ordinary stores, which an XCD's L2 holds
 * back (write-back, not coherent with the other XCDs' L2s), so every holder of a set must sit
 * behind the same L2.  That makes the hand-over cheap: no agent-scope acquire / release, whose
 * fences write back and invalidate the whole L2 (buffer_wbl2 / buffer_inv sc1) — with them the
 * fast seeding ran 11-15% slower (C2 proxy).  Lane 0 takes the set with a relaxed CAS on its owner
 * flag (device-scope atomics are performed past the L2s), probing from slot `start`; a partition
 * holds at least as many sets as its XCD holds waves, so a free set always exists and the probe
 * ends.  On release the wave first waits for its own slot stores to reach the L2
 * (s_waitcnt vmcnt(0)), then stores the new base, waits again, and clears the owner flag, so the
 * next holder reads the new base and finds every slot of this holder in the L2.  A next holder
 * may still see an older copy of a line in its CU's L1: older lines hold older generations,
 * which never match. */
#if DSB_HSET_POOL
#if defined(__HIP_DEVICE_COMPILE__)
static_assert(DSB_HSET_WAVE_U64 == (uint64_t)DSB_HSET_SLOT_U64 * DSB_HSET_SLOTS * DSB_WV, "a pool set holds one wave's tables");
#endif
__device__ __forceinline__ uint32_t dsb_hpool_acquire(const dsb_dindex_t *ix, uint32_t start, uint64_t *gen_base)
{
	uint32_t s = 0, glo = 0, ghi = 0;
	const int fenced = ix->hpool_fenced; /* uniform */
	if (dsb_lane() == 0) {
		/* HW_REG_XCC_ID: dev_init checked that the device's waves report exactly 0..hpool_nx-1
		 * (else hpool_nx is 1 and the hand-over fenced) */
		uint32_t xcc = ((uint32_t)__builtin_amdgcn_s_getreg(20 | (31 << 11)) & 0xfu) % ix->hpool_nx;
		uint32_t mask = ix->hpool_part - 1, base = xcc * ix->hpool_part, q = start & mask;
		for (;;) {
			uint32_t expect = 0;
			if (fenced ? __hip_atomic_compare_exchange_strong(ix->hpool_own + base + q, &expect, 1u, __ATOMIC_ACQUIRE,
									  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
				   : __hip_atomic_compare_exchange_strong(ix->hpool_own + base + q, &expect, 1u, __ATOMIC_RELAXED,
									  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
				break;
			q = (q + 1) & mask;
		}
		s = base + q;
		uint64_t g = __hip_atomic_load(ix->hpool_gen + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		glo = (uint32_t)g;
		ghi = (uint32_t)(g >> 32);
	}
	*gen_base = ((uint64_t)(uint32_t)dsb_wshfl((int)ghi, 0) << 32) | (uint32_t)dsb_wshfl((int)glo, 0);
	if (fenced) /* every lane: no stale line of the set in this CU's L1 / this XCD's L2 */
		__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
	return (uint32_t)dsb_wshfl((int)s, 0);
}
/* the next holder's tags start past `last_gen`, the wave's highest generation */
__device__ __forceinline__ void dsb_hpool_release(const dsb_dindex_t *ix, uint32_t s, uint64_t gen_base, uint32_t last_gen, uint32_t dbg)
{
	uint32_t top = (uint32_t)dsb_wmax((int)last_gen);
	if (ix->hpool_fenced) /* every lane's slot stores written back past this XCD's L2 */
		__builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
	else
		__builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup"); /* keeps the slot stores above the wait */
	__builtin_amdgcn_s_waitcnt(0);                        /* every lane's slot stores are in the L2 */
	if (dsb_lane() == 0) {
		if (!(dbg & DSB_DBG_POOL_NOGEN)) /* tests: keep the base, so the next holder meets live slots */
			__hip_atomic_store(ix->hpool_gen + s, gen_base + top + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		__builtin_amdgcn_s_waitcnt(0);
		__hip_atomic_store(ix->hpool_own + s, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	}
}
#endif

/* the seeding sp_set's first level in LDS (dsb_classify.h dsb_set_insert); 0: every entry in the pool set */
#ifndef DSB_HSET_LDS
#define DSB_HSET_LDS 1
#endif

/* resolve_tree fused into the seeding kernels (wave_phase_read; the host skips the resolve launches,
 * kernels.hip resolve_fused).  Parity-green, but slower on c2l18 (A/B, 3 steps: 517.9k fused vs
 * 523.8k separate): the fused fast-seeding kernel spills 432 B per lane instead of 192, and fast
 * seeding grew by more than the resolve launch it absorbed (642 + 48 -> 715 ms per step).  Off. */
#ifndef DSB_FUSE_RESOLVE
#define DSB_FUSE_RESOLVE 0
#endif
/* the seeding kernels' LDS buffer: the sp_set first level, then the fused resolve's sort arrays */
#define DSB_SEED_LDS_U64 DSB_MAX((DSB_HSET_LDS ? DSB_HSET_L1 * 64u : 1u), (12u * DSB_MAX(DSB_SORT_LDS, DSB_SORT_LDS_SLOW) + 7u) / 8u)

/* Lanes per read of the seeding phases (FAST0/1, SLOW0/1): 64 = a wave per read; 32 = two reads
 * per wave, each on a half-wave group running the state machine of dsb_seed_sm on its own (a
 * read's wave time is set by its longest seed, so the other lanes mostly wait: tools/seed_prof). */
#ifndef DSB_SM_G
#define DSB_SM_G 64
#endif
static_assert(DSB_SM_G == 64 || DSB_SM_G == 32, "lanes per read of the seeding phases: 64 or 32");
#define DSB_PH_SEEDING(PH) ((PH) == DSB_PH_FAST0 || (PH) == DSB_PH_FAST1 || (PH) == DSB_PH_SLOW0 || (PH) == DSB_PH_SLOW1)
#define DSB_PH_LANES(PH) (DSB_PH_SEEDING(PH) ? DSB_SM_G : 64)

/* the scoring phase's LDS: reference windows, the read hash build's slots, the register k-mer
 * match's candidate slots, a window's read range */
__device__ __forceinline__ void dsb_dela_lds(dsb_read_ws *w, uint64_t *dela_lds)
{
	w->lds_hb = (uint8_t *)dela_lds;
	if (DSB_WIN_IN_LDS)
		w->win = (uint8_t *)dela_lds;
	/* the register k-mer match's candidate slots: past the windows, inside the build's area */
	static_assert(DSB_WIN_LDS_BYTES <= DSB_DELA_CAND_OFF && DSB_DELA_CAND_OFF + 128 <= DSB_DELA_LDS_BYTES,
		      "candidate slots must not overlap the windows");
	w->lds_cand = (uint16_t *)((uint8_t *)dela_lds + DSB_DELA_CAND_OFF);
	/* a window's read range (DSB_QCOPY): the LDS past the windows */
	static_assert(!DSB_QCOPY || (DSB_WIN_LDS_BYTES + DSB_QCOPY_BYTES <= DSB_DELA_LDS_BYTES && (DSB_WIN_LDS_BYTES & 7) == 0),
		      "the read-range copy must fit past the windows");
	static_assert(!(DSB_MATCH_BF && DSB_QCOPY), "the candidate slots share the read-range copy's LDS");
	if (DSB_QCOPY)
		w->lds_q = (uint8_t *)dela_lds + DSB_WIN_LDS_BYTES;
}

/* One read of a phase of part A with one wavefront per read (dsb_wave.h), or a group of
 * DSB_PH_LANES(PH) lanes per read: fast seeding (FAST0/FAST1), chaining (RESOLVE_*), scoring
 * (DELA).  `live`: the group has a read (the last wave of a launch may hold fewer).  The last
 * phase publishes the read's summary like k_phase. */
template <int PH, int STATS>
__device__ __forceinline__ void wave_phase_read(const dsb_dindex_t *__restrict__ ix, const uint32_t *__restrict__ len,
						const uint64_t *__restrict__ ws_off, const uint32_t *__restrict__ scale,
						uint8_t *__restrict__ ws, const uint32_t *__restrict__ order, uint32_t t, int live,
						dsb_read_out_t *__restrict__ ro, uint32_t *__restrict__ n_overflow,
						uint64_t *st, uint64_t *tmr_lds, unsigned long long *__restrict__ gstats,
						uint32_t dbg, uint64_t tag)
{
	const int ph = PH;
	constexpr int G = DSB_PH_LANES(PH);
	uint32_t lane = threadIdx.x & (G - 1); /* the lane's index in its read's group */
	uint32_t r = order[t];
	uint64_t tl0 = (DSB_TL && (dbg & DSB_DBG_TIMELINE)) ? __builtin_amdgcn_s_memrealtime() : 0;
	uint32_t L = len[r];
	uint8_t *base = ws + ws_off[r];
	dsb_caps_t cap = dsb_default_caps(L, scale[r]);
	dsb_ws_layout lay = dsb_layout(L, cap);
	dsb_read_ws w;
	dsb_ws_init(&w, ix, base, L, cap);
	dsb_rstate_t *sp = (dsb_rstate_t *)(base + lay.state);
	dsb_rflags_t f;
	dsb_state_load(&w, &f, sp);
	w.dbg = dbg;
	w.launch_tag = tag;
	if (STATS == 1)
		w.stats = st;
	if (STATS == 2)
		w.tmr = tmr_lds;
	int active = live && dsb_phase_active(&w, &f, ph);
#if DSB_HSET_POOL
	/* the seeding wave's sp_set set: taken and handed back by the whole wave (its lanes' tables
	 * serve the reads of all its groups), if any group seeds */
	uint32_t ps = 0;
	uint64_t hs_tag = 0;
	uint64_t *hset = nullptr;
	uint32_t last_gen = 0;
	const int pool_wave = DSB_PH_SEEDING(PH) && __ballot(active) != 0;
	if (pool_wave) {
		/* tests (DSB_DBG_POOL_NOGEN): sets picked by the first group's read length, so a copy of
		 * a read meets the set an earlier copy used */
		uint32_t start = (dbg & DSB_DBG_POOL_NOGEN) ? ((uint32_t)__builtin_amdgcn_readfirstlane((int)L) * 0x9E3779B1u) >> 19
							    : (uint32_t)__builtin_amdgcn_readfirstlane((int)t);
		ps = dsb_hpool_acquire(ix, start, &hs_tag);
		hset = ix->hpool + (uint64_t)ps * DSB_HSET_WAVE_U64;
	}
#endif
	if (active) {
		if (DSB_PH_SEEDING(PH)) {
			/* no clearing: slots carry the set's tag (dsb_set_insert) */
#if !DSB_HSET_POOL
			uint64_t *hset = (uint64_t *)(base + lay.hset);
			uint64_t hs_tag = dsb_hset_tag(&w);
			uint32_t last_gen;
#endif
			/* LDS: per group, 2 x G ints (dsb_seed_sm's owner / max arrays); the sp_set's first level
			 * (dsb_set_insert: DSB_HSET_L1 u64 per lane, 16 KB per wave), reused after the seeding by the
			 * fused resolve's sort arrays */
			__shared__ uint64_t hs_l1[DSB_SEED_LDS_U64];
			if (ph == DSB_PH_FAST0 || ph == DSB_PH_FAST1) {
				__shared__ int32_t sm_lds[2 * 64];
				last_gen = dsb_fast_classify_sm<G>(&w, &w.sd[ph - DSB_PH_FAST0], hset, hs_tag, sm_lds, DSB_HSET_LDS ? hs_l1 : nullptr);
			} else {
				__shared__ int32_t sm_lds2[2 * 64];
				last_gen = dsb_slow_classify_sm<G>(&w, &w.sd[ph == DSB_PH_SLOW0 ? 0 : 1], hset, hs_tag, w.mem, sm_lds2,
								   DSB_HSET_LDS ? hs_l1 : nullptr);
			}
#if !DSB_HSET_POOL
			(void)last_gen;
#endif
			/* the read's resolve right after its seeding (DSB_FUSE_RESOLVE): resolve_tree of the fast
			 * reads after their last fast phase, of the slow reads after each slow phase — the same
			 * per-read steps in the same order as separate launches, but a read with a long resolve
			 * runs it beside the other reads' seeding instead of as the tail of a launch of its own */
			if (DSB_FUSE_RESOLVE && STATS == 0 && G == 64) {
				const int rph = ((ph == DSB_PH_FAST0 && !f.both) || ph == DSB_PH_FAST1) ? DSB_PH_RESOLVE_F
						: ph == DSB_PH_SLOW0 ? DSB_PH_RESOLVE_S0 : ph == DSB_PH_SLOW1 ? DSB_PH_RESOLVE_S1 : -1;
				if (rph >= 0) {
					const uint32_t NS = rph == DSB_PH_RESOLVE_F ? DSB_SORT_LDS : DSB_SORT_LDS_SLOW;
					dsb_wsync();
					w.lds_key = hs_l1;
					w.lds_id = (uint32_t *)(hs_l1 + NS);
					w.lds_n = NS;
					dsb_phase<true>(&w, &f, rph);
				}
			}
		} else if (ph == DSB_PH_RESOLVE_F || ph == DSB_PH_RESOLVE_S0 || ph == DSB_PH_RESOLVE_S1) {
			constexpr uint32_t NS = (PH == DSB_PH_RESOLVE_S0 || PH == DSB_PH_RESOLVE_S1) ? DSB_SORT_LDS_SLOW : DSB_SORT_LDS;
			__shared__ uint64_t sort_key[NS];
			__shared__ uint32_t sort_id[NS];
			w.lds_key = sort_key;
			w.lds_id = sort_id;
			w.lds_n = NS;
			dsb_phase<true>(&w, &f, ph);
		} else if (ph == DSB_PH_DELA) {
			__shared__ uint64_t dela_lds[DSB_DELA_LDS_BYTES / 8];
			dsb_dela_lds(&w, dela_lds);
			dsb_phase<true>(&w, &f, ph);
		} else
			dsb_phase<true>(&w, &f, ph);
	}
#if DSB_HSET_POOL
	if (pool_wave)
		dsb_hpool_release(ix, ps, hs_tag, last_gen, dbg);
#endif
	__syncthreads();
	if (lane == 0) {
		if (active)
			dsb_state_save(&w, &f, sp);
		if (ph == DSB_PH_DELA) {
			dsb_read_out_t o;
			o.n_hit = w.n_hit;
			o.n_anchor = w.n_anc;
			o.fast = w.fast_classify;
			o.status = w.overflow;
			o.reached_update = w.reached_update;
			o.pad = 0;
			o.hit_off = 0;
			ro[r] = o;
			if (w.overflow)
				atomicAdd(n_overflow, 1u);
		}
	}
	if (DSB_TL && (dbg & DSB_DBG_TIMELINE) && lane == 0 && live && t < DSB_TL_STRIDE) {
		unsigned long long *e = gstats + DSB_N_STATS + 4ull * (PH * DSB_TL_STRIDE + t);
		e[0] = tl0;
		e[1] = __builtin_amdgcn_s_memrealtime();
		e[2] = r | ((unsigned long long)PH << 32) | ((unsigned long long)active << 40);
		e[3] = __builtin_amdgcn_s_getreg(4 | (31 << 11)) | /* HW_ID (wave, SIMD, CU, SE), XCC_ID */
		       ((unsigned long long)__builtin_amdgcn_s_getreg(20 | (31 << 11)) << 32);
	}
}

/* A phase of part A, one wave per workgroup: workgroup t runs read order[t] (the seeding phases:
 * 64 / DSB_SM_G reads per workgroup). */
template <int PH, int STATS>
__global__ __launch_bounds__(64, DSB_MINW_WAVE(PH)) void k_wave_phase(const dsb_dindex_t *__restrict__ ix, const uint32_t *__restrict__ len,
						    const uint64_t *__restrict__ ws_off, const uint32_t *__restrict__ scale,
						    uint8_t *__restrict__ ws, const uint32_t *__restrict__ order, uint32_t n,
						    dsb_read_out_t *__restrict__ ro, uint32_t *__restrict__ n_overflow,
						    unsigned long long *__restrict__ gstats, uint32_t dbg,
									      uint64_t tag)
{
	uint32_t lane = threadIdx.x;
	uint64_t st[DSB_ST_N];
	if (STATS == 1) /* work counters (per lane) */
		for (int k = 0; k < DSB_ST_N; k++) st[k] = 0;
	__shared__ uint64_t tmr_lds[DSB_ST_N];
	if (STATS == 2) { /* wave clocks (lane 0, LDS) */
		if (lane < DSB_ST_N)
			tmr_lds[lane] = 0;
		__syncthreads();
	}
	/* DSB_PH_LANES(PH) lanes per read: workgroup b runs reads order[b * 64 / G ...] */
	constexpr int G = DSB_PH_LANES(PH);
	uint32_t t = G == 64 ? blockIdx.x : blockIdx.x * (64 / G) + lane / G, t0 = blockIdx.x * (64 / G);
	if (t0 >= n)
		return;
	int live = t < n;
	wave_phase_read<PH, STATS>(ix, len, ws_off, scale, ws, order, live ? t : t0, live, ro, n_overflow, st, tmr_lds, gstats, dbg,
				   tag);
	if (STATS == 1)
		for (int k = 0; k < DSB_ST_N; k++)
			if (st[k])
				atomicAdd(gstats + DSB_ST_STRIDE * PH + k, (unsigned long long)st[k]);
	if (STATS == 2 && lane < DSB_ST_N && tmr_lds[lane])
		atomicAdd(gstats + DSB_ST_STRIDE * PH + lane, (unsigned long long)tmr_lds[lane]);
}


/* launch signature shared by the lane (k_phase) and wave (k_wave_phase) phase kernels */
typedef void (*dsb_phase_fn)(const dsb_dindex_t *, const uint32_t *, const uint64_t *, const uint32_t *, uint8_t *,
			     const uint32_t *, uint32_t, dsb_read_out_t *, uint32_t *, unsigned long long *, uint32_t,
			     uint64_t);

/*
 * The scoring of a heavy read (many chains of a long read: kernels.hip k_split) over several waves.
 * get_score_M2 (src/cly.c:2816-2844) scores the chains in order, and a chain's scoring can merge a
 * later chain into itself (combine_chain), which zeroes that chain: a later chain's run depends on
 * the earlier ones only through which chains are zeroed.  So:
 *   k_heavy_prep   (a wave per read)   the chains kept and their seed_con_hash (dsb_dela_prep);
 *   k_heavy_spec   (DSB_HEAVY_W waves per read)  every chain scored on its own as if no earlier
 *                  chain had merged anything: a private copy of the chain (dsb_read_ws.spec_ch),
 *                  merged chains only marked (spec_bits), its own sms buffer; w->hit is not written;
 *   k_heavy_fin    (a wave per read)   the chains in order: a chain zeroed by an accepted merge is
 *                  skipped (as in the reference); a chain whose speculative run merged only chains
 *                  that are still live took exactly the reference's path (each combine_chain call
 *                  accepts the first live match in list order, and the live set it ran against
 *                  differs from the true one only by chains it did not pick), so its result and
 *                  merges are applied; any other chain is scored again, in order, by this wave.
 *                  Then the rest of delete_small_score_rst part A (dsb_dela_post).
 * Scratch per read (host-laid out, dsb_heavy_bytes): DSB_HEAVY_MAX_HIT records, then a sms buffer
 * per wave.
 */
#define DSB_HEAVY_W 16
/* the DSB_HEAVY_W waves of a read read one read hash: it must be built before them (k_hash_lds), not
 * by each wave over the shared workspace — k_split sends only reads with dsb_hash_lds_read() here
 * (none when DSB_HASH_LDS is 0) */
#define DSB_HEAVY_MAX_HIT 400
/* launch signatures (kernels.hip takes the kernels from the scoring phase's unit, phase.hip) */
typedef void (*dsb_heavy_prep_fn)(const dsb_dindex_t *, const uint32_t *, const uint64_t *, const uint32_t *, uint8_t *,
				  const uint32_t *, uint32_t, uint32_t);
typedef void (*dsb_heavy_spec_fn)(const dsb_dindex_t *, const uint32_t *, const uint64_t *, const uint32_t *, uint8_t *,
				  const uint32_t *, uint32_t, uint8_t *, const uint64_t *, uint32_t);
typedef void (*dsb_heavy_fin_fn)(const dsb_dindex_t *, const uint32_t *, const uint64_t *, const uint32_t *, uint8_t *,
				 const uint32_t *, uint32_t, uint8_t *, const uint64_t *, dsb_read_out_t *, uint32_t *, uint32_t);
typedef struct {
	dsb_chain_t ch;         /* the chain after its speculative run (sum_score = its score) */
	uint32_t flags;         /* 1 scored, 2 the run overflowed (the finalising wave scores it again) */
	uint32_t pad;
	uint64_t bits[(DSB_HEAVY_MAX_HIT + 63) / 64]; /* chains it merged */
} dsb_heavy_rec;
DSB_HD uint64_t dsb_heavy_bytes(uint32_t L, uint32_t scale)
{
	dsb_caps_t cap = dsb_default_caps(L, scale);
	return dsb_al(sizeof(dsb_heavy_rec) * DSB_HEAVY_MAX_HIT) + DSB_HEAVY_W * dsb_al(sizeof(dsb_spd_t) * (uint64_t)cap.sms);
}

__device__ __forceinline__ void dsb_heavy_ws(const dsb_dindex_t *ix, const uint32_t *len, const uint64_t *ws_off,
					     const uint32_t *scale, uint8_t *ws, uint32_t r, dsb_read_ws *w, dsb_rflags_t *f,
					     dsb_rstate_t **sp, uint32_t dbg)
{
	uint32_t L = len[r];
	uint8_t *base = ws + ws_off[r];
	dsb_caps_t cap = dsb_default_caps(L, scale[r]);
	dsb_ws_layout lay = dsb_layout(L, cap);
	dsb_ws_init(w, ix, base, L, cap);
	*sp = (dsb_rstate_t *)(base + lay.state);
	dsb_state_load(w, f, *sp);
	w->dbg = dbg;
}

template <int V>
__global__ __launch_bounds__(64) void k_heavy_prep(const dsb_dindex_t *__restrict__ ix, const uint32_t *__restrict__ len,
						   const uint64_t *__restrict__ ws_off, const uint32_t *__restrict__ scale,
						   uint8_t *__restrict__ ws, const uint32_t *__restrict__ hl, uint32_t nh, uint32_t dbg)
{
	if (blockIdx.x >= nh)
		return;
	dsb_read_ws w;
	dsb_rflags_t f;
	dsb_rstate_t *sp;
	dsb_heavy_ws(ix, len, ws_off, scale, ws, hl[blockIdx.x], &w, &f, &sp, dbg);
	if (threadIdx.x == 0) { /* scalar work, one lane */
		dsb_dela_prep(&w);
		dsb_state_save(&w, &f, sp);
	}
}

template <int V>
__global__ __launch_bounds__(64, 4) void k_heavy_spec(const dsb_dindex_t *__restrict__ ix, const uint32_t *__restrict__ len,
								  const uint64_t *__restrict__ ws_off, const uint32_t *__restrict__ scale,
								  uint8_t *__restrict__ ws, const uint32_t *__restrict__ hl, uint32_t nh,
								  uint8_t *__restrict__ hs, const uint64_t *__restrict__ hs_off, uint32_t dbg)
{
	uint32_t h = blockIdx.x / DSB_HEAVY_W, part = blockIdx.x % DSB_HEAVY_W, lane = threadIdx.x;
	if (h >= nh)
		return;
	dsb_read_ws w;
	dsb_rflags_t f;
	dsb_rstate_t *sp;
	dsb_heavy_ws(ix, len, ws_off, scale, ws, hl[h], &w, &f, &sp, dbg);
	__shared__ uint64_t dela_lds[DSB_DELA_LDS_BYTES / 8];
	dsb_dela_lds(&w, dela_lds);
	dsb_heavy_rec *rec = (dsb_heavy_rec *)(hs + hs_off[h]);
	w.sms = (dsb_spd_t *)(hs + hs_off[h] + dsb_al(sizeof(dsb_heavy_rec) * DSB_HEAVY_MAX_HIT) +
			      part * dsb_al(sizeof(dsb_spd_t) * (uint64_t)w.cap.sms));
	int key_len = dsb_build_hash_table<true>(&w, (int)w.L); /* built by k_hash_lds: the key length only */
	for (uint32_t i = part; i < w.n_hit; i += DSB_HEAVY_W) {
		dsb_heavy_rec *rc = rec + i;
		if (lane == 0) {
			rc->ch = w.hit[i];
			rc->flags = 0;
		}
		if (lane < (DSB_HEAVY_MAX_HIT + 63) / 64)
			rc->bits[lane] = 0;
		__syncthreads();
		if (w.hit[i].sum_score == 0)
			continue; /* never scored (the reference skips it too) */
		w.spec_ch = &rc->ch;
		w.spec_bits = rc->bits;
		w.overflow = 0;
		int ok = dsb_score_chain<true>(&w, i, w.L, key_len);
		__syncthreads();
		if (lane == 0)
			rc->flags = ok ? 1u : 2u;
	}
}

template <int V>
__global__ __launch_bounds__(64, 4) void k_heavy_fin(const dsb_dindex_t *__restrict__ ix, const uint32_t *__restrict__ len,
								 const uint64_t *__restrict__ ws_off, const uint32_t *__restrict__ scale,
								 uint8_t *__restrict__ ws, const uint32_t *__restrict__ hl, uint32_t nh,
								 uint8_t *__restrict__ hs, const uint64_t *__restrict__ hs_off,
								 dsb_read_out_t *__restrict__ ro, uint32_t *__restrict__ n_overflow, uint32_t dbg)
{
	uint32_t h = blockIdx.x, lane = threadIdx.x;
	if (h >= nh)
		return;
	uint32_t r = hl[h];
	dsb_read_ws w;
	dsb_rflags_t f;
	dsb_rstate_t *sp;
	dsb_heavy_ws(ix, len, ws_off, scale, ws, r, &w, &f, &sp, dbg);
	__shared__ uint64_t dela_lds[DSB_DELA_LDS_BYTES / 8];
	dsb_dela_lds(&w, dela_lds);
	const dsb_heavy_rec *rec = (const dsb_heavy_rec *)(hs + hs_off[h]);
	int key_len = dsb_build_hash_table<true>(&w, (int)w.L);
	constexpr uint32_t NW = (DSB_HEAVY_MAX_HIT + 63) / 64;
	for (uint32_t i = 0; i < w.n_hit; i++) {
		if (w.hit[i].sum_score == 0)
			continue;
		const dsb_heavy_rec *rc = rec + i;
		/* valid: scored without overflow, and every chain it merged still live */
		uint64_t word = lane < NW ? rc->bits[lane] : 0;
		int bad = 0;
		for (uint64_t m = word; m; m &= m - 1)
			bad |= w.hit[lane * 64 + (uint32_t)__builtin_ctzll(m)].sum_score == 0;
		int valid = rc->flags == 1 && dsb_wballot(bad) == 0;
		if (valid) {
			__syncthreads();
			if (lane == 0)
				w.hit[i] = rc->ch;
			for (uint64_t m = word; m; m &= m - 1) { /* the merged chains, zeroed as dsb_comb_merge does */
				dsb_chain_t *c = w.hit + lane * 64 + (uint32_t)__builtin_ctzll(m);
				c->sum_score = 0;
				c->t_st = c->t_ed = c->q_st = c->q_ed = 0;
			}
			__syncthreads();
		} else if (!dsb_score_chain<true>(&w, i, w.L, key_len))
			break; /* overflow: the read is re-run (kernels.hip batch_run) */
	}
	if (!w.overflow)
		dsb_dela_post(&w);
	__syncthreads();
	if (lane == 0) {
		dsb_state_save(&w, &f, sp);
		dsb_read_out_t o;
		o.n_hit = w.n_hit;
		o.n_anchor = w.n_anc;
		o.fast = w.fast_classify;
		o.status = w.overflow;
		o.reached_update = w.reached_update;
		o.pad = 0;
		o.hit_off = 0;
		ro[r] = o;
		if (w.overflow)
			atomicAdd(n_overflow, 1u);
	}
}

#endif
