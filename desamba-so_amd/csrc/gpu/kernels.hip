/*
 * kernels.hip — MI355X (gfx950) kernels of the deSAMBA classify path + the launch shim
 * behind dsb_gpu.h.
 *
 * Pipeline per chunk of reads (input order; chunk size set by the HBM workspace budget):
 *   k_encode   one workgroup per read: ASCII -> 2-bit forward + reverse complement into the
 *              read's workspace, guard bytes (src/cly.c:1245-1254)
 *   k_seed     one wavefront per 64 consecutive k-mer positions of one strand: rolling l_ek-mer,
 *              low-complexity filter, two-table Bloom probe (src/cly.c:359-397, 951-967),
 *              __ballot -> one 64-bit exist word per wave (coalesced store)
 *   k_classA   one lane per read (reads sorted by length): islands, fast/slow FM search,
 *              map_seed, chaining, SDP rescoring (src/cly.c:3059-3124, 2878-2952)
 *   (host)     max_read_l carry = prefix max over reads that reached cly.c:2953 (H2)
 *   k_classB   one lane per read: length-class filter, MEM-score sort, primary detection;
 *              hit records compacted with one atomic bump per read
 * Reads whose dynamic vectors overflow are re-run (encode/seed/A) with 8x workspace.
 */
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <vector>
#include <atomic>
#include <algorithm>
#include "dsb_ws.h"
#include "dsb_gpu.h"

#include "dsb_kern.h"
#include "dsb_debug.h"
#ifndef DSB_TEST_HOOKS /* 1: the test build lib/libdesamba_test.so (the env-reachable test hooks below) */
#define DSB_TEST_HOOKS 0
#endif
static_assert(DSB_ST_N <= DSB_ST_STRIDE, "work counters per phase");

#define HIP_OK(x)                                                                                    \
	do {                                                                                         \
		hipError_t e_ = (x);                                                                 \
		if (e_ != hipSuccess) {                                                              \
			snprintf(err, errn, "%s failed: %s (%s:%d)", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
			return -1;                                                                   \
		}                                                                                    \
	} while (0)

/* ------------------------------------------------------------------ kernels */
__global__ __launch_bounds__(256) void k_encode(const uint8_t *__restrict__ seq, const uint64_t *__restrict__ seq_off,
						 const uint32_t *__restrict__ len, const uint64_t *__restrict__ ws_off,
						 uint8_t *__restrict__ ws, const uint32_t *__restrict__ sel, uint32_t n)
{
	uint32_t i = blockIdx.x;
	if (i >= n)
		return;
	uint32_t r = sel ? sel[i] : i;
	uint32_t L = len[r];
	const uint8_t *s = seq + seq_off[r];
	uint8_t *bin = ws + ws_off[r] + DSB_BIN_GUARD; /* dsb_layout(...).bin == 0 */
	for (uint32_t k = threadIdx.x; k < L; k += blockDim.x) {
		uint8_t b = dsb_cly_bit(s[k]);
		bin[k] = b;
		bin[2 * L - 1 - k] = 3 - b;
	}
	if (threadIdx.x < DSB_BIN_GUARD) {
		int k = DSB_BIN_GUARD - threadIdx.x; /* bin[-k] */
		uint8_t v = DSB_HEAP_PERTURB;
		if (k <= 8)
			v = (uint8_t)(dsb_chunk_header(L) >> (8 * (8 - k)));
		bin[-k] = v;
	}
	for (uint32_t k = threadIdx.x; k < DSB_BIN_TAIL; k += blockDim.x)
		bin[2ull * L + k] = DSB_HEAP_PERTURB;
}

/* one wave = 64 k-mer positions of one strand of one read */
__global__ __launch_bounds__(256) void k_seed(const dsb_dindex_t *__restrict__ ix, const uint32_t *__restrict__ len,
					       const uint64_t *__restrict__ ws_off, uint8_t *__restrict__ ws,
					       const uint64_t *__restrict__ word_off, const uint32_t *__restrict__ sel,
					       uint32_t n, uint64_t total_waves, unsigned long long *__restrict__ gstats)
{
	uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
	uint32_t lane = threadIdx.x & 63;
	if (wave >= total_waves)
		return;
	/* binary search: word_off[i] <= wave < word_off[i+1] */
	uint32_t lo = 0, hi = n;
	while (hi - lo > 1) {
		uint32_t mid = (lo + hi) >> 1;
		if (word_off[mid] <= wave) lo = mid; else hi = mid;
	}
	uint32_t r = sel ? sel[lo] : lo;
	uint32_t L = len[r];
	int l_ek = ix->l_ek;
	uint32_t lk = L - l_ek + 1;
	uint32_t nw = (lk + 63) >> 6;
	uint64_t wi = wave - word_off[lo];
	uint32_t strand = wi >= nw;
	uint32_t word = (uint32_t)(strand ? wi - nw : wi);
	uint8_t *base = ws + ws_off[r];
	const uint8_t *bin = base + DSB_BIN_GUARD + strand * L;
	dsb_ws_layout lay = dsb_layout(L, dsb_default_caps(L, DSB_SCALE_UNIT)); /* ex offsets do not depend on caps */
	uint64_t *ex = (uint64_t *)(base + (strand ? lay.exR : lay.exF));
	uint32_t *pre = (uint32_t *)(base + lay.pre) + (strand ? L : 0);
	(void)pre;
	uint32_t k = word * 64 + lane;
	int e = 0, p1 = 0, p2 = 0;
	if (k < lk) {
		uint64_t km = dsb_kmer_at(bin + k, l_ek, ix->single_base_max);
		if (DSB_SEED_PRE)
			pre[k] = (uint32_t)(km & DSB_PRE_IDX_MASK); /* the seeding's 13-mer prefix (fast / slow J step) */
		if (gstats) { /* work counters: first / second Bloom probes (get_exist_kmer, src/cly.c:951-967) */
			p1 = km != 0;
			p2 = p1 && ((dsb_gld(ix->ek0 + ((dsb_hash64_1(km) & ix->ek_mask) >> 3)) >>
				     (7 - (dsb_hash64_1(km) & ix->ek_mask & 0x7))) & 1);
		}
		e = dsb_exist_kmer(ix, km);
	}
	uint64_t bits = __ballot(e);
	if (lane == 0)
		ex[word] = bits;
	if (gstats) {
		uint64_t b1 = __ballot(p1), b2 = __ballot(p2);
		if (lane == 0) {
			atomicAdd(gstats + DSB_STATS_SEED + DSB_ST_EK1, (unsigned long long)__builtin_popcountll(b1));
			atomicAdd(gstats + DSB_STATS_SEED + DSB_ST_EK2, (unsigned long long)__builtin_popcountll(b2));
		}
	}
}

template <bool STATS>
__global__ __launch_bounds__(64) void k_classB(const dsb_dindex_t *__restrict__ ix, const uint32_t *__restrict__ len,
						const uint64_t *__restrict__ ws_off, const uint32_t *__restrict__ scale,
						uint8_t *__restrict__ ws, const uint32_t *__restrict__ order, uint32_t n,
						const int32_t *__restrict__ mrl, dsb_read_out_t *__restrict__ ro,
						dsb_hit_out_t *__restrict__ hits_out, uint32_t *__restrict__ hit_cursor,
						uint32_t *__restrict__ hit_off, uint32_t *__restrict__ tid_out,
						unsigned long long *__restrict__ gstats)
{
	uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
	if (t >= n)
		return;
	uint32_t r = order[t];
	uint32_t L = len[r];
	dsb_read_ws w;
	dsb_ws_init(&w, ix, ws + ws_off[r], L, dsb_default_caps(L, scale[r]));
	dsb_read_out_t o = ro[r];
	w.n_hit = o.n_hit;
	w.n_anc = o.n_anchor;
	w.fast_classify = o.fast;
	w.overflow = o.status;
	w.reached_update = o.reached_update;
	uint64_t st[DSB_ST_N];
	if (STATS) {
		for (int k = 0; k < DSB_ST_N; k++) st[k] = 0;
		w.stats = st;
	}
	/* hits are staged in the read's own hit_tmp region, then compacted */
	dsb_hit_out_t *stage = (dsb_hit_out_t *)w.hit_tmp;
	dsb_classify_B(&w, mrl[r], &o, stage, DSB_MAX_HITS);
	uint32_t off = atomicAdd(hit_cursor, o.n_hit);
	for (uint32_t k = 0; k < o.n_hit; k++)
		hits_out[off + k] = stage[k];
	hit_off[r] = off;
	o.hit_off = off;
	ro[r] = o;
	/* per-read taxon (meta_analysis' rule); an index loaded without a taxonomy reports 0 */
	tid_out[r] = (ix->ref_tid && ix->p_tid) ? dsb_read_taxon(stage, o.n_hit, ix->ref_tid, ix->p_tid, ix->max_tid) : 0;
	if (STATS)
		for (int k = 0; k < DSB_ST_N; k++)
			atomicAdd(gstats + DSB_STATS_B + k, (unsigned long long)st[k]);
}

/* per-taxon weights (meta_analysis node_count, reference src/cly_mt.c:1352-1362) */
__global__ __launch_bounds__(256) void k_taxon_count(const uint32_t *__restrict__ tid, const uint32_t *__restrict__ weight,
						     uint64_t n, unsigned long long *__restrict__ counts)
{
	uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (i < n)
		atomicAdd(counts + tid[i], weight ? (unsigned long long)weight[i] : 1ull);
}

/* dst[idx[i]] = src[i] (the per-read taxa of the deferred re-runs into the batch's table) */
__global__ __launch_bounds__(256) void k_scatter_u32(uint32_t *__restrict__ dst, const uint32_t *__restrict__ idx,
						     const uint32_t *__restrict__ src, uint32_t n)
{
	uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i < n)
		dst[idx[i]] = src[i];
}

#if DSB_TEST_HOOKS /* device self-tests: the test build only (lib/libdesamba_test.so) */
/* The merge-sort orders the classifier depends on, one array per lane:
 * which 0 chain_cmp_by_pos, 1 chain_cmp_by_MEM_score, 2 chain_cmp_by_score, 3 anchors
 * (Anchor_cmp_by_chr_ID_and_pos), 4 MEM_rst by match_len.  Output: permutation in idx. */
DSB_HD void dsb_selftest_one(dsb_chain_t *H, dsb_chain_t *T, uint32_t *idx, uint32_t *tmpi, uint32_t n, int which)
{
	for (uint32_t k = 0; k < n; k++) idx[k] = k;
	if (which == 0)
		dsb_msort(idx, tmpi, n, [H](uint32_t a, uint32_t b) -> int { return dsb_chain_cmp_by_pos(H + a, H + b); });
	else if (which == 1)
		dsb_msort(idx, tmpi, n, [H](uint32_t a, uint32_t b) -> int { return dsb_chain_cmp_by_MEM_score(H + a, H + b); });
	else if (which == 2)
		dsb_msort(idx, tmpi, n, [H](uint32_t a, uint32_t b) -> int { return dsb_chain_cmp_by_score(H + a, H + b); });
	else if (which == 3) {
		dsb_anchor_t *A = (dsb_anchor_t *)T; /* n anchors fit: sizeof(anchor) <= sizeof(chain) */
		for (uint32_t k = 0; k < n; k++) {
			dsb_anchor_t a;
			memset(&a, 0, sizeof(a));
			a.ref_ID = H[k].ref_ID; a.direction = H[k].with_top_anchor; a.ref_offset = H[k].t_st;
			A[k] = a;
		}
		dsb_msort(idx, tmpi, n, [A](uint32_t a, uint32_t b) -> int { return dsb_anchor_cmp(A + a, A + b); });
	} else {
		dsb_mem_t *M = (dsb_mem_t *)T;
		for (uint32_t k = 0; k < n; k++) {
			dsb_mem_t m;
			memset(&m, 0, sizeof(m));
			m.match_len = (int)H[k].sum_score + (int)H[k].t_st;
			M[k] = m;
		}
		dsb_msort(idx, tmpi, n, [M](uint32_t a, uint32_t b) -> int { return dsb_mem_cmp(M + a, M + b); });
	}
}

__global__ void k_selftest_sort(dsb_chain_t *chains, dsb_chain_t *tmp, uint32_t *idx, uint32_t *tmpi, uint32_t n,
				 uint32_t n_arrays, int which)
{
	uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
	if (t >= n_arrays)
		return;
	size_t o = (size_t)t * n;
	dsb_selftest_one(chains + o, tmp + o, idx + o, tmpi + o, n, which);
}
#endif

/* ------------------------------------------------------------------ host side */
#define DSB_BOUNCE_BYTES ((size_t)32 << 20) /* pinned bounce buffer per context (copy_wait_g) */
/* device buffer that grows (persistent per device context; calls are serialised) */
struct dbuf {
	void *p = nullptr;
	size_t cap = 0;
	int ensure(size_t n, char *err, size_t errn)
	{
		if (n <= cap)
			return 0;
		if (p)
			hipFree(p);
		p = nullptr;
		cap = 0;
		size_t c = n + n / 8 + 4096;
		HIP_OK(hipMalloc(&p, c));
		cap = c;
		return 0;
	}
	void release()
	{
		if (p)
			hipFree(p);
		p = nullptr;
		cap = 0;
	}
	template <typename T> T *as() const { return (T *)p; }
	~dbuf() { release(); }
};

struct dsb_gpu_batch;
struct dsb_gpu_dev {
	int device;
	int slot;                /* index in dsb_index.gpus */
	hipStream_t stream;
	hipStream_t stream2;     /* scoring of the reads that skip slow seeding, beside the slow phases */
	hipStream_t stream3 = nullptr; /* the heavy reads' scoring, beside both (run_split, DSB_HEAVY_SPEC) */
	int prio_hi = 0;
	hipEvent_t ev_a, ev_b, ev_fork, ev_r0, ev_r1, ev_h0, ev_h1;
	pthread_mutex_t mu;
	dsb_dindex_t h;          /* host copy holding device pointers */
	dsb_dindex_t *d;         /* device copy */
	std::vector<void *> allocs;
	dbuf ws_off, scale, ws, wsr, order, word_off, ro, mrl, hits, hit_off, cnt, stats, sel, wo2, slist, rlist, cnt2;
	dbuf vlen, vso, vidx, vtid; /* the deferred overflow re-runs of a batch (batch_run) */
	dbuf hscr, hoff;         /* the heavy reads' scoring scratch and its per-read offsets (run_split) */
	dbuf blist;              /* the scoring reads by cost class, DSB_COST_CLASSES lists of a chunk each (run_split) */
	dbuf cbound;             /* a lower bound of the carried max_read_l before each read of a chunk (k_carry_bound) */
	hipEvent_t evh[2][2];    /* k_hash_lds before the scoring launch, per stream (launch_phase) */
	int evh_used[2] = {0, 0};
	/* streamed batches (read_classify pipeline): uploads on their own stream through pinned
	 * staging, under their own lock, beside the kernels of the batch before */
	hipStream_t cstream;
	pthread_mutex_t umu;
	void *pin[2] = {nullptr, nullptr};
	size_t pin_cap[2] = {0, 0};
	void *bounce = nullptr;   /* pinned bounce buffer of the waited copies (copy_wait_g), under the run lock */
	size_t bounce_cap = 0;
	hipEvent_t pin_ev[2];
	int pin_used[2] = {0, 0};
	int pin_next = 0;
	std::vector<dsb_gpu_batch *> spare; /* recycled batches: their device buffers are reused, never freed mid-pipeline */
	int n_ctx = 1;           /* contexts on this GPU (they split its workspace budget) */
	size_t pipe_budget = 0;  /* chunk workspace budget of a streamed batch (dsb_gpu_fit_contexts) */
};

template <typename T>
static int upload(dsb_gpu_dev *g, const T *src, size_t count, const T **dst, char *err, size_t errn)
{
	void *p = nullptr;
	size_t bytes = count * sizeof(T);
	HIP_OK(hipMalloc(&p, bytes ? bytes : 16));
	if (bytes)
		HIP_OK(hipMemcpy(p, src, bytes, hipMemcpyHostToDevice));
	g->allocs.push_back(p);
	*dst = (const T *)p;
	return 0;
}

extern "C" int dsb_gpu_device_count(void)
{
	int n = 0;
	if (hipGetDeviceCount(&n) != hipSuccess)
		return 0;
	return n;
}

/* the XCC ids (HW_REG_XCC_ID) the waves of this device report, as a bit set */
__global__ __launch_bounds__(64) void k_xcc_probe(uint32_t *seen)
{
	if (threadIdx.x == 0)
		atomicOr(seen, 1u << ((uint32_t)__builtin_amdgcn_s_getreg(20 | (31 << 11)) & 0x1fu));
}

#if DSB_TEST_HOOKS /* tests: the fenced sp_set pool hand-over on any device */
#define DSB_TEST_POOL_FENCED() (getenv("DSB_TEST_POOL_FENCED") != NULL)
#else
#define DSB_TEST_POOL_FENCED() 0
#endif

static int xcc_ids_seen(uint32_t *out, char *err, size_t errn)
{
	uint32_t *d = nullptr;
	HIP_OK(hipMalloc(&d, 4));
	HIP_OK(hipMemset(d, 0, 4));
	k_xcc_probe<<<1 << 15, 64>>>(d); /* 32k one-wave workgroups: every CU of every XCC */
	HIP_OK(hipGetLastError());
	HIP_OK(hipMemcpy(out, d, 4, hipMemcpyDeviceToHost));
	HIP_OK(hipFree(d));
	return 0;
}

/* A device context: streams, events, workspace, and the index tables — its own upload, or
 * those of `share`, an earlier context on the same GPU (several contexts per GPU let batches of
 * one read_classify call run their kernels side by side, each context with its own workspace). */
static int dev_init(dsb_index *ix, int device, const dsb_gpu_dev *share, dsb_gpu_dev **out, char *err, size_t errn)
{
	HIP_OK(hipSetDevice(device));
	dsb_gpu_dev *g = new dsb_gpu_dev();
	*out = g;
	g->device = device;
	pthread_mutex_init(&g->mu, NULL);
	pthread_mutex_init(&g->umu, NULL);
	/* default priority: at the highest one the slow reads' chain was no faster (r06_c2l18/ab_stream_prio.txt) */
	HIP_OK(hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking));
	HIP_OK(hipStreamCreateWithFlags(&g->cstream, hipStreamNonBlocking));
	for (int k = 0; k < 2; k++)
		HIP_OK(hipEventCreateWithFlags(&g->pin_ev[k], hipEventDisableTiming));
	HIP_OK(hipEventCreate(&g->ev_a));
	HIP_OK(hipEventCreate(&g->ev_b));
	/* the pinned bounce buffer of the waited copies (copy_wait_g), once per context */
	HIP_OK(hipHostMalloc(&g->bounce, DSB_BOUNCE_BYTES, hipHostMallocDefault));
	g->bounce_cap = DSB_BOUNCE_BYTES;
	{ /* the split-off scoring yields to the slow phases */
		int least = 0, greatest = 0;
		HIP_OK(hipDeviceGetStreamPriorityRange(&least, &greatest));
		HIP_OK(hipStreamCreateWithPriority(&g->stream2, hipStreamNonBlocking, least));
		g->prio_hi = greatest; /* stream3 is created on first use (run_split, DSB_HEAVY_SPEC) */
	}
	HIP_OK(hipEventCreate(&g->ev_h0));
	HIP_OK(hipEventCreate(&g->ev_h1));
	HIP_OK(hipEventCreate(&g->ev_fork));
	HIP_OK(hipEventCreate(&g->ev_r0));
	HIP_OK(hipEventCreate(&g->ev_r1));
	for (int k = 0; k < 2; k++)
		for (int e = 0; e < 2; e++)
			HIP_OK(hipEventCreate(&g->evh[k][e]));
	if (share) { /* read-only tables: one copy per GPU */
		g->h = share->h;
		g->d = share->d;
		return 0;
	}
	{ /* the HBM the tables and the seeding pool take, against what is free: a clear error now
	   * rather than a failed allocation halfway through the upload */
		size_t need = ((size_t)ix->n_occ_line + 1) * DSB_OCC_LINE_U64 * 8 + ix->n_occ_super * 32 +
			      (((size_t)1 << 26) + 1) * 8 + ix->sa_size * 8 + 2 * ix->ek_size + (ix->n_uni + 2) * 8 +
			      ix->ref_bin_padded + 16 * ix->n_ref + (ix->n_rp + 64) * 8 + 4 * (ix->n_ref + ix->max_tid + 2) +
			      ((size_t)8 * DSB_HSET_WAVE_U64 + 12) * 8192 * (DSB_HSET_POOL ? 1 : 0) + ((size_t)256 << 20);
		size_t fr = 0, tot = 0;
		HIP_OK(hipMemGetInfo(&fr, &tot));
		if (fr < need) {
			snprintf(err, errn, "the index needs %.2f GB of HBM on device %d, %.2f GB of %.2f GB are free "
				 "(another index or another user of the GPU holds the rest)", need / 1e9, device, fr / 1e9, tot / 1e9);
			return -1;
		}
	}
	dsb_dindex_t &h = g->h;
	memset(&h, 0, sizeof(h));
	/* occ lines (128 B per 256 BWT symbols, re-laid out by the loader) + one zero line */
	if (upload(g, ix->occ, (ix->n_occ_line + 1) * DSB_OCC_LINE_U64, &h.occ, err, errn)) return -1;
	h.n_occ_line = ix->n_occ_line;
	if (upload(g, ix->occ_super, ix->n_occ_super * 4, &h.occ_super, err, errn)) return -1;
	memcpy(h.dollar_row, ix->dollar_row, sizeof(h.dollar_row));
	h.n_dollar = ix->n_dollar;
	memcpy(h.rank, ix->rank, sizeof(h.rank));
	if (upload(g, ix->hash_index, (1ull << 26) + 1, &h.hash_index, err, errn)) return -1;
	if (upload(g, ix->sa, ix->sa_size, &h.sa, err, errn)) return -1;
	h.sa_size = ix->sa_size;
	h.dollor_pos = ix->dollor_pos;
	if (upload(g, ix->ek0, ix->ek_size, &h.ek0, err, errn)) return -1;
	if (upload(g, ix->ek1, ix->ek_size, &h.ek1, err, errn)) return -1;
	h.ek_size = ix->ek_size;
	h.ek_mask = ix->ek_mask;
	h.l_ek = ix->l_ek;
	h.single_base_max = ix->single_base_max;
	if (upload(g, ix->uni, ix->n_uni + 2, &h.uni, err, errn)) return -1;
	h.n_uni = ix->n_uni;
	if (upload(g, ix->ref_bin, ix->ref_bin_padded, &h.ref_bin, err, errn)) return -1;
	h.ref_bin_n = ix->ref_bin_n;
	h.ref_bin_padded = ix->ref_bin_padded;
	if (upload(g, ix->ref_seq_offset, ix->n_ref, &h.ref_seq_offset, err, errn)) return -1;
	if (upload(g, ix->ref_seq_l, ix->n_ref, &h.ref_seq_l, err, errn)) return -1;
	h.n_ref = ix->n_ref;
	if (upload(g, ix->r_p, ix->n_rp + 64, &h.r_p, err, errn)) return -1;
	h.n_rp = ix->n_rp;
	if (upload(g, ix->Q_MEM, (size_t)DSB_Q_MEM_PAD, &h.Q_MEM, err, errn)) return -1;
	if (upload(g, ix->Q_LV, (size_t)DSB_LV_DIM * DSB_LV_DIM, &h.Q_LV, err, errn)) return -1;
	h.filter_min_length = ix->filter_min_length;
	h.filter_min_score = ix->filter_min_score;
	h.filter_min_score_LV3 = ix->filter_min_score_LV3;
	if (ix->ref_tid && ix->p_tid) { /* taxonomy (per-read taxa in classB) */
		if (upload(g, ix->ref_tid, ix->n_ref + 1, &h.ref_tid, err, errn)) return -1;
		if (upload(g, ix->p_tid, ix->max_tid + 1, &h.p_tid, err, errn)) return -1;
		h.max_tid = ix->max_tid;
	}
	if (DSB_HSET_POOL) {
		/* the seeding sp_set pool, shared by the contexts on this GPU: a partition per XCD, one
		 * set per wave the XCD can hold (32 per CU), rounded up to a power of two; zero-filled, so
		 * no slot matches a tag before its first writer (generation 0 is never used) */
		hipDeviceProp_t prop;
		HIP_OK(hipGetDeviceProperties(&prop, device));
		int nx = 0, fenced = 0;
		uint32_t seen = 0;
		if (hipDeviceGetAttribute(&nx, hipDeviceAttributeNumberOfXccs, device) != hipSuccess || nx < 1)
			nx = 0;
		if (xcc_ids_seen(&seen, err, errn))
			return -1;
		/* the partition of a wave is its XCC id modulo hpool_nx: correct only when the ids are
		 * exactly 0..nx-1 (one L2 per partition); otherwise one partition with fenced hand-overs */
		if (nx < 1 || nx > 16 || seen != (nx >= 32 ? ~0u : (1u << nx) - 1) || DSB_TEST_POOL_FENCED()) {
			fprintf(stderr, "[dsb] device %d: %d XCCs reported, XCC ids seen %#x: sp_set pool hand-over fenced\n",
				device, nx, seen);
			nx = 1;
			fenced = 1;
		}
		uint64_t per_cu = DSB_MAX(32u, (uint32_t)prop.maxThreadsPerMultiProcessor / 64u);
		uint64_t waves = ((uint64_t)prop.multiProcessorCount + nx - 1) / nx * per_cu, part = 1;
		while (part < waves)
			part <<= 1;
		uint64_t n = part * (uint64_t)nx;
		void *p;
		HIP_OK(hipMalloc(&p, 8 * DSB_HSET_WAVE_U64 * n));
		HIP_OK(hipMemset(p, 0, 8 * DSB_HSET_WAVE_U64 * n));
		g->allocs.push_back(p);
		h.hpool = (uint64_t *)p;
		HIP_OK(hipMalloc(&p, 12 * n));
		HIP_OK(hipMemset(p, 0, 12 * n));
		g->allocs.push_back(p);
		h.hpool_gen = (uint64_t *)p;
		h.hpool_own = (uint32_t *)((uint8_t *)p + 8 * n);
		h.hpool_part = (uint32_t)part;
		h.hpool_nx = (uint32_t)nx;
		h.hpool_fenced = (uint32_t)fenced;
	}
	const dsb_dindex_t *dptr;
	if (upload(g, &h, 1, &dptr, err, errn)) return -1;
	g->d = (dsb_dindex_t *)dptr;
	return 0;
}

static void dev_free(dsb_gpu_dev *g);

/* The devices the index is replicated on: DSB_DEVICES ("all" or a comma list), else
 * DSB_DEVICE, else the current HIP device; `device` >= 0 forces that one. */
extern "C" int dsb_gpu_init(dsb_index *ix, int device, char *err, size_t errn)
{
	int ndev = 0;
	if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
		snprintf(err, errn, "no HIP device visible: the deSAMBA MI355X classify path has no CPU fallback");
		return -1;
	}
	int devs[DSB_MAX_GPUS], n = 0;
	const char *list = getenv("DSB_DEVICES");
	if (device < 0 && list && *list) {
		if (!strcmp(list, "all")) {
			for (int d = 0; d < ndev && n < DSB_MAX_GPUS; d++)
				devs[n++] = d;
		} else {
			for (const char *q = list; *q && n < DSB_MAX_GPUS;) {
				char *e;
				long d = strtol(q, &e, 10);
				if (e == q)
					break;
				devs[n++] = (int)d;
				q = *e == ',' ? e + 1 : e;
			}
		}
	}
	if (n == 0) {
		if (device < 0) {
			const char *e = getenv("DSB_DEVICE");
			if (e)
				device = atoi(e);
			else
				HIP_OK(hipGetDevice(&device));
		}
		devs[n++] = device;
	}
	for (int k = 0; k < n; k++)
		if (devs[k] < 0 || devs[k] >= ndev) {
			snprintf(err, errn, "device %d out of range (%d visible)", devs[k], ndev);
			return -1;
		}
	/* DSB_GPU_CONTEXTS (default 2): contexts per listed GPU, sharing its copy of the index, so
	 * that consecutive batches of a read_classify call overlap on the GPU and fill each other's
	 * phase-kernel tails (the batch API uses the first context only) */
	int per = 2;
	if (const char *e = getenv("DSB_GPU_CONTEXTS"))
		per = DSB_MAX(1, DSB_MIN(8, atoi(e)));
	if (per > 1) {
		int m = 0, d2[DSB_MAX_GPUS];
		for (int k = 0; k < n; k++)
			for (int c = 0; c < per && m < DSB_MAX_GPUS; c++)
				d2[m++] = devs[k];
		memcpy(devs, d2, sizeof(int) * m);
		n = m;
	}
	for (int k = 0; k < n; k++) {
		dsb_gpu_dev *g = nullptr;
		const dsb_gpu_dev *share = nullptr;
		for (int j = 0; j < k && !share; j++)
			if (((dsb_gpu_dev *)ix->gpus[j])->device == devs[k])
				share = (const dsb_gpu_dev *)ix->gpus[j];
		if (dev_init(ix, devs[k], share, &g, err, errn)) {
			if (g)
				dev_free(g);
			for (int j = 0; j < k; j++)
				dev_free((dsb_gpu_dev *)ix->gpus[j]);
			ix->n_gpu = 0;
			ix->gpu = NULL;
			return -1;
		}
		g->slot = k;
		ix->gpus[k] = g;
	}
	ix->n_gpu = n;
	ix->gpu = ix->gpus[0];
	for (int k = 0; k < n; k++) {
		dsb_gpu_dev *g = (dsb_gpu_dev *)ix->gpus[k];
		g->n_ctx = 0;
		for (int j = 0; j < n; j++)
			g->n_ctx += ((dsb_gpu_dev *)ix->gpus[j])->device == g->device;
	}
	return 0;
}

static void batch_destroy(dsb_gpu_batch *b);

static void dev_free(dsb_gpu_dev *g)
{
	hipSetDevice(g->device);
	hipDeviceSynchronize();
	for (dsb_gpu_batch *b : g->spare)
		batch_destroy(b);
	g->spare.clear();
	for (int k = 0; k < 2; k++) {
		if (g->pin[k])
			hipHostFree(g->pin[k]);
		hipEventDestroy(g->pin_ev[k]);
	}
	if (g->bounce)
		hipHostFree(g->bounce);
	hipStreamDestroy(g->cstream);
	pthread_mutex_destroy(&g->umu);
	for (void *p : g->allocs)
		hipFree(p);
	dbuf *bs[] = {&g->ws_off, &g->scale, &g->ws, &g->wsr, &g->order, &g->word_off, &g->ro, &g->mrl, &g->hits,
		      &g->hit_off, &g->cnt, &g->stats, &g->sel, &g->wo2, &g->slist, &g->rlist, &g->cnt2, &g->hscr, &g->hoff, &g->blist, &g->cbound};
	for (dbuf *b : bs)
		b->release();
	hipEventDestroy(g->ev_a);
	hipEventDestroy(g->ev_b);
	hipEventDestroy(g->ev_fork);
	hipEventDestroy(g->ev_r0);
	hipEventDestroy(g->ev_r1);
	hipEventDestroy(g->ev_h0);
	hipEventDestroy(g->ev_h1);
	for (int k = 0; k < 2; k++)
		for (int e = 0; e < 2; e++)
			hipEventDestroy(g->evh[k][e]);
	hipStreamDestroy(g->stream2);
	if (g->stream3)
		hipStreamDestroy(g->stream3);
	hipStreamDestroy(g->stream);
	pthread_mutex_destroy(&g->mu);
	delete g;
}

extern "C" void dsb_gpu_free(dsb_index *ix)
{
	for (int k = 0; k < ix->n_gpu; k++)
		if (ix->gpus[k])
			dev_free((dsb_gpu_dev *)ix->gpus[k]);
	ix->n_gpu = 0;
	ix->gpu = NULL;
}

extern "C" int dsb_gpu_n_devices(const dsb_index *ix) { return ix->n_gpu; }
extern "C" int dsb_gpu_device_id(const dsb_index *ix, int slot)
{
	return slot >= 0 && slot < ix->n_gpu ? ((dsb_gpu_dev *)ix->gpus[slot])->device : -1;
}

static double now_ms(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec * 1e3 + ts.tv_nsec / 1e6;
}

/* the phase kernels live in their own translation units (phase.hip, one per phase) */
extern "C" {
dsb_phase_fn dsb_phase_kernel_0(int wave, int stats);
dsb_phase_fn dsb_phase_kernel_1(int wave, int stats);
dsb_phase_fn dsb_phase_kernel_2(int wave, int stats);
dsb_phase_fn dsb_phase_kernel_3(int wave, int stats);
dsb_phase_fn dsb_phase_kernel_4(int wave, int stats);
dsb_phase_fn dsb_phase_kernel_5(int wave, int stats);
dsb_phase_fn dsb_phase_kernel_6(int wave, int stats);
dsb_phase_fn dsb_phase_kernel_7(int wave, int stats);
dsb_phase_fn dsb_phase_kernel_8(int wave, int stats);
}
static_assert(DSB_PH_N == 9, "phase dispatch table");
static dsb_phase_fn phase_kernel_at(int ph, int wave, int stats)
{
	static dsb_phase_fn (*const get[DSB_PH_N])(int, int) = {
		dsb_phase_kernel_0, dsb_phase_kernel_1, dsb_phase_kernel_2, dsb_phase_kernel_3, dsb_phase_kernel_4,
		dsb_phase_kernel_5, dsb_phase_kernel_6, dsb_phase_kernel_7, dsb_phase_kernel_8};
	return get[ph](wave, stats);
}

static float ev_ms(dsb_gpu_dev *g)
{
	hipEventRecord(g->ev_b, g->stream);
	hipEventSynchronize(g->ev_b);
	float ms = 0;
	hipEventElapsedTime(&ms, g->ev_a, g->ev_b);
	return ms;
}

/* workspace budget for one chunk of reads: most of the HBM left after the index (the
 * workspace already held by this device counts as available) */
static size_t ws_budget(const dsb_gpu_dev *g, int share)
{
	const char *e = getenv("DSB_WS_BUDGET_MB");
	if (e)
		return (size_t)atoll(e) << 20;
	size_t fr = 0, tot = 0;
	if (hipMemGetInfo(&fr, &tot) != hipSuccess)
		return (size_t)8 << 30;
	/* the rest: overflow re-runs (retry buffer), result buffers, streams; the contexts of a GPU
	 * that run the batches of one read_classify call side by side split it (share = their
	 * number).  Fewer, larger chunks pay fewer phase-kernel tails and chunk turnarounds: on the C2
	 * proxy (1M reads) a 192 GB budget (0.7 of free HBM) made 9 chunks, 250 GB 7 chunks:
	 * 650.6k -> 694.4k reads/s (profiles/r04_k). */
	if (share > 1 && g->pipe_budget)
		return g->pipe_budget;
	size_t b = (size_t)((double)(fr + g->ws.cap) * 0.88 / share);
	size_t cap = (size_t)250 << 30;
	return b < cap ? b : cap;
}

/* Before a streamed read_classify call: split the HBM the contexts of each GPU can use for chunk
 * workspaces evenly between them.  A single-batch call may have grown one context's workspace to
 * most of the GPU (ws_budget with share 1); left alone, the other contexts of that GPU would get
 * chunks sized to what is left, and the streamed batches would run in many small chunks (C2 proxy,
 * 100k reads: 326k -> 40k reads/s).  A workspace larger than its share is freed here, under its
 * context's run lock (try-locks: a GPU with a call in flight is left as that call fitted it),
 * and the other buffers a batch of max_reads reads needs are sized here (the workspace itself
 * grows with the batches, by doubling: pre-sizing it to the share held ~90% of the HBM for every
 * loaded index, also for small inputs). */
extern "C" int dsb_gpu_fit_contexts(dsb_index *ix, uint64_t max_reads, char *err, size_t errn)
{
	if (getenv("DSB_WS_BUDGET_MB"))
		return 0;
	for (int k = 0; k < ix->n_gpu; k++) {
		dsb_gpu_dev *g0 = (dsb_gpu_dev *)ix->gpus[k];
		int first = 1;
		for (int j = 0; j < k; j++)
			first &= ((dsb_gpu_dev *)ix->gpus[j])->device != g0->device;
		if (!first) /* this GPU was fitted with its first context */
			continue;
		std::vector<dsb_gpu_dev *> cs;
		for (int j = k; j < ix->n_gpu; j++)
			if (((dsb_gpu_dev *)ix->gpus[j])->device == g0->device)
				cs.push_back((dsb_gpu_dev *)ix->gpus[j]);
		/* try-locks only: a batch of another call in flight holds its context's run lock while it
		 * waits for the carry of its call's batch before, which may need another context's lock;
		 * blocking here on one lock while holding another could close that cycle.  A busy context
		 * means a call is running on this GPU, and that call has fitted the contexts already. */
		size_t got = 0;
		while (got < cs.size() && pthread_mutex_trylock(&cs[got]->mu) == 0)
			got++;
		if (got < cs.size()) {
			while (got-- > 0)
				pthread_mutex_unlock(&cs[got]->mu);
			continue;
		}
		size_t fr = 0, tot = 0, held = 0;
		int rc = hipSetDevice(g0->device) == hipSuccess && hipMemGetInfo(&fr, &tot) == hipSuccess ? 0 : -1;
		for (dsb_gpu_dev *g : cs)
			held += g->ws.cap;
		/* the share, less dbuf::ensure's 1/8 growth margin; 250 GB at most (ws_budget).  A share
		 * within 10% of the one already set is kept: free HBM moves a little from call to call
		 * (staging, result buffers), and a workspace freed for a slightly smaller share is
		 * re-allocated by the next batch (hundreds of ms for ~100 GB) */
		size_t per = (size_t)((double)(fr + held) * 0.88 / cs.size() / 1.13);
		per = std::min(per, (size_t)250 << 30);
		for (dsb_gpu_dev *g : cs) {
			if (rc) {
				g->pipe_budget = 0;
				continue;
			}
			size_t old = g->pipe_budget;
			if (!(old && old <= per + per / 10 && per <= old + old / 10))
				g->pipe_budget = per;
			size_t b = g->pipe_budget;
			if (g->ws.cap > b + b / 4 + 8192) {
				hipDeviceSynchronize(); /* the context's earlier launches may still read it */
				g->ws.release();
			}
			/* the buffers a batch of up to max_reads reads needs, at their full size now: grown
			 * batch by batch they were freed and re-allocated whenever a context met a larger batch
			 * than before, and hipFree waits for the whole GPU (the other context's kernels) */
			uint64_t n = max_reads;
			char e2[256];
			if (b && n &&
			    (g->scale.ensure(4 * n + 4, e2, sizeof(e2)) ||
			     g->ws_off.ensure(8 * n + 8, e2, sizeof(e2)) || g->ro.ensure(sizeof(dsb_read_out_t) * n + 64, e2, sizeof(e2)) ||
			     g->mrl.ensure(4 * n + 4, e2, sizeof(e2)) || g->hit_off.ensure(4 * n + 4, e2, sizeof(e2)) ||
			     g->order.ensure(4 * n + 4, e2, sizeof(e2)) || g->word_off.ensure(8 * n + 16, e2, sizeof(e2)) ||
			     g->hits.ensure(sizeof(dsb_hit_out_t) * 16 * n + 4096, e2, sizeof(e2)) ||
			     g->wsr.ensure((size_t)64 << 20, e2, sizeof(e2))))
				(void)hipGetLastError(); /* not fatal: the batches allocate what they need themselves */
		}
		for (size_t j = cs.size(); j-- > 0;)
			pthread_mutex_unlock(&cs[j]->mu);
	}
	(void)err;
	(void)errn;
	return 0;
}

/* seed-wave prefix over a read list: 2 strands x ceil(lk/64) words for reads >= 40 bp */
static uint64_t seed_words(const std::vector<uint32_t> &len, uint64_t cb, const uint32_t *sel, size_t m, int l_ek,
			   std::vector<uint64_t> &off, uint64_t *positions)
{
	off.resize(m + 1);
	uint64_t tw = 0;
	for (size_t i = 0; i < m; i++) {
		off[i] = tw;
		uint32_t L = len[cb + (sel ? sel[i] : i)];
		if (L >= DSB_MIN_READ_LEN) {
			uint32_t lk = L - l_ek + 1;
			tw += 2ull * ((lk + 63) / 64);
			if (positions)
				*positions += 2ull * lk;
		}
	}
	off[m] = tw;
	return tw;
}

/* Test hooks (DSB_WAVE_DBG bits other than the timeline, DSB_WAVE_PHASES, DSB_TEST_SCALE0) exist
 * only in the test build of the library (lib/libdesamba_test.so, -DDSB_TEST_HOOKS=1): they force
 * staging overflows, sequential wave-loop variants, lane-per-read phases or stale sp_set pool
 * generations.  The production library ignores them. */
static uint32_t wave_dbg(void)
{
	const char *e = getenv("DSB_WAVE_DBG");
	uint32_t d = e ? (uint32_t)strtoul(e, NULL, 0) : 0;
	return DSB_TEST_HOOKS ? d : (d & DSB_DBG_TIMELINE); /* the timeline is a read-only dev tool (DSB_TL builds) */
}

/* phases run with one wavefront per read (DSB_WAVE_PHASES overrides in the test build) */
static uint32_t wave_phases(void)
{
	if (DSB_TEST_HOOKS)
		if (const char *e = getenv("DSB_WAVE_PHASES"))
			return (uint32_t)strtoul(e, NULL, 0);
	return (1u << DSB_PH_FAST0) | (1u << DSB_PH_FAST1) | (1u << DSB_PH_RESOLVE_F) | (1u << DSB_PH_SLOW0) |
	       (1u << DSB_PH_RESOLVE_S0) | (1u << DSB_PH_SLOW1) | (1u << DSB_PH_RESOLVE_S1) | (1u << DSB_PH_DELA);
}

/* Seeding sp_set slots are never cleared.  The GPU build keeps them in a per-GPU pool whose sets
 * carry their own generation base (dsb_hpool_release); a DSB_HSET_POOL=0 build keeps them in each
 * read's workspace, tagged with the launch that wrote them (dsb_hset_tag), so a tag must never
 * repeat on workspace bytes: one counter for the whole process (every context of every GPU: a
 * context's workspace may be re-allocated over bytes another context wrote), and workspace
 * buffers are zero-filled when allocated (tag 0 is never used). */
static std::atomic<uint64_t> g_launch_tag{0};
static uint64_t next_launch_tag(void) { return ++g_launch_tag; }

/* the LDS read-hash build's time (ms_phase[DSB_PH_HASH]) since the last call, taken out of the
 * scoring phase's (the callers time the hash build + scoring launch pair together); the events
 * of launches the callers do not time (overflow re-runs) are dropped with clear = 1 */
#define DSB_PH_HASH 9
#define DSB_PH_HEAVY 10 /* ms_phase: the heavy reads' scoring (run_split), hash build included */
static float hash_ms(dsb_gpu_dev *g, int clear = 0)
{
	float tot = 0;
	for (int si = 0; si < 2; si++)
		if (g->evh_used[si]) {
			float ms = 0;
			if (!clear && hipEventSynchronize(g->evh[si][1]) == hipSuccess &&
			    hipEventElapsedTime(&ms, g->evh[si][0], g->evh[si][1]) == hipSuccess)
				tot += ms;
			g->evh_used[si] = 0;
		}
	return tot;
}

/* one phase of part A over the reads order[0..m) */
/* the resolve phase ph ran inside the seeding kernels before it (dsb_kern.h DSB_FUSE_RESOLVE; not in
 * the stats runs, whose counters stay per phase, nor with lane-per-read seeding kernels) */
static int resolve_fused(int ph, int stats)
{
	if (!DSB_FUSE_RESOLVE || stats || DSB_SM_G != 64)
		return 0;
	uint32_t wp = wave_phases();
	switch (ph) {
	case DSB_PH_RESOLVE_F: return ((wp >> DSB_PH_FAST0) & 1) && ((wp >> DSB_PH_FAST1) & 1);
	case DSB_PH_RESOLVE_S0: return (wp >> DSB_PH_SLOW0) & 1;
	case DSB_PH_RESOLVE_S1: return (wp >> DSB_PH_SLOW1) & 1;
	default: return 0;
	}
}

static void launch_phase(dsb_gpu_dev *g, int ph, int stats, const uint32_t *cl, uint8_t *wsb, const uint32_t *order,
			 uint32_t m, hipStream_t s = 0)
{
	if (!s)
		s = g->stream;
	if (resolve_fused(ph, stats))
		return;
	int wave = (int)((wave_phases() >> ph) & 1);
	dsb_phase_fn fn = phase_kernel_at(ph, wave, stats);
	if (!fn) { /* a lane-per-read phase variant that is not compiled in (build with DSB_LANE_PHASES=1) */
		fprintf(stderr, "[dsb] phase %d: no %s-per-read kernel in this build\n", ph, wave ? "wave" : "lane");
		abort();
	}
	uint32_t dbg = wave_dbg();
	/* every launch gets its own slot tag (used by a DSB_HSET_POOL=0 build only) */
	uint64_t tag = next_launch_tag();
	if (!DSB_HSET_POOL && tag >= (1ull << (64 - DSB_HSET_GEN_BITS))) { /* 2^40 launches: unreachable in practice */
		fprintf(stderr, "[dsb] launch tag space exhausted; reload the index\n");
		abort();
	}
	if (ph == DSB_PH_DELA && DSB_HASH_LDS && m) {
		/* the read hash in LDS (k_hash_lds), then the scoring; timed apart by hash_ms() */
		int si = s == g->stream2;
		hipEventRecord(g->evh[si][0], s);
		if (stats == 1)
			hipLaunchKernelGGL(k_hash_lds<1>, dim3(2 * m), dim3(DSB_HL_WG), 0, s, g->d, cl, g->ws_off.as<uint64_t>(),
					   g->scale.as<uint32_t>(), wsb, order, m, g->stats.as<unsigned long long>());
		else
			hipLaunchKernelGGL(k_hash_lds<0>, dim3(2 * m), dim3(DSB_HL_WG), 0, s, g->d, cl, g->ws_off.as<uint64_t>(),
					   g->scale.as<uint32_t>(), wsb, order, m, g->stats.as<unsigned long long>());
		hipEventRecord(g->evh[si][1], s);
		g->evh_used[si] = 1;
	}
	if (wave) /* a wave per read, or 64 / DSB_SM_G reads per wave in the seeding phases */
		hipLaunchKernelGGL(fn, dim3(((uint64_t)m * DSB_PH_LANES(ph) + 63) / 64), dim3(64), 0, s, g->d, cl,
				   g->ws_off.as<uint64_t>(), g->scale.as<uint32_t>(), wsb, order, m, g->ro.as<dsb_read_out_t>(),
				   g->cnt.as<uint32_t>(), g->stats.as<unsigned long long>(), dbg, tag);
	else
		hipLaunchKernelGGL(fn, dim3(((ph == DSB_PH_ISLAND ? 2 * DSB_MAX(1, DSB_ISLAND_G) : 1) * m + 63) / 64), dim3(64), 0, s, g->d, cl, g->ws_off.as<uint64_t>(),
				   g->scale.as<uint32_t>(), wsb, order, m, g->ro.as<dsb_read_out_t>(), g->cnt.as<uint32_t>(),
				   g->stats.as<unsigned long long>(), dbg, tag);
}

/* a batch of reads resident in HBM (sequences only) + its results */
struct dsb_gpu_batch {
	int slot = 0;                /* device (dsb_index.gpus[slot]) holding the reads */
	hipEvent_t up_ev = nullptr;  /* the upload of a streamed batch (dsb_gpu_batch_stage) */
	int up_pending = 0;
	uint64_t n = 0, tot = 0;
	std::vector<uint32_t> len;
	std::vector<uint64_t> seq_off;
	dbuf seq, d_seq_off, d_len;
	dbuf d_tid, d_w;             /* per-read taxon of the last run (classB), weights for the counts */
	std::vector<dsb_read_out_t> ro;
	std::vector<dsb_hit_out_t> hits;
	std::vector<int32_t> carry; /* max_read_l each read's part B used (src/cly.c:2953) */
	/* per-chunk processing order (longest first), cached: it depends on the lengths only */
	std::vector<uint64_t> ord_cb, ord_ce;
	std::vector<std::vector<uint32_t>> ord;
	/* each read's workspace bytes at capacity scale wsz_scale (dsb_layout), cached: the chunk
	 * partition of a rerun batch sums them instead of laying every read out again (9 ms per 1M) */
	std::vector<uint64_t> wsz;
	uint32_t wsz_scale = 0;
};

static const std::vector<uint32_t> &chunk_order(dsb_gpu_batch *b, uint64_t cb, uint64_t ce)
{
	for (size_t k = 0; k < b->ord.size(); k++)
		if (b->ord_cb[k] == cb && b->ord_ce[k] == ce)
			return b->ord[k];
	if (cb == 0) { /* a new partition of the batch (the workspace budget changed): drop the old one */
		b->ord.clear();
		b->ord_cb.clear();
		b->ord_ce.clear();
	}
	std::vector<uint32_t> order(ce - cb);
	for (uint32_t i = 0; i < ce - cb; i++) order[i] = i;
	const std::vector<uint32_t> &len = b->len;
	std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t c) { return len[cb + a] > len[cb + c]; });
	b->ord_cb.push_back(cb);
	b->ord_ce.push_back(ce);
	b->ord.push_back(std::move(order));
	return b->ord.back();
}

static int batch_upload(dsb_gpu_dev *g, const dsb_reads_t *reads, dsb_gpu_batch *b, dsb_gpu_timing &T, char *err,
			size_t errn)
{
	HIP_OK(hipSetDevice(g->device));
	hipStream_t s = g->stream;
	uint64_t n = reads->n;
	b->n = n;
	b->wsz.clear(); /* new reads: the cached sizes and orders are stale */
	b->ord.clear();
	b->ord_cb.clear();
	b->ord_ce.clear();
	b->len.resize(n);
	b->seq_off.resize(n);
	uint64_t tot = 0;
	for (uint64_t i = 0; i < n; i++) {
		b->seq_off[i] = tot;
		b->len[i] = reads->rec[i].seq_l;
		tot += b->len[i];
	}
	b->tot = tot;
	if (b->seq.ensure(tot + 16, err, errn) || b->d_seq_off.ensure(8 * n + 8, err, errn) ||
	    b->d_len.ensure(4 * n + 4, err, errn))
		return -1;
	double th = now_ms();
	std::vector<uint8_t> stage(tot + 16); /* pack the bases (the arena also holds names/quals) */
	for (uint64_t i = 0; i < n; i++)
		memcpy(stage.data() + b->seq_off[i], reads->rec[i].seq, b->len[i]);
	HIP_OK(hipMemcpyAsync(b->seq.p, stage.data(), tot, hipMemcpyHostToDevice, s));
	HIP_OK(hipMemcpyAsync(b->d_seq_off.p, b->seq_off.data(), 8 * n, hipMemcpyHostToDevice, s));
	HIP_OK(hipMemcpyAsync(b->d_len.p, b->len.data(), 4 * n, hipMemcpyHostToDevice, s));
	HIP_OK(hipStreamSynchronize(s));
	T.ms_h2d += now_ms() - th;
	T.n_reads = n;
	T.n_bases = tot;
	return 0;
}

/* after resolve_f: reads[order[t]] -> slow list (slow seeding still to run) or rest list (scoring
 * next); one atomic per wave, lane order kept inside a wave (per-read results do not depend on
 * the processing order) */
/* The split's lists: the slow reads, and the scoring reads in descending classes of their
 * estimated scoring cost (chains x read length, powers of two): the longest waves start first, so
 * the launch does not end on a few of them (longest-processing-time-first).  On the C2 proxy
 * (5-step A/B, r05_hc) with one class of reads >= 2^16 first the scoring fell 431 -> 386 ms per
 * step; reads with no scoring to do cost 0.  With DSB_HEAVY_SPEC the reads of cost >=
 * DSB_HEAVY_COST go to their own list (scored over several waves each). */
#ifndef DSB_HEAVY_COST
#define DSB_HEAVY_COST (1u << 20) /* chains x read length: ~130 chains of an 8-kb read */
#endif
#define DSB_COST_CLASSES 14 /* class 0: cost < 2^12; class c: [2^(c+11), 2^(c+12)); the last open-ended */
static uint32_t heavy_cost(void)
{
	static int64_t v = -1;
	if (v < 0) {
		const char *e = getenv("DSB_HEAVY_COST");
		v = e ? strtoll(e, NULL, 10) : DSB_HEAVY_COST;
	}
	return (uint32_t)v;
}
DSB_HD uint32_t dsb_cost_class(uint64_t cost)
{
	if (cost < (1u << 12))
		return 0;
	uint32_t c = 63 - (uint32_t)__builtin_clzll(cost) - 11;
	return c < DSB_COST_CLASSES - 1 ? c : DSB_COST_CLASSES - 1;
}

/* Heavy reads deferred to the end of the batch (DSB_HEAVY_DEFER, cost >= DSB_DEFER_COST).  A scoring
 * launch lasts at least as long as its costliest read's wave: on the c2xl proxy the launch's wave clocks
 * summed to the small proxy's, but every launch waited ~140 ms for its heaviest read (one per chunk
 * and list, ten per step).  Such a read leaves the chunk's scoring with status DSB_STATUS_DEFER_HEAVY and
 * is classified again with the batch's deferred overflow re-runs, so the tails of all chunks overlap in
 * one launch.  A read may go only when its own result cannot move the carried max_read_l
 * (src/cly.c:2953): its length is at most a lower bound of the carry before it — the batch's carry-in
 * and the prefix maximum of the lengths of the chunk's earlier reads known to reach the update (fast
 * reads with hits after resolve_f: delete_small_score_rst returns early only without hits), computed by
 * k_carry_bound. */
#define DSB_STATUS_DEFER_HEAVY 64u
#define DSB_CB_WG 1024
__global__ __launch_bounds__(DSB_CB_WG) void k_carry_bound(const uint32_t *__restrict__ len, const uint64_t *__restrict__ ws_off,
							   const uint32_t *__restrict__ scale, const uint8_t *__restrict__ ws, uint32_t n,
							   uint32_t *__restrict__ bound)
{
	__shared__ uint32_t part[DSB_CB_WG];
	uint32_t tid = threadIdx.x, per = (n + DSB_CB_WG - 1) / DSB_CB_WG;
	uint32_t lo = DSB_MIN(n, tid * per), hi = DSB_MIN(n, lo + per);
	auto val = [&](uint32_t i) -> uint32_t { /* read i (input order) reaches the update with its length */
		uint32_t L = len[i];
		dsb_ws_layout lay = dsb_layout(L, dsb_default_caps(L, scale[i]));
		const dsb_rstate_t *sp = (const dsb_rstate_t *)(ws + ws_off[i] + lay.state);
		return (!sp->f.done && !sp->overflow && !sp->f.run_slow && sp->n_hit) ? L : 0u;
	};
	uint32_t m = 0;
	for (uint32_t i = lo; i < hi; i++)
		m = DSB_MAX(m, val(i));
	part[tid] = m;
	__syncthreads();
	for (uint32_t off = 1; off < DSB_CB_WG; off <<= 1) { /* inclusive prefix max over the threads' ranges */
		uint32_t v = tid >= off ? part[tid - off] : 0u;
		__syncthreads();
		part[tid] = DSB_MAX(part[tid], v);
		__syncthreads();
	}
	uint32_t run = tid ? part[tid - 1] : 0u;
	for (uint32_t i = lo; i < hi; i++) {
		bound[i] = run;
		run = DSB_MAX(run, val(i));
	}
}

/* cnt: [0] slow, [1] heavy (spec), [2 + c] class c, [2 + DSB_COST_CLASSES] deferred (DSB_HEAVY_DEFER);
 * class c's reads at classes + c * n */
__global__ __launch_bounds__(64) void k_split(const uint32_t *__restrict__ len, const uint64_t *__restrict__ ws_off,
					      const uint32_t *__restrict__ scale, const uint8_t *__restrict__ ws,
					      const uint32_t *__restrict__ order, uint32_t n, uint32_t *__restrict__ slow_list,
					      uint32_t *__restrict__ heavy_list, uint32_t *__restrict__ classes,
					      uint32_t *__restrict__ cnt, uint32_t heavy, uint32_t defer_cost,
					      const uint32_t *__restrict__ bound, uint32_t carry_in, dsb_read_out_t *__restrict__ ro,
					      uint32_t *__restrict__ n_overflow)
{
	uint32_t t = blockIdx.x * 64 + threadIdx.x, lane = threadIdx.x;
	int act = t < n, slow = 0, hv = 0, df = 0;
	uint32_t r = 0, cls = 0;
	if (act) {
		r = order[t];
		uint32_t L = len[r];
		dsb_ws_layout lay = dsb_layout(L, dsb_default_caps(L, scale[r]));
		const dsb_rstate_t *sp = (const dsb_rstate_t *)(ws + ws_off[r] + lay.state);
		slow = !sp->f.done && !sp->overflow && sp->f.run_slow;
		uint64_t cost = (!slow && !sp->f.done && !sp->overflow) ? (uint64_t)DSB_MIN(sp->n_hit, 400u) * L : 0;
		/* the heavy reads' waves share the read hash k_hash_lds prebuilt: a read whose hash each
		 * wave would build itself (dsb_hash_lds_read false) stays in the one-wave scoring */
		hv = !slow && sp->n_hit && cost >= heavy && dsb_hash_lds_read(L);
		df = !slow && !hv && sp->n_hit && cost >= defer_cost && L <= DSB_MAX(carry_in, bound[r]);
		cls = dsb_cost_class(cost);
		if (df) {
			dsb_read_out_t o = {0, 0, 0, DSB_STATUS_DEFER_HEAVY, 0, 0, 0};
			ro[r] = o;
			atomicAdd(n_overflow, 1u);
		}
	}
	uint64_t lt = lane == 0 ? 0 : (~0ull >> (64 - lane));
	/* slow and heavy lists, then each class present in the wave: one atomic per list per wave */
	int key = !act ? -1 : slow ? DSB_COST_CLASSES : hv ? DSB_COST_CLASSES + 1 : df ? DSB_COST_CLASSES + 2 : (int)cls;
	for (;;) {
		uint64_t live = __ballot(key >= 0);
		if (!live)
			break;
		int k0 = __shfl(key, (int)__builtin_ctzll(live));
		uint64_t m = __ballot(key == k0);
		uint32_t *ctr = k0 == DSB_COST_CLASSES ? cnt : k0 == DSB_COST_CLASSES + 1 ? cnt + 1 :
				k0 == DSB_COST_CLASSES + 2 ? cnt + 2 + DSB_COST_CLASSES : cnt + 2 + k0;
		uint32_t base = 0;
		if (lane == (uint32_t)__builtin_ctzll(m))
			base = atomicAdd(ctr, (uint32_t)__builtin_popcountll(m));
		base = (uint32_t)__shfl((int)base, (int)__builtin_ctzll(m));
		if (key == k0) {
			uint32_t at = base + (uint32_t)__builtin_popcountll(m & lt);
			if (k0 == DSB_COST_CLASSES)
				slow_list[at] = r;
			else if (k0 == DSB_COST_CLASSES + 1)
				heavy_list[at] = r;
			else if (k0 < DSB_COST_CLASSES)
				classes[(uint64_t)k0 * n + at] = r;
			key = -1;
		}
	}
}

/* The split of part A (run_split): after resolve_f the reads that still need slow seeding run
 * their slow phases on the library stream while the scoring of every other read runs on the
 * second stream.  On by default since round 4: on the C2 proxy the slow phases are ~14% of a step
 * (slow0 21 ms per 111k-read chunk, a few thousand long-running waves that leave most CUs idle),
 * and beside the scoring grid they cost little: 543.8k -> 579.7k reads/s (C2, 300k reads, one
 * box, profiles/r04_b).  On the C1 proxy of round 2 (slow phases ~9 ms of 160) it measured 555k
 * vs 564k without.  DSB_SPLIT=0 turns it off. */
static int split_slow(void)
{
	static int v = -1;
	if (v < 0) {
		const char *e = getenv("DSB_SPLIT");
		v = e ? (atoi(e) != 0) : 1;
	}
	return v;
}

/* A copy between the device and pageable host memory on the context's stream, waited for, through
 * the context's pinned bounce buffer.  A pageable copy (hipMemcpy, or hipMemcpyAsync on the
 * stream) waited for the other context's kernels on the GPU: 60-150 ms inside a 250-450 ms
 * read_classify call (the first batch's results, measured with DSB_HOST_TIMING); a pinned copy is
 * a DMA on this stream only.  The bounce buffer has a fixed size, allocated once per context
 * (growing it would hipHostFree, which synchronises the whole device: the other context's kernels);
 * larger copies go in bounce-sized pieces. */
static hipError_t copy_wait_g(dsb_gpu_dev *g, void *dst, const void *src, size_t n, hipMemcpyKind k, hipStream_t s)
{
	if (n == 0)
		return hipSuccess;
	if (!g->bounce) {
		hipError_t e = hipHostMalloc(&g->bounce, DSB_BOUNCE_BYTES, hipHostMallocDefault);
		if (e != hipSuccess) {
			g->bounce = nullptr;
			return e;
		}
		g->bounce_cap = DSB_BOUNCE_BYTES;
	}
	for (size_t o = 0; o < n; o += g->bounce_cap) {
		size_t m = std::min(g->bounce_cap, n - o);
		hipError_t e;
		if (k == hipMemcpyDeviceToHost) {
			e = hipMemcpyAsync(g->bounce, (const uint8_t *)src + o, m, k, s);
			if (e == hipSuccess)
				e = hipStreamSynchronize(s);
			if (e == hipSuccess)
				memcpy((uint8_t *)dst + o, g->bounce, m);
		} else {
			memcpy(g->bounce, (const uint8_t *)src + o, m);
			e = hipMemcpyAsync((uint8_t *)dst + o, g->bounce, m, k, s);
			if (e == hipSuccess)
				e = hipStreamSynchronize(s);
		}
		if (e != hipSuccess)
			return e;
	}
	return hipSuccess;
}

/* The slow phases touch ~2% of the reads and leave most of the GPU idle: after resolve_f the
 * reads are split, the scoring of the rest runs on a second stream while the slow phases and
 * then the slow reads' scoring run on the first.  Returns 1 when the rest of part A ran here,
 * 0 when there was nothing to split (the caller continues phase by phase), -1 on error. */
/* the heavy reads' scoring over several waves per read (dsb_kern.h k_heavy_*); DSB_HEAVY_SPEC=0:
 * one wave per read, the heavy reads first in the scoring launch */
extern "C" void dsb_heavy_kernels(dsb_heavy_prep_fn *prep, dsb_heavy_spec_fn *spec, dsb_heavy_fin_fn *fin);
#ifndef DSB_HEAVY_SPEC_DEFAULT
#define DSB_HEAVY_SPEC_DEFAULT 0
#endif
static int heavy_spec(void)
{
	static int v = -1;
	if (v < 0) {
		const char *e = getenv("DSB_HEAVY_SPEC");
		v = e ? (atoi(e) != 0) : DSB_HEAVY_SPEC_DEFAULT;
	}
	return v;
}

/* DSB_HEAVY_DEFER=1: heavy reads' scoring deferred to the batch's re-run group (k_split), reads of cost
 * >= DSB_DEFER_COST (chains x length) */
#ifndef DSB_DEFER_COST
#define DSB_DEFER_COST (1u << 22)
#endif
static uint32_t defer_cost(void)
{
	static int64_t v = -1;
	if (v < 0) {
		const char *e = getenv("DSB_HEAVY_DEFER");
		const char *c = getenv("DSB_DEFER_COST");
		v = (e && atoi(e)) ? (c ? strtoll(c, NULL, 10) : DSB_DEFER_COST) : UINT32_MAX;
	}
	return (uint32_t)v;
}

static int defer_retries(void);

/* carry_in: the carried max_read_l before the chunk when known (else 0: a lower bound) */
static int run_split(dsb_gpu_dev *g, int stats, const uint32_t *cl, uint8_t *wsb, uint32_t cn, const uint32_t *hlen,
		     const uint32_t *hscale, uint32_t carry_in, dsb_gpu_timing &T, char *err, size_t errn)
{
	hipStream_t s = g->stream;
	/* slist: the slow reads, then (at cn) the heavy scoring reads (DSB_HEAVY_SPEC); blist: the
	 * other scoring reads by cost class; rlist: those, costliest class first */
	const int want_spec = stats == 0 && heavy_spec();
	/* heavy reads deferred to the batch's re-run group (not in stats runs: those count every read's
	 * work in its chunk's phases; not without deferral) */
	const uint32_t dcost = (stats == 0 && defer_retries()) ? defer_cost() : UINT32_MAX;
	if (g->slist.ensure(8ull * cn + 8, err, errn) || g->rlist.ensure(4ull * cn + 4, err, errn) ||
	    g->blist.ensure(4ull * DSB_COST_CLASSES * cn + 4, err, errn) || g->cnt2.ensure(4 * (3 + DSB_COST_CLASSES), err, errn) ||
	    g->cbound.ensure(4ull * cn + 4, err, errn))
		return -1;
	HIP_OK(hipMemsetAsync(g->cnt2.p, 0, 4 * (3 + DSB_COST_CLASSES), s));
	if (dcost != UINT32_MAX)
		k_carry_bound<<<1, DSB_CB_WG, 0, s>>>(cl, g->ws_off.as<uint64_t>(), g->scale.as<uint32_t>(), wsb, cn,
						       g->cbound.as<uint32_t>());
	uint32_t *hl = g->slist.as<uint32_t>() + cn;
	k_split<<<(cn + 63) / 64, 64, 0, s>>>(cl, g->ws_off.as<uint64_t>(), g->scale.as<uint32_t>(), wsb,
					       g->order.as<uint32_t>(), cn, g->slist.as<uint32_t>(), hl, g->blist.as<uint32_t>(),
					       g->cnt2.as<uint32_t>(), want_spec ? heavy_cost() : UINT32_MAX, dcost,
					       g->cbound.as<uint32_t>(), carry_in, g->ro.as<dsb_read_out_t>(), g->cnt.as<uint32_t>());
	HIP_OK(hipGetLastError());
	uint32_t cc[3 + DSB_COST_CLASSES];
	HIP_OK(copy_wait_g(g, cc, g->cnt2.p, sizeof(cc), hipMemcpyDeviceToHost, s));
	uint32_t nr = 0;
	for (int k = 0; k < DSB_COST_CLASSES; k++)
		nr += cc[2 + k];
	uint32_t nh = cc[1], nd = cc[2 + DSB_COST_CLASSES];
	if (cc[0] + nh + nr + nd != cn) {
		snprintf(err, errn, "split: %u + %u + %u + %u reads for a chunk of %u", cc[0], nh, nr, nd, cn);
		return -1;
	}
	T.n_defer_heavy += nd;
	if (cc[0] == 0 || nh + nr == 0)
		return 0;
	/* the rest of the reads' list, costliest class first */
	for (int k = DSB_COST_CLASSES - 1, at = 0; k >= 0; k--)
		if (cc[2 + k]) {
			HIP_OK(hipMemcpyAsync(g->rlist.as<uint32_t>() + at, g->blist.as<uint32_t>() + (uint64_t)k * cn, 4ull * cc[2 + k],
					      hipMemcpyDeviceToDevice, s));
			at += cc[2 + k];
		}
	{ /* reads at or above DSB_HEAVY_COST (their own kernels with DSB_HEAVY_SPEC; else first in the list) */
		uint32_t hc = dsb_cost_class(heavy_cost());
		uint64_t nheavy = nh;
		for (int k = (int)hc; k < DSB_COST_CLASSES; k++)
			nheavy += cc[2 + k];
		T.n_heavy += nheavy;
	}
	static dsb_heavy_prep_fn k_prep;
	static dsb_heavy_spec_fn k_spec;
	static dsb_heavy_fin_fn k_fin;
	if (!k_prep)
		dsb_heavy_kernels(&k_prep, &k_spec, &k_fin);
	const int spec = nh > 0;
	if (spec && !g->stream3)
		HIP_OK(hipStreamCreateWithPriority(&g->stream3, hipStreamNonBlocking, g->prio_hi));
	if (spec) { /* the heavy reads' scratch, laid out per read */
		std::vector<uint32_t> hv(nh);
		HIP_OK(copy_wait_g(g, hv.data(), hl, 4ull * nh, hipMemcpyDeviceToHost, s));
		std::vector<uint64_t> ho(nh);
		uint64_t tot = 0;
		for (uint32_t k = 0; k < nh; k++) {
			ho[k] = tot;
			tot += dsb_heavy_bytes(hlen[hv[k]], hscale[hv[k]]);
		}
		if (g->hscr.ensure(tot + 256, err, errn) || g->hoff.ensure(8ull * nh + 8, err, errn))
			return -1;
		HIP_OK(copy_wait_g(g, g->hoff.p, ho.data(), 8ull * nh, hipMemcpyHostToDevice, s));
	}
	uint32_t c2[2] = {cc[0], nr};
	/* slow0's few workgroups are queued before the scoring grid so that they are dispatched first */
	hipEventRecord(g->ev_fork, s);
	hipEventRecord(g->ev_a, s);
	launch_phase(g, DSB_PH_SLOW0, stats, cl, wsb, g->slist.as<uint32_t>(), c2[0]);
	if (spec) {
		uint32_t dbg = wave_dbg();
		HIP_OK(hipStreamWaitEvent(g->stream3, g->ev_fork, 0));
		hipEventRecord(g->ev_h0, g->stream3);
		hipLaunchKernelGGL(k_hash_lds<0>, dim3(2 * nh), dim3(DSB_HL_WG), 0, g->stream3, g->d, cl, g->ws_off.as<uint64_t>(),
				   g->scale.as<uint32_t>(), wsb, hl, nh, g->stats.as<unsigned long long>());
		hipLaunchKernelGGL(k_prep, dim3(nh), dim3(64), 0, g->stream3, g->d, cl, g->ws_off.as<uint64_t>(),
				   g->scale.as<uint32_t>(), wsb, hl, nh, dbg);
		hipLaunchKernelGGL(k_spec, dim3(nh * DSB_HEAVY_W), dim3(64), 0, g->stream3, g->d, cl, g->ws_off.as<uint64_t>(),
				   g->scale.as<uint32_t>(), wsb, hl, nh, g->hscr.as<uint8_t>(), g->hoff.as<uint64_t>(), dbg);
		hipLaunchKernelGGL(k_fin, dim3(nh), dim3(64), 0, g->stream3, g->d, cl, g->ws_off.as<uint64_t>(),
				   g->scale.as<uint32_t>(), wsb, hl, nh, g->hscr.as<uint8_t>(), g->hoff.as<uint64_t>(),
				   g->ro.as<dsb_read_out_t>(), g->cnt.as<uint32_t>(), dbg);
		hipEventRecord(g->ev_h1, g->stream3);
		HIP_OK(hipGetLastError());
	}
	HIP_OK(hipStreamWaitEvent(g->stream2, g->ev_fork, 0));
	hipEventRecord(g->ev_r0, g->stream2);
	if (c2[1])
		launch_phase(g, DSB_PH_DELA, stats, cl, wsb, g->rlist.as<uint32_t>(), c2[1], g->stream2);
	hipEventRecord(g->ev_r1, g->stream2);
	HIP_OK(hipGetLastError());
	T.ms_phase[DSB_PH_SLOW0] += ev_ms(g);
	for (int ph = DSB_PH_SLOW0 + 1; ph < DSB_PH_N; ph++) {
		hipEventRecord(g->ev_a, s);
		launch_phase(g, ph, stats, cl, wsb, g->slist.as<uint32_t>(), c2[0]);
		T.ms_phase[ph] += ev_ms(g);
		HIP_OK(hipGetLastError());
	}
	HIP_OK(hipStreamWaitEvent(s, g->ev_r1, 0));
	if (spec)
		HIP_OK(hipStreamWaitEvent(s, g->ev_h1, 0));
	hipEventRecord(g->ev_b, s);
	HIP_OK(hipEventSynchronize(g->ev_b));
	float wall = 0, rest = 0, heavy = 0;
	hipEventElapsedTime(&wall, g->ev_fork, g->ev_b);
	hipEventElapsedTime(&rest, g->ev_r0, g->ev_r1);
	if (spec)
		hipEventElapsedTime(&heavy, g->ev_h0, g->ev_h1);
	T.ms_phase[DSB_PH_DELA] += rest; /* both scoring launches; ms_classA takes the overlapped wall time */
	T.ms_phase[DSB_PH_HEAVY] += heavy;
	if (c2[1]) {
		float hm = hash_ms(g); /* both launches' read-hash builds (each timed with its scoring launch) */
		T.ms_phase[DSB_PH_HASH] += hm;
		T.ms_phase[DSB_PH_DELA] -= hm;
	}
	T.ms_classA += wall;
	T.n_launch_dela += 2;
	return 1;
}

/* The scoring of an overflow re-run (retry_view) with its heavy reads (cost >= DSB_RETRY_HEAVY_COST,
 * k_split's rule otherwise) over DSB_HEAVY_W waves each (k_heavy_*) beside the one-wave scoring of the rest
 * (default; DSB_RETRY_SPEC=0: one wave per read).  A re-run group is a few hundred of the batch's
 * costliest reads and its scoring launch lasts as long as the costliest one (43 of the 82 ms of a
 * c2l18 step's re-run tail).  Every phase before the scoring has run for every re-run read, slow
 * ones included, so the list takes any read with chains to score.  c2l18: 541.6k vs 538.6k reads/s
 * (profiles/r06_c2l18/ab_retry_spec.txt). */
#ifndef DSB_RETRY_SPEC_DEFAULT
#define DSB_RETRY_SPEC_DEFAULT 1
#endif
static int retry_spec(void)
{
	static int v = -1;
	if (v < 0) {
		const char *e = getenv("DSB_RETRY_SPEC");
		v = e ? (atoi(e) != 0) : DSB_RETRY_SPEC_DEFAULT;
	}
	return v && DSB_HASH_LDS;
}

/* the re-run's heavy-read threshold (chains x length, DSB_RETRY_HEAVY_COST): 1 = every re-run read with
 * a chain to score.  The re-run's reads are few and costly, and its one-wave tail was a read below
 * the chunk's threshold: c2l18 550.7k reads/s at 1, 550.4k at 2^16, 541.7k at DSB_HEAVY_COST's 2^20
 * (profiles/r06_c2l18/ab_retry_cost.txt) */
#ifndef DSB_RETRY_HEAVY_COST
#define DSB_RETRY_HEAVY_COST 1
#endif
static uint32_t retry_heavy_cost(void)
{
	static int64_t v = -1;
	if (v < 0) {
		const char *e = getenv("DSB_RETRY_HEAVY_COST");
		v = e ? strtoll(e, NULL, 10) : (int64_t)DSB_RETRY_HEAVY_COST;
	}
	return (uint32_t)v;
}

/* cnt: [0] heavy reads (heavy_list), [1] the others (rest_list) */
__global__ __launch_bounds__(64) void k_retry_split(const uint32_t *__restrict__ len, const uint64_t *__restrict__ ws_off,
						    const uint32_t *__restrict__ scale, const uint8_t *__restrict__ ws,
						    const uint32_t *__restrict__ sel, uint32_t n, uint32_t heavy,
						    uint32_t *__restrict__ heavy_list, uint32_t *__restrict__ rest_list,
						    uint32_t *__restrict__ cnt)
{
	uint32_t t = blockIdx.x * 64 + threadIdx.x;
	if (t >= n)
		return;
	uint32_t r = sel[t], L = len[r];
	dsb_ws_layout lay = dsb_layout(L, dsb_default_caps(L, scale[r]));
	const dsb_rstate_t *sp = (const dsb_rstate_t *)(ws + ws_off[r] + lay.state);
	uint64_t cost = (!sp->f.done && !sp->overflow) ? (uint64_t)DSB_MIN(sp->n_hit, 400u) * L : 0;
	if (sp->n_hit && cost >= heavy && dsb_hash_lds_read(L))
		heavy_list[atomicAdd(cnt, 1u)] = r;
	else
		rest_list[atomicAdd(cnt + 1, 1u)] = r;
}

/* the scoring phase of a re-run of the m reads sel[] (device list; hlen / hscale: the view's host
 * lengths and capacity scales by read) -> the number of reads scored over several waves, or -1 */
static int retry_score(dsb_gpu_dev *g, const uint32_t *cl, uint8_t *wsb, const uint32_t *sel, uint32_t m,
		       const uint32_t *hlen, const uint32_t *hscale, char *err, size_t errn)
{
	hipStream_t s = g->stream;
	if (g->slist.ensure(4ull * m + 4, err, errn) || g->rlist.ensure(4ull * m + 4, err, errn) ||
	    g->cnt2.ensure(4 * (3 + DSB_COST_CLASSES), err, errn))
		return -1;
	HIP_OK(hipMemsetAsync(g->cnt2.p, 0, 8, s));
	k_retry_split<<<(m + 63) / 64, 64, 0, s>>>(cl, g->ws_off.as<uint64_t>(), g->scale.as<uint32_t>(), wsb, sel, m,
						   retry_heavy_cost(), g->slist.as<uint32_t>(), g->rlist.as<uint32_t>(),
						   g->cnt2.as<uint32_t>());
	HIP_OK(hipGetLastError());
	uint32_t cc[2];
	HIP_OK(copy_wait_g(g, cc, g->cnt2.p, sizeof(cc), hipMemcpyDeviceToHost, s));
	const uint32_t nh = cc[0], nr = cc[1];
	if (nh + nr != m) {
		snprintf(err, errn, "re-run split: %u + %u reads of %u", nh, nr, m);
		return -1;
	}
	if (!nh) {
		launch_phase(g, DSB_PH_DELA, 0, cl, wsb, sel, m);
		return 0;
	}
	static dsb_heavy_prep_fn k_prep;
	static dsb_heavy_spec_fn k_spec;
	static dsb_heavy_fin_fn k_fin;
	if (!k_prep)
		dsb_heavy_kernels(&k_prep, &k_spec, &k_fin);
	const uint32_t *hl = g->slist.as<uint32_t>();
	std::vector<uint32_t> hv(nh);
	HIP_OK(copy_wait_g(g, hv.data(), hl, 4ull * nh, hipMemcpyDeviceToHost, s));
	std::vector<uint64_t> ho(nh);
	uint64_t tot = 0;
	for (uint32_t k = 0; k < nh; k++) {
		ho[k] = tot;
		tot += dsb_heavy_bytes(hlen[hv[k]], hscale[hv[k]]);
	}
	if (g->hscr.ensure(tot + 256, err, errn) || g->hoff.ensure(8ull * nh + 8, err, errn))
		return -1;
	HIP_OK(copy_wait_g(g, g->hoff.p, ho.data(), 8ull * nh, hipMemcpyHostToDevice, s));
	if (!g->stream3)
		HIP_OK(hipStreamCreateWithPriority(&g->stream3, hipStreamNonBlocking, g->prio_hi));
	const uint32_t dbg = wave_dbg();
	hipEventRecord(g->ev_fork, s);
	HIP_OK(hipStreamWaitEvent(g->stream3, g->ev_fork, 0));
	hipLaunchKernelGGL(k_hash_lds<0>, dim3(2 * nh), dim3(DSB_HL_WG), 0, g->stream3, g->d, cl, g->ws_off.as<uint64_t>(),
			   g->scale.as<uint32_t>(), wsb, hl, nh, g->stats.as<unsigned long long>());
	hipLaunchKernelGGL(k_prep, dim3(nh), dim3(64), 0, g->stream3, g->d, cl, g->ws_off.as<uint64_t>(),
			   g->scale.as<uint32_t>(), wsb, hl, nh, dbg);
	hipLaunchKernelGGL(k_spec, dim3(nh * DSB_HEAVY_W), dim3(64), 0, g->stream3, g->d, cl, g->ws_off.as<uint64_t>(),
			   g->scale.as<uint32_t>(), wsb, hl, nh, g->hscr.as<uint8_t>(), g->hoff.as<uint64_t>(), dbg);
	hipLaunchKernelGGL(k_fin, dim3(nh), dim3(64), 0, g->stream3, g->d, cl, g->ws_off.as<uint64_t>(),
			   g->scale.as<uint32_t>(), wsb, hl, nh, g->hscr.as<uint8_t>(), g->hoff.as<uint64_t>(),
			   g->ro.as<dsb_read_out_t>(), g->cnt.as<uint32_t>(), dbg);
	hipEventRecord(g->ev_h1, g->stream3);
	HIP_OK(hipGetLastError());
	if (nr)
		launch_phase(g, DSB_PH_DELA, 0, cl, wsb, g->rlist.as<uint32_t>(), nr);
	HIP_OK(hipStreamWaitEvent(s, g->ev_h1, 0));
	HIP_OK(hipGetLastError());
	return (int)nh;
}

/* DSB_HOST_TIMING=1 (diagnostic): per batch_run, the host wall time of each section of the chunk
 * loop on stderr (the GPU idles in the sections that end in a synchronisation) */
enum { HS_SIZE, HS_SETUP, HS_PARTA, HS_SYNC_A, HS_RETRY, HS_CARRY_B, HS_D2H, HS_N };
static const char *hs_name[HS_N] = {"size", "setup", "partA_launch", "sync_A+ro", "retry", "carry+classB", "d2h"};
static int host_timing(void)
{
	static int v = -1;
	if (v < 0)
		v = getenv("DSB_HOST_TIMING") ? 1 : 0;
	return v;
}

/* overflow re-runs deferred to the end of a batch when they cannot change the carry (batch_run);
 * DSB_DEFER_RETRY=0 re-runs them chunk by chunk */
static int defer_retries(void)
{
	static int v = -1;
	if (v < 0) {
		const char *e = getenv("DSB_DEFER_RETRY");
		v = e ? (atoi(e) != 0) : 1;
	}
	return v;
}

/* part B (k_classB) of the reads order[0, n) of a view: lengths cl, the context's ws_off / scale /
 * mrl / ro / hit_off arrays, per-read taxa to tid */
static int launch_classB(dsb_gpu_dev *g, dsb_gpu_batch *b, const uint32_t *cl, uint8_t *wsb, const uint32_t *order,
			 uint32_t n, uint32_t *tid, int stats_on, hipStream_t s)
{
	(void)b;
	if (n == 0)
		return 0;
	if (stats_on == 1)
		k_classB<true><<<(n + 63) / 64, 64, 0, s>>>(g->d, cl, g->ws_off.as<uint64_t>(), g->scale.as<uint32_t>(), wsb, order, n,
							 g->mrl.as<int32_t>(), g->ro.as<dsb_read_out_t>(), g->hits.as<dsb_hit_out_t>(),
							 g->cnt.as<uint32_t>(), g->hit_off.as<uint32_t>(), tid,
							 g->stats.as<unsigned long long>());
	else
		k_classB<false><<<(n + 63) / 64, 64, 0, s>>>(g->d, cl, g->ws_off.as<uint64_t>(), g->scale.as<uint32_t>(), wsb, order, n,
							  g->mrl.as<int32_t>(), g->ro.as<dsb_read_out_t>(), g->hits.as<dsb_hit_out_t>(),
							  g->cnt.as<uint32_t>(), g->hit_off.as<uint32_t>(), tid,
							  g->stats.as<unsigned long long>());
	return hipGetLastError() == hipSuccess ? 0 : -1;
}


static int batch_run(dsb_gpu_dev *g, dsb_index *ix, dsb_gpu_batch *b, int *max_read_l, int stats_on,
		     dsb_gpu_timing &T, char *err, size_t errn, const dsb_carry_hooks *hooks = nullptr)
{
	double hs[HS_N] = {0}, hs_t = now_ms();
	dbuf &WS = g->ws;
	auto hs_mark = [&](int k) {
		double t = now_ms();
		hs[k] += t - hs_t;
		hs_t = t;
	};
	HIP_OK(hipSetDevice(g->device));
	hipStream_t s = g->stream;
	if (b->up_pending) { /* a streamed batch: its bases are still on the way on the copy stream */
		HIP_OK(hipStreamWaitEvent(s, b->up_ev, 0));
		b->up_pending = 0;
	}
	uint64_t n = b->n;
	const std::vector<uint32_t> &len = b->len;
	T.n_reads = n;
	T.n_bases = b->tot;
	b->ro.assign(n, dsb_read_out_t());
	b->hits.clear();
	if (n == 0) {
		if (hooks) { /* keep the carry chain of a stream going */
			int c = hooks->carry_in ? hooks->carry_in(hooks->ctx) : *max_read_l;
			if (hooks->carry_out)
				hooks->carry_out(hooks->ctx, c);
			*max_read_l = c;
		}
		return 0;
	}
	if (b->d_tid.ensure(4 * n + 4, err, errn) || g->scale.ensure(4 * n + 4, err, errn) ||
	    g->ro.ensure(sizeof(dsb_read_out_t) * n + 64, err, errn) ||
	    g->mrl.ensure(4 * n + 4, err, errn) || g->hit_off.ensure(4 * n + 4, err, errn) ||
	    g->cnt.ensure(64, err, errn) || g->ws_off.ensure(8 * n + 8, err, errn))
		return -1;
	/* DSB_DBG_TIMELINE (dev tool, DSB_TIMELINE=path): per-read phase timeline after the counters */
	const size_t tl_bytes = (wave_dbg() & DSB_DBG_TIMELINE) ? 8ull * 4 * DSB_PH_N * DSB_TL_STRIDE : 0;
	if (g->stats.ensure(8 * DSB_N_STATS + tl_bytes, err, errn))
		return -1;
	HIP_OK(hipMemsetAsync(g->stats.p, 0, 8 * DSB_N_STATS + tl_bytes, s));
	/* k_seed's probe counters (stats mode 1) go to the island phase's ek1 / ek2 slots */
	unsigned long long *sst = stats_on == 1 ? g->stats.as<unsigned long long>() : nullptr;
	/* DSB_TEST_SCALE0 (test build only): start below the default capacities so that reads overflow and
	 * take the re-run path */
	uint32_t scale0 = DSB_SCALE_UNIT;
	if (DSB_TEST_HOOKS)
		if (const char *e = getenv("DSB_TEST_SCALE0"))
			scale0 = (uint32_t)DSB_MAX(1, atoi(e));
	std::vector<uint32_t> scale(n, scale0);
	/* DSB_TEST_WS_FILL=b (test build only): the chunk workspace and the re-run reads' bytes are filled
	 * with byte b before the kernels run, so that a per-read field the kernels read before writing
	 * shows up (workspace bytes are otherwise an earlier read's, or zero in a fresh allocation) */
	int ws_fill = -1;
	if (DSB_TEST_HOOKS)
		if (const char *e = getenv("DSB_TEST_WS_FILL"))
			ws_fill = (int)(strtol(e, NULL, 0) & 0xff);
	/* DSB_TEST_FORCE_RERUN=k (test build only): every k-th read re-runs as if it had overflowed */
	uint64_t force_rerun = 0;
	if (DSB_TEST_HOOKS)
		if (const char *e = getenv("DSB_TEST_FORCE_RERUN"))
			force_rerun = strtoull(e, NULL, 10);
	std::vector<uint64_t> ws_off(n);
	std::vector<dsb_read_out_t> h_ro(n);
	std::vector<int32_t> &mrl = b->carry;
	mrl.assign(n, 0);
	std::vector<uint32_t> hit_off(n);
	std::vector<uint64_t> word_off;
	dsb_read_out_t *ro = b->ro.data();
	std::vector<dsb_hit_out_t> &hv = b->hits;
	std::vector<uint64_t> deferred; /* overflowed reads whose re-run waits for the end of the batch */
	size_t budget = ws_budget(g, hooks ? g->n_ctx : 1);
	int carry = *max_read_l;
	int l_ek = ix->l_ek;
	/* ---- overflow: re-run the reads i < cn of a view whose flag is set, with 8x capacities in the
	 * retry buffer; the view's host arrays are indexed cb + i, its device lengths / sequence offsets
	 * are cl[i] / cso[i]: one chunk, or the deferred overflows of the whole batch (below) */
	/* diagnostic (DSB_DEBUG_READ): a read's seeds, anchors and chains from its workspace */
	auto debug_dump = [&](uint8_t *base, uint32_t L, uint32_t sc, const dsb_read_out_t &o, const char *tag) {
		dsb_ws_layout lay = dsb_layout(L, dsb_default_caps(L, sc));
		std::vector<uint8_t> hbuf(lay.total);
		HIP_OK(hipMemcpy(hbuf.data(), base, lay.total, hipMemcpyDeviceToHost));
		dsb_read_ws w;
		dsb_ws_init(&w, &g->h, hbuf.data(), L, dsb_default_caps(L, sc));
		w.n_anc = o.n_anchor; w.n_hit = o.n_hit; w.fast_classify = o.fast;
		w.overflow = o.status; w.reached_update = o.reached_update;
		const dsb_sdir_t *sv = (const dsb_sdir_t *)(hbuf.data() + lay.state);
		w.sd[0] = sv[0];
		w.sd[1] = sv[1];
		dsb_debug_dump(stderr, &w, tag);
		return 0;
	};
	auto retry_view = [&](uint32_t cn, uint64_t cb, const std::vector<uint32_t> &vlen, std::vector<uint32_t> &vscale,
			      std::vector<uint64_t> &vws_off, std::vector<dsb_read_out_t> &vro, const uint32_t *cl,
			      const uint64_t *cso, uint8_t *wsb, uint64_t &rused, uint32_t n_over, const uint32_t *vid) -> int {
		/* the batch's read number of view entry i (vid: the deferred re-runs' map) */
		auto rid = [&](uint32_t i) -> unsigned long { return vid ? (unsigned long)vid[i] : (unsigned long)(cb + i); };
		while (n_over) {
			std::vector<uint32_t> sel;
			for (uint32_t i = 0; i < cn; i++)
				if (vro[cb + i].status) sel.push_back(i);
			T.n_retry += sel.size();
			if (host_timing())
				for (uint32_t i : sel)
					fprintf(stderr, "[dsb retry] read %lu L %u scale %u status %#x anchors %u hits %u\n",
						rid(i), vlen[cb + i], vscale[cb + i], vro[cb + i].status,
						vro[cb + i].n_anchor, vro[cb + i].n_hit);
			uint64_t tot2 = 0;
			for (uint32_t i : sel) {
				vscale[cb + i] *= DSB_CAP_RETRY;
				if (vscale[cb + i] > 4096 * DSB_SCALE_UNIT) {
					snprintf(err, errn, "read %lu (length %u) overflows every workspace size (status %#x, %u anchors, %u hits)",
						 rid(i), vlen[cb + i], vro[cb + i].status, vro[cb + i].n_anchor, vro[cb + i].n_hit);
					return -1;
				}
				vws_off[cb + i] = tot2; /* within this round's part of the retry buffer (rebased below) */
				tot2 += dsb_layout(vlen[cb + i], dsb_default_caps(vlen[cb + i], vscale[cb + i])).total;
			}
			/* the re-run reads live in a separate retry buffer (reads of earlier rounds keep their
			 * bytes; growing it copies only those), addressed from the chunk's base pointer: a
			 * read's offset is (retry buffer - chunk buffer) + its place there, modulo 2^64, so
			 * every kernel keeps using ws + ws_off[r] and the chunk workspace is never duplicated */
			if (rused + tot2 + 4096 > g->wsr.cap) {
				void *np = nullptr;
				size_t need = rused + tot2 + (rused + tot2) / 2 + 4096;
				if (!rused) /* nothing to keep: the old buffer goes first */
					g->wsr.release();
				if (hipMalloc(&np, need) != hipSuccess) {
					(void)hipGetLastError();
					need = rused + tot2 + 4096; /* no head room, then */
					if (hipMalloc(&np, need) != hipSuccess) {
						(void)hipGetLastError();
						size_t fr = 0, tot = 0;
						(void)hipMemGetInfo(&fr, &tot);
						snprintf(err, errn,
							 "out of HBM: re-running %zu overflowed reads needs %.1f MB of workspace, %.1f MB free on device %d",
							 sel.size(), need / 1048576.0, fr / 1048576.0, g->device);
						return -1;
					}
				}
				if (!DSB_HSET_POOL) /* launch-tagged sp_set tables: no stale tag in fresh bytes */
					HIP_OK(hipMemsetAsync(np, 0, need, s));
				if (rused)
					HIP_OK(hipMemcpyAsync(np, g->wsr.p, rused, hipMemcpyDeviceToDevice, s));
				HIP_OK(hipStreamSynchronize(s));
				uint64_t delta = (uint64_t)(uintptr_t)np - (uint64_t)(uintptr_t)g->wsr.p;
				for (uint32_t i = 0; i < cn && rused; i++) /* earlier retried reads move with the buffer */
					if (vscale[cb + i] > scale0 && !std::binary_search(sel.begin(), sel.end(), i))
						vws_off[cb + i] += delta;
				g->wsr.release();
				g->wsr.p = np;
				g->wsr.cap = need;
			}
			{
				uint64_t rbase = (uint64_t)(uintptr_t)g->wsr.p - (uint64_t)(uintptr_t)wsb + rused;
				if (host_timing())
					fprintf(stderr, "[dsb retry] view of %u reads: base %p, retry buffer %p (%.1f MB), rbase %#lx\n", cn,
						(void *)wsb, g->wsr.p, g->wsr.cap / 1048576.0, (unsigned long)rbase);
				for (uint32_t i : sel)
					vws_off[cb + i] += rbase;
				if (ws_fill >= 0) /* tests: the re-run reads' bytes as an earlier read's leftovers */
					HIP_OK(hipMemsetAsync((uint8_t *)g->wsr.p + rused, ws_fill, tot2, s));
				rused += tot2;
			}
			HIP_OK(copy_wait_g(g, g->ws_off.p, vws_off.data() + cb, 8ull * cn, hipMemcpyHostToDevice, s));
			HIP_OK(copy_wait_g(g, g->scale.p, vscale.data() + cb, 4ull * cn, hipMemcpyHostToDevice, s));
			std::vector<uint64_t> wo2;
			uint64_t tw2 = seed_words(vlen, cb, sel.data(), sel.size(), l_ek, wo2, nullptr);
			if (g->sel.ensure(4 * sel.size() + 4, err, errn) || g->wo2.ensure(8 * wo2.size() + 16, err, errn))
				return -1;
			HIP_OK(copy_wait_g(g, g->sel.p, sel.data(), 4 * sel.size(), hipMemcpyHostToDevice, s));
			HIP_OK(copy_wait_g(g, g->wo2.p, wo2.data(), 8 * wo2.size(), hipMemcpyHostToDevice, s));
			uint32_t m = (uint32_t)sel.size();
			if (m == 0) {
				snprintf(err, errn, "overflow reported by the phase kernels but no read carries the flag");
				return -1;
			}
			k_encode<<<m, 256, 0, s>>>(b->seq.as<uint8_t>(), cso, cl, g->ws_off.as<uint64_t>(), wsb, g->sel.as<uint32_t>(), m);
			if (tw2 && DSB_ISLAND_G == 0)
				k_seed<<<(uint32_t)((tw2 * 64 + 255) / 256), 256, 0, s>>>(g->d, cl, g->ws_off.as<uint64_t>(), wsb,
											      g->wo2.as<uint64_t>(), g->sel.as<uint32_t>(), m, tw2, nullptr);
			HIP_OK(hipMemsetAsync(g->cnt.p, 0, 64, s));
			const int rspec = retry_spec();
			for (int ph = 0; ph < (rspec ? DSB_PH_DELA : DSB_PH_N); ph++)
				launch_phase(g, ph, false, cl, wsb, g->sel.as<uint32_t>(), m);
			if (rspec) {
				int nh = retry_score(g, cl, wsb, g->sel.as<uint32_t>(), m, vlen.data() + cb, vscale.data() + cb, err, errn);
				if (nh < 0)
					return -1;
				if (host_timing())
					fprintf(stderr, "[dsb retry] %d of %u re-run reads scored over %d waves each\n", nh, m, DSB_HEAVY_W);
			}
			HIP_OK(hipGetLastError());
			/* the re-run went to the non-blocking stream: drain it before the (null-stream) copies */
			HIP_OK(hipStreamSynchronize(s));
			hash_ms(g, 1); /* re-runs are not timed */
			HIP_OK(copy_wait_g(g, &n_over, g->cnt.p, 4, hipMemcpyDeviceToHost, s));
			HIP_OK(copy_wait_g(g, vro.data() + cb, g->ro.p, sizeof(dsb_read_out_t) * cn, hipMemcpyDeviceToHost, s));
			if (const char *e = getenv("DSB_DEBUG_READ")) /* diagnostic: one re-run read's workspace */
				for (uint32_t i : sel)
					if (rid(i) == strtoull(e, NULL, 10))
						debug_dump(wsb + vws_off[cb + i], vlen[cb + i], vscale[cb + i], vro[cb + i], "gpuR");
		}
		return 0;
	};
	hs_mark(HS_SETUP);
	for (uint64_t cb = 0; cb < n;) {
		/* ---- chunk [cb, ce) within the workspace budget, input order */
		uint64_t ce = cb, ws_total = 0;
		if (b->wsz_scale != scale0 || b->wsz.size() != n) {
			b->wsz.resize(n);
			for (uint64_t i = 0; i < n; i++)
				b->wsz[i] = dsb_layout(len[i], dsb_default_caps(len[i], scale0)).total;
			b->wsz_scale = scale0;
		}
		while (ce < n) {
			uint64_t sz = scale[ce] == scale0 ? b->wsz[ce] : dsb_layout(len[ce], dsb_default_caps(len[ce], scale[ce])).total;
			if (ce > cb && ws_total + sz > budget)
				break;
			ws_off[ce] = ws_total;
			ws_total += sz;
			ce++;
		}
		uint32_t cn = (uint32_t)(ce - cb);
		T.n_chunks++;
		hs_mark(HS_SIZE);
		uint64_t rused = 0; /* bytes of the retry buffer holding this chunk's re-run reads */
		void *ws_before = WS.p;
		/* a streamed batch's workspace grows by doubling (up to the context's share): each growth
		 * is a hipFree, which waits for the whole GPU, the other context's kernels included */
		size_t ws_want = ws_total + 4096;
		if (hooks && ws_want > WS.cap)
			ws_want = std::max(ws_want, std::min((size_t)budget, 2 * WS.cap));
		if (WS.ensure(ws_want, err, errn)) {
			/* HBM short (another index, another user of the GPU, a budget above what is free):
			 * the exact size, else a chunk of half the bytes, down to one read; never a wait */
			(void)hipGetLastError();
			if (ws_want > ws_total + 4096 && WS.ensure(ws_total + 4096, err, errn) == 0) {
				/* the doubling did not fit; the chunk itself does */
			} else if (cn > 1) {
				(void)hipGetLastError();
				budget = std::max((size_t)1, (size_t)(ws_total / 2));
				if (hooks)
					g->pipe_budget = budget;
				T.n_ws_shrink++;
				T.n_chunks--;
				continue; /* re-partition from cb */
			} else {
				size_t fr = 0, tot = 0;
				(void)hipMemGetInfo(&fr, &tot);
				snprintf(err, errn, "out of HBM: one read of %u bases needs %.1f MB of workspace, %.1f MB free on device %d",
					 len[cb], ws_total / 1048576.0, fr / 1048576.0, g->device);
				return -1;
			}
		}
		if (g->order.ensure(4 * (size_t)cn + 4, err, errn) || g->word_off.ensure(8 * (size_t)cn + 16, err, errn))
			return -1;
		if (ws_fill >= 0) /* tests: every read's workspace starts as another read's leftovers would */
			HIP_OK(hipMemsetAsync(WS.p, ws_fill, ws_total, s));
		if (!DSB_HSET_POOL && WS.p != ws_before) /* fresh bytes: no stale sp_set slot may carry a live tag */
			HIP_OK(hipMemsetAsync(WS.p, 0, WS.cap, s));
		HIP_OK(copy_wait_g(g, g->ws_off.p, ws_off.data() + cb, 8ull * cn, hipMemcpyHostToDevice, s));
		HIP_OK(copy_wait_g(g, g->scale.p, scale.data() + cb, 4ull * cn, hipMemcpyHostToDevice, s));
		const uint32_t *cl = b->d_len.as<uint32_t>() + cb;
		const uint64_t *cso = b->d_seq_off.as<uint64_t>() + cb;
		/* length-sorted order (longest first) for the one-lane-per-read kernels */
		const std::vector<uint32_t> &order = chunk_order(b, cb, ce);
		HIP_OK(copy_wait_g(g, g->order.p, order.data(), 4ull * cn, hipMemcpyHostToDevice, s));
		uint8_t *wsb = WS.as<uint8_t>();
		hs_mark(HS_SETUP);
		hipEventRecord(g->ev_a, s);
		k_encode<<<cn, 256, 0, s>>>(b->seq.as<uint8_t>(), cso, cl, g->ws_off.as<uint64_t>(), wsb, nullptr, cn);
		T.ms_encode += ev_ms(g);
		HIP_OK(hipGetLastError());
		/* k-mer positions (both strands) of the reads the island scan covers */
		uint64_t tw = seed_words(len, cb, nullptr, cn, l_ek, word_off, &T.seed_positions);
		T.n_launch_phase += 1;
		if (tw && DSB_ISLAND_G == 0) { /* the rounds-1/2 form: k_seed's exist bits, then a two-lane island scan */
			HIP_OK(copy_wait_g(g, g->word_off.p, word_off.data(), 8ull * (cn + 1), hipMemcpyHostToDevice, s));
			hipEventRecord(g->ev_a, s);
			k_seed<<<(uint32_t)((tw * 64 + 255) / 256), 256, 0, s>>>(g->d, cl, g->ws_off.as<uint64_t>(), wsb,
										     g->word_off.as<uint64_t>(), nullptr, cn, tw, sst);
			T.ms_seed += ev_ms(g);
			HIP_OK(hipGetLastError());
		}
		HIP_OK(hipMemsetAsync(g->cnt.p, 0, 64, s));
		/* island, fast seeding, resolve: every read */
		for (int ph = 0; ph < DSB_PH_N; ph++) {
			hipEventRecord(g->ev_a, s);
			launch_phase(g, ph, stats_on, cl, wsb, g->order.as<uint32_t>(), cn);
			float ms = ev_ms(g);
			T.ms_phase[ph] += ms;
			T.ms_classA += ms;
			if (ph == DSB_PH_DELA) {
				T.n_launch_dela++;
				float hm = hash_ms(g);
				T.ms_phase[DSB_PH_HASH] += hm;
				T.ms_phase[DSB_PH_DELA] -= hm;
			}
			HIP_OK(hipGetLastError());
			if (ph == DSB_PH_RESOLVE_F && split_slow()) {
				int r = run_split(g, stats_on, cl, wsb, cn, len.data() + cb, scale.data() + cb,
						  hooks ? 0u : (uint32_t)DSB_MAX(carry, 0), T, err, errn);
				if (r < 0)
					return -1;
				if (r == 1) /* the rest of part A ran split */
					break;
			}
		}
		HIP_OK(hipGetLastError());
		hs_mark(HS_PARTA);
		HIP_OK(hipStreamSynchronize(s));
		uint32_t n_over = 0;
		HIP_OK(copy_wait_g(g, &n_over, g->cnt.p, 4, hipMemcpyDeviceToHost, s));
		HIP_OK(copy_wait_g(g, h_ro.data() + cb, g->ro.p, sizeof(dsb_read_out_t) * cn, hipMemcpyDeviceToHost, s));
		if (DSB_TEST_HOOKS && force_rerun) /* tests: every k-th read of the batch takes the re-run path */
			for (uint32_t i = 0; i < cn; i++)
				if ((cb + i) % force_rerun == 0 && !h_ro[cb + i].status) {
					h_ro[cb + i].status = 1;
					n_over++;
				}
		hs_mark(HS_SYNC_A);
		/* ---- max_read_l carry (src/cly.c:2953): prefix max over reads reaching the update; a
		 * streamed batch takes its carry-in from the batch before it (possibly on another GPU)
		 * once its own part A is done, and hands its carry-out on before its part B */
		if (cb == 0 && hooks && hooks->carry_in)
			carry = hooks->carry_in(hooks->ctx);
		/* ---- overflow: re-run those reads now, or defer them to one re-run at the end of the
		 * batch.  A deferred read's own part A result (reached_update) must not matter to the
		 * carry, i.e. the carry before it is already >= its length; then the chunk's part B runs
		 * for every other read now and the chunk's workspace is free for the next chunk (the
		 * re-run lives in the retry buffer).  A chunk re-run costs a launch of every phase on a
		 * few long-running waves (~10 ms on the C2 proxy, about one read per 110k-read chunk). */
		uint32_t n_def = 0;
		if (n_over && defer_retries()) {
			int c = carry, ok = 1;
			for (uint32_t i = 0; i < cn && ok; i++) {
				if (h_ro[cb + i].status)
					ok = (int)len[cb + i] <= c;
				else if (h_ro[cb + i].reached_update && (int)len[cb + i] > c)
					c = (int)len[cb + i];
			}
			if (ok) {
				for (uint32_t i = 0; i < cn; i++)
					if (h_ro[cb + i].status) {
						deferred.push_back(cb + i);
						n_def++;
					}
				n_over = 0;
			}
		}
		if (n_over && retry_view(cn, cb, len, scale, ws_off, h_ro, cl, cso, wsb, rused, n_over, nullptr))
			return -1;
		hs_mark(HS_RETRY);
		if (getenv("DSB_DEBUG_READ")) { /* diagnostic: dump one read's workspace after stage A */
			uint64_t dr = strtoull(getenv("DSB_DEBUG_READ"), NULL, 10);
			if (dr >= cb && dr < ce)
				debug_dump(wsb + ws_off[dr], len[dr], scale[dr], h_ro[dr], "gpuA");
		}
		uint64_t worst = 0;
		for (uint32_t i = 0; i < cn; i++) {
			if (h_ro[cb + i].reached_update && (int)len[cb + i] > carry)
				carry = (int)len[cb + i];
			mrl[cb + i] = carry;
			worst += h_ro[cb + i].n_hit;
		}
		if (ce == n && hooks && hooks->carry_out)
			hooks->carry_out(hooks->ctx, carry);
		HIP_OK(copy_wait_g(g, g->mrl.p, mrl.data() + cb, 4ull * cn, hipMemcpyHostToDevice, s));
		if (g->hits.ensure(sizeof(dsb_hit_out_t) * worst + 4096, err, errn))
			return -1;
		HIP_OK(hipMemsetAsync(g->cnt.p, 0, 64, s));
		uint32_t cnB = cn;
		if (n_def) { /* part B of this chunk: every read but the deferred ones */
			std::vector<uint32_t> ordB;
			ordB.reserve(cn - n_def);
			for (uint32_t i : order)
				if (!h_ro[cb + i].status)
					ordB.push_back(i);
			cnB = (uint32_t)ordB.size();
			HIP_OK(copy_wait_g(g, g->order.p, ordB.data(), 4ull * cnB, hipMemcpyHostToDevice, s));
		}
		hipEventRecord(g->ev_a, s);
		if (launch_classB(g, b, cl, wsb, g->order.as<uint32_t>(), cnB, b->d_tid.as<uint32_t>() + cb, stats_on, s))
			return -1;
		T.ms_classB += ev_ms(g);
		HIP_OK(hipGetLastError());
		hs_mark(HS_CARRY_B);
		double td = now_ms();
		uint32_t nh = 0;
		HIP_OK(copy_wait_g(g, &nh, g->cnt.p, 4, hipMemcpyDeviceToHost, s));
		HIP_OK(copy_wait_g(g, ro + cb, g->ro.p, sizeof(dsb_read_out_t) * cn, hipMemcpyDeviceToHost, s));
		HIP_OK(copy_wait_g(g, hit_off.data() + cb, g->hit_off.p, 4ull * cn, hipMemcpyDeviceToHost, s));
		uint64_t base = hv.size();
		hv.resize(base + nh);
		if (nh)
			HIP_OK(copy_wait_g(g, hv.data() + base, g->hits.p, sizeof(dsb_hit_out_t) * nh, hipMemcpyDeviceToHost, s));
		for (uint32_t i = 0; i < cn; i++)
			ro[cb + i].hit_off = base + hit_off[cb + i];
		T.ms_d2h += now_ms() - td;
		hs_mark(HS_D2H);
		cb = ce;
	}
	if (host_timing()) {
		fprintf(stderr, "[dsb host] %lu reads, %lu chunks:", (unsigned long)n, (unsigned long)T.n_chunks);
		for (int k = 0; k < HS_N; k++)
			fprintf(stderr, " %s %.1f", hs_name[k], hs[k]);
		fprintf(stderr, " ms\n");
	}
	/* ---- the deferred overflow re-runs of every chunk together, then their part B; in groups whose
	 * re-run workspace (DSB_CAP_RETRY x capacities) fits the HBM the chunk workspace leaves free.  A
	 * repeat-rich reference overflows thousands of reads per call: freeing the chunk workspace (it is
	 * idle now) is cheaper than a failed call */
	if (!deferred.empty()) {
		size_t fr = 0, tot = 0;
		(void)hipMemGetInfo(&fr, &tot);
		uint64_t need_all = 0;
		for (uint64_t r : deferred)
			need_all += dsb_layout(len[r], dsb_default_caps(len[r], scale[r] * DSB_CAP_RETRY)).total;
		/* DSB_TEST_RELEASE_WS (test build): release it whatever the sizes */
		if ((need_all + need_all / 2 > fr + g->wsr.cap || (DSB_TEST_HOOKS && getenv("DSB_TEST_RELEASE_WS"))) &&
		    !hooks) { /* a streamed batch's other context may use it */
			WS.release();
			(void)hipMemGetInfo(&fr, &tot);
			T.n_ws_shrink++;
		}
		uint64_t gcap = std::max<uint64_t>((uint64_t)((fr + g->wsr.cap) * 0.45), 1);
		if (DSB_TEST_HOOKS && getenv("DSB_TEST_RETRY_GROUP_MB")) /* tests: many small groups */
			gcap = strtoull(getenv("DSB_TEST_RETRY_GROUP_MB"), NULL, 10) << 20;
		uint32_t n_groups = 0;
		std::vector<uint32_t> vlen, vscale, vidx;
		std::vector<uint64_t> vws, vso;
		std::vector<dsb_read_out_t> vro;
		std::vector<int32_t> vmrl;
		for (size_t g0 = 0; g0 < deferred.size();) {
		size_t g1 = g0;
		for (uint64_t acc = 0; g1 < deferred.size(); g1++) {
			uint64_t r = deferred[g1];
			uint64_t sz = dsb_layout(len[r], dsb_default_caps(len[r], scale[r] * DSB_CAP_RETRY)).total;
			if (g1 > g0 && acc + sz > gcap)
				break;
			acc += sz;
		}
		uint32_t m = (uint32_t)(g1 - g0);
		const uint64_t *dq = deferred.data() + g0;
		vlen.assign(m, 0);
		vscale.assign(m, 0);
		vidx.assign(m, 0);
		vws.assign(m, 0);
		vso.assign(m, 0);
		vro.resize(m);
		vmrl.assign(m, 0);
		for (uint32_t k = 0; k < m; k++) {
			uint64_t r = dq[k];
			vidx[k] = (uint32_t)r;
			vlen[k] = len[r];
			vscale[k] = scale[r];
			vso[k] = b->seq_off[r];
			vro[k] = h_ro[r]; /* part A's result: the overflow flag set */
			vmrl[k] = mrl[r];
		}
		/* the order / carry / per-read arrays are sized per chunk elsewhere: m (every chunk's
		 * deferred reads) may exceed the largest chunk */
		if (g->vlen.ensure(4ull * m + 4, err, errn) || g->vso.ensure(8ull * m + 8, err, errn) ||
		    g->vidx.ensure(4ull * m + 4, err, errn) || g->vtid.ensure(4ull * m + 4, err, errn) ||
		    g->order.ensure(4ull * m + 4, err, errn) || g->mrl.ensure(4ull * m + 4, err, errn) ||
		    g->ws_off.ensure(8ull * m + 8, err, errn) || g->scale.ensure(4ull * m + 4, err, errn) ||
		    g->ro.ensure(sizeof(dsb_read_out_t) * m + 64, err, errn) || g->hit_off.ensure(4ull * m + 4, err, errn))
			return -1;
		HIP_OK(copy_wait_g(g, g->vlen.p, vlen.data(), 4ull * m, hipMemcpyHostToDevice, s));
		HIP_OK(copy_wait_g(g, g->vso.p, vso.data(), 8ull * m, hipMemcpyHostToDevice, s));
		HIP_OK(copy_wait_g(g, g->vidx.p, vidx.data(), 4ull * m, hipMemcpyHostToDevice, s));
		uint64_t rused = 0;
		/* offsets are relative to a base pointer: the chunk workspace's, or the retry buffer's own
		 * when the chunk workspace was released — allocated here first, for the group's first
		 * round, so that the kernels never get a null base (with a null base and absolute
		 * offsets, four reads of a 1M-read c2l18 batch lost a seed's anchors in the re-run) */
		if (!WS.p) {
			uint64_t need = 0;
			for (uint32_t k = 0; k < m; k++)
				need += dsb_layout(vlen[k], dsb_default_caps(vlen[k], vscale[k] * DSB_CAP_RETRY)).total;
			need += need / 2 + 4096;
			if (need > g->wsr.cap) {
				g->wsr.release();
				void *np = nullptr;
				if (hipMalloc(&np, need) != hipSuccess) {
					(void)hipGetLastError();
					size_t fr2 = 0, tot2 = 0;
					(void)hipMemGetInfo(&fr2, &tot2);
					snprintf(err, errn, "out of HBM: %u deferred re-runs need %.1f MB of workspace, %.1f MB free on device %d",
						 m, need / 1048576.0, fr2 / 1048576.0, g->device);
					return -1;
				}
				g->wsr.p = np;
				g->wsr.cap = need;
			}
		}
		uint8_t *wsb = WS.p ? WS.as<uint8_t>() : (uint8_t *)g->wsr.p;
		const uint32_t *vcl = g->vlen.as<uint32_t>();
		if (retry_view(m, 0, vlen, vscale, vws, vro, vcl, g->vso.as<uint64_t>(), wsb, rused, m, vidx.data()))
			return -1;
		std::vector<uint32_t> vord(m);
		uint64_t worst = 0;
		for (uint32_t k = 0; k < m; k++) {
			vord[k] = k;
			worst += vro[k].n_hit;
		}
		HIP_OK(copy_wait_g(g, g->order.p, vord.data(), 4ull * m, hipMemcpyHostToDevice, s));
		HIP_OK(copy_wait_g(g, g->mrl.p, vmrl.data(), 4ull * m, hipMemcpyHostToDevice, s));
		if (g->hits.ensure(sizeof(dsb_hit_out_t) * worst + 4096, err, errn))
			return -1;
		HIP_OK(hipMemsetAsync(g->cnt.p, 0, 64, s));
		hipEventRecord(g->ev_a, s);
		if (launch_classB(g, b, vcl, wsb, g->order.as<uint32_t>(), m, g->vtid.as<uint32_t>(), stats_on, s))
			return -1;
		k_scatter_u32<<<(m + 255) / 256, 256, 0, s>>>(b->d_tid.as<uint32_t>(), g->vidx.as<uint32_t>(),
								 g->vtid.as<uint32_t>(), m);
		T.ms_classB += ev_ms(g);
		HIP_OK(hipGetLastError());
		uint32_t nh = 0;
		std::vector<uint32_t> voff(m);
		HIP_OK(copy_wait_g(g, &nh, g->cnt.p, 4, hipMemcpyDeviceToHost, s));
		HIP_OK(copy_wait_g(g, vro.data(), g->ro.p, sizeof(dsb_read_out_t) * m, hipMemcpyDeviceToHost, s));
		HIP_OK(copy_wait_g(g, voff.data(), g->hit_off.p, 4ull * m, hipMemcpyDeviceToHost, s));
		uint64_t base = hv.size();
		hv.resize(base + nh);
		if (nh)
			HIP_OK(copy_wait_g(g, hv.data() + base, g->hits.p, sizeof(dsb_hit_out_t) * nh, hipMemcpyDeviceToHost, s));
		for (uint32_t k = 0; k < m; k++) {
			ro[dq[k]] = vro[k];
			ro[dq[k]].hit_off = base + voff[k];
		}
		n_groups++;
		g0 = g1;
		}
		hs_mark(HS_RETRY);
		if (host_timing())
			fprintf(stderr, "[dsb host] %zu deferred re-runs in %u groups (%.1f MB each at most)\n", deferred.size(),
				n_groups, gcap / 1048576.0);
	}
	*max_read_l = carry;
	if (tl_bytes && getenv("DSB_TIMELINE")) {
		std::vector<uint64_t> tl(tl_bytes / 8);
		HIP_OK(copy_wait_g(g, tl.data(), g->stats.as<uint8_t>() + 8 * DSB_N_STATS, tl_bytes, hipMemcpyDeviceToHost, s));
		if (FILE *f = fopen(getenv("DSB_TIMELINE"), "wb")) {
			fwrite(tl.data(), 8, tl.size(), f);
			fclose(f);
		}
	}
	if (stats_on) {
		unsigned long long st[DSB_N_STATS];
		HIP_OK(copy_wait_g(g, st, g->stats.p, sizeof(st), hipMemcpyDeviceToHost, s));
		for (int k = 0; k < DSB_N_STATS; k++) T.stats[k] = st[k];
	}
	return 0;
}

static dsb_gpu_dev *dev_of(const dsb_index *ix, int slot)
{
	return slot >= 0 && slot < ix->n_gpu ? (dsb_gpu_dev *)ix->gpus[slot] : nullptr;
}

extern "C" int dsb_gpu_batch_upload(dsb_index *ix, const dsb_reads_t *reads, dsb_gpu_batch **out, dsb_gpu_timing *tm,
				    char *err, size_t errn)
{
	dsb_gpu_dev *g = dev_of(ix, 0);
	if (!g) {
		snprintf(err, errn, "index not resident on a GPU (dsb_gpu_init not called)");
		return -1;
	}
	dsb_gpu_timing T;
	memset(&T, 0, sizeof(T));
	dsb_gpu_batch *b = new dsb_gpu_batch();
	pthread_mutex_lock(&g->mu);
	int rc = batch_upload(g, reads, b, T, err, errn);
	pthread_mutex_unlock(&g->mu);
	if (tm) {
		tm->ms_h2d += T.ms_h2d;
		tm->n_reads = T.n_reads;
		tm->n_bases = T.n_bases;
	}
	if (rc) {
		delete b;
		return rc;
	}
	*out = b;
	return 0;
}

static int run_locked(dsb_index *ix, dsb_gpu_batch *b, int *max_read_l, int stats_on, dsb_gpu_timing *tm,
		      const dsb_carry_hooks *hooks, char *err, size_t errn)
{
	dsb_gpu_dev *g = dev_of(ix, b->slot);
	if (!g) {
		snprintf(err, errn, "index not resident on a GPU (dsb_gpu_init not called)");
		return -1;
	}
	double t0 = now_ms();
	dsb_gpu_timing T;
	memset(&T, 0, sizeof(T));
	if (hooks && hooks->lock_wait)
		hooks->lock_wait(hooks->ctx);
	pthread_mutex_lock(&g->mu);
	if (hooks && hooks->locked)
		hooks->locked(hooks->ctx);
	int rc = batch_run(g, ix, b, max_read_l, stats_on, T, err, errn, hooks);
	pthread_mutex_unlock(&g->mu);
	T.ms_total = now_ms() - t0;
	if (tm) {
		double h2d = tm->ms_h2d;
		*tm = T;
		tm->ms_h2d += h2d;
	}
	return rc;
}

extern "C" int dsb_gpu_batch_run(dsb_index *ix, dsb_gpu_batch *b, int *max_read_l, int stats_on, dsb_gpu_timing *tm,
				 char *err, size_t errn)
{
	return run_locked(ix, b, max_read_l, stats_on, tm, nullptr, err, errn);
}

extern "C" int dsb_gpu_batch_run_chain(dsb_index *ix, dsb_gpu_batch *b, int stats_on, const dsb_carry_hooks *hooks,
				       dsb_gpu_timing *tm, char *err, size_t errn)
{
	int mrl = 0;
	return run_locked(ix, b, &mrl, stats_on, tm, hooks, err, errn);
}

/* ---- streamed batches (the read_classify pipeline) */
struct gather_ctx {
	const dsb_reads_t *reads;
	const uint64_t *seq_off;
	uint8_t *dst;
	uint64_t per_task;
};

static void gather_task(void *c_, uint64_t t, int worker)
{
	(void)worker;
	const gather_ctx *c = (const gather_ctx *)c_;
	uint64_t lo = t * c->per_task, hi = lo + c->per_task;
	if (hi > c->reads->n)
		hi = c->reads->n;
	for (uint64_t i = lo; i < hi; i++)
		memcpy(c->dst + c->seq_off[i], c->reads->rec[i].seq, c->reads->rec[i].seq_l);
}

/* Upload `reads` to GPU `slot` without the device's run lock: the bases are gathered from the
 * record views into pinned staging by the host pool, then copied on the device's copy stream,
 * so this overlaps the kernels of the batch before.  The batch comes from the device's spare
 * list when there is one (no hipMalloc / hipFree in steady state). */
extern "C" int dsb_gpu_batch_stage(dsb_index *ix, int slot, const dsb_reads_t *reads, dsb_pool *pool,
				   dsb_gpu_batch **out, double *ms_gather, char *err, size_t errn)
{
	dsb_gpu_dev *g = dev_of(ix, slot);
	if (!g) {
		snprintf(err, errn, "no GPU slot %d", slot);
		return -1;
	}
	HIP_OK(hipSetDevice(g->device));
	pthread_mutex_lock(&g->umu);
	int rc = -1;
	dsb_gpu_batch *b = nullptr;
	do {
		if (!g->spare.empty()) {
			b = g->spare.back();
			g->spare.pop_back();
		} else {
			b = new dsb_gpu_batch();
			if (hipEventCreateWithFlags(&b->up_ev, hipEventDisableTiming) != hipSuccess) {
				snprintf(err, errn, "hipEventCreate failed");
				break;
			}
		}
		b->slot = slot;
		b->ord.clear();
		b->ord_cb.clear();
		b->ord_ce.clear();
		b->wsz.clear();
		uint64_t n = reads->n, tot = 0;
		b->n = n;
		b->len.resize(n);
		b->seq_off.resize(n);
		for (uint64_t i = 0; i < n; i++) {
			b->seq_off[i] = tot;
			b->len[i] = reads->rec[i].seq_l;
			tot += b->len[i];
		}
		b->tot = tot;
		if (b->seq.ensure(tot + 16, err, errn) || b->d_seq_off.ensure(8 * n + 8, err, errn) ||
		    b->d_len.ensure(4 * n + 4, err, errn))
			break;
		/* pinned staging k: free once its last copy has completed */
		int k = g->pin_next;
		g->pin_next ^= 1;
		if (g->pin_used[k] && hipEventSynchronize(g->pin_ev[k]) != hipSuccess) {
			snprintf(err, errn, "staging event failed");
			break;
		}
		size_t need = tot + 12 * n + 64;
		if (need > g->pin_cap[k]) {
			if (g->pin[k])
				hipHostFree(g->pin[k]);
			g->pin[k] = nullptr;
			g->pin_cap[k] = 0;
			size_t c = need + need / 4;
			if (hipHostMalloc(&g->pin[k], c, hipHostMallocDefault) != hipSuccess) {
				snprintf(err, errn, "hipHostMalloc(%zu) failed", c);
				break;
			}
			g->pin_cap[k] = c;
		}
		double t0 = now_ms();
		uint8_t *pin = (uint8_t *)g->pin[k];
		gather_ctx gc = {reads, b->seq_off.data(), pin, 0};
		gc.per_task = n / (uint64_t)(4 * dsb_pool_size(pool)) + 1;
		dsb_pool_run(pool, (n + gc.per_task - 1) / gc.per_task, gather_task, &gc);
		uint8_t *meta = pin + ((tot + 15) & ~(uint64_t)15);
		memcpy(meta, b->seq_off.data(), 8 * n);
		memcpy(meta + 8 * n, b->len.data(), 4 * n);
		if (ms_gather)
			*ms_gather += now_ms() - t0;
		hipStream_t cs = g->cstream;
		if (hipMemcpyAsync(b->seq.p, pin, tot, hipMemcpyHostToDevice, cs) != hipSuccess ||
		    hipMemcpyAsync(b->d_seq_off.p, meta, 8 * n, hipMemcpyHostToDevice, cs) != hipSuccess ||
		    hipMemcpyAsync(b->d_len.p, meta + 8 * n, 4 * n, hipMemcpyHostToDevice, cs) != hipSuccess ||
		    hipEventRecord(g->pin_ev[k], cs) != hipSuccess || hipEventRecord(b->up_ev, cs) != hipSuccess) {
			snprintf(err, errn, "batch upload failed");
			break;
		}
		g->pin_used[k] = 1;
		b->up_pending = 1;
		rc = 0;
	} while (0);
	if (rc && b) {
		g->spare.push_back(b);
		b = nullptr;
	}
	pthread_mutex_unlock(&g->umu);
	*out = b;
	return rc;
}

/* give a streamed batch back to its device's spare list (results already consumed) */
extern "C" void dsb_gpu_batch_recycle(dsb_index *ix, dsb_gpu_batch *b)
{
	dsb_gpu_dev *g = dev_of(ix, b->slot);
	pthread_mutex_lock(&g->umu);
	g->spare.push_back(b);
	pthread_mutex_unlock(&g->umu);
}

extern "C" const dsb_read_out_t *dsb_gpu_batch_ro(const dsb_gpu_batch *b) { return b->ro.data(); }
extern "C" const dsb_hit_out_t *dsb_gpu_batch_hits(const dsb_gpu_batch *b) { return b->hits.data(); }
extern "C" const int32_t *dsb_gpu_batch_carry(const dsb_gpu_batch *b) { return b->carry.data(); }
extern "C" uint64_t dsb_gpu_batch_n(const dsb_gpu_batch *b) { return b->n; }
extern "C" uint64_t dsb_gpu_batch_bases(const dsb_gpu_batch *b) { return b->tot; }
extern "C" int dsb_gpu_batch_device(const dsb_index *ix, const dsb_gpu_batch *b)
{
	dsb_gpu_dev *g = dev_of(ix, b->slot);
	return g ? g->device : -1;
}

extern "C" int dsb_gpu_batch_counts(dsb_index *ix, dsb_gpu_batch *b, const uint32_t *weights, uint64_t *dev_counts,
				    uint64_t n_counts, char *err, size_t errn)
{
	dsb_gpu_dev *g = dev_of(ix, b->slot);
	if (!g) {
		snprintf(err, errn, "no GPU");
		return -1;
	}
	pthread_mutex_lock(&g->mu);
	int rc = -1;
	do {
		if (hipSetDevice(g->device) != hipSuccess || !g->h.p_tid || n_counts < ix->max_tid + 1) {
			snprintf(err, errn, "taxon counts: no taxonomy on the device or a table of %lu < max_tid + 1",
				 (unsigned long)n_counts);
			break;
		}
		if (!b->d_tid.p) {
			snprintf(err, errn, "taxon counts before any run of the batch");
			break;
		}
		hipPointerAttribute_t pa;
		if (hipPointerGetAttributes(&pa, dev_counts) != hipSuccess || pa.device != g->device) {
			snprintf(err, errn, "taxon counts: the table is not device memory of GPU %d", g->device);
			break;
		}
		hipStream_t s = g->stream;
		if (hipMemsetAsync(dev_counts, 0, 8 * n_counts, s) != hipSuccess)
			break;
		if (weights) {
			if (b->d_w.ensure(4 * b->n + 4, err, errn) ||
			    hipMemcpyAsync(b->d_w.p, weights, 4 * b->n, hipMemcpyHostToDevice, s) != hipSuccess)
				break;
		}
		if (b->n)
			k_taxon_count<<<(uint32_t)((b->n + 255) / 256), 256, 0, s>>>(b->d_tid.as<uint32_t>(),
				weights ? b->d_w.as<uint32_t>() : nullptr, b->n, (unsigned long long *)dev_counts);
		if (hipGetLastError() != hipSuccess || hipStreamSynchronize(s) != hipSuccess) {
			snprintf(err, errn, "taxon counts: kernel failed");
			break;
		}
		rc = 0;
	} while (0);
	pthread_mutex_unlock(&g->mu);
	return rc;
}

static void batch_destroy(dsb_gpu_batch *b)
{
	if (b->up_ev)
		hipEventDestroy(b->up_ev);
	delete b;
}

extern "C" void dsb_gpu_batch_free(dsb_index *ix, dsb_gpu_batch *b)
{
	dsb_gpu_dev *g = ix ? dev_of(ix, b->slot) : nullptr;
	if (g) {
		pthread_mutex_lock(&g->mu);
		hipSetDevice(g->device);
	}
	batch_destroy(b);
	if (g)
		pthread_mutex_unlock(&g->mu);
}

extern "C" int dsb_gpu_classify(dsb_index *ix, const dsb_reads_t *reads, int *max_read_l, dsb_read_out_t *ro,
				dsb_hit_out_t **hits, uint64_t *n_hits, int stats_on, dsb_gpu_timing *tm, char *err,
				size_t errn)
{
	dsb_gpu_timing T;
	memset(&T, 0, sizeof(T));
	dsb_gpu_batch *b = nullptr;
	double t0 = now_ms();
	if (dsb_gpu_batch_upload(ix, reads, &b, &T, err, errn))
		return -1;
	int rc = dsb_gpu_batch_run(ix, b, max_read_l, stats_on, &T, err, errn);
	if (rc == 0) {
		memcpy(ro, b->ro.data(), sizeof(dsb_read_out_t) * b->n);
		*n_hits = b->hits.size();
		*hits = (dsb_hit_out_t *)malloc(sizeof(dsb_hit_out_t) * (b->hits.size() + 1));
		if (!b->hits.empty())
			memcpy(*hits, b->hits.data(), sizeof(dsb_hit_out_t) * b->hits.size());
	}
	dsb_gpu_batch_free(ix, b);
	T.ms_total = now_ms() - t0;
	if (tm)
		*tm = T;
	return rc;
}

#if DSB_TEST_HOOKS /* device self-tests: the test build only */
/* GPU self-test of the glibc-msort restatement: n_arrays x n random keys sorted on the device
 * and on the host with the same code; returns the number of arrays whose permutation differs. */
extern "C" int dsb_gpu_selftest_sort(uint32_t n, uint32_t n_arrays, int which, uint32_t seed)
{
	char err[256];
	size_t errn = sizeof(err);
	size_t tot = (size_t)n * n_arrays;
	std::vector<dsb_chain_t> h(tot), tmp(tot);
	std::vector<uint32_t> hi(tot), ht(tot), back(tot);
	uint32_t x = seed | 1;
	auto rnd = [&]() { x ^= x << 13; x ^= x >> 17; x ^= x << 5; return x; };
	for (auto &c : h) {
		memset(&c, 0, sizeof(c));
		c.ref_ID = rnd() % 4;
		c.t_st = rnd() % 8;
		c.sum_score = rnd() % 6;
		c.q_st = rnd() % 100;
		c.q_ed = c.q_st + rnd() % 100;
		c.with_top_anchor = rnd() & 1;
		c.indel = rnd() % 3;
	}
	dsb_chain_t *dc, *dt;
	uint32_t *di, *dti;
	HIP_OK(hipMalloc(&dc, tot * sizeof(dsb_chain_t)));
	HIP_OK(hipMalloc(&dt, tot * sizeof(dsb_chain_t)));
	HIP_OK(hipMalloc(&di, tot * 4));
	HIP_OK(hipMalloc(&dti, tot * 4));
	HIP_OK(hipMemcpy(dc, h.data(), tot * sizeof(dsb_chain_t), hipMemcpyHostToDevice));
	k_selftest_sort<<<(n_arrays + 63) / 64, 64>>>(dc, dt, di, dti, n, n_arrays, which);
	HIP_OK(hipDeviceSynchronize());
	HIP_OK(hipMemcpy(back.data(), di, tot * 4, hipMemcpyDeviceToHost));
	(void)hipFree(dc); (void)hipFree(dt); (void)hipFree(di); (void)hipFree(dti);
	int bad = 0;
	for (uint32_t a = 0; a < n_arrays; a++) {
		size_t o = (size_t)a * n;
		dsb_selftest_one(h.data() + o, tmp.data() + o, hi.data() + o, ht.data() + o, n, which);
		if (memcmp(hi.data() + o, back.data() + o, 4ull * n) != 0)
			bad++;
	}
	return bad;
}

/* GPU self-test of the occ re-layout on any .bwt, BWTs past 2^32 rows included: for every row,
 * dsb_occ(r, c) for c = 0..4 and dsb_occ(r, 0xff) with the symbol it reads (7 u64 per row, the
 * layout of oracle/bigbwt.c occ, which runs the reference's own occ on the same file). */
__global__ __launch_bounds__(256) void k_selftest_occ(const dsb_dindex_t *__restrict__ ix, const uint64_t *__restrict__ rows,
							uint64_t n, uint64_t *__restrict__ out)
{
	uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n)
		return;
	uint64_t r = rows[i];
	for (int c = 0; c < 5; c++) {
		uint8_t cc = (uint8_t)c;
		out[7 * i + c] = dsb_occ(ix, r, &cc);
	}
	uint8_t cf = 0xff;
	out[7 * i + 5] = dsb_occ(ix, r, &cf);
	out[7 * i + 6] = cf;
}

extern "C" int dsb_gpu_selftest_occ(const char *dir, uint64_t dollor_pos, const uint64_t *rows, uint64_t n,
				    uint64_t *out, char *err, size_t errn)
{
	dsb_index *ix = (dsb_index *)calloc(1, sizeof(dsb_index));
	if (!ix) {
		snprintf(err, errn, "out of memory");
		return -1;
	}
	int rc = -1;
	if (errn)
		err[0] = 0;
	void *d_occ = nullptr, *d_sup = nullptr, *d_rows = nullptr, *d_out = nullptr, *d_ix = nullptr;
	do {
		if (dsb_index_load_bwt(ix, dir, 0, err, errn))
			break;
		for (uint64_t i = 0; i < n; i++)
			if (rows[i] >= ix->n_occ_line * DSB_OCC_LINE_SYM) {
				snprintf(err, errn, "row %lu past the BWT (%lu rows)", (unsigned long)rows[i],
					 (unsigned long)(ix->n_occ_line * DSB_OCC_LINE_SYM));
				break;
			}
		if (err[0])
			break;
		dsb_dindex_t h;
		memset(&h, 0, sizeof(h));
		size_t occ_b = (ix->n_occ_line + 1) * DSB_OCC_LINE_U64 * 8, sup_b = ix->n_occ_super * 32;
		if (hipMalloc(&d_occ, occ_b) != hipSuccess || hipMalloc(&d_sup, sup_b) != hipSuccess ||
		    hipMalloc(&d_rows, 8 * n + 8) != hipSuccess || hipMalloc(&d_out, 56 * n + 8) != hipSuccess ||
		    hipMalloc(&d_ix, sizeof(h)) != hipSuccess) {
			snprintf(err, errn, "hipMalloc failed (%.2f GB of occ lines)", occ_b / 1e9);
			break;
		}
		h.occ = (const uint64_t *)d_occ;
		h.occ_super = (const uint64_t *)d_sup;
		h.n_occ_line = ix->n_occ_line;
		memcpy(h.dollar_row, ix->dollar_row, sizeof(h.dollar_row));
		h.n_dollar = ix->n_dollar;
		memcpy(h.rank, ix->rank, sizeof(h.rank));
		h.dollor_pos = dollor_pos;
		if (hipMemcpy(d_occ, ix->occ, occ_b, hipMemcpyHostToDevice) != hipSuccess ||
		    hipMemcpy(d_sup, ix->occ_super, sup_b, hipMemcpyHostToDevice) != hipSuccess ||
		    hipMemcpy(d_rows, rows, 8 * n, hipMemcpyHostToDevice) != hipSuccess ||
		    hipMemcpy(d_ix, &h, sizeof(h), hipMemcpyHostToDevice) != hipSuccess) {
			snprintf(err, errn, "upload failed");
			break;
		}
		if (n)
			k_selftest_occ<<<(uint32_t)((n + 255) / 256), 256>>>((const dsb_dindex_t *)d_ix, (const uint64_t *)d_rows, n,
									   (uint64_t *)d_out);
		if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
		    hipMemcpy(out, d_out, 56 * n, hipMemcpyDeviceToHost) != hipSuccess) {
			snprintf(err, errn, "occ self-test kernel failed");
			break;
		}
		rc = 0;
	} while (0);
	for (void *p : {d_occ, d_sup, d_rows, d_out, d_ix})
		if (p)
			(void)hipFree(p);
	dsb_index_free_host_tables(ix);
	free(ix);
	return rc;
}
#endif
