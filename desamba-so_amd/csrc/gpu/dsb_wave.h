/*
 * dsb_wave.h — wave-cooperative helpers (one 64-lane wavefront per read).
 *
 * The per-read scoring (get_score_M2 and its sparse DP) runs with one wavefront per read:
 * the reference's control flow executes uniformly on every lane, while the inner loops
 * (reference-window k-mer lookups, the sparse-DP predecessor scans, the read hash build,
 * window unpacking) are spread over the 64 lanes and recombined in the reference's order
 * with ballots, prefix sums and max-reductions.
 *
 * Kernels using these helpers run one wavefront per workgroup, so dsb_wsync() (a
 * workgroup barrier) orders one lane's global/LDS stores before another lane's loads.
 * On the host (tests/emu) the same code runs as a one-lane "wave" (DSB_WV == 1).
 */
#ifndef DSB_WAVE_H
#define DSB_WAVE_H
#include "dsb_core.h"

#if defined(__HIP_DEVICE_COMPILE__)
/*
 * Reductions and scans use DPP row operations (16-lane rows, VALU latency) plus v_readlane
 * for the four row totals, instead of ds_bpermute shuffles (an LDS round trip per step).
 * All helpers assume the whole wave is active (they are called from wave-uniform code).
 */
#define DSB_WV 64
#define DSB_DPP_ROW_SHR(n) (0x110 + (n))
#define DSB_DPP_ROW_ROR(n) (0x120 + (n))
DSB_HD uint32_t dsb_lane(void) { return __lane_id(); }
DSB_HD void dsb_wsync(void) { __syncthreads(); }
DSB_HD int dsb_rdlane(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
/* max over the wave, returned uniform */
DSB_HD int dsb_wmax(int v)
{
	v = max(v, __builtin_amdgcn_update_dpp(v, v, DSB_DPP_ROW_ROR(1), 0xf, 0xf, false));
	v = max(v, __builtin_amdgcn_update_dpp(v, v, DSB_DPP_ROW_ROR(2), 0xf, 0xf, false));
	v = max(v, __builtin_amdgcn_update_dpp(v, v, DSB_DPP_ROW_ROR(4), 0xf, 0xf, false));
	v = max(v, __builtin_amdgcn_update_dpp(v, v, DSB_DPP_ROW_ROR(8), 0xf, 0xf, false));
	return max(max(dsb_rdlane(v, 0), dsb_rdlane(v, 16)), max(dsb_rdlane(v, 32), dsb_rdlane(v, 48)));
}
/* exclusive prefix sum over the wave; *tot = sum over all lanes */
DSB_HD uint32_t dsb_wscan(uint32_t v, uint32_t *tot)
{
	int x = (int)v;
	x += __builtin_amdgcn_update_dpp(0, x, DSB_DPP_ROW_SHR(1), 0xf, 0xf, true);
	x += __builtin_amdgcn_update_dpp(0, x, DSB_DPP_ROW_SHR(2), 0xf, 0xf, true);
	x += __builtin_amdgcn_update_dpp(0, x, DSB_DPP_ROW_SHR(4), 0xf, 0xf, true);
	x += __builtin_amdgcn_update_dpp(0, x, DSB_DPP_ROW_SHR(8), 0xf, 0xf, true);
	uint32_t r0 = (uint32_t)dsb_rdlane(x, 15), r1 = (uint32_t)dsb_rdlane(x, 31), r2 = (uint32_t)dsb_rdlane(x, 47),
		 r3 = (uint32_t)dsb_rdlane(x, 63);
	uint32_t row = __lane_id() >> 4;
	uint32_t add = (row > 0 ? r0 : 0) + (row > 1 ? r1 : 0) + (row > 2 ? r2 : 0);
	*tot = r0 + r1 + r2 + r3;
	return (uint32_t)x + add - v;
}
DSB_HD uint64_t dsb_wmax64(uint64_t v)
{
	for (int o = 32; o; o >>= 1) {
		uint32_t lo = __shfl_xor((uint32_t)v, o), hi = __shfl_xor((uint32_t)(v >> 32), o);
		uint64_t u = ((uint64_t)hi << 32) | lo;
		v = u > v ? u : v;
	}
	return v;
}
DSB_HD uint64_t dsb_wballot(int p) { return __ballot(p); }
/* the lane of the k-th (0-based) set bit of a wave mask m (k < popcount(m)) */
DSB_HD uint32_t dsb_select64(uint64_t m, uint32_t k)
{
	uint32_t pos = 0;
	for (uint32_t w = 32; w; w >>= 1) {
		uint32_t c = (uint32_t)__builtin_popcountll(m & ((1ull << w) - 1));
		if (k >= c) {
			k -= c;
			m >>= w;
			pos += w;
		}
	}
	return pos;
}
/* *p = max(*p, v) on workgroup-local memory, from any lane */
DSB_HD void dsb_lds_max(int32_t *p, int32_t v) { atomicMax(p, v); }
/* value of lane `src` for a per-lane src (ds_bpermute) */
DSB_HD int dsb_wshfl_any(int v, int src) { return __shfl(v, src); }
/* value of lane `src`; src must be wave-uniform (v_readlane) */
DSB_HD int dsb_wshfl(int v, int src) { return dsb_rdlane(v, src); }
/*
 * Groups of G lanes (G = 16, 32 or 64) that each work on a read of their own (the seeding state
 * machine with DSB_SM_G lanes per read).  Masks are group-local (bit i = lane i of the group), and
 * the helpers work in divergent code as long as a group's lanes are all active or all inactive.
 */
template <int G> DSB_HD uint32_t dsb_glane(void) { return __lane_id() & (G - 1); }
template <int G> DSB_HD uint32_t dsb_gbase(void) { return __lane_id() & (64 - G); }
template <int G> DSB_HD uint64_t dsb_gballot(int p)
{
	uint64_t b = __ballot(p);
	return G == 64 ? b : (b >> dsb_gbase<G>()) & ((1ull << (G & 63)) - 1);
}
/* value of lane q of the group (q the same in the whole group) */
template <int G> DSB_HD int dsb_gshfl(int v, int q)
{
	if (G == 64)
		return dsb_rdlane(v, q);
	if (G == 32) { /* two readlanes (a uniform q, as the loops of both groups run in step) */
		int a = dsb_rdlane(v, q), b = dsb_rdlane(v, 32 + q);
		return __lane_id() < 32 ? a : b;
	}
	return __shfl(v, (int)dsb_gbase<G>() + q);
}
/* value of lane src of the group, src per lane */
template <int G> DSB_HD int dsb_gshfl_any(int v, int src) { return __shfl(v, (int)dsb_gbase<G>() + src); }
/* exclusive prefix sum over the group; *tot = the group's sum */
template <int G> DSB_HD uint32_t dsb_gscan(uint32_t v, uint32_t *tot)
{
	if (G == 64)
		return dsb_wscan(v, tot);
	int x = (int)v;
	x += __builtin_amdgcn_update_dpp(0, x, DSB_DPP_ROW_SHR(1), 0xf, 0xf, true);
	x += __builtin_amdgcn_update_dpp(0, x, DSB_DPP_ROW_SHR(2), 0xf, 0xf, true);
	x += __builtin_amdgcn_update_dpp(0, x, DSB_DPP_ROW_SHR(4), 0xf, 0xf, true);
	x += __builtin_amdgcn_update_dpp(0, x, DSB_DPP_ROW_SHR(8), 0xf, 0xf, true);
	uint32_t r0 = (uint32_t)dsb_rdlane(x, 15), r1 = (uint32_t)dsb_rdlane(x, 31), r2 = (uint32_t)dsb_rdlane(x, 47),
		 r3 = (uint32_t)dsb_rdlane(x, 63);
	uint32_t row = __lane_id() >> 4, add = 0;
	if (G == 32) {
		uint32_t hi = row >> 1;
		add = (row & 1) ? (hi ? r2 : r0) : 0;
		*tot = hi ? r2 + r3 : r0 + r1;
	} else { /* G == 16: one row */
		*tot = row == 0 ? r0 : row == 1 ? r1 : row == 2 ? r2 : r3;
	}
	return (uint32_t)x + add - v;
}
#else
#define DSB_WV 1
DSB_HD uint32_t dsb_lane(void) { return 0; }
template <int G> DSB_HD uint32_t dsb_glane(void) { return 0; }
template <int G> DSB_HD uint32_t dsb_gbase(void) { return 0; }
template <int G> DSB_HD uint64_t dsb_gballot(int p) { return p ? 1 : 0; }
template <int G> DSB_HD int dsb_gshfl(int v, int q) { (void)q; return v; }
template <int G> DSB_HD int dsb_gshfl_any(int v, int src) { (void)src; return v; }
template <int G> DSB_HD uint32_t dsb_gscan(uint32_t v, uint32_t *tot) { *tot = v; return 0; }
DSB_HD void dsb_wsync(void) {}
DSB_HD int dsb_wmax(int v) { return v; }
DSB_HD uint32_t dsb_wscan(uint32_t v, uint32_t *tot) { *tot = v; return 0; }
DSB_HD uint64_t dsb_wmax64(uint64_t v) { return v; }
DSB_HD uint64_t dsb_wballot(int p) { return p ? 1 : 0; }
DSB_HD int dsb_wshfl(int v, int src) { (void)src; return v; }
DSB_HD int dsb_wshfl_any(int v, int src) { (void)src; return v; }
DSB_HD uint32_t dsb_select64(uint64_t m, uint32_t k) { (void)m; (void)k; return 0; }
DSB_HD void dsb_lds_max(int32_t *p, int32_t v) { if (v > *p) *p = v; }
#endif

#endif
