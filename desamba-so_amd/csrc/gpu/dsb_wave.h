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
#define DSB_WV 64
DSB_HD uint32_t dsb_lane(void) { return __lane_id(); }
DSB_HD void dsb_wsync(void) { __syncthreads(); }
DSB_HD int dsb_wmax(int v)
{
	for (int o = 32; o; o >>= 1)
		v = max(v, __shfl_xor(v, o));
	return v;
}
/* exclusive prefix sum over the wave; *tot = sum over all lanes */
DSB_HD uint32_t dsb_wscan(uint32_t v, uint32_t *tot)
{
	uint32_t lane = __lane_id(), x = v;
	for (int o = 1; o < 64; o <<= 1) {
		uint32_t y = __shfl_up(x, o);
		if (lane >= (uint32_t)o)
			x += y;
	}
	*tot = __shfl(x, 63);
	return x - v;
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
DSB_HD int dsb_wshfl(int v, int src) { return __shfl(v, src); }
#else
#define DSB_WV 1
DSB_HD uint32_t dsb_lane(void) { return 0; }
DSB_HD void dsb_wsync(void) {}
DSB_HD int dsb_wmax(int v) { return v; }
DSB_HD uint32_t dsb_wscan(uint32_t v, uint32_t *tot) { *tot = v; return 0; }
DSB_HD uint64_t dsb_wmax64(uint64_t v) { return v; }
DSB_HD uint64_t dsb_wballot(int p) { return p ? 1 : 0; }
DSB_HD int dsb_wshfl(int v, int src) { (void)src; return v; }
#endif

#endif
