/*
 * phase.hip — one phase kernel of classify part A per translation unit: compiled once per
 * phase with -DDSB_PH=<n> (desamba-so_amd/Makefile), so the nine phases build in parallel
 * and each gets its own register allocation.  kernels.hip obtains the kernel through
 * dsb_phase_kernel_<n>(wave, stats).
 *
 * Phase 0 (island scan) runs 2 x DSB_ISLAND_G lanes per read (k_island_g); phases 1-8 run one wavefront per read.  The
 * lane-per-read variants of phases 1-8 are diagnostics only (DSB_WAVE_PHASES) and are
 * compiled in with -DDSB_LANE_PHASES=1.
 */
#include "dsb_kern.h"

#ifndef DSB_PH
#error "compile with -DDSB_PH=<phase number>"
#endif
#ifndef DSB_LANE_PHASES
#define DSB_LANE_PHASES 0
#endif
#define DSB_CAT_(a, b) a##b
#define DSB_CAT(a, b) DSB_CAT_(a, b)

extern "C" dsb_phase_fn DSB_CAT(dsb_phase_kernel_, DSB_PH)(int wave, int stats)
{
#if DSB_PH == 0
	(void)wave;
#if DSB_ISLAND_G > 0 /* 2 x DSB_ISLAND_G lanes per read, probing the Bloom tables itself */
	return stats == 1 ? k_island_g<DSB_ISLAND_G, 1> : k_island_g<DSB_ISLAND_G, 0>;
#else /* two lanes per read over k_seed's exist bits; launched with 2 x reads threads */
	return stats == 1 ? k_island<1> : (stats == 2 ? k_island<2> : k_island<0>);
#endif
#else
	if (wave)
		return stats == 1 ? k_wave_phase<DSB_PH, 1> : (stats == 2 ? k_wave_phase<DSB_PH, 2> : k_wave_phase<DSB_PH, 0>);
#if DSB_LANE_PHASES && DSB_WS_HASH_LDS
#error "lane-per-read phases build the read hash at dsb_hash_kl bits: add -DDSB_WS_HASH_LDS=0"
#endif
#if DSB_LANE_PHASES
	return stats == 1 ? k_phase<DSB_PH, 1> : (stats == 2 ? k_phase<DSB_PH, 2> : k_phase<DSB_PH, 0>);
#else
	return nullptr;
#endif
#endif
}

#if DSB_PH == 8
static_assert(DSB_PH_DELA == 8, "the heavy reads' scoring kernels live in the scoring phase's unit");
/* the heavy reads' scoring (dsb_kern.h k_heavy_*), for kernels.hip run_split */
extern "C" void dsb_heavy_kernels(dsb_heavy_prep_fn *prep, dsb_heavy_spec_fn *spec, dsb_heavy_fin_fn *fin)
{
	*prep = k_heavy_prep<0>;
	*spec = k_heavy_spec<0>;
	*fin = k_heavy_fin<0>;
}
#endif
