/*
 * tests/emu/emu_classify.cpp — TEST-ONLY kernel-logic emulation.
 *
 * Runs the exact per-read device code of desamba-so_amd/csrc/gpu/dsb_classify.h on the
 * host CPU, one read after the other, so that the classify logic can be checked against
 * the reference oracle in a container without a GPU.  It is never linked into
 * libdesamba.so (whose classify path exists only as HIP kernels) and never used by
 * bench.py's timed leg.
 *
 * usage: emu_classify [--stats] [--des|--sam] <index_dir> <reads.fq>  > out.sam
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#ifdef DSB_EMU_PROF /* emu_prof: per-seed state-machine trips (tools/seed_prof.py) */
#include <stdint.h>
struct emu_prof_seed { uint32_t k; uint64_t trips, maps; };
static std::vector<emu_prof_seed> g_prof[2];
static void dsb_emu_prof_seed(int slow, uint32_t k, uint64_t trips, uint64_t maps)
{
	g_prof[slow ? 1 : 0].push_back({k, trips, maps});
}
/* sp_set inserts by the set's fill at the time (l = entries since the last reset / wrap) */
static uint64_t g_ins_hist[512];
static void dsb_emu_prof_insert(int l) { g_ins_hist[l < 512 ? l : 511]++; }
#endif
extern "C" {
#include "../../desamba-so_amd/csrc/dsb_host.h"
}
#include "../../desamba-so_amd/csrc/gpu/dsb_ws.h"
#include "../../desamba-so_amd/csrc/gpu/dsb_debug.h"

int main(int argc, char **argv)
{
	int ai = 1, stats = 0, fmt = DSB_OUT_SAM_FULL;
	for (; ai < argc && argv[ai][0] == '-'; ai++) {
		if (!strcmp(argv[ai], "--stats")) stats = 1;
		else if (!strcmp(argv[ai], "--des")) fmt = DSB_OUT_DES;
		else if (!strcmp(argv[ai], "--sam")) fmt = DSB_OUT_SAM;
		else { fprintf(stderr, "unknown option %s\n", argv[ai]); return 2; }
	}
	if (ai + 2 > argc) {
		fprintf(stderr, "usage: %s [--stats] [--des|--sam] <index_dir> <reads>\n", argv[0]);
		return 2;
	}
	static dsb_index ix;
	memset(&ix, 0, sizeof(ix));
	char err[512];
	if (dsb_index_load_files(&ix, argv[ai], err, sizeof(err))) {
		fprintf(stderr, "%s\n", err);
		return 1;
	}
	ix.filter_min_length = 170;
	ix.filter_min_score = 64;
	ix.filter_min_score_LV3 = 74;
	dsb_mapq_tables(&ix, 0.15, ix.ref_bin_n * 4);
	dsb_dindex_t d;
	dsb_index_host_view(&ix, &d);

	char *buf;
	uint64_t len;
	if (dsb_slurp_path(argv[ai + 1], &buf, &len)) {
		fprintf(stderr, "cannot read %s\n", argv[ai + 1]);
		return 1;
	}
	dsb_reads_t reads;
	memset(&reads, 0, sizeof(reads));
	dsb_parse_reads(buf, len, &reads);

	int max_read_l = 0;
	std::vector<uint8_t> arena;
	dsb_str out = {0, 0, 0};
	std::vector<dsb_hit_out_t> hits(400);
	uint64_t st[DSB_ST_N];
	memset(st, 0, sizeof(st));
	uint64_t n_retry = 0;
	for (uint64_t i = 0; i < reads.n; i++) {
		uint32_t L = reads.rec[i].seq_l;
		const uint8_t *seq = (const uint8_t *)reads.rec[i].seq;
		dsb_read_out_t ro;
		for (uint32_t scale = DSB_SCALE_UNIT;; scale *= DSB_CAP_RETRY) {
			dsb_caps_t cap = dsb_default_caps(L, scale);
			dsb_ws_layout lay = dsb_layout(L, cap);
			arena.assign(lay.total + 256, (uint8_t)(getenv("EMU_FILL") ? strtol(getenv("EMU_FILL"), 0, 0) : 0xEE));
			dsb_read_ws w;
			dsb_ws_init(&w, &d, arena.data(), L, cap);
			if (stats) w.stats = st;
			if (getenv("EMU_DBG")) w.dbg = (uint32_t)strtoul(getenv("EMU_DBG"), 0, 0);
			/* encode (CLY_Bit) + reverse complement + guards (src/cly.c:1245-1254) */
			for (uint32_t k = 0; k < L; k++) w.bin[k] = dsb_cly_bit(seq[k]);
			for (uint32_t k = 0; k < L; k++) w.bin[L + L - 1 - k] = 3 - w.bin[k];
			dsb_bin_guards(w.bin, L);
			/* exist bits (K_seed) */
			if (L >= DSB_MIN_READ_LEN) {
				uint32_t lk = L - d.l_ek + 1;
				uint64_t *ex[2] = {(uint64_t *)w.exF, (uint64_t *)w.exR};
				for (int s = 0; s < 2; s++) {
					memset(ex[s], 0, 8 * dsb_ex_words(L));
					for (uint32_t k = 0; k < lk; k++) {
						uint64_t km = dsb_kmer_at(w.bin + s * L + k, d.l_ek, d.single_base_max);
						((uint32_t *)w.pre)[s * L + k] = (uint32_t)(km & DSB_PRE_IDX_MASK);
						if (dsb_exist_kmer(&d, km)) ex[s][k >> 6] |= 1ull << (k & 63);
					}
				}
			}
			static uint8_t lds_win[DSB_WIN_BYTES + DSB_HB_LDS + 64];
			static dsb_spd_t lds_sms[DSB_SMS_LDS];
			if (getenv("EMU_LDS")) { /* the scoring kernel's LDS layout (separate window / sms prefix) */
				int fill = (int)strtol(getenv("EMU_LDS"), 0, 0); /* garbage left by other workgroups */
				memset(lds_win, fill, sizeof(lds_win));
				memset(lds_sms, fill, sizeof(lds_sms));
				w.win = lds_win; /* the scoring kernel's windows share their LDS with the hash-build slots */
				w.lds_hb = lds_win;
				w.sms_lds = lds_sms;
			}
			if (getenv("EMU_WAVE")) { /* the wave-cooperative code paths, as a one-lane wave */
				dsb_rflags_t f = {0, 0, 0, 0};
				/* one sp_set table for all reads, never cleared, as a set of the GPU's pool
				 * (dsb_kern.h dsb_hpool_release): only its moving generation base keeps it exact */
				static std::vector<uint64_t> hset_store(DSB_HSET_WAVE_U64, 0);
				static uint64_t gen_base = 0;
				uint64_t *hset = hset_store.data();
				/* the first-level table in LDS (garbage at workgroup start; dsb_hset_make clears it);
				 * EMU_HSET_L1=0: none, every entry in the pool set */
				static uint64_t hs_l1_store[DSB_HSET_L1];
				memset(hs_l1_store, 0xA7, sizeof(hs_l1_store));
				uint64_t *hs_l1 = (getenv("EMU_HSET_L1") && !atoi(getenv("EMU_HSET_L1"))) ? nullptr : hs_l1_store;
				for (int ph = 0; ph < DSB_PH_DELA; ph++) {
					if ((ph == DSB_PH_FAST0 || ph == DSB_PH_FAST1) && dsb_phase_active(&w, &f, ph)) {
						static int32_t sm_lds[2];
						gen_base += dsb_fast_classify_sm(&w, &w.sd[ph - DSB_PH_FAST0], hset, gen_base, sm_lds, hs_l1) + 1;
					} else if ((ph == DSB_PH_SLOW0 || ph == DSB_PH_SLOW1) && dsb_phase_active(&w, &f, ph)) {
						static int32_t sm_lds2[2];
						gen_base += dsb_slow_classify_sm(&w, &w.sd[ph == DSB_PH_SLOW0 ? 0 : 1], hset, gen_base, w.mem, sm_lds2, hs_l1) + 1;
					} else if (ph == DSB_PH_RESOLVE_F || ph == DSB_PH_RESOLVE_S0 || ph == DSB_PH_RESOLVE_S1) {
						/* the resolve kernels' LDS sort / M3 staging arrays (garbage between reads) */
						static uint64_t lds_key[DSB_SORT_LDS_SLOW];
						static uint32_t lds_id[DSB_SORT_LDS_SLOW];
						memset(lds_key, 0x5c, sizeof(lds_key));
						memset(lds_id, 0x5c, sizeof(lds_id));
						w.lds_key = lds_key;
						w.lds_id = lds_id;
						w.lds_n = ph == DSB_PH_RESOLVE_F ? DSB_SORT_LDS : DSB_SORT_LDS_SLOW; /* as dsb_kern.h */
						dsb_phase<true>(&w, &f, ph);
						w.lds_key = 0;
						w.lds_id = 0;
					} else
						dsb_phase<true>(&w, &f, ph);
				}
				dsb_phase<true>(&w, &f, DSB_PH_DELA);
			} else
				dsb_classify_A(&w);
#ifdef DSB_EMU_PROF
			if (scale == DSB_SCALE_UNIT) {
				printf("R %lu %u A %u %u", (unsigned long)i, L, (unsigned)w.n_anc, (unsigned)w.fast_classify);
				for (int sl = 0; sl < 2; sl++) {
					printf(" %s", sl ? "|S" : "|F");
					for (const emu_prof_seed &q : g_prof[sl]) printf(" %lu,%lu", (unsigned long)q.trips, (unsigned long)q.maps);
					g_prof[sl].clear();
				}
				printf("\n");
			}
#endif
			if (getenv("DSB_DEBUG_READ") && strtoull(getenv("DSB_DEBUG_READ"), 0, 10) == i)
				dsb_debug_dump(stderr, &w, "emuA");
			if (w.overflow) {
				n_retry++;
				continue;
			}
			int mrl = max_read_l;
			if (w.reached_update && (int)L > mrl) mrl = (int)L;
			dsb_classify_B(&w, mrl, &ro, hits.data(), 400);
			max_read_l = mrl;
			break;
		}
#ifndef DSB_EMU_PROF
		dsb_format_read(&out, &ix, &reads, i, &ro, hits.data(), fmt, 5);
#endif
		if (out.l > (1 << 24)) {
			fwrite(out.s, 1, out.l, stdout);
			out.l = 0;
		}
	}
	fwrite(out.s, 1, out.l, stdout);
#ifdef DSB_EMU_PROF
	printf("INSHIST");
	for (int k = 0; k < 512; k++) printf(" %lu", (unsigned long)g_ins_hist[k]);
	printf("\n");
#endif
	if (stats) {
		fprintf(stderr, "reads %lu retries %lu\n", (unsigned long)reads.n, (unsigned long)n_retry);
		const char *nm[DSB_ST_N] = {"occ", "occ_nib", "memsearch", "sa", "uni", "refpos", "getref_b", "anchor", "chain", "ek1", "ek2", "hash_b", "lookup", "node", "t_mem", "t_map"};
		for (int k = 0; k < DSB_ST_N; k++) fprintf(stderr, "%s %lu\n", nm[k], (unsigned long)st[k]);
	}
	return 0;
}
