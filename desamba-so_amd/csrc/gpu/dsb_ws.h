/*
 * dsb_ws.h — per-read workspace layout in HBM.
 *
 * One contiguous arena per read, carved into 256-B aligned regions.  The host computes
 * each read's arena size and offset (prefix sum over the batch); the kernels carve the
 * same pointers from (base + offset).  Capacities of the dynamic vectors scale with read
 * length; a read that overflows one is re-run with DSB_CAP_RETRY x larger capacities.
 */
#ifndef DSB_WS_H
#define DSB_WS_H
#include "dsb_classify.h"

#define DSB_BIN_GUARD 64   /* bytes before F: the last 8 = glibc chunk header of the reference buffer */
#define DSB_BIN_TAIL 256   /* bytes after R, MALLOC_PERTURB fill */
static_assert(DSB_BIN_TAIL == DSB_BIN_TAIL_BYTES, "the scoring's read-range copy bound (dsb_classify.h)");
#define DSB_STATE_BYTES 128
#define DSB_CAP_RETRY 8
#define DSB_SCALE_UNIT 8   /* capacity scale is fixed point: DSB_SCALE_UNIT = the default capacities */

DSB_HD uint64_t dsb_al(uint64_t x) { return (x + 255) & ~255ull; }

/* the read hash's key bits, which size its head tables: the GPU build's scoring looks the hash up
 * as k_hash_lds built it, at most DSB_HASH_LDS_KL bits (dsb_build_hash_table); the CPU emulator and
 * the lane-per-read phase kernels build it themselves at dsb_hash_kl bits */
#ifndef DSB_WS_HASH_LDS
#define DSB_WS_HASH_LDS DSB_HSET_POOL
#endif
DSB_HD int dsb_key_len(uint32_t q_len)
{
	return DSB_WS_HASH_LDS && dsb_hash_lds_read(q_len) ? dsb_hash_kl_lds(q_len) : dsb_hash_kl(q_len);
}

DSB_HD dsb_caps_t dsb_default_caps(uint32_t L, uint32_t scale)
{
	dsb_caps_t c;
	c.anc = (uint32_t)(((uint64_t)(1024 + (L >> 2)) * scale) / DSB_SCALE_UNIT);
	c.hit = c.anc;
	c.sms = (uint32_t)(((uint64_t)(2048 + (L >> 1)) * scale) / DSB_SCALE_UNIT);
	return c;
}

DSB_HD uint32_t dsb_ex_words(uint32_t L) { return (L >> 6) + 2; }
DSB_HD uint32_t dsb_seed_cap(uint32_t L) { return (L >> 1) + 20 + L / 3 + 64; }

typedef struct {
	uint64_t bin, exF, exR, pre, seeds, anc, anc_tmp, anc_tmp2, sidx, stmp, hit, hit_tmp, sms, hash, sch, win, mem, spset, hset, state, total;
	uint32_t kl;
} dsb_ws_layout;

DSB_HD dsb_ws_layout dsb_layout(uint32_t L, dsb_caps_t cap)
{
	dsb_ws_layout o;
	uint64_t p = 0;
	uint32_t sortn = DSB_MAX(DSB_MAX(cap.anc, cap.hit), 1024u);
	o.bin = p; p = dsb_al(p + DSB_BIN_GUARD + 2ull * L + DSB_BIN_TAIL);
	o.exF = p; p = dsb_al(p + 8ull * dsb_ex_words(L));
	o.exR = p; p = dsb_al(p + 8ull * dsb_ex_words(L));
	o.pre = p; p = dsb_al(p + 8ull * L); /* u32 13-mer prefix value per k-mer position, F then R */
	o.seeds = p; p = dsb_al(p + sizeof(dsb_seed_t) * (uint64_t)dsb_seed_cap(L));
	o.anc = p; p = dsb_al(p + sizeof(dsb_anchor_t) * (uint64_t)cap.anc);
	o.anc_tmp = p; p = dsb_al(p + DSB_MAX(sizeof(dsb_anchor_t) * (uint64_t)cap.anc, sizeof(dsb_mem_t) * 256ull));
	o.anc_tmp2 = p; p = dsb_al(p + sizeof(dsb_anchor_t) * (uint64_t)cap.anc);
	o.sidx = p; p = dsb_al(p + 4ull * sortn);
	o.stmp = p; p = dsb_al(p + 4ull * sortn);
	o.hit = p; p = dsb_al(p + sizeof(dsb_chain_t) * (uint64_t)cap.hit);
	o.hit_tmp = p; p = dsb_al(p + sizeof(dsb_chain_t) * (uint64_t)cap.hit);
	o.sms = p; p = dsb_al(p + sizeof(dsb_spd_t) * (uint64_t)cap.sms);
	o.kl = (uint32_t)dsb_key_len(L);
	o.hash = p; p = dsb_al(p + 2ull * (4ull * (1ull << o.kl) + 4ull * L)); /* per strand: heads + nodes */
	o.sch = p; p = dsb_al(p + sizeof(dsb_sch_t) * (256 + 2 * 400 + 64) + 2 * (DSB_SC_OFF_U16 + DSB_SC_FLAT_U16));
	o.win = p; p = dsb_al(p + DSB_WIN_BYTES);
	o.mem = p; p = dsb_al(p + sizeof(dsb_mem_t) * 16 * 64); /* 16 MEM results per lane (slow seeding) */
	o.spset = p; p = dsb_al(p + 8 * 512);
	o.hset = p; p = dsb_al(p + (DSB_HSET_POOL ? 0 : 8ull * DSB_HSET_WAVE_U64)); /* per-lane sp_set hashes (else the pool) */
	o.state = p; p = dsb_al(p + DSB_STATE_BYTES); /* dsb_rstate_t: state between phase launches */
	o.total = p;
	return o;
}

/* carve the workspace of one read */
DSB_HD void dsb_ws_init(dsb_read_ws *w, const dsb_dindex_t *ix, uint8_t *base, uint32_t L, dsb_caps_t cap)
{
	dsb_ws_layout o = dsb_layout(L, cap);
	w->ix = ix;
	w->L = L;
	w->bin = base + o.bin + DSB_BIN_GUARD;
	w->exF = (const uint64_t *)(base + o.exF);
	w->exR = (const uint64_t *)(base + o.exR);
	w->pre = (const uint32_t *)(base + o.pre);
	w->seeds = (dsb_seed_t *)(base + o.seeds);
	w->anc = (dsb_anchor_t *)(base + o.anc);
	w->n_anc = 0;
	w->anc_hw = 0;
	w->anc_tmp = (dsb_anchor_t *)(base + o.anc_tmp);
	w->anc_tmp2 = (dsb_anchor_t *)(base + o.anc_tmp2);
	w->sidx = (uint32_t *)(base + o.sidx);
	w->stmp = (uint32_t *)(base + o.stmp);
	w->hit = (dsb_chain_t *)(base + o.hit);
	w->n_hit = 0;
	w->hit_tmp = (dsb_chain_t *)(base + o.hit_tmp);
	w->sms = (dsb_spd_t *)(base + o.sms);
	w->n_sms = 0;
	w->sms_lds = 0;
	w->lds_key = 0;
	w->lds_id = 0;
	w->lds_n = 0;
	w->lds_hb = 0;
	w->lds_cand = 0;
	w->lds_q = 0;
	w->spec_ch = 0;
	w->spec_bits = 0;
	uint32_t *h = (uint32_t *)(base + o.hash);
	uint64_t hs = 1ull << o.kl;
	for (int s = 0; s < 2; s++) {
		w->hh[s] = h; h += hs;
		w->hn[s] = h; h += L;
	}
	w->sch = (dsb_sch_t *)(base + o.sch);
	w->sc_off = (uint16_t *)(w->sch + 256 + 2 * 400 + 64);
	w->sc_flat = w->sc_off + DSB_SC_OFF_U16;
	w->win = base + o.win;
	w->mem = (dsb_mem_t *)(base + o.mem);
	w->spset = (uint64_t *)(base + o.spset);
	w->cap = cap;
	w->overflow = 0;
	w->fast_classify = 1;
	w->max_read_l = 0;
	w->reached_update = 0;
	w->stats = 0;
	w->dbg = 0;
	w->launch_tag = 1;
	w->tmr = 0;
}

/* glibc chunk-size word in front of the reference's bin_read = realloc(NULL, 2L+20)
 * (BUFF_REALLOC, src/lib/utils.h:117-122): read by backward extensions past F[0] (H3). */
DSB_HD uint64_t dsb_chunk_header(uint32_t L)
{
	uint64_t req = 2ull * L + 20;
	uint64_t chunk = (req + 8 + 15) & ~15ull;
	if (chunk < 32)
		chunk = 32;
	return chunk | 1; /* PREV_INUSE, main arena */
}

/* Fill the read buffer guards; bases are written separately (encode kernel). */
DSB_HD void dsb_bin_guards(uint8_t *bin, uint32_t L)
{
	uint64_t hdr = dsb_chunk_header(L);
	for (int k = 0; k < 8; k++)
		bin[-8 + k] = (uint8_t)(hdr >> (8 * k));
	for (int k = 9; k <= DSB_BIN_GUARD; k++)
		bin[-k] = DSB_HEAP_PERTURB;
	for (uint32_t k = 0; k < DSB_BIN_TAIL; k++)
		bin[2ull * L + k] = DSB_HEAP_PERTURB;
}

#endif
