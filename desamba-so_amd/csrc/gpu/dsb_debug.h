/*
 * dsb_debug.h — print one read's workspace (seeds, anchors, chains) in the stage-dump format
 * of oracle/harness_ref.c, for diagnosing parity failures (host-side, after a D2H copy).
 */
#ifndef DSB_DEBUG_H
#define DSB_DEBUG_H
#include <stdio.h>
#include "dsb_classify.h"

static inline void dsb_debug_dump(FILE *f, const dsb_read_ws *w, const char *tag)
{
	fprintf(f, "# %s L=%u n_anc=%u n_hit=%u fast=%u overflow=%u reached=%u\n", tag, w->L, w->n_anc, w->n_hit,
		w->fast_classify, w->overflow, w->reached_update);
	for (int s = 0; s < 2; s++) {
		const dsb_sdir_t *sd = w->sd + s;
		fprintf(f, "S %d %u %u %u\n", s, sd->direction, sd->l_seed_v_f, sd->total_score);
		for (uint32_t i = 0; i < sd->l_seed_v_f; i++) {
			const dsb_seed_t *x = w->seeds + sd->seed_off + i;
			fprintf(f, "s %u %u %u\n", x->offset, x->len, (unsigned)x->top);
		}
	}
	for (int s = 0; s < 2; s++) { /* the seeding state machine's per-seed records (dsb_seed_sm: rec, klist,
	                                 * tix, hand in the read-hash region) as the last seeding phase left
	                                 * them, read with either strand's seed count */
		uint32_t m = w->sd[s].l_seed_v_f;
		const uint32_t *rec = w->hh[0];
		for (uint32_t q = 0; q < m; q++)
			fprintf(f, "r%d %u %08x %08x %u %u %u\n", s, q, rec[2 * q], rec[2 * q + 1], rec[2 * m + q], rec[3 * m + q],
				rec[4 * m + q]);
	}
	fprintf(f, "A %s %u\n", tag, w->n_anc);
	for (uint32_t i = 0; i < w->n_anc; i++) {
		const dsb_anchor_t *a = w->anc + i;
		fprintf(f, "a %u %u %u %u %lu %u %d %u %u %u %u %u %u %u\n", (unsigned)a->direction, a->ref_ID, a->ref_offset,
			a->index_in_read, (unsigned long)a->global_offset, (unsigned)a->mtch_len, (int)a->score,
			(unsigned)a->left_len, (unsigned)a->left_ED, (unsigned)a->rigt_len, (unsigned)a->rigt_ED,
			(unsigned)a->seed_ID, (unsigned)a->anchor_useless, (unsigned)a->duplicate);
	}
	fprintf(f, "H %s %u\n", tag, w->n_hit);
	for (uint32_t i = 0; i < w->n_hit; i++) {
		const dsb_chain_t *c = w->hit + i;
		fprintf(f, "h %u %u %d %u %u %u %u %u %u %u %u %u %u\n", c->ref_ID, (unsigned)c->direction, c->q_t_dis,
			c->sum_score, c->anchor_number, (unsigned)c->with_top_anchor, c->t_st, c->t_ed, c->q_st, c->q_ed,
			c->indel, (unsigned)c->primary, (unsigned)c->pri_index);
	}
}
#endif
