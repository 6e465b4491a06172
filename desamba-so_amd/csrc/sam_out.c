/*
 * sam_out.c — record formatting with the reference's byte layout.
 *
 *   SAM / SAM_FULL  output_one_result_sam   (src/cly_mt.c:229-327)
 *   DES             output_one_result_des   (src/cly_mt.c:144-185, print_hit :47-92)
 *   DES_FULL        output_one_result_full  (src/cly_mt.c:187-227)
 *
 * The reference prints uint32 fields with "%d" (negative soft clips such as "-3S" when
 * q_ed > read length); the same integer widths are used here.
 */
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "dsb_host.h"

void dsb_str_put(dsb_str *s, const char *p, uint64_t n)
{
	if (s->l + n + 1 > s->m) {
		uint64_t m = s->m ? s->m : 4096;
		while (m < s->l + n + 1) m <<= 1;
		s->s = realloc(s->s, m);
		s->m = m;
	}
	memcpy(s->s + s->l, p, n);
	s->l += n;
	s->s[s->l] = 0;
}

void dsb_str_printf(dsb_str *s, const char *fmt, ...)
{
	char tmp[1024];
	va_list ap;
	va_start(ap, fmt);
	int n = vsnprintf(tmp, sizeof(tmp), fmt, ap);
	va_end(ap);
	if (n < 0) return;
	if ((size_t)n < sizeof(tmp)) {
		dsb_str_put(s, tmp, (uint64_t)n);
		return;
	}
	char *big = malloc((size_t)n + 1);
	va_start(ap, fmt);
	vsnprintf(big, (size_t)n + 1, fmt, ap);
	va_end(ap);
	dsb_str_put(s, big, (uint64_t)n);
	free(big);
}

static void put_cstr(dsb_str *s, const char *p)
{
	dsb_str_put(s, p, strlen(p));
}

static const char *primary_string[3] = {"PRI", "SEC", "SUP"};

static void print_hit(dsb_str *out, const dsb_hit_out_t *c, const dsb_index *ix, int rst_cnt)
{
	dsb_str_printf(out, "%3d %s %s %20s ts:%-10d te:%-10d qs:%-10d qe:%-10d %-5d\t%d\t\n",
		       rst_cnt, primary_string[(c->primary - 1) % 3], c->direction ? "F" : "R",
		       ix->ref_name[c->ref_ID], (int)c->t_st, (int)c->t_ed, (int)c->q_st, (int)c->q_ed,
		       (int)c->sum_score, (int)c->indel);
}

void dsb_format_read(dsb_str *out, const dsb_index *ix, const dsb_reads_t *r, uint64_t i,
		     const dsb_read_out_t *ro, const dsb_hit_out_t *hits, int format, int max_sec_N)
{
	const dsb_rec_t *rec = r->rec + i;
	/* the strings are views (not NUL-terminated): printed as %s prints them */
	const char *name = rec->name;
	uint64_t name_n = dsb_cstr_len(rec->name, rec->name_l);
	if (format == DSB_OUT_DES || format == DSB_OUT_DES_FULL) {
		dsb_str_put(out, name, name_n);
		dsb_str_printf(out, "\t%s\t%s\t%ld\tn_rst:[%ld]\tn_anc:[%ld]\t\n",
			       ro->n_hit ? "CLASSIFY" : "UNCLASSIFY", ro->fast ? "FAST" : "SLOW",
			       (long)rec->seq_l, (long)ro->n_hit, (long)ro->n_anchor);
		int rst_cnt = 0;
		for (uint32_t k = 0; k < ro->n_hit; k++)
			if (hits[k].pri_index == 0)
				print_hit(out, hits + k, ix, rst_cnt++);
		for (uint32_t k = 0; k < ro->n_hit; k++)
			if (hits[k].pri_index > 0 && (format == DSB_OUT_DES_FULL || hits[k].pri_index <= max_sec_N))
				print_hit(out, hits + k, ix, rst_cnt++);
		put_cstr(out, "\n");
		return;
	}
	int full = format == DSB_OUT_SAM_FULL;
	const char *seq_s = "*", *qual_s = "*";
	uint64_t seq_n = 1, qual_n = 1;
	if (full) {
		seq_s = rec->seq;
		seq_n = dsb_cstr_len(rec->seq, rec->seq_l);
		if (rec->qual) {
			qual_s = rec->qual;
			qual_n = dsb_cstr_len(rec->qual, rec->qual_l);
		} else {
			qual_s = "(null)";
			qual_n = 6;
		}
	}
	if (ro->n_hit == 0) {
		dsb_str_put(out, name, name_n);
		put_cstr(out, "\t4\t*\t0\t0\t*\t*\t0\t0\t");
		dsb_str_put(out, seq_s, seq_n);
		put_cstr(out, "\t");
		dsb_str_put(out, qual_s, qual_n);
		put_cstr(out, "\t\n");
		return;
	}
	uint32_t read_l = rec->seq_l;
	const dsb_hit_out_t *c_s = hits;
	int flag = c_s->direction ? 0 : 0x10;
	int mapQ_PRI;
	if (ro->n_hit == 1 || (uint32_t)(c_s->sum_score - c_s[1].sum_score) > 5)
		mapQ_PRI = 30;
	else
		mapQ_PRI = (int)((uint32_t)(c_s->sum_score - c_s[1].sum_score) << 2);
	dsb_str_put(out, name, name_n);
	dsb_str_printf(out, "\t%d\t%s\t%d\t%d\t%dS%dM%dS\t*\t0\t0\t", flag, ix->ref_name[c_s->ref_ID],
		       (int)c_s->t_st, mapQ_PRI, (int)c_s->q_st, (int)(c_s->q_ed - c_s->q_st),
		       (int)(read_l - c_s->q_ed));
	dsb_str_put(out, seq_s, seq_n);
	put_cstr(out, "\t");
	dsb_str_put(out, qual_s, qual_n);
	dsb_str_printf(out, "\tAS:i:%d\t\n", (int)c_s->sum_score);
	for (int loop = 0; loop <= 1; loop++) {
		for (uint32_t k = 1; k < ro->n_hit; k++) {
			const dsb_hit_out_t *c = hits + k;
			int show = 0;
			int fl = c->direction ? 0 : 0x10;
			int mapQ = 0;
			if (loop == 0 && c->pri_index == 0) {
				show = 1;
				fl += 0x800;
				mapQ = mapQ_PRI < 30 ? mapQ_PRI : 30;
			} else if (loop == 1 && c->pri_index > 0 && c->pri_index <= max_sec_N) {
				show = 1;
				fl += 0x100;
			}
			if (!show) continue;
			dsb_str_put(out, name, name_n);
			dsb_str_printf(out, "\t%d\t%s\t%d\t%d\t%d%c%dM%d%c\t*\t0\t0\t*\t*\tAS:i:%d\t\n", fl,
				       ix->ref_name[c->ref_ID], (int)c->t_st, mapQ, (int)c->q_st, loop == 0 ? 'H' : 'S',
				       (int)(c->q_ed - c->q_st), (int)(read_l - c->q_ed), loop == 0 ? 'H' : 'S',
				       (int)c->sum_score);
		}
	}
}
