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

/* fast appends for the SAM records (the bulk of read_classify's host time): capacity is reserved
 * once per read, then bytes and "%d" integers are written without further checks */
static void str_reserve(dsb_str *s, uint64_t n)
{
	if (s->l + n + 1 > s->m) {
		uint64_t m = s->m ? s->m : 4096;
		while (m < s->l + n + 1) m <<= 1;
		s->s = realloc(s->s, m);
		s->m = m;
	}
}

static inline void raw_put(dsb_str *s, const char *p, uint64_t n)
{
	memcpy(s->s + s->l, p, n);
	s->l += n;
}

static inline void raw_c(dsb_str *s, char c) { s->s[s->l++] = c; }

static inline void raw_d(dsb_str *s, int v) /* printf "%d" */
{
	char b[12];
	int n = 0;
	uint32_t u = v < 0 ? (uint32_t)0 - (uint32_t)v : (uint32_t)v;
	do {
		b[n++] = (char)('0' + u % 10);
		u /= 10;
	} while (u);
	if (v < 0)
		b[n++] = '-';
	char *d = s->s + s->l;
	for (int k = 0; k < n; k++) d[k] = b[n - 1 - k];
	s->l += n;
}

#define RAW_LIT(s, lit) raw_put((s), (lit), sizeof(lit) - 1)

/* SAM_FULL's SEQ and QUAL fields of a record: the views as "%s" prints them, "(null)" for a FASTA
 * record's missing quality (src/cly_mt.c:258-262) */
void dsb_sam_seq_qual(const dsb_rec_t *rec, const char **seq, uint64_t *seq_n, const char **qual, uint64_t *qual_n)
{
	*seq = rec->seq;
	*seq_n = dsb_cstr_len(rec->seq, rec->seq_l);
	if (rec->qual) {
		*qual = rec->qual;
		*qual_n = dsb_cstr_len(rec->qual, rec->qual_l);
	} else {
		*qual = "(null)";
		*qual_n = 6;
	}
}

/* SAM / SAM_FULL records of one read (output_one_result_sam, src/cly_mt.c:229-327).  hole != NULL
 * (SAM_FULL only): SEQ, the tab and QUAL are not written; *hole = the offset in out where those
 * hole_n bytes go (the caller composes them from the record views), so the bulk bytes are copied
 * once, straight into the final output. */
static void format_sam(dsb_str *out, const dsb_index *ix, const dsb_rec_t *rec, const dsb_read_out_t *ro,
		       const dsb_hit_out_t *hits, int full, int max_sec_N, uint64_t *hole, uint64_t *hole_n)
{
	const char *name = rec->name;
	uint64_t name_n = dsb_cstr_len(rec->name, rec->name_l);
	const char *seq_s = "*", *qual_s = "*";
	uint64_t seq_n = 1, qual_n = 1;
	if (full)
		dsb_sam_seq_qual(rec, &seq_s, &seq_n, &qual_s, &qual_n);
	int holed = hole != NULL && full;
	uint64_t body = holed ? 0 : seq_n + 1 + qual_n;
	if (holed)
		*hole_n = seq_n + 1 + qual_n;
	if (ro->n_hit == 0) {
		str_reserve(out, name_n + body + 64);
		raw_put(out, name, name_n);
		RAW_LIT(out, "\t4\t*\t0\t0\t*\t*\t0\t0\t");
		if (holed)
			*hole = out->l;
		else {
			raw_put(out, seq_s, seq_n);
			raw_c(out, '\t');
			raw_put(out, qual_s, qual_n);
		}
		RAW_LIT(out, "\t\n");
		out->s[out->l] = 0;
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
	const char *rn = ix->ref_name[c_s->ref_ID];
	uint64_t rn_n = strlen(rn);
	str_reserve(out, name_n + rn_n + body + 160);
	raw_put(out, name, name_n);
	raw_c(out, '\t');
	raw_d(out, flag);
	raw_c(out, '\t');
	raw_put(out, rn, rn_n);
	raw_c(out, '\t');
	raw_d(out, (int)c_s->t_st);
	raw_c(out, '\t');
	raw_d(out, mapQ_PRI);
	raw_c(out, '\t');
	raw_d(out, (int)c_s->q_st);
	raw_c(out, 'S');
	raw_d(out, (int)(c_s->q_ed - c_s->q_st));
	raw_c(out, 'M');
	raw_d(out, (int)(read_l - c_s->q_ed));
	RAW_LIT(out, "S\t*\t0\t0\t");
	if (holed)
		*hole = out->l;
	else {
		raw_put(out, seq_s, seq_n);
		raw_c(out, '\t');
		raw_put(out, qual_s, qual_n);
	}
	RAW_LIT(out, "\tAS:i:");
	raw_d(out, (int)c_s->sum_score);
	RAW_LIT(out, "\t\n");
	for (int loop = 0; loop <= 1; loop++) {
		for (uint32_t k = 1; k < ro->n_hit; k++) {
			const dsb_hit_out_t *c = hits + k;
			int fl = c->direction ? 0 : 0x10;
			int mapQ = 0;
			if (loop == 0 && c->pri_index == 0) {
				fl += 0x800;
				mapQ = mapQ_PRI < 30 ? mapQ_PRI : 30;
			} else if (loop == 1 && c->pri_index > 0 && c->pri_index <= max_sec_N) {
				fl += 0x100;
			} else
				continue;
			const char *r2 = ix->ref_name[c->ref_ID];
			uint64_t r2_n = strlen(r2);
			char hs = loop == 0 ? 'H' : 'S';
			str_reserve(out, name_n + r2_n + 128);
			raw_put(out, name, name_n);
			raw_c(out, '\t');
			raw_d(out, fl);
			raw_c(out, '\t');
			raw_put(out, r2, r2_n);
			raw_c(out, '\t');
			raw_d(out, (int)c->t_st);
			raw_c(out, '\t');
			raw_d(out, mapQ);
			raw_c(out, '\t');
			raw_d(out, (int)c->q_st);
			raw_c(out, hs);
			raw_d(out, (int)(c->q_ed - c->q_st));
			raw_c(out, 'M');
			raw_d(out, (int)(read_l - c->q_ed));
			raw_c(out, hs);
			RAW_LIT(out, "\t*\t0\t0\t*\t*\tAS:i:");
			raw_d(out, (int)c->sum_score);
			RAW_LIT(out, "\t\n");
		}
	}
	out->s[out->l] = 0;
}

void dsb_format_read_hole(dsb_str *out, const dsb_index *ix, const dsb_reads_t *r, uint64_t i, const dsb_read_out_t *ro,
			  const dsb_hit_out_t *hits, int format, int max_sec_N, uint64_t *hole, uint64_t *hole_n)
{
	const dsb_rec_t *rec = r->rec + i;
	if (hole)
		*hole = UINT64_MAX;
	if (format == DSB_OUT_DES || format == DSB_OUT_DES_FULL) {
		/* the strings are views (not NUL-terminated): printed as %s prints them */
		dsb_str_put(out, rec->name, dsb_cstr_len(rec->name, rec->name_l));
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
	format_sam(out, ix, rec, ro, hits, format == DSB_OUT_SAM_FULL, max_sec_N, hole, hole_n);
}

void dsb_format_read(dsb_str *out, const dsb_index *ix, const dsb_reads_t *r, uint64_t i,
		     const dsb_read_out_t *ro, const dsb_hit_out_t *hits, int format, int max_sec_N)
{
	dsb_format_read_hole(out, ix, r, i, ro, hits, format, max_sec_N, NULL, NULL);
}
