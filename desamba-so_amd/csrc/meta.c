/*
 * meta.c — host restatement of the reference's meta_analysis (src/cly_mt.c:590-1413).
 *
 * Input is the SAM text produced by read_classify.  Steps (reference line ranges):
 *   1. SAM records -> per-record {name, U/C, tid, read length, MAPQ, AS score}; the SEQ of
 *      human records (tid 9606 / 63221 / 741158) is collected (getOneSAM, :687-813;
 *      meta_analysis_core, :1111-1136)
 *   2. one taxid per read: the primary record's tid, replaced by a descendant tid of an
 *      equal-score later record (ana_get_tid, :902-961); weight 1 or read length (:1158)
 *   3. counts sorted by weight (qsort with the 0/1 comparator cmp_count_sort, :584-587,
 *      glibc merge sort = stable descending), lineage weights and child lists (:1192-1222)
 *   4. leaves printed depth-first from roots 0 and 1 (ana_meta_loop_fprint, :846-899)
 *   5. report: no_match share, normalisation, rate-sorted top 3 (+ human > 5 %) (:1344-1411)
 * The record parser keeps the reference's strtok() tokenisation, so empty SAM fields shift
 * the same way they do in the reference.
 */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "dsb_host.h"

#define READ_NAME_LEN 100

typedef struct {
	char name[READ_NAME_LEN];
	char cls;            /* 'C' or 'U' */
	uint32_t tid, read_length, score;
	uint8_t mapq;
} meta_rec;

/* next strtok() token starting at *cur, advancing *cur past it (the reference's idiom) */
static char *tok_at(char **cur, const char *delim)
{
	char *t = strtok(*cur, delim);
	if (t)
		*cur += strlen(t) + 1;
	return t;
}

/* one SAM line -> meta_rec; returns the SEQ token (pointer into line) or NULL */
static char *parse_sam_line(char *line, meta_rec *r)
{
	char *cur = line, *t, *seq = NULL;
	if (!(t = tok_at(&cur, "\t"))) return NULL;
	strncpy(r->name, t, READ_NAME_LEN - 1);
	r->name[READ_NAME_LEN - 1] = 0;
	tok_at(&cur, "\t");                         /* FLAG */
	r->read_length = 0;
	r->score = 0;
	char *rname = tok_at(&cur, "\t");            /* RNAME */
	if (!rname) return NULL;
	if (rname[0] == '*') {
		r->cls = 'U';
		r->tid = 0;
		r->mapq = 0;
		for (int k = 0; k < 6; k++) tok_at(&cur, "\t"); /* POS MAPQ CIGAR * 0 0 */
		seq = tok_at(&cur, "\t");
	} else {
		r->cls = 'C';
		tok_at(&cur, "\t");                 /* POS */
		t = tok_at(&cur, "\t");             /* MAPQ */
		r->mapq = t ? (uint8_t)strtoul(t, NULL, 10) : 0;
		for (int k = 0; k < 4; k++) tok_at(&cur, "\t"); /* CIGAR * 0 0 */
		seq = tok_at(&cur, "\t");
		tok_at(&cur, "\t");                 /* QUAL */
		t = strtok(NULL, ":");              /* tag name, continuing the same strtok scan */
		if (t && ((t[0] == 'A' && t[1] == 'S') || (t[0] == 'N' && t[1] == 'M'))) {
			strtok(NULL, ":");          /* type */
			t = tok_at(&cur, "\t");
			r->score = t ? strtoul(t, NULL, 10) : 0;
			t = strtok(NULL, ":");
			if (t && t[0] == 'm' && t[1] == 's') {
				strtok(NULL, ":");
				t = tok_at(&cur, "\t");
				r->score = t ? strtoul(t, NULL, 10) : 0;
			}
			strtok(NULL, ":");
			tok_at(&cur, "\t");
		}
		/* RNAME "tid|<taxid>|..." -> taxid */
		char *rc = rname;
		char *a = strtok(rname, "|");
		if (a) rc += strlen(rc) + 1;
		char *b = strtok(rc, "|");
		r->tid = b ? strtoul(b, NULL, 10) : 0;
	}
	if (seq)
		r->read_length = (uint32_t)strlen(seq);
	return seq;
}

typedef struct { uint32_t tid; long count; } count_sort;
typedef struct { uint32_t tid, next; } cn_child;
typedef struct { uint64_t weight; uint32_t child_list_begin; } cly_node;

/* glibc msort with cmp_count_sort (a->count < b->count): stable by count descending */
static void sort_counts(count_sort *a, size_t n)
{
	if (n < 2) return;
	count_sort *tmp = malloc(n * sizeof(*a));
	for (size_t w = 1; w < n; w <<= 1) { /* stable bottom-up merge == any stable sort */
		for (size_t lo = 0; lo < n; lo += 2 * w) {
			size_t mid = lo + w < n ? lo + w : n, hi = lo + 2 * w < n ? lo + 2 * w : n;
			size_t i = lo, j = mid, k = lo;
			while (i < mid && j < hi) tmp[k++] = (a[j].count > a[i].count) ? a[j++] : a[i++];
			while (i < mid) tmp[k++] = a[i++];
			while (j < hi) tmp[k++] = a[j++];
		}
		memcpy(a, tmp, n * sizeof(*a));
	}
	free(tmp);
}

typedef struct {
	dsb_str *out;
	const dsb_index *ix;
	cly_node *nodes;
	cn_child *child;
	uint64_t total;
} leaf_ctx;

static void print_leaves(leaf_ctx *c, uint32_t id)
{
	cly_node *nd = c->nodes + id;
	if (nd->weight == 0)
		return;
	float rate = (float)nd->weight / c->total;
	if (nd->child_list_begin != 0) {
		for (uint32_t ch = nd->child_list_begin;; ch = c->child[ch].next) {
			print_leaves(c, c->child[ch].tid);
			if (c->child[ch].next == 0)
				break;
		}
		return;
	}
	const char *type = "microbe";
	if (id == 0 || id == 1)
		type = "no_match";
	else
		for (uint32_t t = id; t != 0xffffffffu; t = c->ix->tax[t].p_tid) {
			if (t == 9606) { type = "human"; break; }
			if (t == 33208 || t == 33090) { type = "animal_and_plant"; break; }
		}
	dsb_str_printf(c->out, "%s\t%s|%s\tnull\t%f\n", type, c->ix->tax[id].name, c->ix->tax[id].rank, rate);
}

typedef struct { char type[256], species[256], tech[256]; float rate; } meta_row;

int dsb_meta_analysis(dsb_index *ix, const char *input, uint64_t input_n, char **output, uint64_t *output_n,
		      int flag, uint64_t max_snapshot_len, char **human_snapshot, uint64_t *human_snapshot_n)
{
	uint64_t max_tid = ix->max_tid;
	/* ---- 1. records (skip '@' header lines) */
	char *text = malloc(input_n + 1);
	memcpy(text, input, input_n);
	text[input_n] = 0;
	dsb_str human = {0, 0, 0};
	meta_rec *recs = NULL;
	uint64_t nrec = 0, mrec = 0;
	char *p = text, *end = text + input_n;
	int in_header = 1;
	while (p < end) {
		char *nl = memchr(p, '\n', (size_t)(end - p));
		char *line_end = nl ? nl + 1 : end;
		size_t ll = (size_t)(line_end - p);
		char *line = malloc(ll + 1);
		memcpy(line, p, ll);
		line[ll] = 0;
		p = line_end;
		if (in_header && line[0] == '@') { free(line); continue; }
		in_header = 0;
		if (nrec == mrec) { mrec = mrec ? 2 * mrec : 1024; recs = realloc(recs, mrec * sizeof(*recs)); }
		meta_rec *r = recs + nrec;
		memset(r, 0, sizeof(*r));
		char *seq = parse_sam_line(line, r);
		if (!seq) { free(line); continue; }
		nrec++;
		if (seq[0] != '*' && (r->tid == 9606 || r->tid == 63221 || r->tid == 741158))
			dsb_str_put(&human, seq, strlen(seq));
		free(line);
	}
	free(text);
	/* ---- 2. one taxid per read, weights */
	uint64_t *node_count = calloc(max_tid + 2, sizeof(uint64_t));
	long total_weight = 0;
	for (uint64_t i = 0; i < nrec;) {
		meta_rec *r = recs + i;
		uint32_t w = ((flag & 1) == 0) ? 1 : r->read_length;
		total_weight += w;
		uint32_t tid = 0, score = 0;
		uint64_t j = i + 1;
		if (r->cls == 'C') {
			if (r->tid <= max_tid) { tid = r->tid; score = r->score; }
			for (; j < nrec; j++) {
				meta_rec *o = recs + j;
				if (strcmp(o->name, r->name) != 0 || score == 0) break;
				if (o->score != score || o->tid > max_tid) continue;
				for (uint32_t pt = o->tid;; pt = ix->tax[pt].p_tid) {
					if (pt == tid) { tid = o->tid; break; }
					if (pt < 1 || pt == 4294967295u) break;
				}
			}
		}
		node_count[tid] += w;
		i = j;
	}
	/* ---- 3. counts, lineage weights, child lists */
	count_sort *srt = malloc(sizeof(count_sort) * (max_tid + 2));
	size_t ns = 0;
	for (uint64_t t = 0; t <= max_tid; t++)
		if (node_count[t]) { srt[ns].tid = (uint32_t)t; srt[ns].count = (long)node_count[t]; ns++; }
	sort_counts(srt, ns);
	cly_node *nodes = calloc(max_tid + 2, sizeof(cly_node));
	cn_child *child = calloc(2 * (max_tid + 2), sizeof(cn_child));
	uint32_t child_count = 1;
	for (size_t i = 0; i < ns; i++) {
		uint32_t c_tid = srt[i].tid;
		for (;;) {
			uint32_t p_tid = ix->tax[c_tid].p_tid;
			nodes[c_tid].weight += node_count[srt[i].tid];
			if (p_tid == 0xffffffffu) break;
			if (nodes[p_tid].child_list_begin == 0) {
				nodes[p_tid].child_list_begin = child_count++;
				child[child_count - 1].tid = c_tid;
			} else {
				uint32_t lb = nodes[p_tid].child_list_begin;
				while (child[lb].tid != c_tid && child[lb].next != 0) lb = child[lb].next;
				if (child[lb].tid != c_tid && child[lb].next == 0) {
					child[lb].next = child_count++;
					child[child_count - 1].tid = c_tid;
				}
			}
			c_tid = p_tid;
		}
	}
	/* ---- 4. leaves */
	dsb_str rows = {0, 0, 0};
	leaf_ctx lc = {&rows, ix, nodes, child, (uint64_t)total_weight};
	if (nrec > 0) {
		print_leaves(&lc, 0);
		print_leaves(&lc, 1);
	}
	/* ---- 5. report */
	if (human.l > 0) {
		*human_snapshot_n = human.l < max_snapshot_len ? human.l : max_snapshot_len;
		*human_snapshot = malloc(*human_snapshot_n + 1);
		memcpy(*human_snapshot, human.s, *human_snapshot_n);
		(*human_snapshot)[*human_snapshot_n] = 0;
	} else {
		*human_snapshot = NULL;
		*human_snapshot_n = 0;
	}
	meta_row *res = NULL;
	size_t nres = 0, mres = 0;
	float no_match_rate = 0;
	for (char *q = rows.s, *qe = rows.s + rows.l; q && q < qe;) {
		char *nl = memchr(q, '\n', (size_t)(qe - q));
		if (nl) *nl = 0;
		meta_row r;
		memset(&r, 0, sizeof(r));
		sscanf(q, "%255[^\t]\t%255[^\t]\t%255[^\t]\t%f", r.type, r.species, r.tech, &r.rate);
		if (strcmp("no_match", r.type) == 0)
			no_match_rate += r.rate;
		else {
			if (nres == mres) { mres = mres ? 2 * mres : 64; res = realloc(res, mres * sizeof(*res)); }
			res[nres++] = r;
		}
		q = nl ? nl + 1 : qe;
	}
	dsb_str out = {0, 0, 0};
	if (no_match_rate > 0.95) {
		dsb_str_printf(&out, "no_match\tnull|null\tnull\t0\n");
	} else {
		for (size_t i = 0; i < nres; i++)
			res[i].rate = res[i].rate / (1 - no_match_rate);
		/* qsort with cmp_MetaRST (rate descending, proper comparator): stable */
		for (size_t i = 1; i < nres; i++) {
			meta_row v = res[i];
			size_t j = i;
			while (j > 0 && res[j - 1].rate < v.rate) { res[j] = res[j - 1]; j--; }
			res[j] = v;
		}
		for (size_t i = 0; i < nres; i++)
			if (i < 3 || (strcmp("human", res[i].type) == 0 && res[i].rate > 0.05))
				dsb_str_printf(&out, "%s\t%s\t%s\t%f\n", res[i].type, res[i].species, res[i].tech, res[i].rate);
	}
	*output_n = out.l;
	*output = calloc(out.l + 1, 1);
	if (out.l) memcpy(*output, out.s, out.l);
	free(out.s); free(rows.s); free(human.s); free(res);
	free(recs); free(node_count); free(srt); free(nodes); free(child);
	return 0;
}
