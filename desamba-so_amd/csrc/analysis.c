/*
 * analysis.c — `desamba_analysis <command> ...`: the reference's documented evaluation commands
 * (`deSAMBA analysis`, reference src/analysis.c:2679-2751 and usage :2684-2689), restated over
 * this library's host code.  Output is byte-identical to the reference's (tests/test_analysis.py
 * runs both on the same files):
 *
 *   ana_meta       <SAM> <nodes.dmp>   per-read taxa (ana_get_tid) counted up the taxonomy tree
 *                                      and printed as a tree of rates   (:1898-1909, :1390-1519)
 *   ana_meta_base  <SAM> <nodes.dmp>   the same weighted by aligned read length, with mapQ
 *                                      (:1911-1922, :1684-1803)
 *   ana_species    <SAM> <taxid> <nodes.dmp>         accuracy of every read against one true
 *   ana_genus      <SAM> <taxid> <nodes.dmp>         taxon at species / genus rank, or at any
 *   ana_sam        <SAM> <taxid> <nodes.dmp> <rank>  rank ("null": the true taxon is an ancestor
 *                                      of the read's), PRIMARY and any record (:1073-1234, :2014-2025)
 *   count_base     <FASTQ>             reads and bases (:2439-2454)
 *   split_fastq    <FASTQ> <start> <step>  every step-th read from start (:2507-2532)
 *   fastq_to_fasta <FASTQ>             (:2651-2662)
 *
 * A trailing argument "print_list" switches the trees to the leaf list of ana_meta_loop_fprint
 * (:1236-1289), as in the reference (:2707).  Files may be gzip'd (the reference opens every
 * input through zlib or stdio; SAM files are read as text).
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#include "dsb_host.h"

#define READ_NAME_LEN 100 /* analysis.c:35 */
#define MIN_SCORE 10      /* analysis.c:1531 */
#define NO_TID 4294967295u

static int print_list = 0; /* ANA_PRINT_USE_LIST, analysis.c:1235 */

/* ---------------------------------------------------------------- taxonomy (:71-118) */
typedef struct {
	uint32_t p_tid;
	char rank[20];
} tax_rank;

static uint32_t load_taxonomy(const char *path, tax_rank **out)
{
	FILE *fp = fopen(path, "r");
	if (!fp) {
		fprintf(stderr, "[desamba_analysis] fail to open file '%s'\n", path);
		exit(1);
	}
	char *line = NULL;
	size_t m = 0;
	uint32_t max_tid = 0;
	while (getline(&line, &m, fp) > 0) /* the last line's taxid */
		max_tid = (uint32_t)strtoul(strtok(line, "\t|"), NULL, 10);
	rewind(fp);
	max_tid += 1000000;
	tax_rank *t = malloc(sizeof(tax_rank) * ((size_t)max_tid + 1));
	for (uint32_t i = 0; i <= max_tid; i++) {
		t[i].p_tid = NO_TID;
		t[i].rank[0] = 0;
	}
	while (getline(&line, &m, fp) > 0) {
		uint32_t tid = (uint32_t)strtoul(strtok(line, "\t|"), NULL, 10);
		t[tid].p_tid = (uint32_t)strtoul(strtok(NULL, "\t|"), NULL, 10);
		snprintf(t[tid].rank, sizeof(t[tid].rank), "%s", strtok(NULL, "\t|"));
	}
	t[1].p_tid = 0; /* the root's parent is 0 */
	strcpy(t[1].rank, "root");
	strcpy(t[0].rank, "CLY_FAIL");
	free(line);
	fclose(fp);
	*out = t;
	return max_tid;
}

/* ---------------------------------------------------------------- SAM -> RST lines (:191-294, :430-464) */
typedef struct {
	char read_name[READ_NAME_LEN + 1];
	char isClassify;
	uint32_t tid, read_length;
	uint8_t MAPQ; /* RST.MAPQ is a uint8_t (:47) */
	uint32_t score;
} rst_t;

static void sam_to_rst(const char *line_in, rst_t *r)
{
	char *line = strdup(line_in);
	char *tok = strtok(line, "\t");
	snprintf(r->read_name, sizeof(r->read_name), "%s", tok ? tok : "");
	strtok(NULL, "\t"); /* flag */
	r->read_length = 0;
	r->score = 0;
	tok = strtok(NULL, "\t");
	if (!tok || tok[0] == '*') {
		r->isClassify = 'U';
		r->tid = 0;
		r->MAPQ = 0;
	} else {
		r->isClassify = 'C';
		char *ref = tok;
		strtok(NULL, "\t"); /* POS */
		tok = strtok(NULL, "\t");
		r->MAPQ = (uint8_t)strtoul(tok ? tok : "0", NULL, 10);
		char *cigar = strtok(NULL, "\t");
		for (int k = 0; k < 5; k++) /* RNEXT, PNEXT, TLEN, SEQ, QUAL */
			strtok(NULL, "\t");
		tok = strtok(NULL, ":");
		if (tok && ((tok[0] == 'A' && tok[1] == 'S') || (tok[0] == 'N' && tok[1] == 'M'))) {
			strtok(NULL, ":");
			tok = strtok(NULL, "\t");
			r->score = (uint32_t)strtoul(tok ? tok : "0", NULL, 10);
			tok = strtok(NULL, ":");
			if (tok && tok[0] == 'm' && tok[1] == 's') {
				strtok(NULL, ":");
				tok = strtok(NULL, "\t");
				r->score = (uint32_t)strtoul(tok ? tok : "0", NULL, 10);
			}
		}
		/* "tid|<taxid>|..." */
		strtok(ref, "|");
		tok = strtok(NULL, "|");
		r->tid = (uint32_t)strtoul(tok ? tok : "0", NULL, 10);
		/* read length: the M, I, S and X counts of the CIGAR */
		int len = 0, n = 0;
		for (const char *c = cigar ? cigar : ""; *c; c++) {
			if (*c >= '0' && *c <= '9')
				n = n * 10 + (*c - '0');
			else {
				if (*c == 'M' || *c == 'I' || *c == 'S' || *c == 'X')
					len += n;
				n = 0;
			}
		}
		r->read_length = (uint32_t)len;
	}
	free(line);
}

/* the dump / reload round trip of dump_des_sam_file + getOneRST: "%s\t%c\t%d\t%d\t%d\t%d" */
typedef struct {
	rst_t *a;
	size_t n, next;
} rst_list;

static void load_rst(const char *sam_path, rst_list *L)
{
	uint64_t len;
	char *buf;
	if (dsb_slurp_path(sam_path, &buf, &len)) {
		fprintf(stderr, "[desamba_analysis] fail to open file '%s'\n", sam_path);
		exit(1);
	}
	memset(L, 0, sizeof(*L));
	size_t m = 0;
	char *p = buf, *end = buf + len;
	int head = 1;
	while (p < end) {
		char *nl = memchr(p, '\n', (size_t)(end - p));
		size_t l = nl ? (size_t)(nl - p) + 1 : (size_t)(end - p);
		if (head && p[0] == '@') { /* skip_sam_head, :338-351 */
			p += l;
			continue;
		}
		head = 0;
		char *line = strndup(p, l);
		if (L->n == m) {
			m = m ? 2 * m : 1024;
			L->a = realloc(L->a, m * sizeof(rst_t));
		}
		sam_to_rst(line, L->a + L->n++);
		free(line);
		p += l;
	}
	free(buf);
	if (head) { /* skip_sam_head's xassert (:343): no record line at all */
		fprintf(stderr, "[skip_sam_head] Read SAM file FAILED\n Abort, line [344]!\n");
		abort();
	}
}

static int next_rst(rst_list *L, rst_t *r) /* getOneRST, :161-189 */
{
	if (L->next >= L->n)
		return -1;
	*r = L->a[L->next++];
	return 0;
}

/* ana_get_tid, :1329-1388 (returns 0 for the last read of the file, as the reference does) */
static uint32_t get_tid(rst_t *r, uint32_t max_tid, rst_list *L, int *eof_, const tax_rank *tax, int *read_len,
			float *coverage)
{
	char old[READ_NAME_LEN + 1];
	uint32_t tid = 0, score = 0;
	*eof_ = 0;
	*read_len = (int)r->read_length;
	if (r->isClassify != 'C') {
		if (next_rst(L, r) < 0)
			*eof_ = -1;
		return 0;
	}
	strcpy(old, r->read_name);
	if (r->tid <= max_tid) {
		tid = r->tid;
		score = r->score;
		*coverage = r->read_length > 0 ? (float)score / r->read_length : 0;
	}
	for (;;) {
		*eof_ = next_rst(L, r);
		if (*eof_ < 0)
			return 0;
		if (strcmp(old, r->read_name) != 0)
			break;
		if (score == 0)
			break;
		if (r->score != score || r->tid > max_tid)
			continue;
		for (uint32_t p = r->tid;;) {
			if (p == tid) {
				tid = r->tid;
				break;
			}
			if (p < 1 || p == NO_TID)
				break;
			p = tax[p].p_tid;
		}
	}
	return tid;
}

/* ---------------------------------------------------------------- tree (:1458-1504, :1236-1316) */
typedef struct {
	uint64_t weight, total_mapQ;
	uint32_t child_list_begin;
} node_t;
typedef struct {
	uint32_t tid, next;
} child_t;
typedef struct {
	uint32_t tid;
	uint64_t w, q;
} sort_t;

/* glibc qsort with the reference's (a->x < b->x) comparators: a stable sort by weight, descending */
static void sort_desc(sort_t *a, size_t n)
{
	sort_t *tmp = malloc((n + 1) * sizeof(*a));
	for (size_t w = 1; w < n; w <<= 1) {
		for (size_t lo = 0; lo < n; lo += 2 * w) {
			size_t mid = lo + w < n ? lo + w : n, hi = lo + 2 * w < n ? lo + 2 * w : n;
			size_t i = lo, j = mid, k = lo;
			while (i < mid && j < hi) tmp[k++] = (a[j].w > a[i].w) ? a[j++] : a[i++];
			while (i < mid) tmp[k++] = a[i++];
			while (j < hi) tmp[k++] = a[j++];
		}
		memcpy(a, tmp, n * sizeof(*a));
	}
	free(tmp);
}

static void build_tree(const tax_rank *tax, uint32_t max_tid, const uint64_t *w, const uint64_t *q, node_t *nodes,
		       child_t *child)
{
	sort_t *s = malloc(sizeof(sort_t) * ((size_t)max_tid + 2));
	size_t n = 0;
	for (uint32_t i = 0; i <= max_tid; i++)
		if (w[i]) {
			s[n].tid = i;
			s[n].w = w[i];
			s[n++].q = q ? q[i] : 0;
		}
	sort_desc(s, n);
	uint32_t child_count = 1;
	for (size_t i = 0; i < n; i++) {
		uint32_t c = s[i].tid;
		nodes[c].weight += w[c];
		nodes[c].total_mapQ += q ? q[c] : 0;
		for (;;) {
			uint32_t p = tax[c].p_tid;
			if (p < 1 || p == NO_TID)
				break;
			nodes[p].weight += w[s[i].tid];
			nodes[p].total_mapQ += q ? q[s[i].tid] : 0;
			if (nodes[p].child_list_begin == 0) {
				nodes[p].child_list_begin = child_count++;
				child[child_count - 1].tid = c;
			} else {
				uint32_t lb = nodes[p].child_list_begin;
				while (child[lb].tid != c && child[lb].next != 0)
					lb = child[lb].next;
				if (child[lb].tid != c && child[lb].next == 0) {
					child[lb].next = child_count++;
					child[child_count - 1].tid = c;
				}
			}
			c = p;
		}
	}
	free(s);
}

static void tree_print(const tax_rank *tax, const node_t *nodes, uint32_t id, const child_t *child, int level,
		       uint64_t total, int is_base)
{
	const node_t *nd = nodes + id;
	float rate = (float)nd->weight / total * 100;
	float map_q = (float)nd->total_mapQ / nd->weight * rate;
	if (rate < 0.01)
		return;
	for (int i = 0; i < level; i++)
		putchar('|');
	if (is_base) /* the node's tax_name is never set: "" */
		printf("%s TID:%d %s %f%%, mapQ:%f\n", tax[id].rank, (int)id, "", rate, map_q);
	else
		printf("%s TID:%d %s %f%%\n", tax[id].rank, (int)id, "", rate);
	if (nd->child_list_begin)
		for (uint32_t c = nd->child_list_begin;; c = child[c].next) {
			tree_print(tax, nodes, child[c].tid, child, level + 1, total, is_base);
			if (child[c].next == 0)
				break;
		}
}

static void leaf_print(const tax_rank *tax, const node_t *nodes, uint32_t id, const child_t *child, int level,
		       uint64_t total)
{
	const node_t *nd = nodes + id;
	if (nd->weight == 0)
		return;
	float rate = (float)nd->weight / total;
	if (nd->child_list_begin) {
		for (uint32_t c = nd->child_list_begin;; c = child[c].next) {
			leaf_print(tax, nodes, child[c].tid, child, level + 1, total);
			if (child[c].next == 0)
				break;
		}
		return;
	}
	const char *type = "microbe";
	if (id == 0 || id == 1)
		type = "no_match";
	else
		for (uint32_t t = id; t != NO_TID; t = tax[t].p_tid) {
			if (t == 9606) { type = "human"; break; }
			if (t == 33208 || t == 33090) { type = "animal_and_plant"; break; }
		}
	printf("%s\t%d|%s\tnull\t%f\n", type, (int)id, tax[id].rank, rate);
	/* DEBUG 1 (desc.h:4): the reference echoes each leaf, indented, on stderr */
	for (int i = 0; i < level; i++)
		fputs("  ", stderr);
	fprintf(stderr, "DEBUG: %s\t%d|%s\tnull\t%f\n", type, (int)id, tax[id].rank, rate);
}

/* ana_meta (:1390-1519) and ana_meta_base_M2 (:1684-1803) over a SAM file (:1898-1922) */
static int ana_meta(const char *sam, const char *nodes_dmp, int by_base)
{
	char tmp[1100];
	snprintf(tmp, sizeof(tmp), "%s.temp", sam); /* the reference's dump file name, printed */
	rst_list L;
	load_rst(sam, &L);
	printf("Current read %s\t", tmp);
	printf("%s\t", tmp);
	tax_rank *tax;
	uint32_t max_tid = load_taxonomy(nodes_dmp, &tax);
	uint64_t *w = calloc((size_t)max_tid + 2, sizeof(uint64_t)), *q = calloc((size_t)max_tid + 2, sizeof(uint64_t));
	int total_reads = 0;
	uint64_t total_base = 0, low_n = 0, low_base = 0;
	rst_t r;
	int eof_ = 0;
	float coverage = 0;
	if (next_rst(&L, &r) < 0) {
		free(L.a);
		free(tax);
		free(w);
		free(q);
		return 0;
	}
	for (;;) {
		total_reads++;
		int read_len = 0;
		int map_q = r.MAPQ;
		uint32_t t = get_tid(&r, max_tid, &L, &eof_, tax, &read_len, &coverage);
		if (t > 0) {
			if (!by_base)
				w[t]++;
			else if (coverage * read_len > MIN_SCORE) {
				total_base += (uint64_t)read_len;
				w[t] += (uint64_t)read_len;
				q[t] += (uint64_t)read_len * (uint64_t)map_q;
				if (coverage < 0.08) {
					low_base += (uint64_t)read_len;
					low_n++;
				}
			}
		}
		if (eof_ < 0)
			break;
	}
	node_t *nodes = calloc((size_t)max_tid + 2, sizeof(node_t));
	child_t *child = calloc(2 * ((size_t)max_tid + 2), sizeof(child_t));
	build_tree(tax, max_tid, w, by_base ? q : NULL, nodes, child);
	uint64_t total = by_base ? total_base : (uint64_t)total_reads;
	printf(by_base ? "Analysis based on base number:\n" : "Data:\n");
	if (print_list)
		leaf_print(tax, nodes, 1, child, 0, total);
	else
		tree_print(tax, nodes, 1, child, 0, total, by_base);
	if (by_base) {
		printf("total_mapped_base_number :%ld\n", (long)total_base);
		printf("low identity read (identity <= 75%%) number :%ld\t", (long)low_n);
		printf("total base %ld\t", (long)low_base);
	} else
		printf("total_read_number :%d\t", total_reads);
	free(nodes);
	free(child);
	free(w);
	free(q);
	free(tax);
	free(L.a);
	return 0;
}

/* ---------------------------------------------------------------- accuracy vs one true taxon */
/* get_tax_by_rank, :1029-1048: the first taxon at `rank` on the path to the root, or 0 */
static uint32_t tax_by_rank(const tax_rank *tax, uint32_t t, const char *rank)
{
	for (uint32_t c = t;;) {
		if (strcmp(tax[c].rank, rank) == 0)
			return c;
		c = tax[c].p_tid;
		if (c <= 1 || c == NO_TID)
			return 0;
	}
}

/* compare_tax, :1051-1065: is `a` on the path from `b` to (below) the root */
static int tax_is_ancestor(const tax_rank *tax, uint32_t a, uint32_t b)
{
	for (uint32_t c = b;;) {
		if (c == a)
			return 1;
		c = tax[c].p_tid;
		if (c <= 1 || c == NO_TID)
			return 0;
	}
}

static int right_classify(const tax_rank *tax, uint32_t right_tax, uint32_t tid, const char *rank, int no_rank)
{
	return no_rank ? tax_is_ancestor(tax, right_tax, tid) : tax_by_rank(tax, tid, rank) == right_tax;
}

/* ana_tax_des (:2014-2025) + ana_tax (:1073-1234): every read of the SAM file should come from
 * `right_tax`; per read "\n<name> " then UM (unmapped), PRI (the primary record is right) or SEC
 * (a later record of the read is), on stdout; the totals and rates on stderr. */
static int ana_tax(const char *sam, uint32_t right_tax, const char *nodes_dmp, const char *rank)
{
	char tmp[1100];
	snprintf(tmp, sizeof(tmp), "%s.temp", sam);
	rst_list L;
	load_rst(sam, &L);
	fprintf(stderr, "%s\t", tmp);
	int no_rank = strcmp(rank, "null") == 0;
	tax_rank *tax;
	load_taxonomy(nodes_dmp, &tax);
	int wrong = 0, total = 0, unmapped = 0, right_first = 0, right_second = 0;
	rst_t r;
	if (next_rst(&L, &r) < 0) {
		free(tax);
		free(L.a);
		return 0;
	}
	for (;;) {
		total++;
		printf("\n%s ", r.read_name);
		if (r.isClassify == 'U') {
			unmapped++;
			printf("UM");
			if (next_rst(&L, &r) < 0)
				break;
			continue;
		}
		int right = right_classify(tax, right_tax, r.tid, rank, no_rank);
		if (right) {
			right_first++;
			printf("PRI");
		}
		char old[READ_NAME_LEN + 1];
		strcpy(old, r.read_name);
		int eof_ = 0;
		for (;;) {
			eof_ = next_rst(&L, &r);
			if (eof_ < 0 || strcmp(old, r.read_name) != 0)
				break;
			if (right)
				continue;
			if (right_classify(tax, right_tax, r.tid, rank, no_rank)) {
				right = 1;
				right_second++;
				printf("SEC");
			}
		}
		if (eof_ < 0)
			break;
		if (!right)
			wrong++;
	}
	(void)wrong;
	fprintf(stderr, "%d\t", total);
	fprintf(stderr, "%d\t", unmapped);
	fprintf(stderr, "%d\t", right_first);
	fprintf(stderr, "%d\t", right_second + right_first);
	fprintf(stderr, "%f%%\t", (float)unmapped / total * 100);
	fprintf(stderr, "%f%%\t", (float)right_first / total * 100);
	fprintf(stderr, "%f%%\t", (float)right_first / (total - unmapped) * 100);
	fprintf(stderr, "%f%%\t", (float)(right_second + right_first) / total * 100);
	fprintf(stderr, "%f%%\n", (float)(right_second + right_first) / (total - unmapped) * 100);
	free(tax);
	free(L.a);
	return 0;
}

/* ---------------------------------------------------------------- FASTQ utilities */
static char *slurp_or_die(const char *path, uint64_t *len)
{
	char *buf;
	if (dsb_slurp_path(path, &buf, len)) {
		fprintf(stderr, "[desamba_analysis] fail to open file '%s'\n", path);
		exit(1);
	}
	return buf;
}

static const char *s_or_null(const char *s) { return s ? s : "(null)"; }

static int count_base(const char *path) /* :2439-2454 */
{
	uint64_t len;
	char *buf = slurp_or_die(path, &len);
	dsb_kseq1 *k = dsb_kseq1_open(buf, len);
	uint64_t reads = 0, bases = 0;
	while (dsb_kseq1_read(k) >= 0) {
		reads++;
		bases += dsb_kseq1_seq_l(k);
	}
	fprintf(stderr, "%s read number: %ld base number %ld ( %f Mbp)\n", path, (long)reads, (long)bases,
		(float)bases / 1000000);
	dsb_kseq1_close(k);
	free(buf);
	return 0;
}

static int split_fastq(const char *path, long begin, long step) /* :2507-2532 */
{
	uint64_t len;
	char *buf = slurp_or_die(path, &len);
	dsb_kseq1 *k = dsb_kseq1_open(buf, len);
	uint64_t total = 0, n = 0;
	while (dsb_kseq1_read(k) >= 0) {
		if ((long)n >= begin && ((long)n - begin) % step == 0) {
			printf("@%s %s\n%s\n+\n%s\n", s_or_null(dsb_kseq1_name(k)), s_or_null(dsb_kseq1_comment(k)),
			       s_or_null(dsb_kseq1_seq(k)), s_or_null(dsb_kseq1_qual(k)));
			total += dsb_kseq1_seq_l(k);
		}
		n++;
	}
	fprintf(stderr, "%s read number: %ld base number %ld ( %f Mbp)\n", path, (long)n, (long)total,
		(float)total / 1000000);
	dsb_kseq1_close(k);
	free(buf);
	return 0;
}

static int fastq_to_fasta(const char *path) /* :2651-2662 */
{
	uint64_t len;
	char *buf = slurp_or_die(path, &len);
	dsb_kseq1 *k = dsb_kseq1_open(buf, len);
	while (dsb_kseq1_read(k) >= 0) {
		printf(">%s %s\n", s_or_null(dsb_kseq1_name(k)), s_or_null(dsb_kseq1_comment(k)));
		printf("%s\n", s_or_null(dsb_kseq1_seq(k)));
	}
	dsb_kseq1_close(k);
	free(buf);
	return 0;
}

static int usage(void)
{
	fprintf(stderr, "usage: desamba_analysis <command> [files] [print_list]\n"
			"  ana_meta       <SAM> <nodes.dmp>\n"
			"  ana_meta_base  <SAM> <nodes.dmp>\n"
			"  ana_species    <SAM> <taxid> <nodes.dmp>\n"
			"  ana_genus      <SAM> <taxid> <nodes.dmp>\n"
			"  ana_sam        <SAM> <taxid> <nodes.dmp> <rank|null>\n"
			"  count_base     <FASTQ>\n"
			"  split_fastq    <FASTQ> <start> <step>\n"
			"  fastq_to_fasta <FASTQ>\n");
	return 1;
}

int main(int argc, char **argv)
{
	if (argc > 1 && !strcmp(argv[argc - 1], "print_list")) {
		print_list = 1;
		fprintf(stderr, "ANA_PRINT_USE_LIST = 1\n");
	}
	if (argc <= 1)
		return usage();
	const char *cmd = argv[1];
	if (!strcmp(cmd, "ana_meta") && argc >= 4)
		return ana_meta(argv[2], argv[3], 0);
	if (!strcmp(cmd, "ana_meta_base") && argc >= 4)
		return ana_meta(argv[2], argv[3], 1);
	if (!strcmp(cmd, "ana_species") && argc >= 5)
		return ana_tax(argv[2], (uint32_t)strtoul(argv[3], NULL, 10), argv[4], "species");
	if (!strcmp(cmd, "ana_genus") && argc >= 5)
		return ana_tax(argv[2], (uint32_t)strtoul(argv[3], NULL, 10), argv[4], "genus");
	if (!strcmp(cmd, "ana_sam") && argc >= 6)
		return ana_tax(argv[2], (uint32_t)strtoul(argv[3], NULL, 10), argv[4], argv[5]);
	if (!strcmp(cmd, "count_base") && argc >= 3)
		return count_base(argv[2]);
	if (!strcmp(cmd, "split_fastq") && argc >= 5) {
		long step = strtol(argv[4], NULL, 10);
		return split_fastq(argv[2], strtol(argv[3], NULL, 10), step > 0 ? step : 1);
	}
	if (!strcmp(cmd, "fastq_to_fasta") && argc >= 3)
		return fastq_to_fasta(argv[2]);
	fprintf(stderr, "command [%s] unsupported!\n\n", cmd);
	return usage();
}
