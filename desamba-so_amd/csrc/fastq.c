/*
 * fastq.c — FASTQ/FASTA parsing with the exact semantics the reference applies on
 * the classify path, as a resumable stream of batches.
 *
 * The reference parses with kseq (src/lib/utils.c:841-977) inside a 3-worker
 * kt_pipeline (src/lib/kthread.c:114-197, src/cly_mt.c:361-381): batch k is read by the
 * worker with the k-th smallest pipeline index into that worker's own array of 5000
 * kseq_t slots (src/cly_mt.c:29-43, 531-547, 977-983).  Two consequences are visible in
 * the output and reproduced here:
 *   - each slot keeps its own `last_char`, so a FASTA record whose header '>' was
 *     consumed by the previous slot is skipped by the next one (every other FASTA record
 *     is dropped);
 *   - a record that fails to parse (kseq_read < 0) ends the batch; a worker whose batch
 *     is empty leaves the pipeline, the others keep reading.
 * SAM_FULL prints qual.s, which for a FASTA record is the slot's previous quality string
 * (or "(null)").
 *
 * The input stays resident (the caller's buffer, an mmap'd file, or inflated gzip text) and
 * records are views into it: a single-line FASTQ record read by a slot whose last_char is 0
 * (the state every FASTQ record leaves behind) is recognised with memchr and not copied (the
 * fast path below takes exactly the bytes kseq_read would).  Every other record (FASTA,
 * multi-line, blank lines, malformed) goes through the byte-level kseq emulation and is
 * copied into the parser's arena, whose chunks never move and live as long as the parser,
 * so stale quality strings of earlier batches stay valid.
 */
#define _GNU_SOURCE
#include <ctype.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>
#include "dsb_host.h"

#define KS_BUFSIZE 100000 /* __kseq_bufsize, utils.c:835 */
#define N_NEEDED 5000     /* cly_mt.c:22 */
#define MAX_READ_SIZE 10000000 /* cly_mt.c:23 */
#define N_WORKERS 3       /* PIPELINE_T_NUM, cly_mt.c:461 */

typedef struct {
	const unsigned char *buf;
	uint64_t len;
	uint64_t begin, end; /* absolute positions of the loaded window */
	int is_eof;
} kstream_emu;

typedef struct { char *s; uint64_t l, m; } kstr;

static void kstr_need(kstr *s, uint64_t n)
{
	if (s->m < n) {
		uint64_t m = n < 64 ? 64 : n;
		m--; m |= m >> 1; m |= m >> 2; m |= m >> 4; m |= m >> 8; m |= m >> 16; m |= m >> 32; m++;
		s->s = realloc(s->s, m);
		s->m = m;
	}
}

/* gzread of one buffer: the whole input is already in memory */
static void ks_refill(kstream_emu *ks)
{
	uint64_t n = ks->len - ks->end;
	if (n > KS_BUFSIZE) n = KS_BUFSIZE;
	ks->begin = ks->end;
	ks->end += n;
	if (n < KS_BUFSIZE) ks->is_eof = 1;
}

/* move the read position forward to `pos`, refilling windows as ks_getc would have */
static void ks_seek(kstream_emu *ks, uint64_t pos)
{
	while (ks->end < pos) {
		uint64_t old_end = ks->end;
		ks_refill(ks);
		if (ks->end == old_end) break;
	}
	ks->begin = pos;
}

static int ks_getc(kstream_emu *ks) /* utils.c:890-900 */
{
	if (ks->is_eof && ks->begin >= ks->end) return -1;
	if (ks->begin >= ks->end) {
		uint64_t old_end = ks->end;
		ks_refill(ks);
		if (ks->end == old_end) return -1;
	}
	return (int)ks->buf[ks->begin++];
}

/* ks_getuntil2, utils.c:841-885; delimiter 0 = isspace */
static int64_t ks_getuntil2(kstream_emu *ks, int delimiter, kstr *str, int *dret, int append)
{
	if (dret) *dret = 0;
	str->l = append ? str->l : 0;
	if (ks->begin >= ks->end && ks->is_eof) return -1;
	for (;;) {
		uint64_t i;
		if (ks->begin >= ks->end) {
			if (!ks->is_eof) {
				uint64_t old_end = ks->end;
				ks_refill(ks);
				if (ks->end == old_end) break;
			} else break;
		}
		if (delimiter > 1) {
			for (i = ks->begin; i < ks->end; ++i)
				if (ks->buf[i] == delimiter) break;
		} else {
			for (i = ks->begin; i < ks->end; ++i)
				if (isspace(ks->buf[i])) break;
		}
		kstr_need(str, str->l + (i - ks->begin) + 1);
		memcpy(str->s + str->l, ks->buf + ks->begin, i - ks->begin);
		str->l += i - ks->begin;
		ks->begin = i + 1;
		if (i < ks->end) {
			if (dret) *dret = ks->buf[i];
			break;
		}
	}
	kstr_need(str, str->l + 1);
	str->s[str->l] = '\0';
	return (int64_t)str->l;
}

typedef struct {
	int last_char;
	const char *qual; /* the slot's qual.s (a stale one for FASTA records); NULL = never set */
	uint32_t qual_l;
} slot_state;

typedef struct { kstr name, comment, seq, qual; } kseq_bufs;

/* kseq_read, utils.c:939-977.  Returns seq.l, -1 (EOF) or -2 (malformed). */
static int64_t kseq_read_emu(kstream_emu *ks, slot_state *st, kseq_bufs *b, int *has_qual)
{
	int c;
	*has_qual = 0;
	if (st->last_char == 0) {
		while ((c = ks_getc(ks)) != -1 && c != '>' && c != '@');
		if (c == -1) return -1;
		st->last_char = c;
	}
	b->comment.l = b->seq.l = b->qual.l = 0;
	if (ks_getuntil2(ks, 0, &b->name, &c, 0) < 0) return -1;
	if (c != '\n') ks_getuntil2(ks, '\n', &b->comment, 0, 0);
	kstr_need(&b->seq, 256);
	while ((c = ks_getc(ks)) != -1 && c != '>' && c != '+' && c != '@') {
		kstr_need(&b->seq, b->seq.l + 2);
		b->seq.s[b->seq.l++] = (char)c;
		ks_getuntil2(ks, '\n', &b->seq, 0, 1);
	}
	if (c == '>' || c == '@') st->last_char = c;
	kstr_need(&b->seq, b->seq.l + 1);
	b->seq.s[b->seq.l] = 0;
	if (c != '+') return (int64_t)b->seq.l; /* FASTA */
	while ((c = ks_getc(ks)) != -1 && c != '\n');
	if (c == -1) return -2;
	b->qual.l = 0;
	while (ks_getuntil2(ks, '\n', &b->qual, 0, 1) >= 0 && b->qual.l < b->seq.l);
	st->last_char = 0;
	*has_qual = 1;
	if (b->seq.l != b->qual.l) return -2;
	return (int64_t)b->seq.l;
}

/* The same record read by a slot whose last_char is 0, when it is one single-line FASTQ
 * record ("@name...\nSEQ\n+...\nQUAL\n", |QUAL| == |SEQ|): the views kseq_read would have
 * copied, without copying.  Returns 1 and advances the stream, or 0 (nothing consumed) when
 * the record is anything else — the byte-level emulation then reads it. */
static int fastq_view(kstream_emu *ks, dsb_rec_t *rec)
{
	const char *buf = (const char *)ks->buf;
	uint64_t len = ks->len, p = ks->begin;
	while (p < len && buf[p] != '@' && buf[p] != '>') p++; /* kseq's header scan */
	if (p >= len || buf[p] != '@') return 0;
	uint64_t h = p + 1;
	const char *nl = memchr(buf + h, '\n', len - h);
	if (!nl) return 0;
	uint64_t e = h;
	while (!isspace((unsigned char)buf[e])) e++; /* name: up to the first isspace (<= the '\n') */
	uint64_t s = (uint64_t)(nl - buf) + 1, plus;
	if (s >= len) return 0;
	uint32_t seq_l = 0;
	char c = buf[s];
	if (c == '+') {
		plus = s;
	} else {
		if (c == '>' || c == '@' || c == '\n') return 0; /* FASTA, or a blank line kseq folds in */
		const char *nl2 = memchr(buf + s, '\n', len - s);
		if (!nl2) return 0;
		plus = (uint64_t)(nl2 - buf) + 1;
		if (plus >= len || buf[plus] != '+') return 0; /* multi-line sequence or FASTA */
		if ((uint64_t)(nl2 - buf) - s > 0xFFFFFFFFull) return 0;
		seq_l = (uint32_t)((uint64_t)(nl2 - buf) - s);
	}
	const char *nl3 = memchr(buf + plus, '\n', len - plus);
	if (!nl3) return 0;
	uint64_t q = (uint64_t)(nl3 - buf) + 1;
	if (q >= len) return 0;
	const char *nl4 = memchr(buf + q, '\n', len - q);
	uint64_t qe = nl4 ? (uint64_t)(nl4 - buf) : len;
	if (qe - q != seq_l) return 0; /* multi-line or malformed quality */
	rec->name = buf + h;
	rec->name_l = (uint32_t)(e - h);
	rec->seq = buf + s;
	rec->seq_l = seq_l;
	rec->qual = buf + q;
	rec->qual_l = seq_l;
	ks_seek(ks, nl4 ? qe + 1 : len);
	return 1;
}

/* ------------------------------------------------------------------ arena */
typedef struct arena_chunk {
	struct arena_chunk *next;
	uint64_t n, m;
	char data[];
} arena_chunk;

static const char *arena_put(arena_chunk **head, const char *s, uint64_t n)
{
	arena_chunk *c = *head;
	if (!c || c->n + n + 1 > c->m) {
		uint64_t m = (uint64_t)4 << 20;
		if (m < n + 1) m = n + 1;
		arena_chunk *nc = malloc(sizeof(arena_chunk) + m);
		nc->next = c;
		nc->n = 0;
		nc->m = m;
		*head = c = nc;
	}
	char *p = c->data + c->n;
	if (n) memcpy(p, s, n);
	p[n] = 0;
	c->n += n + 1;
	return p;
}

static void arena_free(arena_chunk *c)
{
	while (c) {
		arena_chunk *n = c->next;
		free(c);
		c = n;
	}
}

/* ------------------------------------------------------------------ parser */
struct dsb_parser {
	kstream_emu ks;
	slot_state *slots;
	kseq_bufs b;
	int64_t widx[N_WORKERS];
	int alive[N_WORKERS];
	int64_t next_index;
	arena_chunk *arena;
	int fast;
	uint64_t n_fast, n_slow;
	int cur_w;               /* worker whose kt batch is being read (-1: none) */
	long cur_nb, cur_total;  /* its slots used and bases so far */
};

dsb_parser *dsb_parser_new(const char *buf, uint64_t len)
{
	dsb_parser *p = calloc(1, sizeof(*p));
	p->ks.buf = (const unsigned char *)buf;
	p->ks.len = len;
	p->slots = calloc((size_t)N_WORKERS * N_NEEDED, sizeof(slot_state));
	for (int w = 0; w < N_WORKERS; w++) {
		p->widx[w] = w;
		p->alive[w] = 1;
	}
	p->next_index = N_WORKERS;
	p->cur_w = -1;
	p->fast = getenv("DSB_PARSE_SLOW") ? 0 : 1;
	return p;
}

/* the zero-copy fast path on (1) or off (0: every record through the byte-level kseq emulation) */
void dsb_parser_set_fast(dsb_parser *p, int fast)
{
	p->fast = fast;
}

static void reads_push(dsb_reads_t *out, const dsb_rec_t *r)
{
	if (out->n == out->m) {
		out->m = out->m ? out->m * 2 : 1024;
		out->rec = realloc(out->rec, out->m * sizeof(dsb_rec_t));
	}
	out->rec[out->n++] = *r;
}

/* Read one record in the kt_pipeline order: worker w (the alive one with the smallest pipeline
 * index) fills its slots 0, 1, ... until 5000 reads, >= 10 Mbp, or the first kseq_read() < 0
 * ends its batch (cly_mt.c:29-43); a worker whose batch is empty leaves the pipeline.  The
 * batch state is kept in the parser, so a GPU batch may end anywhere inside a kt batch.
 * Returns 1 with *rec filled, 0 at the end of the input. */
static int parse_one(dsb_parser *p, dsb_rec_t *rec)
{
	for (;;) {
		if (p->cur_w < 0) {
			int w = -1;
			for (int k = 0; k < N_WORKERS; k++)
				if (p->alive[k] && (w < 0 || p->widx[k] < p->widx[w])) w = k;
			if (w < 0) return 0;
			p->cur_w = w;
			p->cur_nb = 0;
			p->cur_total = 0;
		}
		if (p->cur_nb < N_NEEDED && p->cur_total < MAX_READ_SIZE) {
			slot_state *st = p->slots + (size_t)p->cur_w * N_NEEDED + p->cur_nb;
			if (p->fast && st->last_char == 0 && fastq_view(&p->ks, rec)) {
				st->qual = rec->qual;
				st->qual_l = rec->qual_l;
				p->cur_total += rec->seq_l;
				p->cur_nb++;
				p->n_fast++;
				return 1;
			}
			int has_qual;
			int64_t rst = kseq_read_emu(&p->ks, st, &p->b, &has_qual);
			if (rst >= 0) {
				rec->name = arena_put(&p->arena, p->b.name.s ? p->b.name.s : "", p->b.name.l);
				rec->name_l = (uint32_t)p->b.name.l;
				rec->seq = arena_put(&p->arena, p->b.seq.s, p->b.seq.l);
				rec->seq_l = (uint32_t)p->b.seq.l;
				if (has_qual) {
					rec->qual = arena_put(&p->arena, p->b.qual.s, p->b.qual.l);
					rec->qual_l = (uint32_t)p->b.qual.l;
					st->qual = rec->qual;
					st->qual_l = rec->qual_l;
				} else { /* FASTA: SAM_FULL prints the slot's stale qual.s, or "(null)" */
					rec->qual = st->qual;
					rec->qual_l = st->qual_l;
				}
				p->cur_total += p->b.seq.l;
				p->cur_nb++;
				p->n_slow++;
				return 1;
			}
		}
		/* the kt batch of worker cur_w ends here */
		if (p->cur_nb == 0)
			p->alive[p->cur_w] = 0;
		else
			p->widx[p->cur_w] = p->next_index++;
		p->cur_w = -1;
	}
}

uint64_t dsb_parser_next(dsb_parser *p, dsb_reads_t *out, uint64_t max_reads, uint64_t max_bases)
{
	uint64_t n0 = out->n, bases = 0;
	dsb_rec_t rec;
	while (out->n - n0 < max_reads && bases < max_bases && parse_one(p, &rec)) {
		reads_push(out, &rec);
		bases += rec.seq_l;
	}
	return out->n - n0;
}

/* input bytes not yet read (an estimate: the reader's window start) */
uint64_t dsb_parser_left(const dsb_parser *p)
{
	return p->ks.len > p->ks.begin ? p->ks.len - p->ks.begin : 0;
}

void dsb_parser_stats(const dsb_parser *p, uint64_t *n_fast, uint64_t *n_slow)
{
	*n_fast = p->n_fast;
	*n_slow = p->n_slow;
}

void dsb_parser_free(dsb_parser *p)
{
	if (!p) return;
	free(p->slots);
	free(p->b.name.s); free(p->b.comment.s); free(p->b.seq.s); free(p->b.qual.s);
	arena_free(p->arena);
	free(p);
}

/* Whole input at once.  The records are views into `buf` (which must outlive `out`) and into
 * an arena `out` owns. */
int dsb_parse_reads(const char *buf, uint64_t len, dsb_reads_t *out)
{
	dsb_parser *p = dsb_parser_new(buf, len);
	while (dsb_parser_next(p, out, UINT64_MAX, UINT64_MAX));
	out->arena_owner = p->arena;
	p->arena = NULL;
	dsb_parser_free(p);
	return 0;
}

void dsb_reads_free(dsb_reads_t *r)
{
	arena_free((arena_chunk *)r->arena_owner);
	free(r->rec);
	free(r->text_owner);
	memset(r, 0, sizeof(*r));
}

/* ------------------------------------------------------------------ one kseq_t */
/* A single kseq_t reading resident text record by record (the evaluation tools' loops,
 * reference src/analysis.c:2439-2678): the strings are the kseq buffers themselves, so a
 * record without a comment shows the previous record's comment and a FASTA record the previous
 * quality, as printf("%s") of the reference prints them (NULL: never set). */
struct dsb_kseq1 {
	kstream_emu ks;
	slot_state st;
	kseq_bufs b;
	int has_qual;
};

dsb_kseq1 *dsb_kseq1_open(const char *buf, uint64_t len)
{
	dsb_kseq1 *k = calloc(1, sizeof(*k));
	k->ks.buf = (const unsigned char *)buf;
	k->ks.len = len;
	return k;
}

int64_t dsb_kseq1_read(dsb_kseq1 *k)
{
	return kseq_read_emu(&k->ks, &k->st, &k->b, &k->has_qual);
}

const char *dsb_kseq1_name(const dsb_kseq1 *k) { return k->b.name.s; }
const char *dsb_kseq1_comment(const dsb_kseq1 *k) { return k->b.comment.s; }
const char *dsb_kseq1_seq(const dsb_kseq1 *k) { return k->b.seq.s; }
const char *dsb_kseq1_qual(const dsb_kseq1 *k) { return k->b.qual.s; }
uint64_t dsb_kseq1_seq_l(const dsb_kseq1 *k) { return k->b.seq.l; }

void dsb_kseq1_close(dsb_kseq1 *k)
{
	if (!k) return;
	free(k->b.name.s); free(k->b.comment.s); free(k->b.seq.s); free(k->b.qual.s);
	free(k);
}

/* ------------------------------------------------------------------ input sources */
static int inflate_all(gzFile gz, char **buf, uint64_t *len, uint64_t hint)
{
	uint64_t m = hint < (1 << 24) ? (1 << 24) : hint, n = 0;
	char *p = malloc(m);
	if (!p) return -1;
	for (;;) {
		if (m - n < 1 << 20) {
			m *= 2;
			char *q = realloc(p, m);
			if (!q) { free(p); return -1; }
			p = q;
		}
		int k = gzread(gz, p + n, (unsigned)((m - n) > (1u << 30) ? (1u << 30) : (m - n)));
		if (k <= 0) break;
		n += (uint64_t)k;
	}
	*buf = p;
	*len = n;
	return 0;
}

int dsb_inflate_if_gzip(const char *in, uint64_t in_n, char **buf, uint64_t *len, int *owned)
{
	*owned = 0;
	if (in_n < 2 || (unsigned char)in[0] != 0x1f || (unsigned char)in[1] != 0x8b) {
		*buf = (char *)in;
		*len = in_n;
		return 0;
	}
	/* gzip: route through a temporary file + gzdopen like read_classify_core (cly_mt.c:1055-1062) */
	FILE *tf = tmpfile();
	if (!tf) return -1;
	if (fwrite(in, 1, in_n, tf) != in_n) { fclose(tf); return -1; }
	rewind(tf);
	gzFile gz = gzdopen(dup(fileno(tf)), "r");
	fclose(tf);
	if (!gz) return -1;
	int rc = inflate_all(gz, buf, len, in_n * 4 + 4096);
	gzclose(gz);
	if (rc) return -1;
	*owned = 1;
	return 0;
}

int dsb_slurp_path(const char *path, char **buf, uint64_t *len)
{
	gzFile gz = gzopen(path, "r");
	if (!gz) return -1;
	int rc = inflate_all(gz, buf, len, 0);
	gzclose(gz);
	return rc;
}

/* Input of read_classify in path mode (input_n == (uint64_t)-1, cly_mt.c:1049-1052): a plain
 * file is mapped, not read (the parser's views point into the mapping); a gzip file is
 * inflated into memory.  Returns 0; *unmap_len > 0 means munmap(*buf, *unmap_len), else free. */
int dsb_open_path(const char *path, char **buf, uint64_t *len, uint64_t *unmap_len)
{
	*unmap_len = 0;
	int fd = open(path, O_RDONLY);
	if (fd < 0) return -1;
	unsigned char magic[2] = {0, 0};
	struct stat sb;
	if (fstat(fd, &sb) == 0 && S_ISREG(sb.st_mode) && sb.st_size > 0 &&
	    pread(fd, magic, 2, 0) == 2 && !(magic[0] == 0x1f && magic[1] == 0x8b)) {
		void *m = mmap(NULL, (size_t)sb.st_size, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0);
		close(fd);
		if (m == MAP_FAILED) return dsb_slurp_path(path, buf, len);
		madvise(m, (size_t)sb.st_size, MADV_SEQUENTIAL);
		*buf = m;
		*len = (uint64_t)sb.st_size;
		*unmap_len = (uint64_t)sb.st_size;
		return 0;
	}
	close(fd);
	return dsb_slurp_path(path, buf, len);
}
