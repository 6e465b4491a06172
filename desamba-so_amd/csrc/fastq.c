/*
 * fastq.c — FASTQ/FASTA parsing with the exact semantics the reference applies on
 * the classify path.
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
 */
#define _GNU_SOURCE
#include <ctype.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
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
	int64_t qual_rec; /* record index whose qual string this slot's qual.s holds, -1 = NULL */
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

static uint64_t arena_put(dsb_reads_t *r, const char *s, uint64_t n)
{
	if (r->arena_n + n + 1 > r->arena_m) {
		uint64_t m = r->arena_m ? r->arena_m : (1u << 20);
		while (m < r->arena_n + n + 1) m <<= 1;
		r->arena = realloc(r->arena, m);
		r->arena_m = m;
	}
	uint64_t off = r->arena_n;
	memcpy(r->arena + off, s, n);
	r->arena[off + n] = 0;
	r->arena_n += n + 1;
	return off;
}

int dsb_parse_reads(const char *buf, uint64_t len, dsb_reads_t *out)
{
	kstream_emu ks = {(const unsigned char *)buf, len, 0, 0, 0};
	slot_state *slots = calloc((size_t)N_WORKERS * N_NEEDED, sizeof(slot_state));
	for (int i = 0; i < N_WORKERS * N_NEEDED; i++) slots[i].qual_rec = -1;
	kseq_bufs b;
	memset(&b, 0, sizeof(b));
	int64_t widx[N_WORKERS];
	int alive[N_WORKERS];
	for (int w = 0; w < N_WORKERS; w++) { widx[w] = w; alive[w] = 1; }
	int64_t next_index = N_WORKERS;
	for (;;) {
		int w = -1;
		for (int k = 0; k < N_WORKERS; k++)
			if (alive[k] && (w < 0 || widx[k] < widx[w])) w = k;
		if (w < 0) break;
		long nb = 0, total = 0;
		for (; nb < N_NEEDED && total < MAX_READ_SIZE; nb++) {
			slot_state *st = slots + (size_t)w * N_NEEDED + nb;
			int has_qual;
			int64_t rst = kseq_read_emu(&ks, st, &b, &has_qual);
			if (rst < 0) break;
			total += b.seq.l;
			if (out->n == out->m) {
				out->m = out->m ? out->m * 2 : 1024;
				out->rec = realloc(out->rec, out->m * sizeof(dsb_rec_t));
			}
			dsb_rec_t *rec = out->rec + out->n;
			rec->name_off = arena_put(out, b.name.s ? b.name.s : "", b.name.l);
			rec->seq_off = arena_put(out, b.seq.s, b.seq.l);
			rec->seq_l = (uint32_t)b.seq.l;
			if (has_qual) {
				rec->qual_off = arena_put(out, b.qual.s, b.qual.l);
				rec->qual_null = 0;
				st->qual_rec = (int64_t)out->n;
			} else if (st->qual_rec >= 0) {
				rec->qual_off = out->rec[st->qual_rec].qual_off; /* stale qual.s */
				rec->qual_null = 0;
			} else {
				rec->qual_off = 0;
				rec->qual_null = 1;
			}
			out->n++;
		}
		if (nb == 0) { alive[w] = 0; continue; }
		widx[w] = next_index++;
	}
	free(slots);
	free(b.name.s); free(b.comment.s); free(b.seq.s); free(b.qual.s);
	return 0;
}

void dsb_reads_free(dsb_reads_t *r)
{
	free(r->arena);
	free(r->rec);
	memset(r, 0, sizeof(*r));
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
	uint64_t m = in_n * 4 + 4096, n = 0;
	char *p = malloc(m);
	for (;;) {
		if (m - n < 1 << 20) { m *= 2; p = realloc(p, m); }
		int k = gzread(gz, p + n, (unsigned)((m - n) > (1u << 30) ? (1u << 30) : (m - n)));
		if (k <= 0) break;
		n += (uint64_t)k;
	}
	gzclose(gz);
	*buf = p;
	*len = n;
	*owned = 1;
	return 0;
}

int dsb_slurp_path(const char *path, char **buf, uint64_t *len)
{
	gzFile gz = gzopen(path, "r");
	if (!gz) return -1;
	uint64_t m = 1 << 24, n = 0;
	char *p = malloc(m);
	for (;;) {
		if (m - n < 1 << 20) { m *= 2; p = realloc(p, m); }
		int k = gzread(gz, p + n, (unsigned)((m - n) > (1u << 30) ? (1u << 30) : (m - n)));
		if (k <= 0) break;
		n += (uint64_t)k;
	}
	gzclose(gz);
	*buf = p;
	*len = n;
	return 0;
}
