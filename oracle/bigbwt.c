/*
 * oracle/bigbwt.c — TEST INFRASTRUCTURE ONLY (tests/test_gpu_bigbwt.py).  Linked against the
 * reference's own objects (oracle/Makefile `bigbwt`), so both the file and the answers come from
 * reference code:
 *
 *   bigbwt gen DIR NSYM SEED
 *       A synthetic BWT string of NSYM symbols (random A/C/G/T with ~1/64 '#' and one '$' at row
 *       NSYM - 1000 (printed)) written in the reference's format by the reference's own builder
 *       functions: bwt_cal_check_point + bwt_str2bwt_occ + bwt_cal_AGCTCounter + write_bwt
 *       (src/bwt.c:110-256): DIR/deSAMBA.bwt (168-B blocks + rank + a zero 13-mer hash index),
 *       .acg, and an empty .sa.  NSYM may exceed 2^32 (the reference's rows are uint64_t,
 *       src/bwt.h:45), which is what the test is for.  Prints "dollar_row R".
 *
 *   bigbwt occ DIR DOLLOR_POS ROWS OUT
 *       load_bwt(DIR) (src/bwt.c:68-104), then for every u64 row r of the file ROWS the
 *       reference's occ (src/bwt.c:43-65): occ(r, c) for c = 0..4 and occ(r, 0xff) with the symbol
 *       it reads, as 7 u64 per row into OUT.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "bwt.h"

static uint64_t xs = 88172645463325252ull;
static inline uint64_t rnd(void)
{
	xs ^= xs << 13;
	xs ^= xs >> 7;
	xs ^= xs << 17;
	return xs;
}

static int gen(const char *dir, uint64_t n, uint64_t seed)
{
	xs ^= seed * 0x9E3779B97F4A7C15ull;
	bwt bt;
	memset(&bt, 0, sizeof(bt));
	char *s = malloc(n);
	if (!s) {
		fprintf(stderr, "out of memory (%lu)\n", (unsigned long)n);
		return 1;
	}
	static const char sym[4] = {'A', 'C', 'G', 'T'};
	for (uint64_t i = 0; i < n; i += 8) {
		uint64_t v = rnd();
		for (int k = 0; k < 8 && i + k < n; k++) {
			uint8_t b = (uint8_t)(v >> (8 * k));
			s[i + k] = (b & 0xfc) == 0 ? '#' : sym[b & 3]; /* '#' with probability 1/64 */
		}
	}
	uint64_t dollar = n - 1000;
	s[dollar] = '$';
	bt.hash_index = calloc((1ull << 26) + 1, 8);
	bt.sa_size = 0;
	bt.sa_taxon = malloc(8);
	build_BWT(&bt, s, n, (char *)dir);
	write_bwt(&bt, dir);
	printf("dollar_row %lu\n", (unsigned long)dollar);
	return 0;
}

static int occ_rows(const char *dir, uint64_t dollor_pos, const char *rows_path, const char *out_path)
{
	bwt bt;
	memset(&bt, 0, sizeof(bt));
	load_bwt(&bt, dir);
	bt.DOLLOR_POS = dollor_pos;
	FILE *f = fopen(rows_path, "rb");
	if (!f)
		return 1;
	fseek(f, 0, SEEK_END);
	uint64_t n = (uint64_t)ftell(f) / 8;
	fseek(f, 0, SEEK_SET);
	uint64_t *rows = malloc(8 * n + 8), *out = malloc(56 * n + 8);
	if (fread(rows, 8, n, f) != n)
		return 1;
	fclose(f);
	for (uint64_t i = 0; i < n; i++) {
		for (uint8_t c = 0; c < 5; c++) {
			uint8_t cc = c;
			out[7 * i + c] = occ(&bt, rows[i], &cc);
		}
		uint8_t cf = 0xff;
		out[7 * i + 5] = occ(&bt, rows[i], &cf);
		out[7 * i + 6] = cf;
	}
	f = fopen(out_path, "wb");
	if (!f || fwrite(out, 56, n, f) != n)
		return 1;
	fclose(f);
	return 0;
}

int main(int argc, char **argv)
{
	if (argc == 5 && !strcmp(argv[1], "gen"))
		return gen(argv[2], strtoull(argv[3], NULL, 10), strtoull(argv[4], NULL, 10));
	if (argc == 6 && !strcmp(argv[1], "occ"))
		return occ_rows(argv[2], strtoull(argv[3], NULL, 10), argv[4], argv[5]);
	fprintf(stderr, "usage: bigbwt gen DIR NSYM SEED | bigbwt occ DIR DOLLOR_POS ROWS OUT\n");
	return 2;
}
