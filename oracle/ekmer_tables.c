/*
 * oracle/ekmer_tables.c — TEST INFRASTRUCTURE ONLY: (re)compute an index's e-kmer Bloom tables
 * (deSAMBA.exk0 / .exk1 / .exki) for any table size, restating the reference builder's
 * get_EXIST_kmer + set_ekmer_par (reference src/idx.c:966-1027):
 *
 *   for every unitig, every l_ek-mer of its string (2-bit, first base high; no complexity
 *   filter at build time): bit hash64_1(kmer) & mask of table 0 and hash64_2(kmer) & mask of
 *   table 1, MSB-first within a byte (0x80 >> (h & 7));  e_kmer_size selects l_ek and the mask:
 *   128 MB -> 16 / MASK_30, 256 MB -> 17 / MASK_31, 512 MB -> 17 / MASK_32, 1 GB -> 18 / MASK_33 ...
 *
 * The unitig strings are not stored in the index; they are read back from the packed reference
 * at each unitig's first REF_POS (deSAMBA.unv / .ref_p / .ref_b, idx.c:1089-1096: unitigs are
 * forward substrings of the reference; CONSIDER_BOTH_ORIENTATION is off, desc.h:6).
 * Checked against the reference builder's own tables (same size) before any other use:
 * `ekmer_tables <idx> <size> <out> --check` must print "identical".
 *
 * Used to make the l_ek-17 / MASK_31 variant of the C1 proxy index (tests/test_gpu_c2.py),
 * which the reference classifier then loads as it would a builder-made index of >= 238.6 M k-mers.
 *
 *   ekmer_tables <index_dir> <e_kmer_size_bytes> <out_dir> [--check]
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t hash64_1(uint64_t key) /* reference src/lib/utils.c:1067-1077 */
{
	key = (~key + (key << 21));
	key = key ^ key >> 24;
	key = ((key + (key << 3)) + (key << 8));
	key = key ^ key >> 14;
	key = ((key + (key << 2)) + (key << 4));
	key = key ^ key >> 28;
	key = (key + (key << 31));
	return key;
}

static uint64_t hash64_2(uint64_t key) /* reference src/lib/utils.c:1080-1091 */
{
	key += ~(key << 32);
	key ^= (key >> 22);
	key += ~(key << 13);
	key ^= (key >> 8);
	key += (key << 3);
	key ^= (key >> 15);
	key += ~(key << 27);
	key ^= (key >> 31);
	return key;
}

static void *slurp(const char *dir, const char *suffix, uint64_t *n_bytes)
{
	char p[4096];
	snprintf(p, sizeof(p), "%s/deSAMBA%s", dir, suffix);
	FILE *f = fopen(p, "rb");
	if (!f) {
		perror(p);
		exit(1);
	}
	fseek(f, 0, SEEK_END);
	long n = ftell(f);
	rewind(f);
	void *b = malloc((size_t)n + 8);
	if (fread(b, 1, (size_t)n, f) != (size_t)n) {
		fprintf(stderr, "short read %s\n", p);
		exit(1);
	}
	fclose(f);
	*n_bytes = (uint64_t)n;
	return b;
}

static void write_file(const char *dir, const char *suffix, const void *p, uint64_t n)
{
	char path[4096];
	snprintf(path, sizeof(path), "%s/deSAMBA%s", dir, suffix);
	FILE *f = fopen(path, "wb");
	if (!f || fwrite(p, 1, n, f) != n) {
		perror(path);
		exit(1);
	}
	fclose(f);
}

int main(int argc, char **argv)
{
	if (argc < 4) {
		fprintf(stderr, "usage: %s <index_dir> <e_kmer_size_bytes> <out_dir> [--check]\n", argv[0]);
		return 2;
	}
	uint64_t size = strtoull(argv[2], NULL, 10);
	int check = argc > 4 && !strcmp(argv[4], "--check");
	/* set_ekmer_par, src/idx.c:966-982 */
	int l_ek;
	uint64_t mask;
	switch (size) {
	case 1ull << 27: l_ek = 16; mask = 0x3fffffffull; break;
	case 1ull << 28: l_ek = 17; mask = 0x7fffffffull; break;
	case 1ull << 29: l_ek = 17; mask = 0xffffffffull; break;
	case 1ull << 30: l_ek = 18; mask = 0x1ffffffffull; break;
	case 1ull << 31: l_ek = 18; mask = 0x3ffffffffull; break;
	case 1ull << 32: l_ek = 19; mask = 0x7ffffffffull; break;
	case 1ull << 33: l_ek = 19; mask = 0xfffffffffull; break;
	default: l_ek = 20; mask = 0x1fffffffffull; break;
	}
	uint64_t nb;
	uint8_t *unv = slurp(argv[1], ".unv", &nb);
	uint64_t n_uni = *(uint64_t *)unv;
	const uint32_t *uni = (const uint32_t *)(unv + 8); /* {ref_list, length} */
	uint8_t *rp = slurp(argv[1], ".ref_p", &nb);
	uint64_t n_rp = *(uint64_t *)rp;
	const uint64_t *refpos = (const uint64_t *)(rp + 8);
	uint8_t *rb = slurp(argv[1], ".ref_b", &nb);
	uint64_t n_rb = *(uint64_t *)rb;
	const uint8_t *ref = rb + 8;
	uint8_t *t0 = calloc(size, 1), *t1 = calloc(size, 1);
	if (!t0 || !t1) {
		fprintf(stderr, "out of memory\n");
		return 1;
	}
	uint64_t kmask = (l_ek == 32) ? ~0ull : ((1ull << (2 * l_ek)) - 1), n_kmer = 0;
	for (uint64_t u = 0; u < n_uni; u++) {
		uint32_t rl = uni[2 * u], len = uni[2 * u + 1];
		if (rl >= n_rp || len < (uint32_t)l_ek)
			continue;
		uint64_t off = refpos[rl] & ((1ull << 40) - 1);
		if ((off + len + 3) / 4 > n_rb)
			continue;
		uint64_t km = 0;
		for (uint32_t i = 0; i < len; i++) {
			uint64_t g = off + i;
			uint64_t b = (ref[g >> 2] >> (6 - 2 * (g & 3))) & 3;
			km = ((km << 2) | b) & kmask;
			if (i + 1 >= (uint32_t)l_ek) {
				uint64_t h1 = hash64_1(km) & mask, h2 = hash64_2(km) & mask;
				t0[h1 >> 3] |= (uint8_t)(0x80 >> (h1 & 7));
				t1[h2 >> 3] |= (uint8_t)(0x80 >> (h2 & 7));
				n_kmer++;
			}
		}
	}
	if (check) {
		uint64_t n0, n1, ni;
		uint8_t *r0 = slurp(argv[1], ".exk0", &n0), *r1 = slurp(argv[1], ".exk1", &n1);
		uint8_t *ri = slurp(argv[1], ".exki", &ni);
		int same = n0 == size && n1 == size && *(uint64_t *)ri == size && !memcmp(r0, t0, size) &&
			   !memcmp(r1, t1, size);
		printf("%s (%lu unitigs, %lu l_ek-mers, l_ek %d)\n", same ? "identical" : "DIFFERENT",
		       (unsigned long)n_uni, (unsigned long)n_kmer, l_ek);
		return same ? 0 : 1;
	}
	write_file(argv[3], ".exk0", t0, size);
	write_file(argv[3], ".exk1", t1, size);
	write_file(argv[3], ".exki", &size, 8);
	printf("wrote %s/deSAMBA.exk{0,1,i}: %lu unitigs, %lu l_ek-mers, l_ek %d, %lu-byte tables\n", argv[3],
	       (unsigned long)n_uni, (unsigned long)n_kmer, l_ek, (unsigned long)size);
	return 0;
}
