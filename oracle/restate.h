/*
 * oracle/restate.h — TEST INFRASTRUCTURE ONLY: this repository's own plain-C restatement of
 * the primitives on deSAMBA's classify hot path, written from the reference's algorithm
 * (file:line citations below, paths relative to /root/reference/src).  It is a checker:
 * tests/ link it (through oracle/_ref/restate_check) and compare it with the reference's own
 * compiled functions; the product (desamba-so_amd/) never includes or links it.
 *
 * Layouts are the reference's on-disk ones (168-B occ blocks, 2-bit MSB-first reference,
 * u64 REF_POS bitfields), not the HBM layouts of the GPU path, so the restatement is
 * independent of the product's data structures.
 */
#ifndef DSB_RESTATE_H
#define DSB_RESTATE_H
#include <stddef.h>
#include <stdint.h>

/* CLY_Bit (cly.c:16-34): A0 C1 G2 T3, anything else -> 1 */
uint8_t rs_cly_bit(uint8_t c);
/* getIsland's encoding (cly.c:1245-1254): F at bin[0,L), reverse complement at bin[L,2L) */
void rs_encode_read(const char *seq, uint32_t L, uint8_t *bin);
/* store_kmers (cly.c:359-397): n rolling l-mers, 0 when a base count reaches single_base_max */
void rs_store_kmers(const uint8_t *bin, uint32_t n, int l, int single_base_max, uint64_t *out);
/* hash64_1 / hash64_2 (lib/utils.c:1067-1091) */
uint64_t rs_hash64_1(uint64_t key);
uint64_t rs_hash64_2(uint64_t key);
/* get_exist_kmer (cly.c:951-967) */
int rs_exist_kmer(const uint8_t *ek0, const uint8_t *ek1, uint64_t kmer, uint64_t hash_mask);

/* FM index in the reference's file layout (bwt.c:32-42, 68-104) */
typedef struct {
	const uint8_t *bwt_occ;      /* 168-B blocks: u64 count[5] + 128 B of 4-bit symbols */
	uint64_t rank[6];            /* rank[5] = rank[0] - 1 (bwt.c:81) */
	const uint64_t *hash_index;  /* 13-mer prefix -> [sp, ep) */
	uint64_t dollor_pos;
} rs_fm_t;
/* occ (bwt.c:43-65); *c == 0xff: c := symbol at r, '$' (5) returns dollor_pos */
uint64_t rs_occ(const rs_fm_t *fm, uint64_t r, uint8_t *c);

/* MEM_rst (cly.c:614-622) */
typedef struct {
	int match_len;
	uint64_t sp, sa_sp;
	int sa_sp_l, kmer_index, read_offset;
} rs_mem_t;
/* SP_SET (cly.c:1275-1293) */
typedef struct {
	uint64_t *set;
	int l, m;
} rs_spset_t;
int rs_spset_insert(uint64_t node, rs_spset_t *s);
/* bwt_single_search (cly.c:1339-1378) and bwt_MEM_search (cly.c:1383-1442); `string` points
 * into a 2-bit read and is read backwards */
void rs_single_search(const rs_fm_t *fm, uint64_t sp, const uint8_t *string, int max_match_len, rs_spset_t *set,
		      rs_mem_t *out);
int rs_mem_search(const rs_fm_t *fm, const uint8_t *string, uint64_t pre_v, int max_rst, int l_min, int l_max,
		  rs_spset_t *set, rs_mem_t *out);

/* get_ref (cly.c:434-461) over the 2-bit MSB-first packed reference */
void rs_get_ref(const uint8_t *ref_bin, uint8_t *out, uint64_t uni_offset, uint32_t length, int forward);
/* get_uni (cly.c:466-491): unitig table {ref_list, length}, REF_POS u64 {offset:40, ...} */
typedef struct { uint32_t unitig_ID, offset; } rs_sa_t;
typedef struct { uint32_t ref_list, length; } rs_uni_t;
uint32_t rs_get_uni(const rs_sa_t *sa, const rs_uni_t *uni, const uint64_t *r_p, uint64_t bwt_pos, int search_l,
		    uint64_t *global_offset, uint32_t *uni_offset);
/* lv_extd (cly.c:505-604): banded Landau-Vishkin edit distance, at most 4 errors.  Writes
 * and restores terminators at ref[ref_length] / query[query_length]. */
int32_t rs_lv_extd(uint8_t *ref, int32_t ref_length, uint8_t *query, int32_t query_length);

/* glibc 2.35 qsort (msort_with_tmp: top-down, n1 = n/2, left element when cmp <= 0) */
void rs_msort(void *base, size_t n, size_t size, int (*cmp)(const void *, const void *));

#endif
