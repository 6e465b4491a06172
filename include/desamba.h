/*
 * desamba.h — drop-in C-ABI of the MI355X deSAMBA classifier.
 *
 * Exactly the three entry points an existing libdesamba.so consumer binds with dlsym
 * (reference main_test.c:30-32); each declaration below replaces the one cited.
 * Ownership and argument meaning are unchanged: outputs are malloc'd by the library and
 * released by the caller with free().
 */
#ifndef DESAMBA_H
#define DESAMBA_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Replaces reference desamba.h:10 (impl. src/cly_mt.c:1238-1274).
 * Loads <dirPath>/deSAMBA.* plus nodes.dmp / names.dmp and makes the index resident in the
 * HBM of the current (or $DSB_DEVICE) GPU.  *idx receives an opaque handle.  Exits the
 * process with a message on a missing file or when no GPU is visible. */
void load_index(void **idx, const char *dirPath);

/* Replaces reference desamba.h:23 (impl. src/cly_mt.c:1309-1316, 1041-1081).
 * input/input_n: FASTQ/FASTA text of input_n bytes (gzip accepted), or a file path when
 * input_n == (uint64_t)-1.  *output: malloc'd, zero-filled, NUL-terminated SAM_FULL text of
 * *output_n bytes (no header).  input_n == 0: *output_n = 0 and *output untouched.
 * thread_id selects per-caller state; concurrent calls need distinct thread_ids. */
void read_classify(void *idx, char *input, uint64_t input_n, char **output, uint64_t *output_n, int thread_id,
		   int thread_num);

/* Replaces reference desamba.h:45 (impl. src/cly_mt.c:1329-1414).
 * Summarises read_classify output per taxon: top-3 (+ human > 5 %) report lines
 * "[type]\t[name|rank]\tnull\t[rate]\n", or "no_match\tnull|null\tnull\t0\n".
 * *human_snapshot: malloc'd concatenated human read bases (<= max_snapshot_len) or NULL. */
#define META_USE_READ_NUM 0
#define META_USE_BASE_NUM 1
void meta_analysis(void *idx, char *input, uint64_t input_n, char **output, uint64_t *output_n, int thread_id,
		   int flag, uint64_t max_snapshot_len, char **human_snapshot, uint64_t *human_snapshot_n);

#ifdef __cplusplus
}
#endif
#endif
