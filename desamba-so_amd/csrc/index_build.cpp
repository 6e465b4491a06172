/*
 * index_build.cpp — `desamba_index <SortedKmer> <Reference> <IndexDir>`: the jellyfish-free index
 * builder.  Same inputs and the same index files, byte for byte, as the
 * reference's `deSAMBA index` (reference src/idx.c:884-1101, 1163-1282; src/bwt.c:106-277):
 *
 *   kmer.srt    [u64 n][n sorted distinct forward 31-mers]  (tools/simulate.py writes it; the
 *               reference pipeline gets it from jellyfish + `deSAMBA kmersort`)
 *   Reference   FASTA (plain or gzip), read with the kseq rules of the classify path
 *
 * The stages and what makes each one reproducible:
 *   1. edges    de Bruijn in/out edges of every 31-mer from the ACGT runs of the reference
 *               (build_deb, idx.c:125-239): the reference splits the work over 16 threads by
 *               k-mer suffix; here positions are split over threads and the edge bits are
 *               OR-ed atomically — the same bits whatever the split.
 *   2. labels   unitig start / end flags (setLabel, idx.c:392-512): flag ORs, order-free.
 *   3. unitigs  walks from every start k-mer (get_uni_v, idx.c:723-854): unitig ids, lengths,
 *               start / end k-mers and each k-mer's preceding character (the '$' of the first
 *               unitig), over successors found by one merge pass per first base (walk_unitigs_nx).
 *   4. ref lists REF_UNI records per reference segment, stable-sorted by unitig id, and the
 *               unitigs' ref_list offsets (set_ref_lists, idx.c:554-706), packed reference.
 *   5. BWT      the 30 suffix ("special") k-mers of every unitig sorted with the reference's
 *               own merge schedule (ksort_stable_mt, utils.c:396-510: 15 chunks, bottom-up
 *               merges, ties to the left; spkmer_cmp_l, idx.c:856-880, orders the strings
 *               suffix + '#' lexicographically, so the last levels' merges are cut at merge-path
 *               points and run in parallel) — then
 *               merged with the k-mers into the BWT string and its 13-mer hash index
 *               (merge_kmer, idx.c:345-389; idx.c:933-962).
 *   6. FM index occ check points per 256 symbols, 4-bit BWT, ACGT counters (bwt.c:109-190),
 *               written in 168-byte blocks (bwt.c:193-256).
 *   7. SA       the LF walk from '$' (bwt_cal_SA, idx.c:1163-1237) over a one-cache-line-per-64-
 *               rows rank structure; it also yields the unitig string.
 *   8. Bloom    e-kmer tables from the unitig string (get_EXIST_kmer, idx.c:986-1026), OR-ed
 *               atomically by threads.
 *   9. files    write_idx (idx.c:1046-1101).
 *
 * Bytes the reference leaves undefined and this builder writes as zero: REF_INFO name bytes
 * after the terminator (strcpy into realloc'd memory, idx.c:590), and, when the BWT has at most
 * 256 blocks, the unused tail of the last 128-byte BWT block (bwt.c:226-229 copies the short
 * last block into a reused buffer; with more than 256 blocks those bytes are the same offsets of
 * block n-257, which this builder reproduces).  tests/test_index_build.py compares every file
 * with the reference builder's output, those bytes excepted.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <errno.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/time.h>
#include <atomic>
#include <algorithm>
#include <string>
#include <thread>
#include <vector>

extern "C" {
#include "dsb_host.h"
}

namespace {

constexpr int K = 31;           /* B_KMER */
constexpr int LPRE = 13;        /* L_PRE_IDX */
constexpr int PRE_MOVE = (K - LPRE) * 2; /* 36 */
constexpr uint32_t MIN_UNI_L = 35;
constexpr uint64_t MASK60 = ~(3ull << ((K - 1) * 2)); /* clears the first base of a 31-mer */
constexpr int N_UNI_PARTS = 16;  /* N_T_UNI_V, idx.c:767 */
constexpr int N_SP_SORT = 15;    /* ksort_stable_mt(..., 15), idx.c:928 */
constexpr int N_RU_SORT = 16;    /* idx.c:668 */
const char CHARS[6] = {'A', 'C', 'G', 'T', '#', '$'};

uint8_t BIT[256];    /* ACGT (either case) -> 0..3, anything else 4 (idx.c:9-27) */
uint8_t BIN_BIT[256]; /* ACGT -> 0..3, anything else 0 (idx.c:29-47) */

/* kmerInfo bits, idx.c:52-59: 0-3 out edges, 4-7 in edges, 8 end, 9 start, 10-12 last char */
constexpr uint16_t F_END = 1u << 8, F_START = 1u << 9;

int g_threads = 8;
double t_start;

double now()
{
	struct timeval tv;
	gettimeofday(&tv, nullptr);
	return tv.tv_sec + tv.tv_usec * 1e-6;
}

[[noreturn]] void die(const char *msg, const char *arg = "")
{
	fprintf(stderr, "[desamba_index] error: %s%s\n", msg, arg);
	exit(1);
}

void note(const char *what)
{
	fprintf(stderr, "[desamba_index] %-28s %8.2f s\n", what, now() - t_start);
}

template <class F> void par_for(uint64_t n, int nt, F f)
{
	/* f(lo, hi, t) over nt contiguous slices */
	if (nt <= 1 || n < 2) {
		f(0, n, 0);
		return;
	}
	std::vector<std::thread> th;
	for (int t = 0; t < nt; t++) {
		uint64_t lo = n * t / nt, hi = n * (t + 1) / nt;
		th.emplace_back([=] { f(lo, hi, t); });
	}
	for (auto &x : th) x.join();
}

template <class F> void par_tasks(uint64_t n, int nt, F f)
{
	/* f(i) for i < n, handed out dynamically */
	std::atomic<uint64_t> next{0};
	std::vector<std::thread> th;
	for (int t = 0; t < std::max(1, nt); t++)
		th.emplace_back([&] {
			for (uint64_t i; (i = next.fetch_add(1)) < n;) f(i);
		});
	for (auto &x : th) x.join();
}

inline void or16(uint16_t *p, uint16_t v) { __atomic_fetch_or(p, v, __ATOMIC_RELAXED); }
inline uint16_t ld16(const uint16_t *p) { return __atomic_load_n(p, __ATOMIC_RELAXED); }
inline int popc4(unsigned x) { return __builtin_popcount(x & 15u); }

/* ------------------------------------------------------------------ k-mer table */
struct Kmers {
	uint64_t n = 0;
	std::vector<uint64_t> v;     /* sorted distinct 31-mers */
	std::vector<uint16_t> info;  /* kmerInfo */
	std::vector<uint64_t> bucket; /* first index of each 13-mer prefix, 2^26 + 1 (getCounter, idx.c:95-110) */

	uint64_t find(uint64_t key) const
	{
		uint64_t p = key >> PRE_MOVE, lo = bucket[p], hi = bucket[p + 1], end = hi;
		while (lo < hi) {
			uint64_t mid = lo + ((hi - lo) >> 1);
			if (v[mid] < key)
				lo = mid + 1;
			else
				hi = mid;
		}
		if (lo == end || v[lo] != key) {
			char b[40];
			snprintf(b, sizeof b, "%016llx", (unsigned long long)key);
			die("a reference 31-mer is missing from the sorted k-mer file: ", b);
		}
		return lo;
	}
	/* find() of n keys at once: the bucket words, then the keys' search ranges, are prefetched for
	 * the whole batch before any search runs, so the batch's cache misses overlap instead of
	 * following one another key by key (the de Bruijn edge pass does one search per position) */
	void find_batch(const uint64_t *key, uint64_t *loc, int n) const
	{
		uint64_t p[64];
		for (int k = 0; k < n; k++) {
			p[k] = key[k] >> PRE_MOVE;
			__builtin_prefetch(&bucket[p[k]]);
		}
		for (int k = 0; k < n; k++) {
			uint64_t lo = bucket[p[k]], hi = bucket[p[k] + 1];
			__builtin_prefetch(&v[lo]);
			__builtin_prefetch(&v[lo + ((hi - lo) >> 1)]);
			if (hi > lo)
				__builtin_prefetch(&v[hi - 1]);
		}
		for (int k = 0; k < n; k++)
			loc[k] = find(key[k]);
	}
};

/* ------------------------------------------------------------------ reference */
struct RefSeq {
	std::string name;
	uint64_t off, len; /* into Ref::bases */
};
struct Ref {
	std::vector<char> bases; /* all sequences back to back, each followed by a NUL */
	std::vector<RefSeq> seqs;
	uint64_t total = 0;      /* sum of sequence lengths (build_deb's len_ref) */
};

void load_reference(const char *path, Ref &r)
{
	char *buf;
	uint64_t len, unmap_len;
	if (dsb_open_path(path, &buf, &len, &unmap_len))
		die("cannot read the reference ", path);
	dsb_kseq1 *k = dsb_kseq1_open(buf, len);
	int64_t l;
	while ((l = dsb_kseq1_read(k)) >= 0) {
		RefSeq s;
		s.name = dsb_kseq1_name(k);
		s.len = dsb_kseq1_seq_l(k);
		s.off = r.bases.size();
		const char *q = dsb_kseq1_seq(k);
		r.bases.insert(r.bases.end(), q, q + s.len);
		r.bases.push_back(0);
		r.total += s.len;
		if (s.name.size() >= 128)
			die("reference name longer than 127 bytes (REF_INFO.ref_name[128], idx.c:590): ", s.name.c_str());
		r.seqs.push_back(std::move(s));
	}
	dsb_kseq1_close(k);
	if (unmap_len)
		munmap(buf, unmap_len);
	else
		free(buf);
}

/* ------------------------------------------------------------------ 0: the k-mer list */
/* SortedKmer "-": the sorted distinct forward 31-mers of every ACGT run (either case) of the
 * reference, computed here instead of read from a kmer.srt (the file tools/simulate.py writes, and
 * what the reference's idx_sort makes from a non-canonical jellyfish count, idx_sort.c:101-204).
 * Parallel: positions in 1 Mbp tasks, k-mers bucketed by their first four bases (two passes:
 * count, then place), each bucket sorted and de-duplicated on its own, buckets concatenated. */
void kmers_from_reference(const Ref &ref, Kmers &km)
{
	constexpr uint64_t CHUNK = 1 << 20;
	constexpr int NB = 256;
	struct Task { uint32_t seq; uint64_t lo, hi; };
	std::vector<Task> tasks;
	for (uint32_t i = 0; i < ref.seqs.size(); i++)
		for (uint64_t lo = 0; lo < ref.seqs[i].len; lo += CHUNK)
			tasks.push_back({i, lo, std::min(ref.seqs[i].len, lo + CHUNK)});
	const uint64_t mask = (1ull << 62) - 1;
	/* the k-mers starting in [lo, hi) of one sequence: f(value) for each one made of ACGT only */
	auto each = [&](const Task &t, auto &&f) {
		const char *b = ref.bases.data() + ref.seqs[t.seq].off;
		uint64_t len = ref.seqs[t.seq].len, v = 0;
		int run = 0;
		uint64_t j0 = t.lo >= 30 ? t.lo - 30 : 0; /* the run of bases before the first start position */
		for (uint64_t j = j0; j < len && j < t.hi + 30; j++) {
			uint8_t c = BIT[(uint8_t)b[j]];
			if (c > 3) {
				run = 0;
				continue;
			}
			v = ((v << 2) | c) & mask;
			if (++run >= 31 && j - 30 >= t.lo && j - 30 < t.hi)
				f(v);
		}
	};
	std::vector<uint64_t> cnt(tasks.size() * NB, 0);
	par_tasks(tasks.size(), g_threads, [&](uint64_t i) {
		uint64_t *c = cnt.data() + i * NB;
		each(tasks[i], [&](uint64_t v) { c[v >> 54]++; });
	});
	std::vector<uint64_t> bstart(NB + 1, 0), pos(tasks.size() * NB);
	{
		uint64_t o = 0;
		for (int bk = 0; bk < NB; bk++) {
			bstart[bk] = o;
			for (uint64_t i = 0; i < tasks.size(); i++) {
				pos[i * NB + bk] = o;
				o += cnt[i * NB + bk];
			}
		}
		bstart[NB] = o;
	}
	std::vector<uint64_t>().swap(cnt);
	std::vector<uint64_t> all(bstart[NB]);
	par_tasks(tasks.size(), g_threads, [&](uint64_t i) {
		uint64_t *p = pos.data() + i * NB;
		each(tasks[i], [&](uint64_t v) { all[p[v >> 54]++] = v; });
	});
	std::vector<uint64_t> uniq(NB);
	par_tasks(NB, g_threads, [&](uint64_t bk) {
		uint64_t *a = all.data() + bstart[bk], *e = all.data() + bstart[bk + 1];
		std::sort(a, e);
		uniq[bk] = (uint64_t)(std::unique(a, e) - a);
	});
	uint64_t n = 0;
	for (int bk = 0; bk < NB; bk++) { /* concatenate the buckets' distinct values in place */
		if (n != bstart[bk])
			memmove(all.data() + n, all.data() + bstart[bk], 8 * uniq[bk]);
		n += uniq[bk];
	}
	all.resize(n);
	all.shrink_to_fit();
	km.v.swap(all);
	km.n = n;
}

/* ------------------------------------------------------------------ 1-2: edges and labels */
void build_edges(const Ref &ref, Kmers &km, std::vector<uint64_t> &heads, std::vector<uint64_t> &tails)
{
	/* per position j of an ACGT run [st, en) with j + 31 <= en (build_deb, idx.c:151-233):
	 *   in edge  s[j-1] when j > st,  out edge s[j+31] when j + 31 < en,
	 *   heads when j == st,  tails when j + 31 == en */
	constexpr uint64_t CHUNK = 1 << 20;
	struct Task { uint32_t seq; uint64_t lo, hi; };
	std::vector<Task> tasks;
	for (uint32_t i = 0; i < ref.seqs.size(); i++)
		for (uint64_t lo = 0; lo < ref.seqs[i].len; lo += CHUNK)
			tasks.push_back({i, lo, std::min(ref.seqs[i].len, lo + CHUNK)});
	std::vector<std::vector<uint64_t>> th(tasks.size()), tt(tasks.size());
	uint16_t *info = km.info.data();
	par_tasks(tasks.size(), g_threads, [&](uint64_t ti) {
		const Task &t = tasks[ti];
		const RefSeq &rs = ref.seqs[t.seq];
		const uint8_t *s = (const uint8_t *)ref.bases.data() + rs.off;
		uint64_t L = rs.len;
		auto acgt = [&](uint64_t p) { return p < L && BIT[s[p]] < 4; };
		uint64_t key = 0;
		int run = 0; /* ACGT bases ending at j + 30 */
		uint64_t j0 = t.lo;
		/* prime the rolling k-mer with the 30 bases before position t.lo + 30 */
		for (uint64_t p = j0; p < j0 + K - 1 && p < L; p++) {
			if (BIT[s[p]] < 4) {
				key = ((key << 2) | BIT[s[p]]) & ((1ull << (2 * K)) - 1);
				run++;
			} else {
				key = 0;
				run = 0;
			}
		}
		/* positions are searched in batches of NB (km.find_batch), then applied in order */
		constexpr int NB = 32;
		uint64_t bkey[NB], bloc[NB], bpos[NB];
		int nb = 0;
		auto flush = [&] {
			km.find_batch(bkey, bloc, nb);
			for (int q = 0; q < nb; q++) {
				uint64_t j = bpos[q], loc = bloc[q];
				bool first = !(j > 0 && BIT[s[j - 1]] < 4);
				bool last = !acgt(j + K);
				uint16_t e = 0;
				if (!first)
					e |= (uint16_t)(1u << (BIT[s[j - 1]] + 4));
				if (!last)
					e |= (uint16_t)(1u << BIT[s[j + K]]);
				if (e)
					or16(info + loc, e);
				if (first)
					th[ti].push_back(loc);
				if (last)
					tt[ti].push_back(loc);
			}
			nb = 0;
		};
		for (uint64_t j = j0; j < t.hi; j++) {
			uint64_t p = j + K - 1;
			if (p >= L)
				break;
			if (BIT[s[p]] < 4) {
				key = ((key << 2) | BIT[s[p]]) & ((1ull << (2 * K)) - 1);
				run++;
			} else {
				key = 0;
				run = 0;
			}
			if (run < K)
				continue;
			bkey[nb] = key;
			bpos[nb] = j;
			if (++nb == NB)
				flush();
		}
		flush();
	});
	for (auto &v : th) heads.insert(heads.end(), v.begin(), v.end());
	for (auto &v : tt) tails.insert(tails.end(), v.begin(), v.end());
}

uint64_t set_labels(Kmers &km, const std::vector<uint64_t> &heads, const std::vector<uint64_t> &tails)
{
	uint16_t *info = km.info.data();
	const uint64_t *v = km.v.data();
	auto preds = [&](uint64_t i, uint16_t in_edges) { /* setEnd on every predecessor */
		for (unsigned j = 0; j < 4; j++)
			if (in_edges >> j & 1)
				or16(info + km.find((v[i] >> 2) | ((uint64_t)j << ((K - 1) * 2))), F_END);
	};
	auto succs = [&](uint64_t i, uint16_t out_edges) { /* setStart on every successor */
		for (unsigned j = 0; j < 4; j++)
			if (out_edges >> j & 1)
				or16(info + km.find(((v[i] & MASK60) << 2) | j), F_START);
	};
	/* cutOffMulEdges, idx.c:392-438 (edge bits no longer change: the flag ORs commute) */
	par_for(km.n, g_threads, [&](uint64_t lo, uint64_t hi, int) {
		for (uint64_t i = lo; i < hi; i++) {
			uint16_t x = ld16(info + i);
			int in = popc4(x >> 4), out = popc4(x);
			if (in != 1) {
				or16(info + i, F_START);
				preds(i, (x >> 4) & 15);
			}
			if (out != 1) {
				or16(info + i, F_END);
				succs(i, x & 15);
			}
		}
	});
	/* handleFrstLastKmer, idx.c:440-489 */
	par_for(heads.size(), g_threads, [&](uint64_t lo, uint64_t hi, int) {
		for (uint64_t k = lo; k < hi; k++) {
			uint64_t i = heads[k];
			or16(info + i, F_START);
			preds(i, (ld16(info + i) >> 4) & 15);
		}
	});
	par_for(tails.size(), g_threads, [&](uint64_t lo, uint64_t hi, int) {
		for (uint64_t k = lo; k < hi; k++) {
			uint64_t i = tails[k];
			or16(info + i, F_END);
			succs(i, ld16(info + i) & 15);
		}
	});
	std::atomic<uint64_t> n_end{0};
	par_for(km.n, g_threads, [&](uint64_t lo, uint64_t hi, int) {
		uint64_t c = 0;
		for (uint64_t i = lo; i < hi; i++) c += (info[i] & F_END) != 0;
		n_end += c;
	});
	return n_end;
}

/* ------------------------------------------------------------------ 3: unitigs */
struct Unitigs {
	std::vector<uint32_t> len;    /* per unitig */
	std::vector<uint64_t> start;  /* start k-mer (sorted) */
	std::vector<uint64_t> end;    /* end k-mer (sp_kmer_ori) */
};

void walk_unitigs(Kmers &km, uint64_t n_uni, Unitigs &u)
{
	/* get_uni_v_worker, idx.c:723-765, over the reference's 16 index ranges */
	uint16_t *info = km.info.data();
	const uint64_t *v = km.v.data();
	uint64_t step = km.n / N_UNI_PARTS;
	std::vector<Unitigs> part(N_UNI_PARTS);
	par_tasks(N_UNI_PARTS, g_threads, [&](uint64_t t) {
		uint64_t lo = step * t, hi = (t == N_UNI_PARTS - 1) ? km.n : step * (t + 1);
		uint16_t last = (lo == 0) ? (uint16_t)(5u << 10) : (uint16_t)(4u << 10);
		Unitigs &p = part[t];
		for (uint64_t i = lo; i < hi; i++) {
			if (!(ld16(info + i) & F_START))
				continue;
			or16(info + i, last);
			uint64_t loc = i;
			uint32_t L = K;
			uint16_t x;
			while (!((x = ld16(info + loc)) & F_END)) {
				last = (uint16_t)((v[loc] >> ((K - 1) * 2)) << 10);
				unsigned nc = 0;
				while (!((x >> nc) & 1)) {
					if (++nc >= 4)
						die("unitig walk reached a k-mer without an out edge");
				}
				loc = km.find(((v[loc] & MASK60) << 2) | nc);
				or16(info + loc, last);
				L++;
			}
			p.end.push_back(v[loc]);
			last = (uint16_t)(4u << 10);
			p.len.push_back(L);
			p.start.push_back(v[i]);
		}
	});
	for (auto &p : part) {
		u.len.insert(u.len.end(), p.len.begin(), p.len.end());
		u.start.insert(u.start.end(), p.start.begin(), p.start.end());
		u.end.insert(u.end.end(), p.end.begin(), p.end.end());
	}
	if (u.len.size() != n_uni)
		die("unitig count differs from the number of end k-mers");
}

/* The same walks without a search per step.
 *
 * Successors: a k-mer x that is not an end has exactly one out edge c, and its successor is
 * ((x & MASK60) << 2) | c.  The k-mers with one first base are a contiguous range of the sorted
 * list, and over such a range that key increases with the index, so every successor of a slice of
 * the list is found by one forward merge over the list (nx[i], sequential reads) instead of a
 * bucketed binary search per walk step (several dependent cache misses each: 80 of the 182 s of
 * the c2l18 build, 179 of 470 s for c2xl, in the range form above).
 *
 * Preceding characters: the walk ORs into every k-mer after a unitig's first the first base of
 * the k-mer it came from.  A successor y of a non-end x has exactly one in edge (setLabel marks x
 * an end when y has in != 1 or is a sequence head, idx.c:392-489), and that edge's character is
 * x's first base; so a walk step reads only nx[] and y's flags.  Unitig starts take '#', except the
 * first start of the whole list, which the reference's range 0 gives '$' (idx.c:741-745).
 *
 * Unitig ids follow the start k-mers' order in the list in both forms (the ranges are contiguous
 * and walked in order), so the starts are handed out in slices and the slices concatenated. */
template <class IX> void walk_unitigs_nx(Kmers &km, uint64_t n_uni, Unitigs &u)
{
	uint16_t *info = km.info.data();
	const uint64_t *v = km.v.data();
	const uint64_t n = km.n;
	std::vector<IX> nx(n);
	constexpr uint64_t SLICE = 1 << 22;
	const uint64_t n_sl = (n + SLICE - 1) / SLICE;
	par_tasks(n_sl, g_threads, [&](uint64_t s) {
		uint64_t lo = s * SLICE, hi = std::min(n, lo + SLICE), j = 0;
		int grp = -1;
		for (uint64_t i = lo; i < hi; i++) {
			uint16_t x = ld16(info + i);
			if (x & F_END)
				continue;
			unsigned c = (unsigned)__builtin_ctz(x & 15u);
			if ((x & 15u) == 0)
				die("unitig walk reached a k-mer without an out edge");
			uint64_t key = ((v[i] & MASK60) << 2) | c;
			int b = (int)(v[i] >> ((K - 1) * 2));
			if (b != grp) { /* a new first-base range: the merge restarts at a search */
				grp = b;
				j = (uint64_t)(std::lower_bound(v, v + n, key) - v);
			}
			while (j < n && v[j] < key)
				j++;
			if (j == n || v[j] != key) {
				char t[40];
				snprintf(t, sizeof t, "%016llx", (unsigned long long)key);
				die("a successor 31-mer is missing from the k-mer list: ", t);
			}
			nx[i] = (IX)j;
		}
	});
	uint64_t first_start = n;
	for (uint64_t i = 0; i < n; i++)
		if (ld16(info + i) & F_START) {
			first_start = i;
			break;
		}
	/* each thread advances UW walks of its slice in turn, the next k-mer's successor index and
	 * flags prefetched UW - 1 steps of the other walks before they are needed (one dependent cache
	 * miss per step otherwise: 113 of the c2xl build's 322 s); the slice's unitigs keep the order of
	 * their start k-mers */
	constexpr int UW = 16;
	std::vector<Unitigs> part(n_sl);
	par_tasks(n_sl, g_threads, [&](uint64_t s) {
		uint64_t lo = s * SLICE, hi = std::min(n, lo + SLICE);
		Unitigs &p = part[s];
		uint64_t ns = 0;
		for (uint64_t i = lo; i < hi; i++)
			ns += (ld16(info + i) & F_START) != 0;
		p.len.resize(ns);
		p.start.resize(ns);
		p.end.resize(ns);
		/* a walk's current k-mer is `loc`; `pend`: its preceding character is still to be OR-ed
		 * (done on the walk's next turn, when its flags line has arrived) */
		struct Walk { uint64_t i, loc, slot; uint32_t L; int live, pend; };
		uint64_t next = lo, slot = 0;
		auto start = [&](Walk &x) {
			while (next < hi && !(ld16(info + next) & F_START))
				next++;
			x.live = next < hi;
			if (!x.live)
				return;
			x.i = x.loc = next++;
			x.slot = slot++;
			x.L = K;
			x.pend = 0;
			or16(info + x.i, (uint16_t)((x.i == first_start ? 5u : 4u) << 10));
			__builtin_prefetch(&nx[x.loc]);
		};
		Walk w[UW];
		int live = 0;
		for (int j = 0; j < UW; j++) {
			start(w[j]);
			live += w[j].live;
		}
		while (live) {
			for (int j = 0; j < UW; j++) {
				Walk &x = w[j];
				if (!x.live)
					continue;
				uint16_t f = ld16(info + x.loc);
				if (x.pend) {
					unsigned in = (f >> 4) & 15u;
					if (popc4(in) != 1)
						die("unitig walk: a successor without exactly one in edge");
					or16(info + x.loc, (uint16_t)((unsigned)__builtin_ctz(in) << 10));
					x.pend = 0;
				}
				if (!(f & F_END)) { /* one step: the successor's flags and successor index prefetched */
					uint64_t nl = nx[x.loc];
					__builtin_prefetch(info + nl);
					__builtin_prefetch(&nx[nl]);
					x.loc = nl;
					x.L++;
					x.pend = 1;
					continue;
				}
				p.end[x.slot] = v[x.loc];
				p.len[x.slot] = x.L;
				p.start[x.slot] = v[x.i];
				start(x);
				live -= !x.live;
			}
		}
	});
	for (auto &p : part) {
		u.len.insert(u.len.end(), p.len.begin(), p.len.end());
		u.start.insert(u.start.end(), p.start.begin(), p.start.end());
		u.end.insert(u.end.end(), p.end.begin(), p.end.end());
	}
	if (u.len.size() != n_uni)
		die("unitig count differs from the number of end k-mers");
}

/* ------------------------------------------------------------------ 4: reference lists */
#pragma pack(push, 1)
struct UnitigRec { uint32_t ref_list, length; };                    /* UNITIG, idx.h:33-37 */
struct RefUni { uint32_t direction : 1, ref_ID : 31; uint32_t uid, ref_offset; }; /* REF_UNI, idx.h:39-43 */
struct RefInfo { char ref_name[128]; uint64_t seq_l, seq_offset; }; /* REF_INFO, idx.h:28-32 */
struct SaTaxon { uint32_t unitig_ID, offset; };                     /* SA_taxon, bwt.h:9-12 */
#pragma pack(pop)
static_assert(sizeof(RefUni) == 12 && sizeof(RefInfo) == 144 && sizeof(UnitigRec) == 8, "layouts");

void ref_lists(const Ref &ref, const Kmers &km, const Unitigs &u, std::vector<UnitigRec> &uv, std::vector<RefUni> &ru,
	       std::vector<uint8_t> &ref_bin)
{
	/* set_ref_lists, idx.c:554-706 (CONSIDER_BOTH_ORIENTATION is off, desc.h:6) */
	uint64_t n_uni = u.len.size();
	std::vector<std::vector<RefUni>> per(ref.seqs.size());
	par_tasks(ref.seqs.size(), g_threads, [&](uint64_t id) {
		const RefSeq &rs = ref.seqs[id];
		const uint8_t *s = (const uint8_t *)ref.bases.data() + rs.off;
		uint64_t L = rs.len;
		for (uint64_t g = 0; g < L; ++g) {
			if (BIT[s[g]] >= 4)
				continue;
			uint64_t st = g;
			while (BIT[s[++g]] != 4 && g < L)
				;
			if (st + K > g)
				continue;
			for (;;) {
				uint64_t key = 0;
				for (int k = 0; k < K; k++) key = (key << 2) | BIT[s[st + k]];
				uint64_t loc = km.find(key);
				if (!(km.info[loc] & F_START))
					die("reference walk: a unitig does not start where the previous one ended");
				auto it = std::lower_bound(u.start.begin(), u.start.end(), key);
				if (it == u.start.end() || *it != key)
					die("reference walk: start k-mer without a unitig");
				uint32_t uid = (uint32_t)(it - u.start.begin());
				uint32_t ul = u.len[uid];
				if (ul >= MIN_UNI_L) {
					RefUni r;
					r.direction = 1; /* FORWARD, utils.h:66 */
					r.ref_ID = (uint32_t)id;
					r.uid = uid;
					r.ref_offset = (uint32_t)st;
					per[id].push_back(r);
				}
				st += ul - K + 1;
				if (st + K > g) {
					if (st + K != g + 1)
						die("reference walk: unitigs overrun an ACGT run");
					break;
				}
			}
		}
	});
	for (auto &p : per) ru.insert(ru.end(), p.begin(), p.end());
	/* ksort_stable_mt with REF_UNITIG_cmp_by_UNITIG_ID: a total preorder, so any stable sort
	 * gives the reference's order (ascending unitig id, reference order within one) */
	std::stable_sort(ru.begin(), ru.end(), [](const RefUni &a, const RefUni &b) { return a.uid < b.uid; });
	(void)N_RU_SORT;
	uv.assign(n_uni + 1000 + 1, UnitigRec{0, 0});
	for (uint64_t i = 0; i < n_uni; i++) uv[i].length = u.len[i];
	uint32_t old = UINT32_MAX;
	for (uint32_t r = 0; r < ru.size(); r++) {
		uint32_t c = ru[r].uid;
		if (old != c) {
			if (uv[c].ref_list != 0) {
				if (uv[c].ref_list != r)
					die("ref_list bookkeeping differs from the reference's assertion");
			} else
				uv[c].ref_list = r;
			uv[c + 1].ref_list = r + 1;
			old = c;
		} else
			uv[c + 1].ref_list++;
	}
	uv[n_uni].length = 0;
	uv[n_uni].ref_list = (uint32_t)ru.size();
	uv.resize(n_uni + 1);
	/* packed reference, 2 bits per base, first base high, across sequence boundaries */
	ref_bin.assign((ref.total + 3) >> 2, 0);
	uint8_t *rb = ref_bin.data();
	std::vector<uint64_t> g0(ref.seqs.size());
	for (uint64_t i = 0, o = 0; i < ref.seqs.size(); i++) {
		g0[i] = o;
		o += ref.seqs[i].len;
	}
	par_tasks(ref.seqs.size(), g_threads, [&](uint64_t id) {
		const uint8_t *s = (const uint8_t *)ref.bases.data() + ref.seqs[id].off;
		for (uint64_t i = 0; i < ref.seqs[id].len; i++) {
			uint64_t g = g0[id] + i;
			uint8_t b = (uint8_t)(BIN_BIT[s[i]] << (6 - 2 * (g & 3)));
			if (b)
				__atomic_fetch_or(rb + (g >> 2), b, __ATOMIC_RELAXED);
		}
	});
}

/* ------------------------------------------------------------------ 5: special k-mers, BWT */
struct SpK {
	uint64_t v;   /* value[8] as a little-endian u64 */
	int8_t pos;   /* sp_pos */
	int8_t last;  /* last_char */
};

/* spkmer_cmp_l, idx.c:856-880 */
inline int sp_cmp(const SpK &a, const SpK &b)
{
	if (a.pos < b.pos) {
		int mv = (b.pos - a.pos) << 1;
		return a.v <= (b.v >> mv) ? 1 : -1;
	}
	if (a.pos > b.pos) {
		int mv = (a.pos - b.pos) << 1;
		return (a.v >> mv) < b.v ? 1 : -1;
	}
	return a.v < b.v ? 1 : (a.v > b.v ? -1 : 0);
}

/* one pass of ksort_stable_step (utils.c:396-461): runs of `w` elements merged pairwise,
 * the left element taken when cmp(left, right) >= 0, a trailing lone run copied.
 *
 * spkmer_cmp_l orders the strings "the last sp_pos bases of the k-mer, then '#'" lexicographically
 * with '#' below every base (cmp 1: a before b, -1: after, 0: the same string), a total preorder,
 * so "cmp(left, right) >= 0" is the stable merge rule and the merge path can be cut anywhere: the
 * last levels (a few huge merges, one thread each in the reference's schedule) are split into
 * segments at merge-path points found by binary search (the smallest i on output diagonal k with
 * B[k-i-1] before A[i]) and the segments merged in parallel — the same output element by element.
 * DSB_INDEX_SERIAL_MERGE=1 merges each pair on one thread (the check). */
void merge_pass(const SpK *from, SpK *to, uint64_t n, uint64_t w, int nt)
{
	uint64_t pairs = 0;
	for (uint64_t b = 0; b + w < n; b += 2 * w) pairs++;
	auto merge_seg = [&](const SpK *a, uint64_t na, const SpK *b, uint64_t nb, SpK *o) {
		uint64_t p1 = 0, p2 = 0, p = 0;
		while (p1 < na && p2 < nb) {
			if (sp_cmp(a[p1], b[p2]) >= 0)
				o[p++] = a[p1++];
			else
				o[p++] = b[p2++];
		}
		while (p1 < na) o[p++] = a[p1++];
		while (p2 < nb) o[p++] = b[p2++];
	};
	/* elements of A among the first k outputs of merging A and B */
	auto split = [&](const SpK *a, uint64_t na, const SpK *b, uint64_t nb, uint64_t k) -> uint64_t {
		uint64_t lo = k > nb ? k - nb : 0, hi = std::min(k, na);
		while (lo < hi) {
			uint64_t mid = lo + ((hi - lo) >> 1);
			if (sp_cmp(a[mid], b[k - mid - 1]) < 0) /* B[k-mid-1] goes before A[mid] */
				hi = mid;
			else
				lo = mid + 1;
		}
		return lo;
	};
	const char *ser = getenv("DSB_INDEX_SERIAL_MERGE");
	uint64_t segs = (nt > 1 && pairs < (uint64_t)nt * 4 && !(ser && *ser == '1')) ? ((uint64_t)nt * 8 + pairs - 1) / pairs : 1;
	auto one = [&](uint64_t q) {
		uint64_t k = q / segs, sg = q % segs;
		uint64_t b1 = k * 2 * w, e1 = b1 + w, b2 = e1, e2 = std::min(b2 + w, n);
		const SpK *A = from + b1, *B = from + b2;
		uint64_t na = e1 - b1, nb = e2 - b2, tot = na + nb;
		uint64_t k0 = tot * sg / segs, k1 = tot * (sg + 1) / segs;
		uint64_t i0 = split(A, na, B, nb, k0), i1 = split(A, na, B, nb, k1);
		merge_seg(A + i0, i1 - i0, B + (k0 - i0), (k1 - i1) - (k0 - i0), to + b1 + k0);
	};
	if (nt > 1 && pairs * segs > 1)
		par_tasks(pairs * segs, nt, one);
	else
		for (uint64_t q = 0; q < pairs * segs; q++) one(q);
	uint64_t b = pairs * 2 * w;
	if (b < n)
		memcpy(to + b, from + b, (n - b) * sizeof(SpK));
}

/* ksort_stable_step(base, n, ., cmp, w0): bottom-up from runs of w0 */
void ksort_step(SpK *a, SpK *tmp, uint64_t n, uint64_t w0, int nt)
{
	SpK *from = a, *to = tmp;
	for (uint64_t w = w0; w < n; w <<= 1) {
		merge_pass(from, to, n, w, nt);
		std::swap(from, to);
	}
	if (from != a)
		memcpy(a, from, n * sizeof(SpK));
}

/* ksort_stable_mt(base, n, ., cmp, 15), utils.c:490-510 */
void sort_special(std::vector<SpK> &sp)
{
	uint64_t n = sp.size();
	std::vector<SpK> tmp(n);
	uint64_t m = n / N_SP_SORT;
	if (m == 0)
		die("fewer special k-mers than sort chunks (the reference's sort would not terminate)");
	par_tasks(N_SP_SORT, g_threads, [&](uint64_t t) {
		uint64_t lo = m * t, cnt = (t == N_SP_SORT - 1) ? n - m * t : m;
		ksort_step(sp.data() + lo, tmp.data() + lo, cnt, 1, 1);
	});
	ksort_step(sp.data(), tmp.data(), n, m, g_threads);
}

struct Bwt {
	uint64_t len = 0;
	std::vector<uint8_t> code;        /* 0-5: A C G T # $ */
	std::vector<uint64_t> hash_index; /* compressed, 2^26 + 1 */
};

void build_bwt_string(const Kmers &km, const Unitigs &u, Bwt &bw)
{
	uint64_t n_uni = u.len.size(), n_sp = n_uni * (K - 1);
	/* genSpKmers, idx.c:514-526: the 30 prefixes of each unitig's end k-mer */
	std::vector<SpK> sp(n_sp);
	par_for(n_uni, g_threads, [&](uint64_t lo, uint64_t hi, int) {
		for (uint64_t i = lo; i < hi; i++) {
			uint64_t kv = u.end[i], mask = (1ull << ((K - 1) * 2)) - 1;
			SpK *p = sp.data() + i * (K - 1);
			for (int pos = K - 1; pos > 0; pos--, p++, mask >>= 2) {
				p->v = kv & mask;
				p->pos = (int8_t)pos;
				p->last = (int8_t)((kv >> (pos << 1)) & 3);
			}
		}
	});
	note("special k-mers");
	sort_special(sp);
	note("special k-mers sorted");
	bw.len = n_uni + km.n + n_sp;
	bw.code.resize(bw.len);
	uint8_t *c = bw.code.data();
	for (uint64_t i = 0; i < n_uni; i++) c[i] = (uint8_t)(u.end[i] & 3);
	/* merge_kmer, idx.c:345-389 + the hash index (idx.c:933-959) */
	const uint64_t HSZ = 1ull << (2 * LPRE + 1);
	std::vector<uint64_t> h(HSZ, UINT64_MAX);
	uint64_t pre = UINT64_MAX, pos = n_uni, b = 0;
	auto store_hash = [&](uint64_t key, uint64_t idx) {
		if (key != pre) {
			h[key << 1] = idx;
			h[(key << 1) + 1] = idx + 1;
			pre = key;
		} else
			++h[(key << 1) + 1];
	};
	auto emit_kmer = [&](uint64_t i) {
		unsigned lc = (km.info[i] >> 10) & 7;
		if (lc > 5)
			die("k-mer with an undefined preceding character");
		c[pos] = (uint8_t)lc;
		store_hash(km.v[i] >> PRE_MOVE, pos);
		pos++;
	};
	for (const SpK &s : sp) {
		uint64_t key = s.v << ((K - s.pos) << 1);
		while (b < km.n && km.v[b] < key) emit_kmer(b++);
		c[pos] = (uint8_t)s.last;
		if (s.pos >= LPRE)
			store_hash(s.v >> ((s.pos - LPRE) << 1), pos);
		pos++;
	}
	while (b < km.n) emit_kmer(b++);
	if (pos != bw.len)
		die("BWT length mismatch");
	bw.hash_index.assign((1ull << (2 * LPRE)) + 1, 0);
	uint64_t pv = 0;
	for (uint64_t i = 0; i < HSZ; i += 2) {
		if (h[i] != UINT64_MAX) {
			bw.hash_index[i >> 1] = h[i];
			pv = h[i + 1];
		} else
			bw.hash_index[i >> 1] = pv;
	}
	bw.hash_index.back() = pv;
}

/* ------------------------------------------------------------------ 6-7: FM index, SA walk */
/* rank structure: one 48-byte line per 64 rows — three bit planes of the symbol codes and the
 * counts of A C G T # before the line since the start of its 2^32-row superblock (u32), plus the
 * absolute counts at every superblock start (u64): BWTs past 2^32 rows (the reference's rows are
 * uint64_t, src/bwt.h:45) */
struct RankLine {
	uint64_t plane[3];
	uint32_t cnt[5];
	uint32_t pad;
};
static_assert(sizeof(RankLine) == 48, "rank line");
#ifndef RANK_SB_SHIFT
#define RANK_SB_SHIFT 32 /* tests build it at 16 too (bin/desamba_index_sb16) */
#endif

struct Rank {
	std::vector<RankLine> line;
	std::vector<uint64_t> sb; /* 5 per 2^32 rows */
	uint64_t C[5];
	void build(const uint8_t *code, uint64_t n, const uint64_t *rank)
	{
		uint64_t nl = (n + 64) / 64, lines_per_sb = 1ull << (RANK_SB_SHIFT - 6);
		line.assign(nl, RankLine{});
		sb.assign(5 * ((nl + lines_per_sb - 1) / lines_per_sb), 0);
		/* superblocks in parallel: counts per superblock first, then the lines */
		uint64_t nsb = sb.size() / 5;
		std::vector<uint64_t> tot(6 * nsb, 0);
		par_tasks(nsb, g_threads, [&](uint64_t k) {
			uint64_t lo = k << RANK_SB_SHIFT, hi = std::min(n, (k + 1) << RANK_SB_SHIFT);
			for (uint64_t i = lo; i < hi; i++) tot[6 * k + code[i]]++;
		});
		for (uint64_t k = 1; k < nsb; k++)
			for (int c = 0; c < 5; c++) sb[5 * k + c] = sb[5 * (k - 1) + c] + tot[6 * (k - 1) + c];
		par_for(nl, g_threads, [&](uint64_t l0, uint64_t l1, int) {
			if (l0 >= l1)
				return;
			/* counts before line l0 within its superblock */
			uint64_t sbl = (l0 / lines_per_sb) * lines_per_sb;
			uint32_t cnt[6] = {0, 0, 0, 0, 0, 0};
			for (uint64_t i = sbl * 64; i < std::min(n, l0 * 64); i++) cnt[code[i]]++;
			for (uint64_t l = l0; l < l1; l++) {
				if (l % lines_per_sb == 0)
					memset(cnt, 0, sizeof(cnt));
				RankLine &r = line[l];
				for (int c = 0; c < 5; c++) r.cnt[c] = cnt[c];
				for (uint64_t i = l * 64; i < std::min(n, l * 64 + 64); i++) {
					uint8_t x = code[i];
					for (int b = 0; b < 3; b++) r.plane[b] |= (uint64_t)((x >> b) & 1) << (i & 63);
					cnt[x]++;
				}
			}
		});
		for (int c = 0; c < 5; c++) C[c] = rank[c];
	}
	inline uint8_t sym(uint64_t r) const
	{
		const RankLine &l = line[r >> 6];
		unsigned s = r & 63;
		return (uint8_t)(((l.plane[0] >> s) & 1) | (((l.plane[1] >> s) & 1) << 1) | (((l.plane[2] >> s) & 1) << 2));
	}
	/* build_LFC, bwt.c:171-190: C[c] + occurrences of c in rows [0, r) */
	inline uint64_t lf(uint64_t r, uint8_t c) const
	{
		const RankLine &l = line[r >> 6];
		uint64_t m0 = (c & 1) ? l.plane[0] : ~l.plane[0];
		uint64_t m1 = (c & 2) ? l.plane[1] : ~l.plane[1];
		uint64_t m2 = (c & 4) ? l.plane[2] : ~l.plane[2];
		uint64_t eq = m0 & m1 & m2 & ((1ull << (r & 63)) - 1);
		return C[c] + sb[5 * (r >> RANK_SB_SHIFT) + c] + l.cnt[c] + (uint64_t)__builtin_popcountll(eq);
	}
};

struct Fm {
	uint64_t rank[5];
	std::vector<uint64_t> occ; /* 5 per 256-symbol block */
};

void fm_checkpoints(const Bwt &bw, Fm &fm)
{
	/* bwt_cal_check_point, bwt.c:109-138 */
	uint64_t nb = (bw.len + 255) / 256;
	fm.occ.assign(nb * 5, 0);
	uint64_t t[6] = {0, 0, 0, 0, 0, 0};
	for (uint64_t b = 0; b < nb; b++) {
		for (int j = 0; j < 5; j++) fm.occ[b * 5 + j] = t[j];
		for (uint64_t i = b * 256; i < std::min(bw.len, b * 256 + 256); i++) t[bw.code[i]]++;
	}
	fm.rank[0] = t[4] + t[5];
	fm.rank[1] = fm.rank[0] + t[0];
	fm.rank[2] = fm.rank[1] + t[1];
	fm.rank[3] = fm.rank[2] + t[2];
	fm.rank[4] = 0;
}

/* bwt_cal_SA, idx.c:1163-1237, as the reference runs it: one LF walk from '$' backwards over
 * the whole text (DSB_INDEX_SERIAL_SA=1; the check of sa_walk_par) */
void sa_walk_serial(const Bwt &bw, const Rank &rk, const std::vector<UnitigRec> &uv, std::vector<SaTaxon> &sa,
		    std::vector<uint8_t> &uni)
{
	uint64_t sa_size = (bw.len + 7) / 8;
	sa.assign(sa_size, SaTaxon{0, 0});
	std::vector<uint8_t> filled(sa_size, 0);
	uni.assign(bw.len, 0);
	int64_t cnt = (int64_t)bw.len - 1;
	uint32_t uid = (uint32_t)(uv.size() - 2);
	uint32_t offset = uv[uid].length - 1;
	uint64_t occ = uv.size() - 2; /* DOLLOR_POS */
	auto put_sa = [&](uint64_t r, uint32_t id, uint32_t off) {
		if ((r & 7) == 0) {
			sa[r >> 3] = SaTaxon{id, off};
			filled[r >> 3] = 1;
		}
	};
	uni[cnt--] = 5;
	uint8_t c = rk.sym(occ);
	uni[cnt--] = c;
	put_sa(occ, uid, offset);
	offset--;
	for (;;) {
		occ = rk.lf(occ, c);
		c = rk.sym(occ);
		if (c == 4) {
			if (uid == 0)
				break;
			uid--;
			if (offset != UINT32_MAX)
				die("SA walk: unitig offset not exhausted at '#'");
			offset = uv[uid].length;
		}
		if (c == 5) {
			if (offset != UINT32_MAX)
				die("SA walk: unitig offset not exhausted at '$'");
			break;
		}
		if (cnt < 0)
			die("SA walk longer than the BWT");
		uni[cnt--] = c;
		put_sa(occ, uid, offset);
		offset--;
	}
	if ((occ & 7) == 0) {
		uint32_t id = (uint32_t)(uv.size() - 2);
		sa[occ >> 3] = SaTaxon{id, uv[id].length};
		filled[occ >> 3] = 1;
	}
	if (cnt != -1)
		die("SA walk did not cover the BWT");
	for (uint64_t i = 0; i < sa_size; i++)
		if (!filled[i])
			die("SA walk left a sample unset");
}

/* The same samples and unitig string from n_uni independent walks.  The text the walk reads is
 * U_0 # U_1 # ... # U_{n-1} $; BWT row i < n_uni is the separator after U_i (merge_kmer emits
 * those rows first, in unitig order: idx.c:924-925), whose BWT symbol is U_i's last base.  The
 * serial walk stores, for every row r, the (unitig, offset) of r's BWT symbol (the separator after
 * U_i being offset len_i of U_i) — so walking back from row i through U_i's len_i bases gives
 * rows whose symbols are U_i[len_i - 1 .. 0], and one more LF step the row whose symbol is the
 * separator before U_i: (i - 1, len_{i-1}), or for i = 0 the '$' the serial walk assigns after
 * its loop ((n - 1, len_{n-1})).  Each walk is a chain of dependent LF steps; the chains run in
 * parallel. */
void sa_walk_par(const Bwt &bw, const Rank &rk, const std::vector<UnitigRec> &uv, std::vector<SaTaxon> &sa,
		 std::vector<uint8_t> &uni)
{
	uint64_t n = uv.size() - 1, sa_size = (bw.len + 7) / 8;
	sa.assign(sa_size, SaTaxon{0, 0});
	std::vector<uint8_t> filled(sa_size, 0);
	uni.assign(bw.len, 0);
	std::vector<uint64_t> st(n + 1);
	for (uint64_t u = 0, s = 0; u <= n; u++) {
		st[u] = s;
		s += (uint64_t)uv[u].length + 1;
	}
	if (st[n] != bw.len)
		die("unitig lengths do not add up to the BWT length");
	/* each thread advances SA_G walks of its block in turn: a step's one cache miss (the rank line
	 * of the next row) is prefetched SA_G - 1 steps of the other walks before it is needed */
	constexpr int SA_G = 16;
	struct Walk { uint64_t i, r; uint32_t len, k; int live; };
	std::atomic<int> bad{0};
	par_tasks((n + 1023) / 1024, g_threads, [&](uint64_t blk) {
		uint64_t next = blk * 1024, end = std::min(n, blk * 1024 + 1024);
		auto start = [&](Walk &x) {
			x.live = next < end;
			if (!x.live)
				return;
			x.i = next++;
			x.len = uv[x.i].length;
			x.r = x.i;
			x.k = 0;
			__builtin_prefetch(&rk.line[x.r >> 6]);
		};
		Walk w[SA_G];
		int live = 0;
		for (int j = 0; j < SA_G; j++) {
			start(w[j]);
			live += w[j].live;
		}
		while (live) {
			for (int j = 0; j < SA_G; j++) {
				Walk &x = w[j];
				if (!x.live)
					continue;
				uint8_t c = rk.sym(x.r);
				if (x.k < x.len) { /* U_i[len - 1 - k] */
					if (c > 3) {
						bad = 1;
						return;
					}
					uint32_t off = x.len - 1 - x.k;
					uni[st[x.i] + off] = c;
					if ((x.r & 7) == 0) {
						sa[x.r >> 3] = SaTaxon{(uint32_t)x.i, off};
						filled[x.r >> 3] = 1;
					}
					x.r = rk.lf(x.r, c);
					__builtin_prefetch(&rk.line[x.r >> 6]);
					x.k++;
					continue;
				}
				if (c != 4 && c != 5) { /* the separator before U_i */
					bad = 2;
					return;
				}
				uni[st[x.i] + x.len] = (x.i == n - 1) ? 5 : 4;
				if ((x.r & 7) == 0) {
					uint32_t id = x.i ? (uint32_t)(x.i - 1) : (uint32_t)(n - 1);
					sa[x.r >> 3] = SaTaxon{id, uv[id].length};
					filled[x.r >> 3] = 1;
				}
				start(x);
				live -= !x.live;
			}
		}
	});
	if (bad)
		die(bad == 1 ? "SA walk met a separator inside a unitig" : "SA walk: a unitig does not end at a separator");
	for (uint64_t i = 0; i < sa_size; i++)
		if (!filled[i])
			die("SA walk left a sample unset");
}

/* ------------------------------------------------------------------ 8: e-kmer Bloom tables */
uint64_t hash64_1(uint64_t key) /* reference src/lib/utils.c:1067-1077 */
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
uint64_t hash64_2(uint64_t key) /* reference src/lib/utils.c:1080-1091 */
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

struct Ekmer {
	uint64_t size;
	int l_ek;
	uint64_t mask;
	std::vector<uint8_t> t0, t1;
};

void ekmer_params(uint64_t n_kmer, Ekmer &ek)
{
	/* get_EXIST_kmer's size choice + set_ekmer_par, idx.c:966-997 */
	static const uint64_t size[8] = {1ull << 27, 1ull << 28, 1ull << 29, 1ull << 30,
					 1ull << 31, 1ull << 32, 1ull << 33, 1ull << 34};
	static const int lek[8] = {16, 17, 17, 18, 18, 19, 19, 20};
	int k = 7;
	for (int i = 0; i < 8; i++)
		if (n_kmer < (1ull << (31 + i)) / 9) {
			k = i;
			break;
		}
	ek.size = size[k];
	ek.l_ek = lek[k];
	ek.mask = (1ull << (30 + k)) - 1; /* MASK_30 .. MASK_37 */
}

void ekmer_tables(const std::vector<UnitigRec> &uv, const std::vector<uint8_t> &uni, Ekmer &ek)
{
	/* get_EXIST_kmer, idx.c:1008-1025: every l_ek-mer inside every unitig of the unitig string */
	ek.t0.assign(ek.size, 0);
	ek.t1.assign(ek.size, 0);
	uint64_t n = uv.size() - 1, L = (uint64_t)ek.l_ek;
	uint64_t kmask = (1ull << (2 * L)) - 1;
	std::vector<uint64_t> st(n + 1);
	for (uint64_t u = 0, s = 0; u <= n; u++) {
		st[u] = s;
		s += (uint64_t)uv[u].length + 1;
	}
	uint8_t *t0 = ek.t0.data(), *t1 = ek.t1.data();
	const uint8_t *us = uni.data();
	par_tasks((n + 4095) / 4096, g_threads, [&](uint64_t blk) {
		for (uint64_t u = blk * 4096; u < std::min(n, blk * 4096 + 4096); u++) {
			uint64_t s = st[u], e = s + uv[u].length - L + 1;
			uint64_t kmer = 0;
			for (uint64_t i = 0; i + 1 < L; i++) kmer = (kmer << 2) | us[s + i];
			for (uint64_t i = s; i < e; i++) {
				kmer = ((kmer << 2) | us[i + L - 1]) & kmask;
				uint64_t h1 = hash64_1(kmer) & ek.mask, h2 = hash64_2(kmer) & ek.mask;
				__atomic_fetch_or(t0 + (h1 >> 3), (uint8_t)(0x80u >> (h1 & 7)), __ATOMIC_RELAXED);
				__atomic_fetch_or(t1 + (h2 >> 3), (uint8_t)(0x80u >> (h2 & 7)), __ATOMIC_RELAXED);
			}
		}
	});
}

/* ------------------------------------------------------------------ 9: files */
struct Out {
	std::string dir;
	FILE *open(const char *suffix)
	{
		std::string p = dir + (dir.empty() || dir.back() != '/' ? "/" : "") + "deSAMBA" + suffix;
		FILE *f = fopen(p.c_str(), "wb");
		if (!f)
			die("cannot write ", p.c_str());
		setvbuf(f, nullptr, _IOFBF, 1 << 22);
		return f;
	}
	static void put(FILE *f, const void *p, uint64_t n)
	{
		if (n && fwrite(p, 1, n, f) != n)
			die("short write");
	}
};

void write_bwt(Out &o, const Bwt &bw, const Fm &fm, const std::vector<SaTaxon> &sa)
{
	/* write_bwt, bwt.c:193-256 */
	uint64_t nb = (bw.len + 255) / 256, lbin = (bw.len + 1) >> 1;
	std::vector<uint8_t> bin(nb * 128, 0); /* bwt_str2bwt_occ, bwt.c:140-154: low nibble first */
	for (uint64_t i = 0; i + 1 < bw.len; i += 2) bin[i >> 1] = (uint8_t)((bw.code[i + 1] << 4) | bw.code[i]);
	if (bw.len & 1)
		bin[bw.len >> 1] = (uint8_t)(0xF0 | bw.code[bw.len - 1]);
	uint64_t last_copy = lbin - (nb - 1) * 128; /* bytes of the last block taken from the BWT */
	if (nb > 256) /* the rest of the last block: the buffer bytes of block nb - 257 */
		memcpy(bin.data() + (nb - 1) * 128 + last_copy, bin.data() + (nb - 257) * 128 + last_copy, 128 - last_copy);
	FILE *f = o.open(".bwt");
	uint64_t byte_len = nb * 168;
	Out::put(f, &byte_len, 8);
	for (uint64_t b = 0; b < nb; b++) {
		Out::put(f, fm.occ.data() + b * 5, 40);
		Out::put(f, bin.data() + b * 128, 128);
	}
	Out::put(f, fm.rank, 40);
	Out::put(f, bw.hash_index.data(), bw.hash_index.size() * 8);
	fclose(f);
	/* ACGT counters, bwt.c:168-182 */
	f = o.open(".acg");
	uint64_t n16 = 1 << 16;
	Out::put(f, &n16, 8);
	std::vector<uint8_t> t(n16);
	for (unsigned j = 0; j < 5; j++) {
		unsigned m = 0x1111u * j;
		for (unsigned i = 0; i < n16; i++) {
			unsigned x = i ^ m, z = 0;
			for (int k = 0; k < 4; k++, x >>= 4) z += (x & 15) == 0;
			t[i] = (uint8_t)z;
		}
		Out::put(f, t.data(), n16);
	}
	fclose(f);
	f = o.open(".sa");
	uint64_t n = sa.size();
	Out::put(f, &n, 8);
	Out::put(f, sa.data(), n * sizeof(SaTaxon));
	fclose(f);
}

void write_rest(Out &o, const Ekmer &ek, const std::vector<UnitigRec> &uv, const Ref &ref,
		const std::vector<uint8_t> &ref_bin, const std::vector<RefUni> &ru)
{
	/* write_idx, idx.c:1049-1100 */
	FILE *f = o.open(".exk0");
	Out::put(f, ek.t0.data(), ek.size);
	fclose(f);
	f = o.open(".exk1");
	Out::put(f, ek.t1.data(), ek.size);
	fclose(f);
	f = o.open(".exki");
	Out::put(f, &ek.size, 8);
	fclose(f);
	f = o.open(".unv");
	uint64_t n = uv.size();
	Out::put(f, &n, 8);
	Out::put(f, uv.data(), n * sizeof(UnitigRec));
	fclose(f);
	f = o.open(".ref_b");
	n = ref_bin.size();
	Out::put(f, &n, 8);
	Out::put(f, ref_bin.data(), n);
	fclose(f);
	f = o.open(".ref_i");
	n = ref.seqs.size();
	Out::put(f, &n, 8);
	std::vector<uint64_t> seq_off(n);
	for (uint64_t i = 0, s = 0; i < n; i++) {
		RefInfo r;
		memset(&r, 0, sizeof r);
		memcpy(r.ref_name, ref.seqs[i].name.c_str(), ref.seqs[i].name.size() + 1);
		r.seq_l = ref.seqs[i].len;
		r.seq_offset = s;
		seq_off[i] = s;
		s += ref.seqs[i].len;
		Out::put(f, &r, sizeof r);
	}
	fclose(f);
	f = o.open(".ref_p");
	n = ru.size();
	Out::put(f, &n, 8);
	std::vector<uint64_t> rp(n);
	for (uint64_t i = 0; i < n; i++) /* REF_POS {global_offset:40, ref_ID:23, direction:1}, idx.h:45-51 */
		rp[i] = ((seq_off[ru[i].ref_ID] + ru[i].ref_offset) & ((1ull << 40) - 1)) |
			((uint64_t)(ru[i].ref_ID & ((1u << 23) - 1)) << 40) | ((uint64_t)ru[i].direction << 63);
	Out::put(f, rp.data(), n * 8);
	fclose(f);
}

int usage()
{
	fprintf(stderr,
		"Usage: desamba_index [-t threads] <SortedKmer> <Reference> <IndexDir>\n"
		"  SortedKmer  kmer.srt: [u64 n][n sorted distinct 31-mers] (tools/simulate.py reference), or -:\n"
		"              the distinct forward 31-mers of the reference's ACGT runs, computed here\n"
		"  Reference   FASTA (plain or gzip), all reference sequences in one file\n"
		"  IndexDir    output directory (created); the same files as `deSAMBA index`\n");
	return 1;
}

} // namespace

int main(int argc, char **argv)
{
	int a = 1;
	const char *te = getenv("DSB_HOST_THREADS");
	g_threads = te ? atoi(te) : (int)std::max(1u, std::min(32u, std::thread::hardware_concurrency()));
	if (a + 1 < argc && !strcmp(argv[a], "-t")) {
		g_threads = atoi(argv[a + 1]);
		a += 2;
	}
	if (argc - a != 3)
		return usage();
	g_threads = std::max(1, g_threads);
	const char *kpath = argv[a], *rpath = argv[a + 1];
	Out out{argv[a + 2]};
	t_start = now();
	for (int i = 0; i < 256; i++) BIT[i] = 4, BIN_BIT[i] = 0;
	const char *acgt = "ACGT", *lc = "acgt";
	for (int i = 0; i < 4; i++) {
		BIT[(uint8_t)acgt[i]] = BIT[(uint8_t)lc[i]] = (uint8_t)i;
		BIN_BIT[(uint8_t)acgt[i]] = BIN_BIT[(uint8_t)lc[i]] = (uint8_t)i;
	}
	if (mkdir(out.dir.c_str(), 0755) && errno != EEXIST)
		die("cannot create ", out.dir.c_str());

	Kmers km;
	Ref ref;
	if (!strcmp(kpath, "-")) { /* the k-mer list from the reference itself */
		load_reference(rpath, ref);
		note("reference loaded");
		kmers_from_reference(ref, km);
		note("k-mers from the reference");
	} else {
		FILE *f = fopen(kpath, "rb");
		if (!f || fread(&km.n, 8, 1, f) != 1)
			die("cannot read ", kpath);
		km.v.resize(km.n);
		if (fread(km.v.data(), 8, km.n, f) != km.n)
			die("short k-mer file ", kpath);
		fclose(f);
		for (uint64_t i = 1; i < km.n; i++)
			if (km.v[i] <= km.v[i - 1])
				die("k-mer file not sorted / not distinct: ", kpath);
		note("k-mers loaded");
		load_reference(rpath, ref);
		note("reference loaded");
	}
	km.info.assign(km.n, 0);
	km.bucket.assign((1ull << (2 * LPRE)) + 2, 0);
	for (uint64_t i = 0; i < km.n; i++) km.bucket[(km.v[i] >> PRE_MOVE) + 1]++;
	for (uint64_t i = 1; i < km.bucket.size(); i++) km.bucket[i] += km.bucket[i - 1];
	std::vector<uint64_t> heads, tails;
	build_edges(ref, km, heads, tails);
	note("de Bruijn edges");
	uint64_t n_uni = set_labels(km, heads, tails);
	note("unitig labels");
	Unitigs u;
	{
		const char *rw = getenv("DSB_INDEX_RANGE_WALK"); /* the reference's 16 ranges with a search per step */
		if (rw && *rw == '1')
			walk_unitigs(km, n_uni, u);
		else if (km.n < (1ull << 32))
			walk_unitigs_nx<uint32_t>(km, n_uni, u);
		else
			walk_unitigs_nx<uint64_t>(km, n_uni, u);
	}
	note("unitigs");
	std::vector<UnitigRec> uv;
	std::vector<RefUni> ru;
	std::vector<uint8_t> ref_bin;
	ref_lists(ref, km, u, uv, ru, ref_bin);
	note("reference lists");
	Bwt bw;
	build_bwt_string(km, u, bw);
	note("BWT string + hash index");
	{
		std::vector<uint64_t>().swap(km.bucket);
		std::vector<uint16_t>().swap(km.info);
	}
	Fm fm;
	fm_checkpoints(bw, fm);
	std::vector<SaTaxon> sa;
	std::vector<uint8_t> uni;
	{
		Rank rk;
		rk.build(bw.code.data(), bw.len, fm.rank);
		note("rank structure");
		const char *ser = getenv("DSB_INDEX_SERIAL_SA");
		if (ser && *ser == '1')
			sa_walk_serial(bw, rk, uv, sa, uni);
		else
			sa_walk_par(bw, rk, uv, sa, uni);
	}
	note("SA walk");
	write_bwt(out, bw, fm, sa);
	note("BWT / SA written");
	Ekmer ek;
	ekmer_params(km.n, ek);
	ekmer_tables(uv, uni, ek);
	note("e-kmer tables");
	write_rest(out, ek, uv, ref, ref_bin, ru);
	note("done");
	fprintf(stderr, "[desamba_index] %llu k-mers, %llu unitigs, BWT %llu symbols, l_ek %d\n",
		(unsigned long long)km.n, (unsigned long long)n_uni, (unsigned long long)bw.len, ek.l_ek);
	return 0;
}
