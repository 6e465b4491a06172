// tools/gather_calib.hip — measurement tool (GPU box): what rocprofv3's TCC FETCH_SIZE / WRITE_SIZE
// count for the access kinds the classify kernels make, so that the PMC traffic of a kernel can
// be split into its random gathers and scattered stores.
//
// Kernels (each one launch, 64-thread blocks, enough waves to fill the chip):
//   k_gather  N random 4-byte loads over a table of T bytes (dependent pairs: load, then a load
//             at an address derived from the loaded value, as a hash-list walk does)
//   k_scatter N random 4-byte stores over a table of T bytes
//   k_stream  T bytes read once, coalesced (the reference point for the FETCH correction)
//   k_build   the scoring kernel's read-hash build pattern: each wave owns a table of O KB (a
//             read's list heads) and each lane does old = t[key]; t[key] = f(old) at random keys
//
//   gather_calib <table_MB> <million_accesses> [own_KB]
// prints one line per kernel: accesses, HIP-event time; the per-access bytes come from a
// separate `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` pass over the same command.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>

#define CK(x)                                                                                     \
	do {                                                                                      \
		hipError_t e_ = (x);                                                              \
		if (e_ != hipSuccess) {                                                           \
			fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
			exit(1);                                                                  \
		}                                                                                 \
	} while (0)

__device__ inline uint64_t mix(uint64_t x)
{
	x ^= x >> 33;
	x *= 0xff51afd7ed558ccdull;
	x ^= x >> 33;
	x *= 0xc4ceb9fe1a85ec53ull;
	x ^= x >> 33;
	return x;
}

__global__ __launch_bounds__(64) void k_gather(const uint32_t *__restrict__ t, uint64_t words, uint64_t per_lane,
					       uint32_t *__restrict__ sink)
{
	uint64_t id = (uint64_t)blockIdx.x * 64 + threadIdx.x;
	uint32_t acc = 0;
	for (uint64_t k = 0; k < per_lane; k += 2) {
		uint64_t a = mix(id * 0x9E3779B97F4A7C15ull + k) % words;
		uint32_t v = t[a];
		uint64_t b = mix(a ^ v ^ k) % words; /* dependent, like head -> node */
		acc += t[b];
	}
	if (acc == 0x12345678u)
		sink[0] = acc;
}

__global__ __launch_bounds__(64) void k_scatter(uint32_t *__restrict__ t, uint64_t words, uint64_t per_lane)
{
	uint64_t id = (uint64_t)blockIdx.x * 64 + threadIdx.x;
	for (uint64_t k = 0; k < per_lane; k++) {
		uint64_t a = mix(id * 0x9E3779B97F4A7C15ull + k + 7) % words;
		t[a] = (uint32_t)(id + k);
	}
}

__global__ __launch_bounds__(64) void k_build(uint32_t *__restrict__ t, uint32_t own_words, uint64_t per_lane)
{
	uint64_t id = (uint64_t)blockIdx.x * 64 + threadIdx.x;
	uint32_t *own = t + (uint64_t)blockIdx.x * own_words;
	for (uint64_t k = 0; k < per_lane; k++) {
		uint32_t a = (uint32_t)(mix(id * 0x9E3779B97F4A7C15ull + k + 11) & (own_words - 1));
		uint32_t old = own[a];
		own[a] = old + (uint32_t)k;
	}
}

__global__ __launch_bounds__(256) void k_stream(const uint4 *__restrict__ t, uint64_t n, uint32_t *__restrict__ sink)
{
	uint64_t id = (uint64_t)blockIdx.x * 256 + threadIdx.x, stride = (uint64_t)gridDim.x * 256;
	uint32_t acc = 0;
	for (uint64_t i = id; i < n; i += stride) {
		uint4 v = t[i];
		acc ^= v.x ^ v.y ^ v.z ^ v.w;
	}
	if (acc == 0x12345678u)
		sink[0] = acc;
}

int main(int argc, char **argv)
{
	uint64_t mb = argc > 1 ? strtoull(argv[1], 0, 10) : 1024;
	uint64_t acc_m = argc > 2 ? strtoull(argv[2], 0, 10) : 256;
	uint64_t own_kb = argc > 3 ? strtoull(argv[3], 0, 10) : 32; /* power of two */
	uint64_t bytes = mb << 20, words = bytes / 4;
	uint32_t *t, *sink;
	CK(hipMalloc(&t, bytes));
	CK(hipMalloc(&sink, 64));
	CK(hipMemset(t, 1, bytes));
	uint64_t lanes = 64ull * 16384; /* 16384 one-wave blocks: 16 waves per CU on 256 CUs, in flight */
	uint64_t per_lane = (acc_m * 1000000ull + lanes - 1) / lanes;
	per_lane += per_lane & 1;
	hipEvent_t a, b;
	CK(hipEventCreate(&a));
	CK(hipEventCreate(&b));
	float ms;
	/* warm-up */
	k_stream<<<4096, 256>>>((const uint4 *)t, bytes / 16, sink);
	CK(hipDeviceSynchronize());

	CK(hipEventRecord(a));
	k_gather<<<(uint32_t)(lanes / 64), 64>>>(t, words, per_lane, sink);
	CK(hipEventRecord(b));
	CK(hipEventSynchronize(b));
	CK(hipEventElapsedTime(&ms, a, b));
	printf("k_gather  table %lu MB  loads %lu  %.3f ms  %.2f G loads/s\n", (unsigned long)mb,
	       (unsigned long)(lanes * per_lane), ms, lanes * per_lane / (ms * 1e6));

	CK(hipEventRecord(a));
	k_scatter<<<(uint32_t)(lanes / 64), 64>>>(t, words, per_lane);
	CK(hipEventRecord(b));
	CK(hipEventSynchronize(b));
	CK(hipEventElapsedTime(&ms, a, b));
	printf("k_scatter table %lu MB  stores %lu  %.3f ms  %.2f G stores/s\n", (unsigned long)mb,
	       (unsigned long)(lanes * per_lane), ms, lanes * per_lane / (ms * 1e6));

	uint32_t own_words = (uint32_t)(own_kb * 256);
	if ((uint64_t)own_words * 4 * (lanes / 64) <= bytes) {
		CK(hipEventRecord(a));
		k_build<<<(uint32_t)(lanes / 64), 64>>>(t, own_words, per_lane);
		CK(hipEventRecord(b));
		CK(hipEventSynchronize(b));
		CK(hipEventElapsedTime(&ms, a, b));
		printf("k_build   own %lu KB per wave  updates %lu  %.3f ms  %.2f G updates/s\n", (unsigned long)own_kb,
		       (unsigned long)(lanes * per_lane), ms, lanes * per_lane / (ms * 1e6));
	}

	CK(hipEventRecord(a));
	k_stream<<<4096, 256>>>((const uint4 *)t, bytes / 16, sink);
	CK(hipEventRecord(b));
	CK(hipEventSynchronize(b));
	CK(hipEventElapsedTime(&ms, a, b));
	printf("k_stream  table %lu MB  bytes %lu  %.3f ms  %.1f GB/s\n", (unsigned long)mb, (unsigned long)bytes, ms,
	       bytes / (ms * 1e6));
	CK(hipFree(t));
	CK(hipFree(sink));
	return 0;
}
