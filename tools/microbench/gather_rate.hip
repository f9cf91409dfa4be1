/*
 * gather_rate — random-gather ceiling of one MI355X (the roofline of a
 * lookup-bound kernel).  Every lane issues K independent loads of W bytes at
 * uniformly random, W-aligned offsets of a table of S bytes, so the rate is
 * set by the memory level that serves the table (L2 / Infinity Cache / HBM)
 * and by the per-CU address/tag rate, not by latency.
 *
 *   hipcc --offload-arch=gfx950 -O3 gather_rate.hip -o gather_rate
 *   ./gather_rate            -> one JSON line per (S, W)
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x)                                                                         \
	do {                                                                             \
		hipError_t e_ = (x);                                                     \
		if (e_ != hipSuccess) {                                                  \
			fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));          \
			return 1;                                                        \
		}                                                                        \
	} while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x)
{
	x ^= x >> 16;
	x *= 0x7feb352du;
	x ^= x >> 15;
	x *= 0x846ca68bu;
	x ^= x >> 16;
	return x;
}

template <int W, int K>
__global__ __launch_bounds__(256) void gather(const uint4 *tab, uint32_t mask, uint32_t iters, uint32_t *out)
{
	const uint32_t t = blockIdx.x * 256 + threadIdx.x;
	uint32_t acc = 0, h = mix(t * 0x9E3779B9u + 1);
	for (uint32_t it = 0; it < iters; it++) {
		uint32_t v[K];
#pragma unroll
		for (int k = 0; k < K; k++) {
			h = mix(h + k);
			const uint32_t i = h & mask; /* in W-byte units */
			if (W == 16) {
				const uint4 x = tab[i];
				v[k] = x.x ^ x.y ^ x.z ^ x.w;
			} else {
				v[k] = reinterpret_cast<const uint32_t *>(tab)[i];
			}
		}
#pragma unroll
		for (int k = 0; k < K; k++)
			acc += v[k];
	}
	if (acc == 0x12345678u)
		out[t] = acc;
}

template <int W>
static int run(const uint4 *tab, size_t bytes, uint32_t *out, int cus)
{
	constexpr int K = 8;
	const uint32_t mask = (uint32_t)(bytes / W - 1);
	const uint32_t blocks = cus * 8, iters = 64;
	hipEvent_t a, b;
	CHECK(hipEventCreate(&a));
	CHECK(hipEventCreate(&b));
	hipLaunchKernelGGL((gather<W, K>), dim3(blocks), dim3(256), 0, 0, tab, mask, iters, out);
	CHECK(hipEventRecord(a));
	const int reps = 5;
	for (int r = 0; r < reps; r++)
		hipLaunchKernelGGL((gather<W, K>), dim3(blocks), dim3(256), 0, 0, tab, mask, iters, out);
	CHECK(hipEventRecord(b));
	CHECK(hipEventSynchronize(b));
	float ms = 0;
	CHECK(hipEventElapsedTime(&ms, a, b));
	const double loads = (double)blocks * 256 * iters * K * reps;
	printf("{\"table_bytes\": %zu, \"width\": %d, \"gloads_per_s\": %.1f, \"ms\": %.3f}\n", bytes, W,
	       loads / (ms * 1e-3) / 1e9, ms / reps);
	fflush(stdout);
	return 0;
}

int main()
{
	int dev = 0, cus = 0;
	CHECK(hipGetDevice(&dev));
	CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
	const size_t maxb = (size_t)1 << 32;
	uint4 *tab;
	uint32_t *out;
	CHECK(hipMalloc((void **)&tab, maxb));
	CHECK(hipMemset(tab, 1, maxb));
	CHECK(hipMalloc((void **)&out, (size_t)cus * 8 * 256 * 4));
	const size_t sizes[] = {(size_t)256 << 10, (size_t)1 << 20, (size_t)2 << 20, (size_t)4 << 20,
				(size_t)16 << 20, (size_t)64 << 20, (size_t)128 << 20, maxb};
	for (size_t s : sizes) {
		if (run<4>(tab, s, out, cus) || run<16>(tab, s, out, cus))
			return 1;
	}
	CHECK(hipFree(tab));
	CHECK(hipFree(out));
	return 0;
}
