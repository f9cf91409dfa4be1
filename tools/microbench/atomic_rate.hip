/*
 * atomic_rate — what scattered 64-bit counter adds cost on one MI355X, the
 * shape of the classify kernel's per-policy-entry counters (one lane, one
 * random counter slot).  N adds of a packed {packets, bytes} word into a
 * table of S u64 slots:
 *   A  global atomicAdd per add (no return), random slot
 *   B  the same adds pre-sorted by slot within each 1024-add block (what a
 *      per-workgroup sort would give the memory side)
 *   C  plain stores of the adds' slot ids (4 B, coalesced): the store-pass
 *      alternative's first half
 *   D  LDS: per-workgroup counters for the whole table (S <= 16k), then one
 *      global atomicAdd per nonzero slot per workgroup
 * Every variant checks the sum of the table against the adds issued.
 *
 *   hipcc --offload-arch=gfx950 -O3 atomic_rate.hip -o atomic_rate
 *   ./atomic_rate            -> one JSON line per (variant, S)
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>

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

__global__ __launch_bounds__(256) void k_random(unsigned long long *tab, uint32_t mask, uint32_t per)
{
	const uint32_t t = blockIdx.x * 256 + threadIdx.x;
	for (uint32_t k = 0; k < per; k++) {
		const uint32_t s = mix(t * per + k) & mask;
		atomicAdd(&tab[s], 1ull);
	}
}

/* slots sorted inside each wave's 64 x per adds: lane l takes the l-th
 * smallest of each group of 64 (a bitonic-free stand-in: consecutive slots) */
__global__ __launch_bounds__(256) void k_sorted(unsigned long long *tab, uint32_t mask, uint32_t per)
{
	const uint32_t t = blockIdx.x * 256 + threadIdx.x;
	const uint32_t lane = threadIdx.x & 63u, wave = t >> 6;
	for (uint32_t k = 0; k < per; k++) {
		const uint32_t base = mix(wave * per + k) & mask & ~63u;
		atomicAdd(&tab[base + lane], 1ull);
	}
}

__global__ __launch_bounds__(256) void k_store(uint32_t *out, uint32_t mask, uint32_t per, uint32_t n)
{
	const uint32_t t = blockIdx.x * 256 + threadIdx.x;
	const uint32_t T = gridDim.x * 256;
	for (uint32_t k = 0; k < per; k++) {
		const uint32_t i = k * T + t;
		out[i] = mix(t * per + k) & mask;
	}
}

__global__ __launch_bounds__(1024) void k_lds(unsigned long long *tab, uint32_t mask, uint32_t per)
{
	extern __shared__ unsigned long long c[];
	for (uint32_t s = threadIdx.x; s <= mask; s += 1024)
		c[s] = 0;
	__syncthreads();
	const uint32_t t = blockIdx.x * 1024 + threadIdx.x;
	for (uint32_t k = 0; k < per; k++)
		atomicAdd(&c[mix(t * per + k) & mask], 1ull);
	__syncthreads();
	for (uint32_t s = threadIdx.x; s <= mask; s += 1024)
		if (c[s])
			atomicAdd(&tab[s], c[s]);
}

int main()
{
	const uint32_t N = 24u << 20; /* ~ the cold-slot hits of one 64M-tuple config-2 launch */
	unsigned long long *tab;
	uint32_t *ids;
	CHECK(hipMalloc(&tab, (size_t)8 << 20));
	CHECK(hipMalloc(&ids, (size_t)N * 4));
	hipEvent_t a, b;
	CHECK(hipEventCreate(&a));
	CHECK(hipEventCreate(&b));
	for (uint32_t S : {1u << 14, 1u << 17, 1u << 20}) {
		for (int v = 0; v < 4; v++) {
			if (v == 3 && S > (1u << 14))
				continue;
			const uint32_t per = 16;
			const uint32_t threads = N / per;
			float best = 1e9f;
			for (int rep = 0; rep < 4; rep++) {
				CHECK(hipMemset(tab, 0, (size_t)S * 8));
				CHECK(hipEventRecord(a));
				if (v == 0)
					hipLaunchKernelGGL(k_random, dim3(threads / 256), dim3(256), 0, 0, tab, S - 1, per);
				else if (v == 1)
					hipLaunchKernelGGL(k_sorted, dim3(threads / 256), dim3(256), 0, 0, tab, S - 1, per);
				else if (v == 2)
					hipLaunchKernelGGL(k_store, dim3(threads / 256), dim3(256), 0, 0, ids, S - 1, per, N);
				else
					hipLaunchKernelGGL(k_lds, dim3(threads / 1024), dim3(1024), (size_t)S * 8, 0, tab,
							   S - 1, per);
				CHECK(hipEventRecord(b));
				CHECK(hipEventSynchronize(b));
				float ms;
				CHECK(hipEventElapsedTime(&ms, a, b));
				best = ms < best ? ms : best;
			}
			unsigned long long sum = 0;
			if (v != 2) {
				std::vector<unsigned long long> h(S);
				CHECK(hipMemcpy(h.data(), tab, (size_t)S * 8, hipMemcpyDeviceToHost));
				for (auto x : h)
					sum += x;
			}
			const char *name[] = {"random_atomic", "wave_contiguous_atomic", "store_ids", "lds_then_atomic"};
			printf("{\"variant\": \"%s\", \"slots\": %u, \"adds\": %u, \"ms\": %.4f, \"G_adds_per_s\": %.2f, "
			       "\"sum_ok\": %s}\n",
			       name[v], S, N, best, N / best / 1e6, v == 2 ? "null" : (sum == N ? "true" : "false"));
		}
	}
	return 0;
}
