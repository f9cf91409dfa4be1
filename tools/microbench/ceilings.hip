/*
 * ceilings — the measured transaction ceilings of one MI355X that bound the
 * classification kernels (bench.py's roofline):
 *
 *   gather  every lane issues K independent loads of W bytes (4 / 8 / 16) at
 *           uniformly random, W-aligned offsets of a table of S bytes.  The
 *           rate is set by the level that serves the table (L1 / L2 /
 *           Infinity Cache / HBM) and the per-CU address and tag rate.  The
 *           best (K, occupancy) per (S, W) is the ceiling of that tier.
 *   atomic  no-return 64-bit atomicAdd of a packed {packets, bytes} word at
 *           a uniformly random slot of a table of S u64 slots: the shape of
 *           the classify kernels' cold counter adds (memory-side atomics).
 *   stream  coalesced 16-B-per-lane read of 4 GiB, and a 16-B-per-lane write:
 *           the column streams' ceiling.
 *
 *   hipcc --offload-arch=gfx950 -O3 ceilings.hip -o ceilings
 *   ./ceilings            -> one JSON line per measurement (tools/ceilings.py
 *                            folds them into profiles/ceilings.json)
 *
 * Every loop carries its result into a store the compiler cannot drop.
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

template <int W, int K, int BS>
__global__ __launch_bounds__(BS) void gather(const uint4 *tab, uint64_t mask, uint32_t iters, uint32_t *out)
{
	const uint32_t t = blockIdx.x * BS + threadIdx.x;
	uint32_t acc = 0, h = mix(t * 0x9E3779B9u + 1);
	for (uint32_t it = 0; it < iters; it++) {
		uint32_t v[K];
#pragma unroll
		for (int k = 0; k < K; k++) {
			h = mix(h + k);
			/* two draws for tables past 2^32 units are not needed: S <= 4 GiB */
			const uint64_t i = (uint64_t)h & mask; /* in W-byte units */
			if constexpr (W == 16) {
				const uint4 x = tab[i];
				v[k] = x.x ^ x.y ^ x.z ^ x.w;
			} else if constexpr (W == 8) {
				const uint2 x = reinterpret_cast<const uint2 *>(tab)[i];
				v[k] = x.x ^ x.y;
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

__global__ __launch_bounds__(256) void k_atomic(unsigned long long *tab, uint32_t mask, uint32_t per)
{
	const uint32_t t = blockIdx.x * 256 + threadIdx.x;
	uint32_t h = mix(t * 0x9E3779B9u + 7);
	for (uint32_t k = 0; k < per; k++) {
		h = mix(h + k);
		/* packed {packets << 37 | bytes} as the classify kernels add it */
		atomicAdd(&tab[h & mask], (1ull << 37) | (64 + (h >> 26)));
	}
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_read(const u32x4 *p, size_t n, uint32_t *out)
{
	uint32_t acc = 0;
	for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
		const u32x4 x = __builtin_nontemporal_load(p + i);
		acc ^= x.x + x.y + x.z + x.w;
	}
	if (acc == 0x12345678u)
		out[threadIdx.x] = acc;
}

__global__ __launch_bounds__(256) void k_write(u32x4 *p, size_t n)
{
	for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
		__builtin_nontemporal_store(u32x4{(uint32_t)i, 1u, 2u, 3u}, p + i);
}

static hipEvent_t ev_a, ev_b;

template <typename F> static float best_ms(F launch, int reps)
{
	float best = 1e30f;
	launch(); /* warm */
	for (int r = 0; r < reps; r++) {
		(void)hipEventRecord(ev_a);
		launch();
		(void)hipEventRecord(ev_b);
		(void)hipEventSynchronize(ev_b);
		float ms = 0;
		(void)hipEventElapsedTime(&ms, ev_a, ev_b);
		best = ms < best ? ms : best;
	}
	return best;
}

template <int W, int K, int BS>
static void run_gather(const uint4 *tab, size_t bytes, uint32_t *out, int cus, int per_cu)
{
	const uint64_t mask = bytes / W - 1;
	const uint32_t blocks = cus * per_cu, iters = 512 / K;
	const float ms = best_ms(
		[&] { hipLaunchKernelGGL((gather<W, K, BS>), dim3(blocks), dim3(BS), 0, 0, tab, mask, iters, out); }, 5);
	const double loads = (double)blocks * BS * iters * K;
	printf("{\"kind\": \"gather\", \"table_bytes\": %zu, \"width\": %d, \"k\": %d, \"threads_per_cu\": %d, "
	       "\"g_per_s\": %.2f, \"ms\": %.4f}\n",
	       bytes, W, K, BS * per_cu, loads / (ms * 1e-3) / 1e9, ms);
	fflush(stdout);
}

/* A of every 8 loads (16 B) per lane from table [0, small), 8 - A from [0, big) */
template <int A>
__global__ __launch_bounds__(256) void gather_mix(const uint4 *tab, uint64_t mask_s, uint64_t mask_b, uint32_t iters,
						  uint32_t *out)
{
	const uint32_t t = blockIdx.x * 256 + threadIdx.x;
	uint32_t acc = 0, h = mix(t * 0x9E3779B9u + 3);
	for (uint32_t it = 0; it < iters; it++) {
		uint32_t v[8];
#pragma unroll
		for (int k = 0; k < 8; k++) {
			h = mix(h + k);
			const uint4 x = tab[(uint64_t)h & (k < A ? mask_s : mask_b)];
			v[k] = x.x ^ x.y ^ x.z ^ x.w;
		}
#pragma unroll
		for (int k = 0; k < 8; k++)
			acc += v[k];
	}
	if (acc == 0x12345678u)
		out[t] = acc;
}

template <int A> static void run_mix(const uint4 *tab, size_t small, size_t big, uint32_t *out, int cus)
{
	const uint32_t blocks = cus * 8, iters = 64;
	const float ms = best_ms(
		[&] {
			hipLaunchKernelGGL(gather_mix<A>, dim3(blocks), dim3(256), 0, 0, tab, small / 16 - 1, big / 16 - 1,
					   iters, out);
		},
		5);
	const double loads = (double)blocks * 256 * iters * 8;
	printf("{\"kind\": \"mix\", \"small_bytes\": %zu, \"big_bytes\": %zu, \"small_frac\": %.4f, "
	       "\"g_per_s\": %.2f, \"ms\": %.4f}\n",
	       small, big, A / 8.0, loads / (ms * 1e-3) / 1e9, ms);
	fflush(stdout);
}

template <int W> static void sweep_width(const uint4 *tab, size_t s, uint32_t *out, int cus)
{
	run_gather<W, 8, 256>(tab, s, out, cus, 8);   /* 32 waves per CU */
	run_gather<W, 16, 256>(tab, s, out, cus, 8);
	run_gather<W, 8, 1024>(tab, s, out, cus, 1);  /* 16 waves per CU, one workgroup */
	run_gather<W, 4, 256>(tab, s, out, cus, 8);
}

int main()
{
	int dev = 0, cus = 0, clk = 0;
	CHECK(hipGetDevice(&dev));
	CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
	CHECK(hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev));
	hipDeviceProp_t prop;
	CHECK(hipGetDeviceProperties(&prop, dev));
	printf("{\"kind\": \"device\", \"name\": \"%s\", \"arch\": \"%s\", \"cus\": %d, \"clock_khz\": %d}\n", prop.name,
	       prop.gcnArchName, cus, clk);
	CHECK(hipEventCreate(&ev_a));
	CHECK(hipEventCreate(&ev_b));
	const size_t maxb = (size_t)4 << 30;
	uint4 *tab;
	uint32_t *out;
	CHECK(hipMalloc((void **)&tab, maxb));
	CHECK(hipMemset(tab, 1, maxb));
	CHECK(hipMalloc((void **)&out, (size_t)cus * 8 * 1024 * 4));

	/* streams first (they also flush the caches) */
	{
		const size_t n = maxb / 16;
		const float r = best_ms([&] { hipLaunchKernelGGL(k_read, dim3(cus * 16), dim3(256), 0, 0, (const u32x4 *)tab, n, out); }, 5);
		const float w = best_ms([&] { hipLaunchKernelGGL(k_write, dim3(cus * 16), dim3(256), 0, 0, (u32x4 *)tab, n); }, 5);
		printf("{\"kind\": \"stream\", \"bytes\": %zu, \"read_gbs\": %.1f, \"write_gbs\": %.1f}\n", maxb,
		       maxb / (r * 1e-3) / 1e9, maxb / (w * 1e-3) / 1e9);
		fflush(stdout);
		CHECK(hipMemset(tab, 1, maxb));
	}
	const size_t KB = 1024, MB = KB * KB;
	const size_t sizes[] = {16 * KB, 64 * KB, 256 * KB, 1 * MB,   2 * MB,   3 * MB,   4 * MB,  6 * MB,
				8 * MB,  12 * MB, 16 * MB,  24 * MB,  32 * MB,  48 * MB,  64 * MB, 96 * MB,
				128 * MB, 192 * MB, 256 * MB, 384 * MB, 512 * MB, 1024 * MB, maxb};
	for (size_t s : sizes) {
		sweep_width<16>(tab, s, out, cus);
		sweep_width<8>(tab, s, out, cus);
		sweep_width<4>(tab, s, out, cus);
	}
	/* mixes: A of every 8 loads per lane from a small table, the rest from a
	 * large one -- checks that the time of a mix is no less than the sum of
	 * its parts at their own tier's rate (bench.py composes the bound so) */
	for (size_t big : {64 * MB, maxb}) {
		run_mix<1>(tab, 2 * MB, big, out, cus);
		run_mix<2>(tab, 2 * MB, big, out, cus);
		run_mix<4>(tab, 2 * MB, big, out, cus);
		run_mix<6>(tab, 2 * MB, big, out, cus);
		run_mix<7>(tab, 2 * MB, big, out, cus);
	}
	/* packed u64 counter atomics */
	unsigned long long *ctr = reinterpret_cast<unsigned long long *>(tab);
	const uint32_t per = 16, threads = (24u << 20) / per;
	for (uint32_t S : {1u << 14, 1u << 17, 1u << 20, 1u << 24}) {
		CHECK(hipMemset(ctr, 0, (size_t)S * 8));
		const float ms = best_ms(
			[&] { hipLaunchKernelGGL(k_atomic, dim3(threads / 256), dim3(256), 0, 0, ctr, S - 1, per); }, 5);
		/* every add carries packets = 1 in bits 37..: the table's packet sum
		 * must equal the adds issued (6 launches: best_ms's warm-up + 5) */
		std::vector<unsigned long long> h(S);
		CHECK(hipMemcpy(h.data(), ctr, (size_t)S * 8, hipMemcpyDeviceToHost));
		unsigned long long pk = 0;
		for (auto x : h)
			pk += x >> 37;
		printf("{\"kind\": \"atomic\", \"slots\": %u, \"adds\": %u, \"g_per_s\": %.3f, \"ms\": %.4f, "
		       "\"sum_ok\": %s}\n",
		       S, threads * per, threads * per / (ms * 1e-3) / 1e9, ms,
		       pk == 6ull * threads * per ? "true" : "false");
		fflush(stdout);
	}
	CHECK(hipFree(tab));
	CHECK(hipFree(out));
	return 0;
}
