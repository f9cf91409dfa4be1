// Debug: run v6_lookup on the device against a freshly built table.
#include "../../cilium_amd/csrc/host.cpp"
#include "../../cilium_amd/csrc/kernels.hip"

/* variant: no early return, result carried in a variable */
__device__ uint32_t v6_lookup_b(const v6_lpm &t, uint4 a)
{
	if (!t.root)
		return 0;
	const uint32_t top = ((a.x & 0xFFu) << 8) | ((a.x >> 8) & 0xFFu);
	const uint2 r = t.root[top];
	uint32_t res = 0;
	if (r.x) {
		const uint4 m = reinterpret_cast<const uint4 *>(t.masks)[r.x];
		uint64_t hi = ((uint64_t)m.w << 32) | m.z, lo = ((uint64_t)m.y << 32) | m.x;
		while ((hi | lo) && !res) {
			uint32_t L[4];
#pragma unroll
			for (int j = 0; j < 4; j++) {
				uint32_t len = 0;
				if (hi) {
					int bit = 63 - __clzll(hi);
					hi &= ~(1ull << bit);
					len = 17u + 64u + (uint32_t)bit;
				} else if (lo) {
					int bit = 63 - __clzll(lo);
					lo &= ~(1ull << bit);
					len = 17u + (uint32_t)bit;
				}
				L[j] = len;
			}
#pragma unroll
			for (int j = 0; j < 4; j++) {
				if (L[j] && !res) {
					uint4 key = mask6(a, L[j]);
					uint32_t bi = hash16(key.x, key.y, key.z, key.w, L[j]) & t.set.bucket_mask;
					const uint4 *p = reinterpret_cast<const uint4 *>(t.set.slots) + (size_t)bi * 4u;
					uint4 bk[4] = {p[0], p[1], p[2], p[3]};
					res = set16_resolve(t.set, bk, bi, key, 1u | (L[j] << 8));
				}
			}
		}
	}
	return res ? res : r.y;
}

__global__ void kprobe_b(v6_lpm t, const uint4 *q, uint32_t *out, int n)
{
	int i = threadIdx.x;
	if (i < n)
		out[i] = v6_lookup_b(t, q[i]);
}

__global__ void kclz(uint32_t *out)
{
	uint64_t x = 0x80000000ull;
	out[0] = (uint32_t)__clzll(x);
	out[1] = (uint32_t)__builtin_clzll(x);
	uint64_t y = 0x800000000000ull;
	out[2] = (uint32_t)__clzll(y);
}

__global__ void kprobe(v6_lpm t, const uint4 *q, uint32_t *out, int n)
{
	int i = threadIdx.x;
	if (i < n) {
		uint4 a = q[i];
		const uint32_t top = ((a.x & 0xFFu) << 8) | ((a.x >> 8) & 0xFFu);
		out[3 * i] = v6_lookup(t, a);
		out[3 * i + 1] = t.root[top].x;
		out[3 * i + 2] = t.root[top].y;
	}
}

int main()
{
	cgpu_config cfg;
	cgpu_config_default(&cfg);
	cgpu_ctx *c;
	if (cgpu_ctx_create(&cfg, -1, &c))
		return 1;
	cgpu_cidr_key k{};
	k.prefixlen = 16; k.addr[0] = 0x20; k.addr[1] = 0x01; k.addr[2] = 5;
	cgpu_cidr_update(c, CGPU_CIDR_V6_DYN, &k, 0);
	k.prefixlen = 48; k.addr[2] = 1; k.addr[5] = 7;
	cgpu_cidr_update(c, CGPU_CIDR_V6_DYN, &k, 0);
	V6Build b;
	build_pf6(c, b);
	void *droot, *dmask, *dset, *dq, *dout;
	(void)hipMalloc(&droot, b.root.size() * 4);
	(void)hipMalloc(&dmask, b.masks.size() * 4);
	(void)hipMalloc(&dset, b.set.slots.size() * sizeof(set16_slot));
	(void)hipMemcpy(droot, b.root.data(), b.root.size() * 4, hipMemcpyHostToDevice);
	(void)hipMemcpy(dmask, b.masks.data(), b.masks.size() * 4, hipMemcpyHostToDevice);
	(void)hipMemcpy(dset, b.set.slots.data(), b.set.slots.size() * sizeof(set16_slot), hipMemcpyHostToDevice);
	v6_lpm t{(const uint2 *)droot, (const uint32_t *)dmask, nullptr,
		 addr_set16{(const set16_slot *)dset, b.set.mask, b.set.max_probe}, (uint32_t)(b.masks.size() / 4)};
	uint8_t q[2][16] = {{0x20, 0x01, 0, 140, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12},
			    {0x20, 0x01, 1, 0, 0, 7, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12}};
	(void)hipMalloc(&dq, 32);
	(void)hipMalloc(&dout, 64);
	(void)hipMemcpy(dq, q, 32, hipMemcpyHostToDevice);
	hipLaunchKernelGGL(kprobe, dim3(1), dim3(64), 0, 0, t, (const uint4 *)dq, (uint32_t *)dout, 2);
	uint32_t out[6];
	(void)hipMemcpy(out, dout, 24, hipMemcpyDeviceToHost);
	printf("host root[0x2001] = {%u, %08x}\n", b.root[2 * 0x2001], b.root[2 * 0x2001 + 1]);
	for (int i = 0; i < 2; i++)
		printf("dev q%d: lookup=%08x root={%u,%08x}\n", i, out[3 * i], out[3 * i + 1], out[3 * i + 2]);
	hipLaunchKernelGGL(kprobe_b, dim3(1), dim3(64), 0, 0, t, (const uint4 *)dq, (uint32_t *)dout, 2);
	(void)hipMemcpy(out, dout, 8, hipMemcpyDeviceToHost);
	printf("variant b: q0=%08x q1=%08x\n", out[0], out[1]);
	hipLaunchKernelGGL(kclz, dim3(1), dim3(1), 0, 0, (uint32_t *)dout);
	(void)hipMemcpy(out, dout, 12, hipMemcpyDeviceToHost);
	printf("clzll(0x80000000)=%u builtin=%u clzll(1<<47)=%u\n", out[0], out[1], out[2]);
	return 0;
}
