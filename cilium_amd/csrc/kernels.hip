/*
 * kernels.hip — gfx950 kernels of the classification path.
 *
 * One lane per tuple, grid-stride over SoA columns (coalesced 1/2/4-byte
 * loads of every column, both addresses loaded and selected per lane).
 * The path is memory-latency bound (dependent gathers into HBM/L2-resident
 * tables, no arithmetic to speak of), so there is no MFMA: the levers are
 * waves in flight, independent loads issued together, and 64-byte-aligned
 * table buckets (one cache-line sector per probe).  See DESIGN.md §4.
 */
#include "cgpu.h"
#include "launch.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>

#define DROP_POLICY (-133)           /* bpf/lib/common.h:240 */
#define DROP_CT_UNKNOWN_PROTO (-137) /* bpf/lib/common.h:244 */
#define DROP_NO_SERVICE (-158)      /* bpf/lib/common.h:265 */
#define XDP_DROP 1
#define XDP_PASS 2
/* CGPU_VERDICT_XDP_DROP: an ingress tuple the netdev's XDP prefilter dropped
 * (cgpu_classify_v4_cascade; stage 8) */
#define VERDICT_XDP_DROP (-4097)
#define TC_ACT_OK 0
#define TC_ACT_REDIRECT 7

namespace {

constexpr int BLOCK = 256;

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

/* Streamed column access: with NTL the loads / stores carry the nontemporal
 * hint (`nt`), so the 26 B/tuple stream does not evict table lines. */
typedef uint32_t v4u_t __attribute__((ext_vector_type(4)));
typedef uint32_t v2u_t __attribute__((ext_vector_type(2)));
/* one column element, nontemporal (streams past the table lines in L2) */
template <typename T> __device__ __forceinline__ uint32_t ntl(const T *p)
{
	return (uint32_t)__builtin_nontemporal_load(p);
}

template <bool NTL> __device__ __forceinline__ uint4 ld_x4(const void *p)
{
	if (NTL) {
		const v4u_t v = __builtin_nontemporal_load(static_cast<const v4u_t *>(p));
		return make_uint4(v.x, v.y, v.z, v.w);
	}
	return *static_cast<const uint4 *>(p);
}
template <bool NTL> __device__ __forceinline__ uint2 ld_x2(const void *p)
{
	if (NTL) {
		const v2u_t v = __builtin_nontemporal_load(static_cast<const v2u_t *>(p));
		return make_uint2(v.x, v.y);
	}
	return *static_cast<const uint2 *>(p);
}
template <bool NTL> __device__ __forceinline__ uint32_t ld_x1(const void *p)
{
	if (NTL)
		return __builtin_nontemporal_load(static_cast<const uint32_t *>(p));
	return *static_cast<const uint32_t *>(p);
}
template <bool NTL> __device__ __forceinline__ void st_x4(void *p, uint32_t a, uint32_t b, uint32_t c, uint32_t d)
{
	if (NTL) {
		v4u_t v = {a, b, c, d};
		__builtin_nontemporal_store(v, static_cast<v4u_t *>(p));
	} else {
		*static_cast<uint4 *>(p) = make_uint4(a, b, c, d);
	}
}
template <bool NTL> __device__ __forceinline__ void st_x1(void *p, uint32_t a)
{
	if (NTL)
		__builtin_nontemporal_store(a, static_cast<uint32_t *>(p));
	else
		*static_cast<uint32_t *>(p) = a;
}

/* Run-node search of the compressed LPM (tables.h lpm16c): q0..q3 hold the
 * node's words (only the first 1 / 2 / 4 loaded for kind 0 / 1 / 2). */
__device__ __forceinline__ uint32_t lpmc_search(uint4 q0, uint4 q1, uint4 q2, uint4 q3, uint32_t kind,
						uint32_t x)
{
	const uint32_t w[16] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w,
				q2.x, q2.y, q2.z, q2.w, q3.x, q3.y, q3.z, q3.w};
	const uint32_t nb = kind == 0 ? 1u : (kind == 1 ? 2u : 5u);
	uint32_t cnt = 0;
#pragma unroll
	for (uint32_t i = 0; i < 5; i++)
		if (i < nb)
			cnt += (x >= (w[i] & 0xFFFFu) ? 1u : 0u) + (x >= (w[i] >> 16) ? 1u : 0u);
	const uint32_t idx = nb + cnt;
	uint32_t v = w[1];
#pragma unroll
	for (uint32_t j = 2; j < 16; j++)
		v = j == idx ? w[j] : v;
	return v;
}

/* Longest-prefix lookup of a network-order IPv4 address in the compressed
 * ipcache table (tables.h lpm16c): the /16's inline run node (x16), or on
 * overflow its d16-style entry, a 256-entry array per address byte (at most
 * two levels) and one run node.  dict: the leaf dictionary (LDS copy or
 * t.dict).  Returns the DIR-encoded leaf (0 = no match). */
__device__ __forceinline__ uint32_t lpmc_lookup(const lpm16c &t, const uint32_t *dict, uint32_t addr_be)
{
	const uint32_t h = bswap32(addr_be);
	const uint4 q = reinterpret_cast<const uint4 *>(t.x16)[h >> 16];
	if (!(q.w & LPMC_OVERFLOW)) {
		const uint32_t x = h & 0xFFFFu;
		const uint32_t cnt = (x >= (q.x & 0xFFFFu) ? 1u : 0u) + (x >= (q.x >> 16) ? 1u : 0u) +
				     (x >= (q.y & 0xFFFFu) ? 1u : 0u) + (x >= (q.y >> 16) ? 1u : 0u);
		const uint64_t v = ((uint64_t)q.w << 32) | q.z;
		return dict[(uint32_t)(v >> (12u * cnt)) & 0xFFFu];
	}
	constexpr uint32_t ARR = (DIR_TAG_GROUP >> LPMC_KIND_SHIFT) | 3u;
	uint32_t e = q.x;
	bool lvl8 = false;
	if ((e >> LPMC_KIND_SHIFT) == ARR) {
		e = t.nodes[(size_t)(e & LPMC_OFF_MASK) * 4u + ((h >> 8) & 255u)];
		lvl8 = true;
		if ((e >> LPMC_KIND_SHIFT) == ARR)
			e = t.nodes[(size_t)(e & LPMC_OFF_MASK) * 4u + (h & 255u)];
	}
	if ((e & DIR_TAG_MASK) == DIR_TAG_GROUP) {
		const uint32_t kind = (e >> LPMC_KIND_SHIFT) & 3u;
		const uint4 *nd = reinterpret_cast<const uint4 *>(t.nodes) + (e & LPMC_OFF_MASK);
		const uint4 q0 = nd[0];
		const uint4 q1 = kind ? nd[1] : make_uint4(0, 0, 0, 0);
		const uint4 q2 = kind == 2 ? nd[2] : make_uint4(0, 0, 0, 0);
		const uint4 q3 = kind == 2 ? nd[3] : make_uint4(0, 0, 0, 0);
		e = lpmc_search(q0, q1, q2, q3, kind, lvl8 ? (h & 255u) : (h & 0xFFFFu));
	}
	return e;
}

/* Resolve a lookup in the single-slot (neighbourhood) policy table whose home
 * slot b is already in registers (tables.h POL_HOP): returns the counter slot
 * or -1 (map_lookup_elem NULL); *z receives ep | proxy_port << 16.  Further
 * (dependent) loads only for the hop bits beyond the home slot itself. */
__device__ __forceinline__ int pol_resolve1(const pol_table &t, uint4 sl, uint32_t b, uint32_t lo,
					    uint32_t hi, uint32_t ep, uint32_t *z)
{
	uint32_t hop = sl.w >> POL_HOP_SHIFT;
	if ((hop & 1u) && sl.x == lo && sl.y == hi && (sl.z & 0xFFFFu) == ep) {
		*z = sl.z;
		return (int)(sl.w & POL_CTR_MASK);
	}
	hop &= ~1u;
	const uint4 *tab = reinterpret_cast<const uint4 *>(t.slots);
	int r = -1;
	while (hop && r < 0) {
		const uint32_t j = __builtin_ctz(hop);
		hop &= hop - 1u;
		const uint4 x = tab[(b + j) & t.bucket_mask];
		if (x.x == lo && x.y == hi && (x.z & 0xFFFFu) == ep) {
			*z = x.z;
			r = (int)(x.w & POL_CTR_MASK);
		}
	}
	return r;
}

/* Policy hash probe: exact 8-byte policy_key + endpoint.  Returns the
 * counter slot, or -1 (map_lookup_elem NULL); *z receives ep|proxy<<16. */
__device__ __forceinline__ int pol_lookup(const pol_table &t, uint32_t lo, uint32_t hi, uint32_t ep,
					  uint32_t *z)
{
	const uint32_t b = pol_hash(lo, hi, ep) & t.bucket_mask;
	return pol_resolve1(t, reinterpret_cast<const uint4 *>(t.slots)[b], b, lo, hi, ep, z);
}

/* The group slot of {id, ep | dir << 16} whose home slot g (index b) is in
 * registers (tables.h pol_groups), or {0, 0, EMPTY, 0} when the endpoint's
 * map holds no key of that identity and direction. */
__device__ __forceinline__ uint4 pg_resolve(const pol_groups &t, uint4 g, uint32_t b, uint32_t id, uint32_t ed)
{
	uint32_t hop = g.y >> POL_HOP_SHIFT;
	if ((hop & 1u) && g.x == id && (g.y & 0x1FFFFu) == ed)
		return g;
	hop &= ~1u;
	uint4 r = make_uint4(0, 0, POL_CTR_EMPTY, 0);
	while (hop) {
		const uint32_t j = __builtin_ctz(hop);
		hop &= hop - 1u;
		const uint4 x = t.slots[(b + j) & t.mask];
		if (x.x == id && (x.y & 0x1FFFFu) == ed) {
			r = x;
			break;
		}
	}
	return r;
}

__device__ __forceinline__ bool set4_has(const addr_set4 &t, uint32_t a)
{
	uint32_t b = mix32(a, 0x5e7) & t.bucket_mask;
	for (uint32_t p = 0; p < t.max_probe; p++) {
		const uint4 *bk = reinterpret_cast<const uint4 *>(t.slots) + (size_t)b * 4u;
		uint4 s[4];
#pragma unroll
		for (int k = 0; k < 4; k++)
			s[k] = bk[k];
#pragma unroll
		for (int k = 0; k < 4; k++) {
			if (!s[k].y)
				return false;
			if (s[k].x == a)
				return true;
			if (!s[k].w)
				return false;
			if (s[k].z == a)
				return true;
		}
		b = (b + 1) & t.bucket_mask;
	}
	return false;
}

/* check_v4 of the netdev's XDP program for a pre-parsed IPv4 packet
 * (bpf_xdp.c:97-121): saddr covered by the dyn LPM or a fix /32
 * (CIDR4_FILTER; pf4c is their any-match union) -> XDP_DROP, else daddr must
 * be a local endpoint (check_v4_endpoint :88-95).  true = XDP_PASS. */
/* slots of a pf4x half-node below x: u16 lanes k0.. of the four words */
__device__ __forceinline__ uint32_t pf4x_below(uint4 q, uint32_t x, bool skip_header)
{
	return (!skip_header && (q.x & 0xFFFFu) < x ? 1u : 0u) + ((q.x >> 16) < x ? 1u : 0u) +
	       ((q.y & 0xFFFFu) < x ? 1u : 0u) + ((q.y >> 16) < x ? 1u : 0u) + ((q.z & 0xFFFFu) < x ? 1u : 0u) +
	       ((q.z >> 16) < x ? 1u : 0u) + ((q.w & 0xFFFFu) < x ? 1u : 0u) + ((q.w >> 16) < x ? 1u : 0u);
}

/* the deny set covers saddr (network order): pf4x (tables.h PF4X_*), with
 * pf4c for the /16s of more than 15 boundaries */
__device__ __forceinline__ bool pf4_covered(const cgpu_snapshot &s, uint32_t sa)
{
	const uint32_t h = bswap32(sa), x = h & 0xFFFFu;
	const uint4 q = s.pf4x[2u * (h >> 16)];
	if (q.x & PF4X_OVF)
		return lpmc_lookup(s.pf4c, s.pf4c.dict, sa) != 0;
	uint32_t c = pf4x_below(q, x, true) + (q.x & 1u);
	if (q.x & PF4X_TWO)
		c += pf4x_below(s.pf4x[2u * (h >> 16) + 1u], x, false);
	return c & 1u;
}

__device__ __forceinline__ bool xdp_pass4(const cgpu_snapshot &s, uint32_t sa, uint32_t da)
{
	if (s.pf4_enabled && s.pf4x && pf4_covered(s, sa))
		return false;
	return set4_has(s.ep4, da);
}

/* Resolve a 16-byte-key probe whose first bucket is loaded: returns the
 * slot's entry word (pad[0], nonzero for prefix sets) or 0 on a miss. */
__device__ __forceinline__ uint32_t set16_resolve(const addr_set16 &t, uint4 k0, uint4 m0, uint4 k1, uint4 m1,
						  uint32_t b, uint4 key, uint32_t want)
{
	for (uint32_t p = 0;;) {
		if (!(m0.x & 1u))
			return 0;
		if (m0.x == want && k0.x == key.x && k0.y == key.y && k0.z == key.z && k0.w == key.w)
			return m0.y;
		if (!(m1.x & 1u))
			return 0;
		if (m1.x == want && k1.x == key.x && k1.y == key.y && k1.z == key.z && k1.w == key.w)
			return m1.y;
		if (++p >= t.max_probe)
			return 0;
		b = (b + 1) & t.bucket_mask;
		const uint4 *bk = reinterpret_cast<const uint4 *>(t.slots) + (size_t)b * 4u;
		k0 = bk[0];
		m0 = bk[1];
		k1 = bk[2];
		m1 = bk[3];
	}
}

/* set16_resolve with only the bucket's first slot loaded (k0, m0): the
 * second slot is read when the first holds another key */
__device__ __forceinline__ uint32_t set16_resolve_first(const addr_set16 &t, uint4 k0, uint4 m0, uint32_t b,
							uint4 key, uint32_t want)
{
	if (!(m0.x & 1u))
		return 0;
	if (m0.x == want && k0.x == key.x && k0.y == key.y && k0.z == key.z && k0.w == key.w)
		return m0.y;
	const uint4 *bk = reinterpret_cast<const uint4 *>(t.slots) + (size_t)b * 4u;
	return set16_resolve(t, make_uint4(0, 0, 0, 0), make_uint4(1u | (want ^ 0xFF00u), 0, 0, 0), bk[2], bk[3], b,
			     key, want);
}

/* The IPv6 address words as stored (network-order bytes, little-endian u32
 * view) -> host-order words (x = address bits 0..31), the prefix-key domain
 * of tables.h pfx6_hash */
__device__ __forceinline__ uint4 v6_host_words(uint4 a)
{
	return make_uint4(bswap32(a.x), bswap32(a.y), bswap32(a.z), bswap32(a.w));
}

/* ---- IPv6 ipcache trie (tables.h v6_lpm) ---- */

/* (ah, al) <= (bh, bl) as 64-bit values */
__device__ __forceinline__ bool le64(uint32_t ah, uint32_t al, uint32_t bh, uint32_t bl)
{
	return ah < bh || (ah == bh && al <= bl);
}

/* the line of x (= address bits 32..63) in the /32 node {ex, ey}; outside:
 * x lies outside the node's window (its label is the line's outer slot) */
__device__ __forceinline__ uint32_t v6t_line(uint32_t ex, uint32_t ey, uint32_t x, bool &outside)
{
	const uint32_t w = (ey & 31u) + 9u, s = (ey >> 5) & 7u;
	const uint32_t rel = x - (ey & ~511u);
	outside = w < 32u ? (rel >> w) != 0u : false;
	const uint32_t sh = w - (s == V6T_LONG ? 0u : s);
	const uint32_t k = outside || sh >= 32u ? 0u : rel >> sh;
	return (ex & V6T_LINE_MASK) + (s == V6T_LONG ? 0u : k);
}

/* The label of x in a node line whose first four 16-B units are q0..q3
 * (tables.h v6_lpm): the region r = #{slot i < x, i < V6T_NB}; 128-B lines
 * read label r as one more word of the line, 64-B lines hold it in q2, q3. */
__device__ __forceinline__ uint32_t v6t_label(const uint32_t *pool, uint32_t line, bool out, uint4 q0, uint4 q1,
					      uint4 q2, uint4 q3, uint32_t x)
{
	static_assert(V6T_NB == 15u || V6T_NB == 7u, "node lines of 15 or 7 boundaries");
	if constexpr (V6T_NB == 15u) {
		const uint32_t c = (q0.x < x) + (q0.y < x) + (q0.z < x) + (q0.w < x) + (q1.x < x) + (q1.y < x) +
				   (q1.z < x) + (q1.w < x) + (q2.x < x) + (q2.y < x) + (q2.z < x) + (q2.w < x) +
				   (q3.x < x) + (q3.y < x) + (q3.z < x);
		return out ? q3.w : pool[V6T_LW * line + 16u + c];
	} else {
		const uint32_t c = (q0.x < x) + (q0.y < x) + (q0.z < x) + (q0.w < x) + (q1.x < x) + (q1.y < x) +
				   (q1.z < x);
		const uint32_t lo = c & 1u ? (c & 2u ? q2.w : q2.y) : (c & 2u ? q2.z : q2.x);
		const uint32_t hi = c & 1u ? (c & 2u ? q3.w : q3.y) : (c & 2u ? q3.z : q3.x);
		return out ? q1.w : (c & 4u ? hi : lo);
	}
}

/* a V6T_LONG node: n boundaries (b - 1) and n + 1 labels from line + 1 on,
 * binary-searched */
__device__ __forceinline__ uint32_t v6t_long(const uint32_t *pool, uint32_t line, uint32_t n, uint32_t x)
{
	const uint32_t *b = pool + V6T_LW * (line + 1u);
	uint32_t lo = 0, hi = n; /* count of b[i] < x */
	while (lo < hi) {
		const uint32_t m = (lo + hi) >> 1;
		if (b[m] < x)
			lo = m + 1u;
		else
			hi = m;
	}
	return b[n + lo];
}

/* a /64 list (tables.h v6_lpm h64): label of the low 64 bits (xh, xl) */
__device__ __forceinline__ uint32_t v6t_list64(const uint32_t *pool, uint32_t off, uint32_t xh, uint32_t xl)
{
	const uint32_t *p = pool + 4u * off;
	const uint32_t n = p[0];
	uint32_t c = 0;
	for (uint32_t i = 0; i < n; i++)
		c += le64(p[4u + 2u * i], p[5u + 2u * i], xh, xl) ? 1u : 0u;
	return p[4u + 2u * n + c];
}

/* the /64 record of w's /64 (or V6T_FALL): home slot s0 / s1 loaded */
__device__ __forceinline__ uint32_t v6t_rec(const v6_lpm &t, uint4 w, uint32_t home, uint4 s0, uint4 s1)
{
	uint32_t hop = s0.w >> POL_HOP_SHIFT;
	bool found = (hop & 1u) && s0.x == w.x && s0.y == w.y;
	hop &= ~1u;
	while (hop && !found) {
		const uint32_t k = (home + (uint32_t)__builtin_ctz(hop)) & t.m64;
		hop &= hop - 1u;
		const uint4 x = t.h64[2u * k];
		if (x.x == w.x && x.y == w.y) {
			s0 = x;
			s1 = t.h64[2u * k + 1u];
			found = true;
		}
	}
	if (!found)
		return V6T_FALL;
	if ((s0.z & DIR_TAG_MASK) == DIR_TAG_GROUP)
		return v6t_list64(t.pool, s0.z & DIR_PAYLOAD_MASK, w.z, w.w);
	return le64(s1.x, s1.y, w.z, w.w) && le64(w.z, w.w, s1.z, s1.w) ? s0.z : V6T_FALL;
}

/* IPv6 longest-prefix lookup (tables.h v6_lpm), one lane, every level from
 * global memory.  a: the address as stored.  Returns the DIR-encoded entry
 * (0 = no match). */
__device__ __forceinline__ uint32_t v6_lookup(const v6_lpm &t, uint4 a)
{
	if (!t.root)
		return 0;
	const uint4 w = v6_host_words(a);
	uint32_t e = t.root[w.x >> 16];
	if ((e & DIR_TAG_MASK) == DIR_TAG_GROUP)
		e = t.b24[(e & DIR_PAYLOAD_MASK) * 256u + ((w.x >> 8) & 0xFFu)];
	if ((e & DIR_TAG_MASK) != DIR_TAG_GROUP)
		return e;
	const uint2 n = t.b32[(e & DIR_PAYLOAD_MASK) * 256u + (w.x & 0xFFu)];
	if ((n.x & DIR_TAG_MASK) != DIR_TAG_GROUP)
		return n.x;
	bool out;
	const uint32_t line = v6t_line(n.x, n.y, w.y, out);
	const uint4 *q = reinterpret_cast<const uint4 *>(t.pool) + (V6T_LW / 4u) * line;
	const uint4 q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
	uint32_t lab;
	if (((n.y >> 5) & 7u) == V6T_LONG)
		lab = v6t_long(t.pool, line, q0.x, w.y);
	else
		lab = v6t_label(t.pool, line, out, q0, q1, q2, q3, w.y);
	if (n.x & V6T_DEEP) {
		const uint32_t home = mix32(w.x, w.y) & t.m64;
		const uint32_t r = v6t_rec(t, w, home, t.h64[2u * home], t.h64[2u * home + 1u]);
		if (r != V6T_FALL)
			lab = r;
	}
	return lab;
}

/* ---- service load balancer (bpf/lib/lb.h, bpf/bpf_lb.c) ---- */

/* frontend slot of {addr, dport} (tables.h lb_table); w == 0: no frontend */
__device__ __forceinline__ uint4 lb_fe_resolve(const lb_table &t, uint32_t home, uint4 s, uint32_t addr,
					      uint32_t dport)
{
	uint32_t hop = s.w >> POL_HOP_SHIFT;
	if ((hop & 1u) && s.x == addr && (s.y & 0xFFFFu) == dport)
		return s;
	hop &= ~1u;
	uint4 r = make_uint4(0, 0, 0, 0);
	while (hop && !r.w) {
		const uint32_t j = __builtin_ctz(hop);
		hop &= hop - 1u;
		const uint4 x = t.fe[(home + j) & t.fe_mask];
		if (x.x == addr && (x.y & 0xFFFFu) == dport)
			r = x;
	}
	return r;
}

__device__ __forceinline__ uint4 lb_frontend(const lb_table &t, uint32_t addr, uint32_t dport)
{
	const uint32_t home = lb_hash(addr, dport) & t.fe_mask;
	return lb_fe_resolve(t, home, t.fe[home], addr, dport);
}

/* map_lookup_elem(&cilium_lb4_services, {addr, dport, slave}) given the
 * frontend f of {addr, dport}; *v = {target, port | count << 16,
 * rev_nat | weight << 16, present}.  For slave 0 only the count is kept
 * (its only reader is lb4_lookup_service). */
__device__ __forceinline__ bool lb_entry(const lb_table &t, uint4 f, uint32_t slave, uint4 *v)
{
	if (!f.w)
		return false;
	if (slave == 0) {
		*v = make_uint4(0, f.y & 0xFFFF0000u, 0, 1);
		return true;
	}
	if (slave > (f.w & 0xFFFFu))
		return false;
	*v = t.be[f.z + slave - 1u];
	return v->w != 0;
}

/* map_lookup_elem(&cilium_lb4_services, {addr, dport, slave}) as a full row
 * (slave 0 included: the LB_FE_MASTER row), for lb4_lookup_slave of the
 * stateful service step, whose slave comes from a conntrack entry */
__device__ __forceinline__ bool lb_row(const lb_table &t, uint4 f, uint32_t slave, uint4 *v)
{
	if (!f.w)
		return false;
	const uint32_t ns = f.w & 0xFFFFu;
	if (slave == 0) {
		if (!(f.w & LB_FE_MASTER))
			return false;
		*v = t.be[f.z + ns];
		return true;
	}
	if (slave > ns)
		return false;
	*v = t.be[f.z + slave - 1u];
	return v->w != 0;
}

/* lb4_lookup_service (lb.h:604-635): the L4 key {addr, *kd, slave} if its
 * count is nonzero, else *kd = 0 and the L3 key; *f: the frontend searched
 * last.  *probes counts map lookups as the reference issues them. */
__device__ __forceinline__ bool lb_service(const cgpu_snapshot &s, uint32_t addr, uint32_t *kd,
					   uint32_t slave, uint4 *v, uint4 *f, uint32_t *probes)
{
	if ((s.lb_flags & CGPU_LB_L4) && *kd) {
		*f = lb_frontend(s.lb, addr, *kd);
		(*probes)++;
		if (lb_entry(s.lb, *f, slave, v) && (v->y >> 16))
			return true;
		*kd = 0;
	}
	if (s.lb_flags & CGPU_LB_L3) {
		*f = lb_frontend(s.lb, addr, *kd);
		(*probes)++;
		if (lb_entry(s.lb, *f, slave, v) && (v->y >> 16))
			return true;
	}
	return false;
}

/* map_lookup_elem(&cilium_lb6_services, {addr, dport, slave}) (tables.h
 * lb6_table): tg = target, val = {port | count << 16, rev_nat | weight << 16,
 * present, 0}; slave 0 carries only the master's count, or with FULL0 the
 * master's stored row (the stateful service step).  f = fold6(addr). */
template <bool FULL0 = false>
__device__ __forceinline__ bool lb6_get(const lb6_table &t, uint4 addr, uint32_t f, uint32_t dport,
					uint32_t slave, uint4 &tg, uint4 &val)
{
	const uint32_t home = lb6_hash(f, dport) & t.fe_mask;
	uint4 m = t.fe[2u * home + 1u];
	uint32_t hop = m.z >> POL_HOP_SHIFT;
	bool found = false;
	if (hop & 1u) {
		const uint4 a = t.fe[2u * home];
		found = a.x == addr.x && a.y == addr.y && a.z == addr.z && a.w == addr.w && (m.x & 0xFFFFu) == dport;
	}
	hop &= ~1u;
	while (hop && !found) {
		const uint32_t k = (home + (uint32_t)__builtin_ctz(hop)) & t.fe_mask;
		hop &= hop - 1u;
		const uint4 a = t.fe[2u * k], mk = t.fe[2u * k + 1u];
		if (a.x == addr.x && a.y == addr.y && a.z == addr.z && a.w == addr.w && (mk.x & 0xFFFFu) == dport) {
			m = mk;
			found = true;
		}
	}
	if (!found || !(m.z & LB_FE_USED))
		return false;
	if (slave == 0) {
		if (FULL0) { /* the stored master row (LB_FE_MASTER) */
			if (!(m.z & LB_FE_MASTER))
				return false;
			const uint32_t r = m.y + (m.z & 0xFFFFu);
			tg = t.be[2u * r];
			val = t.be[2u * r + 1u];
			return true;
		}
		tg = make_uint4(0, 0, 0, 0);
		val = make_uint4(m.x & 0xFFFF0000u, 0, 1, 0);
		return true;
	}
	if (slave > (m.z & 0xFFFFu))
		return false;
	const uint32_t r = m.y + slave - 1u;
	tg = t.be[2u * r];
	val = t.be[2u * r + 1u];
	return val.z != 0;
}

/* lb6_lookup_service (lb.h:351-380): the L4 key if its count is nonzero,
 * else *kd = 0 and the L3 key */
__device__ __forceinline__ bool lb6_service(const cgpu_snapshot &s, uint4 addr, uint32_t f, uint32_t *kd,
					    uint32_t slave, uint4 &tg, uint4 &val)
{
	if ((s.lb_flags & CGPU_LB_L4) && *kd) {
		if (lb6_get(s.lb6, addr, f, *kd, slave, tg, val) && (val.x >> 16))
			return true;
		*kd = 0;
	}
	if (s.lb_flags & CGPU_LB_L3)
		if (lb6_get(s.lb6, addr, f, *kd, slave, tg, val) && (val.x >> 16))
			return true;
	return false;
}

struct lb6_res {
	int32_t ret; /* 0 not load-balanced, CGPU_LB_XLATED, DROP_NO_SERVICE */
	uint4 tdaddr;
	uint32_t dport;
};

/*
 * The service step of ipv6_l3_from_lxc (bpf_lxc.c:117-139) with an empty
 * conntrack table: lb6_extract_key (lb.h:334-349), lb6_lookup_service,
 * lb6_local (lb.h:426-483).  Raw (network-order) address words in and out;
 * same decisions as oracle/cgpu_oracle.c lb6_one, which the golden vectors
 * of the reference pin.  No loopback case on IPv6.
 */
__device__ __forceinline__ lb6_res lb6_one(const cgpu_snapshot &s, uint4 da, uint32_t dp, uint32_t proto,
					   uint32_t hash)
{
	lb6_res r{0, da, dp};
	uint32_t kd = 0;
	if (s.lb_flags & CGPU_LB_L4) { /* extract_l4_port (lb.h:191-215) */
		if (proto == 6u || proto == 17u)
			kd = dp;
		else if (proto != 1u && proto != 58u)
			return r;
	}
	const uint32_t f = fold6(da.x, da.y, da.z, da.w);
	/* no frontend has this address (tables.h lb6_table.vip): every key misses */
	const uint32_t vb = lb6_vip_bit(f) & s.lb6.vip_mask;
	if (!((s.lb6.vip[vb >> 5] >> (vb & 31u)) & 1u))
		return r;
	uint4 tg, val;
	if (!lb6_service(s, da, f, &kd, 0, tg, val))
		return r;
	if (s.ct_proto_gate && proto != 58u && proto != 6u && proto != 17u) {
		/* lb6_local's CT_SERVICE ct_lookup6: DROP_CT_UNKNOWN_PROTO ->
		 * DROP_NO_SERVICE (conntrack.h:376-378, lb.h:436-456) */
		r.ret = DROP_NO_SERVICE;
		return r;
	}
	uint32_t slave = hash % (val.x >> 16) + 1u; /* lb6_select_slave, lb.h:124-156 */
	if (!lb6_get(s.lb6, da, f, kd, slave, tg, val)) { /* lb6_lookup_slave, lb.h:382-396 */
		/* lb.h:462-469: the key keeps the slave just tried */
		if (!lb6_service(s, da, f, &kd, slave, tg, val)) {
			r.ret = DROP_NO_SERVICE;
			return r;
		}
	}
	r.ret = CGPU_LB_XLATED;
	r.tdaddr = tg; /* tuple->daddr = svc->target (lb.h:475) */
	const uint32_t port = val.x & 0xFFFFu;
	if ((s.lb_flags & CGPU_LB_L4) && port && kd != port && (proto == 6u || proto == 17u))
		r.dport = port; /* lb6_xlate (lb.h:410-420); ct_lookup6 reloads it */
	return r;
}

struct lb_res {
	int32_t ret;
	uint32_t saddr, daddr, tdaddr, dport, rev_nat, slave, probes;
};

/*
 * One tuple through the service step.  MODE CGPU_LB_NETDEV: bpf_lb.c
 * handle_ipv4 (:118-170); CGPU_LB_LXC: lb4_local as handle_ipv4_from_lxc
 * calls it (bpf_lxc.c:444-460) with an empty conntrack table (CT_NEW).
 * Same decisions as oracle/cgpu_oracle.c lb4_one, which the golden vectors
 * of the reference pin.  tdaddr is tuple.daddr afterwards (LXC: the service
 * address is kept on loopback).
 */
template <int MODE, bool VIP = true>
__device__ __forceinline__ lb_res lb4_one(const cgpu_snapshot &s, uint32_t sa, uint32_t da, uint32_t dp,
					  uint32_t proto, uint32_t hash)
{
	lb_res r = {0, sa, da, da, dp, 0, 0, 0};
	uint32_t kd = 0;
	/* lb4_extract_key / extract_l4_port (lb.h:192-216): under LB_L4 only
	 * TCP/UDP carry a port, ICMP/ICMPv6 go on with 0, the rest are
	 * DROP_UNKNOWN_L4 = not load-balanced */
	if (s.lb_flags & CGPU_LB_L4) {
		if (proto == 6u || proto == 17u)
			kd = dp;
		else if (proto != 1u && proto != 58u)
			return r;
	}
	/* no frontend has this address (tables.h lb_table.vip): every key
	 * lb4_lookup_service would try misses */
	const uint32_t vb = lb_vip_bit(da) & s.lb.vip_mask;
	if (VIP && !((s.lb.vip[vb >> 5] >> (vb & 31u)) & 1u)) {
		r.probes = ((s.lb_flags & CGPU_LB_L4) && kd ? 1u : 0u) + ((s.lb_flags & CGPU_LB_L3) ? 1u : 0u);
		return r;
	}
	uint4 f, v;
	if (!lb_service(s, da, &kd, 0, &v, &f, &r.probes))
		return r;
	if (MODE == CGPU_LB_LXC && s.ct_proto_gate && proto != 1u && proto != 6u && proto != 17u) {
		/* lb4_local's CT_SERVICE ct_lookup4: DROP_CT_UNKNOWN_PROTO ->
		 * DROP_NO_SERVICE (conntrack.h:526-528, lb.h:711-731) */
		r.ret = DROP_NO_SERVICE;
		return r;
	}
	uint32_t slave = hash % (v.y >> 16) + 1u; /* lb4_select_slave, lb.h:158-190 */
	uint4 b;
	r.probes++;
	if (!lb_entry(s.lb, f, slave, &b)) { /* lb4_lookup_slave, lb.h:637-651 */
		if (MODE == CGPU_LB_NETDEV) {
			r.ret = DROP_NO_SERVICE;
			return r;
		}
		/* lb4_local fallback (lb.h:737-744): the key keeps the slave */
		if (!lb_service(s, da, &kd, slave, &b, &f, &r.probes)) {
			r.ret = DROP_NO_SERVICE;
			return r;
		}
		slave = hash % (b.y >> 16) + 1u;
	}
	r.slave = slave;
	r.rev_nat = b.z & 0xFFFFu;
	r.daddr = b.x;
	if (MODE == CGPU_LB_LXC) {
		if (sa == b.x) { /* loopback source NAT, lb.h:753-771 */
			r.saddr = s.ipv4_loopback;
			r.ret = CGPU_LB_XLATED_LOOPBACK;
		} else {
			r.tdaddr = b.x;
			r.ret = CGPU_LB_XLATED;
		}
	} else {
		r.tdaddr = b.x;
		r.ret = TC_ACT_REDIRECT;
	}
	const uint32_t port = b.y & 0xFFFFu;
	if ((s.lb_flags & CGPU_LB_L4) && port && kd != port && (proto == 6u || proto == 17u))
		r.dport = port; /* lb4_xlate, lb.h:685-694 */
	return r;
}

/*
 * lb4_one<CGPU_LB_LXC> for the Q tuples of a lane, with each step's gathers
 * issued together: the first frontend home slots, the L3 retry after a failed
 * L4 key (lb.h:604-635), then the chosen backend rows.  A tuple whose backend
 * row is missing (the lb4_local fallback, lb.h:737-744) or whose frontend
 * needs it leaves for lb4_one itself, so every decision is lb4_one's.  Only
 * what the classify cascade reads comes back: *drop (DROP_NO_SERVICE), the
 * translated tuple.daddr and dport.
 * XDP (cgpu_classify_v4_cascade): the ingress tuples (xin, disjoint from act)
 * take check_v4 in the same stages, so the prefilter adds no dependent round
 * trip: their /16 deny node rides with the egress tuples' vip-bitmap words,
 * their endpoint bucket (and a /16's second half-node) with the frontend
 * slots; xpass[u] = XDP_PASS (true where !xin[u]).  Same decisions as
 * xdp_pass4.
 */
template <int Q, bool XDP = false>
__device__ __forceinline__ void lb4_lxc_q(const cgpu_snapshot &s, const uint32_t *sa, uint32_t *da, uint32_t *dp,
					  const uint32_t *proto, const uint32_t *h, const bool *act, bool *drop,
					  const bool *xin = nullptr, bool *xpass = nullptr)
{
	constexpr uint32_t NONE = 0, L4K = 1, L3K = 2, RETRY = 3, FOUND = 4, SLOW = 5;
	const lb_table &t = s.lb;
	const bool l4 = s.lb_flags & CGPU_LB_L4, l3 = s.lb_flags & CGPU_LB_L3;
	const bool pf = XDP && s.pf4_enabled && s.pf4x;
	uint32_t st[Q], kd[Q], home[Q];
	uint4 f[Q];
#pragma unroll
	for (int u = 0; u < Q; u++) {
		st[u] = NONE;
		kd[u] = 0;
		home[u] = 0;
		drop[u] = false;
		if (!act[u])
			continue;
		if (l4) { /* lb4_extract_key / extract_l4_port (lb.h:192-216) */
			if (proto[u] == 6u || proto[u] == 17u)
				kd[u] = dp[u];
			else if (proto[u] != 1u && proto[u] != 58u)
				continue;
		}
		if (l4 && kd[u])
			st[u] = L4K;
		else if (l3)
			st[u] = L3K;
		else
			continue;
		home[u] = lb_vip_bit(da[u]) & t.vip_mask;
	}
	/* no frontend has this address (tables.h lb_table.vip): every key of
	 * lb4_lookup_service misses, the tuple is not load-balanced.  XDP: the
	 * ingress tuples' /16 deny nodes in the same stage (into f) */
	uint32_t vw[Q];
#pragma unroll
	for (int u = 0; u < Q; u++) {
		vw[u] = st[u] != NONE ? t.vip[home[u] >> 5] : 0u;
		if (XDP)
			f[u] = (xin[u] && pf) ? s.pf4x[2u * (bswap32(sa[u]) >> 16)] : make_uint4(0, 0, 0, 0);
	}
	/* XDP: the first half-node's count (bit 0: parity) and what the rest of
	 * the decision needs: XN_TWO the second half-node, XN_OVF the pf4c
	 * lookup, XN_EP the endpoint bucket (the deny set passed, or may) */
	constexpr uint32_t XN_TWO = 2u, XN_OVF = 4u, XN_EP = 8u;
	uint32_t xc[Q];
#pragma unroll
	for (int u = 0; u < Q; u++) {
		xc[u] = 0;
		if (!XDP || !xin[u])
			continue;
		if (!pf) {
			xc[u] = XN_EP;
			continue;
		}
		const uint4 q = f[u];
		if (q.x & PF4X_OVF) {
			xc[u] = XN_OVF | XN_EP;
			continue;
		}
		xc[u] = (pf4x_below(q, bswap32(sa[u]) & 0xFFFFu, true) + (q.x & 1u)) & 1u;
		if (q.x & PF4X_TWO)
			xc[u] |= XN_TWO | XN_EP;
		else if (!(xc[u] & 1u))
			xc[u] |= XN_EP;
	}
#pragma unroll
	for (int u = 0; u < Q; u++) {
		if (!((vw[u] >> (home[u] & 31u)) & 1u))
			st[u] = NONE;
		home[u] = lb_hash(da[u], kd[u]) & t.fe_mask;
	}
	/* the frontend home slots; XDP: the ingress tuples' endpoint buckets
	 * (first 16 B: slots 0 and 1) into f, their second half-nodes into x2 */
	uint4 x2[XDP ? Q : 1];
#pragma unroll
	for (int u = 0; u < Q; u++) {
		if (XDP && xin[u]) {
			f[u] = (xc[u] & XN_EP)
				       ? reinterpret_cast<const uint4 *>(s.ep4.slots)[(size_t)(mix32(da[u], 0x5e7) & s.ep4.bucket_mask) * 4u]
				       : make_uint4(0, 0, 0, 0);
			x2[XDP ? u : 0] = (xc[u] & XN_TWO) ? s.pf4x[2u * (bswap32(sa[u]) >> 16) + 1u] : make_uint4(0, 0, 0, 0);
			continue;
		}
		f[u] = st[u] != NONE ? t.fe[home[u]] : make_uint4(0, 0, 0, 0);
	}
	if constexpr (XDP) {
#pragma unroll
		for (int u = 0; u < Q; u++) {
			xpass[u] = true;
			if (!xin[u])
				continue;
			bool deny;
			if (xc[u] & XN_OVF)
				deny = lpmc_lookup(s.pf4c, s.pf4c.dict, sa[u]) != 0u;
			else if (xc[u] & XN_TWO)
				deny = ((xc[u] + pf4x_below(x2[u], bswap32(sa[u]) & 0xFFFFu, false)) & 1u) != 0u;
			else
				deny = (xc[u] & 1u) != 0u;
			if (deny) {
				xpass[u] = false;
				continue;
			}
			/* check_v4_endpoint: slots 0 / 1 of the home bucket decide
			 * unless both are used and neither holds da */
			const uint4 w = f[u];
			if (!w.y || w.x == da[u] || !w.w || w.z == da[u])
				xpass[u] = w.y && (w.x == da[u] || (w.w && w.z == da[u]));
			else
				xpass[u] = set4_has(s.ep4, da[u]);
		}
	}
#pragma unroll
	for (int u = 0; u < Q; u++) {
		if (st[u] == NONE)
			continue;
		f[u] = lb_fe_resolve(t, home[u], f[u], da[u], kd[u]);
		if (f[u].w && (f[u].y >> 16)) {
			st[u] = FOUND;
		} else if (st[u] == L4K && l3) {
			kd[u] = 0;
			st[u] = RETRY;
			home[u] = lb_hash(da[u], 0u) & t.fe_mask;
		} else {
			st[u] = NONE;
		}
	}
#pragma unroll
	for (int u = 0; u < Q; u++)
		if (st[u] == RETRY)
			f[u] = t.fe[home[u]];
#pragma unroll
	for (int u = 0; u < Q; u++) {
		if (st[u] != RETRY)
			continue;
		f[u] = lb_fe_resolve(t, home[u], f[u], da[u], 0u);
		st[u] = f[u].w && (f[u].y >> 16) ? FOUND : NONE;
	}
	uint32_t bi[Q];
#pragma unroll
	for (int u = 0; u < Q; u++) {
		bi[u] = 0;
		if (st[u] != FOUND)
			continue;
		if (s.ct_proto_gate && proto[u] != 1u && proto[u] != 6u && proto[u] != 17u) {
			drop[u] = true; /* lb4_local's CT_SERVICE lookup (conntrack.h:526-528) */
			st[u] = NONE;
			continue;
		}
		const uint32_t slave = h[u] % (f[u].y >> 16) + 1u; /* lb4_select_slave, lb.h:158-190 */
		if (slave > (f[u].w & 0xFFFFu))
			st[u] = SLOW;
		else
			bi[u] = f[u].z + slave - 1u;
	}
	uint4 b[Q];
#pragma unroll
	for (int u = 0; u < Q; u++)
		b[u] = st[u] == FOUND ? t.be[bi[u]] : make_uint4(0, 0, 0, 0);
#pragma unroll
	for (int u = 0; u < Q; u++) {
		if (st[u] == FOUND && !b[u].w)
			st[u] = SLOW;
		if (st[u] == FOUND) {
			if (sa[u] != b[u].x) /* else loopback source NAT: daddr stays (lb.h:753-771) */
				da[u] = b[u].x;
			const uint32_t port = b[u].y & 0xFFFFu;
			if (l4 && port && kd[u] != port && (proto[u] == 6u || proto[u] == 17u))
				dp[u] = port; /* lb4_xlate, lb.h:685-694 */
		} else if (st[u] == SLOW) {
			const lb_res r = lb4_one<CGPU_LB_LXC, false>(s, sa[u], da[u], dp[u], proto[u], h[u]);
			if (r.ret == DROP_NO_SERVICE) {
				drop[u] = true;
			} else {
				da[u] = r.tdaddr;
				dp[u] = r.dport;
			}
		}
	}
}

template <int MODE> __global__ __launch_bounds__(BLOCK) void k_lb4(cgpu_snapshot s, lb4_args a)
{
	const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
	for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < a.n; i += stride) {
		const uint32_t sa = a.saddr[i], da = a.daddr[i], dp = a.dport[i], pr = a.proto[i];
		const uint32_t h = a.hash ? a.hash[i] : flow_hash(sa, da, a.sport[i], dp, pr);
		const lb_res r = lb4_one<MODE>(s, sa, da, dp, pr, h);
		a.ret[i] = r.ret;
		if (a.saddr_out)
			a.saddr_out[i] = r.saddr;
		if (a.daddr_out)
			a.daddr_out[i] = r.daddr;
		if (a.dport_out)
			a.dport_out[i] = (uint16_t)r.dport;
		if (a.rev_nat_out)
			a.rev_nat_out[i] = (uint16_t)r.rev_nat;
		if (a.slave_out)
			a.slave_out[i] = (uint16_t)r.slave;
	}
}

/* ---- IPv6 any-match cover (tables.h cover6) ---- */

__device__ __forceinline__ bool c6_node64(const uint32_t *pool, uint32_t off, uint32_t xh, uint32_t xl)
{
	const uint4 *nd = reinterpret_cast<const uint4 *>(pool) + off;
	const uint32_t nb = nd[0].x;
	uint32_t cnt = 0;
	for (uint32_t k = 0; k < nb; k += 8) {
		uint4 q[4];
#pragma unroll
		for (uint32_t j = 0; j < 4; j++)
			q[j] = k + 2 * j < nb ? nd[1 + k / 2 + j] : make_uint4(0, 0, 0, 0);
#pragma unroll
		for (uint32_t j = 0; j < 4; j++) {
			const uint32_t i = k + 2 * j;
			cnt += (i < nb && le64(q[j].x, q[j].y, xh, xl) ? 1u : 0u) +
			       (i + 1 < nb && le64(q[j].z, q[j].w, xh, xl) ? 1u : 0u);
		}
	}
	return cnt & 1u;
}

__device__ __forceinline__ uint32_t entry_label(const uint32_t *vals, uint32_t e)
{
	uint32_t p = e & DIR_PAYLOAD_MASK;
	return (e & DIR_TAG_MASK) == DIR_TAG_INDIRECT ? vals[p] : p;
}

template <typename T> __device__ __forceinline__ T wave_sum(T v)
{
#pragma unroll
	for (int off = 32; off > 0; off >>= 1)
		v += __shfl_xor(v, off, 64);
	return v;
}

/*
 * Stateless classification (see cgpu.h cgpu_classify_v4 / _v6).
 *   egress : bpf_lxc.c:484-505 (v4) / :170-191 (v6)
 *            dstID = ipcache(daddr) | CLUSTER | WORLD
 *   ingress: bpf_netdev.c:374-404 (v4) / :203-211 (v6) src identity from ipcache(saddr)
 *   policy : bpf/lib/policy.h:46-110 (3 probes, issued in the reference's
 *            order: probe k+1 only after probe k missed), collapsed to
 *            DROP_POLICY by policy_can_access_ingress / policy_can_egress
 *   gate   : bpf/lib/conntrack.h DROP_CT_UNKNOWN_PROTO
 *   metrics: bpf/lib/drop.h:104 update_metrics(len, dir, -reason); forwarded
 *            at the verdict with reason 0
 * A speculative schedule (all three policy buckets loaded before the first
 * was resolved) was measured 1.4x slower: the extra random loads cost more
 * address-unit (TA) time than the shorter dependence chain saved.
 */
struct cls_args {
	const void *saddr, *daddr; /* u32 (v4) or uint4 (v6) per tuple */
	const uint16_t *dport;
	const uint8_t *proto, *flags;
	const uint32_t *len;
	const uint16_t *ep;
	int32_t *verdict;
	uint32_t *identity;
	uint8_t *stage;
	uint64_t *delta;
	uint64_t n;
	uint64_t *pk; /* packed cold-slot accumulator (k_classify_x4 only) */
	int lb;       /* v4: egress service step first (cgpu_classify_v4_lb) */
	const uint16_t *sport;
	const uint32_t *hash;
	uint32_t cc_n; /* k_classify_x4: cold-slot cache entries in LDS (cc_entries, or 0) */
	/* k_classify_x4 FR (frames): the tuple count is *n_dev - n_off, at most n */
	const uint32_t *n_dev;
	uint64_t n_off;
	/* k_classify_x4 IPCE: the ipcache entries k_ipc6_pre wrote, [n] */
	uint32_t *ipc_e;
	int xdp; /* v4 with lb: the XDP prefilter before every ingress tuple (cgpu_classify_v4_cascade) */
};

/* The identity resolution and the three-probe policy cascade for one tuple
 * that passed the protocol gate (shared by k_classify and k_frames).
 *   egress : dstID = ipcache(daddr) label | CLUSTER | WORLD (bpf_lxc.c:484-500
 *            v4, :170-187 v6)
 *   ingress: src = ipcache(saddr) label when the handed-in identity is
 *            reserved and the label is not CLUSTER (nor HOST on v4)
 *            (bpf_netdev.c:374-398 / :203-211); v4 secctx quirk (:278-290)
 *   policy : policy.h:46-110, negative collapsed to DROP_POLICY
 * v: verdict; id: label given to policy; st: 1 exact, 2 L3-only, 3 wildcard,
 * 0 miss; ctr: the hit entry's counter slot or -1. */
#ifndef CGPU_POLICY_Q_PROBES
#define CGPU_POLICY_Q_PROBES 0
#endif

struct decision {
	int32_t v;
	uint32_t id, st;
	int ctr;
};

template <int V6>
__device__ __forceinline__ decision decide(const cgpu_snapshot &s, bool egress, bool frag, uint32_t sa4,
					   uint32_t da4, uint4 sa6, uint4 da6, uint32_t dport, uint32_t proto,
					   uint32_t ep)
{
	decision d;
	const uint32_t eg = egress ? (1u << 24) : 0u;
	const uint32_t hi4 = dport | (proto << 16) | eg;
	uint32_t e, label;
	bool in_cluster;
	if (V6) {
		const uint4 ad = egress ? da6 : sa6;
		e = v6_lookup(s.ipc6, ad);
		label = entry_label(s.ipc6.vals, e);
		/* ipv6_match_prefix_64(daddr, ROUTER_IP), bpf/lib/ipv6.h:166-175 */
		in_cluster = ad.x == s.router_ip64[0] && ad.y == s.router_ip64[1];
	} else {
		const uint32_t ad = egress ? da4 : sa4;
		e = lpmc_lookup(s.ipc4c, s.ipc4c.dict, ad);
		label = entry_label(s.ipc4c.vals, e);
		in_cluster = (ad & s.ipv4_cluster_mask) == s.ipv4_cluster_range;
	}
	if (egress) {
		if (e && label)
			d.id = label;
		else if (in_cluster)
			d.id = s.cluster_id;
		else
			d.id = s.world_id;
	} else {
		/* the lookup above ran unconditionally; it only decides when the
		 * handed-in identity is reserved */
		uint32_t src = s.ingress_src_identity;
		if (src < s.health_id && e && label && label != s.cluster_id && (V6 || label != s.host_id))
			src = label;
		d.id = (!V6 && s.ingress_secctx_world) ? s.world_id : src;
	}
	uint32_t z = 0;
	int ctr = -1;
	d.st = 0;
	if (CGPU_POLICY_Q_PROBES) {
		if (!frag) {
			ctr = pol_lookup(s.pol, d.id, hi4, ep, &z);
			d.st = 1;
		}
		if (ctr < 0) {
			ctr = pol_lookup(s.pol, d.id, eg, ep, &z);
			d.st = 2;
		}
	} else {
		/* as policy_q: the {identity, endpoint, direction} group slot gives
		 * probe 2 and the bloom that gates probe 1 */
		const uint32_t ed = ep | (egress ? 1u << 16 : 0u);
		const uint32_t bg = pg_hash(d.id, ed) & s.pg.mask;
		const uint4 grp = pg_resolve(s.pg, s.pg.slots[bg], bg, d.id, ed);
		const uint32_t bl = pg_bloom(dport, proto);
		if (!frag && (grp.w & bl) == bl) {
			ctr = pol_lookup(s.pol, d.id, hi4, ep, &z);
			d.st = 1;
		}
		if (ctr < 0) {
			d.st = 2;
			if ((grp.z & POL_CTR_MASK) != POL_CTR_EMPTY) {
				ctr = (int)(grp.z & POL_CTR_MASK);
				z = 0;
			}
		}
	}
	if (ctr < 0 && !frag) {
		ctr = pol_lookup(s.pol, 0u, hi4, ep, &z);
		d.st = 3;
	}
	if (ctr >= 0) {
		d.v = d.st == 2 ? 0 : (int32_t)(z >> 16);
	} else {
		d.st = 0;
		d.v = DROP_POLICY;
	}
	d.ctr = ctr;
	return d;
}

/* The policy cascade of decide<> (probe 1 {id, dport, proto, dir} unless a
 * fragment, probe 2 {id, any port, dir}, probe 3 {any identity, dport,
 * proto, dir} unless a fragment) for Q tuples whose identity d[u].id is
 * set, each stage's Q gathers issued together, through the group table as
 * k_classify_x4 (tables.h pol_groups): one gather of the {identity,
 * endpoint, direction} group slot gives probe 2 (its L3 key) and a bloom
 * over the group's (dport, proto) that admits probe 1 only where an exact
 * key can exist; probe 3 gathers directly.  Same results as the three
 * probes in order (GROUP false: the probes themselves, for kernels at their
 * register limit - the group slots' registers spill k_ct_finish, 2.18 ->
 * 2.36 ms, profiles/r4_i/; CGPU_POLICY_Q_PROBES: every caller, A/B). */
template <int Q, bool GROUP = true>
__device__ __forceinline__ void policy_q(const cgpu_snapshot &s, const bool (&act)[Q], const bool (&eg)[Q],
					 const bool (&frag)[Q], const uint32_t (&dport)[Q], const uint32_t (&proto)[Q],
					 const uint32_t (&ep)[Q], decision (&d)[Q])
{
	uint32_t hi4[Q], egw[Q], z[Q], b[Q];
	int ctr[Q];
	uint4 sl[Q];
	const uint4 *ptab = reinterpret_cast<const uint4 *>(s.pol.slots);
	const uint32_t pm = s.pol.bucket_mask;
#pragma unroll
	for (int u = 0; u < Q; u++) {
		egw[u] = eg[u] ? (1u << 24) : 0u;
		hi4[u] = dport[u] | (proto[u] << 16) | egw[u];
		z[u] = 0;
		ctr[u] = -1;
		d[u].st = 0;
	}
	if (CGPU_POLICY_Q_PROBES || !GROUP) {
		/* probe 1: {id, dport, proto, dir} (not for fragments) */
#pragma unroll
		for (int u = 0; u < Q; u++) {
			b[u] = pol_hash(d[u].id, hi4[u], ep[u]) & pm;
			sl[u] = (act[u] && !frag[u]) ? ptab[b[u]] : make_uint4(0, 0, 0, 0);
		}
#pragma unroll
		for (int u = 0; u < Q; u++)
			if (act[u] && !frag[u]) {
				ctr[u] = pol_resolve1(s.pol, sl[u], b[u], d[u].id, hi4[u], ep[u], &z[u]);
				d[u].st = 1;
			}
		/* probe 2: {id, any port, dir} */
#pragma unroll
		for (int u = 0; u < Q; u++) {
			b[u] = pol_hash(d[u].id, egw[u], ep[u]) & pm;
			sl[u] = (act[u] && ctr[u] < 0) ? ptab[b[u]] : make_uint4(0, 0, 0, 0);
		}
#pragma unroll
		for (int u = 0; u < Q; u++)
			if (act[u] && ctr[u] < 0) {
				ctr[u] = pol_resolve1(s.pol, sl[u], b[u], d[u].id, egw[u], ep[u], &z[u]);
				d[u].st = 2;
			}
	} else {
		/* the group slot: probe 2 and the bloom that gates probe 1 */
		uint4 grp[Q];
		bool need[Q];
#pragma unroll
		for (int u = 0; u < Q; u++) {
			grp[u] = make_uint4(0, 0, POL_CTR_EMPTY, 0);
			b[u] = pg_hash(d[u].id, ep[u] | (eg[u] ? 1u << 16 : 0u)) & s.pg.mask;
			if (act[u])
				grp[u] = s.pg.slots[b[u]];
		}
#pragma unroll
		for (int u = 0; u < Q; u++) {
			need[u] = false;
			if (!act[u])
				continue;
			grp[u] = pg_resolve(s.pg, grp[u], b[u], d[u].id, ep[u] | (eg[u] ? 1u << 16 : 0u));
			const uint32_t bl = pg_bloom(dport[u], proto[u]);
			need[u] = !frag[u] && (grp[u].w & bl) == bl;
		}
		/* probe 1: {id, dport, proto, dir} (policy.h:61-72), if the bloom admits it */
#pragma unroll
		for (int u = 0; u < Q; u++) {
			b[u] = pol_hash(d[u].id, hi4[u], ep[u]) & pm;
			sl[u] = need[u] ? ptab[b[u]] : make_uint4(0, 0, 0, 0);
		}
#pragma unroll
		for (int u = 0; u < Q; u++) {
			if (need[u]) {
				ctr[u] = pol_resolve1(s.pol, sl[u], b[u], d[u].id, hi4[u], ep[u], &z[u]);
				d[u].st = 1;
			}
			/* probe 2: {id, any port, dir} (policy.h:74-83), the group's L3 key */
			if (act[u] && ctr[u] < 0) {
				d[u].st = 2;
				if ((grp[u].z & POL_CTR_MASK) != POL_CTR_EMPTY) {
					ctr[u] = (int)(grp[u].z & POL_CTR_MASK);
					z[u] = 0;
				}
			}
		}
	}
	/* probe 3: {any identity, dport, proto, dir} (not for fragments) */
#pragma unroll
	for (int u = 0; u < Q; u++) {
		b[u] = pol_hash(0u, hi4[u], ep[u]) & pm;
		sl[u] = (act[u] && ctr[u] < 0 && !frag[u]) ? ptab[b[u]] : make_uint4(0, 0, 0, 0);
	}
#pragma unroll
	for (int u = 0; u < Q; u++) {
		if (act[u] && ctr[u] < 0 && !frag[u]) {
			ctr[u] = pol_resolve1(s.pol, sl[u], b[u], 0u, hi4[u], ep[u], &z[u]);
			d[u].st = 3;
		}
		if (ctr[u] >= 0) {
			d[u].v = d[u].st == 2 ? 0 : (int32_t)(z[u] >> 16);
		} else {
			d[u].st = 0;
			d[u].v = DROP_POLICY;
		}
		d[u].ctr = ctr[u];
	}
}

/* decide<0> for Q tuples of one lane, stage by stage: each stage (the /16
 * run node, the leaf, policy probe 1, 2, 3) issues the Q tuples' gathers
 * together, so a wave has Q x 64 independent loads in flight where decide
 * has 64.  Same results as decide<0> tuple by tuple (the stateful path's
 * prep and finish passes; the dictionary is read from global memory). */
template <int Q>
__device__ __forceinline__ void ident4_q(const cgpu_snapshot &s, const uint32_t *dict, const bool (&act)[Q],
					 const bool (&eg)[Q], const uint32_t (&sa)[Q], const uint32_t (&da)[Q],
					 decision (&d)[Q])
{
	const lpm16c &t = s.ipc4c;
	uint32_t h[Q], e[Q];
	uint4 q[Q];
#pragma unroll
	for (int u = 0; u < Q; u++) {
		h[u] = bswap32(eg[u] ? da[u] : sa[u]);
		q[u] = act[u] ? reinterpret_cast<const uint4 *>(t.x16)[h[u] >> 16] : make_uint4(0, 0, 0, 0);
	}
#pragma unroll
	for (int u = 0; u < Q; u++) {
		if (!(q[u].w & LPMC_OVERFLOW)) {
			const uint32_t x = h[u] & 0xFFFFu;
			const uint32_t cnt = (x >= (q[u].x & 0xFFFFu) ? 1u : 0u) + (x >= (q[u].x >> 16) ? 1u : 0u) +
					     (x >= (q[u].y & 0xFFFFu) ? 1u : 0u) + (x >= (q[u].y >> 16) ? 1u : 0u);
			const uint64_t v = ((uint64_t)q[u].w << 32) | q[u].z;
			e[u] = act[u] ? dict[(uint32_t)(v >> (12u * cnt)) & 0xFFFu] : 0u;
		} else {
			e[u] = lpmc_lookup(t, t.dict, eg[u] ? da[u] : sa[u]);
		}
	}
#pragma unroll
	for (int u = 0; u < Q; u++) {
		const uint32_t label = entry_label(t.vals, e[u]);
		const uint32_t ad = eg[u] ? da[u] : sa[u];
		const bool in_cluster = (ad & s.ipv4_cluster_mask) == s.ipv4_cluster_range;
		if (eg[u]) {
			d[u].id = (e[u] && label) ? label : (in_cluster ? s.cluster_id : s.world_id);
		} else {
			uint32_t src = s.ingress_src_identity;
			if (src < s.health_id && e[u] && label && label != s.cluster_id && label != s.host_id)
				src = label;
			d[u].id = s.ingress_secctx_world ? s.world_id : src;
		}
	}
}

template <int Q>
__device__ __forceinline__ void decide4_q(const cgpu_snapshot &s, const bool (&act)[Q], const bool (&eg)[Q],
					  const bool (&frag)[Q], const uint32_t (&sa)[Q], const uint32_t (&da)[Q],
					  const uint32_t (&dport)[Q], const uint32_t (&proto)[Q],
					  const uint32_t (&ep)[Q], decision (&d)[Q])
{
	ident4_q<Q>(s, s.ipc4c.dict, act, eg, sa, da, d);
	policy_q<Q>(s, act, eg, frag, dport, proto, ep, d);
}

/* Packed per-workgroup counter: packets in bits 41..63, bytes in 0..40.
 * Exact while a workgroup adds < 2^23 hits of < 2^18 bytes to one slot
 * (the launcher bounds tuples per workgroup; longer packets take the
 * global path). */
#define PK_SHIFT 41
#define PK_BYTES_MASK ((1ull << PK_SHIFT) - 1ull)
#define PK_MAX_LEN (1u << 18)

/*
 * CTR = 0: two global u64 atomics per policy hit (packets, bytes).
 * CTR = 1: hits on hot slots [0, s.hot_slots) (L3-only / wildcard keys) go
 *          to one packed LDS atomic; the workgroup flushes its LDS counters
 *          to the delta buffer once at the end; cold slots as CTR = 0.
 */
template <int V6, int CTR, int NT>
__global__ __launch_bounds__(NT) void k_classify(cgpu_snapshot s, cls_args a)
{
	extern __shared__ __attribute__((aligned(16))) uint64_t lctr[];
	/* metrics {reason 0 / 133 / 137 / 158} x {ingress, egress} */
	uint64_t mcnt[8] = {0, 0, 0, 0, 0, 0, 0, 0}, mbyt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
	const uint64_t stride = (uint64_t)gridDim.x * NT;
	uint64_t *pctr = a.delta;
	if (CTR == 1) {
		for (uint32_t k = threadIdx.x; k < s.hot_slots; k += NT)
			lctr[k] = 0;
		__syncthreads();
	}

	for (uint64_t i = (uint64_t)blockIdx.x * NT + threadIdx.x; i < a.n; i += stride) {
		const uint32_t fl = a.flags[i];
		const uint32_t proto = a.proto[i];
		const uint32_t len = a.len[i];
		uint32_t dport = a.dport[i];
		const uint32_t ep = a.ep[i];
		const bool egress = fl & 1u;
		int32_t v;
		uint32_t id;
		uint32_t st = 0;
		/* egress service step (bpf_lxc.c:444-469): ipcache resolves
		 * tuple.daddr afterwards and policy sees the rewritten dport */
		bool lbdrop = false;
		uint32_t eda = 0;
		uint4 lda6{}; /* v6: the (translated) raw daddr */
		if (V6 && egress) {
			lda6 = static_cast<const uint4 *>(a.daddr)[i];
			if (a.lb) {
				const uint4 sa6 = static_cast<const uint4 *>(a.saddr)[i];
				const uint32_t h = a.hash ? a.hash[i]
							  : flow_hash(fold6(sa6.x, sa6.y, sa6.z, sa6.w),
								      fold6(lda6.x, lda6.y, lda6.z, lda6.w), a.sport[i],
								      dport, proto);
				const lb6_res r = lb6_one(s, lda6, dport, proto, h);
				if (r.ret == DROP_NO_SERVICE) {
					lbdrop = true;
				} else {
					lda6 = r.tdaddr;
					dport = r.dport;
				}
			}
		}
		/* config 5 whole: the netdev's XDP prefilter before an ingress
		 * tuple reaches from_netdev (bpf_xdp.c:180-184) */
		bool xdpdrop = false;
		if (!V6) {
			eda = static_cast<const uint32_t *>(a.daddr)[i];
			if (a.xdp && !egress)
				xdpdrop = !xdp_pass4(s, static_cast<const uint32_t *>(a.saddr)[i], eda);
			if (a.lb && egress) {
				const uint32_t sa = static_cast<const uint32_t *>(a.saddr)[i];
				const uint32_t h = a.hash ? a.hash[i] : flow_hash(sa, eda, a.sport[i], dport, proto);
				const lb_res r = lb4_one<CGPU_LB_LXC>(s, sa, eda, dport, proto, h);
				if (r.ret == DROP_NO_SERVICE) {
					lbdrop = true;
				} else {
					eda = r.tdaddr;
					dport = r.dport;
				}
			}
		}
		/* ct_lookup{4,6} protocol gate: ICMP (v4: 1, v6: 58), TCP, UDP */
		const bool gated = s.ct_proto_gate && proto != (V6 ? 58u : 1u) && proto != 6u &&
				   proto != 17u;

		if (xdpdrop) {
			/* XDP_DROP: nothing counted, nothing notified */
			v = VERDICT_XDP_DROP;
			id = 0;
			st = 8;
		} else if (lbdrop) {
			v = DROP_NO_SERVICE;
			id = 0;
			st = 6;
		} else if (gated) {
			v = DROP_CT_UNKNOWN_PROTO;
			id = 0;
			st = 4;
		} else {
			/* IPv6 passes is_fragment = false (bpf_lxc.c:787-789) */
			const bool frag = !V6 && !egress && ((fl >> 1) & 1u);
			uint4 sa6{}, da6{};
			uint32_t sa4 = 0;
			if (V6) {
				if (egress)
					da6 = lda6;
				else
					sa6 = static_cast<const uint4 *>(a.saddr)[i];
			} else if (!egress) {
				sa4 = static_cast<const uint32_t *>(a.saddr)[i];
			}
			const decision d = decide<V6>(s, egress, frag, sa4, eda, sa6, da6, dport, proto, ep);
			v = d.v;
			id = d.id;
			st = d.st;
			if (d.ctr >= 0) {
				const uint32_t c = (uint32_t)d.ctr;
				if (CTR == 1 && c < s.hot_slots && len < PK_MAX_LEN) {
					atomicAdd((unsigned long long *)&lctr[c],
						  (1ull << PK_SHIFT) | (unsigned long long)len);
				} else {
					atomicAdd((unsigned long long *)&pctr[2u * c], 1ull);
					atomicAdd((unsigned long long *)&pctr[2u * c + 1u],
						  (unsigned long long)len);
				}
			}
		}
		a.verdict[i] = v;
		a.identity[i] = id;
		if (a.stage)
			a.stage[i] = (uint8_t)st;
		/* a proxy redirect (v > 0) traces TRACE_TO_PROXY: no metrics */
		const uint32_t r = (v > 0 || xdpdrop) ? 4u : v == 0 ? 0u : (v == DROP_POLICY ? 1u : (v == DROP_NO_SERVICE ? 3u : 2u));
		const uint32_t idx = r * 2u + (egress ? 1u : 0u);
#pragma unroll
		for (int k = 0; k < 8; k++) {
			mcnt[k] += (idx == (uint32_t)k) ? 1u : 0u;
			mbyt[k] += (idx == (uint32_t)k) ? len : 0u;
		}
	}

	/* metrics: wave-reduce, one atomic per nonzero {reason, dir} per wave */
	uint64_t *met = a.delta + 2ull * s.n_ctr_slots;
	const uint32_t reasons[4] = {0u, 133u, 137u, 158u};
#pragma unroll
	for (int k = 0; k < 8; k++) {
		uint64_t c = wave_sum(mcnt[k]);
		uint64_t b = wave_sum(mbyt[k]);
		if ((threadIdx.x & 63) == 0 && c) {
			uint32_t key = (reasons[k >> 1] * 4u + ((k & 1) ? 2u : 1u)) * 2u;
			atomicAdd((unsigned long long *)&met[key], (unsigned long long)c);
			atomicAdd((unsigned long long *)&met[key + 1], (unsigned long long)b);
		}
	}
	if (CTR == 1) {
		__syncthreads();
		for (uint32_t k = threadIdx.x; k < s.hot_slots; k += NT) {
			const uint64_t v = lctr[k];
			if (v) {
				atomicAdd((unsigned long long *)&pctr[2u * k], v >> PK_SHIFT);
				atomicAdd((unsigned long long *)&pctr[2u * k + 1u], v & PK_BYTES_MASK);
			}
		}
	}
}


/* Packed per-slot accumulator of k_classify_x4 (pk): one u64 per counter
 * slot, packets in bits 37..63, bytes in 0..36.  Exact while one launch adds
 * at most PKC_CHUNK = 2^26 hits of < 2^11 bytes to a slot (2^26 * 2047 <
 * 2^37): the launcher caps a launch at PKC_CHUNK tuples and unpacks pk into
 * the delta buffer after it.  A packet of >= PKC_MAX_LEN bytes takes the
 * two-word path into delta directly.  Each stream has its own pk buffer
 * (host.cpp), so concurrent calls on one context never share the bound. */
#define PKC_SHIFT 37
#ifndef CC_PROBE
/* linear probes of the LDS cold-slot cache: 1 (direct-mapped) measured
 * fastest, config 2 1.771 / 1.734 / 1.752 / 1.763 ms at 4 / 1 / 2 / 3
 * (profiles/r4_x/): a second probe rarely finds room the first did not
 * and costs an LDS round trip on every miss */
#define CC_PROBE 1
#endif
#define PKC_BYTES_MASK ((1ull << PKC_SHIFT) - 1ull)
#define PKC_MAX_LEN (1u << 11)
#define PKC_CHUNK (1ull << 26)

/* timing-only tool builds (tools/diag_ab.py; wrong results): confine a
 * gather to the first 1024 entries of its table, i.e. make it an L2 hit */
#ifdef CGPU_DIAG_P1_SMALL
#define DIAG_P1(b) ((b) & 1023u)
#else
#define DIAG_P1(b) (b)
#endif
#ifdef CGPU_DIAG_P2_SMALL
#define DIAG_P2(b) ((b) & 1023u)
#else
#define DIAG_P2(b) (b)
#endif
#ifdef CGPU_DIAG_LPM_SMALL
#define DIAG_LPM(b) ((b) & 1023u)
#else
#define DIAG_LPM(b) (b)
#endif

/* IPv6 ipcache lookups of Q tuples per lane for the x4 schedule
 * (k_classify_x4<.., V6>; tables.h v6_lpm), level by level with the Q
 * tuples' loads of a level in flight together:
 *   root: the GROUP bitmap and ranks in LDS (lds; a leaf root reads its
 *         entry from global memory at the next level);
 *   b24:  the u16 blocks in LDS when staged (lds24), else global;
 *   b32:  one 8-byte gather;
 *   node: the line's four boundary units (64 B) and, for a /32 with /65+
 *         prefixes, the /64's h64 home slot, together; then the label word.
 * w: host-order address words; act false: e = 0. */
#ifndef V6T_LDS_B24
#define V6T_LDS_B24 96u /* b24 blocks staged in LDS at most (48 KiB) */
#endif

/* b24 blocks the x4 kernel stages in LDS (0: b24 read from global memory) */
__host__ __device__ __forceinline__ uint32_t v6t_lds_b24(const v6_lpm &t)
{
	return t.root && t.b24_16 && t.n_b24 <= V6T_LDS_B24 ? t.n_b24 : 0u;
}

/* LDS words of the x4 kernel's staged trie levels */
__host__ __device__ __forceinline__ uint32_t v6t_lds_words(const v6_lpm &t)
{
	return t.root ? V6T_RBITS_WORDS + v6t_lds_b24(t) * 128u : 0u;
}

/* bloom words the lookup pre-pass stages behind them (0: none) */
__host__ __device__ __forceinline__ uint32_t v6t_lds_bloom(const v6_lpm &t)
{
	return t.root && t.bl64 && t.bl64_mask < V6T_BLOOM_MAX_WORDS ? t.bl64_mask + 1u : 0u;
}

/* 1: the x4 lookups read a node's whole 128-B line (boundaries, outer AND
 * the 16 region labels) in one go and select the label in registers, so a
 * lookup has no dependent label load; 0: the 64-B
 * boundary half, then the label word */
#ifndef CGPU_V6T_FULL_LINE
#define CGPU_V6T_FULL_LINE 0
#endif

__device__ __forceinline__ uint32_t sel16(const uint4 &a, const uint4 &b, const uint4 &c, const uint4 &d, uint32_t i)
{
	const uint4 v = (i & 8u) ? ((i & 4u) ? d : c) : ((i & 4u) ? b : a);
	const uint32_t lo = (i & 1u) ? v.y : v.x, hi = (i & 1u) ? v.w : v.z;
	return (i & 2u) ? hi : lo;
}

/* bl: the /64 bloom staged in LDS (v6_lpm.bl64), or NULL: probe h64 for
 * every tuple under a deep /32 */
template <int Q>
__device__ __forceinline__ void v6t_lookup_q(const v6_lpm &t, const uint32_t *lds, bool lds24,
					     const uint4 (&w)[Q], const bool (&act)[Q], uint32_t (&e)[Q],
					     const uint32_t *bl = nullptr)
{
	const uint16_t *rank = reinterpret_cast<const uint16_t *>(lds + 2048u);
	const uint16_t *b16 = reinterpret_cast<const uint16_t *>(lds + V6T_RBITS_WORDS);
	const uint32_t *src[Q];
	bool leaf[Q];
	uint32_t b32i[Q];
	/* root and (staged) b24 in LDS: each tuple ends with the global word it
	 * needs (a leaf of root / b24, or an unstaged b24 entry) or a b32 block */
#pragma unroll
	for (int u = 0; u < Q; u++) {
		src[u] = nullptr;
		leaf[u] = false;
		b32i[u] = 0xFFFFFFFFu;
		e[u] = 0;
		if (!act[u] || !t.root)
			continue;
		const uint32_t r = w[u].x >> 16, wd = lds[r >> 5], bit = 1u << (r & 31u);
		if (!(wd & bit)) {
			src[u] = t.root + r;
			leaf[u] = true;
			continue;
		}
		const uint32_t blk = rank[r >> 5] + __popc(wd & (bit - 1u));
		const uint32_t x24 = blk * 256u + ((w[u].x >> 8) & 0xFFu);
		if (lds24) {
			const uint32_t c = b16[x24];
			if (c & 0x8000u) {
				b32i[u] = c & 0x7FFFu;
			} else {
				src[u] = t.b24 + x24;
				leaf[u] = true;
			}
		} else {
			src[u] = t.b24 + x24;
		}
	}
	uint32_t g[Q];
#pragma unroll
	for (int u = 0; u < Q; u++)
		g[u] = src[u] ? *src[u] : 0u;
#pragma unroll
	for (int u = 0; u < Q; u++) {
		if (!src[u])
			continue;
		if (!leaf[u] && (g[u] & DIR_TAG_MASK) == DIR_TAG_GROUP)
			b32i[u] = g[u] & DIR_PAYLOAD_MASK; /* an unstaged b24 GROUP */
		else
			e[u] = g[u];
	}
	/* b32 */
	uint2 n[Q];
#pragma unroll
	for (int u = 0; u < Q; u++)
		n[u] = b32i[u] != 0xFFFFFFFFu ? t.b32[b32i[u] * 256u + (w[u].x & 0xFFu)] : make_uint2(0, 0);
	bool node[Q], deep[Q], out[Q];
	uint32_t line[Q], home[Q];
	uint4 q0[Q], q1[Q], q2[Q], q3[Q], h0[Q], h1[Q];
	constexpr bool FULL = CGPU_V6T_FULL_LINE && V6T_NB == 15u;
	uint4 q4[FULL ? Q : 1], q5[FULL ? Q : 1], q6[FULL ? Q : 1], q7[FULL ? Q : 1];
#pragma unroll
	for (int u = 0; u < Q; u++) {
		node[u] = b32i[u] != 0xFFFFFFFFu && (n[u].x & DIR_TAG_MASK) == DIR_TAG_GROUP;
		if (b32i[u] != 0xFFFFFFFFu && !node[u])
			e[u] = n[u].x;
#ifdef CGPU_DIAG_V6_NO_H64 /* timing-only tool build: the /64 records never read (wrong results) */
		deep[u] = false;
#else
		deep[u] = node[u] && (n[u].x & V6T_DEEP);
		if (bl && deep[u]) {
			const uint32_t h = mix32(w[u].x, w[u].y), m = v6_bloom_bits(h);
			deep[u] = (bl[v6_bloom_word(h, t.bl64_mask)] & m) == m;
		}
#endif
		out[u] = false;
		line[u] = node[u] ? v6t_line(n[u].x, n[u].y, w[u].y, out[u]) : 0u;
		home[u] = mix32(w[u].x, w[u].y) & t.m64;
	}
	/* the node line and the /64 home slot together */
#pragma unroll
	for (int u = 0; u < Q; u++) {
		q0[u] = q1[u] = q2[u] = q3[u] = h0[u] = h1[u] = make_uint4(0, 0, 0, 0);
		if constexpr (FULL)
			q4[u] = q5[u] = q6[u] = q7[u] = make_uint4(0, 0, 0, 0);
		if (node[u]) {
			const uint4 *q = reinterpret_cast<const uint4 *>(t.pool) + (V6T_LW / 4u) * line[u];
			q0[u] = q[0];
			q1[u] = q[1];
			q2[u] = q[2];
			q3[u] = q[3];
			if constexpr (FULL) {
				q4[u] = q[4];
				q5[u] = q[5];
				q6[u] = q[6];
				q7[u] = q[7];
			}
		}
		if (deep[u]) {
			h0[u] = t.h64[2u * home[u]];
			h1[u] = t.h64[2u * home[u] + 1u];
		}
	}
	uint32_t lab[Q];
#pragma unroll
	for (int u = 0; u < Q; u++) {
		lab[u] = 0;
		if (!node[u])
			continue;
		if (((n[u].y >> 5) & 7u) == V6T_LONG) {
			lab[u] = v6t_long(t.pool, line[u], q0[u].x, w[u].y);
		} else if constexpr (FULL) {
			const uint32_t x = w[u].y;
			const uint32_t c = (q0[u].x < x) + (q0[u].y < x) + (q0[u].z < x) + (q0[u].w < x) +
					   (q1[u].x < x) + (q1[u].y < x) + (q1[u].z < x) + (q1[u].w < x) +
					   (q2[u].x < x) + (q2[u].y < x) + (q2[u].z < x) + (q2[u].w < x) +
					   (q3[u].x < x) + (q3[u].y < x) + (q3[u].z < x);
			lab[u] = out[u] ? q3[u].w : sel16(q4[u], q5[u], q6[u], q7[u], c);
		} else {
			lab[u] = v6t_label(t.pool, line[u], out[u], q0[u], q1[u], q2[u], q3[u], w[u].y);
		}
	}
#pragma unroll
	for (int u = 0; u < Q; u++) {
		if (!node[u])
			continue;
		uint32_t r = V6T_FALL;
		if (deep[u])
			r = v6t_rec(t, w[u], home[u], h0[u], h1[u]);
		e[u] = r != V6T_FALL ? r : lab[u];
	}
}


/*
 * IPv4 classification, four consecutive tuples per lane per step.
 * Same semantics as k_classify<0, 1, NT> (the reference cascade of
 * policy.h:46-110 behind the identity resolution of bpf_lxc.c:484-500 /
 * bpf_netdev.c:374-404).  Differences are all in the memory schedule:
 *   - every column is read with one 4/8/16-byte load per lane (the wave reads
 *     256 B .. 1 KiB contiguous per instruction instead of 64 B .. 256 B);
 *   - the four tuples of a lane advance stage by stage (x16, node, probe 1,
 *     probe 2, probe 3), so each stage has four independent gathers in flight;
 *   - a hit on a cold counter slot is ONE packed u64 atomic (pk), not two.
 * Lane t of the grid (T lanes) handles tuples 4 * (j * T + t) + {0..3} at
 * step j.  The launcher guarantees 16-byte aligned 4-byte columns, 8-byte
 * aligned 2-byte columns and 4-byte aligned 1-byte columns; the one partial
 * group at the end of the batch is read element by element.
 */
/* frames on the x4 schedule (launch_classify_frames): flag bits of the
 * parsed columns.  FRF_DEC: the parse ended the frame (daddr column = its
 * status); FRF_V6: an IPv6 frame, classified by the compacted v6 pass */
#define FRAME_NOT_CLASSIFIED 1   /* CGPU_FRAME_NOT_CLASSIFIED */
#define DROP_SNAPLEN (-4096)     /* CGPU_DROP_SNAPLEN */
#define FRF_DEC 0x80u
#define FRF_V6 0x40u
/* The first 64 bytes of a frame slot as 16 little-endian words: Ethernet,
 * the IPv4 header without options / the IPv6 header, and the L4 type and
 * ports right behind them.  Offsets are compile-time constants after
 * inlining, so the words stay in VGPRs. */
struct fwin {
	uint32_t w[16];
	__device__ __forceinline__ uint32_t b(int o) const { return (w[o >> 2] >> ((o & 3) * 8)) & 0xffu; }
	/* raw (memory-order) u16 at an even offset */
	__device__ __forceinline__ uint32_t h(int o) const { return (w[o >> 2] >> ((o & 2) * 8)) & 0xffffu; }
	/* raw u32 at an even offset */
	__device__ __forceinline__ uint32_t d(int o) const
	{
		return (o & 2) ? ((w[o >> 2] >> 16) | (w[(o >> 2) + 1] << 16)) : w[o >> 2];
	}
};

struct ftuple {
	int32_t status; /* 0 reached policy, FRAME_NOT_CLASSIFIED, or a drop */
	uint32_t fam;   /* 4 / 6 / 0 */
	uint4 sa, da;   /* IPv4 in .x */
	uint32_t dport, proto;
	bool frag;
};

/* endpoints whose rows the frame parse stages in LDS (8 KiB): the egress
 * SMAC / DMAC / SIP checks then read LDS, not a global load that would wait
 * behind the frame loads */
#define FR_LXC_LDS 256u
/* the x4 schedule's cold-slot atomics of a full quad go out behind the next
 * quad's column loads: config 2 1.612 -> 1.592 ms, v6 2.688 -> 2.661
 * (deferring the output stores as well: 2.08 ms, spills; profiles/r6_n/) */
#ifndef CGPU_X4_DEFER_COLD
#define CGPU_X4_DEFER_COLD 1
#endif
#ifndef CGPU_FF_H
#define CGPU_FF_H 2 /* fused frames: slots loaded together (1, 2, 4) */
#endif
#define FF_H CGPU_FF_H
#ifndef CGPU_FF_STAGE
#define CGPU_FF_STAGE 1 /* fused frames: coalesced tile loads handed out through LDS */
#endif
/* fused frames' LDS rows per wave: 64 slots x 80 B */
#define FF_STG_U4 320u
/* fused frames: staging buffers shared by a workgroup's 16 waves (0: one
 * per wave) */
#ifndef CGPU_FF_POOL
#define CGPU_FF_POOL 4
#endif

__device__ __forceinline__ ftuple parse_frame_w(const cgpu_snapshot &s, const fwin &W, const uint8_t *f,
						uint32_t len, uint32_t cap, bool egress, uint32_t ep,
						const uint4 *lxc);

/* a wave-uniform 64-bit value into scalar registers */
__device__ __forceinline__ uint64_t wave_uniform64(uint64_t x)
{
	const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
	const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
	return ((uint64_t)hi << 32) | lo;
}

/* FR: 0 tuple columns; 1 the columns k_frames_cols parsed (a parse-ended
 * frame's status in its daddr column); 2 fused frames: the kernel parses
 * the 64-byte frame slots itself (a.saddr = the slots; lane l of a wave
 * handles frames i0 + 64 u + l, so each load instruction covers 64
 * consecutive slots and each output store 64 consecutive frames), IPv6
 * frames compacted to fx for the v6 pass */
template <int NT, bool NTL = false, int Q = 4, int MINW = 1, bool LB = false, bool V6 = false,
	  int FR = 0, bool IPCE = false, bool XDP = false>
__global__ __launch_bounds__(NT, MINW) void k_classify_x4(cgpu_snapshot s, cls_args a0, uint64_t *pk, frames_x4 fx)
{
	constexpr bool FF = FR == 2;
	static_assert(!XDP || (LB && !V6), "the XDP prefilter: the IPv4 cascade");
	static_assert(!FF || (Q == 4 && !V6 && !LB), "fused frames: the v4 x4 schedule");
	cls_args a = a0;
	if (FR && a0.n_dev) {
		const uint64_t c = *a0.n_dev;
		a.n = c > a0.n_off ? min(c - a0.n_off, a0.n) : 0;
	}
	/* per-tuple flag word */
	/* F_XDP (with F_LBDROP, which ends the tuple's lookups): the XDP
	 * prefilter dropped an ingress tuple (cgpu_classify_v4_cascade) */
	constexpr uint32_t F_OK = 1u, F_EG = 2u, F_GATED = 4u, F_FRAG = 8u, F_LVL8 = 16u, F_LBDROP = 32u,
			   F_DEC = 64u, F_XDP = 128u;
	extern __shared__ __attribute__((aligned(16))) uint64_t lctr[];
	/* drop metrics (send_drop_notify -> update_metrics, drop.h:94-118):
	 * [reason 133 / 137 / 158][ingress, egress] x {count, bytes} in LDS
	 * (index 0..3 unused); forwards (verdict 0: TRACE_TO_LXC / _STACK,
	 * trace.h) per lane in registers, wave-reduced at the end; a proxy
	 * redirect (verdict > 0, TRACE_TO_PROXY) counts nothing */
	__shared__ unsigned long long lmet[16];
	uint32_t fwd_n[2] = {0u, 0u};
	uint64_t fwd_b[2] = {0ull, 0ull};
	const uint64_t T = (uint64_t)gridDim.x * NT;
	const uint64_t t0 = (uint64_t)blockIdx.x * NT + threadIdx.x;
	uint64_t *pctr = a.delta;
	const uint4 *ptab = reinterpret_cast<const uint4 *>(s.pol.slots);
	const uint32_t pmask = s.pol.bucket_mask;
	/* after the hot counters: v4 the LPM leaf dictionary; v6 the ipcache
	 * trie's root bitmap and ranks, then its b24 blocks as u16 (if staged) */
	uint32_t *ldict = reinterpret_cast<uint32_t *>(lctr + s.hot_slots);
	const uint32_t n24 = V6 && !IPCE ? v6t_lds_b24(s.ipc6) : 0u;
	/* cold-slot cache (x4_lds_layout): cc_n u64 packed counts, then cc_n u32
	 * tags (slot + 1, 0 = free) */
	const uint32_t lds_words = V6 ? (IPCE ? 0u : v6t_lds_words(s.ipc6)) : s.ipc4c.n_dict;
	uint64_t *ccv = lctr + s.hot_slots + ((lds_words + 1u) >> 1);
	uint32_t *cck = reinterpret_cast<uint32_t *>(ccv + a.cc_n);
	/* fused frames: the endpoints' rows (16-byte aligned) and each lane's
	 * four parse statuses, after the cold-slot cache (launch_x4's LDS) */
	uint4 *lxl = reinterpret_cast<uint4 *>((reinterpret_cast<uintptr_t>(cck + a.cc_n) + 15u) & ~(uintptr_t)15u);
	int16_t *fst = reinterpret_cast<int16_t *>(lxl + (FF ? 2u * FR_LXC_LDS : 0u));
	/* fused frames: this wave's staging rows, after the statuses */
	uint4 *stg0 = reinterpret_cast<uint4 *>(fst + (FF ? NT * Q : 0));
#if CGPU_FF_POOL
	/* CGPU_FF_POOL staging buffers shared by the workgroup's waves (a wave
	 * holds one only between its tile's LDS write and read), then their
	 * busy flags: the LDS the per-wave rows took goes to hot counter slots */
	uint32_t *pool_busy = reinterpret_cast<uint32_t *>(stg0 + CGPU_FF_POOL * FF_STG_U4);
	if (FF && threadIdx.x < CGPU_FF_POOL)
		pool_busy[threadIdx.x] = 0u;
	uint4 *stg = stg0;
#else
	uint4 *stg = stg0 + (threadIdx.x >> 6) * FF_STG_U4;
#endif
	if constexpr (FF) {
		for (uint32_t k = threadIdx.x; k < 2u * s.n_lxc; k += NT)
			lxl[k] = s.lxc[k];
	}
	for (uint32_t k = threadIdx.x; k < s.hot_slots; k += NT)
		lctr[k] = 0;
	for (uint32_t k = threadIdx.x; k < a.cc_n; k += NT) {
		ccv[k] = 0;
		cck[k] = 0;
	}
	if (threadIdx.x < 16)
		lmet[threadIdx.x] = 0;
	if (V6) {
		if (s.ipc6.root && !IPCE) {
			for (uint32_t k = threadIdx.x; k < V6T_RBITS_WORDS; k += NT)
				ldict[k] = s.ipc6.rbits[k];
			const uint32_t *b16 = reinterpret_cast<const uint32_t *>(s.ipc6.b24_16);
			for (uint32_t k = threadIdx.x; k < n24 * 128u; k += NT)
				ldict[V6T_RBITS_WORDS + k] = b16[k];
		}
	} else {
		for (uint32_t k = threadIdx.x; k < s.ipc4c.n_dict; k += NT)
			ldict[k] = s.ipc4c.dict[k];
	}
	__syncthreads();

	const uint32_t lane = threadIdx.x & 63u;
	/* CGPU_X4_DEFER_COLD: a quad's cold-slot atomics (into pk) are issued
	 * after the next quad's column loads, so the wait for those loads does
	 * not wait for them too (vmcnt retires in issue order) */
	constexpr bool DEFER = CGPU_X4_DEFER_COLD && !FF && Q == 4;
	uint32_t dcs[DEFER ? Q : 1], dln[DEFER ? Q : 1];
#pragma unroll
	for (int u = 0; u < (DEFER ? Q : 1); u++)
		dcs[u] = 0xFFFFFFFFu, dln[u] = 0u;
	auto defer_flush = [&]() {
		if constexpr (DEFER) {
#pragma unroll
			for (int u = 0; u < Q; u++)
				if (dcs[u] != 0xFFFFFFFFu) {
					atomicAdd((unsigned long long *)&pk[dcs[u]], (1ull << PKC_SHIFT) | (unsigned long long)dln[u]);
					dcs[u] = 0xFFFFFFFFu;
				}
		}
	};
	for (uint64_t g = t0;; g += T) {
		/* FF: i0 = the wave's first frame, frame u of the lane at iu(u) */
		const uint64_t i0 = FF ? wave_uniform64((g - lane) * Q) : g * Q;
		/* FF: wave-uniform, every lane of the wave stages its part of the
		 * tile; a lane past the batch carries no tuple (F_OK clear) */
		const bool live = i0 < a.n;
		if (!live) {
			defer_flush();
			break;
		}
		const bool full = FF ? false : i0 + Q <= a.n;
		if (!full || Q != 4)
			defer_flush(); /* (a full quad's go out behind its column loads) */
		/* FF: a scalar base (i0 + 64 u) plus the lane */
		auto iu = [&](int u) -> uint64_t { return FF ? (i0 + 64u * (uint32_t)u) + lane : i0 + (uint64_t)u; };
		/* decode: hi4 = the policy key's upper word {dport, proto, egress}
		 * (policy.h:61-64), fw = flag word, ad = the looked-up address */
		/* QA: the vector-load branches below are written for Q = 4; arrays
		 * they fill are sized for them whatever Q (dead when Q != 4) */
		constexpr int QA = Q < 4 ? 4 : Q;
		uint32_t fw[Q], ad[Q], hi4[Q], ep[QA], len[QA];
		uint4 ad6[Q];
		{
			uint32_t fl[QA], proto[QA], dport[QA], sa[QA], da[QA];
			if constexpr (FF) {
				/* the frames' 64-byte slots and len / flags / ep, all in
				 * flight together, then the parse (parse_frame_w) of each */
				const uint8_t *fd = static_cast<const uint8_t *>(a.saddr);
				uint4 raw[FF_H][4];
				uint32_t flv[Q];
#pragma unroll
				for (int u = 0; u < Q; u++) {
					const bool ok = iu(u) < a.n;
					const uint64_t i = ok ? iu(u) : i0;
					len[u] = a.len[i];
					flv[u] = a.flags[i];
					ep[u] = a.ep[i];
				}
#pragma unroll
				for (int u = 0; u < Q; u++) {
					const bool ok = iu(u) < a.n;
					const uint64_t i = ok ? iu(u) : i0;
					/* FF_H frames' slots in flight at a time (registers) */
					if (u % FF_H == 0) {
#pragma unroll
						for (int h = 0; h < FF_H; h++) {
#if CGPU_FF_STAGE
							/* the wave's tile of 64 slots as four coalesced
							 * 1-KiB loads: load k, lane l = slot 16 k + l / 4,
							 * quarter l % 4 */
							const uint64_t t = i0 + 64u * (uint32_t)(u + h);
#pragma unroll
							for (int k = 0; k < 4; k++)
								raw[h][k] = t + 16u * k + (lane >> 2) < a.n
										    ? ld_x4<NTL>(fd + t * 64u + 1024u * k + 16u * lane)
										    : make_uint4(0, 0, 0, 0);
#else
							const bool okh = iu(u + h) < a.n;
							const uint64_t ih = okh ? iu(u + h) : i0;
#pragma unroll
							for (int k = 0; k < 4; k++)
								raw[h][k] = okh ? ld_x4<NTL>(fd + ih * 64u + 16u * k) : make_uint4(0, 0, 0, 0);
#endif
						}
					}
					fwin W;
#if CGPU_FF_STAGE
#if CGPU_FF_POOL
					/* take a free staging buffer (lane 0 for the wave) */
					uint32_t pb = 0;
					if (lane == 0) {
						const uint32_t w0 = (threadIdx.x >> 6) % CGPU_FF_POOL;
						for (bool got = false; !got;) {
#pragma unroll 1
							for (uint32_t t = 0; t < CGPU_FF_POOL && !got; t++) {
								const uint32_t b = (w0 + t) % CGPU_FF_POOL;
								uint32_t z0 = 0u;
								if (__hip_atomic_compare_exchange_strong(&pool_busy[b], &z0, 1u, __ATOMIC_ACQUIRE,
													 __ATOMIC_RELAXED,
													 __HIP_MEMORY_SCOPE_WORKGROUP)) {
									pb = b;
									got = true;
								}
							}
							if (!got)
								__builtin_amdgcn_s_sleep(1);
						}
					}
					pb = (uint32_t)__shfl((int)pb, 0, 64);
					stg = stg0 + pb * FF_STG_U4;
#endif
					/* each lane's slot through the wave's LDS rows (64 slots of
					 * 80 B: conflict-free 16-B reads) */
#pragma unroll
					for (int k = 0; k < 4; k++)
						stg[(16u * k + (lane >> 2)) * 5u + (lane & 3u)] = raw[u % FF_H][k];
					__builtin_amdgcn_wave_barrier();
#pragma unroll
					for (int q = 0; q < 4; q++) {
						const uint4 v = stg[lane * 5u + q];
						W.w[4 * q] = v.x;
						W.w[4 * q + 1] = v.y;
						W.w[4 * q + 2] = v.z;
						W.w[4 * q + 3] = v.w;
					}
					__builtin_amdgcn_wave_barrier();
#if CGPU_FF_POOL
					/* the reads above are done before the buffer is free */
					if (lane == 0)
						__hip_atomic_store(&pool_busy[pb], 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
#endif
#else
#pragma unroll
					for (int k = 0; k < 4; k++) {
						W.w[4 * k] = raw[u % FF_H][k].x;
						W.w[4 * k + 1] = raw[u % FF_H][k].y;
						W.w[4 * k + 2] = raw[u % FF_H][k].z;
						W.w[4 * k + 3] = raw[u % FF_H][k].w;
					}
#endif
					const bool egress = flv[u] & 1u;
					const ftuple t = parse_frame_w(s, W, fd + i * 64u, len[u], min(len[u], 64u), egress, ep[u], lxl);
					const bool v6 = t.status == 0 && t.fam != 4u;
					fl[u] = egress ? 1u : 0u;
					sa[u] = da[u] = dport[u] = proto[u] = 0u;
					/* the status the output reports (0 for an IPv6 frame's
					 * placeholder, which the v6 pass overwrites) */
					fst[threadIdx.x * Q + u] = (int16_t)t.status;
					if (t.status != 0) {
						fl[u] |= FRF_DEC;
					} else if (!v6) {
						sa[u] = t.sa.x;
						da[u] = t.da.x;
						dport[u] = t.dport;
						proto[u] = t.proto;
						fl[u] |= t.frag ? 2u : 0u;
					} else {
						fl[u] |= FRF_V6;
					}
					/* wave-aggregated rows of the IPv6 frames (fr_emit) */
					const bool m6 = ok && v6;
					const uint64_t m = __ballot(m6);
					if (m) {
						const int leader = __ffsll((unsigned long long)m) - 1;
						uint32_t base = 0;
						if ((int)lane == leader)
							base = atomicAdd(fx.n6, (uint32_t)__popcll(m));
						base = __shfl(base, leader, 64);
						if (m6) {
							const uint32_t j = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
							fx.sa6[j] = t.sa;
							fx.da6[j] = t.da;
							fx.dport6[j] = (uint16_t)t.dport;
							fx.proto6[j] = (uint8_t)t.proto;
							fx.fl6[j] = (uint8_t)(egress ? 1u : 0u);
							fx.len6[j] = len[u];
							fx.ep6[j] = (uint16_t)ep[u];
							fx.idx6[j] = (uint32_t)(a.n_off + i);
						}
					}
				}
			} else if (full && Q == 4) {
				const uint32_t f4 = ld_x1<NTL>(a.flags + i0);
				const uint32_t p4 = ld_x1<NTL>(a.proto + i0);
				const uint2 d4 = ld_x2<NTL>(a.dport + i0);
				const uint2 e4 = ld_x2<NTL>(a.ep + i0);
				const uint4 l4 = ld_x4<NTL>(a.len + i0);
				const uint4 s4 = V6 ? make_uint4(0, 0, 0, 0)
						    : ld_x4<NTL>(static_cast<const uint32_t *>(a.saddr) + i0);
				const uint4 a4 = V6 ? make_uint4(0, 0, 0, 0)
						    : ld_x4<NTL>(static_cast<const uint32_t *>(a.daddr) + i0);
				defer_flush(); /* behind the loads just issued */
				const uint32_t dd[4] = {d4.x & 0xFFFFu, d4.x >> 16, d4.y & 0xFFFFu, d4.y >> 16};
				const uint32_t ee[4] = {e4.x & 0xFFFFu, e4.x >> 16, e4.y & 0xFFFFu, e4.y >> 16};
				const uint32_t ll[4] = {l4.x, l4.y, l4.z, l4.w};
				const uint32_t ss[4] = {s4.x, s4.y, s4.z, s4.w};
				const uint32_t aa[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
				for (int u = 0; u < Q; u++) {
					fl[u] = (f4 >> (8 * u)) & 0xFFu;
					proto[u] = (p4 >> (8 * u)) & 0xFFu;
					dport[u] = dd[u];
					ep[u] = ee[u];
					len[u] = ll[u];
					sa[u] = ss[u];
					da[u] = aa[u];
				}
			} else if (full && Q == 2) {
				const uint32_t f2 = *reinterpret_cast<const uint16_t *>(a.flags + i0);
				const uint32_t p2 = *reinterpret_cast<const uint16_t *>(a.proto + i0);
				const uint32_t d2 = ld_x1<NTL>(a.dport + i0);
				const uint32_t e2 = ld_x1<NTL>(a.ep + i0);
				const uint2 l2 = ld_x2<NTL>(a.len + i0);
				const uint2 s2 = V6 ? make_uint2(0, 0)
						    : ld_x2<NTL>(static_cast<const uint32_t *>(a.saddr) + i0);
				const uint2 a2 = V6 ? make_uint2(0, 0)
						    : ld_x2<NTL>(static_cast<const uint32_t *>(a.daddr) + i0);
				const uint32_t dd[2] = {d2 & 0xFFFFu, d2 >> 16}, ee[2] = {e2 & 0xFFFFu, e2 >> 16};
				const uint32_t ll[2] = {l2.x, l2.y}, ss[2] = {s2.x, s2.y}, aa[2] = {a2.x, a2.y};
#pragma unroll
				for (int u = 0; u < Q; u++) {
					fl[u] = (f2 >> (8 * u)) & 0xFFu;
					proto[u] = (p2 >> (8 * u)) & 0xFFu;
					dport[u] = dd[u];
					ep[u] = ee[u];
					len[u] = ll[u];
					sa[u] = ss[u];
					da[u] = aa[u];
				}
			} else {
#pragma unroll
				for (int u = 0; u < Q; u++) {
					const uint64_t i = i0 + u < a.n ? i0 + u : i0;
					fl[u] = a.flags[i];
					proto[u] = a.proto[i];
					dport[u] = a.dport[i];
					ep[u] = a.ep[i];
					len[u] = a.len[i];
					sa[u] = V6 ? 0u : static_cast<const uint32_t *>(a.saddr)[i];
					da[u] = V6 ? 0u : static_cast<const uint32_t *>(a.daddr)[i];
				}
			}
			uint32_t lbf[Q];
#pragma unroll
			for (int u = 0; u < Q; u++)
				lbf[u] = 0;
			if (V6) {
				/* the looked-up address only: daddr egress, saddr ingress */
#pragma unroll
				for (int u = 0; u < Q; u++) {
					const uint64_t i = i0 + u < a.n ? i0 + u : i0;
					if constexpr (IPCE) { /* the pre-pass looked the address up */
						ad6[u] = make_uint4(0, 0, 0, 0);
						continue;
					}
					uint4 raw = ld_x4<NTL>(static_cast<const uint4 *>((fl[u] & 1u) ? a.daddr : a.saddr) + i);
					if (LB && live && (fl[u] & 1u) && i0 + u < a.n) {
						/* egress service step first (bpf_lxc.c:117-149) */
						uint32_t h;
						if (a.hash) {
							h = a.hash[i];
						} else {
							const uint4 sr = ld_x4<NTL>(static_cast<const uint4 *>(a.saddr) + i);
							h = flow_hash(fold6(sr.x, sr.y, sr.z, sr.w), fold6(raw.x, raw.y, raw.z, raw.w),
								      a.sport[i], dport[u], proto[u]);
						}
						const lb6_res r = lb6_one(s, raw, dport[u], proto[u], h);
						if (r.ret == DROP_NO_SERVICE) {
							lbf[u] = F_LBDROP;
						} else {
							raw = r.tdaddr;
							dport[u] = r.dport;
						}
					}
					ad6[u] = v6_host_words(raw);
				}
			}
			if (LB && !V6) {
				/* egress service step first (bpf_lxc.c:444-469): the
				 * translated tuple.daddr and dport feed ipcache / policy */
				uint32_t hh[QA], sp[QA];
#pragma unroll
				for (int u = 0; u < Q; u++)
					hh[u] = sp[u] = 0;
				if (full && Q == 4) {
					if (a.hash) {
						const uint4 h4 = ld_x4<NTL>(a.hash + i0);
						hh[0] = h4.x, hh[1] = h4.y, hh[2] = h4.z, hh[3] = h4.w;
					} else {
						const uint2 s4 = ld_x2<NTL>(a.sport + i0);
						sp[0] = s4.x & 0xFFFFu, sp[1] = s4.x >> 16;
						sp[2] = s4.y & 0xFFFFu, sp[3] = s4.y >> 16;
					}
				} else {
#pragma unroll
					for (int u = 0; u < Q; u++) {
						const uint64_t i = i0 + u < a.n ? i0 + u : i0;
						if (a.hash)
							hh[u] = a.hash[i];
						else
							sp[u] = a.sport[i];
					}
				}
				bool act[Q], drop[Q];
#pragma unroll
				for (int u = 0; u < Q; u++) {
					act[u] = (fl[u] & 1u) && i0 + u < a.n;
					if (!a.hash)
						hh[u] = flow_hash(sa[u], da[u], sp[u], dport[u], proto[u]);
				}
				/* XDP (config 5 whole): the netdev's XDP prefilter (bpf_xdp.c
				 * check_v4) before an ingress tuple reaches from_netdev
				 * (bpf_netdev.c:470), in the service step's stages */
				bool in[Q], pass[Q];
#pragma unroll
				for (int u = 0; u < Q; u++)
					in[u] = XDP && !(fl[u] & 1u) && i0 + u < a.n;
				lb4_lxc_q<Q, XDP>(s, sa, da, dport, proto, hh, act, drop, in, pass);
#pragma unroll
				for (int u = 0; u < Q; u++) {
					if (drop[u])
						lbf[u] = F_LBDROP;
					if (XDP && !pass[u])
						lbf[u] = F_LBDROP | F_XDP;
				}
			}
#pragma unroll
			for (int u = 0; u < Q; u++) {
				const bool eg = fl[u] & 1u;
				/* frames: a frame the parse ended runs no lookup (F_GATED
				 * masks them) and reports its status (its daddr column,
				 * re-read at the output: 0 for an IPv6 frame's placeholder) */
				const bool dec = FR && !V6 && (fl[u] & (FRF_DEC | FRF_V6));
				if (dec)
					lbf[u] |= F_DEC | F_GATED;
				/* ct_lookup{4,6} protocol gate: ICMP (v4: 1, v6: 58), TCP, UDP */
				const bool gated = s.ct_proto_gate && proto[u] != (V6 ? 58u : 1u) && proto[u] != 6u &&
						   proto[u] != 17u;
				/* IPv6 passes is_fragment = false (bpf_lxc.c:787-789) */
				fw[u] = (live && iu(u) < a.n ? F_OK : 0u) | (eg ? F_EG : 0u) | (gated ? F_GATED : 0u) | lbf[u] |
					(!V6 && !eg && ((fl[u] >> 1) & 1u) ? F_FRAG : 0u);
				ad[u] = eg ? da[u] : sa[u];
				hi4[u] = dport[u] | (proto[u] << 16) | (eg ? (1u << 24) : 0u);
			}
		}
		/* ipcache lookup (eps.h:56-80) */
		uint32_t e[Q];
		if (V6) {
			bool act[Q];
#pragma unroll
			for (int u = 0; u < Q; u++)
				act[u] = (fw[u] & (F_OK | F_GATED | F_LBDROP)) == F_OK;
#ifdef CGPU_DIAG_V6_NO_TRIE /* timing-only tool build: wrong identities */
#pragma unroll
			for (int u = 0; u < Q; u++)
				e[u] = act[u] ? (DIR_TAG_DIRECT | 2u) : 0u;
#else
			if constexpr (IPCE) {
				uint32_t pe[QA];
				if (full && Q == 4) {
					const uint4 v = ld_x4<NTL>(a.ipc_e + i0);
					pe[0] = v.x, pe[1] = v.y, pe[2] = v.z, pe[3] = v.w;
				} else if (full && Q == 2) {
					const uint2 v = ld_x2<NTL>(a.ipc_e + i0);
					pe[0] = v.x, pe[1] = v.y;
				} else {
#pragma unroll
					for (int u = 0; u < Q; u++)
						pe[u] = a.ipc_e[i0 + u < a.n ? i0 + u : i0];
				}
#pragma unroll
				for (int u = 0; u < Q; u++)
					e[u] = act[u] ? pe[u] : 0u;
			} else {
				v6t_lookup_q<Q>(s.ipc6, ldict, n24 != 0u, ad6, act, e);
			}
#endif
		} else {
			/* v4: the /16's inline node (x16), then the compressed LPM */
			{
				/* one 16-byte gather: the /16's inline run node (tables.h) */
				uint4 q[Q];
#pragma unroll
				for (int u = 0; u < Q; u++) {
					q[u] = make_uint4(0, 0, 0, 0);
					if ((fw[u] & (F_OK | F_GATED | F_LBDROP)) == F_OK)
						q[u] = reinterpret_cast<const uint4 *>(s.ipc4c.x16)[DIAG_LPM(bswap32(ad[u]) >> 16)];
				}
#pragma unroll
				for (int u = 0; u < Q; u++) {
					if (q[u].w & LPMC_OVERFLOW) {
						e[u] = q[u].x;
						continue;
					}
					const uint32_t x = bswap32(ad[u]) & 0xFFFFu;
					const uint32_t cnt = (x >= (q[u].x & 0xFFFFu) ? 1u : 0u) + (x >= (q[u].x >> 16) ? 1u : 0u) +
							     (x >= (q[u].y & 0xFFFFu) ? 1u : 0u) + (x >= (q[u].y >> 16) ? 1u : 0u);
					const uint64_t v = ((uint64_t)q[u].w << 32) | q[u].z;
					e[u] = (fw[u] & (F_OK | F_GATED | F_LBDROP)) == F_OK ? ldict[(uint32_t)(v >> (12u * cnt)) & 0xFFFu] : 0u;
				}
			}
			{
				/* compressed LPM (tables.h lpm16c): arrays (rare), then one run node */
				constexpr uint32_t ARR = (DIR_TAG_GROUP >> LPMC_KIND_SHIFT) | 3u;
#pragma unroll
				for (int u = 0; u < Q; u++)
					if ((e[u] >> LPMC_KIND_SHIFT) == ARR) {
						e[u] = s.ipc4c.nodes[(size_t)(e[u] & LPMC_OFF_MASK) * 4u +
								     ((bswap32(ad[u]) >> 8) & 255u)];
						fw[u] |= F_LVL8; /* below an array: x is the last byte */
					}
#pragma unroll
				for (int u = 0; u < Q; u++)
					if ((e[u] >> LPMC_KIND_SHIFT) == ARR)
						e[u] = s.ipc4c.nodes[(size_t)(e[u] & LPMC_OFF_MASK) * 4u + (bswap32(ad[u]) & 255u)];
				/* the first 32 bytes of every node in flight together; the
				 * rare 64-byte node reads its second half one tuple at a time */
				uint4 q[Q][2];
#pragma unroll
				for (int u = 0; u < Q; u++) {
					q[u][0] = q[u][1] = make_uint4(0, 0, 0, 0);
					if ((e[u] & DIR_TAG_MASK) == DIR_TAG_GROUP) {
						const uint4 *nd = reinterpret_cast<const uint4 *>(s.ipc4c.nodes) +
								  (e[u] & LPMC_OFF_MASK);
						q[u][0] = nd[0];
						if ((e[u] >> LPMC_KIND_SHIFT) & 3u)
							q[u][1] = nd[1];
					}
				}
#pragma unroll
				for (int u = 0; u < Q; u++) {
					if ((e[u] & DIR_TAG_MASK) != DIR_TAG_GROUP)
						continue;
					const uint32_t kind = (e[u] >> LPMC_KIND_SHIFT) & 3u;
					uint4 q2 = make_uint4(0, 0, 0, 0), q3 = q2;
					if (kind == 2) {
						const uint4 *nd = reinterpret_cast<const uint4 *>(s.ipc4c.nodes) +
								  (e[u] & LPMC_OFF_MASK);
						q2 = nd[2];
						q3 = nd[3];
					}
					const uint32_t h = bswap32(ad[u]);
					e[u] = lpmc_search(q[u][0], q[u][1], q2, q3, kind,
							   (fw[u] & F_LVL8) ? (h & 255u) : (h & 0xFFFFu));
				}
			}
		}
		/* identity (bpf_lxc.c:488-496 / bpf_netdev.c:374-404) */
		uint32_t id[QA];
#pragma unroll
		for (int u = 0; u < Q; u++) {
			const uint32_t label = entry_label(V6 ? s.ipc6.vals : s.ipc4c.vals, e[u]);
			/* v6: ipv6_match_prefix_64(daddr, ROUTER_IP), bpf/lib/ipv6.h:166-175
			 * (ad6: host-order words) */
			const bool in_cluster = V6 ? ad6[u].x == bswap32(s.router_ip64[0]) &&
							     ad6[u].y == bswap32(s.router_ip64[1])
						   : (ad[u] & s.ipv4_cluster_mask) == s.ipv4_cluster_range;
			if (fw[u] & F_EG) {
				if (e[u] && label)
					id[u] = label;
				else if (in_cluster)
					id[u] = s.cluster_id;
				else
					id[u] = s.world_id;
			} else {
				uint32_t src = s.ingress_src_identity;
				if (src < s.health_id && e[u] && label && label != s.cluster_id && (V6 || label != s.host_id))
					src = label;
				id[u] = (!V6 && s.ingress_secctx_world) ? s.world_id : src;
			}
		}
		/* The cascade of policy.h:46-110 over the group of {ep, id, dir}
		 * (tables.h pol_groups): one gather of the group slot gives probe 2
		 * (the L3 key) and a bloom over the group's (dport, proto); probe 1
		 * gathers the exact key only when the bloom admits it; probe 3
		 * (identity 0) gathers directly.  Stages and counters are the
		 * reference's: st = the probe that hit. */
		int ctr[Q];
		uint32_t z[Q], st[QA], bk[Q], need[Q];
		uint4 sl[Q], grp[Q];
#pragma unroll
		for (int u = 0; u < Q; u++) {
			ctr[u] = -1;
			z[u] = 0;
			st[u] = 0;
			grp[u] = make_uint4(0, 0, POL_CTR_EMPTY, 0);
			if ((fw[u] & (F_OK | F_GATED | F_LBDROP)) == F_OK) {
				bk[u] = pg_hash(id[u], ep[u] | (hi4[u] >> 24) << 16) & s.pg.mask;
				grp[u] = s.pg.slots[DIAG_P2(bk[u])];
			}
		}
#pragma unroll
		for (int u = 0; u < Q; u++) {
			if ((fw[u] & (F_OK | F_GATED | F_LBDROP)) != F_OK)
				continue;
			grp[u] = pg_resolve(s.pg, grp[u], bk[u], id[u], ep[u] | (hi4[u] >> 24) << 16);
			const uint32_t bl = pg_bloom(hi4[u] & 0xFFFFu, (hi4[u] >> 16) & 0xFFu);
			need[u] = !(fw[u] & F_FRAG) && (grp[u].w & bl) == bl;
		}
		/* probe 1: exact {id, dport, proto, dir} (policy.h:61-72) */
#pragma unroll
		for (int u = 0; u < Q; u++)
			if ((fw[u] & (F_OK | F_GATED | F_LBDROP)) == F_OK && need[u]) {
				bk[u] = pol_hash(id[u], hi4[u], ep[u]) & pmask;
				sl[u] = ptab[DIAG_P1(bk[u])];
			}
#pragma unroll
		for (int u = 0; u < Q; u++)
			if ((fw[u] & (F_OK | F_GATED | F_LBDROP)) == F_OK && need[u]) {
				ctr[u] = pol_resolve1(s.pol, sl[u], bk[u], id[u], hi4[u], ep[u], &z[u]);
				st[u] = 1;
			}
		/* probe 2: L3-only {id, 0, 0, dir} (policy.h:74-83), from the group */
#pragma unroll
		for (int u = 0; u < Q; u++)
			if ((fw[u] & (F_OK | F_GATED | F_LBDROP)) == F_OK && ctr[u] < 0) {
				st[u] = 2;
				if ((grp[u].z & POL_CTR_MASK) != POL_CTR_EMPTY) {
					ctr[u] = (int)(grp[u].z & POL_CTR_MASK);
					z[u] = 0;
				}
			}
		/* probe 3: identity-wildcard L4 {0, dport, proto, dir} (policy.h:85-96) */
#pragma unroll
		for (int u = 0; u < Q; u++)
			if ((fw[u] & (F_OK | F_GATED | F_LBDROP | F_FRAG)) == F_OK && ctr[u] < 0) {
				bk[u] = pol_hash(0u, hi4[u], ep[u]) & pmask;
				sl[u] = ptab[bk[u]];
			}
#pragma unroll
		for (int u = 0; u < Q; u++)
			if ((fw[u] & (F_OK | F_GATED | F_LBDROP | F_FRAG)) == F_OK && ctr[u] < 0) {
				ctr[u] = pol_resolve1(s.pol, sl[u], bk[u], 0u, hi4[u], ep[u], &z[u]);
				st[u] = 3;
			}
		/* counters, outputs, metrics */
		int32_t v[QA];
		uint64_t *metg = a.delta + 2ull * s.n_ctr_slots;
#pragma unroll
		for (int u = 0; u < Q; u++) {
			if (FR && (fw[u] & F_DEC)) {
				/* k_frames' rules: NOT_CLASSIFIED counts nothing (stage 7), an
				 * IPv6 frame's placeholder is overwritten by the v6 pass */
				id[u] = 0;
				v[u] = 0;
				st[u] = 0;
				if (!(fw[u] & F_OK))
					continue; /* a tail lane repeating tuple i0: no status, no metrics */
				const int32_t sv = FF ? (int32_t)fst[threadIdx.x * Q + u]
						      : (int32_t)static_cast<const uint32_t *>(a.daddr)[i0 + u];
				if (sv == 0 || sv == FRAME_NOT_CLASSIFIED) {
					v[u] = 0;
					st[u] = sv ? 7u : 0u;
				} else {
					v[u] = sv;
					st[u] = sv == DROP_CT_UNKNOWN_PROTO ? 4u : 5u;
					if (sv != DROP_SNAPLEN) {
						const uint32_t reason = (uint32_t)(-sv) & 0xffu;
						const uint32_t key = (reason * 4u + ((fw[u] & F_EG) ? 2u : 1u)) * 2u;
						atomicAdd((unsigned long long *)&metg[key], 1ull);
						atomicAdd((unsigned long long *)&metg[key + 1], (unsigned long long)len[u]);
					}
				}
				continue;
			}
			if (XDP && (fw[u] & F_XDP)) {
				/* XDP_DROP: nothing counted, nothing notified */
				v[u] = VERDICT_XDP_DROP;
				id[u] = 0;
				st[u] = 8;
			} else if (fw[u] & F_LBDROP) {
				v[u] = DROP_NO_SERVICE;
				id[u] = 0;
				st[u] = 6;
			} else if (fw[u] & F_GATED) {
				v[u] = DROP_CT_UNKNOWN_PROTO;
				id[u] = 0;
				st[u] = 4;
			} else if (ctr[u] >= 0) {
				const uint32_t c = (uint32_t)ctr[u];
				if (len[u] >= PKC_MAX_LEN) {
					atomicAdd((unsigned long long *)&pctr[2u * c], 1ull);
					atomicAdd((unsigned long long *)&pctr[2u * c + 1u], (unsigned long long)len[u]);
				} else if (c < s.hot_slots) {
					atomicAdd((unsigned long long *)&lctr[c],
						  (1ull << PK_SHIFT) | (unsigned long long)len[u]);
				} else {
#ifndef CGPU_DIAG_NO_COLD /* timing-only tool build (tools/diag_ab.py): counters wrong */
					/* the workgroup's cold-slot cache: a global atomic
					 * executes at the memory side (one 64-B request each,
					 * MI355X_MICROARCH.md), so hits aggregate in LDS and
					 * each touched slot costs one atomic at the end; a
					 * slot that finds no free entry in CC_PROBE goes global */
					bool done = false;
					if (a.cc_n) {
						uint32_t j = __umulhi(c * 0x9E3779B1u, a.cc_n);
#pragma unroll
						for (int p = 0; p < CC_PROBE && !done; p++, j++) {
							j = j == a.cc_n ? 0u : j;
							uint32_t t = cck[j];
							if (t == 0u) {
								const uint32_t o = atomicCAS(&cck[j], 0u, c + 1u);
								t = o == 0u ? c + 1u : o;
							}
							if (t == c + 1u) {
								atomicAdd((unsigned long long *)&ccv[j],
									  (1ull << PK_SHIFT) | (unsigned long long)len[u]);
								done = true;
							}
						}
					}
					if (!done) {
						if constexpr (DEFER) {
							dcs[u] = c;
							dln[u] = len[u];
						} else {
							atomicAdd((unsigned long long *)&pk[c],
								  (1ull << PKC_SHIFT) | (unsigned long long)len[u]);
						}
					}
#endif
				}
				v[u] = st[u] == 2 ? 0 : (int32_t)(z[u] >> 16);
			} else {
				st[u] = 0;
				v[u] = DROP_POLICY;
			}
			if ((fw[u] & F_OK) && v[u] == 0) {
				const uint32_t e = (fw[u] & F_EG) ? 1u : 0u;
				fwd_n[e] += 1u;
				fwd_b[e] += len[u];
			}
			if ((fw[u] & (F_OK | (XDP ? F_XDP : 0u))) == F_OK && v[u] < 0) {
				const uint32_t mr = v[u] == DROP_POLICY ? 1u : (v[u] == DROP_NO_SERVICE ? 3u : 2u);
				const uint32_t mi = (mr * 2u + ((fw[u] & F_EG) ? 1u : 0u)) * 2u;
				atomicAdd(&lmet[mi], 1ull);
				atomicAdd(&lmet[mi + 1u], (unsigned long long)len[u]);
			}
		}
		if constexpr (FF) {
#pragma unroll
			for (int u = 0; u < Q; u++)
				if (fw[u] & F_OK) {
					const uint64_t i = iu(u);
					if (NTL) {
						__builtin_nontemporal_store(v[u], a.verdict + i);
						__builtin_nontemporal_store(id[u], a.identity + i);
					} else {
						a.verdict[i] = v[u];
						a.identity[i] = id[u];
					}
					if (a.stage)
						a.stage[i] = (uint8_t)st[u];
				}
		} else if (full && Q == 4) {
#ifdef CGPU_DIAG_STORE_SC1 /* write-through stores that leave the XCD's L2 */
			{
				const auto rv = __builtin_amdgcn_make_buffer_rsrc(a.verdict, 0, (int)(a.n * 4u), 0x00020000);
				const auto ri = __builtin_amdgcn_make_buffer_rsrc(a.identity, 0, (int)(a.n * 4u), 0x00020000);
				v4u_t vv = {(uint32_t)v[0], (uint32_t)v[1], (uint32_t)v[2], (uint32_t)v[3]};
				v4u_t vi = {id[0], id[1], id[2], id[3]};
				__builtin_amdgcn_raw_buffer_store_b128(vv, rv, (int)(i0 * 4u), 0, 16);
				__builtin_amdgcn_raw_buffer_store_b128(vi, ri, (int)(i0 * 4u), 0, 16);
			}
#else
			st_x4<NTL>(a.verdict + i0, (uint32_t)v[0], (uint32_t)v[1], (uint32_t)v[2], (uint32_t)v[3]);
			st_x4<NTL>(a.identity + i0, id[0], id[1], id[2], id[3]);
#endif
			if (a.stage)
				st_x1<NTL>(a.stage + i0, st[0] | (st[1] << 8) | (st[2] << 16) | (st[3] << 24));
		} else if (full && Q == 2) {
			*reinterpret_cast<int2 *>(a.verdict + i0) = make_int2(v[0], v[1]);
			*reinterpret_cast<uint2 *>(a.identity + i0) = make_uint2(id[0], id[1]);
			if (a.stage)
				*reinterpret_cast<uint16_t *>(a.stage + i0) = (uint16_t)(st[0] | (st[1] << 8));
		} else {
#pragma unroll
			for (int u = 0; u < Q; u++)
				if (fw[u] & F_OK) {
					a.verdict[i0 + u] = v[u];
					a.identity[i0 + u] = id[u];
					if (a.stage)
						a.stage[i0 + u] = (uint8_t)st[u];
				}
		}
	}

	uint64_t *met = a.delta + 2ull * s.n_ctr_slots;
#pragma unroll
	for (int e = 0; e < 2; e++) {
		const uint64_t c = wave_sum((uint64_t)fwd_n[e]);
		const uint64_t b = wave_sum(fwd_b[e]);
		if ((threadIdx.x & 63) == 0 && c) {
			atomicAdd((unsigned long long *)&met[(e + 1u) * 2u], (unsigned long long)c);
			atomicAdd((unsigned long long *)&met[(e + 1u) * 2u + 1u], (unsigned long long)b);
		}
	}
	__syncthreads();
	if (threadIdx.x >= 4 && threadIdx.x < 16 && lmet[threadIdx.x]) {
		const uint32_t reasons[4] = {0u, 133u, 137u, 158u};
		const uint32_t c = threadIdx.x >> 1;
		const uint32_t key = (reasons[c >> 1] * 4u + ((c & 1) ? 2u : 1u)) * 2u + (threadIdx.x & 1u);
		atomicAdd((unsigned long long *)&met[key], lmet[threadIdx.x]);
	}
	__syncthreads();
	/* one packed atomic per touched hot slot: PK (LDS) -> PKC (pk) format;
	 * a workgroup's bytes per slot stay < 2^37 (<= 2^26 tuples of < 2^11) */
	for (uint32_t k = threadIdx.x; k < s.hot_slots; k += NT) {
		const uint64_t x = lctr[k];
		if (x)
			atomicAdd((unsigned long long *)&pk[k],
				  ((x >> PK_SHIFT) << PKC_SHIFT) | (x & PK_BYTES_MASK));
	}
	for (uint32_t k = threadIdx.x; k < a.cc_n; k += NT) {
		const uint32_t t = cck[k];
		const uint64_t x = ccv[k];
		if (t && x)
			atomicAdd((unsigned long long *)&pk[t - 1u],
				  ((x >> PK_SHIFT) << PKC_SHIFT) | (x & PK_BYTES_MASK));
	}
}

/* ------------------------------------------------------------------ */
/* raw Ethernet frames -> policy tuple -> verdict   */
/* ------------------------------------------------------------------ */
#define DROP_INVALID_SMAC (-130) /* bpf/lib/common.h:237-264 */
#define DROP_INVALID_DMAC (-131)
#define DROP_INVALID_SIP (-132)
#define DROP_INVALID (-134)
#define DROP_CT_INVALID_HDR (-135)
#define DROP_UNKNOWN_L3 (-139)
#define DROP_UNKNOWN_TARGET (-150)
#define DROP_INVALID_EXTHDR (-156)
#define DROP_FRAG_NOSUPPORT (-157)
#define EFAULT_LOAD (-14)        /* bpf_skb_load_bytes past skb->len */


/* A header read of [off, off + sz): the reference bounds it by skb->len
 * (revalidate_data / skb_load_bytes) and returns `err` past it; within len
 * the bytes must also lie in the stored slot (cap = min(len, stride)). */
__device__ __forceinline__ int32_t fchk(uint32_t off, uint32_t sz, uint32_t len, uint32_t cap, int32_t err)
{
	return off + sz > len ? err : (off + sz > cap ? DROP_SNAPLEN : 0);
}

/* One frame through the endpoint programs' steps before ipcache (cgpu.h
 * cgpu_frames_parse).  Window reads when the L4 header sits right behind
 * an option-less IPv4 / extension-less IPv6 header, global loads (L2) for
 * IPv4 options and IPv6 extension headers. */
__device__ __forceinline__ ftuple parse_frame_w(const cgpu_snapshot &s, const fwin &W, const uint8_t *f,
						uint32_t len, uint32_t cap, bool egress, uint32_t ep,
						const uint4 *lxc);

__device__ __forceinline__ ftuple parse_frame(const cgpu_snapshot &s, const uint8_t *f, uint32_t len,
					      uint32_t cap, bool egress, uint32_t ep)
{
	fwin W;
#pragma unroll
	for (int k = 0; k < 4; k++) {
		const uint4 v = ld_x4<true>(f + 16 * k);
		W.w[4 * k] = v.x;
		W.w[4 * k + 1] = v.y;
		W.w[4 * k + 2] = v.z;
		W.w[4 * k + 3] = v.w;
	}
	return parse_frame_w(s, W, f, len, cap, egress, ep, s.lxc);
}

/* the same with the frame's first 64 bytes already in W; lxc = the
 * endpoints' rows (s.lxc, or a copy in LDS) */
__device__ __forceinline__ ftuple parse_frame_w(const cgpu_snapshot &s, const fwin &W, const uint8_t *f,
						uint32_t len, uint32_t cap, bool egress, uint32_t ep,
						const uint4 *lxc)
{
	ftuple t;
	t.status = 0;
	t.fam = 0;
	t.sa = uint4{0, 0, 0, 0};
	t.da = uint4{0, 0, 0, 0};
	t.dport = 0;
	t.proto = 0;
	t.frag = false;
	if (len < 14u) { /* no Ethernet header to dispatch on */
		t.status = DROP_INVALID;
		return t;
	}
	/* skb->protocol dispatch: egress bpf_lxc.c:690-710 (ARP to the ARP
	 * responder, others DROP_UNKNOWN_L3); ingress bpf_netdev.c:494-521
	 * (non-IP passed to the stack) */
	const uint32_t et = W.h(12);
	const bool v4 = et == 0x0008u;
	if (!v4 && et != 0xDD86u) {
		t.status = (egress && et != 0x0608u) ? DROP_UNKNOWN_L3 : FRAME_NOT_CLASSIFIED;
		return t;
	}
	t.fam = v4 ? 4u : 6u;
	/* revalidate_data: ETH_HLEN + sizeof(iphdr / ipv6hdr) <= len
	 * (bpf/lib/common.h:71-91); the window holds both headers */
	if (len < (v4 ? 34u : 54u)) {
		t.status = DROP_INVALID;
		return t;
	}
	if (v4) {
		t.sa.x = W.d(26);
		t.da.x = W.d(30);
		t.proto = W.b(23);
	} else {
		t.sa = uint4{W.d(22), W.d(26), W.d(30), W.d(34)};
		t.da = uint4{W.d(38), W.d(42), W.d(46), W.d(50)};
		t.proto = W.b(20);
	}
	if (egress && !v4 && t.proto == 58u) {
		/* handle_ipv6 (bpf_lxc.c:364-389), before ipv6_l3_from_lxc and its
		 * endpoint checks: an ICMPv6 frame needs its icmp6hdr (DROP_INVALID),
		 * then icmp6_handle (lib/icmp6.h:390-412) hands a neighbour
		 * solicitation and an echo request to ROUTER_IP to the responders
		 * (tail calls: the frame leaves classification, as ARP does).  The
		 * NS responder drops an unknown target (ACTION_UNKNOWN_ICMP6_NS,
		 * DROP_UNKNOWN_TARGET) and reads the ND option at 78 (icmp6.h:
		 * 148-204).  The ND target lies past the window: byte loads (rare). */
		int32_t r = len < 62u ? DROP_INVALID : 0;
		if (!r) {
			const uint32_t type = W.b(54);
			if (type == 135u) {
				r = fchk(62u, 16u, len, cap, DROP_INVALID);
				if (!r) {
					uint32_t diff = 0;
#pragma unroll
					for (int k = 0; k < 4; k++) {
						const uint32_t w = (uint32_t)f[62 + 4 * k] | (uint32_t)f[63 + 4 * k] << 8 |
								   (uint32_t)f[64 + 4 * k] << 16 |
								   (uint32_t)f[65 + 4 * k] << 24;
						diff |= w ^ s.router_ip[k];
					}
					r = diff ? DROP_UNKNOWN_TARGET : fchk(78u, 8u, len, cap, DROP_INVALID);
					if (!r)
						r = FRAME_NOT_CLASSIFIED;
				}
			} else if (type == 128u && t.da.x == s.router_ip[0] && t.da.y == s.router_ip[1] &&
				   t.da.z == s.router_ip[2] && t.da.w == s.router_ip[3]) {
				r = FRAME_NOT_CLASSIFIED;
			}
		}
		if (r) {
			t.status = r;
			return t;
		}
	}
	if (egress && ep < s.n_lxc) {
		/* SMAC / DMAC / SIP checks of the endpoint (bpf_lxc.c:431-437,
		 * :100-105; lib/lxc.h:31-89) */
		const uint4 i0 = lxc[2u * ep];
		const uint32_t verify = (i0.y >> 16) & 0xffu;
		if ((verify & CGPU_VERIFY_SMAC) && (W.d(6) != i0.x || W.h(10) != (i0.y & 0xffffu))) {
			t.status = DROP_INVALID_SMAC;
			return t;
		}
		if ((verify & CGPU_VERIFY_DMAC) && (W.d(0) != s.node_mac_lo || W.h(4) != s.node_mac_hi)) {
			t.status = DROP_INVALID_DMAC;
			return t;
		}
		if (verify & CGPU_VERIFY_SIP) {
			bool ok;
			if (v4) {
				ok = t.sa.x == i0.z;
			} else {
				const uint4 i1 = lxc[2u * ep + 1u];
				ok = t.sa.x == i0.w && t.sa.y == i1.x && t.sa.z == i1.y && t.sa.w == i1.z;
			}
			if (!ok) {
				t.status = DROP_INVALID_SIP;
				return t;
			}
		}
	}
	uint32_t l4;
	bool inwin;
	if (v4) {
		/* ipv4_hdrlen (ipv4.h:45-48): ihl * 4, not validated by the
		 * reference; ipv4_is_fragment (ipv4.h:50-61): ingress only,
		 * policy_can_egress4 passes false */
		l4 = 14u + 4u * (W.b(14) & 15u);
		inwin = l4 == 34u;
		t.frag = !egress && (W.h(20) & 0xFFBFu) != 0u;
	} else {
		/* ipv6_hdrlen (ipv6.h:61-98): at most IPV6_MAX_HEADERS (4)
		 * extension headers.  The length rule follows the reference
		 * exactly: the AUTH formula applies when the NEXT header is AUTH. */
		uint32_t nh = t.proto, off = 40u;
		int32_t r = 1;
		for (int k = 0; k < 4 && r == 1; k++) {
			if (nh == 59u) {
				r = DROP_INVALID_EXTHDR;
			} else if (nh == 44u) {
				r = DROP_FRAG_NOSUPPORT;
			} else if (nh == 0u || nh == 43u || nh == 51u || nh == 60u) {
				const uint32_t o = 14u + off;
				r = fchk(o, 2, len, cap, DROP_INVALID);
				if (!r) {
					const uint32_t hl = f[o + 1];
					nh = f[o];
					off += nh == 51u ? (hl + 2u) << 2 : (hl + 1u) << 3;
					r = 1;
				}
			} else {
				r = 0;
			}
		}
		if (r == 1)
			r = DROP_INVALID_EXTHDR;
		if (r) {
			t.status = r;
			return t;
		}
		t.proto = nh;
		l4 = 14u + off;
		inwin = l4 == 54u;
	}
	int32_t r;
	/* extract_l4_port of lb{4,6}_extract_key under LB_L4 (lib/lb.h:192-215,
	 * :590-599): TCP/UDP load the dport; a short frame returns the -EFAULT
	 * of skb_load_bytes, which the egress program returns */
	if (egress && (s.lb_flags & CGPU_LB_L4) && (t.proto == 6u || t.proto == 17u) &&
	    (r = fchk(l4 + 2u, 2, len, cap, EFAULT_LOAD))) {
		t.status = r;
		return t;
	}
	/* ct_lookup{4,6} (conntrack.h:470-528 / :317-378) for the CT_NEW tuple:
	 * built reversed, both lookups miss, the reverse leaves tuple.dport =
	 * the packet's dport.  ICMP echo request: sport = type -> dport 8
	 * (ICMPv6: 128); echo reply and other types: 0.  TCP also loads the
	 * flags at l4 + 12 (bounds only: the action does not reach policy).
	 * Without CONNTRACK the stubs leave the tuple ports 0. */
	if (s.ct_proto_gate) {
		if (t.proto == (v4 ? 1u : 58u)) {
			if ((r = fchk(l4, 1, len, cap, DROP_CT_INVALID_HDR))) {
				t.status = r;
				return t;
			}
			const uint32_t type = inwin ? (v4 ? W.b(34) : W.b(54)) : (uint32_t)f[l4];
			t.dport = type == (v4 ? 8u : 128u) ? type : 0u;
		} else if (t.proto == 6u || t.proto == 17u) {
			if ((r = fchk(l4, t.proto == 6u ? 14u : 4u, len, cap, DROP_CT_INVALID_HDR))) {
				t.status = r;
				return t;
			}
			t.dport = inwin ? (v4 ? W.h(36) : W.h(56))
					: (uint32_t) * reinterpret_cast<const uint16_t *>(f + l4 + 2u);
		} else {
			t.status = DROP_CT_UNKNOWN_PROTO;
		}
	}
	return t;
}

/*
 * MODE 0: cgpu_frames_parse — write the policy tuple columns.
 * MODE 1: cgpu_classify_frames — parse, then decide<> (the cgpu_classify_v4 /
 *         _v6 decision) with the k_classify<.., CTR = 1> counters (hot
 *         policy slots in LDS) and metrics.  One frame per lane; v4 and v6
 *         frames of a batch share waves.
 */
template <int MODE, int NT>
__global__ __launch_bounds__(NT) void k_frames(cgpu_snapshot s, frames_args a)
{
	extern __shared__ __attribute__((aligned(16))) uint64_t lctr[];
	/* metrics {reason 0 / 133 / 137} x {ingress, egress}; others direct */
	uint64_t mcnt[6] = {0, 0, 0, 0, 0, 0}, mbyt[6] = {0, 0, 0, 0, 0, 0};
	uint64_t *met = MODE == 1 ? a.delta + 2ull * s.n_ctr_slots : nullptr;
	if (MODE == 1) {
		for (uint32_t k = threadIdx.x; k < s.hot_slots; k += NT)
			lctr[k] = 0;
		__syncthreads();
	}
	const uint64_t gstride = (uint64_t)gridDim.x * NT;
	for (uint64_t i = (uint64_t)blockIdx.x * NT + threadIdx.x; i < a.n; i += gstride) {
		const uint32_t len = a.len[i];
		const bool egress = a.flags[i] & 1u;
		const uint32_t ep = a.ep[i];
		const ftuple t = parse_frame(s, a.data + i * (uint64_t)a.stride, len, min(len, a.stride), egress, ep);
		if (MODE == 0) {
			a.status[i] = t.status;
			if (a.family)
				a.family[i] = (uint8_t)t.fam;
			if (a.saddr16)
				reinterpret_cast<uint4 *>(a.saddr16)[i] = t.sa;
			if (a.daddr16)
				reinterpret_cast<uint4 *>(a.daddr16)[i] = t.da;
			if (a.dport)
				a.dport[i] = (uint16_t)t.dport;
			if (a.proto)
				a.proto[i] = (uint8_t)t.proto;
			if (a.tflags)
				a.tflags[i] = (uint8_t)((egress ? 1u : 0u) | (t.frag ? 2u : 0u));
			continue;
		}
		int32_t v;
		uint32_t id = 0, st;
		if (t.status == 0) {
			const decision d = t.fam == 4u
				? decide<0>(s, egress, t.frag, t.sa.x, t.da.x, uint4{}, uint4{}, t.dport, t.proto, ep)
				: decide<1>(s, egress, false, 0u, 0u, t.sa, t.da, t.dport, t.proto, ep);
			v = d.v;
			id = d.id;
			st = d.st;
			if (d.ctr >= 0) {
				const uint32_t c = (uint32_t)d.ctr;
				if (c < s.hot_slots && len < PK_MAX_LEN) {
					atomicAdd((unsigned long long *)&lctr[c],
						  (1ull << PK_SHIFT) | (unsigned long long)len);
				} else if (len < PKC_MAX_LEN) {
					/* one packed atomic (launch_classify_frames unpacks) */
					atomicAdd((unsigned long long *)&a.pk[c],
						  (1ull << PKC_SHIFT) | (unsigned long long)len);
				} else {
					atomicAdd((unsigned long long *)&a.delta[2u * c], 1ull);
					atomicAdd((unsigned long long *)&a.delta[2u * c + 1u], (unsigned long long)len);
				}
			}
		} else if (t.status == FRAME_NOT_CLASSIFIED) {
			v = 0;
			st = 7;
		} else {
			v = t.status;
			st = v == DROP_CT_UNKNOWN_PROTO ? 4u : 5u;
		}
		a.verdict[i] = v;
		a.identity[i] = id;
		if (a.stage)
			a.stage[i] = (uint8_t)st;
		/* not classified, snap-length, or a proxy redirect (TRACE_TO_PROXY
		 * counts nothing): no metrics */
		if (st == 7u || v == DROP_SNAPLEN || v > 0)
			continue;
		/* update_metrics(len, dir, -reason) (bpf/lib/drop.h:104), reason as u8 */
		const uint32_t reason = v < 0 ? (uint32_t)(-v) & 0xffu : 0u;
		const uint32_t dir = egress ? 1u : 0u;
		const int b = reason == 0u ? 0 : reason == 133u ? 1 : reason == 137u ? 2 : -1;
		if (b < 0) {
			const uint32_t key = (reason * 4u + dir + 1u) * 2u;
			atomicAdd((unsigned long long *)&met[key], 1ull);
			atomicAdd((unsigned long long *)&met[key + 1], (unsigned long long)len);
		} else {
#pragma unroll
			for (int k = 0; k < 6; k++) {
				const bool hit = k == 2 * b + (int)dir;
				mcnt[k] += hit ? 1u : 0u;
				mbyt[k] += hit ? len : 0u;
			}
		}
	}
	if (MODE == 0)
		return;
	const uint32_t reasons[3] = {0u, 133u, 137u};
#pragma unroll
	for (int k = 0; k < 6; k++) {
		const uint64_t c = wave_sum(mcnt[k]);
		const uint64_t b = wave_sum(mbyt[k]);
		if ((threadIdx.x & 63) == 0 && c) {
			const uint32_t key = (reasons[k >> 1] * 4u + ((k & 1) ? 2u : 1u)) * 2u;
			atomicAdd((unsigned long long *)&met[key], (unsigned long long)c);
			atomicAdd((unsigned long long *)&met[key + 1], (unsigned long long)b);
		}
	}
	__syncthreads();
	for (uint32_t k = threadIdx.x; k < s.hot_slots; k += NT) {
		const uint64_t v = lctr[k];
		if (v) {
			atomicAdd((unsigned long long *)&a.delta[2u * k], v >> PK_SHIFT);
			atomicAdd((unsigned long long *)&a.delta[2u * k + 1u], v & PK_BYTES_MASK);
		}
	}
}

/* delta[2s] += pk[s] >> 37; delta[2s+1] += pk[s] & (2^37-1); pk[s] = 0 */
__global__ __launch_bounds__(256) void k_unpack(uint64_t *delta, uint64_t *pk, uint32_t lo, uint32_t hi)
{
	for (uint32_t s = lo + blockIdx.x * blockDim.x + threadIdx.x; s < hi; s += gridDim.x * blockDim.x) {
		if (!pk[s])
			continue;
		/* atomic: classify calls on other streams may add meanwhile */
		const uint64_t x = atomicExch((unsigned long long *)&pk[s], 0ull);
		const uint64_t np = x >> PKC_SHIFT, nb = x & PKC_BYTES_MASK;
		atomicAdd((unsigned long long *)&delta[2u * s], np);
		atomicAdd((unsigned long long *)&delta[2u * s + 1u], nb);
	}
}

/* XDP prefilter IPv4 (bpf/bpf_xdp.c:97-121, :158-178) */
__global__ __launch_bounds__(BLOCK) void k_prefilter_v4(cgpu_snapshot s, prefilter_args a)
{
	const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
	for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < a.n; i += stride) {
		const uint32_t f = a.flags[i];
		const uint32_t sa = a.saddr4[i], da = a.daddr4[i];
		uint8_t v;
		if (f == 2u) {
			v = XDP_PASS;
		} else if (f != 0u) {
			v = XDP_DROP;
		} else {
			v = xdp_pass4(s, sa, da) ? XDP_PASS : XDP_DROP;
		}
		a.verdict[i] = v;
	}
}

/*
 * XDP prefilter IPv6, Q packets per lane with the cover lookup advanced
 * stage by stage across them (root, b24, b32, interval node, /64 record,
 * endpoint bucket), so each stage has Q independent gathers in flight per
 * lane: bpf/bpf_xdp.c:132-156 (any deny prefix covers saddr -> XDP_DROP),
 * then check_v6_endpoint :123-130.
 */

/*
 * The /32 interval nodes (tables.h cover6 node32) of Q packets per lane, read
 * cooperatively: each owner lane picks the line of its x's sub-range, the 8
 * lanes of an octet take the octet's 8 lines in turn, lane j loading 16-B
 * unit j, so one load instruction touches one 128-B line per node.  A line is
 * parity-coded, so lane j only counts its 4 slots below x and puts the
 * count's parity in bit o of a word; three DPP xors over the octet leave all
 * 8 parities in every lane and owner lane o keeps bit o.  COVER6_LONG nodes
 * are scanned by their owner.  Every lane of the wave must call this
 * (cross-lane reads).
 */
__device__ __forceinline__ uint32_t octet_xor(uint32_t v)
{
	v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);  /* quad_perm 1,0,3,2 */
	v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);  /* quad_perm 2,3,0,1 */
	v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false); /* row_half_mirror */
	return v;
}

__device__ __forceinline__ uint32_t c6_below4(uint4 q, uint32_t x)
{
	return (q.x < x ? 1u : 0u) + (q.y < x ? 1u : 0u) + (q.z < x ? 1u : 0u) + (q.w < x ? 1u : 0u);
}

template <int Q>
__device__ __forceinline__ void c6_node32_coop(const uint32_t *pool, const uint32_t (&e)[Q], const uint32_t (&x)[Q],
					       uint32_t (&tag)[Q], bool (&hit)[Q])
{
	const int lane = (int)__lane_id();
	const uint32_t j = (uint32_t)lane & 7u;
	const int base = lane & ~7;
	const uint4 *P = reinterpret_cast<const uint4 *>(pool) + j;
#pragma unroll
	for (int u = 0; u < Q; u++) {
		const bool node = tag[u] == COVER6_NODE;
		if (!__any(node))
			continue;
		const uint32_t split = (e[u] >> 27) & 7u;
		const uint32_t sub = split == COVER6_LONG ? 0u : (uint32_t)((uint64_t)x[u] >> (32u - split));
		/* the line to read; 0 (all 0xFFFFFFFF) when none, so the loads
		 * need no branch */
		const uint32_t mine = node && split != COVER6_LONG ? (e[u] & 0x1FFFFFFu) + sub : 0u;
		uint32_t acc = 0;
#pragma unroll
		for (int o = 0; o < 8; o++) {
			const uint32_t lo = __shfl(mine, base | o), xo = __shfl(x[u], base | o);
			acc |= (c6_below4(P[lo * 8u], xo) & 1u) << o;
		}
		acc = octet_xor(acc);
		if (node) {
			uint32_t par = (acc >> j) & 1u;
			if (split == COVER6_LONG) {
				const uint4 *n = reinterpret_cast<const uint4 *>(pool) + (size_t)(e[u] & 0x1FFFFFFu) * 8u;
				const uint32_t nb = n[0].x;
				par = 0;
				for (uint32_t k = 1; k <= (nb + 3) / 4; k++)
					par ^= c6_below4(n[k], x[u]) & 1u;
			}
			par ^= sub ? 0u : (e[u] >> 25) & 1u;
			hit[u] = par != 0u;
			tag[u] = !par && ((e[u] >> 26) & 1u) ? COVER6_DEEP : COVER6_NONE;
		}
	}
}

/* set16_has whose first bucket's keys and tag words are already loaded
 * (tag 0: exact keys); m0 / m1: the first words of the two mask units */
__device__ __forceinline__ bool set16_has_first(const addr_set16 &t, uint4 k0, uint32_t m0, uint4 k1, uint32_t m1,
						uint32_t b, uint4 key)
{
	bool res = false, done = false;
	for (uint32_t p = 0; !done;) {
		if (!(m0 & 1u)) {
			done = true;
		} else if (m0 == 1u && k0.x == key.x && k0.y == key.y && k0.z == key.z && k0.w == key.w) {
			res = done = true;
		} else if (!(m1 & 1u)) {
			done = true;
		} else if (m1 == 1u && k1.x == key.x && k1.y == key.y && k1.z == key.z && k1.w == key.w) {
			res = done = true;
		} else if (++p >= t.max_probe) {
			done = true;
		} else {
			b = (b + 1) & t.bucket_mask;
			const uint4 *bk = reinterpret_cast<const uint4 *>(t.slots) + (size_t)b * 4u;
			k0 = bk[0];
			m0 = bk[1].x;
			k1 = bk[2];
			m1 = bk[3].x;
		}
	}
	return res;
}

/* a u16 LDS entry (tables.h cover6 root16 / b24_16) as a cover6 entry */
__device__ __forceinline__ uint32_t c6_from16(uint32_t r)
{
	return r >= 2u ? (COVER6_DEEP << 30) | (r - 2u) : (r ? COVER6_FULL << 30 : 0u);
}

/* mode (k_prefilter_v6_q): 0 the root in global memory; 1 lds = root16;
 * 2 lds = rbits then the b24_16 blocks (root and b24 resolved in LDS) */
template <int Q, int mode>
__device__ __forceinline__ void cover6_any_q(const cover6 &t, const uint32_t *lds, const uint4 (&a)[Q],
					     const bool (&act)[Q], bool (&hit)[Q])
{
	uint32_t w0[Q], w1[Q], w2[Q], w3[Q], e[Q], tag[Q];
#pragma unroll
	for (int u = 0; u < Q; u++) {
		w0[u] = bswap32(a[u].x);
		w1[u] = bswap32(a[u].y);
		w2[u] = bswap32(a[u].z);
		w3[u] = bswap32(a[u].w);
		e[u] = 0u;
		if (!act[u] || !t.root)
			continue;
		const uint32_t x = w0[u] >> 16;
		if constexpr (mode == 2) {
			/* root bitmaps and rank, then the /16's b24 block: all LDS */
			const uint32_t deep = lds[x >> 5], full = lds[2048u + (x >> 5)];
			const uint32_t bit = 1u << (x & 31u);
			if (full & bit) {
				e[u] = COVER6_FULL << 30;
			} else if (deep & bit) {
				const uint32_t rank = reinterpret_cast<const uint16_t *>(lds + 4096u)[x >> 5] +
						      __popc(deep & (bit - 1u));
				const uint16_t *b24 = reinterpret_cast<const uint16_t *>(lds + COVER6_RBITS_WORDS);
				e[u] = c6_from16(b24[rank * 256u + ((w0[u] >> 8) & 0xFFu)]);
			}
		} else if constexpr (mode == 1) {
			e[u] = c6_from16(reinterpret_cast<const uint16_t *>(lds)[x]);
		} else {
			e[u] = t.root[x];
		}
	}
	/* the direct-indexed levels: bits 16..23 (unless resolved in LDS), 24..31 */
	if constexpr (mode != 2) {
#pragma unroll
		for (int u = 0; u < Q; u++)
			if ((e[u] >> 30) == COVER6_DEEP)
				e[u] = t.b24[(e[u] & 0x3FFFFFFFu) * 256u + ((w0[u] >> 8) & 0xFFu)];
	}
#pragma unroll
	for (int u = 0; u < Q; u++)
		if ((e[u] >> 30) == COVER6_DEEP)
			e[u] = t.b32[(e[u] & 0x3FFFFFFFu) * 256u + (w0[u] & 0xFFu)];
#pragma unroll
	for (int u = 0; u < Q; u++) {
		tag[u] = e[u] >> 30;
		hit[u] = tag[u] == COVER6_FULL;
	}
#ifndef CGPU_DIAG_PF6_NO_NODE /* timing-only tool build (tools/diag_ab.py): wrong verdicts */
	c6_node32_coop<Q>(t.pool, e, w1, tag, hit);
#endif
	/* /64 records */
	uint4 s0[Q], s1[Q];
	uint32_t home[Q];
#pragma unroll
	for (int u = 0; u < Q; u++) {
		home[u] = mix32(w0[u], w1[u]) & t.m64;
		s0[u] = s1[u] = make_uint4(0, 0, 0, 0);
		if (tag[u] == COVER6_DEEP) {
			s0[u] = t.h64[2u * home[u]];
			s1[u] = t.h64[2u * home[u] + 1u];
		}
	}
#pragma unroll
	for (int u = 0; u < Q; u++) {
		if (tag[u] != COVER6_DEEP)
			continue;
		uint32_t hop = s0[u].w >> POL_HOP_SHIFT;
		bool found = (hop & 1u) && s0[u].x == w0[u] && s0[u].y == w1[u];
		hop &= ~1u;
		while (hop && !found) {
			const uint32_t j = __builtin_ctz(hop);
			hop &= hop - 1u;
			const uint32_t k = (home[u] + j) & t.m64;
			const uint4 x = t.h64[2u * k];
			if (x.x == w0[u] && x.y == w1[u]) {
				s0[u] = x;
				s1[u] = t.h64[2u * k + 1u];
				found = true;
			}
		}
		if (found) {
			const uint32_t tg = s0[u].z >> 30;
			if (tg == COVER6_FULL)
				hit[u] = le64(s1[u].x, s1[u].y, w2[u], w3[u]) && le64(w2[u], w3[u], s1[u].z, s1[u].w);
			else if (tg == COVER6_NODE)
				hit[u] = c6_node64(t.pool, s0[u].z & 0x3FFFFFFFu, w2[u], w3[u]);
		}
	}
}

#ifdef CGPU_DIAG_PF6_PREFETCH /* timing-only tool build (tools/diag_ab.py) */
#define PF6_PREFETCH true
#else
#define PF6_PREFETCH false /* measured slower: the extra registers spill (r2) */
#endif
#ifdef CGPU_DIAG_PF6_Q /* timing-only tool build: packets per lane */
#define PF6_Q CGPU_DIAG_PF6_Q
#else
#define PF6_Q 3 /* 3 > 4 > 2 measured (r2, config 3) */
#endif

/* Q packets per lane; mode: the LDS staging of the cover's top levels
 * (cover6_any_q).  The /32 node reads are octet-cooperative
 * (c6_node32_coop), so the loop trip count is uniform per wave; lanes past
 * the batch end carry inactive packets. */
template <int Q, int NT, int mode>
__global__ __launch_bounds__(NT) void k_prefilter_v6_q(cgpu_snapshot s, prefilter_args a)
{
	const uint4 *sa16 = reinterpret_cast<const uint4 *>(a.saddr16);
	const uint4 *da16 = reinterpret_cast<const uint4 *>(a.daddr16);
	/* LDS: the endpoint bloom filter, then the cover's staged levels (mode) */
	extern __shared__ __attribute__((aligned(16))) uint32_t lbloom[];
	uint32_t *lc = lbloom + s.ep6_bloom_mask + 1u; /* 16-B aligned: >= 64 words */
	for (uint32_t k = threadIdx.x; k <= s.ep6_bloom_mask; k += NT)
		lbloom[k] = s.ep6_bloom[k];
	if constexpr (mode == 1) {
		for (uint32_t k = threadIdx.x; k < 65536u * 2u / 16u; k += NT)
			reinterpret_cast<uint4 *>(lc)[k] = reinterpret_cast<const uint4 *>(s.pf6.root16)[k];
	} else if constexpr (mode == 2) {
		for (uint32_t k = threadIdx.x; k < COVER6_RBITS_WORDS / 4u; k += NT)
			reinterpret_cast<uint4 *>(lc)[k] = reinterpret_cast<const uint4 *>(s.pf6.rbits)[k];
		for (uint32_t k = threadIdx.x; k < s.pf6.n_b24 * 256u * 2u / 16u; k += NT)
			reinterpret_cast<uint4 *>(lc + COVER6_RBITS_WORDS)[k] =
				reinterpret_cast<const uint4 *>(s.pf6.b24_16)[k];
	}
	__syncthreads();
	const uint64_t T = (uint64_t)gridDim.x * NT;
	const uint64_t lane = threadIdx.x & 63u;
	/* wave-step g covers packets [g * Q, g * Q + 64 Q): packet u of a lane
	 * is g * Q + 64 u + lane, so each column load of a wave reads 64
	 * consecutive packets (1 KiB of addresses, 64 B of flags) */
	/* PF6_PREFETCH: the source addresses and flags of the wave's next step
	 * are loaded while this one resolves */
	uint4 nsa[Q];
	uint32_t nf[Q];
	auto load_src = [&](uint64_t g, uint4 (&sa)[Q], uint32_t (&f)[Q]) {
#pragma unroll
		for (int u = 0; u < Q; u++) {
			const uint64_t i = std::min<uint64_t>(g * Q + 64u * u + lane, a.n - 1);
			const v4u_t x = __builtin_nontemporal_load(reinterpret_cast<const v4u_t *>(sa16 + i));
			sa[u] = make_uint4(x.x, x.y, x.z, x.w);
			f[u] = a.flags[i];
		}
	};
	const uint64_t g0 = (uint64_t)blockIdx.x * NT + threadIdx.x - lane;
	if (PF6_PREFETCH && g0 * Q < a.n)
		load_src(g0, nsa, nf);
	for (uint64_t g = g0; g * Q < a.n; g += T) {
		uint4 sa[Q], da[Q];
		uint32_t f[Q];
		uint64_t ix[Q];
		bool act[Q], hit[Q];
		if (PF6_PREFETCH) {
#pragma unroll
			for (int u = 0; u < Q; u++) {
				sa[u] = nsa[u];
				f[u] = nf[u];
			}
			if ((g + T) * Q < a.n)
				load_src(g + T, nsa, nf);
		} else {
			load_src(g, sa, f);
		}
#pragma unroll
		for (int u = 0; u < Q; u++)
			ix[u] = g * Q + 64u * u + lane;
#pragma unroll
		for (int u = 0; u < Q; u++) {
			const uint64_t i = ix[u] < a.n ? ix[u] : a.n - 1;
			const v4u_t y = __builtin_nontemporal_load(reinterpret_cast<const v4u_t *>(da16 + i));
			da[u] = make_uint4(y.x, y.y, y.z, y.w);
			act[u] = ix[u] < a.n && f[u] == 0u && s.pf6_enabled;
#ifdef CGPU_DIAG_PF6_NO_COVER /* timing-only tool build: wrong verdicts */
			act[u] = false;
#endif
		}
		cover6_any_q<Q, mode>(s.pf6, lc, sa, act, hit);
		/* check_v6_endpoint: cilium_lxc on daddr; the LDS bloom filter
		 * settles most misses, the rest load their first bucket together */
		uint4 k0[Q], k1[Q];
		uint32_t m0[Q], m1[Q], b[Q];
		bool need[Q];
#pragma unroll
		for (int u = 0; u < Q; u++) {
			const uint32_t h = pfx6_hash(da[u].x, da[u].y, da[u].z, da[u].w, 0u);
			const uint32_t bits = v6_bloom_bits(h);
			b[u] = h & s.ep6.bucket_mask;
			need[u] = ix[u] < a.n && f[u] == 0u && !hit[u] &&
				  (lbloom[v6_bloom_word(h, s.ep6_bloom_mask)] & bits) == bits;
#ifdef CGPU_DIAG_PF6_NO_EP /* timing-only tool build: wrong verdicts */
			need[u] = false;
#endif
			const uint4 *p = reinterpret_cast<const uint4 *>(s.ep6.slots) + (size_t)b[u] * 4u;
			const uint32_t *pw = reinterpret_cast<const uint32_t *>(p);
			k0[u] = need[u] ? p[0] : make_uint4(0, 0, 0, 0);
			m0[u] = need[u] ? pw[4] : 0u;
			k1[u] = need[u] ? p[2] : make_uint4(0, 0, 0, 0);
			m1[u] = need[u] ? pw[12] : 0u;
		}
#pragma unroll
		for (int u = 0; u < Q; u++) {
			if (ix[u] >= a.n)
				continue;
			uint8_t v;
			if (f[u] == 2u) {
				v = XDP_PASS;
			} else if (f[u] != 0u || hit[u] || !need[u]) {
				v = XDP_DROP;
			} else {
				v = set16_has_first(s.ep6, k0[u], m0[u], k1[u], m1[u], b[u], da[u]) ? XDP_PASS : XDP_DROP;
			}
			a.verdict[ix[u]] = v;
		}
	}
}

__global__ void k_fold(uint64_t *totals, uint64_t *delta, uint64_t n)
{
	for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
	     i += (uint64_t)gridDim.x * blockDim.x) {
		uint64_t d = delta[i];
		if (d) {
			totals[i] += d;
			delta[i] = 0;
		}
	}
}

__global__ void k_slot_init(uint64_t *totals, uint64_t *delta, const uint32_t *slot,
			    const uint64_t *pk, const uint64_t *by, uint32_t n)
{
	uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i < n) {
		uint32_t sl = slot[i];
		totals[2u * sl] = pk[i];
		totals[2u * sl + 1u] = by[i];
		delta[2u * sl] = 0;
		delta[2u * sl + 1u] = 0;
	}
}

/* device side of the table verification sum (tables.h table_sum_word) over
 * one part: `bytes` bytes from word w0 of the buffer (a trailing partial
 * word counts its bytes only) */
__global__ __launch_bounds__(256) void k_table_sum(const uint64_t *buf, uint64_t w0, uint64_t bytes, uint64_t *out)
{
	uint64_t acc = 0;
	const uint64_t nw = (bytes + 7u) / 8u;
	const uint64_t stride = (uint64_t)gridDim.x * 256u;
	for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < nw; i += stride) {
		uint64_t w = __builtin_nontemporal_load(buf + w0 + i);
		const uint64_t rem = bytes - 8u * i;
		if (rem < 8u)
			w &= (1ull << (8u * rem)) - 1ull;
		acc += table_sum_word(w, w0 + i);
	}
	acc = wave_sum(acc);
	if ((threadIdx.x & 63) == 0 && acc)
		atomicAdd((unsigned long long *)out, (unsigned long long)acc);
}

unsigned grid_for(uint64_t n)
{
	uint64_t blocks = (n + BLOCK - 1) / BLOCK;
	/* 256 CUs x 8 resident 256-thread blocks; grid-stride beyond that */
	const uint64_t cap = 256ull * 8ull;
	return (unsigned)(blocks < cap ? (blocks ? blocks : 1) : cap);
}

} // namespace

/* k_classify_x4 reads columns as 4/8/16-byte vectors at tuple index
 * multiples of 4: the column base pointers must be aligned to match. */
static bool x4_aligned(const cls_args &a)
{
	const uintptr_t a16 = (uintptr_t)a.saddr | (uintptr_t)a.daddr | (uintptr_t)a.len |
			      (uintptr_t)a.verdict | (uintptr_t)a.identity | (uintptr_t)a.hash;
	const uintptr_t a8 = (uintptr_t)a.dport | (uintptr_t)a.ep | (uintptr_t)a.sport;
	const uintptr_t a4 = (uintptr_t)a.proto | (uintptr_t)a.flags | (uintptr_t)a.stage;
	return !(a16 & 15) && !(a8 & 7) && !(a4 & 3);
}

/* Workgroups of NT threads of kernel `kern` that stay resident on the
 * current device with `lds` bytes of dynamic LDS (CUs x occupancy); cached
 * per (device, kernel, lds). */
static unsigned resident_blocks(const void *kern, int NT, size_t lds)
{
	static std::mutex mu;
	static std::map<std::tuple<int, const void *, size_t>, unsigned> cache;
	int dev = 0;
	(void)hipGetDevice(&dev);
	std::lock_guard<std::mutex> g(mu);
	auto key = std::make_tuple(dev, kern, lds);
	auto it = cache.find(key);
	if (it != cache.end())
		return it->second;
	int cus = 0, per_cu = 0;
	if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
		cus = 256;
	if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, NT, lds) != hipSuccess || per_cu <= 0)
		per_cu = 1;
	const unsigned r = (unsigned)(cus * per_cu);
	cache[key] = r;
	return r;
}

/* x4 schedule: one persistent-size grid (every workgroup resident, so the
 * per-workgroup LDS counter flush is paid once per resident workgroup) per
 * launch of <= PKC_CHUNK tuples, then the unpack of pk into delta. */
/* dynamic LDS of a k_classify_x4 workgroup: 160 KiB per CU less the static
 * metrics block and some slack */
#define X4_LDS_BUDGET (156u * 1024u)

/* cold-slot cache entries (12 B each: packed count + tag) in the LDS left
 * under X4_LDS_BUDGET by `used` bytes: a multiple of 64, at most 16384,
 * none below 512 (any count: the probe start is a multiply-high of the slot
 * hash, the probe wraps at the end) */
static uint32_t cc_entries(size_t used)
{
	if (used >= X4_LDS_BUDGET)
		return 0u;
	const size_t n = std::min<size_t>((X4_LDS_BUDGET - used) / 12u, 16384u) & ~(size_t)63u;
	return n >= 512u ? (uint32_t)n : 0u;
}

/* The snapshot a launch sees with at most `max_hot` LDS counter slots: hits
 * on slots past it take the kernels' cold path (the counts are the same,
 * only where they accumulate changes), so LDS never overflows whatever
 * hot_counter_slots is. */
static cgpu_snapshot with_lds_hot(const cgpu_snapshot &s, size_t max_hot)
{
	cgpu_snapshot r = s;
	r.hot_slots = (uint32_t)std::min<size_t>(s.hot_slots, max_hot);
	return r;
}

/* cgpu_classify_v6's ipcache pass on the x4 schedule: every tuple's
 * looked-up address (daddr egress, saddr ingress, bpf_lxc.c:170-187 /
 * bpf_netdev.c:203-211) through the trie (v6t_lookup_q), its DIR entry to
 * e[i].  Kept out of k_classify_x4 so that the trie walk's dependent loads
 * run at this kernel's occupancy (few registers, no counter LDS) instead of
 * the classify kernel's; the classify kernel then reads 4 bytes per tuple
 * instead of the address.  Lane-interleaved: load instruction u of a wave
 * covers 64 consecutive tuples. */
#ifndef CGPU_IPC6_MINW
#define CGPU_IPC6_MINW 1 /* workgroups per CU the register budget aims at */
#endif
#ifndef CGPU_IPC6_SPEC
#define CGPU_IPC6_SPEC 1 /* addresses loaded beside the direction flag (0: behind it) */
#endif
/* svc_out[i].x: SVC_* | LBS_* << 8 | slave << 16; .y target; .z the dport
 * rewrite (0 none) | rev_nat_index << 16 */
#define SVC_NONE 0u
#define SVC_XLATED 1u
#define SVC_DROP 2u

template <int Q, int NT>
__global__ __launch_bounds__(NT, CGPU_IPC6_MINW) void k_ipc6_pre(cgpu_snapshot s, const uint4 *sa, const uint4 *da,
						 const uint8_t *flags, uint32_t *e_out, uint64_t n,
						 const uint4 *svc)
{
	/* svc (the IPv6 service path, or NULL): an egress packet lb6_local
	 * translated is looked up on its target (svc[2i + 1]) */
	extern __shared__ __attribute__((aligned(16))) uint32_t lt[];
	const uint32_t n24 = v6t_lds_b24(s.ipc6);
	const uint32_t nbl = v6t_lds_bloom(s.ipc6);
	uint32_t *lbl = lt + v6t_lds_words(s.ipc6);
	if (s.ipc6.root) {
		for (uint32_t k = threadIdx.x; k < V6T_RBITS_WORDS; k += NT)
			lt[k] = s.ipc6.rbits[k];
		const uint32_t *b16 = reinterpret_cast<const uint32_t *>(s.ipc6.b24_16);
		for (uint32_t k = threadIdx.x; k < n24 * 128u; k += NT)
			lt[V6T_RBITS_WORDS + k] = b16[k];
		for (uint32_t k = threadIdx.x; k < nbl; k += NT)
			lbl[k] = s.ipc6.bl64[k];
	}
	__syncthreads();
	const uint64_t T = (uint64_t)gridDim.x * NT;
	for (uint64_t g = (uint64_t)blockIdx.x * NT + threadIdx.x; g < n; g += T * Q) {
		uint4 w[Q];
		bool act[Q], eg[Q];
		uint32_t e[Q];
#if CGPU_IPC6_SPEC
		/* both addresses (and the service outcome) are loaded with the
		 * direction flag, not behind it: one round trip less per tuple for
		 * 16 more bytes of stream (k_ipc6_pre 1.62 ms, round 5) */
		uint4 xs[Q], xd[Q], so[Q], st[Q];
#pragma unroll
		for (int u = 0; u < Q; u++) {
			const uint64_t i = g + (uint64_t)u * T;
			act[u] = i < n;
			const uint64_t j = act[u] ? i : 0u;
			eg[u] = flags[j] & 1u;
			xs[u] = ld_x4<true>(sa + j);
			xd[u] = ld_x4<true>(da + j);
			if (svc) {
				so[u] = svc[2u * j];
				st[u] = svc[2u * j + 1u];
			}
		}
#pragma unroll
		for (int u = 0; u < Q; u++) {
			uint4 x = eg[u] ? xd[u] : xs[u];
			if (svc && eg[u] && (so[u].x & 3u) == SVC_XLATED)
				x = st[u];
			w[u] = act[u] ? v6_host_words(x) : make_uint4(0, 0, 0, 0);
		}
#else
#pragma unroll
		for (int u = 0; u < Q; u++) {
			const uint64_t i = g + (uint64_t)u * T;
			act[u] = i < n;
			w[u] = make_uint4(0, 0, 0, 0);
			eg[u] = false;
			if (act[u]) {
				eg[u] = flags[i] & 1u;
				uint4 x = ld_x4<true>((eg[u] ? da : sa) + i);
				if (svc && eg[u] && (svc[2u * i].x & 3u) == SVC_XLATED)
					x = svc[2u * i + 1u];
				w[u] = v6_host_words(x);
			}
		}
#endif
		v6t_lookup_q<Q>(s.ipc6, lt, n24 != 0u, w, act, e, nbl ? lbl : nullptr);
#pragma unroll
		for (int u = 0; u < Q; u++) {
			const uint64_t i = g + (uint64_t)u * T;
			if (!act[u])
				continue;
			/* the classify kernel reads no address: an egress tuple's
			 * fallback identity (no match or a label-0 match) is folded in
			 * here, as a DIRECT entry of cluster_id when the address lies in
			 * ROUTER_IP's /64 (ipv6_match_prefix_64, bpf/lib/ipv6.h:166-175;
			 * bpf_lxc.c:170-187), else no match (WORLD_ID) */
			uint32_t ev = e[u];
			if (eg[u] && !(ev && entry_label(s.ipc6.vals, ev))) {
				const bool in_cluster = w[u].x == bswap32(s.router_ip64[0]) &&
							w[u].y == bswap32(s.router_ip64[1]);
				ev = in_cluster ? (DIR_TAG_DIRECT | s.cluster_id) : 0u;
			}
			e_out[i] = ev;
		}
	}
}

#ifndef CGPU_DIAG_IPC6_PRE_Q
#define CGPU_DIAG_IPC6_PRE_Q 2
#endif

static hipError_t launch_ipc6_pre(const cgpu_snapshot &s, const cls_args &a, hipStream_t st)
{
	constexpr int NT = 1024, Q = CGPU_DIAG_IPC6_PRE_Q;
	const size_t lds = (size_t)(v6t_lds_words(s.ipc6) + v6t_lds_bloom(s.ipc6)) * 4u;
	const unsigned res = resident_blocks((const void *)k_ipc6_pre<Q, NT>, NT, lds);
	const unsigned g = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((a.n + Q * NT - 1) / (Q * NT), res));
	hipLaunchKernelGGL((k_ipc6_pre<Q, NT>), dim3(g), dim3(NT), lds, st, s, static_cast<const uint4 *>(a.saddr),
			   static_cast<const uint4 *>(a.daddr), a.flags, a.ipc_e, a.n, nullptr);
	return hipGetLastError();
}

/* tuples per lane of the config-5 cascade kernel: 2 (its service step and
 * prefilter share stages; at 4 the kernel spilled 19 VGPRs with the stages
 * apart and 101 with them shared): 3.18 -> 3.02 ms per 64M tuples, of which
 * sharing the stages 0.015 (profiles/r6_l/) */
#ifndef CGPU_XDP_Q
#define CGPU_XDP_Q 2
#endif
template <bool LB, bool V6, int FR = 0, bool IPCE = false, bool XDP = false>
static hipError_t launch_x4(const cgpu_snapshot &s0, const cls_args &a, hipStream_t st,
			    const frames_x4 &fx = frames_x4{})
{
	constexpr bool FF = FR == 2;
	constexpr int NT = 1024;
	if constexpr (IPCE) {
		hipError_t e = launch_ipc6_pre(s0, a, st);
		if (e != hipSuccess)
			return e;
	}
	/* LDS: hot counters + the ipcache leaf dictionary (v4) / the staged trie
	 * levels (v6 without the pre-pass) */
	size_t fixed = V6 ? (IPCE ? 0u : (size_t)v6t_lds_words(s0.ipc6) * 4u) : (size_t)s0.ipc4c.n_dict * 4u;
	fixed = (fixed + 7u) & ~(size_t)7u;
	/* fused frames: the endpoint rows (+ alignment) and 4 statuses per lane */
	const size_t ff = FF ? 16u + 2u * FR_LXC_LDS * 16u + (size_t)NT * 4u * 2u +
				       (CGPU_FF_STAGE ? (size_t)(CGPU_FF_POOL ? CGPU_FF_POOL : NT / 64) * FF_STG_U4 * 16u + 64u
						      : 0u)
			     : 0u;
	fixed += ff;
	const cgpu_snapshot s = with_lds_hot(s0, fixed < X4_LDS_BUDGET ? (X4_LDS_BUDGET - fixed) / 8u : 0u);
	size_t lds = (size_t)s.hot_slots * 8u + fixed;
	/* the cold-slot cache takes the LDS one workgroup per CU leaves free
	 * (the resident grid runs one 1024-thread workgroup per CU) */
	const uint32_t cc_n = (s.schedule & CGPU_SCHED_NO_CCACHE) ? 0u : cc_entries(lds);
	lds += (size_t)cc_n * 12u;
#ifdef CGPU_DIAG_LDS_PAD /* timing-only: fewer resident workgroups per CU */
	lds += CGPU_DIAG_LDS_PAD;
#endif
#ifdef CGPU_DIAG_V6_Q /* timing-only tool build (tools/diag_ab.py): v6 tuples per lane */
	constexpr int Q = V6 && !IPCE ? CGPU_DIAG_V6_Q : 4;
#else
	constexpr int Q = V6 && !IPCE ? 2 : XDP ? CGPU_XDP_Q : 4; /* in-kernel v6 lookups: the trie's line registers */
#endif
	const void *kern = (const void *)k_classify_x4<NT, true, Q, 1, LB, V6, FR, IPCE, XDP>;
	static_assert(!FF || Q == 4, "fused frames: Q = 4");
	const unsigned res = resident_blocks(kern, NT, lds);
	/* LDS packed counters: <= 2^22 tuples per workgroup (PK_SHIFT) */
	const uint64_t chunk = std::min<uint64_t>(PKC_CHUNK, (uint64_t)res << 22);
	for (uint64_t off = 0; off < a.n; off += chunk) {
		cls_args c = a;
		c.cc_n = cc_n;
		const uint64_t m = std::min<uint64_t>(a.n - off, chunk);
		c.n = m;
		c.verdict += off;
		c.identity += off;
		if (c.stage)
			c.stage += off;
		c.flags += off;
		c.len += off;
		c.ep += off;
		if (FF) { /* a.saddr = the 64-byte frame slots */
			c.saddr = static_cast<const char *>(a.saddr) + off * 64u;
		} else {
			c.dport += off;
			c.proto += off;
			c.saddr = static_cast<const char *>(a.saddr) + off * (V6 ? 16 : 4);
			c.daddr = static_cast<const char *>(a.daddr) + off * (V6 ? 16 : 4);
		}
		if (c.sport)
			c.sport += off;
		if (c.hash)
			c.hash += off;
		if (c.ipc_e)
			c.ipc_e += off;
		c.n_off = off;
		const unsigned g = (unsigned)std::min<uint64_t>((m + Q * NT - 1) / (Q * NT), res);
		hipLaunchKernelGGL((k_classify_x4<NT, true, Q, 1, LB, V6, FR, IPCE, XDP>), dim3(g), dim3(NT), lds, st, s, c,
				   a.pk, fx);
		if (s.cold_hi) {
			const unsigned ug = std::min<unsigned>((s.cold_hi + 255) / 256, 1024);
			hipLaunchKernelGGL(k_unpack, dim3(ug), dim3(256), 0, st, a.delta, a.pk, 0u, s.cold_hi);
		}
	}
	return hipGetLastError();
}

/* The context's cgpu_config.schedule selects the schedule (every schedule
 * computes the reference's results, tests/test_gpu_parity.py):
 *   default: k_classify_x4 -- four tuples per lane, vector column loads, LDS
 *      hot counters + one packed atomic per cold hit, resident grid (needs
 *      aligned columns, else the per-lane kernel)
 *   CGPU_SCHED_PER_LANE: one tuple per lane, LDS hot counters
 *   CGPU_SCHED_GLOBAL_CTR: global atomics for every hit, 256-thread workgroups */
template <int V6>
static hipError_t launch_classify(const cgpu_snapshot &s0, cls_args a, hipStream_t st)
{
	if (s0.schedule & CGPU_SCHED_GLOBAL_CTR) {
		hipLaunchKernelGGL((k_classify<V6, 0, BLOCK>), dim3(grid_for(a.n)), dim3(BLOCK), 0, st, s0, a);
		return hipGetLastError();
	}
	if (!(s0.schedule & CGPU_SCHED_PER_LANE) && a.pk && x4_aligned(a)) {
		if (V6)
			return a.lb ? launch_x4<true, true>(s0, a, st)
				    : (a.ipc_e ? launch_x4<false, true, false, true>(s0, a, st) : launch_x4<false, true>(s0, a, st));
		if (a.lb)
			return a.xdp ? launch_x4<true, false, 0, false, true>(s0, a, st) : launch_x4<true, false>(s0, a, st);
		return launch_x4<false, false>(s0, a, st);
	}
	/* LDS counters: 1024-thread workgroups, <= 2 per CU (LDS), and at most
	 * 2^22 tuples per workgroup (packed-counter exactness) */
	constexpr int NT = 1024;
	const cgpu_snapshot s = with_lds_hot(s0, X4_LDS_BUDGET / 8u);
	const size_t lds = (size_t)s.hot_slots * 8u;
	const uint64_t cap = 2ull * 256ull;
	const uint64_t per_launch = cap * (1ull << 22); /* k_classify<.., 1, ..> never touches pk */
	for (uint64_t off = 0; off < a.n; off += per_launch) {
		cls_args c = a;
		const uint64_t m = std::min<uint64_t>(a.n - off, per_launch);
		c.n = m;
		c.verdict += off;
		c.identity += off;
		if (c.stage)
			c.stage += off;
		c.dport += off;
		c.proto += off;
		c.flags += off;
		c.len += off;
		c.ep += off;
		c.saddr = static_cast<const char *>(a.saddr) + off * (V6 ? 16 : 4);
		c.daddr = static_cast<const char *>(a.daddr) + off * (V6 ? 16 : 4);
		if (c.sport)
			c.sport += off;
		if (c.hash)
			c.hash += off;
		const unsigned g = (unsigned)std::min<uint64_t>((m + NT - 1) / NT, cap);
		hipLaunchKernelGGL((k_classify<V6, 1, NT>), dim3(g), dim3(NT), lds, st, s, c);
	}
	return hipGetLastError();
}

hipError_t launch_classify_v4(const cgpu_snapshot &s, const classify_v4_args &x, hipStream_t st)
{
	cls_args c{x.saddr, x.daddr, x.dport, x.proto, x.flags, x.len, x.ep, x.verdict, x.identity,
		   x.stage, x.delta, x.n, x.pk, x.lb, x.sport, x.hash};
	c.xdp = x.lb ? x.xdp : 0;
	return launch_classify<0>(s, c, st);
}

hipError_t launch_classify_v6(const cgpu_snapshot &s, const classify_v6_args &x, hipStream_t st)
{
	cls_args c{x.saddr16, x.daddr16, x.dport, x.proto, x.flags, x.len, x.ep, x.verdict, x.identity,
		   x.stage, x.delta, x.n, x.pk, x.lb, x.sport, x.hash};
	c.ipc_e = x.ipc_e;
	return launch_classify<1>(s, c, st);
}

hipError_t launch_lb4(const cgpu_snapshot &s, const lb4_args &a, hipStream_t st)
{
	if (a.mode == CGPU_LB_NETDEV)
		hipLaunchKernelGGL(k_lb4<CGPU_LB_NETDEV>, dim3(grid_for(a.n)), dim3(BLOCK), 0, st, s, a);
	else
		hipLaunchKernelGGL(k_lb4<CGPU_LB_LXC>, dim3(grid_for(a.n)), dim3(BLOCK), 0, st, s, a);
	return hipGetLastError();
}

hipError_t launch_prefilter_v4(const cgpu_snapshot &s, const prefilter_args &a, hipStream_t st)
{
	hipLaunchKernelGGL(k_prefilter_v4, dim3(grid_for(a.n)), dim3(BLOCK), 0, st, s, a);
	return hipGetLastError();
}

hipError_t launch_prefilter_v6(const cgpu_snapshot &s, const prefilter_args &a, hipStream_t st)
{
	/* four packets per lane, octet-cooperative node reads, a resident grid
	 * of 1024-thread workgroups (the LDS root is loaded once per
	 * workgroup).  A/B on config 3 (Gpps, round 1): Q=4 coop 24.8; Q=4
	 * per-lane nodes 21.1; Q=4 fitted to 5 waves/SIMD 20.4; Q=2 20.9. */
	constexpr int NT = 1024;
	constexpr size_t LDS_MAX = 160u * 1024u;
	/* stage the deepest cover levels that fit next to the bloom filter */
	const size_t bloom = (size_t)(s.ep6_bloom_mask + 1u) * 4u;
	const size_t l2 = (size_t)COVER6_RBITS_WORDS * 4u + (size_t)s.pf6.n_b24 * 512u;
	/* CGPU_SCHED_PF6_LDS caps the mode (every mode computes the same
	 * verdicts; tests/test_gpu_parity.py runs each) */
	const uint32_t cap = (s.schedule >> 4) & 3u;
	const int max_mode = cap ? (int)cap - 1 : 2;
	int mode = 0;
	size_t lds = bloom;
	if (max_mode >= 2 && s.pf6.rbits && bloom + l2 <= LDS_MAX) {
		mode = 2;
		lds += l2;
	} else if (max_mode >= 1 && s.pf6.root16 && bloom + 65536u * 2u <= LDS_MAX) {
		mode = 1;
		lds += 65536u * 2u;
	}
	const void *kern = mode == 2 ? (const void *)k_prefilter_v6_q<PF6_Q, NT, 2>
			   : mode == 1 ? (const void *)k_prefilter_v6_q<PF6_Q, NT, 1> : (const void *)k_prefilter_v6_q<PF6_Q, NT, 0>;
	const unsigned res = resident_blocks(kern, NT, lds);
	const unsigned g = (unsigned)std::min<uint64_t>((a.n + PF6_Q * NT - 1) / (PF6_Q * NT), res);
	if (mode == 2)
		hipLaunchKernelGGL((k_prefilter_v6_q<PF6_Q, NT, 2>), dim3(g ? g : 1), dim3(NT), lds, st, s, a);
	else if (mode == 1)
		hipLaunchKernelGGL((k_prefilter_v6_q<PF6_Q, NT, 1>), dim3(g ? g : 1), dim3(NT), lds, st, s, a);
	else
		hipLaunchKernelGGL((k_prefilter_v6_q<PF6_Q, NT, 0>), dim3(g ? g : 1), dim3(NT), lds, st, s, a);
	return hipGetLastError();
}

hipError_t launch_frames_parse(const cgpu_snapshot &s, const frames_args &a, hipStream_t st)
{
	hipLaunchKernelGGL((k_frames<0, BLOCK>), dim3(grid_for(a.n)), dim3(BLOCK), 0, st, s, a);
	return hipGetLastError();
}

/* frames -> the x4 schedule: the header parse writes policy-tuple columns
 * (IPv4 frames in place, frames the parse ended flagged FRF_DEC with their
 * status, IPv6 frames compacted to their own columns with their index),
 * then k_classify_x4 runs over the IPv4 columns and, on the device-side
 * count, over the IPv6 ones, whose results are scattered back */

/* one tile of 64 frames in 64-byte slots: the wave's four coalesced 1-KiB
 * loads (lane l holds bytes [1024 k + 16 l, +16) of the tile) and the
 * lane's own len / flags / ep */
struct fr_tile {
	uint4 v[4];
	uint32_t len, fl, ep;
};

__device__ __forceinline__ void fr_fetch(const frames_args &a, uint64_t i0, uint32_t lane, fr_tile &t)
{
	const uint64_t i = i0 + lane;
	const uint64_t bytes = i0 < a.n ? min((uint64_t)64, a.n - i0) * 64u : 0u;
	const uint8_t *base = a.data + i0 * 64u;
#pragma unroll
	for (int k = 0; k < 4; k++) {
		const uint32_t off = 1024u * k + 16u * lane;
		t.v[k] = off < bytes ? ld_x4<true>(base + off) : make_uint4(0, 0, 0, 0);
	}
	const bool valid = i < a.n;
	t.len = valid ? a.len[i] : 0u;
	t.fl = valid ? a.flags[i] : 0u;
	t.ep = valid ? a.ep[i] : 0u;
}

/* frame i's policy-tuple columns (or its FRF_DEC status / its compacted
 * IPv6 row) from its parse */
__device__ __forceinline__ void fr_emit(const cgpu_snapshot &s, const frames_args &a, const frames_x4 &c,
					const uint4 *lxc, const fwin &W, uint64_t i, uint32_t len, uint32_t flv,
					uint32_t ep)
{
	const bool valid = i < a.n;
	const bool egress = valid && (flv & 1u);
	const ftuple t = parse_frame_w(s, W, a.data + i * (uint64_t)a.stride, len, min(len, a.stride), egress, ep, lxc);
	uint32_t fl = egress ? 1u : 0u, sa = 0, da = 0, dp = 0, pr = 0;
	const bool v6 = t.status == 0 && t.fam != 4u;
	if (t.status != 0) {
		fl |= FRF_DEC;
		da = (uint32_t)t.status;
	} else if (!v6) {
		sa = t.sa.x;
		da = t.da.x;
		dp = t.dport;
		pr = t.proto;
		fl |= t.frag ? 2u : 0u;
	} else {
		fl |= FRF_V6;
	}
	/* wave-aggregated slot of the IPv6 frames */
	const uint64_t m = __ballot(valid && v6);
	if (m) {
		const int leader = __ffsll((unsigned long long)m) - 1;
		uint32_t base = 0;
		if ((int)__lane_id() == leader)
			base = atomicAdd(c.n6, (uint32_t)__popcll(m));
		base = __shfl(base, leader, 64);
		if (valid && v6) {
			const uint32_t j = base + (uint32_t)__popcll(m & ((1ull << __lane_id()) - 1ull));
			c.sa6[j] = t.sa;
			c.da6[j] = t.da;
			c.dport6[j] = (uint16_t)t.dport;
			c.proto6[j] = (uint8_t)t.proto;
			c.fl6[j] = (uint8_t)(egress ? 1u : 0u);
			c.len6[j] = len;
			c.ep6[j] = (uint16_t)ep;
			c.idx6[j] = (uint32_t)i;
		}
	}
	if (!valid)
		return;
	c.sa4[i] = sa;
	c.da4[i] = da;
	c.dport[i] = (uint16_t)dp;
	c.proto[i] = (uint8_t)pr;
	c.fl[i] = (uint8_t)fl;
}

template <bool LXL>
__global__ __launch_bounds__(256) void k_frames_cols(cgpu_snapshot s, frames_args a, frames_x4 c)
{
	/* 64-byte slots: a wave reads its 64 frames as four fully coalesced
	 * 1-KiB loads and hands each lane its frame through LDS (rows of 17
	 * words: conflict-free reads); per-lane 16-byte loads of 64 separate
	 * slots cost one address-unit pass per lane and load.  Software-
	 * pipelined: the next tile's slots and len / flags / ep are in flight
	 * while this tile is parsed, and the endpoint rows come from LDS, so a
	 * tile costs one memory round trip, not three. */
	__shared__ uint32_t stg[4][64 * 17];
	__shared__ uint4 lxl[LXL ? 2u * FR_LXC_LDS : 1u];
	if constexpr (LXL) {
		for (uint32_t k = threadIdx.x; k < 2u * s.n_lxc; k += 256u)
			lxl[k] = s.lxc[k];
		__syncthreads();
	}
	const uint4 *lxc = LXL ? static_cast<const uint4 *>(lxl) : s.lxc;
	const uint32_t wv = threadIdx.x >> 6, lane = __lane_id();
	const uint64_t stride = (uint64_t)gridDim.x * 256u;
	uint64_t i0 = (uint64_t)blockIdx.x * 256u + wv * 64u;
	if (a.stride == 64u) {
		fr_tile cur;
		fr_fetch(a, i0, lane, cur);
		for (; i0 < a.n; i0 += stride) {
			fr_tile nxt;
			fr_fetch(a, i0 + stride, lane, nxt);
#pragma unroll
			for (int k = 0; k < 4; k++) {
				const uint32_t off = 1024u * k + 16u * lane;
				uint32_t *d = &stg[wv][(off >> 6) * 17u + ((off & 63u) >> 2)];
				d[0] = cur.v[k].x;
				d[1] = cur.v[k].y;
				d[2] = cur.v[k].z;
				d[3] = cur.v[k].w;
			}
			__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
			__builtin_amdgcn_wave_barrier();
			__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
			fwin W;
#pragma unroll
			for (int j = 0; j < 16; j++)
				W.w[j] = stg[wv][lane * 17u + j];
			__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
			__builtin_amdgcn_wave_barrier();
			__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
			fr_emit(s, a, c, lxc, W, i0 + lane, cur.len, cur.fl, cur.ep);
			cur = nxt;
		}
		return;
	}
	for (; i0 < a.n; i0 += stride) {
		const uint64_t i = i0 + lane;
		const bool valid = i < a.n;
		fwin W;
		if (valid) {
			const uint8_t *f = a.data + i * (uint64_t)a.stride;
#pragma unroll
			for (int k = 0; k < 4; k++) {
				const uint4 v = ld_x4<true>(f + 16 * k);
				W.w[4 * k] = v.x;
				W.w[4 * k + 1] = v.y;
				W.w[4 * k + 2] = v.z;
				W.w[4 * k + 3] = v.w;
			}
		}
		fr_emit(s, a, c, lxc, W, i, valid ? a.len[i] : 0u, valid ? a.flags[i] : 0u, valid ? a.ep[i] : 0u);
	}
}

__global__ __launch_bounds__(256) void k_frames_scatter6(frames_x4 c, int32_t *verdict, uint32_t *identity,
							 uint8_t *stage)
{
	const uint32_t n6 = *c.n6;
	for (uint32_t j = blockIdx.x * 256u + threadIdx.x; j < n6; j += gridDim.x * 256u) {
		const uint32_t i = c.idx6[j];
		verdict[i] = c.v6[j];
		identity[i] = c.id6[j];
		if (stage)
			stage[i] = c.st6[j];
	}
}

static size_t frames_x4_layout(uint64_t n, size_t *off)
{
	/* column element sizes, each column rounded to 256 bytes */
	static const size_t el[17] = {4, 4, 2, 1, 1, 16, 16, 2, 1, 1, 4, 2, 4, 4, 4, 1, 4};
	size_t t = 0;
	for (int k = 0; k < 17; k++) {
		off[k] = t;
		t += ((k == 16 ? 1 : n) * el[k] + 255) & ~(size_t)255;
	}
	return t;
}

size_t frames_x4_bytes(uint64_t n)
{
	size_t off[17];
	return frames_x4_layout(n, off);
}

frames_x4 frames_x4_carve(void *base, uint64_t n)
{
	size_t o[17];
	frames_x4_layout(n, o);
	char *b = static_cast<char *>(base);
	return frames_x4{reinterpret_cast<uint32_t *>(b + o[0]), reinterpret_cast<uint32_t *>(b + o[1]),
			 reinterpret_cast<uint16_t *>(b + o[2]), reinterpret_cast<uint8_t *>(b + o[3]),
			 reinterpret_cast<uint8_t *>(b + o[4]), reinterpret_cast<uint4 *>(b + o[5]),
			 reinterpret_cast<uint4 *>(b + o[6]), reinterpret_cast<uint16_t *>(b + o[7]),
			 reinterpret_cast<uint8_t *>(b + o[8]), reinterpret_cast<uint8_t *>(b + o[9]),
			 reinterpret_cast<uint32_t *>(b + o[10]), reinterpret_cast<uint16_t *>(b + o[11]),
			 reinterpret_cast<uint32_t *>(b + o[12]), reinterpret_cast<int32_t *>(b + o[13]),
			 reinterpret_cast<uint32_t *>(b + o[14]), reinterpret_cast<uint8_t *>(b + o[15]),
			 reinterpret_cast<uint32_t *>(b + o[16])};
}

hipError_t launch_classify_frames_x4(const cgpu_snapshot &s, const frames_args &a, const frames_x4 &c,
				     hipStream_t st)
{
	hipError_t e = hipMemsetAsync(c.n6, 0, 4, st);
	if (e != hipSuccess)
		return e;
	if (a.stride == 64u && s.n_lxc <= FR_LXC_LDS && !((uintptr_t)a.data & 15u) &&
	    !(s.schedule & CGPU_SCHED_FRAMES_SPLIT)) {
		/* fused: the classify kernel parses the slots itself (no tuple
		 * columns written and re-read), the IPv6 frames as below.  Each
		 * wave reads its 64-slot tile as four coalesced 1-KiB loads and
		 * hands the slots out through LDS (CGPU_FF_STAGE): 2.64 against
		 * 2.81 ms per 64M frames for the two passes, 2.96 with per-lane
		 * slot loads (profiles/r5_j/) */
		cls_args f4{a.data, nullptr, nullptr, nullptr, a.flags, a.len, a.ep, a.verdict, a.identity, a.stage,
			    a.delta, a.n, a.pk, 0, nullptr, nullptr};
		if ((e = launch_x4<false, false, 2>(s, f4, st, c)) != hipSuccess)
			return e;
		cls_args c6{c.sa6, c.da6, c.dport6, c.proto6, c.fl6, c.len6, c.ep6, c.v6, c.id6,
			    a.stage ? c.st6 : nullptr, a.delta, a.n, a.pk, 0, nullptr, nullptr};
		c6.n_dev = c.n6;
		if ((e = launch_x4<false, true, 1>(s, c6, st)) != hipSuccess)
			return e;
		hipLaunchKernelGGL(k_frames_scatter6, dim3(grid_for(a.n)), dim3(BLOCK), 0, st, c, a.verdict,
				   a.identity, a.stage);
		return hipGetLastError();
	}
	/* a streaming pass: up to 8 resident 256-thread blocks per CU (25 KiB
	 * LDS each) so enough slot loads are in flight */
	const unsigned gf = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((a.n + BLOCK - 1) / BLOCK, 256u * 8u * 4u));
	if (s.n_lxc <= FR_LXC_LDS)
		hipLaunchKernelGGL(k_frames_cols<true>, dim3(gf), dim3(BLOCK), 0, st, s, a, c);
	else
		hipLaunchKernelGGL(k_frames_cols<false>, dim3(gf), dim3(BLOCK), 0, st, s, a, c);
	cls_args c4{c.sa4, c.da4, c.dport, c.proto, c.fl, a.len, a.ep, a.verdict, a.identity, a.stage,
		    a.delta, a.n, a.pk, 0, nullptr, nullptr};
	if (!x4_aligned(c4))
		return hipErrorInvalidValue;
	if ((e = launch_x4<false, false, 1>(s, c4, st)) != hipSuccess)
		return e;
	cls_args c6{c.sa6, c.da6, c.dport6, c.proto6, c.fl6, c.len6, c.ep6, c.v6, c.id6,
		    a.stage ? c.st6 : nullptr, a.delta, a.n, a.pk, 0, nullptr, nullptr};
	c6.n_dev = c.n6;
	if ((e = launch_x4<false, true, 1>(s, c6, st)) != hipSuccess)
		return e;
	hipLaunchKernelGGL(k_frames_scatter6, dim3(grid_for(a.n)), dim3(BLOCK), 0, st, c, a.verdict, a.identity,
			   a.stage);
	return hipGetLastError();
}

/* as the k_classify<.., CTR = 1> launcher: 1024-thread workgroups, <= 2 per
 * CU (LDS), at most 2^22 frames per workgroup (packed LDS counters) */
hipError_t launch_classify_frames(const cgpu_snapshot &s0, const frames_args &a, hipStream_t st)
{
	constexpr int NT = 1024;
	const cgpu_snapshot s = with_lds_hot(s0, X4_LDS_BUDGET / 8u);
	const size_t lds = (size_t)s.hot_slots * 8u;
	const uint64_t cap = 2ull * 256ull;
	/* cold-slot hits go to the packed per-stream accumulator pk, exact for
	 * <= PKC_CHUNK frames between unpacks */
	const uint64_t per_launch = std::min<uint64_t>(cap * (1ull << 22), PKC_CHUNK);
	static_assert(PKC_CHUNK <= 512ull * (1ull << 22), "frames chunk within the LDS packing bound");
	for (uint64_t off = 0; off < a.n; off += per_launch) {
		frames_args c = a;
		const uint64_t m = std::min<uint64_t>(a.n - off, per_launch);
		c.n = m;
		c.data += off * a.stride;
		c.len += off;
		c.flags += off;
		c.ep += off;
		c.verdict += off;
		c.identity += off;
		if (c.stage)
			c.stage += off;
		const unsigned g = (unsigned)std::min<uint64_t>((m + NT - 1) / NT, cap);
		hipLaunchKernelGGL((k_frames<1, NT>), dim3(g), dim3(NT), lds, st, s, c);
		if (s.cold_hi) {
			const unsigned ug = std::min<unsigned>((s.cold_hi + 255) / 256, 1024);
			hipLaunchKernelGGL(k_unpack, dim3(ug), dim3(256), 0, st, a.delta, a.pk, 0u, s.cold_hi);
		}
	}
	return hipGetLastError();
}

hipError_t launch_table_sum(const void *buf, size_t off, size_t bytes, uint64_t *out, hipStream_t st)
{
	const uint64_t nw = (bytes + 7u) / 8u;
	if (!nw)
		return hipSuccess;
	const unsigned g = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((nw + 255) / 256, 4096));
	hipLaunchKernelGGL(k_table_sum, dim3(g), dim3(256), 0, st, static_cast<const uint64_t *>(buf), off / 8u,
			   (uint64_t)bytes, out);
	return hipGetLastError();
}

hipError_t launch_fold(uint64_t *totals, uint64_t *delta, uint64_t n, hipStream_t st)
{
	unsigned g = (unsigned)std::min<uint64_t>((n + 255) / 256, 1024);
	hipLaunchKernelGGL(k_fold, dim3(g ? g : 1), dim3(256), 0, st, totals, delta, n);
	return hipGetLastError();
}

/* host-resident batches (host.cpp cgpu_classify_v4_host): a chunk's columns
 * read from, and its outputs stored into, the caller's page-locked host
 * buffers by the CUs (16 B per lane, four in flight per lane, coalesced
 * PCIe requests) in place of DMA copies, so every step of the pipeline is a
 * kernel the queues order on the device */
__global__ __launch_bounds__(256) void k_copy_host(uint4 *dst, const uint4 *src, uint64_t n16, uint8_t *dtail,
						   const uint8_t *stail, uint32_t ntail)
{
	const uint64_t stride = (uint64_t)gridDim.x * 256u;
	uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
	for (; i + 3 * stride < n16; i += 4 * stride) {
		const uint4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
		dst[i] = a;
		dst[i + stride] = b;
		dst[i + 2 * stride] = c;
		dst[i + 3 * stride] = d;
	}
	for (; i < n16; i += stride)
		dst[i] = src[i];
	if (blockIdx.x == 0 && threadIdx.x < ntail)
		dtail[threadIdx.x] = stail[threadIdx.x];
}

hipError_t launch_copy_host(void *dst, const void *src, uint64_t bytes, hipStream_t st)
{
	if ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15u)
		return hipErrorInvalidValue;
	if (!bytes)
		return hipSuccess;
	const uint64_t n16 = bytes >> 4;
	const unsigned g = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n16 + 1023) / 1024, 128));
	hipLaunchKernelGGL(k_copy_host, dim3(g), dim3(256), 0, st, static_cast<uint4 *>(dst),
			   static_cast<const uint4 *>(src), n16, static_cast<uint8_t *>(dst) + (n16 << 4),
			   static_cast<const uint8_t *>(src) + (n16 << 4), (uint32_t)(bytes & 15u));
	return hipGetLastError();
}

/* blocks per segment row of the host copies (timing-only A/B builds vary it,
 * tools/host_ab.py) */
#ifndef CGPU_HS_COPY_G
#define CGPU_HS_COPY_G 128
#endif

/* every column of a chunk in ONE launch: segment blockIdx.y, the blocks of
 * a row grid-stride over it (a launch per column left ~10 us gaps between
 * seven small kernels per chunk, profiles/r4_ah) */
__global__ __launch_bounds__(256) void k_copy_host_multi(copy_segs d)
{
	const copy_seg g = d.seg[blockIdx.y];
	const uint64_t n16 = g.bytes >> 4;
	uint4 *dst = static_cast<uint4 *>(g.dst);
	const uint4 *src = static_cast<const uint4 *>(g.src);
	const uint64_t stride = (uint64_t)gridDim.x * 256u;
	uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
	for (; i + 3 * stride < n16; i += 4 * stride) {
		const uint4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], e = src[i + 3 * stride];
		dst[i] = a;
		dst[i + stride] = b;
		dst[i + 2 * stride] = c;
		dst[i + 3 * stride] = e;
	}
	for (; i < n16; i += stride)
		dst[i] = src[i];
	const uint32_t tail = (uint32_t)(g.bytes & 15u);
	if (blockIdx.x == 0 && threadIdx.x < tail)
		static_cast<uint8_t *>(g.dst)[(n16 << 4) + threadIdx.x] =
			static_cast<const uint8_t *>(g.src)[(n16 << 4) + threadIdx.x];
}

hipError_t launch_copy_host_multi(const copy_segs &d, hipStream_t st)
{
	uint64_t most = 0;
	for (uint32_t k = 0; k < d.n; k++) {
		if ((reinterpret_cast<uintptr_t>(d.seg[k].dst) | reinterpret_cast<uintptr_t>(d.seg[k].src)) & 15u)
			return hipErrorInvalidValue;
		most = std::max(most, d.seg[k].bytes);
	}
	if (!d.n || !most)
		return hipSuccess;
	/* the longest segment sets the row width; shorter rows' spare blocks exit */
	const unsigned g = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(((most >> 4) + 1023) / 1024,
									     CGPU_HS_COPY_G));
	hipLaunchKernelGGL(k_copy_host_multi, dim3(g, d.n), dim3(256), 0, st, d);
	return hipGetLastError();
}

hipError_t launch_slot_init(uint64_t *totals, uint64_t *delta, const uint32_t *slot,
			    const uint64_t *pk, const uint64_t *by, uint32_t n, hipStream_t st)
{
	hipLaunchKernelGGL(k_slot_init, dim3((n + 255) / 256), dim3(256), 0, st, totals, delta, slot,
			   pk, by, n);
	return hipGetLastError();
}

/* ======================================================================= */
/* Conntrack on the classification path                  */
/*                                                                          */
/* cgpu_classify_v4_ct in four steps on one stream:                         */
/*  1 k_ct_prep    per packet (parallel): the reply-direction tuple of      */
/*                 ct_lookup4, the ct action, whether policy allows the     */
/*                 forward tuple (no counters), and the conntrack GROUP =   */
/*                 the packet's unordered address pair: every CT key a      */
/*                 packet reads or writes (forward, reply, ICMP related)    */
/*                 carries that pair, so groups never share a key.          */
/*  2 radix sort of (group, packet index): stable, so each group's packets  */
/*                 stay in batch order; then the group heads are selected.  */
/*  3 k_ct_walk    one lane per group replays its packets IN ORDER against  */
/*                 the device CT map (lookups, entry updates, creates,      */
/*                 deletes) = the sequential semantics of the reference.    */
/*  4 k_ct_finish  per packet (parallel): policy on the tuple ct_lookup4    */
/*                 left (reply tuple for CT_REPLY / CT_RELATED) with the    */
/*                 entry counters, the reply/related skip, the verdict and  */
/*                 the metrics.                                             */
/*                                                                          */
/* Memory protocol of the map (per-XCD L2s are not coherent): a slot's tag  */
/* changes only by agent-scope atomics (EMPTY -> LIVE, LIVE -> TOMB,        */
/* TOMB -> LIVE; never back to EMPTY, so a lane that once saw a slot in use */
/* never sees it empty again); key words and entry rows are written         */
/* write-through (sc1) and read past L1 (nt); a key is only ever inserted,  */
/* updated or deleted by the lane that owns its group.                      */
/* ======================================================================= */
#include <hipcub/hipcub.hpp>

#define CT_LIFETIME_TCP 21600u /* bpf/lib/conntrack.h:31-35 */
#define CT_LIFETIME_NONTCP 60u
#define CT_SYN_TIMEOUT 60u
#define CT_CLOSE_TIMEOUT 10u
#define CT_REPORT_INTERVAL 5u
#define DROP_CT_CREATE_FAILED (-155) /* bpf/lib/common.h:262 */
#define CTB_RX_CLOSING 1u
#define CTB_TX_CLOSING 2u
#define CTB_SEEN_NON_SYN 16u
#define TUPLE_F_IN 1u      /* conntrack.h:63-66 */
#define TUPLE_F_RELATED 2u
#define CT_NEW 0u          /* common.h:331-336 */
#define CT_ESTABLISHED 1u
#define CT_REPLY 2u
#define CT_RELATED 3u
#define CT_FAIL 0x80u      /* walker -> finish: the create failed */
/* rec meta bits (rec.w >> 16) */
#define CTM_EGRESS 1u
#define CTM_ACT_CREATE 2u
#define CTM_ACT_CLOSE 4u
#define CTM_TCP 8u
#define CTM_GATED 16u
#define CTM_ALLOWED 32u
#define CTM_FRAG 64u
/* ct_args.pcls: a service-path packet's phase-2 class */
#define PCL_P2A 1u   /* runs in phase 2a (an ordinary pair) */
#define PCL_P2B 2u   /* runs in phase 2b (a special pair) */
#define PCL_ADDRX 4u /* owes an address entry to another pair */
#define PCL_RELX 8u  /* a create may owe its ICMP entry */
/* packets per lane of the conntrack prep / finish passes (timing-only tool
 * builds vary it, tools/diag_ab.py) */
#ifndef CGPU_CT_Q
#define CGPU_CT_Q 4
#endif
/* ... of the finish pass alone (3: its 1024-thread workgroups spill 33-54
 * VGPRs at Q = 4; ct 11.70 -> 11.12 ms, ct6 15.19 -> 14.50, ctlb 20.38 ->
 * 19.65, ctlb6 22.16 -> 21.28, profiles/r5_m/ab_fin_*.log), and its
 * workgroup size */
#ifndef CGPU_CT_FQ
#define CGPU_CT_FQ 3
#endif
#ifndef CGPU_CT_FNT
#define CGPU_CT_FNT 1024
#endif
/* phase 2b groups an address entry no phase-2 packet can read by its whole
 * key (k_ct_owed_bloom); 0: by its pair (A/B) */
#ifndef CGPU_OWED_BY_KEY
#define CGPU_OWED_BY_KEY 1
#endif
/* the service paths' forward decisions: 0 inside the per-packet prep, 1 a
 * k_ct_decq pass after it (Q packets per lane).  Measured slower (ctlb
 * 25.19 -> 25.53 ms, ctlb6 24.13 -> 26.93: the v6 pass stages the trie
 * levels in LDS per 256-thread workgroup, profiles/r4_o/): kept for A/B */
#ifndef CGPU_CT_SVC_DECQ
#define CGPU_CT_SVC_DECQ 0
#endif
/* the service path's prep: Q packets per lane (k_ct_prep_svc_q), 1 = the
 * per-lane k_ct_prep */
#ifndef CGPU_CT_SVC_Q
#define CGPU_CT_SVC_Q 2
#endif
/* ... IPv6 (k_ct_prep6's per-lane decide<1> walks the trie from global
 * memory: 32 GB of HBM traffic per 64M packets, profiles/r4_prof/ctlb6):
 * 1 = k_ct_decq on a resident grid of 1024-thread workgroups, the trie
 * levels staged in LDS once per CU as k_ipc6_pre.  Measured slower too,
 * 24.10 -> 24.75 ms (profiles/r4_s/): off */
#ifndef CGPU_CT_SVC_DECQ6
#define CGPU_CT_SVC_DECQ6 0
#endif
/* ... IPv6: 1 = the trie pre-pass on the translated addresses, then
 * k_ct_prep6_q<SVC> (as the plain IPv6 path) */
#ifndef CGPU_CT_SVC_PRE6
#define CGPU_CT_SVC_PRE6 1
#endif
/* the stateful service step (cgpu_classify_v4_ctlb) */
#define CTM_PHASE2 128u   /* the packet's address pair may hold owed address entries: phase 2 */
#define CTM_ADDRX 256u    /* its address entry lies in another pair: owed to phase 2 */
#define CTM_SVCDROP 512u  /* lb4_local returned DROP_NO_SERVICE */
#define CT_ADDRP 0x40u    /* walker -> phase 2: the address entry of this create is owed */
#define CTM_RELX 1024u    /* grouped by connection in phase 1: the ICMP entry a create
			   * writes is reserved and owed to phase 2 */
#define CT_RELP 0x20u     /* walker -> phase 2: the ICMP entry of this create is owed */
/* Group-default results (CGPU_CT_DFLT, every conntrack path): the prep marks
 * every packet's result CT_DFLT.  A packet's orientation is a fixed function
 * of its tuple that flips for the reversed tuple and is 0 for the usual
 * initiator (ephemeral source port above the service port; an ICMP echo
 * request).  When the group's first decided packet created or found its
 * entry in orientation 0 (ESTABLISHED / NEW for orientation 0, REPLY for 1),
 * the phase-1 walker stores none of the group's results that equal the
 * orientation default -- ESTABLISHED for orientation 0, REPLY for 1 -- and
 * the finish resolves CT_DFLT from the record's tuple alone.  Groups of the
 * other orientation store every result.  Exact for any mix of connections
 * in a group: a packet whose result is not the default is stored.  Saves
 * most of the walker's scattered result stores with no lookup in the
 * finish (a group bitmap read there cost 0.27 ms: profiles/r6_p/, r7_a/). */
#define CT_DFLT 0x10u
#ifndef CGPU_CT_DFLT
#define CGPU_CT_DFLT 1
#endif
/* a packet's orientation (any fixed function of its key) and its group key,
 * as k_ct_prep_q computed it (ct_conn_group over the record's tuple) */
/* z = sport | dport << 16 (TCP / UDP ports in network order, the ICMP /
 * ICMPv6 type word as ct_lookup4 / ct_lookup6 build it), `tie` = saddr <
 * daddr for the reversed-invariant tie */
__device__ __forceinline__ uint32_t ct_orient(uint32_t z, uint32_t proto, bool tie)
{
	uint32_t sp = z & 0xFFFFu, dp = z >> 16;
	if (proto != 1u && proto != 58u) {
		sp = __builtin_bswap16((uint16_t)sp);
		dp = __builtin_bswap16((uint16_t)dp);
		if (sp != dp)
			return sp < dp ? 1u : 0u; /* the initiator's source port is the higher */
	} else if (sp != dp) {
		return sp > dp ? 1u : 0u; /* an echo request carries its type as dport */
	}
	return tie ? 1u : 0u;
}
#define CTB_LB_LOOPBACK 8u /* struct ct_entry lb_loopback (common.h:389) */
#define TUPLE_F_SERVICE 4u /* conntrack.h:66 */
/* rec word 2 .w of the service path: lb_loopback | address-entry mode << 1 */
#define LBF_LOOPBACK 1u
#define AM_NONE 0u
#define AM_INLINE 1u /* same address pair: written by the create itself */
#define AM_DEFER 2u  /* other pair: capacity reserved, written in phase 2 */
#define LBS_ENTRY 1u /* lb_loopback came from the conntrack entry */
#define LBS_SNAT 2u  /* saddr == target: loopback source NAT (lb.h:753-767) */

/* 8-byte write-through store (global_store_dwordx2 sc1) */
__device__ __forceinline__ void st_wt64(void *p, uint32_t lo, uint32_t hi)
{
	__hip_atomic_store(static_cast<uint64_t *>(p), (uint64_t)lo | ((uint64_t)hi << 32),
			   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt32(void *p, uint32_t v)
{
	__hip_atomic_store(static_cast<uint32_t *>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

/* one struct ct_entry row: a,b = rx/tx packets|bytes, c = {lifetime,
 * bits | rev_nat << 16, slave | tx_flags_seen << 16 | rx_flags_seen << 24,
 * src_sec_id}, d = {last_tx_report, last_rx_report} (the row's last 8 bytes
 * are padding) */
struct ct_row {
	uint4 a, b, c;
	uint2 d;
};

__device__ __forceinline__ ct_row ct_row_load(const ct_table &T, uint32_t slot)
{
	const uint4 *p = T.vals + 4u * slot;
	const uint4 d = ld_x4<true>(p + 3);
	return ct_row{ld_x4<true>(p), ld_x4<true>(p + 1), ld_x4<true>(p + 2), uint2{d.x, d.y}};
}

/* Write-through stores complete asynchronously: a later load of the same
 * bytes by this lane (after the entry was evicted from its cache and is
 * probed again) could be served from memory before the store lands.  The
 * lane's cache therefore marks stores pending (ct_cache.pend) and the next
 * probe of the map first waits for them (ct_pend_wait): a store burst never
 * stalls the walk itself, only a later cache miss does, which reads the
 * map anyway.  Other lanes never read this lane's keys or rows (a slot's
 * tag changes by atomics only; a deleted slot is retired with a wait,
 * ct_erase). */
__device__ __forceinline__ void ct_row_store(const ct_table &T, uint32_t slot, const ct_row &e)
{
	uint32_t *p = reinterpret_cast<uint32_t *>(T.vals + 4u * slot);
	st_wt64(p + 0, e.a.x, e.a.y);
	st_wt64(p + 2, e.a.z, e.a.w);
	st_wt64(p + 4, e.b.x, e.b.y);
	st_wt64(p + 6, e.b.z, e.b.w);
	st_wt64(p + 8, e.c.x, e.c.y);
	st_wt64(p + 10, e.c.z, e.c.w);
	st_wt64(p + 12, e.d.x, e.d.y);
}

__device__ __forceinline__ void ct_pend_wait(uint32_t &pend)
{
	if (pend) {
		__builtin_amdgcn_s_waitcnt(0);
		pend = 0;
	}
}

__device__ __forceinline__ void add64(uint32_t &lo, uint32_t &hi, uint32_t v)
{
	const uint64_t x = ((uint64_t)hi << 32 | lo) + v;
	lo = (uint32_t)x;
	hi = (uint32_t)(x >> 32);
}

/* __ct_update_timeout, conntrack.h:104-161 (seen = union tcp_flags.lower_bits) */
__device__ __forceinline__ void ct_touch(ct_row &e, uint32_t now, uint32_t lifetime, bool ingress,
					 uint32_t seen)
{
	e.c.x = now + lifetime;
	const uint32_t sh = ingress ? 24u : 16u;
	const uint32_t acc = (e.c.z >> sh) & 0xFFu;
	const uint32_t last = ingress ? e.d.y : e.d.x;
	seen = (seen | acc) & 0xFFu;
	if (last + CT_REPORT_INTERVAL < now || acc != seen) {
		if (ingress)
			e.d.y = now;
		else
			e.d.x = now;
		e.c.z = (e.c.z & ~(0xFFu << sh)) | (seen << sh);
	}
}

/* ct_update_timeout, conntrack.h:169-185.  w = union tcp_flags as loaded:
 * .syn (like .fin and .rst, a bit-field member of a union) is bit 0. */
__device__ __forceinline__ void ct_timeout(ct_row &e, uint32_t now, bool tcp, bool ingress, uint32_t w)
{
	uint32_t lifetime = CT_LIFETIME_NONTCP;
	if (tcp) {
		if (!(w & 1u))
			e.c.y |= CTB_SEEN_NON_SYN;
		lifetime = (e.c.y & CTB_SEEN_NON_SYN) ? CT_LIFETIME_TCP : CT_SYN_TIMEOUT;
	}
	ct_touch(e, now, lifetime, ingress, w >> 8);
}

/* __ct_lookup's update of a found entry, conntrack.h:205-256 (with
 * CONNTRACK_ACCOUNTING) */
__device__ __forceinline__ void ct_hit(ct_row &e, uint32_t meta, bool ingress, uint32_t w,
				       uint32_t len, uint32_t now)
{
	const bool tcp = meta & CTM_TCP;
	if ((e.c.y & 3u) != 3u) /* ct_entry_alive */
		ct_timeout(e, now, tcp, ingress, w);
	if (ingress) {
		add64(e.a.x, e.a.y, 1u);
		add64(e.a.z, e.a.w, len);
	} else {
		add64(e.b.x, e.b.y, 1u);
		add64(e.b.z, e.b.w, len);
	}
	if (meta & CTM_ACT_CREATE) {
		if (e.c.y & 3u) {
			e.c.y &= ~3u; /* ct_reset_closing */
			ct_timeout(e, now, tcp, ingress, w);
		}
	} else if (meta & CTM_ACT_CLOSE) {
		e.c.y |= ingress ? CTB_RX_CLOSING : CTB_TX_CLOSING;
		if ((e.c.y & 3u) == 3u)
			ct_touch(e, now, CT_CLOSE_TIMEOUT, ingress, w >> 8);
	}
}

__device__ __forceinline__ uint4 sel4(bool t, uint4 a, uint4 b)
{
	return uint4{t ? a.x : b.x, t ? a.y : b.y, t ? a.z : b.z, t ? a.w : b.w};
}

/* The two maps' key slots (tables.h ct_table), as traits of one walker:
 *   CtK4 cilium_ct4_global: keys[h] = {daddr, saddr, dport | sport << 16,
 *        nexthdr | flags << 8 | tag << 16} (struct ipv4_ct_tuple, 16 B)
 *   CtK6 cilium_ct6_global: keys[4h .. 4h + 3] = {dport | sport << 16,
 *        nexthdr | flags << 8 | tag << 16, 0, 0}, {daddr}, {saddr}, {0}
 *        (struct ipv6_ct_tuple in one 64-B line: a probe is one line)
 * In a lane's cache the upper half of the meta word (the tag in the map)
 * holds the CTC_* state instead. */
struct CtK4 {
	typedef uint4 key;
	static constexpr int V6 = 0;
	static constexpr bool SVC = false;  /* entries carry the service's slave / lb_loopback */
	static constexpr bool ADDR = false; /* creates write ct_create4's address entry */
	__device__ static uint32_t &meta(key &k) { return k.w; }
	__device__ static uint32_t cmeta(const key &k) { return k.w; }
	__device__ static uint32_t hash(const key &k) { return ct_hash(k.x, k.y, k.z, k.w); }
	__device__ static bool same(const key &s, const key &k)
	{
		return s.x == k.x && s.y == k.y && s.z == k.z && (s.w & 0xFFFFu) == (k.w & 0xFFFFu);
	}
	__device__ static uint32_t *tagp(const ct_table &T, uint32_t h) { return &T.keys[h].w; }
	__device__ static key load(const ct_table &T, uint32_t h) { return ld_x4<true>(T.keys + h); }
	/* the key words (not the meta word) again, at the coherence point */
	__device__ static void reload(const ct_table &T, uint32_t h, key &s)
	{
		const uint64_t xy = __hip_atomic_load(reinterpret_cast<uint64_t *>(T.keys + h), __ATOMIC_RELAXED,
						      __HIP_MEMORY_SCOPE_AGENT);
		s.x = (uint32_t)xy;
		s.y = (uint32_t)(xy >> 32);
		s.z = __hip_atomic_load(&T.keys[h].z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	}
	__device__ static void store(const ct_table &T, uint32_t h, const key &k)
	{
		uint32_t *p = reinterpret_cast<uint32_t *>(T.keys + h);
		st_wt64(p, k.x, k.y);
		st_wt32(p + 2, k.z);
	}
	__device__ static void clear(const ct_table &T, uint32_t h)
	{
		uint32_t *p = reinterpret_cast<uint32_t *>(T.keys + h);
		st_wt64(p, 0u, 0u);
		st_wt32(p + 2, 0u);
	}
	__device__ static key sel(bool t, const key &a, const key &b) { return sel4(t, a, b); }
	/* ipv4_ct_tuple_reverse, conntrack.h:414-431 */
	__device__ static key reversed(const key &k)
	{
		return uint4{k.y, k.x, (k.z >> 16) | (k.z << 16), k.w ^ (TUPLE_F_IN << 8)};
	}
	/* ct_create4's ICMP entry relating errors, conntrack.h:722-733 */
	__device__ static key related(const key &k)
	{
		return uint4{k.x, k.y, 0u, 1u | ((((k.w >> 8) & 0xFFu) | TUPLE_F_RELATED) << 8)};
	}
};

struct CtK6 {
	struct key {
		uint4 d, s;
		uint32_t p, m;
	};
	static constexpr int V6 = 1;
	static constexpr bool SVC = false;
	static constexpr bool ADDR = false;
	__device__ static uint32_t &meta(key &k) { return k.m; }
	__device__ static uint32_t cmeta(const key &k) { return k.m; }
	__device__ static uint32_t hash(const key &k)
	{
		return ct_hash(fold6(k.d.x, k.d.y, k.d.z, k.d.w), fold6(k.s.x, k.s.y, k.s.z, k.s.w), k.p, k.m);
	}
	__device__ static bool same(const key &a, const key &b)
	{
		return a.p == b.p && (a.m & 0xFFFFu) == (b.m & 0xFFFFu) && a.d.x == b.d.x && a.d.y == b.d.y &&
		       a.d.z == b.d.z && a.d.w == b.d.w && a.s.x == b.s.x && a.s.y == b.s.y && a.s.z == b.s.z &&
		       a.s.w == b.s.w;
	}
	__device__ static uint32_t *tagp(const ct_table &T, uint32_t h) { return &T.keys[4u * h].y; }
	__device__ static key load(const ct_table &T, uint32_t h)
	{
		const uint4 m = ld_x4<true>(T.keys + 4u * h);
		return key{ld_x4<true>(T.keys + 4u * h + 1u), ld_x4<true>(T.keys + 4u * h + 2u), m.x, m.y};
	}
	__device__ static uint4 load_coherent4(const uint4 *q)
	{
		const uint64_t lo = __hip_atomic_load(reinterpret_cast<const uint64_t *>(q), __ATOMIC_RELAXED,
						      __HIP_MEMORY_SCOPE_AGENT);
		const uint64_t hi = __hip_atomic_load(reinterpret_cast<const uint64_t *>(q) + 1, __ATOMIC_RELAXED,
						      __HIP_MEMORY_SCOPE_AGENT);
		return uint4{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
	}
	__device__ static void reload(const ct_table &T, uint32_t h, key &s)
	{
		s.p = __hip_atomic_load(&T.keys[4u * h].x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		s.d = load_coherent4(T.keys + 4u * h + 1u);
		s.s = load_coherent4(T.keys + 4u * h + 2u);
	}
	__device__ static void store(const ct_table &T, uint32_t h, const key &k)
	{
		uint32_t *p = reinterpret_cast<uint32_t *>(T.keys + 4u * h);
		st_wt32(p, k.p);
		st_wt64(p + 4, k.d.x, k.d.y);
		st_wt64(p + 6, k.d.z, k.d.w);
		st_wt64(p + 8, k.s.x, k.s.y);
		st_wt64(p + 10, k.s.z, k.s.w);
	}
	__device__ static void clear(const ct_table &T, uint32_t h)
	{
		store(T, h, key{uint4{0u, 0u, 0u, 0u}, uint4{0u, 0u, 0u, 0u}, 0u, 0u});
	}
	__device__ static key sel(bool t, const key &a, const key &b)
	{
		return key{sel4(t, a.d, b.d), sel4(t, a.s, b.s), t ? a.p : b.p, t ? a.m : b.m};
	}
	/* ipv6_ct_tuple_reverse, conntrack.h:265-285 */
	__device__ static key reversed(const key &k)
	{
		return key{k.s, k.d, (k.p >> 16) | (k.p << 16), k.m ^ (TUPLE_F_IN << 8)};
	}
	/* ct_create6's ICMPv6 entry relating errors, conntrack.h:617-629 */
	__device__ static key related(const key &k)
	{
		return key{k.d, k.s, 0u, 58u | ((((k.m >> 8) & 0xFFu) | TUPLE_F_RELATED) << 8)};
	}
};

/* cilium_ct4_global behind the stateful service step: CtK4's key slots,
 * records of 3 x 16 B (the service's ct_state) and ct_create4's address
 * entry */
struct CtK4S : CtK4 {
	static constexpr bool SVC = true;
	static constexpr bool ADDR = true;
};
/* cilium_ct6_global behind the IPv6 service step (ct_create6 writes no
 * address entry) */
struct CtK6S : CtK6 {
	static constexpr bool SVC = true;
};

/* Probe for k (low 16 bits of the meta word = nexthdr | flags << 8).
 * Returns the slot or -1; *free_at = the first tombstone on the chain, else
 * the empty slot that ended it (where an insert of k may start). */
template <class K>
__device__ __forceinline__ int ct_find(const ct_table &T, const typename K::key &k, uint32_t *free_at,
				       uint32_t &pend)
{
	ct_pend_wait(pend);
	uint32_t h = K::hash(k) & T.mask;
	uint32_t ff = 0xFFFFFFFFu;
	for (uint32_t probe = 0; probe <= T.mask; probe++) {
		typename K::key s = K::load(T, h);
		uint32_t tag = K::meta(s) >> 16;
#ifdef CGPU_DIAG_CT_COHERENT_PROBE /* timing-only tool build: every slot read at the coherence point */
		if (true) {
#else
		if (tag == CT_TAG_EMPTY) {
#endif
			/* the chain ends only on an EMPTY read at the coherence point:
			 * the plain load may be a line this XCD's L2 holds from before
			 * another XCD's lane claimed the slot (a claim's CAS happens at
			 * memory), which would end the chain early and hide a key this
			 * lane inserted past it.  Tags never return to EMPTY, so one
			 * agent-scope re-read settles it; key words written after a
			 * claim are re-read the same way. */
			K::meta(s) = __hip_atomic_load(K::tagp(T, h), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			tag = K::meta(s) >> 16;
			if (tag == CT_TAG_EMPTY) {
				*free_at = ff != 0xFFFFFFFFu ? ff : h;
				return -1;
			}
			K::reload(T, h, s);
		}
		if (tag == CT_TAG_LIVE && K::same(s, k))
			return (int)h;
		if (tag == CT_TAG_TOMB && ff == 0xFFFFFFFFu)
			ff = h;
		h = (h + 1u) & T.mask;
	}
	*free_at = ff;
	return -1;
}

/* Per-workgroup accounting of the map's live / tombstone counts.  One
 * global word takes every insert's capacity check otherwise (~10^2 atomics
 * per us on one address): a workgroup instead reserves capacity from
 * count[0] in chunks and keeps the rest in LDS, and nets its tombstone and
 * delete changes in LDS, all flushed once at the end.  Exact while the map
 * is not about to fill; at the edge an unused reservation of another
 * workgroup can fail a create early (the documented order dependence).
 * The chunk (T.res_chunk) is sized by the host so that all waves'
 * outstanding reservations stay under a quarter of the headroom. */
struct ct_acct {
	int *res;   /* LDS: reserved, unused capacity */
	int *live;  /* LDS: live entries removed (deletes), to return */
	int *tombs; /* LDS: tombstone delta */
};

__device__ __forceinline__ bool ct_take(const ct_table &T, const ct_acct &A)
{
	if (atomicSub(A.res, 1) > 0)
		return true;
	atomicAdd(A.res, 1);
	/* one refill per wave for all the lanes that found the pool empty:
	 * a refill per lane would hold 64 chunks per wave */
	const uint64_t m = __ballot(1);
	const int leader = __ffsll((unsigned long long)m) - 1;
	const uint32_t need = (uint32_t)__popcll(m);
	const bool lead = (int)__lane_id() == leader;
	uint32_t got = 0;
	if (lead) {
		const uint32_t ask = need + T.res_chunk - 1u;
		if (atomicAdd(&T.count[0], ask) + ask <= T.max) {
			got = ask;
		} else {
			atomicSub(&T.count[0], ask);
			got = 0xFFFFFFFFu; /* at the edge: one exact check per lane */
		}
	}
	got = __shfl(got, leader, 64);
	if (got != 0xFFFFFFFFu) {
		if (lead && got > need)
			atomicAdd(A.res, (int)(got - need));
		return true;
	}
	if (atomicAdd(&T.count[0], 1u) < T.max)
		return true;
	atomicSub(&T.count[0], 1u);
	return false;
}


/* ---- LRU mode (cgpu_config.ct_lru) ----
 * The reference declares CT_MAP4 / CT_MAP6 as BPF_MAP_TYPE_LRU_HASH on every
 * kernel with LRU maps (bpf/bpf_lxc.c:53-75, probe bpf/probes/raw_lru_map.t),
 * so a full map evicts instead of failing ct_create.  Its victim is the
 * kernel's per-CPU LRU list's; ours is an entry none of this batch's
 * packets can touch: every key a packet of the batch may look up or create
 * (reply, forward and ICMP tuples; the service path's service, address and
 * ICMP tuples) is marked in a bloom filter before the walks, and a create
 * that finds the map full scans the slots from a hashed start for a live
 * entry outside the filter.  So every packet of the batch gets the result
 * the map it started from gives it, whatever was evicted; across batches an
 * entry idle in one batch may be gone in the next, as an LRU-evicted one. */
#ifndef CT_EVICT_SCAN
#define CT_EVICT_SCAN 4096u
#endif

template <class K> __device__ __forceinline__ uint32_t ct_bbit(const typename K::key &k)
{
	return ct_fmix(K::hash(k) ^ 0x2545F491u);
}

template <class K> __device__ __forceinline__ bool ct_in_batch(const ct_table &T, const typename K::key &k)
{
	const uint32_t b = ct_bbit<K>(k);
	return (T.bloom[(b >> 5) & T.bloom_mask] >> (b & 31u)) & 1u;
}

template <class K> __device__ __forceinline__ void ct_mark(uint32_t *bloom, uint32_t mask, const typename K::key &k)
{
	const uint32_t b = ct_bbit<K>(k);
	uint32_t *w = bloom + ((b >> 5) & mask);
	const uint32_t m = 1u << (b & 31u);
	if (!(*w & m)) /* most marks repeat a connection's: read before the atomic */
		atomicOr(w, m);
}

/* evict one live entry outside the batch's filter: its capacity passes to
 * the caller's create (the live count does not change), the slot becomes a
 * tombstone as a delete leaves it (claimed first, so no prober compares
 * and no insert reuses it while its words are cleared) */
template <class K> __device__ __forceinline__ bool ct_evict(const ct_table &T, const ct_acct &A, uint32_t start)
{
	uint32_t h = start & T.mask;
	for (uint32_t probe = 0; probe < CT_EVICT_SCAN; probe++, h = (h + 1u) & T.mask) {
		const uint32_t tw = __hip_atomic_load(K::tagp(T, h), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		if ((tw >> 16) != CT_TAG_LIVE)
			continue;
		typename K::key s{};
		K::reload(T, h, s);
		K::meta(s) = tw;
		if (ct_in_batch<K>(T, s))
			continue;
		if (atomicCAS(K::tagp(T, h), tw, (CT_TAG_CLAIM << 16) | (tw & 0xFFFFu)) != tw)
			continue;
		K::clear(T, h);
		__builtin_amdgcn_s_waitcnt(0);
		__hip_atomic_exchange(K::tagp(T, h), CT_TAG_TOMB << 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		atomicAdd(A.tombs, 1);
		return true;
	}
	return false;
}

/* ct_take, and in LRU mode an eviction when the map is full */
template <class K> __device__ __forceinline__ bool ct_take_k(const ct_table &T, const ct_acct &A, uint32_t seed)
{
	if (ct_take(T, A))
		return true;
	return T.lru && ct_evict<K>(T, A, ct_fmix(seed ^ (blockIdx.x * 256u + threadIdx.x) * 0x9E3779B1u));
}

/* Insert absent k at the first free slot from `from` on (htab_map_update_elem
 * of a new key: -E2BIG past max_elem).  Returns the slot or -1. */
template <class K, bool TAKE = true>
__device__ __forceinline__ int ct_insert(const ct_table &T, const ct_acct &A, const typename K::key &k,
					 uint32_t from)
{
	if (TAKE && !ct_take_k<K>(T, A, K::hash(k)))
		return -1;
	uint32_t h = from & T.mask;
	for (uint32_t probe = 0; probe <= T.mask; probe++) {
		typename K::key s = K::load(T, h);
		const uint32_t tag = K::meta(s) >> 16;
		if (tag == CT_TAG_EMPTY || tag == CT_TAG_TOMB) {
			const uint32_t expect = tag << 16;
			const uint32_t want = (K::cmeta(k) & 0xFFFFu) | (CT_TAG_LIVE << 16);
			/* LRU mode: the slot turns LIVE only once its key words are
			 * written (claimed first), so an eviction never judges a key it
			 * reads half-written */
			const uint32_t first = T.lru ? (K::cmeta(k) & 0xFFFFu) | (CT_TAG_CLAIM << 16) : want;
			if (atomicCAS(K::tagp(T, h), expect, first) == expect) {
				if (tag == CT_TAG_TOMB)
					atomicSub(A.tombs, 1);
				K::store(T, h, k); /* pending: the caller marks it (ctc_update) */
				if (T.lru) {
					__builtin_amdgcn_s_waitcnt(0);
					__hip_atomic_exchange(K::tagp(T, h), want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
				}
				return (int)h;
			}
		}
		h = (h + 1u) & T.mask;
	}
	atomicAdd(A.res, 1);
	return -1;
}

/* map_delete_elem: the row and key words are retired before the tag turns
 * into a tombstone another lane may claim.  Every store to the map is
 * write-through, so draining this lane's outstanding stores (vmcnt 0) is
 * the whole release: no L2 write-back (an agent-scope release fence would
 * write back the XCD's entire L2 for every delete). */
template <class K> __device__ __forceinline__ void ct_erase(const ct_table &T, const ct_acct &A, uint32_t slot)
{
	if (T.lru) /* claimed first: an eviction's CAS of the LIVE tag then fails */
		__hip_atomic_exchange(K::tagp(T, slot), CT_TAG_CLAIM << 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	K::clear(T, slot);
	__builtin_amdgcn_s_waitcnt(0);
	__hip_atomic_exchange(K::tagp(T, slot), CT_TAG_TOMB << 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	atomicAdd(A.live, 1);
	atomicAdd(A.tombs, 1);
}

struct ct_args {
	const uint32_t *saddr, *daddr; /* IPv6: 16 bytes per packet */
	const uint16_t *sport, *dport;
	const uint8_t *proto;
	const uint16_t *l4;
	const uint8_t *flags;
	const uint32_t *len;
	const uint16_t *ep;
	int32_t *verdict;
	uint8_t *ct_ret;
	uint32_t *identity;
	uint8_t *stage;
	uint64_t *delta;
	uint64_t n;
	uint32_t now;
	/* scratch */
	uint4 *rec;                  /* [2n] (IPv4) / [4n] (IPv6) per packet, batch order */
	uint32_t *gkey, *gkey_sorted; /* [n] */
	uint32_t *idx, *idx_sorted;   /* [n] */
	uint8_t *head;               /* [n] */
	uint32_t *heads, *n_heads;   /* [n], [1] */
	const uint32_t *gpos, *glen; /* [n_heads] group start / length, longest first */
	/* the stateful service step (cgpu_classify_v4_ctlb) */
	const uint32_t *hash;        /* skb->hash or NULL (cgpu_flow_hash) */
	uint4 *svc_out;              /* [n] lb4_local's outcome per packet */
	uint32_t *ctl;               /* [4] flags: violation, phase-2 packets, owed entries */
	uint32_t *xdaddr;            /* [n] optional: frame daddr after the service step */
	uint16_t *xdport;            /* [n] optional: frame dport after it */
	uint32_t serial;             /* one group for the whole batch (see launch_ctlb) */
	uint8_t *f2;                 /* [2n] phase-2 candidate flags (plain path) */
	uint8_t *pcls;               /* [n] service path: phase-2 class, PCL_* (k_ct_prep) */
	uint64_t *pk;                /* packed per-slot counters (k_ct_finish, k_unpack) */
	uint32_t dflt; /* nonzero: group-default results (CGPU_CT_DFLT) */
};

/* One packet's record, written by k_ct_prep{,6} and read by the walker and
 * k_ct_finish (batch order):
 *   IPv4 (2 x 16 B): {daddr, saddr, z, nexthdr | tflags << 8 | meta << 16},
 *                    {w | port << 16, len, sec, cst}
 *   IPv6 (4 x 16 B): {daddr}, {saddr}, {z, nexthdr | tflags << 8 | meta << 16,
 *                    w | port << 16, len}, {sec, cst, rev_nat, 0}
 * z = the reply-direction tuple's dport | sport << 16 (ct_lookup's first
 * lookup), w = the L4 word (TCP header bytes 12-13 / ICMP type), port = the
 * forward decision's proxy port, sec = src_sec_id of a created entry, cst =
 * counter slot + 1 | stage << 24 of the forward decision, rev_nat = the
 * reverse NAT index an IPv6 ingress entry is created with. */
struct ct_pkt {
	uint32_t meta, w, len, sec, revnat, port, cst, dport, proto;
	uint32_t sa4, da4;
	uint4 sa6, da6;
	/* the service's ct_state (CtK4S): slave, lb_loopback | mode << 1, addr,
	 * svc_addr */
	uint32_t slave, lbf, addr, svc_addr;
};

template <class K> struct ct_rec;
template <> struct ct_rec<CtK4> {
	static constexpr uint32_t RW = 2;
	uint4 r0, r1;
	__device__ static ct_rec load(const uint4 *rec, uint32_t i, bool nt)
	{
		return nt ? ct_rec{ld_x4<true>(rec + 2u * i), ld_x4<true>(rec + 2u * i + 1u)}
			  : ct_rec{rec[2u * i], rec[2u * i + 1u]};
	}
	__device__ CtK4::key key() const { return uint4{r0.x, r0.y, r0.z, r0.w & 0xFFFFu}; }
	__device__ uint32_t meta() const { return r0.w >> 16; }
	__device__ ct_pkt pkt() const
	{
		return ct_pkt{r0.w >> 16, r1.x & 0xFFFFu, r1.y, r1.z, 0u, r1.x >> 16, r1.w, r0.z & 0xFFFFu,
			      r0.w & 0xFFu, r0.y, r0.x, uint4{}, uint4{}};
	}
};
/*   IPv4 behind the service step (3 x 16 B): the IPv4 record, then
 *                    {rev_nat | slave << 16, addr, svc_addr, lbf} */
template <> struct ct_rec<CtK4S> {
	static constexpr uint32_t RW = 3;
	uint4 r0, r1, r2;
	__device__ static ct_rec load(const uint4 *rec, uint32_t i, bool nt)
	{
		const uint4 *p = rec + 3u * i;
		return nt ? ct_rec{ld_x4<true>(p), ld_x4<true>(p + 1), ld_x4<true>(p + 2)}
			  : ct_rec{p[0], p[1], p[2]};
	}
	__device__ CtK4::key key() const { return uint4{r0.x, r0.y, r0.z, r0.w & 0xFFFFu}; }
	__device__ uint32_t meta() const { return r0.w >> 16; }
	__device__ ct_pkt pkt() const
	{
		return ct_pkt{r0.w >> 16, r1.x & 0xFFFFu, r1.y, r1.z, r2.x & 0xFFFFu, r1.x >> 16, r1.w,
			      r0.z & 0xFFFFu, r0.w & 0xFFu, r0.y, r0.x, uint4{}, uint4{},
			      r2.x >> 16, r2.w, r2.y, r2.z};
	}
};
template <> struct ct_rec<CtK6> {
	static constexpr uint32_t RW = 4;
	uint4 r0, r1, r2, r3;
	__device__ static ct_rec load(const uint4 *rec, uint32_t i, bool nt)
	{
		const uint4 *p = rec + 4u * i;
		return nt ? ct_rec{ld_x4<true>(p), ld_x4<true>(p + 1), ld_x4<true>(p + 2), ld_x4<true>(p + 3)}
			  : ct_rec{p[0], p[1], p[2], p[3]};
	}
	__device__ CtK6::key key() const { return CtK6::key{r0, r1, r2.x, r2.y & 0xFFFFu}; }
	__device__ uint32_t meta() const { return r2.y >> 16; }
	__device__ ct_pkt pkt() const
	{
		return ct_pkt{r2.y >> 16, r2.z & 0xFFFFu, r2.w, r3.x, r3.z, r2.z >> 16, r3.y, r2.x & 0xFFFFu,
			      r2.y & 0xFFu, 0u, 0u, r1, r0};
	}
};

/* ct_create4's address entry (conntrack.h:697-725) of forward tuple k for
 * the egress direction: daddr := state->addr; on loopback flags :=
 * TUPLE_F_IN and saddr := state->svc_addr */
__device__ __forceinline__ uint4 ct_addr_key(uint4 k, const ct_pkt &q)
{
	k.x = q.addr;
	if (q.lbf & LBF_LOOPBACK) {
		k.w = (k.w & ~0xFF00u) | (TUPLE_F_IN << 8);
		k.y = q.svc_addr;
	}
	return k;
}

/*   IPv6 behind the service step: the IPv6 record with {sec, cst, rev_nat,
 *                    slave | lbf << 16} as its last word */
template <> struct ct_rec<CtK6S> {
	static constexpr uint32_t RW = 4;
	uint4 r0, r1, r2, r3;
	__device__ static ct_rec load(const uint4 *rec, uint32_t i, bool nt)
	{
		const uint4 *p = rec + 4u * i;
		return nt ? ct_rec{ld_x4<true>(p), ld_x4<true>(p + 1), ld_x4<true>(p + 2), ld_x4<true>(p + 3)}
			  : ct_rec{p[0], p[1], p[2], p[3]};
	}
	__device__ CtK6::key key() const { return CtK6::key{r0, r1, r2.x, r2.y & 0xFFFFu}; }
	__device__ uint32_t meta() const { return r2.y >> 16; }
	__device__ ct_pkt pkt() const
	{
		return ct_pkt{r2.y >> 16, r2.z & 0xFFFFu, r2.w, r3.x, r3.z, r2.z >> 16, r3.y, r2.x & 0xFFFFu,
			      r2.y & 0xFFu, 0u, 0u, r1, r0, r3.w & 0xFFFFu, r3.w >> 16, 0u, 0u};
	}
};

/* CGPU_CT_DFLT: a walked packet's orientation from its record (ct_orient) */
__device__ __forceinline__ bool ct6_lt(const uint4 &a, const uint4 &b)
{
	if (a.x != b.x)
		return a.x < b.x;
	if (a.y != b.y)
		return a.y < b.y;
	if (a.z != b.z)
		return a.z < b.z;
	return a.w < b.w;
}
template <class K> struct ct_dflt {
	static constexpr bool ON = CGPU_CT_DFLT != 0;
	__device__ static uint32_t orient(const ct_rec<K> &r)
	{
		if constexpr (K::V6 != 0) /* {daddr, saddr, {z, proto | ...}} */
			return ct_orient(r.r2.x, r.r2.y & 0xFFu, ct6_lt(r.r1, r.r0));
		else /* {daddr, saddr, z, proto | ...} */
			return ct_orient(r.r0.z, r.r0.w & 0xFFu, r.r0.y < r.r0.x);
	}
};

/* set a batch-wide flag word (0 -> 1): the launcher only asks whether any
 * packet set it.  One plain store per wave that needs it (performed in the
 * XCD's L2; every writer writes the same value): an atomic per packet (or
 * per wave) on one word serialises at the memory side (~88 per us,
 * MI355X_MICROARCH.md), 3 ms per 16M packets of the service path. */
__device__ __forceinline__ void ct_flag(uint32_t *w)
{
	const uint64_t m = __ballot(1);
	if ((int)__lane_id() == __ffsll((unsigned long long)m) - 1)
		*w = 1u;
}

/* ct_lookup4's tuple setup, conntrack.h:461-528.  SVC (cgpu_classify_v4_ctlb):
 * egress packets first take lb4_local's outcome (svc_out, the service walk):
 * the frame's daddr / dport as lb4_xlate left them, tuple.daddr (the service
 * address is kept on loopback, lb.h:769-770), the ct_state ct_create4 will
 * store; a packet whose address entry lies in another address pair owes it
 * to phase 2 (CTM_ADDRX), and a packet whose own pair can receive such
 * entries runs in phase 2 (CTM_PHASE2).  SERIAL: one group for the batch. */
/* one packet of k_ct_prep before and after its forward decision (the
 * per-lane kernel and the Q-interleaved service prep share them) */
struct prep4 {
	uint32_t fl, pr, len, sa, ep, w, da, dp, tfl, z, meta, r2x, addr, saddr2, lbf;
	bool egress, frag, dec; /* dec: the packet takes the forward decision */
};

template <bool SVC, bool SERIAL>
__device__ __forceinline__ bool prep4_pre(const cgpu_snapshot &s, const ct_args &a, uint64_t i, prep4 &p)
{
	constexpr uint32_t RW = SVC ? 3u : 2u;
	p.fl = a.flags[i];
	p.pr = a.proto[i];
	p.len = a.len[i];
	p.sa = a.saddr[i];
	p.ep = a.ep[i];
	p.w = a.l4[i];
	p.da = a.daddr[i];
	p.dp = a.dport[i];
	p.egress = p.fl & 1u;
	p.tfl = p.egress ? TUPLE_F_IN : 0u;
	p.z = 0;
	p.meta = p.egress ? CTM_EGRESS : 0u;
	p.r2x = p.addr = p.saddr2 = p.lbf = 0;
	const uint32_t &fl = p.fl, &pr = p.pr, &len = p.len, &sa = p.sa;
	uint32_t &w = p.w, &da = p.da, &dp = p.dp, &tfl = p.tfl, &z = p.z, &meta = p.meta, &r2x = p.r2x,
		 &addr = p.addr, &saddr2 = p.saddr2, &lbf = p.lbf;
	const bool egress = p.egress;
	uint32_t xd = da;
	if constexpr (SVC) {
		const uint4 so = egress ? a.svc_out[i] : make_uint4(SVC_NONE, 0, 0, 0);
		if ((so.x & 3u) == SVC_DROP) {
			a.identity[i] = 0;
			if (a.xdaddr)
				a.xdaddr[i] = da;
			if (a.xdport)
				a.xdport[i] = (uint16_t)dp;
			uint4 *r = a.rec + RW * i;
			r[0] = uint4{da, sa, 0u, pr | ((CTM_EGRESS | CTM_GATED | CTM_SVCDROP) << 16)};
			r[1] = uint4{0u, len, 0u, 0u};
			r[2] = uint4{0u, 0u, 0u, 0u};
			a.gkey[i] = SERIAL ? 0u : ct_fmix((uint32_t)i ^ 0x5bd1e995u);
			a.idx[i] = (uint32_t)i;
			if constexpr (!SERIAL)
				a.pcls[i] = 0u; /* dropped: no phase-2 class (the scratch is reused) */
			return false;
		}
		if ((so.x & 3u) == SVC_XLATED) {
			const uint32_t lbs = (so.x >> 8) & 3u, tg = so.y;
			const bool lb = lbs != 0;
			xd = tg;
			if (!lb)
				da = tg; /* tuple->daddr = svc->target */
			if (so.z & 0xFFFFu)
				dp = so.z & 0xFFFFu; /* lb4_xlate's port rewrite */
			addr = (lbs & LBS_SNAT) ? s.ipv4_loopback : tg;
			saddr2 = (lbs & LBS_SNAT) ? sa : 0u;
			/* the address entry's pair {addr, loopback ? svc_addr : daddr}
			 * against the packet's own {saddr, daddr} */
			const uint32_t b = lb ? saddr2 : da;
			const bool same = (addr == sa && b == da) || (addr == da && b == sa);
			/* ct_create4 writes no address entry for addr 0 (a slave-0
			 * master row carries target 0), conntrack.h:697 */
			const uint32_t am = !addr ? AM_NONE : (same || SERIAL) ? AM_INLINE : AM_DEFER;
			lbf = (lb ? LBF_LOOPBACK : 0u) | (am << 1);
			r2x = (so.z >> 16) | (so.x & 0xFFFF0000u);
		}
		if (a.xdaddr)
			a.xdaddr[i] = xd;
		if (a.xdport)
			a.xdport[i] = (uint16_t)dp;
	}
	if (pr == 1u) {
		const uint32_t type = w & 0xFFu;
		if (type == 3u || type == 11u || type == 12u) /* DEST_UNREACH, TIME_EXCEEDED, PARAMETERPROB */
			tfl |= TUPLE_F_RELATED;
		else if (type == 0u) /* ECHOREPLY: tuple->dport = ICMP_ECHO */
			z = 8u;
		else {
			if (type == 8u) /* ECHO: tuple->sport = type */
				z = 8u << 16;
			meta |= CTM_ACT_CREATE;
		}
	} else if (pr == 6u || pr == 17u) {
		/* skb_load_bytes(off, &tuple->dport, 4): dport <- sport, sport <- dport */
		z = (uint32_t)a.sport[i] | (dp << 16);
		if (pr == 6u) {
			meta |= CTM_TCP | ((w & 1u) ? CTM_ACT_CLOSE : CTM_ACT_CREATE);
		} else {
			meta |= CTM_ACT_CREATE;
		}
	} else {
		meta |= CTM_GATED;
	}
	if (pr != 6u)
		w = 0; /* union tcp_flags stays zero (conntrack.h:448) */
	p.frag = !egress && ((fl >> 1) & 1u);
	p.dec = !(meta & CTM_GATED);
	return true;
}

template <bool SVC, bool SERIAL>
__device__ __forceinline__ void prep4_post(const cgpu_snapshot &s, const ct_args &a, uint64_t i, const prep4 &p,
					   const decision &d, bool conn)
{
	constexpr uint32_t RW = SVC ? 3u : 2u;
	const uint32_t &pr = p.pr, &len = p.len, &sa = p.sa, &ep = p.ep, &w = p.w, &da = p.da, &tfl = p.tfl, &z = p.z,
		       &r2x = p.r2x, &addr = p.addr, &saddr2 = p.saddr2, &lbf = p.lbf;
	uint32_t meta = p.meta;
	const bool egress = p.egress;
	uint32_t sec = 0, port = 0, cst = 0, id = 0;
	if (p.dec) {
		/* the forward tuple's decision (what CT_NEW / CT_ESTABLISHED packets
		 * see); k_ct_finish bumps its counter */
		if (p.frag)
			meta |= CTM_FRAG;
		if (egress)
			sec = ep < s.n_lxc ? s.lxc[2u * ep + 1u].w : 0u; /* SECLABEL */
		if constexpr (!SVC || !CGPU_CT_SVC_DECQ) {
			if (d.v >= 0) {
				meta |= CTM_ALLOWED;
				port = (uint32_t)d.v;
			}
			id = d.id;
			if (!egress)
				sec = d.id;
			cst = (uint32_t)(d.ctr + 1) | (d.st << 24);
		} /* SVC: k_ct_decq, Q packets per lane */
	}
	uint32_t g = ct_group(sa, da);
	if constexpr (!SVC) {
		/* phase 1 by connection (TCP / UDP ports, ICMP echo ids): only
		 * the ICMP entries of creates (owed) and the ICMP errors that
		 * read them (phase 2) share an address pair's keys across
		 * connections */
		bool p2 = false;
		if (!(meta & CTM_GATED)) {
			if (pr == 1u && (tfl & TUPLE_F_RELATED)) {
				meta |= CTM_PHASE2;
				p2 = true;
			} else {
				meta |= CTM_RELX;
				g = ct_conn_group(g, z, pr);
			}
		}
		/* phase-2 candidates 2i (the packet) and 2i + 1 (its owed ICMP
		 * entry, set by the walker) */
		reinterpret_cast<uint16_t *>(a.f2)[i] = p2 ? 1u : 0u;
	}
	if constexpr (SVC) {
		if (!SERIAL && !(meta & CTM_GATED)) {
			/* pairs an address entry can land in: {T, T}, {IPV4_LOOPBACK,
			 * x}, {target, 0} (ct_create4's addr / svc_addr rewrites) */
			const uint32_t lo = s.ipv4_loopback;
			/* ... and, grouping by connection (conn), ICMP errors, which
			 * read the ICMP entries the creates of every connection of
			 * their pair owe */
			const bool special = sa == da || !sa || !da || sa == lo || da == lo;
			const bool p2 = special || (conn && pr == 1u && (tfl & TUPLE_F_RELATED));
			if ((lbf >> 1) == AM_DEFER) {
				meta |= CTM_ADDRX;
				ct_flag(&a.ctl[2]);
				if (special)
					ct_flag(&a.ctl[0]); /* owes into phase 2b from phase 2b */
			}
			if (p2) {
				meta |= CTM_PHASE2;
				ct_flag(&a.ctl[1]);
				g = ct_fmix((uint32_t)i ^ 0x5bd1e995u);
			} else if (conn) {
				/* phase 1 by connection (an address entry of the same
				 * pair is the forward key itself: tuple.daddr is the
				 * target already), the ICMP entry owed */
				meta |= CTM_RELX;
				ct_flag(&a.ctl[2]);
				g = ct_conn_group(g, z, pr);
			}
		}
	}
	a.identity[i] = id;
	if (!SERIAL && CGPU_CT_DFLT && a.dflt)
		a.ct_ret[i] = CT_DFLT; /* as k_ct_prep_q */
	uint4 *r = a.rec + RW * i;
	r[0] = uint4{da, sa, z, pr | (tfl << 8) | (meta << 16)};
	r[1] = uint4{w | (port << 16), len, sec, cst};
	if constexpr (SVC)
		r[2] = uint4{r2x, addr, saddr2, lbf};
	a.gkey[i] = SERIAL ? 0u : (meta & CTM_GATED) ? ct_fmix((uint32_t)i ^ 0x5bd1e995u) : g;
	a.idx[i] = (uint32_t)i;
	if constexpr (SVC && !SERIAL) {
		/* what k_ct_owed_flags selects by, in one byte instead of the
		 * record's first line */
		const bool live = !(meta & CTM_GATED);
		const uint32_t lo = s.ipv4_loopback;
		const bool special = sa == da || !sa || !da || sa == lo || da == lo;
		const bool p2 = live && (meta & CTM_PHASE2);
		a.pcls[i] = (uint8_t)((p2 && !special ? PCL_P2A : 0u) | (p2 && special ? PCL_P2B : 0u) |
				      (live && (meta & CTM_ADDRX) ? PCL_ADDRX : 0u) |
				      (live && (meta & CTM_RELX) ? PCL_RELX : 0u));
	}
}

template <bool SVC, bool SERIAL>
__global__ __launch_bounds__(256) void k_ct_prep(cgpu_snapshot s, ct_args a, bool conn = false)
{
	const uint64_t stride = (uint64_t)gridDim.x * 256u;
	for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < a.n; i += stride) {
		prep4 p;
		if (!prep4_pre<SVC, SERIAL>(s, a, i, p))
			continue;
		decision d{};
		if (p.dec && (!SVC || !CGPU_CT_SVC_DECQ))
			d = decide<0>(s, p.egress, p.frag, p.sa, p.da, uint4{}, uint4{}, p.z >> 16, p.pr, p.ep);
		prep4_post<SVC, SERIAL>(s, a, i, p, d, conn);
	}
}

/* k_ct_prep<true, false> (the service path) with Q packets per lane: the
 * forward decisions through decide4_q, every lookup stage's gathers of the
 * lane's packets in flight together */
template <int Q>
__global__ __launch_bounds__(256) void k_ct_prep_svc_q(cgpu_snapshot s, ct_args a, bool conn)
{
	const uint64_t T = (uint64_t)gridDim.x * 256u;
	for (uint64_t g = (uint64_t)blockIdx.x * 256u + threadIdx.x; g < a.n; g += T * Q) {
		prep4 p[Q];
		bool act[Q], dec[Q], eg[Q], frag[Q];
		uint32_t sa[Q], da[Q], fdp[Q], pr[Q], ep[Q];
#pragma unroll
		for (int u = 0; u < Q; u++) {
			const uint64_t i = g + (uint64_t)u * T;
			act[u] = i < a.n && prep4_pre<true, false>(s, a, i, p[u]);
			dec[u] = act[u] && p[u].dec;
			eg[u] = act[u] && p[u].egress;
			frag[u] = act[u] && p[u].frag;
			sa[u] = act[u] ? p[u].sa : 0u;
			da[u] = act[u] ? p[u].da : 0u;
			fdp[u] = act[u] ? p[u].z >> 16 : 0u;
			pr[u] = act[u] ? p[u].pr : 0u;
			ep[u] = act[u] ? p[u].ep : 0u;
		}
		decision d[Q];
		decide4_q<Q>(s, dec, eg, frag, sa, da, fdp, pr, ep, d);
#pragma unroll
		for (int u = 0; u < Q; u++)
			if (act[u])
				prep4_post<true, false>(s, a, g + (uint64_t)u * T, p[u], d[u], conn);
	}
}

/* k_ct_prep<false, false> (the plain IPv4 path) with Q packets per lane:
 * the forward decisions through decide4_q; packet i = g + u * (threads),
 * so every column load of a wave covers 64 consecutive packets */
template <int Q>
__global__ __launch_bounds__(256) void k_ct_prep_q(cgpu_snapshot s, ct_args a)
{
	const uint64_t T = (uint64_t)gridDim.x * 256u;
	for (uint64_t g = (uint64_t)blockIdx.x * 256u + threadIdx.x; g < a.n; g += T * Q) {
		bool act[Q], dec[Q], eg[Q], frag[Q];
		uint32_t sa[Q], da[Q], fdp[Q], pr[Q], ep[Q], meta[Q], tfl[Q], z[Q], w[Q], len[Q];
#pragma unroll
		for (int u = 0; u < Q; u++) {
			const uint64_t i = g + (uint64_t)u * T;
			act[u] = i < a.n;
			const uint64_t j = act[u] ? i : 0u;
			/* columns stream past the tables: nontemporal, so they do not
			 * evict the LPM / policy lines from L2 */
			const uint32_t fl = ntl(a.flags + j);
			pr[u] = ntl(a.proto + j);
			len[u] = ntl(a.len + j);
			sa[u] = ntl(a.saddr + j);
			da[u] = ntl(a.daddr + j);
			ep[u] = ntl(a.ep + j);
			w[u] = ntl(a.l4 + j);
			const uint32_t dp = ntl(a.dport + j), sp = ntl(a.sport + j);
			eg[u] = fl & 1u;
			tfl[u] = eg[u] ? TUPLE_F_IN : 0u;
			meta[u] = eg[u] ? CTM_EGRESS : 0u;
			z[u] = 0;
			if (pr[u] == 1u) { /* as k_ct_prep */
				const uint32_t type = w[u] & 0xFFu;
				if (type == 3u || type == 11u || type == 12u)
					tfl[u] |= TUPLE_F_RELATED;
				else if (type == 0u)
					z[u] = 8u;
				else {
					if (type == 8u)
						z[u] = 8u << 16;
					meta[u] |= CTM_ACT_CREATE;
				}
			} else if (pr[u] == 6u || pr[u] == 17u) {
				z[u] = sp | (dp << 16);
				meta[u] |= pr[u] == 6u ? (CTM_TCP | ((w[u] & 1u) ? CTM_ACT_CLOSE : CTM_ACT_CREATE))
						       : CTM_ACT_CREATE;
			} else {
				meta[u] |= CTM_GATED;
			}
			if (pr[u] != 6u)
				w[u] = 0;
			frag[u] = !eg[u] && ((fl >> 1) & 1u);
			if (frag[u] && !(meta[u] & CTM_GATED))
				meta[u] |= CTM_FRAG;
			dec[u] = act[u] && !(meta[u] & CTM_GATED);
			fdp[u] = z[u] >> 16;
		}
		decision d[Q];
		decide4_q<Q>(s, dec, eg, frag, sa, da, fdp, pr, ep, d);
#pragma unroll
		for (int u = 0; u < Q; u++) {
			if (!act[u])
				continue;
			const uint64_t i = g + (uint64_t)u * T;
			uint32_t sec = 0, port = 0, cst = 0, id = 0, m = meta[u];
			if (dec[u]) {
				if (d[u].v >= 0) {
					m |= CTM_ALLOWED;
					port = (uint32_t)d[u].v;
				}
				id = d[u].id;
				sec = eg[u] ? (ep[u] < s.n_lxc ? s.lxc[2u * ep[u] + 1u].w : 0u) : d[u].id;
				cst = (uint32_t)(d[u].ctr + 1) | (d[u].st << 24);
			}
			uint32_t gk = ct_group(sa[u], da[u]);
			bool p2 = false;
			if (dec[u]) {
				if (pr[u] == 1u && (tfl[u] & TUPLE_F_RELATED)) {
					m |= CTM_PHASE2;
					p2 = true;
				} else {
					m |= CTM_RELX;
					gk = ct_conn_group(gk, z[u], pr[u]);
				}
			}
			reinterpret_cast<uint16_t *>(a.f2)[i] = p2 ? 1u : 0u;
			if (CGPU_CT_DFLT && a.dflt)
				a.ct_ret[i] = CT_DFLT; /* the walker stores only non-default results */
			a.identity[i] = id;
			uint4 *r = a.rec + 2u * i;
			r[0] = uint4{da[u], sa[u], z[u], pr[u] | (tfl[u] << 8) | (m << 16)};
			r[1] = uint4{w[u] | (port << 16), len[u], sec, cst};
			a.gkey[i] = (m & CTM_GATED) ? ct_fmix((uint32_t)i ^ 0x5bd1e995u) : gk;
			a.idx[i] = (uint32_t)i;
		}
	}
}

/* k_ct_prep6<false> (the plain IPv6 path) with Q packets per lane, the
 * ipcache entries from the pre-pass (k_ipc6_pre, egress fallback folded in)
 * and the policy cascades through policy_q */
template <int Q, bool SVC = false>
__global__ __launch_bounds__(256) void k_ct_prep6_q(cgpu_snapshot s, ct_args a, const uint32_t *ipc_e)
{
	const uint64_t T = (uint64_t)gridDim.x * 256u;
	const uint4 *sa16 = reinterpret_cast<const uint4 *>(a.saddr);
	const uint4 *da16 = reinterpret_cast<const uint4 *>(a.daddr);
	for (uint64_t g = (uint64_t)blockIdx.x * 256u + threadIdx.x; g < a.n; g += T * Q) {
		bool act[Q], dec[Q], eg[Q], frag[Q];
		uint32_t fdp[Q], pr[Q], ep[Q], meta[Q], tfl[Q], z[Q], w[Q], len[Q];
		/* SVC: lb6_local's outcome (svc_out[2i], target svc_out[2i + 1]):
		 * drop, translated, and the dport as lb6_xlate left it */
		bool drop[Q], xl[Q];
		uint32_t dpx[Q];
		decision d[Q];
#pragma unroll
		for (int u = 0; u < Q; u++) {
			const uint64_t i = g + (uint64_t)u * T;
			act[u] = i < a.n;
			const uint64_t j = act[u] ? i : 0u;
			const uint32_t fl = ntl(a.flags + j), sp = ntl(a.sport + j);
			uint32_t dp = ntl(a.dport + j);
			drop[u] = xl[u] = false;
			if constexpr (SVC) {
				if (fl & 1u) {
					const uint4 so = a.svc_out[2u * j];
					drop[u] = (so.x & 3u) == SVC_DROP;
					xl[u] = (so.x & 3u) == SVC_XLATED;
					if (xl[u] && (so.y & 0xFFFFu))
						dp = so.y & 0xFFFFu; /* lb6_xlate's port rewrite */
				}
			}
			dpx[u] = dp;
			pr[u] = ntl(a.proto + j);
			len[u] = ntl(a.len + j);
			ep[u] = ntl(a.ep + j);
			w[u] = ntl(a.l4 + j);
			eg[u] = fl & 1u;
			frag[u] = false; /* no fragment flag on IPv6 (bpf_lxc.c:787-789) */
			tfl[u] = eg[u] ? TUPLE_F_IN : 0u;
			meta[u] = eg[u] ? CTM_EGRESS : 0u;
			z[u] = 0;
			if (pr[u] == 58u) { /* as k_ct_prep6 */
				const uint32_t type = w[u] & 0xFFu;
				if (type >= 1u && type <= 4u)
					tfl[u] |= TUPLE_F_RELATED;
				else if (type == 129u)
					z[u] = 128u;
				else {
					if (type == 128u)
						z[u] = 128u << 16;
					meta[u] |= CTM_ACT_CREATE;
				}
			} else if (pr[u] == 6u || pr[u] == 17u) {
				z[u] = sp | (dp << 16);
				meta[u] |= pr[u] == 6u ? (CTM_TCP | ((w[u] & 1u) ? CTM_ACT_CLOSE : CTM_ACT_CREATE))
						       : CTM_ACT_CREATE;
			} else {
				meta[u] |= CTM_GATED;
			}
			if (pr[u] != 6u)
				w[u] = 0;
			dec[u] = act[u] && !drop[u] && !(meta[u] & CTM_GATED);
			fdp[u] = z[u] >> 16;
			/* decide<1>'s identity from the pre-pass entry (SVC: looked up
			 * on the translated daddr) */
			const uint32_t e = ntl(ipc_e + j);
			const uint32_t label = entry_label(s.ipc6.vals, e);
			if (eg[u]) {
				d[u].id = (e && label) ? label : s.world_id; /* cluster fallback folded into e */
			} else {
				uint32_t src = s.ingress_src_identity;
				if (src < s.health_id && e && label && label != s.cluster_id)
					src = label;
				d[u].id = src;
			}
		}
		policy_q<Q>(s, dec, eg, frag, fdp, pr, ep, d);
#pragma unroll
		for (int u = 0; u < Q; u++) {
			if (!act[u])
				continue;
			const uint64_t i = g + (uint64_t)u * T;
			const uint4 sa = ld_x4<true>(sa16 + i);
			uint4 da = ld_x4<true>(da16 + i);
			uint32_t rev = eg[u] ? 0u : (da.w & 0xFFFFu), svcw = 0; /* svcw: slave | lbf << 16 */
			if constexpr (SVC) {
				if (drop[u]) { /* as k_ct_prep6<true> */
					a.identity[i] = 0;
					reinterpret_cast<uint16_t *>(a.f2)[i] = 0u;
					if (a.xdaddr)
						reinterpret_cast<uint4 *>(a.xdaddr)[i] = da;
					if (a.xdport)
						a.xdport[i] = (uint16_t)dpx[u];
					uint4 *r = a.rec + 4u * i;
					r[0] = da;
					r[1] = sa;
					r[2] = uint4{0u, pr[u] | ((CTM_EGRESS | CTM_GATED | CTM_SVCDROP) << 16), 0u, len[u]};
					r[3] = uint4{0u, 0u, 0u, 0u};
					a.gkey[i] = ct_fmix((uint32_t)i ^ 0x5bd1e995u);
					a.idx[i] = (uint32_t)i;
					continue;
				}
				if (xl[u]) {
					const uint4 so = a.svc_out[2u * i];
					da = a.svc_out[2u * i + 1u]; /* tuple->daddr = svc->target (lb.h:475) */
					rev = so.y >> 16;
					svcw = (so.x >> 16) | ((((so.x >> 8) & LBS_ENTRY) ? LBF_LOOPBACK : 0u) << 16);
				}
				if (a.xdaddr)
					reinterpret_cast<uint4 *>(a.xdaddr)[i] = da;
				if (a.xdport)
					a.xdport[i] = (uint16_t)dpx[u];
			}
			uint32_t sec = 0, port = 0, cst = 0, id = 0, m = meta[u];
			if (dec[u]) {
				if (d[u].v >= 0) {
					m |= CTM_ALLOWED;
					port = (uint32_t)d[u].v;
				}
				id = d[u].id;
				sec = eg[u] ? (ep[u] < s.n_lxc ? s.lxc[2u * ep[u] + 1u].w : 0u) : d[u].id;
				cst = (uint32_t)(d[u].ctr + 1) | (d[u].st << 24);
			}
			uint32_t gk = ct_group(fold6(sa.x, sa.y, sa.z, sa.w), fold6(da.x, da.y, da.z, da.w));
			bool p2 = false;
			if (dec[u]) {
				if (pr[u] == 58u && (tfl[u] & TUPLE_F_RELATED)) {
					m |= CTM_PHASE2;
					p2 = true;
				} else {
					m |= CTM_RELX;
					gk = ct_conn_group(gk, z[u], pr[u]);
				}
			}
			reinterpret_cast<uint16_t *>(a.f2)[i] = p2 ? 1u : 0u;
			if (CGPU_CT_DFLT && a.dflt)
				a.ct_ret[i] = CT_DFLT; /* as k_ct_prep_q */
			a.identity[i] = id;
			uint4 *r = a.rec + 4u * i;
			r[0] = da;
			r[1] = sa;
			r[2] = uint4{z[u], pr[u] | (tfl[u] << 8) | (m << 16), w[u] | (port << 16), len[u]};
			r[3] = uint4{sec, cst, rev, svcw};
			a.gkey[i] = (m & CTM_GATED) ? ct_fmix((uint32_t)i ^ 0x5bd1e995u) : gk;
			a.idx[i] = (uint32_t)i;
		}
	}
}

/* The forward tuple's decision for the service paths' records (k_ct_prep /
 * k_ct_prep6 with SVC leave it out of their per-packet lanes): Q packets per
 * lane, packet i = g + u * (threads), every lookup stage's gathers in flight
 * together (decide4_q; v6 the trie walk with its levels in LDS as
 * k_ipc6_pre, then policy_q).  Patches the record as the per-packet prep
 * writes it: CTM_ALLOWED, the proxy port, src_sec_id (ingress: the source
 * identity), the counter slot | stage, and the identity column. */
template <class K, int Q, int NT>
__global__ __launch_bounds__(NT) void k_ct_decq(cgpu_snapshot s, ct_args a)
{
	constexpr bool V6 = K::V6 != 0;
	constexpr uint32_t RW = ct_rec<K>::RW;
	extern __shared__ __attribute__((aligned(16))) uint32_t lt[];
	uint32_t n24 = 0, nbl = 0;
	uint32_t *lbl = lt;
	if constexpr (V6) {
		n24 = v6t_lds_b24(s.ipc6);
		nbl = v6t_lds_bloom(s.ipc6);
		lbl = lt + v6t_lds_words(s.ipc6);
		if (s.ipc6.root) {
			for (uint32_t k = threadIdx.x; k < V6T_RBITS_WORDS; k += NT)
				lt[k] = s.ipc6.rbits[k];
			const uint32_t *b16 = reinterpret_cast<const uint32_t *>(s.ipc6.b24_16);
			for (uint32_t k = threadIdx.x; k < n24 * 128u; k += NT)
				lt[V6T_RBITS_WORDS + k] = b16[k];
			for (uint32_t k = threadIdx.x; k < nbl; k += NT)
				lbl[k] = s.ipc6.bl64[k];
		}
	} else {
		for (uint32_t k = threadIdx.x; k < s.ipc4c.n_dict; k += NT)
			lt[k] = s.ipc4c.dict[k];
	}
	__syncthreads();
	const uint64_t T = (uint64_t)gridDim.x * NT;
	for (uint64_t g = (uint64_t)blockIdx.x * NT + threadIdx.x; g < a.n; g += T * Q) {
		bool act[Q], eg[Q], frag[Q];
		uint32_t sa[Q], da[Q], dp[Q], pr[Q], ep[Q];
		uint4 w6[Q], rm[Q], rd[Q];
		decision d[Q];
#pragma unroll
		for (int u = 0; u < Q; u++) {
			const uint64_t i = g + (uint64_t)u * T;
			const uint64_t j = i < a.n ? i : 0u;
			const uint4 *r = a.rec + RW * j;
			/* v4: r0 = {daddr, saddr, z, proto | meta}, r1 = {w | port, len,
			 * sec, cst}; v6: r2 = {z, proto | meta, w | port, len}, r3 =
			 * {sec, cst, rev_nat, svcw} */
			rm[u] = V6 ? r[2] : r[0];
			rd[u] = V6 ? r[3] : r[1];
			const uint32_t meta = (V6 ? rm[u].y : rm[u].w) >> 16;
			act[u] = i < a.n && !(meta & CTM_GATED);
			eg[u] = meta & CTM_EGRESS;
			frag[u] = meta & CTM_FRAG;
			dp[u] = V6 ? rm[u].x >> 16 : rm[u].z >> 16;
			pr[u] = (V6 ? rm[u].y : rm[u].w) & 0xFFu;
			ep[u] = a.ep[j];
			sa[u] = V6 ? 0u : rm[u].y;
			da[u] = V6 ? 0u : rm[u].x;
			w6[u] = make_uint4(0, 0, 0, 0);
			if (V6)
				w6[u] = v6_host_words(eg[u] ? r[0] : r[1]);
		}
		if constexpr (V6) {
			/* decide<1>'s identity (bpf_lxc.c:170-187 / bpf_netdev.c:203-211) */
			uint32_t e[Q];
			v6t_lookup_q<Q>(s.ipc6, lt, n24 != 0u, w6, act, e, nbl ? lbl : nullptr);
#pragma unroll
			for (int u = 0; u < Q; u++) {
				const uint32_t label = entry_label(s.ipc6.vals, e[u]);
				const bool in_cluster = w6[u].x == bswap32(s.router_ip64[0]) &&
							w6[u].y == bswap32(s.router_ip64[1]);
				if (eg[u]) {
					d[u].id = (e[u] && label) ? label : (in_cluster ? s.cluster_id : s.world_id);
				} else {
					uint32_t src = s.ingress_src_identity;
					if (src < s.health_id && e[u] && label && label != s.cluster_id)
						src = label;
					d[u].id = src;
				}
			}
		} else {
			ident4_q<Q>(s, lt, act, eg, sa, da, d);
		}
		policy_q<Q>(s, act, eg, frag, dp, pr, ep, d);
#pragma unroll
		for (int u = 0; u < Q; u++) {
			const uint64_t i = g + (uint64_t)u * T;
			if (!act[u])
				continue;
			const uint32_t allowed = d[u].v >= 0 ? (CTM_ALLOWED << 16) : 0u;
			const uint32_t port = d[u].v >= 0 ? (uint32_t)d[u].v << 16 : 0u;
			const uint32_t cst = (uint32_t)(d[u].ctr + 1) | (d[u].st << 24);
			uint4 *r = a.rec + RW * i;
			if (V6) {
				r[2] = make_uint4(rm[u].x, rm[u].y | allowed, rm[u].z | port, rm[u].w);
				r[3] = make_uint4(eg[u] ? rd[u].x : d[u].id, cst, rd[u].z, rd[u].w);
			} else {
				r[0] = make_uint4(rm[u].x, rm[u].y, rm[u].z, rm[u].w | allowed);
				r[1] = make_uint4(rd[u].x | port, rd[u].y, eg[u] ? rd[u].z : d[u].id, cst);
			}
			a.identity[i] = d[u].id;
		}
	}
}

template <class K> static void launch_ct_decq(const cgpu_snapshot &s, const ct_args &a, hipStream_t st)
{
	if (!(K::V6 ? CGPU_CT_SVC_DECQ6 : CGPU_CT_SVC_DECQ))
		return;
	if constexpr (K::V6 != 0) {
		/* as k_ipc6_pre: the staged levels once per CU */
		constexpr int Q = 2, NT = 1024;
		const size_t lds = (size_t)(v6t_lds_words(s.ipc6) + v6t_lds_bloom(s.ipc6)) * 4u;
		const unsigned res = resident_blocks((const void *)k_ct_decq<K, Q, NT>, NT, lds);
		const unsigned g = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((a.n + Q * NT - 1) / (Q * NT), res));
		hipLaunchKernelGGL((k_ct_decq<K, Q, NT>), dim3(g), dim3(NT), lds, st, s, a);
	} else {
		constexpr int Q = CGPU_CT_Q;
		const size_t lds = (size_t)s.ipc4c.n_dict * 4u;
		const unsigned g = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((a.n + 256 * Q - 1) / (256 * Q), 8192));
		hipLaunchKernelGGL((k_ct_decq<K, Q, 256>), dim3(g), dim3(256), lds, st, s, a);
	}
}

/* phase 2 of the service path, in two sub-phases: candidate 4i = packet i
 * if it runs in phase 2, 4i + 1 = packet i's owed address entry (kept
 * whatever phase 1 decided: the walk checks CT_ADDRP), 4i + 2 = the ICMP
 * entry phase 1 owed (CT_RELP).  Phase 2a: the ICMP errors of ordinary
 * pairs and the ICMP entries (all in ordinary pairs); phase 2b: the special
 * pairs ({a, a}, 0, IPV4_LOOPBACK) - their packets and the address entries,
 * which only land there.  2a writes and reads ordinary pairs only and may
 * owe into 2b, 2b runs after it; a 2b packet that owes runs the batch
 * serially.  The plain path's flags come from its prep and walk (ct_args.f2,
 * two per packet). */
__global__ __launch_bounds__(256) void k_ct_owed_flags(ct_args a, uint32_t *f4, uint32_t phase)
{
	const uint64_t stride = (uint64_t)gridDim.x * 256u;
	for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < a.n; i += stride) {
		/* the packet's class (k_ct_prep: phase-2 packet of an ordinary /
		 * special pair, owes an address entry, owes its ICMP entry) */
		const uint32_t c = a.pcls[i];
		uint32_t f;
		if (phase == 0u) {
			const bool rel = (c & PCL_RELX) && (a.ct_ret[i] & CT_RELP);
			f = (c & PCL_P2A ? 1u : 0u) | (rel ? 1u << 16 : 0u);
		} else {
			f = (c & PCL_P2B ? 1u : 0u) | (c & PCL_ADDRX ? 1u << 8 : 0u);
		}
		f4[i] = f;
	}
}

/* group key of each selected candidate: the address pair (packet: its own,
 * owed entry: the entry's), or, when no packet runs in phase 2, the owed
 * entry's whole key (blind BPF_ANY writes of different keys commute) */
/* Phase 2b of the service path: the pairs its PACKETS run in (candidates
 * of kind 0), as a bloom filter over their pair hashes: an owed address
 * entry whose pair has no such packet is a blind BPF_ANY write that no
 * phase-2 read sees, so k_ct_owed_keys groups it by its whole key (entries
 * of one key stay in batch order) instead of serialising the pair's */
#define OWED_BLOOM_WORDS (1u << 15) /* 2^20 bits */
#define LH_B 256u /* head ranges of the device-side longest-first ordering */
template <class K> __global__ __launch_bounds__(256) void k_ct_owed_bloom(ct_args a, uint32_t m, uint32_t *bl)
{
	for (uint32_t j = blockIdx.x * 256u + threadIdx.x; j < m; j += gridDim.x * 256u) {
		const uint32_t v = a.idx[j];
		if ((v & 3u) != 0u)
			continue;
		const uint4 k = ct_rec<K>::load(a.rec, v >> 2, false).key();
		const uint32_t h = ct_group(k.x, k.y);
		atomicOr(&bl[(h >> 5) & (OWED_BLOOM_WORDS - 1u)], 1u << (h & 31u));
	}
}

/* bl (the service path's phase 2b): k_ct_owed_bloom's filter, or nullptr */
template <class K>
__global__ __launch_bounds__(256) void k_ct_owed_keys(ct_args a, uint32_t m, uint32_t by_key,
						     const uint32_t *bl = nullptr)
{
	for (uint32_t j = blockIdx.x * 256u + threadIdx.x; j < m; j += gridDim.x * 256u) {
		const uint32_t v = a.idx[j], i = K::ADDR ? v >> 2 : v >> 1;
		const ct_rec<K> r = ct_rec<K>::load(a.rec, i, false);
		if constexpr (K::ADDR) {
			uint4 k = r.key();
			if ((v & 3u) == 1u)
				k = ct_addr_key(CtK4::reversed(k), r.pkt());
			else if ((v & 3u) == 2u)
				k = CtK4::related(CtK4::reversed(k));
			const uint32_t h = ct_group(k.x, k.y);
			const bool alone = bl && (v & 3u) == 1u &&
					   !((bl[(h >> 5) & (OWED_BLOOM_WORDS - 1u)] >> (h & 31u)) & 1u);
			a.gkey[j] = (by_key || alone) ? ct_hash(k.x, k.y, k.z, k.w) : h;
		} else if constexpr (K::V6 != 0) {
			/* an ICMP entry carries its packet's pair */
			const typename K::key k = r.key();
			a.gkey[j] = ct_group(fold6(k.d.x, k.d.y, k.d.z, k.d.w), fold6(k.s.x, k.s.y, k.s.z, k.s.w));
		} else {
			const uint4 k = r.key();
			a.gkey[j] = ct_group(k.x, k.y);
		}
	}
}

/* length of every group (keys) and its start (values), for the longest-
 * first sort */
__global__ __launch_bounds__(256) void k_ct_lens(const uint32_t *heads, uint32_t nh, uint64_t n,
						 uint32_t *len, uint32_t *pos)
{
	for (uint32_t h = blockIdx.x * 256u + threadIdx.x; h < nh; h += gridDim.x * 256u) {
		const uint32_t p0 = heads[h];
		len[h] = (uint32_t)((h + 1u < nh ? (uint64_t)heads[h + 1u] : n) - p0);
		pos[h] = p0;
	}
}

/* a group starts where the SORTED bits of the key change (keys that agree
 * on them are one group even if their other bits differ) */
__global__ __launch_bounds__(256) void k_ct_heads(const uint32_t *g, uint8_t *head, uint64_t n, uint32_t mask)
{
	const uint64_t stride = (uint64_t)gridDim.x * 256u;
	for (uint64_t p = (uint64_t)blockIdx.x * 256u + threadIdx.x; p < n; p += stride)
		head[p] = (p == 0 || ((g[p] ^ g[p - 1]) & mask)) ? 1u : 0u;
}

/* ct_lookup6's tuple setup (conntrack.h:308-378) and the forward tuple's
 * decision, as k_ct_prep; IPv6 has no fragment flag (bpf_lxc.c:787-789) and
 * an ingress entry carries the reverse NAT index ipv6_policy derives from
 * the destination address, daddr.s6_addr32[3] & 0xFFFF (bpf_lxc.c:748). */
template <bool SVC>
__global__ __launch_bounds__(256) void k_ct_prep6(cgpu_snapshot s, ct_args a)
{
	const uint64_t stride = (uint64_t)gridDim.x * 256u;
	const uint4 *sa16 = reinterpret_cast<const uint4 *>(a.saddr);
	const uint4 *da16 = reinterpret_cast<const uint4 *>(a.daddr);
	for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < a.n; i += stride) {
		const uint32_t fl = a.flags[i], pr = a.proto[i], len = a.len[i], ep = a.ep[i];
		uint32_t w = a.l4[i], dp = a.dport[i];
		const uint4 sa = ld_x4<true>(sa16 + i);
		uint4 da = ld_x4<true>(da16 + i);
		const bool egress = fl & 1u;
		uint32_t tfl = egress ? TUPLE_F_IN : 0u, z = 0, meta = egress ? CTM_EGRESS : 0u;
		uint32_t svcw = 0; /* slave | lbf << 16 */
		uint32_t rev = egress ? 0u : (da.w & 0xFFFFu);
		if constexpr (SVC) {
			/* lb6_local's outcome (svc_out[2i], target svc_out[2i + 1]) */
			const uint4 so = egress ? a.svc_out[2u * i] : make_uint4(SVC_NONE, 0, 0, 0);
			if ((so.x & 3u) == SVC_DROP) {
				a.identity[i] = 0;
				reinterpret_cast<uint16_t *>(a.f2)[i] = 0u;
				if (a.xdaddr)
					reinterpret_cast<uint4 *>(a.xdaddr)[i] = da;
				if (a.xdport)
					a.xdport[i] = (uint16_t)dp;
				uint4 *r = a.rec + 4u * i;
				r[0] = da;
				r[1] = sa;
				r[2] = uint4{0u, pr | ((CTM_EGRESS | CTM_GATED | CTM_SVCDROP) << 16), 0u, len};
				r[3] = uint4{0u, 0u, 0u, 0u};
				a.gkey[i] = ct_fmix((uint32_t)i ^ 0x5bd1e995u);
				a.idx[i] = (uint32_t)i;
				continue;
			}
			if ((so.x & 3u) == SVC_XLATED) {
				da = a.svc_out[2u * i + 1u]; /* tuple->daddr = svc->target (lb.h:475) */
				if (so.y & 0xFFFFu)
					dp = so.y & 0xFFFFu; /* lb6_xlate's port rewrite */
				rev = so.y >> 16;
				svcw = (so.x >> 16) | ((((so.x >> 8) & LBS_ENTRY) ? LBF_LOOPBACK : 0u) << 16);
			}
			if (a.xdaddr)
				reinterpret_cast<uint4 *>(a.xdaddr)[i] = da;
			if (a.xdport)
				a.xdport[i] = (uint16_t)dp;
		}
		if (pr == 58u) {
			const uint32_t type = w & 0xFFu;
			if (type >= 1u && type <= 4u) /* DEST_UNREACH, PKT_TOOBIG, TIME_EXCEED, PARAMPROB */
				tfl |= TUPLE_F_RELATED;
			else if (type == 129u) /* ECHO_REPLY: tuple->dport = ICMPV6_ECHO_REQUEST */
				z = 128u;
			else {
				if (type == 128u) /* ECHO_REQUEST: tuple->sport = type */
					z = 128u << 16;
				meta |= CTM_ACT_CREATE;
			}
		} else if (pr == 6u || pr == 17u) {
			z = (uint32_t)a.sport[i] | (dp << 16);
			if (pr == 6u)
				meta |= CTM_TCP | ((w & 1u) ? CTM_ACT_CLOSE : CTM_ACT_CREATE);
			else
				meta |= CTM_ACT_CREATE;
		} else {
			meta |= CTM_GATED;
		}
		if (pr != 6u)
			w = 0; /* union tcp_flags stays zero (conntrack.h:294) */
		uint32_t sec = 0, port = 0, cst = 0, id = 0;
		if (!(meta & CTM_GATED)) {
			if (egress)
				sec = ep < s.n_lxc ? s.lxc[2u * ep + 1u].w : 0u; /* SECLABEL */
			if constexpr (!SVC || !CGPU_CT_SVC_DECQ6) {
				const decision d = decide<1>(s, egress, false, 0u, 0u, sa, da, z >> 16, pr, ep);
				if (d.v >= 0) {
					meta |= CTM_ALLOWED;
					port = (uint32_t)d.v;
				}
				id = d.id;
				if (!egress)
					sec = d.id;
				cst = (uint32_t)(d.ctr + 1) | (d.st << 24);
			} /* SVC: k_ct_decq, Q packets per lane */
		}
		uint32_t g = ct_group(fold6(sa.x, sa.y, sa.z, sa.w), fold6(da.x, da.y, da.z, da.w));
		{ /* phase 1 by connection, as k_ct_prep (ct_create6 writes no address
		   * entry, so the service path groups the same way) */
			bool p2 = false;
			if (!(meta & CTM_GATED)) {
				if (pr == 58u && (tfl & TUPLE_F_RELATED)) {
					meta |= CTM_PHASE2;
					p2 = true;
				} else {
					meta |= CTM_RELX;
					g = ct_conn_group(g, z, pr);
				}
			}
			reinterpret_cast<uint16_t *>(a.f2)[i] = p2 ? 1u : 0u;
		}
		a.identity[i] = id;
		uint4 *r = a.rec + 4u * i;
		r[0] = da;
		r[1] = sa;
		r[2] = uint4{z, pr | (tfl << 8) | (meta << 16), w | (port << 16), len};
		r[3] = uint4{sec, cst, rev, svcw};
		a.gkey[i] = (meta & CTM_GATED) ? ct_fmix((uint32_t)i ^ 0x5bd1e995u) : g;
		a.idx[i] = (uint32_t)i;
	}
}

/* A lane's cache of the map entries its group touched.  The lane owns every
 * key of its group (no other lane inserts, updates or deletes one), so a
 * cached entry - present with its row, or absent with the slot an insert
 * may start from - stays exact for the whole group: a connection's packets
 * cost one probe per distinct key instead of one per packet.  Rows are
 * written back (write-through) when evicted and at the end of the group.
 * CTC entries, round-robin replacement, every access an unrolled select so
 * the cache lives in VGPRs. */
#ifndef CTC
#define CTC 4 /* 3 ways measured 14 % slower (more re-probes) */
#endif
#ifndef CGPU_CT_CREATE_LOOP
#define CGPU_CT_CREATE_LOOP 1 /* the service step's creates through one update call site */
#endif
#define CTC_VALID 0x10000u
#define CTC_NEG 0x20000u
#define CTC_DIRTY 0x40000u

/* One cache entry.  The CTC entries are SEPARATE locals of the walker (not
 * an array, not members of one aggregate) and every access below names
 * them one by one: with an array, instcombine folds the unrolled
 * selects back into a dynamically indexed load and the cache lands in
 * scratch memory.  The key's meta word carries nexthdr | flags << 8 |
 * CTC_*. */
template <class K> struct ctc_ent {
	typename K::key key;
	uint32_t pos;
	ct_row row;
};

template <class K> struct ct_cache {
	ctc_ent<K> &e0, &e1;
#if CTC >= 3
	ctc_ent<K> &e2;
#endif
#if CTC == 4
	ctc_ent<K> &e3;
#endif
	uint32_t next;
	uint32_t pend; /* map stores of this lane not yet waited for */
};

template <class K, typename F> __device__ __forceinline__ void ctc_each(ct_cache<K> &c, F &&f)
{
	f(c.e0, 0);
	f(c.e1, 1);
#if CTC >= 3
	f(c.e2, 2);
#endif
#if CTC == 4
	f(c.e3, 3);
#endif
}

/* Every helper reads all entries unconditionally and writes them back
 * through selects: a branch per entry would let SimplifyCFG sink the four
 * identical stores into one store through a phi of entry addresses, which
 * again keeps the cache out of registers. */
__device__ __forceinline__ bool ctc_dirty(uint32_t w)
{
	return (w & (CTC_VALID | CTC_NEG | CTC_DIRTY)) == (CTC_VALID | CTC_DIRTY);
}

template <class K> __device__ __forceinline__ void ctc_flush(const ct_table &T, ct_cache<K> &c)
{
	ctc_each(c, [&](ctc_ent<K> &e, int) {
		const uint32_t w = K::meta(e.key), p = e.pos;
		const ct_row r = e.row;
		if (ctc_dirty(w)) {
			ct_row_store(T, p, r);
			c.pend = 1;
		}
		K::meta(e.key) = 0;
	});
	c.next = 0;
}

template <class K> __device__ __forceinline__ uint32_t ctc_state(ct_cache<K> &c, int i)
{
	uint32_t w = 0;
	ctc_each(c, [&](ctc_ent<K> &e, int j) { w = i == j ? K::meta(e.key) : w; });
	return w;
}

template <class K> __device__ __forceinline__ uint32_t ctc_pos(ct_cache<K> &c, int i)
{
	uint32_t p = 0;
	ctc_each(c, [&](ctc_ent<K> &e, int j) { p = i == j ? e.pos : p; });
	return p;
}

__device__ __forceinline__ ct_row selrow(bool t, const ct_row &a, const ct_row &b)
{
	return ct_row{sel4(t, a.a, b.a), sel4(t, a.b, b.b), sel4(t, a.c, b.c),
		      uint2{t ? a.d.x : b.d.x, t ? a.d.y : b.d.y}};
}

template <class K> __device__ __forceinline__ ct_row ctc_row(ct_cache<K> &c, int i)
{
	ct_row r{};
	ctc_each(c, [&](ctc_ent<K> &e, int j) { r = selrow(i == j, e.row, r); });
	return r;
}

/* entry i := present at pos with row r (dirty) */
template <class K> __device__ __forceinline__ void ctc_put(ct_cache<K> &c, int i, uint32_t pos, const ct_row &r)
{
	ctc_each(c, [&](ctc_ent<K> &e, int j) {
		const bool t = i == j;
		K::meta(e.key) = t ? (K::meta(e.key) & 0xFFFFu) | CTC_VALID | CTC_DIRTY : K::meta(e.key);
		e.pos = t ? pos : e.pos;
		e.row = selrow(t, r, e.row);
	});
}

/* entry i := absent, inserts may start at pos */
template <class K> __device__ __forceinline__ void ctc_drop(ct_cache<K> &c, int i, uint32_t pos)
{
	ctc_each(c, [&](ctc_ent<K> &e, int j) {
		const bool t = i == j;
		K::meta(e.key) = t ? (K::meta(e.key) & 0xFFFFu) | CTC_VALID | CTC_NEG : K::meta(e.key);
		e.pos = t ? pos : e.pos;
	});
}

/* the cache entry of k, probing the map on a miss */
template <class K>
__device__ __forceinline__ int ctc_get(const ct_table &T, ct_cache<K> &c, const typename K::key &k)
{
	int hit = -1;
	ctc_each(c, [&](ctc_ent<K> &e, int j) {
		hit = ((K::meta(e.key) & CTC_VALID) && K::same(e.key, k)) ? j : hit;
	});
	if (hit >= 0)
		return hit;
	const int v = (int)c.next;
	c.next = v + 1 == CTC ? 0u : (uint32_t)v + 1u;
	uint32_t from;
	const int slot = ct_find<K>(T, k, &from, c.pend);
	ct_row r{};
	if (slot >= 0)
		r = ct_row_load(T, (uint32_t)slot);
	/* write back the victim (a different key: the probe above cannot have
	 * read its row) */
	uint32_t vw = 0, vp = 0;
	ct_row vr{};
	ctc_each(c, [&](ctc_ent<K> &e, int j) {
		vw = j == v ? K::meta(e.key) : vw;
		vp = j == v ? e.pos : vp;
		vr = selrow(j == v, e.row, vr);
	});
	if (ctc_dirty(vw)) {
		ct_row_store(T, vp, vr);
		c.pend = 1;
	}
	typename K::key nk = k;
	K::meta(nk) = (K::cmeta(k) & 0xFFFFu) | CTC_VALID | (slot < 0 ? CTC_NEG : 0u);
	const uint32_t np = slot >= 0 ? (uint32_t)slot : from;
	ctc_each(c, [&](ctc_ent<K> &e, int j) {
		const bool t = j == v;
		e.key = K::sel(t, nk, e.key);
		e.pos = t ? np : e.pos;
		e.row = selrow(t, r, e.row);
	});
	return v;
}

/* the cache entry of k, or -1 (no probe) */
template <class K> __device__ __forceinline__ int ctc_find(ct_cache<K> &c, const typename K::key &k)
{
	int hit = -1;
	ctc_each(c, [&](ctc_ent<K> &e, int j) {
		hit = ((K::meta(e.key) & CTC_VALID) && K::same(e.key, k)) ? j : hit;
	});
	return hit;
}

/* One probe chain of ct_find, advanced a slot per round so that the chains
 * of several keys have their loads in flight together.  slot: -3 not
 * probed, -2 running, -1 absent (inserts may start at ff), else found. */
struct ct_chain {
	uint32_t h, ff, n;
	int slot;
};

/* s = the slot as loaded; cm = its meta word re-read at the coherence point
 * when the plain read was EMPTY (ct_find's rule) */
template <class K>
__device__ __forceinline__ void ct_chain_eval(const ct_table &T, const typename K::key &k, typename K::key s,
					      uint32_t cm, ct_chain &ch)
{
	if (ch.slot != -2)
		return;
	uint32_t tag = K::meta(s) >> 16;
	if (tag == CT_TAG_EMPTY) {
		K::meta(s) = cm;
		tag = cm >> 16;
		if (tag == CT_TAG_EMPTY) {
			ch.slot = -1;
			if (ch.ff == 0xFFFFFFFFu)
				ch.ff = ch.h;
			return;
		}
		K::reload(T, ch.h, s);
	}
	if (tag == CT_TAG_LIVE && K::same(s, k)) {
		ch.slot = (int)ch.h;
		return;
	}
	if (tag == CT_TAG_TOMB && ch.ff == 0xFFFFFFFFu)
		ch.ff = ch.h;
	ch.h = (ch.h + 1u) & T.mask;
	if (++ch.n > T.mask)
		ch.slot = -1;
}

template <class K>
__device__ __forceinline__ void ct_find3(const ct_table &T, const typename K::key &k0, const typename K::key &k1,
					 const typename K::key &k2, ct_chain &c0, ct_chain &c1, ct_chain &c2,
					 uint32_t &pend)
{
	ct_pend_wait(pend);
	c0.h = K::hash(k0) & T.mask;
	c1.h = K::hash(k1) & T.mask;
	c2.h = K::hash(k2) & T.mask;
	while (c0.slot == -2 || c1.slot == -2 || c2.slot == -2) {
		typename K::key s0 = k0, s1 = k1, s2 = k2;
		if (c0.slot == -2)
			s0 = K::load(T, c0.h);
		if (c1.slot == -2)
			s1 = K::load(T, c1.h);
		if (c2.slot == -2)
			s2 = K::load(T, c2.h);
		uint32_t m0 = 0, m1 = 0, m2 = 0;
		if (c0.slot == -2 && (K::meta(s0) >> 16) == CT_TAG_EMPTY)
			m0 = __hip_atomic_load(K::tagp(T, c0.h), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		if (c1.slot == -2 && (K::meta(s1) >> 16) == CT_TAG_EMPTY)
			m1 = __hip_atomic_load(K::tagp(T, c1.h), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		if (c2.slot == -2 && (K::meta(s2) >> 16) == CT_TAG_EMPTY)
			m2 = __hip_atomic_load(K::tagp(T, c2.h), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		ct_chain_eval<K>(T, k0, s0, m0, c0);
		ct_chain_eval<K>(T, k1, s1, m1, c1);
		ct_chain_eval<K>(T, k2, s2, m2, c2);
	}
}

/* put probed key k (chain ch, row r) into the cache, in the next entry
 * round-robin that holds none of the wanted keys k0..k2 */
template <class K>
__device__ __forceinline__ void ctc_install(const ct_table &T, ct_cache<K> &c, const typename K::key &k,
					    const ct_chain &ch, const ct_row &r, const typename K::key &k0,
					    const typename K::key &k1, const typename K::key &k2)
{
	if (ch.slot == -3 || ctc_find<K>(c, k) >= 0)
		return;
	uint32_t keep = 0;
	ctc_each(c, [&](ctc_ent<K> &e, int j) {
		const bool v = K::meta(e.key) & CTC_VALID;
		if (v && (K::same(e.key, k0) || K::same(e.key, k1) || K::same(e.key, k2)))
			keep |= 1u << j;
	});
	int v = -1;
#pragma unroll
	for (int t = 0; t < CTC; t++) {
		int j = (int)c.next + t;
		j = j >= CTC ? j - CTC : j;
		v = (v < 0 && !((keep >> j) & 1u)) ? j : v;
	}
	c.next = v + 1 == CTC ? 0u : (uint32_t)v + 1u;
	uint32_t vw = 0, vp = 0;
	ct_row vr{};
	ctc_each(c, [&](ctc_ent<K> &e, int j) {
		vw = j == v ? K::meta(e.key) : vw;
		vp = j == v ? e.pos : vp;
		vr = selrow(j == v, e.row, vr);
	});
	if (ctc_dirty(vw)) {
		ct_row_store(T, vp, vr);
		c.pend = 1;
	}
	typename K::key nk = k;
	K::meta(nk) = (K::cmeta(k) & 0xFFFFu) | CTC_VALID | (ch.slot < 0 ? CTC_NEG : 0u);
	const uint32_t np = ch.slot >= 0 ? (uint32_t)ch.slot : ch.ff;
	ctc_each(c, [&](ctc_ent<K> &e, int j) {
		const bool t = j == v;
		e.key = K::sel(t, nk, e.key);
		e.pos = t ? np : e.pos;
		e.row = selrow(t, r, e.row);
	});
}

/* The keys a step will need (w0..w2 select them), probed together when
 * the cache lacks them: a new connection's reply key, forward key and ICMP
 * key cost one round of loads instead of three dependent probes */
template <class K>
__device__ __forceinline__ void ctc_prefetch(const ct_table &T, ct_cache<K> &c, const typename K::key &k0,
					     const typename K::key &k1, const typename K::key &k2, bool w0, bool w1,
					     bool w2)
{
#ifndef CGPU_CT_PREFETCH
	/* off: probing the step's keys together measured slower than probing
	 * them as the step needs them (ct config 21.9 -> 18.5 ms per 64M-packet
	 * batch, profiles/r3_ct_ab): the extra chains cost more than the latency
	 * they overlap, and most packets need only the reply key */
	return;
#endif
	ct_chain c0{0, 0xFFFFFFFFu, 0, -3}, c1 = c0, c2 = c0;
	/* one probe per distinct key: an ICMP error's forward key IS its
	 * related key (ports 0, RELATED set), and two cache entries of one key
	 * would lose updates and insert it twice */
	w1 = w1 && !(w0 && K::same(k1, k0));
	w2 = w2 && !(w0 && K::same(k2, k0)) && !(w1 && K::same(k2, k1));
	if (w0 && ctc_find<K>(c, k0) < 0)
		c0.slot = -2;
	if (w1 && ctc_find<K>(c, k1) < 0)
		c1.slot = -2;
	if (w2 && ctc_find<K>(c, k2) < 0)
		c2.slot = -2;
	if (c0.slot == -3 && c1.slot == -3 && c2.slot == -3)
		return;
	ct_find3<K>(T, k0, k1, k2, c0, c1, c2, c.pend);
	ct_row r0{}, r1{}, r2{};
	if (c0.slot >= 0)
		r0 = ct_row_load(T, (uint32_t)c0.slot);
	if (c1.slot >= 0)
		r1 = ct_row_load(T, (uint32_t)c1.slot);
	if (c2.slot >= 0)
		r2 = ct_row_load(T, (uint32_t)c2.slot);
	ctc_install<K>(T, c, k0, c0, r0, k0, k1, k2);
	ctc_install<K>(T, c, k1, c1, r1, k0, k1, k2);
	ctc_install<K>(T, c, k2, c2, r2, k0, k1, k2);
}

/* BPF_ANY update of k (ct_create's map_update_elem) through the cache */
template <class K>
__device__ __forceinline__ bool ctc_update(const ct_table &T, const ct_acct &A, ct_cache<K> &c,
					   const typename K::key &k, const ct_row &e)
{
	const int i = ctc_get<K>(T, c, k);
	uint32_t pos = ctc_pos(c, i);
	if (ctc_state(c, i) & CTC_NEG) {
		const int slot = pos == 0xFFFFFFFFu ? -1 : ct_insert<K>(T, A, k, pos);
		if (slot < 0)
			return false;
		pos = (uint32_t)slot;
		c.pend = 1;
	}
	ctc_put(c, i, pos, e);
	return true;
}

/* BPF_ANY update of k whose capacity was reserved earlier (an owed address
 * entry): an insert consumes the reservation, an existing key returns it */
template <class K>
__device__ __forceinline__ void ctc_update_owed(const ct_table &T, const ct_acct &A, ct_cache<K> &c,
						const typename K::key &k, const ct_row &e)
{
	const int i = ctc_get<K>(T, c, k);
	uint32_t pos = ctc_pos(c, i);
	if (ctc_state(c, i) & CTC_NEG) {
		const int slot = pos == 0xFFFFFFFFu ? -1 : ct_insert<K, false>(T, A, k, pos);
		if (slot < 0)
			return; /* no free slot on the chain: the slot table is 2x CT_MAP_SIZE */
		pos = (uint32_t)slot;
		c.pend = 1;
	} else {
		atomicAdd(A.live, 1);
	}
	ctc_put(c, i, pos, e);
}

/* the entry ct_create4 writes for packet q (before the ICMP entry's
 * seen_non_syn) */
template <class K> __device__ __forceinline__ ct_row ct_new_row(const ct_pkt &q, bool ingress, uint32_t now)
{
	const bool tcp = q.meta & CTM_TCP;
	ct_row e{};
	ct_timeout(e, now, tcp, ingress, tcp ? 1u : 0u); /* seen_flags.syn = is_tcp: bit 0 */
	if (ingress)
		e.a = uint4{1u, 0u, q.len, 0u};
	else
		e.b = uint4{1u, 0u, q.len, 0u};
	e.c.y |= q.revnat << 16; /* rev_nat_index */
	if (K::SVC) {
		if (q.lbf & LBF_LOOPBACK)
			e.c.y |= CTB_LB_LOOPBACK;
		e.c.z |= q.slave;
	}
	e.c.w = q.sec; /* src_sec_id */
	return e;
}

/* One packet of a group: ct_lookup4 / ct_lookup6 (conntrack.h:441-561 /
 * :288-412) and ct_create4 / ct_create6 (:653-744 / :588-639), with the
 * policy outcome of the endpoint programs (bpf_lxc.c:506-537 / :918-937,
 * :192-203 / :776-800).  k = the reply-direction tuple of the first lookup. */
template <class K>
__device__ __forceinline__ uint32_t ct_step(const ct_table &T, const ct_acct &A, ct_cache<K> &c,
					   typename K::key k, const ct_pkt &q, uint32_t now)
{
	const uint32_t meta = q.meta;
	const bool ingress = !(meta & CTM_EGRESS);
	{
		/* reply key not cached, or cached absent: fetch it, the forward key
		 * and (when the packet may create) the ICMP key in one round */
		const int c1 = ctc_find<K>(c, k);
		if (c1 < 0 || (ctc_state(c, c1) & CTC_NEG)) {
			const typename K::key fk = K::reversed(k);
			ctc_prefetch<K>(T, c, k, fk, K::related(fk), c1 < 0, true, (meta & CTM_ALLOWED) != 0);
		}
	}
	int ci = ctc_get<K>(T, c, k);
	uint32_t ret;
	if (!(ctc_state(c, ci) & CTC_NEG)) {
		ret = ((K::cmeta(k) >> 8) & TUPLE_F_RELATED) ? CT_RELATED : CT_REPLY;
	} else {
		k = K::reversed(k);
		ci = ctc_get<K>(T, c, k);
		ret = (ctc_state(c, ci) & CTC_NEG) ? CT_NEW : CT_ESTABLISHED;
	}
	if (ret != CT_NEW) {
		ct_row e = ctc_row(c, ci);
		ct_hit(e, meta, ingress, q.w, q.len, now);
		ctc_put(c, ci, ctc_pos(c, ci), e);
	}
	if (ret < CT_REPLY && !(meta & CTM_ALLOWED)) {
		if (ret == CT_ESTABLISHED) { /* ct_delete4 / ct_delete6 */
			const uint32_t slot = ctc_pos(c, ci);
			ct_erase<K>(T, A, slot);
			ctc_drop(c, ci, slot);
		}
		return ret;
	}
	if (ret != CT_NEW)
		return ret;
	/* ct_create: the forward entry, the address entry (service step only),
	 * then the ICMP entry relating errors */
	const ct_row e = ct_new_row<K>(q, ingress, now);
	uint32_t owed = 0;
	if (K::ADDR && CGPU_CT_CREATE_LOOP) {
	/* the service step's creates in order, t = 0 the forward entry, 1 the
	 * address entry, 2 the ICMP entry, through ONE map-update call site:
	 * three inlined copies took the CtK4S walker to 256 VGPRs with spills,
	 * one 186 (the plain walkers keep the straight line, which fits their
	 * occupancy budget) */
#pragma unroll 1
	for (int t = 0; t < 3; t++) {
		typename K::key kt = k;
		ct_row et = e;
		if (t == 1) {
			if constexpr (!K::ADDR) {
				continue;
			} else {
				const uint32_t am = q.lbf >> 1;
				if (am == AM_INLINE) {
					kt = ct_addr_key(k, q);
				} else {
					/* AM_DEFER: the entry lies in another address pair's
					 * group: reserve its capacity now (the reference's
					 * update fails here when the map is full), write it
					 * in phase 2 */
					if (am == AM_DEFER) {
						if (!ct_take_k<K>(T, A, K::hash(k)))
							return CT_NEW | CT_FAIL;
						owed = CT_ADDRP;
					}
					continue;
				}
			}
		} else if (t == 2) {
			et.c.y |= CTB_SEEN_NON_SYN;
			if (meta & CTM_RELX) {
				/* the ICMP entry lies in the address pair's phase-2 group:
				 * reserve its capacity now (where the reference's update
				 * would fail), write it in phase 2 in batch order */
				if (!ct_take_k<K>(T, A, K::hash(k)))
					return CT_NEW | CT_FAIL | owed;
				return CT_NEW | CT_RELP | owed;
			}
			kt = K::related(k);
		}
		if (!ctc_update<K>(T, A, c, kt, et))
			return CT_NEW | CT_FAIL | owed;
	}
	return CT_NEW | owed;
	}
	if (!ctc_update<K>(T, A, c, k, e))
		return CT_NEW | CT_FAIL;
	if constexpr (K::ADDR) {
		const uint32_t am = q.lbf >> 1;
		if (am == AM_INLINE) {
			if (!ctc_update<K>(T, A, c, ct_addr_key(k, q), e))
				return CT_NEW | CT_FAIL;
		} else if (am == AM_DEFER) {
			if (!ct_take_k<K>(T, A, K::hash(k)))
				return CT_NEW | CT_FAIL;
			owed = CT_ADDRP;
		}
	}
	ct_row e2 = e;
	e2.c.y |= CTB_SEEN_NON_SYN;
	if (meta & CTM_RELX) {
		if (!ct_take_k<K>(T, A, K::hash(k)))
			return CT_NEW | CT_FAIL | owed;
		return CT_NEW | CT_RELP | owed;
	}
	if (!ctc_update<K>(T, A, c, K::related(k), e2))
		return CT_NEW | CT_FAIL | owed;
	return CT_NEW | owed;
}

/* ---- the stateful service step: lb4_local with CONNTRACK (lb.h:700-775) ----
 * Its conntrack keys carry TUPLE_F_SERVICE (4) and nothing else in the
 * datapath builds such a key (ct_lookup4 sets TUPLE_F_IN / TUPLE_F_OUT |
 * RELATED for CT_EGRESS / CT_INGRESS; ct_create4's address entry TUPLE_F_IN
 * or the tuple's flags), so the service keyspace is disjoint from the
 * endpoint's and the service step of the whole batch runs as its own walk
 * BEFORE the conntrack walk: packets grouped by the unordered pair {saddr,
 * service address} (the service entry and its ICMP entry carry it), each
 * group in batch order.  Its result per packet (the slave, the backend row,
 * loopback) feeds the conntrack path's prep. */

/* A service packet's record (3 x 16 B, batch order):
 *   {VIP, saddr, z, nexthdr | (TUPLE_F_SERVICE | RELATED) << 8 | meta << 16},
 *   {w, len, hash, kd | master count << 16},
 *   {frontend base, frontend nslaves | flags, dport (the frame's), 0}
 * z = the service tuple's ports as ct_lookup4 loads them; kd = key.dport
 * after lb4_lookup_service (0 after an L3 fallback). */
struct ct_srec {
	uint4 r0, r1, r2;
	__device__ static ct_srec load(const uint4 *rec, uint32_t i, bool)
	{
		const uint4 *p = rec + 3u * i;
		return ct_srec{p[0], p[1], p[2]};
	}
	__device__ uint32_t meta() const { return r0.w >> 16; }
};


/* lb4_extract_key + lb4_lookup_service (lb.h:590-635) for every egress
 * packet; service packets get their CT_SERVICE record, their group key (in
 * gkey_sorted, batch order) and a set f2 flag: only they are compacted,
 * sorted and walked (about a fifth of the bench's packets) */
__global__ __launch_bounds__(256) void k_svc_prep(cgpu_snapshot s, ct_args a)
{
	const uint64_t stride = (uint64_t)gridDim.x * 256u;
	const bool l4 = s.lb_flags & CGPU_LB_L4;
	for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < a.n; i += stride) {
		const uint32_t fl = a.flags[i], pr = a.proto[i];
		const uint32_t sa = a.saddr[i], da = a.daddr[i], dp = a.dport[i];
		uint4 out = make_uint4(SVC_NONE, 0, 0, 0);
		bool svc = false;
		uint4 f = make_uint4(0, 0, 0, 0), v;
		uint32_t kd = 0;
		if (fl & 1u) {
			bool skip = false;
			if (l4) { /* extract_l4_port (lb.h:192-216) */
				if (pr == 6u || pr == 17u)
					kd = dp;
				else if (pr != 1u && pr != 58u)
					skip = true; /* DROP_UNKNOWN_L4: skip_service_lookup */
			}
			const uint32_t vb = lb_vip_bit(da) & s.lb.vip_mask;
			uint32_t probes = 0;
			if (!skip && ((s.lb.vip[vb >> 5] >> (vb & 31u)) & 1u))
				svc = lb_service(s, da, &kd, 0, &v, &f, &probes);
		}
		uint4 r0 = make_uint4(0, 0, 0, CTM_GATED << 16), r1 = make_uint4(0, 0, 0, 0),
		      r2 = make_uint4(0, 0, 0, 0);
		if (svc) {
			/* ct_lookup4(..., CT_SERVICE, ...)'s tuple (conntrack.h:462-530) */
			const uint32_t w = a.l4[i];
			uint32_t tfl = TUPLE_F_SERVICE, z = 0, meta = 0;
			bool ok = true;
			if (pr == 1u) {
				const uint32_t type = w & 0xFFu;
				if (type == 3u || type == 11u || type == 12u)
					tfl |= TUPLE_F_RELATED;
				else if (type == 0u)
					z = 8u;
				else {
					if (type == 8u)
						z = 8u << 16;
					meta |= CTM_ACT_CREATE;
				}
			} else if (pr == 6u || pr == 17u) {
				z = (uint32_t)a.sport[i] | (dp << 16);
				meta |= pr == 6u ? (CTM_TCP | ((w & 1u) ? CTM_ACT_CLOSE : CTM_ACT_CREATE)) : CTM_ACT_CREATE;
			} else {
				ok = false; /* DROP_CT_UNKNOWN_PROTO -> DROP_NO_SERVICE (lb.h:728-730) */
			}
			if (ok) {
				const uint32_t h = a.hash ? a.hash[i] : flow_hash(sa, da, a.sport[i], dp, pr);
				r0 = make_uint4(da, sa, z, pr | (tfl << 8) | (meta << 16));
				r1 = make_uint4(pr == 6u ? w : 0u, a.len[i], h, kd | (v.y & 0xFFFF0000u));
				r2 = make_uint4(f.z, f.w & 0xFFFFFFu, dp, 0u);
			} else {
				out.x = SVC_DROP;
			}
		}
		const bool walk = !((r0.w >> 16) & CTM_GATED);
		if (walk) {
			uint4 *r = a.rec + 3u * i;
			r[0] = r0;
			r[1] = r1;
			r[2] = r2;
			a.gkey_sorted[i] = ct_group(sa, da);
		}
		a.f2[i] = walk ? 1u : 0u;
		a.svc_out[i] = out;
	}
}

/* dst[j] = src[idx[j]], j < m (the compacted service packets' group keys) */
__global__ __launch_bounds__(256) void k_gather_u32(const uint32_t *src, const uint32_t *idx, uint32_t *dst,
						    uint32_t m)
{
	for (uint32_t j = blockIdx.x * 256u + threadIdx.x; j < m; j += gridDim.x * 256u)
		dst[j] = src[idx[j]];
}

/* One service packet of a group: lb4_local (lb.h:700-775) against the map.
 * k = the CT_SERVICE tuple; no forward lookup for CT_SERVICE (conntrack.h:
 * 553-558). */
__device__ __forceinline__ uint4 ct_svc_step(const cgpu_snapshot &s, const ct_table &T, const ct_acct &A,
					     ct_cache<CtK4> &c, const ct_srec &r, uint32_t now)
{
	const uint4 k = uint4{r.r0.x, r.r0.y, r.r0.z, r.r0.w & 0xFFFFu};
	const uint32_t meta = r.r0.w >> 16, w = r.r1.x, len = r.r1.y, h = r.r1.z;
	uint32_t kd = r.r1.w & 0xFFFFu;
	const uint32_t pr = r.r0.w & 0xFFu;
	uint4 f = uint4{r.r0.x, kd | (r.r1.w & 0xFFFF0000u), r.r2.x, r.r2.y};
	const uint4 drop = make_uint4(SVC_DROP, 0, 0, 0);
	uint32_t slave, lbs = 0;
	if (ctc_find<CtK4>(c, k) < 0) /* the service key and its ICMP key in one round */
		ctc_prefetch<CtK4>(T, c, k, CtK4::related(k), k, true, true, false);
	int ci = ctc_get<CtK4>(T, c, k);
	if (!(ctc_state(c, ci) & CTC_NEG)) { /* CT_REPLY / CT_RELATED: the stored state */
		ct_row e = ctc_row(c, ci);
		ct_hit(e, meta, false, w, len, now);
		ctc_put(c, ci, ctc_pos(c, ci), e);
		if (e.c.y & CTB_LB_LOOPBACK)
			lbs |= LBS_ENTRY;
		slave = e.c.z & 0xFFFFu;
	} else { /* CT_NEW: lb4_select_slave, ct_create4(CT_SERVICE) -- fail closed */
		slave = h % (r.r1.w >> 16) + 1u;
		const bool tcp = meta & CTM_TCP;
		ct_row e{};
		ct_timeout(e, now, tcp, false, tcp ? 1u : 0u);
		e.b = uint4{1u, 0u, len, 0u};
		e.c.z = slave;
		if (!ctc_update<CtK4>(T, A, c, k, e))
			return drop;
		e.c.y |= CTB_SEEN_NON_SYN;
		if (!ctc_update<CtK4>(T, A, c, CtK4::related(k), e))
			return drop;
	}
	uint4 b;
	if (!lb_row(s.lb, f, slave, &b)) {
		/* lb4_lookup_slave missed: lb4_lookup_service with key.slave kept,
		 * a new slave from its count, ct_update4_slave (lb.h:737-744) */
		uint32_t probes = 0;
		if (!lb_service(s, r.r0.x, &kd, slave, &b, &f, &probes))
			return drop;
		slave = h % (b.y >> 16) + 1u;
		ci = ctc_get<CtK4>(T, c, k);
		if (!(ctc_state(c, ci) & CTC_NEG)) {
			ct_row e = ctc_row(c, ci);
			e.c.z = (e.c.z & 0xFFFF0000u) | slave;
			ctc_put(c, ci, ctc_pos(c, ci), e);
		}
	}
	if (r.r0.y == b.x)
		lbs |= LBS_SNAT;
	const uint32_t port = b.y & 0xFFFFu;
	const uint32_t rw = ((s.lb_flags & CGPU_LB_L4) && port && kd != port && (pr == 6u || pr == 17u)) ? port : 0u;
	return make_uint4(SVC_XLATED | (lbs << 8) | (slave << 16), b.x, rw | ((b.z & 0xFFFFu) << 16), 0u);
}

/* The IPv6 service step: lb6_local with CONNTRACK (lb.h:426-483) over
 * cilium_ct6_global.  A service packet's record (4 x 16 B):
 *   {VIP}, {saddr}, {z, nexthdr | (TUPLE_F_SERVICE | RELATED) << 8 | meta << 16,
 *   w, len}, {hash, kd | master count << 16, fold6(VIP), dport}
 * Result: svc_out[2i] = {SVC_* | LBS_* << 8 | slave << 16, the dport rewrite
 * | rev_nat << 16, 0, 0}, svc_out[2i + 1] = the target. */
struct ct_srec6 {
	uint4 r0, r1, r2, r3;
	__device__ static ct_srec6 load(const uint4 *rec, uint32_t i, bool)
	{
		const uint4 *p = rec + 4u * i;
		return ct_srec6{p[0], p[1], p[2], p[3]};
	}
	__device__ uint32_t meta() const { return r2.y >> 16; }
};

__global__ __launch_bounds__(256) void k_svc_prep6(cgpu_snapshot s, ct_args a)
{
	const uint64_t stride = (uint64_t)gridDim.x * 256u;
	const bool l4 = s.lb_flags & CGPU_LB_L4;
	const uint4 *sa16 = reinterpret_cast<const uint4 *>(a.saddr);
	const uint4 *da16 = reinterpret_cast<const uint4 *>(a.daddr);
	for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < a.n; i += stride) {
		const uint32_t fl = a.flags[i], pr = a.proto[i], dp = a.dport[i];
		const uint4 sa = ld_x4<true>(sa16 + i), da = ld_x4<true>(da16 + i);
		uint4 out = make_uint4(SVC_NONE, 0, 0, 0);
		bool svc = false;
		uint4 tg, val;
		uint32_t kd = 0, f = 0;
		if (fl & 1u) {
			bool skip = false;
			if (l4) { /* extract_l4_port (lb.h:192-216) */
				if (pr == 6u || pr == 17u)
					kd = dp;
				else if (pr != 1u && pr != 58u)
					skip = true;
			}
			f = fold6(da.x, da.y, da.z, da.w);
			const uint32_t vb = lb6_vip_bit(f) & s.lb6.vip_mask;
			if (!skip && ((s.lb6.vip[vb >> 5] >> (vb & 31u)) & 1u))
				svc = lb6_service(s, da, f, &kd, 0, tg, val);
		}
		uint4 *r = a.rec + 4u * i;
		uint4 r2 = make_uint4(0, CTM_GATED << 16, 0, 0), r3 = make_uint4(0, 0, 0, 0);
		if (svc) {
			/* ct_lookup6(..., CT_SERVICE, ...)'s tuple (conntrack.h:308-378) */
			const uint32_t w = a.l4[i];
			uint32_t tfl = TUPLE_F_SERVICE, z = 0, meta = 0;
			bool ok = true;
			if (pr == 58u) {
				const uint32_t type = w & 0xFFu;
				if (type >= 1u && type <= 4u)
					tfl |= TUPLE_F_RELATED;
				else if (type == 129u)
					z = 128u;
				else {
					if (type == 128u)
						z = 128u << 16;
					meta |= CTM_ACT_CREATE;
				}
			} else if (pr == 6u || pr == 17u) {
				z = (uint32_t)a.sport[i] | (dp << 16);
				meta |= pr == 6u ? (CTM_TCP | ((w & 1u) ? CTM_ACT_CLOSE : CTM_ACT_CREATE)) : CTM_ACT_CREATE;
			} else {
				ok = false; /* DROP_CT_UNKNOWN_PROTO -> DROP_NO_SERVICE (lb.h:453-455) */
			}
			if (ok) {
				const uint32_t h = a.hash ? a.hash[i]
							  : flow_hash(fold6(sa.x, sa.y, sa.z, sa.w), f, a.sport[i], dp, pr);
				r2 = make_uint4(z, pr | (tfl << 8) | (meta << 16), pr == 6u ? w : 0u, a.len[i]);
				r3 = make_uint4(h, kd | (val.x & 0xFFFF0000u), f, dp);
			} else {
				out.x = SVC_DROP;
			}
		}
		const bool walk = !((r2.y >> 16) & CTM_GATED);
		if (walk) { /* as k_svc_prep: only service packets are walked */
			r[0] = da;
			r[1] = sa;
			r[2] = r2;
			r[3] = r3;
			a.gkey_sorted[i] = ct_group(fold6(sa.x, sa.y, sa.z, sa.w), f);
		}
		a.f2[i] = walk ? 1u : 0u;
		a.svc_out[2u * i] = out;
	}
}

__device__ __forceinline__ uint4 ct_svc_step6(const cgpu_snapshot &s, const ct_table &T, const ct_acct &A,
					      ct_cache<CtK6> &c, const ct_srec6 &r, uint32_t now, uint4 &tg)
{
	const CtK6::key k{r.r0, r.r1, r.r2.x, r.r2.y & 0xFFFFu};
	const uint32_t meta = r.r2.y >> 16, w = r.r2.z, len = r.r2.w, h = r.r3.x, f = r.r3.z;
	uint32_t kd = r.r3.y & 0xFFFFu;
	const uint32_t pr = r.r2.y & 0xFFu;
	const uint4 drop = make_uint4(SVC_DROP, 0, 0, 0);
	uint32_t slave, lbs = 0;
	if (ctc_find<CtK6>(c, k) < 0)
		ctc_prefetch<CtK6>(T, c, k, CtK6::related(k), k, true, true, false);
	int ci = ctc_get<CtK6>(T, c, k);
	if (!(ctc_state(c, ci) & CTC_NEG)) {
		ct_row e = ctc_row(c, ci);
		ct_hit(e, meta, false, w, len, now);
		ctc_put(c, ci, ctc_pos(c, ci), e);
		if (e.c.y & CTB_LB_LOOPBACK)
			lbs |= LBS_ENTRY;
		slave = e.c.z & 0xFFFFu;
	} else { /* CT_NEW: lb6_select_slave, ct_create6(CT_SERVICE) -- fail closed */
		slave = h % (r.r3.y >> 16) + 1u;
		const bool tcp = meta & CTM_TCP;
		ct_row e{};
		ct_timeout(e, now, tcp, false, tcp ? 1u : 0u);
		e.b = uint4{1u, 0u, len, 0u};
		e.c.z = slave;
		if (!ctc_update<CtK6>(T, A, c, k, e))
			return drop;
		e.c.y |= CTB_SEEN_NON_SYN;
		if (!ctc_update<CtK6>(T, A, c, CtK6::related(k), e))
			return drop;
	}
	uint4 val;
	if (!lb6_get<true>(s.lb6, r.r0, f, kd, slave, tg, val)) {
		/* lb6_lookup_slave missed: lb6_lookup_service with key.slave kept,
		 * a new slave from its count, ct_update6_slave (lb.h:462-469) */
		if (!lb6_service(s, r.r0, f, &kd, slave, tg, val))
			return drop;
		slave = h % (val.x >> 16) + 1u;
		ci = ctc_get<CtK6>(T, c, k);
		if (!(ctc_state(c, ci) & CTC_NEG)) {
			ct_row e = ctc_row(c, ci);
			e.c.z = (e.c.z & 0xFFFF0000u) | slave;
			ctc_put(c, ci, ctc_pos(c, ci), e);
		}
	}
	const uint32_t port = val.x & 0xFFFFu;
	const uint32_t rw = ((s.lb_flags & CGPU_LB_L4) && port && kd != port && (pr == 6u || pr == 17u)) ? port : 0u;
	return make_uint4(SVC_XLATED | (lbs << 8) | (slave << 16), rw | ((val.y & 0xFFFFu) << 16), 0u, 0u);
}

#ifndef CT_RETB
#define CT_RETB 16 /* results a walker lane buffers before storing them */
#endif

/* LRU mode: the keys packet i's conntrack step can look up or create (the
 * reply tuple, the forward tuple, its ICMP tuple) into the batch's filter */
template <class K> __global__ __launch_bounds__(256) void k_ct_mark(ct_args a, uint32_t *bloom, uint32_t mask)
{
	for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < a.n; i += (uint64_t)gridDim.x * 256u) {
		const ct_rec<K> r = ct_rec<K>::load(a.rec, (uint32_t)i, true);
		if (r.meta() & CTM_GATED)
			continue;
		const typename K::key k = r.key();
		const typename K::key fk = K::reversed(k);
		ct_mark<K>(bloom, mask, k);
		ct_mark<K>(bloom, mask, fk);
		ct_mark<K>(bloom, mask, K::related(fk));
	}
}

/* walks: WALK_PKT the conntrack path's packets; WALK_SVC the service step
 * (K = CtK4, ct_srec records, result into svc_out); WALK_OWED phase 2 of the
 * service path: candidates c = packet << 1 | kind, kind 0 a packet whose
 * address pair may hold owed entries, kind 1 an owed address entry */
/* workgroups per CU the service-path walker (CtK4S) is compiled for: its
 * creates through one update call site need 186 VGPRs (2 waves per SIMD);
 * 3 caps it at 168 with ~10 spilled: ctlb 20.83 -> 20.64 ms
 * (profiles/r5_k/ab_ctlb_minb.log; round 4: 1 -> 2, r4_f) */
#ifndef CGPU_WALK_MINB_SVC
#define CGPU_WALK_MINB_SVC 3
#endif
/* ... and the other walkers (1: the compiler's choice, A/B) */
#ifndef CGPU_WALK_W
#define CGPU_WALK_W 1
#endif

#define WALK_PKT 0
#define WALK_SVC 1
#define WALK_OWED 2

#ifdef CGPU_DIAG_WALK_CLOCK
/* timing-only tool build (tools/ct_scan.py): per wave of the last walk
 * {start, end (s_memrealtime, 100 MHz), steps of its busiest lane, steps of
 * all its lanes} */
__device__ unsigned long long g_walk_diag[4 * 8192];
extern "C" __attribute__((visibility("default"))) int cgpu_diag_walk_clock(unsigned long long *out, size_t n)
{
	return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_walk_diag), std::min<size_t>(n, 4 * 8192) * 8) == hipSuccess
		       ? 0
		       : -5;
}
#endif

template <class K, int MODE>
__global__ __launch_bounds__(256, K::ADDR ? CGPU_WALK_MINB_SVC : CGPU_WALK_W) void k_ct_walk(cgpu_snapshot s, ct_table T, ct_args a)
{
#ifdef CGPU_DIAG_WALK_CLOCK
	const unsigned long long dg_t0 = __builtin_amdgcn_s_memrealtime();
	uint32_t dg_steps = 0;
#endif
	using R = std::conditional_t<MODE == WALK_SVC, std::conditional_t<K::V6 != 0, ct_srec6, ct_srec>,
				     ct_rec<K>>;
	constexpr bool DFLT = MODE == WALK_PKT && ct_dflt<K>::ON;
	__shared__ int s_acct[3];
	/* each lane's last CT_RETB results (packet index, ct result), stored
	 * together: a scattered 1-byte store is a memory-side write whose
	 * completion every later load wait of the lane also waits for (vmcnt
	 * counts stores), so storing per packet put one write latency into every
	 * step (1.4 ms of a 12.3 ms step, profiles/r3_session_h/ab_ct_ret.log);
	 * CT_RETB stores issued back to back cost about one */
	__shared__ uint32_t s_ri[CT_RETB][256];
	__shared__ uint8_t s_rr[CT_RETB][256];
	uint32_t nret = 0;
	auto ret_flush = [&]() {
		for (uint32_t k = 0; k < nret; k++) {
			const uint32_t i = s_ri[k][threadIdx.x], ret = s_rr[k][threadIdx.x];
#if defined(CGPU_DIAG_NO_RET) /* timing only: the walk without its result stores */
#elif defined(CGPU_DIAG_RET_SMALL) /* timing only: the stores into 1 MiB */
			a.ct_ret[i & 0xFFFFFu] = (uint8_t)ret;
#elif defined(CGPU_DIAG_RET_NT)
			__builtin_nontemporal_store((uint8_t)ret, a.ct_ret + i);
#else
			a.ct_ret[i] = (uint8_t)ret;
#endif
			if (!K::ADDR && MODE == WALK_PKT && (ret & CT_RELP))
				a.f2[2u * i + 1u] = 1u; /* its ICMP entry is owed to phase 2 */
		}
		nret = 0;
	};
	if (threadIdx.x < 3)
		s_acct[threadIdx.x] = 0;
	__syncthreads();
	const ct_acct A{&s_acct[0], &s_acct[1], &s_acct[2]};
	const uint32_t nh = *a.n_heads;
	const uint32_t stride = gridDim.x * 256u;
#if CTC == 4
	ctc_ent<K> e0{}, e1{}, e2{}, e3{};
	ct_cache<K> c{e0, e1, e2, e3, 0u, 0u};
#elif CTC == 3
	ctc_ent<K> e0{}, e1{}, e2{};
	ct_cache<K> c{e0, e1, e2, 0u, 0u};
#else
	ctc_ent<K> e0{}, e1{};
	ct_cache<K> c{e0, e1, 0u, 0u};
#endif
	/* phase-2 candidates: v = packet << 1 | kind (plain path: kind 1 = the
	 * ICMP entry), v = packet << 2 | kind (service path: kind 1 = the address
	 * entry, 2 = the ICMP entry) */
	auto pkt_of = [](uint32_t v) { return MODE == WALK_OWED ? (K::ADDR ? v >> 2 : v >> 1) : v; };
	/* groups longest first (a.glen / a.gpos, sorted by length): the
	 * elephants start in the first round and the rest fill in behind */
	for (uint32_t h = blockIdx.x * 256u + threadIdx.x; h < nh; h += stride) {
		const uint64_t p0 = a.gpos[h];
		const uint64_t p1 = p0 + a.glen[h];
		/* CGPU_CT_DFLT: the group's orientation (-1: not yet decided) */
		int gb = -1;
		/* packets in batch order through the sort permutation, software-
		 * pipelined: the record of p + 1 and the index of p + 2 are in
		 * flight while packet p runs */
		uint32_t n1 = a.idx_sorted[p0];
		uint32_t n2 = p0 + 1u < p1 ? a.idx_sorted[p0 + 1u] : n1;
		uint32_t n3 = p0 + 2u < p1 ? a.idx_sorted[p0 + 2u] : n1;
		R r1 = R::load(a.rec, pkt_of(n1), false);
		R r2 = p0 + 1u < p1 ? R::load(a.rec, pkt_of(n2), false) : r1;
		for (uint64_t p = p0; p < p1; p++) {
			/* records two packets ahead and the index three ahead are in
			 * flight while packet p runs */
			const uint32_t v = n1;
			const uint32_t i = pkt_of(v);
			const R r = r1;
			n1 = n2;
			r1 = r2;
			if (p + 2u < p1) {
				n2 = n3;
				r2 = R::load(a.rec, pkt_of(n2), false);
				if (p + 3u < p1)
					n3 = a.idx_sorted[p + 3u];
			}
			const uint32_t meta = r.meta();
			if (meta & CTM_GATED)
				continue;
#ifdef CGPU_DIAG_WALK_CLOCK
			dg_steps++;
#endif
			if constexpr (MODE == WALK_SVC) {
				if constexpr (K::V6 != 0) {
					uint4 tg = make_uint4(0, 0, 0, 0);
					const uint4 o = ct_svc_step6(s, T, A, c, r, a.now, tg);
					a.svc_out[2u * i] = o;
					a.svc_out[2u * i + 1u] = tg;
				} else {
					a.svc_out[i] = ct_svc_step(s, T, A, c, r, a.now);
				}
			} else {
				const ct_pkt q = r.pkt();
				if constexpr (MODE == WALK_OWED) {
					const uint32_t kind = K::ADDR ? (v & 3u) : (v & 1u) << 1;
					if (kind != 0u) {
						/* an owed entry of packet i's create: kind 1 its
						 * address entry, kind 2 its ICMP entry.  One update
						 * call site for both (each inlined copy of the map
						 * update costs the walker registers) */
						const typename K::key fk = K::reversed(r.key());
						const bool addr = K::ADDR && kind == 1u;
						if (a.ct_ret[i] & (addr ? CT_ADDRP : CT_RELP)) {
							ct_row e = ct_new_row<K>(q, !addr && !(q.meta & CTM_EGRESS), a.now);
							if (!addr)
								e.c.y |= CTB_SEEN_NON_SYN;
							typename K::key k = K::related(fk);
							if constexpr (K::ADDR) {
								if (addr)
									k = ct_addr_key(fk, q);
							}
							ctc_update_owed<K>(T, A, c, k, e);
						}
						continue;
					}
				}
				if (MODE == WALK_PKT && (meta & CTM_PHASE2))
					continue;
				const uint32_t ret = ct_step<K>(T, A, c, r.key(), q, a.now);
#ifdef CGPU_DIAG_RET_DEFAULT /* timing only: no store where the result is the direction's default */
				if (ret == ((meta & CTM_EGRESS) ? CT_ESTABLISHED : CT_REPLY))
					continue;
#endif
				if constexpr (DFLT) {
					if (a.dflt) {
						const uint32_t o = ct_dflt<K>::orient(r);
						if (gb < 0 && ret <= CT_REPLY)
							gb = (int)(ret == CT_REPLY ? o ^ 1u : o);
						if (gb == 0 && ret == (o ? CT_REPLY : CT_ESTABLISHED))
							continue; /* the orientation default: nothing stored */
					}
				}
				s_ri[nret][threadIdx.x] = i;
				s_rr[nret][threadIdx.x] = (uint8_t)ret;
				if (++nret == CT_RETB)
					ret_flush();
			}
		}
		ctc_flush(T, c);
	}
	ret_flush();
#ifdef CGPU_DIAG_WALK_CLOCK
	{
		uint32_t mx = dg_steps;
		for (int o = 32; o > 0; o >>= 1)
			mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, 64));
		const uint64_t sum = wave_sum((uint64_t)dg_steps);
		const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
		const uint32_t w = (blockIdx.x * 256u + threadIdx.x) >> 6;
		if ((threadIdx.x & 63) == 0 && w < 8192u && MODE == WALK_PKT) {
			g_walk_diag[4u * w] = dg_t0;
			g_walk_diag[4u * w + 1u] = t1;
			g_walk_diag[4u * w + 2u] = mx;
			g_walk_diag[4u * w + 3u] = sum;
		}
	}
#endif
	__syncthreads();
	if (threadIdx.x == 0) {
		const int back = s_acct[0] + s_acct[1]; /* unused reservation + deletes */
		if (back)
			atomicSub(&T.count[0], (uint32_t)back);
		if (s_acct[2])
			atomicAdd(&T.count[1], (uint32_t)s_acct[2]);
	}
}

/* policy on the tuple ct_lookup left, counters, the reply / related skip.
 * CT_NEW / CT_ESTABLISHED packets reuse the prep's forward decision; only
 * CT_REPLY / CT_RELATED ones run the cascade again, on the reply tuple.
 * Hot counter slots accumulate in LDS (packed, as k_classify CTR = 1). */
template <int NT, class K, int Q>
__global__ __launch_bounds__(NT) void k_ct_finish(cgpu_snapshot s, ct_args a, uint32_t cc_n, uint64_t lo,
						   uint64_t hi)
{
	extern __shared__ __attribute__((aligned(16))) uint64_t lctr[];
	/* metrics {reason 0 / 133 / 137 / 155 [/ 158]} x {ingress, egress} */
	constexpr int NM = K::SVC ? 10 : 8;
	uint64_t mcnt[NM] = {}, mbyt[NM] = {};
	/* LDS: the hot counter slots, then the cold-slot cache (as k_classify_x4:
	 * cc_n packed counts, cc_n tags = slot + 1): each touched cold slot costs
	 * one packed memory-side atomic per workgroup instead of one per hit; a
	 * hit the cache cannot take is one packed atomic into pk (PKC format;
	 * the launcher unpacks pk into delta after every PKC_CHUNK packets), as
	 * k_classify_x4 does: two unpacked atomics per hit made this kernel issue
	 * 30M memory-side atomics per 64M packets (profiles/r4_prof/ct) */
	uint64_t *ccv = lctr + s.hot_slots;
	uint32_t *cck = reinterpret_cast<uint32_t *>(ccv + cc_n);
	for (uint32_t k = threadIdx.x; k < s.hot_slots; k += NT)
		lctr[k] = 0;
	for (uint32_t k = threadIdx.x; k < cc_n; k += NT) {
		ccv[k] = 0;
		cck[k] = 0;
	}
	__syncthreads();
	/* Q packets per lane (packet g + u * threads): the CT_REPLY / CT_RELATED
	 * packets' policy cascades run stage-interleaved (policy_q) */
	const uint64_t T = (uint64_t)gridDim.x * NT;
	for (uint64_t g = lo + (uint64_t)blockIdx.x * NT + threadIdx.x; g < hi; g += T * Q) {
		ct_pkt q[Q];
		uint32_t c[Q], ep[Q], dp[Q], pr[Q];
		bool act[Q], rep[Q], eg[Q], frag[Q];
		decision d[Q];
#pragma unroll
		for (int u = 0; u < Q; u++) {
			const uint64_t i = g + (uint64_t)u * T;
			act[u] = i < hi;
			const uint64_t j = act[u] ? i : 0u;
			/* batch order: records and the walker's results stream in */
			const ct_rec<K> rr = ct_rec<K>::load(a.rec, (uint32_t)j, true);
			q[u] = rr.pkt();
			c[u] = ntl(a.ct_ret + j) & ~(CT_ADDRP | CT_RELP);
			if constexpr (ct_dflt<K>::ON) {
				if (c[u] == CT_DFLT && a.dflt) /* the orientation default (the walker stored nothing) */
					c[u] = ct_dflt<K>::orient(rr) ? CT_REPLY : CT_ESTABLISHED;
			}
			ep[u] = ntl(a.ep + j);
			eg[u] = q[u].meta & CTM_EGRESS;
			frag[u] = q[u].meta & CTM_FRAG;
			rep[u] = act[u] && !(q[u].meta & CTM_GATED) && (c[u] & 3u) >= CT_REPLY;
			dp[u] = q[u].dport;
			pr[u] = q[u].proto;
			/* the reply tuple keeps the packet's addresses and direction, so
			 * its identity is the one the prep resolved (decide<>'s identity
			 * depends on neither port nor protocol) */
			d[u].id = rep[u] ? ntl(a.identity + j) : 0u;
		}
		policy_q<Q, false>(s, rep, eg, frag, dp, pr, ep, d);
#pragma unroll
		for (int u = 0; u < Q; u++) {
			if (!act[u])
				continue;
			const uint64_t i = g + (uint64_t)u * T;
			const uint32_t meta = q[u].meta;
			const bool egress = eg[u];
			const uint32_t len = q[u].len;
			int32_t v;
			uint32_t st = 4, cr = 255u;
			if (meta & CTM_GATED) {
				v = DROP_CT_UNKNOWN_PROTO; /* ct_lookup default case */
				if (K::SVC && (meta & CTM_SVCDROP)) {
					v = DROP_NO_SERVICE; /* lb4_local failed closed (lb.h:715-744) */
					st = 6;
				}
			} else {
				cr = c[u] & 3u;
				int ctr;
				if (cr >= CT_REPLY) {
					ctr = d[u].ctr;
					st = d[u].st;
					v = (egress && d[u].v > 0) ? d[u].v : 0;
				} else {
					ctr = (int)(q[u].cst & 0xFFFFFFu) - 1;
					st = q[u].cst >> 24;
					if (!(meta & CTM_ALLOWED))
						v = DROP_POLICY;
					else if (c[u] & CT_FAIL)
						v = DROP_CT_CREATE_FAILED;
					else
						v = (int32_t)q[u].port;
				}
				if (ctr >= 0) {
					const uint32_t cs = (uint32_t)ctr;
					bool done = false;
					/* only packets of < PKC_MAX_LEN bytes may enter the LDS
					 * sums: they are flushed into pk, whose byte field holds
					 * PKC_CHUNK packets of < 2^11 bytes (as k_classify_x4) */
					if (len < PKC_MAX_LEN) {
						if (cs < s.hot_slots) {
							atomicAdd((unsigned long long *)&lctr[cs],
								  (1ull << PK_SHIFT) | (unsigned long long)len);
							done = true;
						} else if (cc_n) {
							uint32_t j = __umulhi(cs * 0x9E3779B1u, cc_n);
#pragma unroll
							for (int p = 0; p < CC_PROBE && !done; p++, j++) {
								j = j == cc_n ? 0u : j;
								uint32_t t = cck[j];
								if (t == 0u) {
									const uint32_t o = atomicCAS(&cck[j], 0u, cs + 1u);
									t = o == 0u ? cs + 1u : o;
								}
								if (t == cs + 1u) {
									atomicAdd((unsigned long long *)&ccv[j],
										  (1ull << PK_SHIFT) | (unsigned long long)len);
									done = true;
								}
							}
						}
					}
					if (!done) {
						if (len < PKC_MAX_LEN) {
							atomicAdd((unsigned long long *)&a.pk[cs],
								  (1ull << PKC_SHIFT) | (unsigned long long)len);
						} else { /* exact two-word path, never packed */
							atomicAdd((unsigned long long *)&a.delta[2u * cs], 1ull);
							atomicAdd((unsigned long long *)&a.delta[2u * cs + 1u],
								  (unsigned long long)len);
						}
					}
				}
			}
			a.verdict[i] = v;
			a.ct_ret[i] = (uint8_t)cr;
			if (a.stage)
				a.stage[i] = (uint8_t)st;
			/* a proxy redirect (v > 0) traces TRACE_TO_PROXY: no metrics */
			const uint32_t r = v > 0 ? 5u : v == 0 ? 0u : (v == DROP_POLICY ? 1u : (v == DROP_CT_UNKNOWN_PROTO ? 2u : (v == DROP_NO_SERVICE ? 4u : 3u)));
			const uint32_t idx = r * 2u + (egress ? 1u : 0u);
#pragma unroll
			for (int k = 0; k < NM; k++) {
				mcnt[k] += (idx == (uint32_t)k) ? 1u : 0u;
				mbyt[k] += (idx == (uint32_t)k) ? len : 0u;
			}
		}
	}
	uint64_t *met = a.delta + 2ull * s.n_ctr_slots;
	const uint32_t reasons[5] = {0u, 133u, 137u, 155u, 158u};
#pragma unroll
	for (int k = 0; k < NM; k++) {
		const uint64_t cn = wave_sum(mcnt[k]);
		const uint64_t by = wave_sum(mbyt[k]);
		if ((threadIdx.x & 63) == 0 && cn) {
			const uint32_t key = (reasons[k >> 1] * 4u + ((k & 1) ? 2u : 1u)) * 2u;
			atomicAdd((unsigned long long *)&met[key], (unsigned long long)cn);
			atomicAdd((unsigned long long *)&met[key + 1], (unsigned long long)by);
		}
	}
	__syncthreads();
	/* one packed atomic per touched slot: PK (LDS) -> PKC (pk) format; a
	 * workgroup's bytes per slot stay < 2^37 (< 2^26 packets of < 2^11 =
	 * PKC_MAX_LEN; every packet of PKC_MAX_LEN bytes or more went to delta
	 * directly above) */
	for (uint32_t k = threadIdx.x; k < s.hot_slots; k += NT) {
		const uint64_t x = lctr[k];
		if (x)
			atomicAdd((unsigned long long *)&a.pk[k], ((x >> PK_SHIFT) << PKC_SHIFT) | (x & PK_BYTES_MASK));
	}
	for (uint32_t k = threadIdx.x; k < cc_n; k += NT) {
		const uint32_t t = cck[k];
		const uint64_t x = ccv[k];
		if (t && x)
			atomicAdd((unsigned long long *)&a.pk[t - 1u],
				  ((x >> PK_SHIFT) << PKC_SHIFT) | (x & PK_BYTES_MASK));
	}
}

/* ctmap.GC's RemoveExpired filter (pkg/maps/ctmap/ctmap.go:273-367,
 * doFiltering: an entry whose lifetime < time is deleted) over the device
 * map, one lane per slot: the map stays on the device (the host path pulls
 * and pushes both arrays, ~0.7 GB each way at config-2 sizes).  The slot
 * turns into a tombstone as a batch's delete does; the live / tombstone
 * counts and the number deleted are netted per workgroup. */
template <class K> __global__ __launch_bounds__(256) void k_ct_gc(ct_table T, uint32_t time, uint32_t *deleted)
{
	__shared__ uint32_t s_del;
	if (threadIdx.x == 0)
		s_del = 0;
	__syncthreads();
	uint32_t del = 0;
	for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i <= T.mask; i += gridDim.x * 256u) {
		const uint32_t tag = *K::tagp(T, i) >> 16;
		if (tag != CT_TAG_LIVE || T.vals[4u * i + 2u].x >= time)
			continue;
		K::clear(T, i);
		*K::tagp(T, i) = CT_TAG_TOMB << 16;
		del++;
	}
	del = (uint32_t)wave_sum((uint64_t)del);
	if ((threadIdx.x & 63u) == 0 && del)
		atomicAdd(&s_del, del);
	__syncthreads();
	if (threadIdx.x == 0 && s_del) {
		atomicAdd(deleted, s_del);
		atomicSub(&T.count[0], s_del);
		atomicAdd(&T.count[1], s_del);
	}
}

/* Compaction of a map whose tombstones lengthen the probe chains: every
 * live slot of src re-inserted into the empty table dst (same size), its
 * row with it; dst's tombstone count is 0, its live count src's. */
template <class K> __global__ __launch_bounds__(256) void k_ct_rehash(ct_table src, ct_table dst)
{
	for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i <= src.mask; i += gridDim.x * 256u) {
		if ((*K::tagp(src, i) >> 16) != CT_TAG_LIVE)
			continue;
		typename K::key k = K::load(src, i);
		const uint32_t want = (K::cmeta(k) & 0xFFFFu) | (CT_TAG_LIVE << 16);
		uint32_t h = K::hash(k) & dst.mask;
		while (atomicCAS(K::tagp(dst, h), CT_TAG_EMPTY, want) != CT_TAG_EMPTY)
			h = (h + 1u) & dst.mask;
		K::store(dst, h, k);
		const uint4 *sv = src.vals + 4u * i;
		uint4 *dv = dst.vals + 4u * h;
		dv[0] = sv[0];
		dv[1] = sv[1];
		dv[2] = sv[2];
		dv[3] = sv[3];
	}
}

hipError_t launch_ct_gc(const ct_table &T, bool v6, uint32_t time, uint32_t *deleted, hipStream_t st)
{
	const unsigned g = (unsigned)std::min<uint64_t>(((uint64_t)T.mask + 256u) / 256u, 8192);
	if (v6)
		hipLaunchKernelGGL(k_ct_gc<CtK6>, dim3(g), dim3(256), 0, st, T, time, deleted);
	else
		hipLaunchKernelGGL(k_ct_gc<CtK4>, dim3(g), dim3(256), 0, st, T, time, deleted);
	return hipGetLastError();
}

/* dst: zeroed keys (tags EMPTY), vals and count set by the caller */
hipError_t launch_ct_rehash(const ct_table &src, const ct_table &dst, bool v6, hipStream_t st)
{
	const unsigned g = (unsigned)std::min<uint64_t>(((uint64_t)src.mask + 256u) / 256u, 8192);
	if (v6)
		hipLaunchKernelGGL(k_ct_rehash<CtK6>, dim3(g), dim3(256), 0, st, src, dst);
	else
		hipLaunchKernelGGL(k_ct_rehash<CtK4>, dim3(g), dim3(256), 0, st, src, dst);
	return hipGetLastError();
}

/* group-key bits the conntrack radix sort orders (CGPU_SCHED_CT_SORT_BITS) */
static int ct_sort_bits(const cgpu_snapshot &s)
{
	const int b = (int)((s.schedule >> 8) & 63u);
	return b ? std::max(8, std::min(32, b)) : 24;
}

/* Ordered stream compaction of byte flags (the group heads, the phase-2
 * candidates): the indices of the set flags, in index order.  Three small
 * launches, count per 4096-flag block -> one-block scan of the counts ->
 * emit, read the flags twice at streaming rate; hipcub's DeviceSelect over
 * a counting iterator took 0.77 ms per 64M flags and 1.43 ms per 128M
 * (profiles/r3_ct). */
#define SEL_T 16u            /* flags per thread: one 16-byte load */
#define SEL_B (256u * SEL_T) /* flags per block */

__device__ __forceinline__ uint32_t sel_bits(const uint8_t *f, uint64_t n, uint64_t i0)
{
	uint32_t bits = 0;
	if (i0 + SEL_T <= n) {
		const uint4 v = *reinterpret_cast<const uint4 *>(f + i0);
		const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
		for (int k = 0; k < 4; k++)
#pragma unroll
			for (int b = 0; b < 4; b++)
				bits |= ((w[k] >> (8 * b)) & 0xFFu) ? 1u << (4 * k + b) : 0u;
	} else {
		for (uint32_t j = 0; j < SEL_T; j++)
			bits |= (i0 + j < n && f[i0 + j]) ? 1u << j : 0u;
	}
	return bits;
}

__global__ __launch_bounds__(256) void k_sel_count(const uint8_t *f, uint64_t n, uint32_t *bc)
{
	__shared__ uint32_t ws[4];
	const uint64_t i0 = ((uint64_t)blockIdx.x * 256u + threadIdx.x) * SEL_T;
	const uint32_t c = wave_sum((uint32_t)__popc(sel_bits(f, n, i0)));
	if ((threadIdx.x & 63u) == 0)
		ws[threadIdx.x >> 6] = c;
	__syncthreads();
	if (threadIdx.x == 0)
		bc[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

/* one workgroup: exclusive scan of the nb block counts in place, the total
 * to *count */
__global__ __launch_bounds__(1024) void k_sel_scan(uint32_t *bc, uint32_t nb, uint32_t *count)
{
	__shared__ uint32_t sc[1024];
	uint32_t carry = 0;
	for (uint32_t base = 0; base < nb; base += 1024u) {
		const uint32_t k = base + threadIdx.x;
		const uint32_t v = k < nb ? bc[k] : 0u;
		sc[threadIdx.x] = v;
		__syncthreads();
		for (uint32_t o = 1; o < 1024u; o <<= 1) {
			const uint32_t t = threadIdx.x >= o ? sc[threadIdx.x - o] : 0u;
			__syncthreads();
			sc[threadIdx.x] += t;
			__syncthreads();
		}
		if (k < nb)
			bc[k] = carry + sc[threadIdx.x] - v;
		carry += sc[1023];
		__syncthreads();
	}
	if (threadIdx.x == 0)
		*count = carry;
}

__global__ __launch_bounds__(256) void k_sel_emit(const uint8_t *f, uint64_t n, const uint32_t *bc, uint32_t *out)
{
	__shared__ uint32_t ws[4];
	const uint32_t lane = __lane_id(), wv = threadIdx.x >> 6;
	const uint64_t i0 = ((uint64_t)blockIdx.x * 256u + threadIdx.x) * SEL_T;
	uint32_t bits = sel_bits(f, n, i0);
	const uint32_t c = (uint32_t)__popc(bits);
	uint32_t x = c; /* inclusive scan over the wave */
	for (int o = 1; o < 64; o <<= 1) {
		const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
		x += lane >= (uint32_t)o ? y : 0u;
	}
	if (lane == 63u)
		ws[wv] = x;
	__syncthreads();
	uint32_t pos = bc[blockIdx.x] + x - c;
	for (uint32_t w = 0; w < wv; w++)
		pos += ws[w];
	while (bits) {
		const uint32_t j = (uint32_t)__ffs(bits) - 1u;
		bits &= bits - 1u;
		out[pos++] = (uint32_t)(i0 + j);
	}
}

static uint64_t sel_blocks(uint64_t n)
{
	return (n + SEL_B - 1) / SEL_B;
}

/* out[0, *count) = the indices i < n with f[i] != 0, ascending; bc = nb
 * words of scratch */
static hipError_t ct_select(const uint8_t *f, uint64_t n, uint32_t *out, uint32_t *count, uint32_t *bc,
			    hipStream_t st)
{
	const uint64_t nb = sel_blocks(n);
	if (!nb)
		return hipMemsetAsync(count, 0, 4, st);
	hipLaunchKernelGGL(k_sel_count, dim3((unsigned)nb), dim3(256), 0, st, f, n, bc);
	hipLaunchKernelGGL(k_sel_scan, dim3(1), dim3(1024), 0, st, bc, (uint32_t)nb, count);
	hipLaunchKernelGGL(k_sel_emit, dim3((unsigned)nb), dim3(256), 0, st, f, n, bc, out);
	return hipGetLastError();
}

/* scratch for the sort of n packets (hipcub) and for the block counts of the
 * selections (the 4n phase-2 candidates of the service path at most) */
size_t ct_temp_bytes(uint64_t n)
{
	size_t a = 0;
	(void)hipcub::DeviceRadixSort::SortPairs(nullptr, a, (const uint32_t *)nullptr, (uint32_t *)nullptr,
						 (const uint32_t *)nullptr, (uint32_t *)nullptr, (int)n);
	/* ... and phase 2b's bloom filter (k_ct_owed_bloom) */
	return std::max<size_t>(std::max<size_t>(a, sel_blocks(4 * n) * 4u + 4u),
				std::max<size_t>((size_t)OWED_BLOOM_WORDS * 4u, (size_t)LH_B * 32u * 4u));
}

static ct_args ct_args_of(const ct_launch &L)
{
	ct_args a{static_cast<const uint32_t *>(L.saddr), static_cast<const uint32_t *>(L.daddr), L.sport,
		  L.dport, L.proto, L.l4, L.flags, L.len, L.ep,
		  L.verdict, L.ct_ret, L.identity, L.stage, L.delta, L.n, L.now,
		  L.rec, L.gkey, L.gkey_sorted, L.idx, L.idx_sorted, L.head, L.heads,
		  L.n_heads};
	a.hash = L.hash;
	a.svc_out = L.svc_out;
	a.ctl = L.ctl;
	a.xdaddr = static_cast<uint32_t *>(L.xdaddr);
	a.xdport = L.xdport;
	a.f2 = L.flags2;
	a.pcls = L.pcls;
	a.pk = L.pk;
	a.dflt = L.dflt;
	return a;
}

/* 1: groups ordered longest first by power-of-two length buckets on the
 * device (no host read of the group count, no sort of the lengths); 0: the
 * lengths radix-sorted exactly, after a host read.  The IPv6 walks keep the
 * exact order: ct 12.29 -> 12.16 ms and ctlb 22.40 -> 22.04 with the
 * buckets, ct6 15.70 -> 15.88 (profiles/r4_ad/) */
#ifndef CGPU_CT_LH
#define CGPU_CT_LH 1
#endif

/* Groups longest first, ordered on the device (the group count stays in
 * device memory: no host round trip between the sort and the walk).  A
 * group's bucket is the highest set bit of its length; the buckets are laid
 * out longest first, so the elephants start in the walker's first round.
 * LH_B workgroups each own a contiguous range of the group heads: count the
 * range's buckets (k_ct_lhist), one workgroup turns the LH_B x 32 counts
 * into offsets (k_ct_lscan), and each range places its groups in head order
 * inside every bucket (k_ct_lplace: ranks from wave ballots, so the layout
 * is deterministic). */
__device__ __forceinline__ void lh_range(uint32_t nh, uint32_t b, uint32_t &lo, uint32_t &hi)
{
	lo = (uint32_t)((uint64_t)nh * b / LH_B);
	hi = (uint32_t)((uint64_t)nh * (b + 1u) / LH_B);
}

__device__ __forceinline__ uint32_t lh_len(const uint32_t *heads, uint32_t k, uint32_t nh, uint64_t n)
{
	return (uint32_t)((k + 1u < nh ? (uint64_t)heads[k + 1u] : n) - heads[k]);
}

__global__ __launch_bounds__(256) void k_ct_lhist(const uint32_t *heads, const uint32_t *n_heads, uint64_t n,
						  uint32_t *bh)
{
	__shared__ uint32_t h[32];
	if (threadIdx.x < 32)
		h[threadIdx.x] = 0;
	__syncthreads();
	uint32_t lo, hi;
	lh_range(*n_heads, blockIdx.x, lo, hi);
	const uint32_t nh = *n_heads;
	for (uint32_t k = lo + threadIdx.x; k < hi; k += 256u)
		atomicAdd(&h[31 - __clz(lh_len(heads, k, nh, n))], 1u);
	__syncthreads();
	if (threadIdx.x < 32)
		bh[blockIdx.x * 32u + threadIdx.x] = h[threadIdx.x];
}

/* one workgroup: bh[b][bucket] := where range b's groups of that bucket
 * start, buckets longest first, ranges in order inside a bucket */
__global__ __launch_bounds__(256) void k_ct_lscan(uint32_t *bh)
{
	__shared__ uint32_t c[LH_B * 32u];
	__shared__ uint32_t base[32];
	for (uint32_t k = threadIdx.x; k < LH_B * 32u; k += 256u)
		c[k] = bh[k];
	__syncthreads();
	if (threadIdx.x < 32) { /* per bucket: ranges' exclusive prefix, the total */
		uint32_t run = 0;
		for (uint32_t b = 0; b < LH_B; b++) {
			const uint32_t x = c[b * 32u + threadIdx.x];
			c[b * 32u + threadIdx.x] = run;
			run += x;
		}
		base[threadIdx.x] = run;
	}
	__syncthreads();
	if (threadIdx.x == 0) {
		uint32_t o = 0;
		for (int k = 31; k >= 0; k--) {
			const uint32_t t = base[k];
			base[k] = o;
			o += t;
		}
	}
	__syncthreads();
	for (uint32_t k = threadIdx.x; k < LH_B * 32u; k += 256u)
		bh[k] = c[k] + base[k & 31u];
}

__global__ __launch_bounds__(256) void k_ct_lplace(const uint32_t *heads, const uint32_t *n_heads, uint64_t n,
						   const uint32_t *bh, uint32_t *glen, uint32_t *gpos)
{
	__shared__ uint32_t off[32];
	__shared__ uint32_t wc[4][32];
	const uint32_t nh = *n_heads, lane = __lane_id(), wv = threadIdx.x >> 6;
	uint32_t lo, hi;
	lh_range(nh, blockIdx.x, lo, hi);
	if (threadIdx.x < 32)
		off[threadIdx.x] = bh[blockIdx.x * 32u + threadIdx.x];
	__syncthreads();
	for (uint32_t t0 = lo; t0 < hi; t0 += 256u) {
		const uint32_t k = t0 + threadIdx.x;
		const bool act = k < hi;
		const uint32_t len = act ? lh_len(heads, k, nh, n) : 1u;
		const uint32_t bk = act ? 31u - (uint32_t)__clz(len) : 32u;
		uint32_t rank = 0;
		const uint64_t below = (1ull << lane) - 1ull;
		for (uint32_t b = 0; b < 32u; b++) {
			const uint64_t m = __ballot(bk == b);
			if (bk == b)
				rank = (uint32_t)__popcll(m & below);
			if (lane == 0)
				wc[wv][b] = (uint32_t)__popcll(m);
		}
		__syncthreads();
		if (act) {
			uint32_t at = off[bk] + rank;
			for (uint32_t w = 0; w < wv; w++)
				at += wc[w][bk];
			glen[at] = len;
			gpos[at] = heads[k];
		}
		__syncthreads();
		if (threadIdx.x < 32)
			off[threadIdx.x] += wc[0][threadIdx.x] + wc[1][threadIdx.x] + wc[2][threadIdx.x] + wc[3][threadIdx.x];
		__syncthreads();
	}
}

/* (gkey, idx)[0, m) -> groups in batch order, longest first: a.idx_sorted
 * the permutation, a.gpos / a.glen per group; *nh (host) the group count, 0 when ordered on the
 * device (the walk reads it from device memory) */
static hipError_t ct_group_sort(const cgpu_snapshot &s, const ct_launch &L, ct_args &a, uint64_t m,
				uint32_t *nh, hipStream_t st, bool exact = false)
{
	const unsigned g = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((m + 255) / 256, 8192));
	size_t tb = L.temp_bytes;
	/* 24 key bits: three passes; pairs sharing a 24-bit hash merge into
	 * one group, which only lengthens that lane's walk */
	const int bits = ct_sort_bits(s);
	hipError_t e = hipcub::DeviceRadixSort::SortPairs(L.temp, tb, L.gkey, L.gkey_sorted, L.idx,
							   L.idx_sorted, (int)m, 0, bits, st);
	if (e != hipSuccess)
		return e;
	const uint32_t mask = bits >= 32 ? 0xFFFFFFFFu : ((1u << bits) - 1u);
	hipLaunchKernelGGL(k_ct_heads, dim3(g), dim3(256), 0, st, L.gkey_sorted, L.head, m, mask);
	e = ct_select(L.head, m, L.heads, L.n_heads, static_cast<uint32_t *>(L.temp), st);
	if (e != hipSuccess)
		return e;
	*nh = 0;
	if (CGPU_CT_LH && !exact) {
		/* gkey / idx are free again: (length, start) of the groups,
		 * longest first; temp holds the range counts */
		uint32_t *bh = static_cast<uint32_t *>(L.temp);
		hipLaunchKernelGGL(k_ct_lhist, dim3(LH_B), dim3(256), 0, st, L.heads, L.n_heads, (uint64_t)m, bh);
		hipLaunchKernelGGL(k_ct_lscan, dim3(1), dim3(256), 0, st, bh);
		hipLaunchKernelGGL(k_ct_lplace, dim3(LH_B), dim3(256), 0, st, L.heads, L.n_heads, (uint64_t)m,
				   (const uint32_t *)bh, L.gkey, L.idx);
		a.glen = L.gkey;
		a.gpos = L.idx;
		return hipGetLastError();
	}
	/* groups longest first: gkey / idx are free again and hold (length,
	 * start) before the sort, gkey_sorted / idx the sorted pairs after */
	e = hipMemcpyAsync(nh, L.n_heads, 4, hipMemcpyDeviceToHost, st);
	if (e != hipSuccess || (e = hipStreamSynchronize(st)) != hipSuccess)
		return e;
	const unsigned gh = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((*nh + 255) / 256, 8192));
	hipLaunchKernelGGL(k_ct_lens, dim3(gh), dim3(256), 0, st, L.heads, *nh, m, L.gkey, L.heads_pos);
	tb = L.temp_bytes;
	e = hipcub::DeviceRadixSort::SortPairsDescending(L.temp, tb, L.gkey, L.gkey_sorted, L.heads_pos,
							 L.idx, (int)*nh, 0, 32, st);
	if (e != hipSuccess)
		return e;
	a.glen = L.gkey_sorted;
	a.gpos = L.idx;
	return hipSuccess;
}


/* walker grid: 8192 workgroups of 4 waves, ~4 rounds of the resident
 * ~2300: a lane takes fewer groups, so the walk's tail is shorter (2048:
 * +0.35 ms on --config ct, +0.44 ms on ctlb, profiles/r5_i/ab_grid_*.log) */
#ifndef CT_WALK_GRID
#define CT_WALK_GRID 8192
#endif

template <class K> static hipError_t launch_ct_finish(const cgpu_snapshot &s, const ct_args &a, hipStream_t st)
{
	/* <= 2^23 packets per workgroup keeps the packed LDS counters exact */
	constexpr int NF = CGPU_CT_FNT, Q = CGPU_CT_FQ;
	const uint64_t gf = std::max<uint64_t>(std::min<uint64_t>((a.n + NF * Q - 1) / (NF * Q), 512), (a.n >> 22) + 1);
	const cgpu_snapshot sf = with_lds_hot(s, X4_LDS_BUDGET / 8u);
	/* the cold-slot cache in the LDS the hot slots leave */
	const size_t hot = (size_t)sf.hot_slots * 8u;
	const uint32_t cc_n = (s.schedule & CGPU_SCHED_NO_CCACHE) ? 0u : cc_entries(hot);
	/* pk stays exact for PKC_CHUNK packets per slot: unpack after each chunk */
	for (uint64_t lo = 0; lo < a.n; lo += PKC_CHUNK) {
		const uint64_t hi = std::min<uint64_t>(a.n, lo + PKC_CHUNK);
		hipLaunchKernelGGL((k_ct_finish<NF, K, Q>), dim3((unsigned)gf), dim3(NF), hot + (size_t)cc_n * 12u, st,
				   sf, a, cc_n, lo, hi);
		hipError_t e = hipGetLastError();
		if (e != hipSuccess)
			return e;
		if (s.cold_hi) {
			const unsigned ug = std::min<unsigned>((s.cold_hi + 255) / 256, 1024);
			hipLaunchKernelGGL(k_unpack, dim3(ug), dim3(256), 0, st, a.delta, a.pk, 0u, s.cold_hi);
			if ((e = hipGetLastError()) != hipSuccess)
				return e;
		}
	}
	return hipSuccess;
}

/* phase 2 of the plain paths (and of the IPv6 service path): the ICMP
 * errors and the owed ICMP entries of the creates, grouped by address pair,
 * in batch order (the prep and the walk set the candidate flags) */
template <class K>
static hipError_t ct_phase2(const cgpu_snapshot &s, const ct_table &T, const ct_launch &L, ct_args &a,
			    hipStream_t st)
{
	hipError_t e = ct_select(L.flags2, 2 * L.n, L.idx, L.n_heads, static_cast<uint32_t *>(L.temp), st);
	if (e != hipSuccess)
		return e;
	uint32_t m = 0, nh = 0;
	e = hipMemcpyAsync(&m, L.n_heads, 4, hipMemcpyDeviceToHost, st);
	if (e != hipSuccess || (e = hipStreamSynchronize(st)) != hipSuccess)
		return e;
	if (!m)
		return hipSuccess;
	const unsigned gm = (unsigned)std::min<uint64_t>((m + 255) / 256, 8192);
	hipLaunchKernelGGL(k_ct_owed_keys<K>, dim3(gm), dim3(256), 0, st, a, m, 0u);
	e = ct_group_sort(s, L, a, m, &nh, st, K::V6 != 0);
	if (e != hipSuccess)
		return e;
	hipLaunchKernelGGL((k_ct_walk<K, WALK_OWED>), dim3(CT_WALK_GRID), dim3(256), 0, st, s, T, a);
	return hipGetLastError();
}

template <class K>
static hipError_t launch_ct(const cgpu_snapshot &s, const ct_table &T, const ct_launch &L, hipStream_t st)
{
	ct_args a = ct_args_of(L);
	/* the IPv6 preps: the trie pre-pass (its entries into idx_sorted, free
	 * until the group sort) when it can fold the egress fallback identity */
	const bool pre6 = s.cluster_id && s.cluster_id <= DIR_PAYLOAD_MASK;
	/* the orientation-default results (CT_DFLT) with the Q preps */
	if (!CGPU_CT_DFLT || (K::V6 && !pre6))
		a.dflt = 0u;
	const unsigned g = (unsigned)std::min<uint64_t>((L.n + 255) / 256, 8192);
	if (K::V6) {
		if (pre6) {
			constexpr int NT = 1024, QP = CGPU_DIAG_IPC6_PRE_Q, Q = 4;
			const size_t lds = (size_t)(v6t_lds_words(s.ipc6) + v6t_lds_bloom(s.ipc6)) * 4u;
			const unsigned res = resident_blocks((const void *)k_ipc6_pre<QP, NT>, NT, lds);
			const unsigned gp = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((L.n + QP * NT - 1) / (QP * NT), res));
			hipLaunchKernelGGL((k_ipc6_pre<QP, NT>), dim3(gp), dim3(NT), lds, st, s,
					   static_cast<const uint4 *>(L.saddr), static_cast<const uint4 *>(L.daddr), L.flags,
					   L.idx_sorted, L.n, nullptr);
			const unsigned gq = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((L.n + 256 * Q - 1) / (256 * Q), 8192));
			hipLaunchKernelGGL((k_ct_prep6_q<Q>), dim3(gq), dim3(256), 0, st, s, a, L.idx_sorted);
		} else {
			hipLaunchKernelGGL(k_ct_prep6<false>, dim3(g), dim3(256), 0, st, s, a);
		}
	} else {
		constexpr int Q = CGPU_CT_Q;
		const unsigned gq = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((L.n + 256 * Q - 1) / (256 * Q), 8192));
		hipLaunchKernelGGL((k_ct_prep_q<Q>), dim3(gq), dim3(256), 0, st, s, a);
	}
	if (T.lru) {
		/* LRU mode: every key the batch can touch into the filter the
		 * evictions avoid (the prep's records are complete) */
		hipError_t e0 = hipMemsetAsync(const_cast<uint32_t *>(T.bloom), 0, ((size_t)T.bloom_mask + 1u) * 4u, st);
		if (e0 != hipSuccess)
			return e0;
		hipLaunchKernelGGL(k_ct_mark<K>, dim3(g), dim3(256), 0, st, a, const_cast<uint32_t *>(T.bloom),
				   T.bloom_mask);
	}
	uint32_t nh;
	hipError_t e = ct_group_sort(s, L, a, L.n, &nh, st, K::V6 != 0);
	if (e != hipSuccess)
		return e;
	hipLaunchKernelGGL((k_ct_walk<K, WALK_PKT>), dim3(CT_WALK_GRID), dim3(256), 0, st, s, T, a);
	if ((e = ct_phase2<K>(s, T, L, a, st)) != hipSuccess)
		return e;
	return launch_ct_finish<K>(s, a, st);
}

hipError_t launch_classify_v4_ct(const cgpu_snapshot &s, const ct_table &T, const ct_launch &L,
				 hipStream_t st)
{
	return launch_ct<CtK4>(s, T, L, st);
}

hipError_t launch_classify_v6_ct(const cgpu_snapshot &s, const ct_table &T, const ct_launch &L,
				 hipStream_t st)
{
	return launch_ct<CtK6>(s, T, L, st);
}

/* the service walk over the packets k_svc_prep{,6} flagged: compacted (the
 * count sizes the radix sort: a host read), their keys gathered, grouped,
 * walked */
template <class K>
static hipError_t ct_svc_walk(const cgpu_snapshot &s, const ct_table &T, const ct_launch &L, ct_args &a,
			      hipStream_t st)
{
	hipError_t e = ct_select(L.flags2, L.n, L.idx, L.n_heads, static_cast<uint32_t *>(L.temp), st);
	if (e != hipSuccess)
		return e;
	uint32_t m = 0;
	e = hipMemcpyAsync(&m, L.n_heads, 4, hipMemcpyDeviceToHost, st);
	if (e != hipSuccess || (e = hipStreamSynchronize(st)) != hipSuccess)
		return e;
	if (!m)
		return hipSuccess;
	const unsigned gm = (unsigned)std::min<uint64_t>((m + 255) / 256, 8192);
	hipLaunchKernelGGL(k_gather_u32, dim3(gm), dim3(256), 0, st, (const uint32_t *)L.gkey_sorted,
			   (const uint32_t *)L.idx, L.gkey, m);
	uint32_t nh;
	if ((e = ct_group_sort(s, L, a, m, &nh, st, K::V6 != 0)) != hipSuccess)
		return e;
	hipLaunchKernelGGL((k_ct_walk<K, WALK_SVC>), dim3(CT_WALK_GRID), dim3(256), 0, st, s, T, a);
	return hipGetLastError();
}

/* cgpu_classify_v6_ctlb: the IPv6 service walk (k_svc_prep6, WALK_SVC over
 * CtK6), then the IPv6 conntrack path with the service's state: phase 1 by
 * connection, phase 2 the ICMPv6 errors and owed ICMPv6 entries by address
 * pair, as the plain path (ct_create6 writes no address entry) */
hipError_t launch_classify_v6_ctlb(const cgpu_snapshot &s, const ct_table &T, const ct_launch &L,
				   hipStream_t st)
{
	ct_args a = ct_args_of(L);
	const unsigned g = (unsigned)std::min<uint64_t>((L.n + 255) / 256, 8192);
	hipLaunchKernelGGL(k_svc_prep6, dim3(g), dim3(256), 0, st, s, a);
	uint32_t nh;
	hipError_t e = ct_svc_walk<CtK6>(s, T, L, a, st);
	if (e != hipSuccess)
		return e;
	if (CGPU_CT_SVC_PRE6 && s.cluster_id && s.cluster_id <= DIR_PAYLOAD_MASK && !CGPU_CT_SVC_DECQ6) {
		/* as the plain IPv6 path: the ipcache lookups (on the translated
		 * daddr) through the trie pre-pass into idx_sorted (free between
		 * the service walk and the group sort), then Q packets per lane */
		constexpr int NT = 1024, QP = CGPU_DIAG_IPC6_PRE_Q, Q = 4;
		const size_t lds = (size_t)(v6t_lds_words(s.ipc6) + v6t_lds_bloom(s.ipc6)) * 4u;
		const unsigned res = resident_blocks((const void *)k_ipc6_pre<QP, NT>, NT, lds);
		const unsigned gp = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((L.n + QP * NT - 1) / (QP * NT), res));
		hipLaunchKernelGGL((k_ipc6_pre<QP, NT>), dim3(gp), dim3(NT), lds, st, s,
				   static_cast<const uint4 *>(L.saddr), static_cast<const uint4 *>(L.daddr), L.flags,
				   L.idx_sorted, L.n, static_cast<const uint4 *>(a.svc_out));
		const unsigned gq = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((L.n + 256 * Q - 1) / (256 * Q), 8192));
		hipLaunchKernelGGL((k_ct_prep6_q<Q, true>), dim3(gq), dim3(256), 0, st, s, a, L.idx_sorted);
	} else {
		a.dflt = 0u; /* k_ct_prep6 stores every result */
		hipLaunchKernelGGL(k_ct_prep6<true>, dim3(g), dim3(256), 0, st, s, a);
		launch_ct_decq<CtK6S>(s, a, st);
	}
	e = ct_group_sort(s, L, a, L.n, &nh, st, true);
	if (e != hipSuccess)
		return e;
	hipLaunchKernelGGL((k_ct_walk<CtK6S, WALK_PKT>), dim3(CT_WALK_GRID), dim3(256), 0, st, s, T, a);
	if ((e = ct_phase2<CtK6S>(s, T, L, a, st)) != hipSuccess)
		return e;
	return launch_ct_finish<CtK6S>(s, a, st);
}

/*
 * cgpu_classify_v4_ctlb: the service walk, then the conntrack path.
 *   1 k_svc_prep + group sort + k_ct_walk<WALK_SVC>: lb4_local for every
 *     service packet, groups = {saddr, service address}, in batch order.
 *   2 k_ct_prep<SVC>: the translated tuples (svc_out), their decisions and
 *     the ct_state their creates store.
 *   3 group sort + k_ct_walk<WALK_PKT> (phase 1): every packet outside the
 *     pairs address entries can land in and but ICMP errors, grouped by
 *     connection; an address entry of another pair and the ICMP entry of
 *     every create are reserved and owed (CT_ADDRP, CT_RELP).
 *   4 phase 2 (only when something is owed or runs in it): the owed
 *     entries and the phase-2 packets, grouped by address pair, in batch
 *     order: 2a the ordinary pairs (ICMP errors, owed ICMP entries), then 2b
 *     the special pairs (their packets, the owed address entries, which
 *     land only there; see k_ct_owed_flags).
 *   5 k_ct_finish.
 * A batch where a packet of the special pairs (addresses 0 / IPV4_LOOPBACK
 * as endpoints or service backends) itself owes an address entry runs the
 * conntrack path as ONE group (exact, serial).
 */
hipError_t launch_classify_v4_ctlb(const cgpu_snapshot &s, const ct_table &T, const ct_launch &L,
				   hipStream_t st)
{
	ct_args a = ct_args_of(L);
	const unsigned g = (unsigned)std::min<uint64_t>((L.n + 255) / 256, 8192);
	hipLaunchKernelGGL(k_svc_prep, dim3(g), dim3(256), 0, st, s, a);
	uint32_t nh;
	hipError_t e = ct_svc_walk<CtK4>(s, T, L, a, st);
	if (e != hipSuccess)
		return e;
	e = hipMemsetAsync(a.ctl, 0, 16, st);
	if (e != hipSuccess)
		return e;
	if (CGPU_CT_SVC_Q > 1) {
		constexpr int Q = CGPU_CT_SVC_Q > 1 ? CGPU_CT_SVC_Q : 2;
		const unsigned gq = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((L.n + 256 * Q - 1) / (256 * Q), 8192));
		hipLaunchKernelGGL((k_ct_prep_svc_q<Q>), dim3(gq), dim3(256), 0, st, s, a, true);
	} else {
		hipLaunchKernelGGL((k_ct_prep<true, false>), dim3(g), dim3(256), 0, st, s, a, true);
	}
	uint32_t ctl[4];
	e = hipMemcpyAsync(ctl, a.ctl, 16, hipMemcpyDeviceToHost, st);
	if (e != hipSuccess || (e = hipStreamSynchronize(st)) != hipSuccess)
		return e;
	const bool serial = ctl[0] != 0;
	if (serial) {
		a.dflt = 0u; /* one group: every result stored */
		hipLaunchKernelGGL((k_ct_prep<true, true>), dim3(g), dim3(256), 0, st, s, a);
	}
	launch_ct_decq<CtK4S>(s, a, st);
	e = ct_group_sort(s, L, a, L.n, &nh, st);
	if (e != hipSuccess)
		return e;
	hipLaunchKernelGGL((k_ct_walk<CtK4S, WALK_PKT>), dim3(CT_WALK_GRID), dim3(256), 0, st, s, T, a);
	if (!serial && (ctl[1] || ctl[2])) {
		const unsigned g2 = (unsigned)std::min<uint64_t>((L.n + 255) / 256, 8192);
		for (uint32_t ph = 0; ph < 2u; ph++) {
			hipLaunchKernelGGL(k_ct_owed_flags, dim3(g2), dim3(256), 0, st, a,
					   reinterpret_cast<uint32_t *>(L.flags2), ph);
			e = ct_select(L.flags2, 4 * L.n, L.idx, L.n_heads, static_cast<uint32_t *>(L.temp), st);
			if (e != hipSuccess)
				return e;
			uint32_t m = 0;
			e = hipMemcpyAsync(&m, L.n_heads, 4, hipMemcpyDeviceToHost, st);
			if (e != hipSuccess || (e = hipStreamSynchronize(st)) != hipSuccess)
				return e;
			if (!m)
				continue;
			const unsigned gm = (unsigned)std::min<uint64_t>((m + 255) / 256, 8192);
			/* 2b: the address entries of pairs no phase-2 packet reads go by
			 * key (the filter in temp, free between the selection and the
			 * sort) */
			uint32_t *bl = nullptr;
			if (ph == 1u && CGPU_OWED_BY_KEY) {
				bl = static_cast<uint32_t *>(L.temp);
				if ((e = hipMemsetAsync(bl, 0, OWED_BLOOM_WORDS * 4u, st)) != hipSuccess)
					return e;
				hipLaunchKernelGGL(k_ct_owed_bloom<CtK4S>, dim3(gm), dim3(256), 0, st, a, m, bl);
			}
			hipLaunchKernelGGL(k_ct_owed_keys<CtK4S>, dim3(gm), dim3(256), 0, st, a, m, 0u,
					   (const uint32_t *)bl);
			e = ct_group_sort(s, L, a, m, &nh, st);
			if (e != hipSuccess)
				return e;
			hipLaunchKernelGGL((k_ct_walk<CtK4S, WALK_OWED>), dim3(CT_WALK_GRID), dim3(256), 0, st, s, T, a);
		}
	}
	return launch_ct_finish<CtK4S>(s, a, st);
}

/* ======================================================================= */
/* L3 MapState compilation                               */
/* The batched selector match behind computeDesiredL3PolicyMapEntries      */
/* (pkg/endpoint/policy.go:317-390): one lane per (endpoint, identity).    */
/* ======================================================================= */
struct l3_dev {
	const cgpu_selector *sel;
	const cgpu_requirement *req;
	const uint32_t *val;
	const uint32_t *rule_subject, *rule_clauses;
	uint32_t n_rules;
	const cgpu_l3_clause *cl;
	const uint32_t *ep_off, *id_off;
	const cgpu_label *ep_lab, *id_lab;
	uint32_t n_ep, n_id, flags;
	uint8_t *subj;  /* [n_ep][n_rules] rule subject matches the endpoint */
	uint8_t *allow; /* [n_ep][n_id] */
	const uint32_t *ep_flags; /* per-endpoint enforcement (cgpu_mapstate_sync) or nullptr */
	const cgpu_l4_filter *flt;
	const uint32_t *flt_sels;
	uint32_t n_flt;
	uint64_t *l4bits;
};

/* EndpointSelector.Matches (api/selector.go:277-302) of labels [l0, l1):
 * Requirement.Matches (k8s labels/selector.go:193-208) with
 * LabelArray.Has / Get (pkg/labels/array.go:92-130: the first label whose
 * key, for the "any" source, or "source.key" matches) */
__device__ __forceinline__ bool l3_match(const l3_dev &P, uint32_t s, const cgpu_label *lab, uint32_t l0,
					 uint32_t l1)
{
	const cgpu_selector S = P.sel[s];
	if (S.match_all)
		return true;
	for (uint32_t q = 0; q < S.n_reqs; q++) {
		const cgpu_requirement R = P.req[S.reqs_off + q];
		int hit = -1;
		for (uint32_t l = l0; l < l1 && hit < 0; l++) {
			const cgpu_label L = lab[l];
			if ((R.any_source ? L.key : L.ext_key) == R.key)
				hit = (int)L.value;
		}
		bool in = false;
		if (hit >= 0)
			for (uint32_t v = 0; v < R.n_values; v++)
				in |= P.val[R.values_off + v] == (uint32_t)hit;
		const bool has = hit >= 0;
		bool ok;
		if (R.op == CGPU_SEL_IN)
			ok = has && in;
		else if (R.op == CGPU_SEL_NOT_IN)
			ok = !(has && in);
		else if (R.op == CGPU_SEL_EXISTS)
			ok = has;
		else
			ok = !has;
		if (!ok)
			return false;
	}
	return true;
}

/* rule subjects against every endpoint: the EndpointSelector is matched
 * against ctx.To (ingress) and ctx.From (egress), both the endpoint */
__global__ __launch_bounds__(256) void k_l3_subject(l3_dev P)
{
	const uint64_t n = (uint64_t)P.n_ep * P.n_rules;
	for (uint64_t t = (uint64_t)blockIdx.x * 256u + threadIdx.x; t < n; t += (uint64_t)gridDim.x * 256u) {
		const uint32_t e = (uint32_t)(t / P.n_rules), r = (uint32_t)(t % P.n_rules);
		P.subj[t] = l3_match(P, P.rule_subject[r], P.ep_lab, P.ep_off[e], P.ep_off[e + 1]) ? 1u : 0u;
	}
}

/* Repository.Allows{Ingress,Egress}LabelAccess (repository.go:80-130,
 * :443-490) over rule.canReach{Ingress,Egress} (rule.go:323-405): a rule
 * with a failing Requires ends the walk Denied; one whose Endpoints match
 * without ToPorts makes it Allowed; Allowed only if the walk ends Allowed */
__global__ __launch_bounds__(256) void k_l3_pairs(l3_dev P)
{
	const uint64_t n = (uint64_t)P.n_ep * P.n_id;
	for (uint64_t t = (uint64_t)blockIdx.x * 256u + threadIdx.x; t < n; t += (uint64_t)gridDim.x * 256u) {
		const uint32_t e = (uint32_t)(t / P.n_id), i = (uint32_t)(t % P.n_id);
		const uint32_t l0 = P.id_off[i], l1 = P.id_off[i + 1];
		int dec0 = 0, dec1 = 0; /* 0 undecided, 1 allowed, -1 denied */
		for (uint32_t r = 0; r < P.n_rules && (dec0 >= 0 || dec1 >= 0); r++) {
			if (!P.subj[(uint64_t)e * P.n_rules + r])
				continue;
			bool den0 = false, den1 = false, al0 = false, al1 = false;
			for (uint32_t c = P.rule_clauses[r]; c < P.rule_clauses[r + 1]; c++) {
				const cgpu_l3_clause C = P.cl[c];
				const bool live = C.dir == CGPU_L3_INGRESS ? dec0 >= 0 : dec1 >= 0;
				if (!live || (C.kind == CGPU_L3_ALLOWS && C.has_ports))
					continue;
				const bool m = l3_match(P, C.selector, P.id_lab, l0, l1);
				if (C.kind == CGPU_L3_REQUIRES && !m) {
					if (C.dir == CGPU_L3_INGRESS)
						den0 = true;
					else
						den1 = true;
				} else if (C.kind == CGPU_L3_ALLOWS && m) {
					if (C.dir == CGPU_L3_INGRESS)
						al0 = true;
					else
						al1 = true;
				}
			}
			if (dec0 >= 0)
				dec0 = den0 ? -1 : (al0 ? 1 : dec0);
			if (dec1 >= 0)
				dec1 = den1 ? -1 : (al1 ? 1 : dec1);
		}
		const uint32_t fl = P.ep_flags ? P.ep_flags[e] : P.flags;
		P.allow[t] = (uint8_t)(((!(fl & CGPU_L3_INGRESS_ENFORCED) || dec0 == 1) ? 1u : 0u) |
				       ((!(fl & CGPU_L3_EGRESS_ENFORCED) || dec1 == 1) ? 2u : 0u));
	}
}

/* computeDesiredL4PolicyMapEntries (pkg/endpoint/policy.go:110-129,143-192):
 * a filter yields the key {identity, port, proto, dir} for every identity
 * one of its Endpoints selectors matches (getSecurityIdentities).  One wave
 * per (filter, 64 consecutive identities): each lane ORs the filter's
 * selectors over its identity's labels and the wave's ballot is the bitmap
 * word, so the output is 1 bit per pair and the store is one u64 per wave. */
__global__ __launch_bounds__(256) void k_ms_l4(l3_dev P)
{
	const uint32_t lane = threadIdx.x & 63u;
	const uint64_t nw = ((uint64_t)P.n_id + 63u) >> 6;
	const uint64_t n = (uint64_t)P.n_flt * nw;
	for (uint64_t w = ((uint64_t)blockIdx.x * 256u + threadIdx.x) >> 6; w < n;
	     w += ((uint64_t)gridDim.x * 256u) >> 6) {
		const uint32_t f = (uint32_t)(w / nw);
		const uint32_t i = (uint32_t)((w % nw) << 6) + lane;
		bool m = false;
		if (i < P.n_id) {
			const cgpu_l4_filter F = P.flt[f];
			const uint32_t l0 = P.id_off[i], l1 = P.id_off[i + 1];
			for (uint32_t k = 0; k < F.n_sels && !m; k++)
				m = l3_match(P, P.flt_sels[F.sels_off + k], P.id_lab, l0, l1);
		}
		const uint64_t b = __ballot(m);
		if (lane == 0)
			P.l4bits[w] = b;
	}
}

hipError_t launch_l3_compile(const l3_launch &L, hipStream_t st)
{
	const l3_dev P{L.sel, L.req, L.val, L.rule_subject, L.rule_clauses, L.n_rules, L.cl,
		       L.ep_off, L.id_off, L.ep_lab, L.id_lab, L.n_ep, L.n_id, L.flags, L.subj, L.allow,
		       L.ep_flags, L.flt, L.flt_sels, L.n_flt, L.l4bits};
	const uint64_t ns = (uint64_t)L.n_ep * L.n_rules, np = (uint64_t)L.n_ep * L.n_id;
	if (ns)
		hipLaunchKernelGGL(k_l3_subject, dim3((unsigned)std::min<uint64_t>((ns + 255) / 256, 8192)),
				   dim3(256), 0, st, P);
	if (np)
		hipLaunchKernelGGL(k_l3_pairs, dim3((unsigned)std::min<uint64_t>((np + 255) / 256, 16384)),
				   dim3(256), 0, st, P);
	const uint64_t nfw = (uint64_t)L.n_flt * (((uint64_t)L.n_id + 63u) >> 6); /* waves */
	if (nfw && L.l4bits)
		hipLaunchKernelGGL(k_ms_l4, dim3((unsigned)std::min<uint64_t>((nfw + 3) / 4, 16384)),
				   dim3(256), 0, st, P);
	return hipGetLastError();
}
