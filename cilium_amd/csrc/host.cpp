/*
 * host.cpp — C ABI (include/cgpu.h): host mirror of the reference maps,
 * table compiler (mirror -> HBM snapshot), counters, batch launch wrappers.
 *
 * The host mirror is the authoritative copy of every table (SURVEY §5:
 * "the host keeps the authoritative table mirror, so the device can be
 * rebuilt from it at any time"); cgpu_commit() compiles it into the device
 * layouts of tables.h and publishes the result as an immutable snapshot.
 * Map semantics follow the kernel maps the reference programs:
 *   BPF_MAP_TYPE_LPM_TRIE  kernel/bpf/lpm_trie.c (ipcache, prefilter dyn)
 *   BPF_MAP_TYPE_HASH      kernel/bpf/hashtab.c  (policy, prefilter fix, lxc)
 */
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <cerrno>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/cgpu.h"
#include "launch.h"
#include "tables.h"

#define CGPU_EXPORT extern "C" __attribute__((visibility("default")))

static_assert(sizeof(cgpu_policy_key) == 8, "policy_key layout");
static_assert(sizeof(cgpu_policy_entry) == 24, "policy_entry layout");
static_assert(sizeof(cgpu_ipcache_key) == 24, "ipcache_key layout");
static_assert(sizeof(cgpu_remote_endpoint_info) == 8, "remote_endpoint_info layout");
static_assert(sizeof(cgpu_endpoint_key) == 20, "endpoint_key layout");
static_assert(sizeof(pol_slot) == 16, "policy slot");
static_assert(sizeof(set16_slot) == 32, "set16 slot");
static_assert(sizeof(cgpu_lb4_key) == 8, "lb4_key layout");
static_assert(sizeof(cgpu_lb4_service) == 12, "lb4_service layout");
static_assert(sizeof(cgpu_lb6_key) == 20, "lb6_key layout");
static_assert(sizeof(cgpu_lb6_service) == 24, "lb6_service layout");

namespace {

thread_local std::string g_last_error;

int fail(int err, const char *fmt, ...)
{
	char buf[512];
	va_list ap;
	va_start(ap, fmt);
	vsnprintf(buf, sizeof(buf), fmt, ap);
	va_end(ap);
	g_last_error = buf;
	return err;
}

#define HIP_OR_EIO(expr)                                                                  \
	do {                                                                              \
		hipError_t e_ = (expr);                                                   \
		if (e_ != hipSuccess)                                                     \
			return fail(-EIO, "%s: %s", #expr, hipGetErrorString(e_));        \
	} while (0)

/* ---------------- LPM canonical keys (kernel lpm_trie identity) ---------- */
template <size_t N> struct LpmKey {
	uint32_t plen;
	std::array<uint8_t, N> data;
	bool operator<(const LpmKey &o) const
	{
		if (data != o.data)
			return data < o.data;
		return plen < o.plen;
	}
	bool operator==(const LpmKey &o) const { return plen == o.plen && data == o.data; }
};

template <size_t N> LpmKey<N> lpm_canon(uint32_t plen, const uint8_t *data)
{
	LpmKey<N> k;
	k.plen = plen;
	for (size_t i = 0; i < N; i++) {
		uint32_t bit0 = (uint32_t)i * 8;
		uint8_t b = data[i];
		if (plen <= bit0)
			b = 0;
		else if (plen < bit0 + 8)
			b &= (uint8_t)(0xFFu << (8 - (plen - bit0)));
		k.data[i] = b;
	}
	return k;
}

/* does the first `bits` bits of a and b agree (MSB first per byte) */
static bool prefix_eq(const uint8_t *a, const uint8_t *b, uint32_t bits)
{
	uint32_t i = 0;
	for (; i + 8 <= bits; i += 8)
		if (a[i / 8] != b[i / 8])
			return false;
	if (i < bits) {
		uint8_t m = (uint8_t)(0xFFu << (8 - (bits - i)));
		if ((a[i / 8] ^ b[i / 8]) & m)
			return false;
	}
	return true;
}

static uint32_t next_pow2(uint64_t x)
{
	uint32_t p = 1;
	while (p < x)
		p <<= 1;
	return p;
}

static inline uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

struct IpcEntry {
	cgpu_ipcache_key raw;
	cgpu_remote_endpoint_info val;
};
struct PolEntry {
	uint16_t proxy_port;
	uint32_t slot;
	uint64_t first_epoch; /* first snapshot whose inputs hold this key */
};
struct SlotInit {
	uint32_t slot;
	uint64_t packets, bytes;
};

/* ---------------- DIR-24-8 builder ---------------- */
struct Dir248 {
	std::vector<uint32_t> tbl24, tbl8, vals;
	void init() { tbl24.assign(DIR_TBL24_ENTRIES, 0u); tbl8.clear(); vals.clear(); }
	uint32_t encode(uint32_t label)
	{
		if (label < (1u << DIR_TAG_SHIFT))
			return DIR_TAG_DIRECT | label;
		vals.push_back(label);
		return DIR_TAG_INDIRECT | (uint32_t)(vals.size() - 1);
	}
	/* apply in ascending rank order; len in [0, 32], addr host order */
	void apply(uint32_t addr, uint32_t len, uint32_t enc)
	{
		if (len <= 24) {
			uint32_t cnt = 1u << (24 - len);
			uint32_t base = len == 0 ? 0 : ((addr >> 8) & ~(cnt - 1));
			std::fill(tbl24.begin() + base, tbl24.begin() + base + cnt, enc);
			return;
		}
		uint32_t idx = addr >> 8, e = tbl24[idx];
		if ((e & DIR_TAG_MASK) != DIR_TAG_GROUP) {
			uint32_t g = (uint32_t)(tbl8.size() / 256);
			tbl8.resize(tbl8.size() + 256, e);
			tbl24[idx] = DIR_TAG_GROUP | g;
		}
		uint32_t g = tbl24[idx] & DIR_PAYLOAD_MASK;
		uint32_t cnt = 1u << (32 - len);
		uint32_t lo = (addr & 255u) & ~(cnt - 1);
		std::fill(tbl8.begin() + g * 256 + lo, tbl8.begin() + g * 256 + lo + cnt, enc);
	}
};

/* ---------------- DIR-24-8 -> compressed LPM (tables.h lpm16c) ----------
 * Compiled from the host DIR-24-8 image one /16 at a time, so that a commit
 * of a few ipcache changes recompiles only the /16s their prefixes cover
 * (patch); nodes of replaced /16s become garbage until the next full build. */
struct Lpm16cBuild {
	std::vector<uint32_t> d16, nodes, x16, dict;
	std::unordered_map<uint32_t, uint32_t> code; /* leaf -> dict index */
	size_t nodes_at_build = 0;
	/* run list over one block: (start, leaf) with distinct neighbours */
	typedef std::vector<std::pair<uint32_t, uint32_t>> Runs;
	static void push(Runs &r, uint32_t start, uint32_t v)
	{
		if (r.empty() || r.back().second != v)
			r.push_back({start, v});
	}
	/* a run node of kind 0..2 for <= LPMC_MAX_RUN_BOUNDS boundaries */
	uint32_t emit_node(const Runs &r)
	{
		const uint32_t k = (uint32_t)r.size() - 1;
		const uint32_t kind = k <= 2 ? 0u : (k <= 4 ? 1u : 2u);
		const uint32_t nb = kind == 0 ? 1u : (kind == 1 ? 2u : 5u);
		const uint32_t words = kind == 0 ? 4u : (kind == 1 ? 8u : 16u);
		const uint32_t off = (uint32_t)(nodes.size() / 4);
		nodes.resize(nodes.size() + words, 0u);
		uint32_t *w = &nodes[(size_t)off * 4];
		for (uint32_t i = 0; i < 2 * nb; i++) {
			uint32_t b = i < k ? r[i + 1].first : 0xFFFFu;
			w[i / 2] |= (i & 1) ? (b << 16) : b;
		}
		for (uint32_t i = 0; i <= 2 * nb && nb + i < words; i++)
			w[nb + i] = r[std::min<uint32_t>(i, k)].second;
		return DIR_TAG_GROUP | (kind << LPMC_KIND_SHIFT) | off;
	}
	uint32_t emit_array(const uint32_t *ent)
	{
		const uint32_t off = (uint32_t)(nodes.size() / 4);
		nodes.insert(nodes.end(), ent, ent + 256);
		return DIR_TAG_GROUP | (3u << LPMC_KIND_SHIFT) | off;
	}
	/* entry for 256 leaves over the last address byte */
	uint32_t byte_level(const uint32_t *leaf)
	{
		Runs r;
		for (uint32_t j = 0; j < 256; j++)
			push(r, j, leaf[j]);
		if (r.size() == 1)
			return r[0].second;
		if (r.size() - 1 <= LPMC_MAX_RUN_BOUNDS)
			return emit_node(r);
		return emit_array(leaf);
	}
	/* the runs of /16 p (stops collecting past LPMC_MAX_RUN_BOUNDS + 1) */
	static Runs runs16(uint32_t p, const std::vector<uint32_t> &tbl24, const std::vector<uint32_t> &tbl8)
	{
		Runs r;
		const uint32_t *t = &tbl24[(size_t)p * 256];
		for (uint32_t j = 0; j < 256 && r.size() <= LPMC_MAX_RUN_BOUNDS + 1; j++) {
			if ((t[j] & DIR_TAG_MASK) != DIR_TAG_GROUP) {
				push(r, j << 8, t[j]);
				continue;
			}
			const uint32_t *g = &tbl8[(size_t)(t[j] & DIR_PAYLOAD_MASK) * 256];
			for (uint32_t b = 0; b < 256; b++)
				push(r, (j << 8) | b, g[b]);
		}
		return r;
	}
	/* d16 entry of /16 p (emits its nodes) */
	uint32_t entry16(uint32_t p, const Runs &r, const std::vector<uint32_t> &tbl24,
			 const std::vector<uint32_t> &tbl8)
	{
		if (r.size() == 1)
			return r[0].second;
		if (r.size() - 1 <= LPMC_MAX_RUN_BOUNDS)
			return emit_node(r);
		const uint32_t *t = &tbl24[(size_t)p * 256];
		uint32_t ent[256];
		for (uint32_t j = 0; j < 256; j++)
			ent[j] = (t[j] & DIR_TAG_MASK) != DIR_TAG_GROUP
					 ? t[j]
					 : byte_level(&tbl8[(size_t)(t[j] & DIR_PAYLOAD_MASK) * 256]);
		return emit_array(ent);
	}
	/* x16[p]: inline when <= 4 run starts and every leaf has a dict code */
	void inline16(uint32_t p, const Runs &r)
	{
		uint32_t *w = &x16[(size_t)p * 4];
		w[0] = w[1] = w[2] = w[3] = 0;
		bool inl = r.size() <= 5;
		for (size_t i = 0; inl && i < r.size(); i++)
			inl = code.count(r[i].second) != 0;
		if (!inl) {
			w[0] = d16[p];
			w[3] = LPMC_OVERFLOW;
			return;
		}
		const uint32_t k = (uint32_t)r.size() - 1;
		uint64_t v = 0;
		for (uint32_t i = 0; i < 4; i++) {
			uint32_t b = i < k ? r[i + 1].first : 0xFFFFu;
			w[i / 2] |= (i & 1) ? (b << 16) : b;
		}
		for (uint32_t i = 0; i < 5; i++)
			v |= (uint64_t)code.at(r[std::min(i, k)].second) << (12 * i);
		w[2] = (uint32_t)v;
		w[3] = (uint32_t)(v >> 32);
	}
	/* full build: dictionary = the LPMC_DICT most frequent leaves of
	 * inline-able /16s */
	void build(const std::vector<uint32_t> &tbl24, const std::vector<uint32_t> &tbl8)
	{
		d16.assign(65536, 0u);
		nodes.clear();
		std::vector<Runs> all(65536);
		for (uint32_t p = 0; p < 65536; p++) {
			all[p] = runs16(p, tbl24, tbl8);
			d16[p] = entry16(p, all[p], tbl24, tbl8);
		}
		std::map<uint32_t, uint64_t> freq;
		for (auto &r : all)
			if (r.size() <= 5)
				for (auto &x : r)
					freq[x.second]++;
		std::vector<std::pair<uint64_t, uint32_t>> byf;
		for (auto &kv : freq)
			byf.push_back({kv.second, kv.first});
		std::sort(byf.begin(), byf.end(), [](const std::pair<uint64_t, uint32_t> &a,
						     const std::pair<uint64_t, uint32_t> &b) {
			return a.first != b.first ? a.first > b.first : a.second < b.second;
		});
		dict.clear();
		code.clear();
		for (auto &f : byf) {
			if (dict.size() >= LPMC_DICT)
				break;
			code[f.second] = (uint32_t)dict.size();
			dict.push_back(f.second);
		}
		x16.assign((size_t)65536 * 4, 0u);
		for (uint32_t p = 0; p < 65536; p++)
			inline16(p, all[p]);
		nodes_at_build = nodes.size();
	}
	/* recompile /16s [lo, hi] after their DIR-24-8 entries changed; new
	 * leaves join the dictionary while it has room */
	void patch(uint32_t lo, uint32_t hi, const std::vector<uint32_t> &tbl24, const std::vector<uint32_t> &tbl8)
	{
		for (uint32_t p = lo; p <= hi; p++) {
			const Runs r = runs16(p, tbl24, tbl8);
			d16[p] = entry16(p, r, tbl24, tbl8);
			if (r.size() <= 5)
				for (auto &x : r)
					if (!code.count(x.second) && dict.size() < LPMC_DICT) {
						code[x.second] = (uint32_t)dict.size();
						dict.push_back(x.second);
					}
			inline16(p, r);
		}
	}
	/* replaced nodes outweigh live ones: time for a full build */
	bool bloated() const { return nodes.size() > 2 * nodes_at_build + (1u << 16); }
};

struct Rank4 {
	uint32_t rank; /* < 32: static-part entry (acts as /0 below every IP prefix) */
	uint32_t addr; /* host order */
	uint32_t len;
	uint32_t label;
};

/* ---------------- device arena ---------------- */
struct Arena {
	std::vector<std::pair<const void *, size_t>> parts; /* host src, bytes */
	std::vector<size_t> offs;
	size_t total = 0;
	size_t add(const void *src, size_t bytes)
	{
		size_t off = (total + 255) & ~(size_t)255;
		parts.push_back({src, bytes});
		offs.push_back(off);
		total = off + bytes;
		return off;
	}
};

} // namespace

/* ======================================================================= */
/* compiler: mirror -> device layouts                                        */
/* ======================================================================= */
namespace {

uint64_t fnv(uint64_t h, const void *p, size_t n)
{
	const uint8_t *b = (const uint8_t *)p;
	for (size_t i = 0; i < n; i++)
		h = (h ^ b[i]) * 0x100000001b3ull;
	return h;
}

/* ipcache -> DIR-24-8 for IPv4 lookups (ipcache_lookup4, eps.h:70-80):
 * a lookup key is {prefixlen 64, pad 0, family 1, ip4, zero pad words}.
 * An entry is a candidate iff its prefixlen <= 64 and its first prefixlen
 * bits equal the lookup key's.  Entries with prefixlen < 32 end inside the
 * static {pad, family} part: they match every IPv4 address and rank below
 * any entry that reaches the address bits.  Returns false for a key that
 * IPv4 lookups never match. */
static const uint8_t kStaticV4[4] = {0, 0, 0, 1};
bool ipc4_candidate(const cgpu_ipcache_key &raw, uint32_t label, Rank4 *r)
{
	const uint32_t p = raw.prefixlen;
	const uint8_t *data = (const uint8_t *)&raw + 4;
	if (p > 64 || !prefix_eq(data, kStaticV4, std::min<uint32_t>(p, 32)))
		return false;
	r->label = label;
	r->rank = p;
	if (p < 32) {
		r->addr = 0;
		r->len = 0;
	} else {
		r->len = p - 32;
		uint32_t a;
		memcpy(&a, data + 4, 4);
		r->addr = bswap32(a) & (r->len ? ~0u << (32 - r->len) : 0u);
	}
	return true;
}

void build_dir(std::vector<Rank4> cand, Dir248 &d, bool any_match)
{
	std::stable_sort(cand.begin(), cand.end(),
			 [](const Rank4 &a, const Rank4 &b) { return a.rank < b.rank; });
	d.init();
	for (auto &r : cand)
		d.apply(r.addr, r.len, any_match ? (DIR_TAG_DIRECT | 1u) : d.encode(r.label));
}

/* One ipcache change recompiled over the address range of its prefix: the
 * range is refilled with the best entry covering all of it (shorter
 * prefixes or static-part entries), then every entry inside the range is
 * re-applied in rank order -- for each address the highest-ranked covering
 * entry wins, exactly as in the full build. */
struct Ipc4Patch {
	uint32_t addr, len;     /* host order, IP prefix length */
	bool has_cover;
	uint32_t cover_label;
	std::vector<Rank4> subs;
};

void apply_ipc4_patch(const Ipc4Patch &pt, Dir248 &d, Lpm16cBuild &lc)
{
	d.apply(pt.addr, pt.len, pt.has_cover ? d.encode(pt.cover_label) : 0u);
	std::vector<Rank4> subs = pt.subs;
	std::stable_sort(subs.begin(), subs.end(), [](const Rank4 &a, const Rank4 &b) { return a.rank < b.rank; });
	for (auto &r : subs)
		d.apply(r.addr, r.len, d.encode(r.label));
	const uint32_t last = pt.len ? pt.addr + ((pt.len == 32 ? 1u : (1u << (32 - pt.len))) - 1u) : 0xFFFFFFFFu;
	lc.patch(pt.addr >> 16, last >> 16, d.tbl24, d.tbl8);
}

/* prefilter v4 any-match: dyn4 (if CIDR4_LPM_PREFILTER) + fix4 keys with
 * prefixlen 32 (a hash key with another prefixlen never equals the lookup
 * key {32, saddr}); both lead to XDP_DROP (bpf_xdp.c:107-117). */
struct PfIn {
	bool fix4, dyn4, fix6, dyn6;
	std::vector<cgpu_cidr_key> dyn4k, fix4k, dyn6k, fix6k;
};

std::vector<Rank4> pf4_candidates(const PfIn &in)
{
	std::vector<Rank4> cand;
	if (!in.fix4)
		return cand;
	if (in.dyn4)
		for (auto &k : in.dyn4k) {
			uint32_t a;
			memcpy(&a, k.addr, 4);
			const uint32_t h = bswap32(a);
			cand.push_back(Rank4{k.prefixlen, k.prefixlen ? h & (~0u << (32 - k.prefixlen)) : 0u,
					     k.prefixlen, 1});
		}
	for (auto &k : in.fix4k) {
		if (k.prefixlen != 32)
			continue;
		uint32_t a;
		memcpy(&a, k.addr, 4);
		cand.push_back(Rank4{32, bswap32(a), 32, 1});
	}
	return cand;
}

/* ---- policy table (tables.h pol_table): neighbourhood hashing ---- */
struct PolKey {
	uint32_t lo, hi, z, slot; /* key words, ep | proxy << 16, counter slot */
};

#ifndef CGPU_LB_SLOTS_PER_FE
#define CGPU_LB_SLOTS_PER_FE 2
#endif

/* policy table slots per key at a full build (power-of-two rounded) */
#ifndef CGPU_POL_SLOTS_PER_KEY
#define CGPU_POL_SLOTS_PER_KEY 8
#endif

struct PolBuild {
	std::vector<pol_slot> slots;
	uint32_t mask = 0;
	size_t count = 0;
	bool used(uint32_t i) const { return (slots[i & mask].ctr & POL_CTR_MASK) != POL_CTR_EMPTY; }
	/* place one key; false when no free slot can be brought into its
	 * neighbourhood.  Hopscotch insertion: the nearest free slot past the
	 * neighbourhood is moved towards the home slot by relocating keys whose
	 * own neighbourhood still covers it (a key's hop bit lives in ITS home
	 * slot; a slot's own hop bits stay where they are), so the table holds
	 * its keys at up to 50 % load (first-fit needed 512k slots for config 2's
	 * 64k keys even at 2 slots per key) */
	bool insert(const PolKey &k)
	{
		const uint32_t home = pol_hash(k.lo, k.hi, k.z & 0xFFFFu) & mask;
		uint32_t d = 0;
		const uint32_t limit = std::min<uint32_t>(mask + 1u, 4096u);
		while (d < limit && used(home + d))
			d++;
		if (d == limit)
			return false;
		while (d >= POL_HOP) {
			/* free slot f = home + d: move a key of home h2 = f - j (j < HOP)
			 * that sits at h2 + o, o < j, into f */
			const uint32_t f = (home + d) & mask;
			bool moved = false;
			for (uint32_t j = POL_HOP - 1; j >= 1 && !moved; j--) {
				const uint32_t h2 = (f - j) & mask;
				const uint32_t hop2 = slots[h2].ctr >> POL_HOP_SHIFT;
				for (uint32_t o = 0; o < j; o++) {
					if (!((hop2 >> o) & 1u))
						continue;
					pol_slot &src = slots[(h2 + o) & mask], &dst = slots[f];
					dst.key_lo = src.key_lo;
					dst.key_hi = src.key_hi;
					dst.ep_proxy = src.ep_proxy;
					dst.ctr = (dst.ctr & ~POL_CTR_MASK) | (src.ctr & POL_CTR_MASK);
					src.key_lo = src.key_hi = src.ep_proxy = 0;
					src.ctr = (src.ctr & ~POL_CTR_MASK) | POL_CTR_EMPTY;
					slots[h2].ctr = (slots[h2].ctr & ~(1u << (POL_HOP_SHIFT + o))) | (1u << (POL_HOP_SHIFT + j));
					d -= j - o;
					moved = true;
					break;
				}
			}
			if (!moved)
				return false;
		}
		pol_slot &sl = slots[(home + d) & mask];
		sl.key_lo = k.lo;
		sl.key_hi = k.hi;
		sl.ep_proxy = k.z;
		sl.ctr = (sl.ctr & ~POL_CTR_MASK) | k.slot;
		slots[home].ctr |= 1u << (POL_HOP_SHIFT + d);
		count++;
		return true;
	}
	/* remove {lo, hi, ep} if present (the slot keeps its own hop bits) */
	bool erase(uint32_t lo, uint32_t hi, uint32_t ep)
	{
		const uint32_t home = pol_hash(lo, hi, ep) & mask;
		const uint32_t hop = slots[home].ctr >> POL_HOP_SHIFT;
		for (uint32_t d = 0; d < POL_HOP; d++) {
			if (!((hop >> d) & 1u))
				continue;
			pol_slot &sl = slots[(home + d) & mask];
			if (sl.key_lo == lo && sl.key_hi == hi && (sl.ep_proxy & 0xFFFFu) == ep) {
				sl.key_lo = sl.key_hi = sl.ep_proxy = 0;
				sl.ctr = (sl.ctr & ~POL_CTR_MASK) | POL_CTR_EMPTY;
				slots[home].ctr &= ~(1u << (POL_HOP_SHIFT + d));
				count--;
				return true;
			}
		}
		return false;
	}
	/* CGPU_POL_SLOTS_PER_KEY slots per key: at 8 (<= 12.5 % load) nearly
	 * every key sits in its home slot, one gather per probe.  Denser tables
	 * measured slower although smaller (config 2, one session, no rebalance:
	 * 2 MiB 1.80 ms, 4 MiB 1.75, 8 MiB 1.72; profiles/r6_d/ab.log): a key
	 * displaced from its home slot costs a dependent second gather */
	void build(const std::vector<PolKey> &keys)
	{
		uint32_t nb = next_pow2(std::max<uint64_t>(64, (uint64_t)CGPU_POL_SLOTS_PER_KEY * keys.size() + 2));
		for (;;) {
			slots.assign(nb, pol_slot{0, 0, 0, POL_CTR_EMPTY});
			mask = nb - 1;
			count = 0;
			bool ok = true;
			for (auto &k : keys)
				if (!(ok = insert(k)))
					break; /* a neighbourhood is full: grow */
			if (ok)
				return;
			nb *= 2;
		}
	}
	bool overloaded() const { return 2 * count + 2 > slots.size(); }
};

/* ---- policy groups (tables.h pol_groups) ---- */
struct PgBuild {
	std::vector<uint4> slots;
	uint32_t mask = 0;
	size_t count = 0;
	static bool groupable(const PolKey &k) { return !((k.hi >> 25) & 0x7Fu); } /* pad bits 0 */
	static uint32_t ep_dir(const PolKey &k) { return (k.z & 0xFFFFu) | (((k.hi >> 24) & 1u) << 16); }
	/* the group slot of (id, ep | dir << 16), inserted if absent; -1: full */
	int64_t find(uint32_t id, uint32_t ed, bool add)
	{
		const uint32_t home = pg_hash(id, ed) & mask;
		const uint32_t hop = slots[home].y >> POL_HOP_SHIFT;
		for (uint32_t d = 0; d < POL_HOP; d++) {
			const uint4 &x = slots[(home + d) & mask];
			if (((hop >> d) & 1u) && x.x == id && (x.y & 0x1FFFFu) == ed)
				return (home + d) & mask;
		}
		if (!add)
			return -1;
		uint32_t d = 0;
		while (d < POL_HOP && (slots[(home + d) & mask].y & PG_USED))
			d++;
		if (d == POL_HOP)
			return -1;
		uint4 &x = slots[(home + d) & mask];
		x.x = id;
		x.y = (x.y & 0xFF000000u) | ed | PG_USED;
		x.z = POL_CTR_EMPTY;
		x.w = 0;
		slots[home].y |= 1u << (POL_HOP_SHIFT + d);
		count++;
		return (home + d) & mask;
	}
	/* key k (present): its bloom bits, and the counter slot of an L3 key */
	bool add(const PolKey &k)
	{
		if (!groupable(k))
			return true;
		const int64_t g = find(k.lo, ep_dir(k), true);
		if (g < 0)
			return false;
		const uint32_t dport = k.hi & 0xFFFFu, proto = (k.hi >> 16) & 0xFFu;
		slots[g].w |= pg_bloom(dport, proto);
		if (!dport && !proto)
			slots[g].z = k.slot;
		return true;
	}
	/* key k deleted: an L3 key leaves its group (bloom bits stay) */
	void remove(const PolKey &k)
	{
		if (!groupable(k) || (k.hi & 0xFFFFFFu))
			return;
		const int64_t g = find(k.lo, ep_dir(k), false);
		if (g >= 0)
			slots[g].z = POL_CTR_EMPTY;
	}
	void build(const std::vector<PolKey> &keys)
	{
		std::set<std::pair<uint32_t, uint32_t>> groups;
		for (auto &k : keys)
			if (groupable(k))
				groups.insert({k.lo, ep_dir(k)});
		uint32_t nb = next_pow2(std::max<uint64_t>(64, 2 * groups.size() + 2));
		for (;;) {
			slots.assign(nb, uint4{0, 0, POL_CTR_EMPTY, 0});
			mask = nb - 1;
			count = 0;
			bool ok = true;
			for (auto &k : keys)
				if (!(ok = add(k)))
					break;
			if (ok)
				return;
			nb *= 2;
		}
	}
	bool overloaded() const { return 2 * count + 2 > slots.size(); }
};

struct Set4Build {
	std::vector<set4_slot> slots;
	uint32_t mask = 0, max_probe = 1;
};
struct Set16Build {
	std::vector<set16_slot> slots;
	uint32_t mask = 0, max_probe = 1;
};

void build_set4(const std::vector<uint32_t> &keys, Set4Build &b)
{
	uint32_t nb = next_pow2(std::max<uint64_t>(8, keys.size() / 4 + 1));
	b.slots.assign((size_t)nb * 8, set4_slot{0, 0});
	b.mask = nb - 1;
	b.max_probe = 1;
	for (uint32_t a : keys) {
		uint32_t bk = mix32(a, 0x5e7) & b.mask, probe = 1;
		for (;;) {
			set4_slot *s = &b.slots[(size_t)bk * 8];
			int k = 0;
			while (k < 8 && s[k].used)
				k++;
			if (k < 8) {
				s[k] = set4_slot{a, 1};
				break;
			}
			bk = (bk + 1) & b.mask;
			probe++;
		}
		b.max_probe = std::max(b.max_probe, probe);
	}
}

/* keys: 4 u32 words + tag + entry (tag goes to `used` bits 8..15 and is
 * hashed as salt; entry goes to pad[0]); pfx6: bucket by pfx6_hash (v6_lpm
 * prefix keys), else hash16 */
void build_set16(const std::vector<std::array<uint32_t, 6>> &keys, Set16Build &b, bool pfx6 = false)
{
	uint32_t nb = next_pow2(std::max<uint64_t>(8, keys.size() + 1));
	b.slots.assign((size_t)nb * 2, set16_slot{});
	b.mask = nb - 1;
	b.max_probe = 1;
	for (auto &k : keys) {
		uint32_t bk = (pfx6 ? pfx6_hash(k[0], k[1], k[2], k[3], k[4]) : hash16(k[0], k[1], k[2], k[3], k[4])) &
			      b.mask,
			 probe = 1;
		for (;;) {
			set16_slot *s = &b.slots[(size_t)bk * 2];
			int j = 0;
			while (j < 2 && (s[j].used & 1))
				j++;
			if (j < 2) {
				set16_slot v{};
				memcpy(v.a, k.data(), 16);
				v.used = 1u | (k[4] << 8);
				v.pad[0] = k[5];
				s[j] = v;
				break;
			}
			bk = (bk + 1) & b.mask;
			probe++;
		}
		b.max_probe = std::max(b.max_probe, probe);
	}
}

struct Rank6 {
	uint32_t rank; /* apply order: < 32 static-part entries, else 32 + len */
	uint32_t len;  /* IP prefix length 0..128 (static entries: 0) */
	std::array<uint8_t, 16> addr;
	uint32_t label;
};

struct V6Build {
	std::vector<uint32_t> root, b24, b32, pool, vals, rbits;
	std::vector<uint16_t> b24_16; /* empty: not representable */
	std::vector<std::array<uint32_t, 8>> h64;
	uint32_t m64 = 0;
	std::vector<uint32_t> bl64; /* bloom of the /64s with records (tables.h v6_lpm) */
	bool any = false;
	bool too_big = false; /* node lines past V6T_LINE_MASK */
};

uint32_t v6_encode(std::vector<uint32_t> &vals, uint32_t label)
{
	if (label < (1u << DIR_TAG_SHIFT))
		return DIR_TAG_DIRECT | label;
	vals.push_back(label);
	return DIR_TAG_INDIRECT | (uint32_t)(vals.size() - 1);
}

/* a prefix of the v6 trie: address as two host-order halves, the rank it
 * applies in (tables.h v6_lpm: later ranks paint over earlier ones) */
struct T6 {
	uint64_t hi, lo;
	uint32_t len, rank, enc;
};

/* Piecewise-constant labels over [0, end): start -> label.  Painting the
 * prefixes of one range in rank order leaves the highest-ranked cover of
 * every point (prefix intervals nest or are disjoint). */
typedef unsigned __int128 u128;
struct Runs {
	std::map<u128, uint32_t> m;
	u128 end;
	Runs(u128 e, uint32_t base) : end(e) { m[0] = base; }
	uint32_t at(u128 x) const { return std::prev(m.upper_bound(x))->second; }
	void paint(u128 a, u128 b, uint32_t lab) /* [a, b) */
	{
		const uint32_t after = b < end ? at(b) : 0u;
		m.erase(m.lower_bound(a), m.lower_bound(b));
		m[a] = lab;
		if (b < end)
			m[b] = after;
	}
	/* boundaries (points > 0 where the label changes) and the label from each */
	void cuts(std::vector<std::pair<u128, uint32_t>> &out, uint32_t &first) const
	{
		out.clear();
		first = m.begin()->second;
		uint32_t cur = first;
		for (auto it = std::next(m.begin()); it != m.end(); ++it)
			if (it->second != cur) {
				out.push_back({it->first, it->second});
				cur = it->second;
			}
	}
};

/* the /32 node over bits 32..63 (tables.h v6_lpm): returns the b32 entry */
static uint2 v6t_node32(V6Build &b, const std::vector<const T6 *> &ps, uint32_t l32, bool deep)
{
	Runs r((u128)1 << 32, l32);
	for (const T6 *p : ps) /* rank order */
		if (p->len > 32 && p->len <= 64) {
			const uint64_t st = (uint32_t)p->hi;
			r.paint(st, st + (1ull << (64 - p->len)), p->enc);
		}
	std::vector<std::pair<u128, uint32_t>> cut;
	uint32_t first;
	r.cuts(cut, first);
	if (cut.empty() && !deep)
		return make_uint2(first, 0u);
	const uint32_t last = cut.empty() ? first : cut.back().second;
	/* the window: least aligned [base, base + 2^w), w >= 9, holding every
	 * boundary, whose outside (below: first, above: last) has one label */
	uint32_t w = 9, base = 0, outer = first;
	for (;; w++) {
		if (w == 32) {
			base = 0;
			outer = first;
			break;
		}
		const uint64_t lo = cut.empty() ? 0 : (uint64_t)cut.front().first;
		const uint64_t hi = cut.empty() ? 0 : (uint64_t)cut.back().first;
		base = (uint32_t)(lo & ~((1ull << w) - 1));
		const uint64_t top = (uint64_t)base + (1ull << w);
		if (hi > top)
			continue;
		const bool below = base > 0, above = top < (1ull << 32);
		if (below && above && first != last)
			continue;
		outer = below ? first : last;
		break;
	}
	b.pool.resize((b.pool.size() + V6T_LW - 1) / V6T_LW * V6T_LW, 0u);
	const size_t line = b.pool.size() / V6T_LW;
	uint32_t s = 0;
	for (; s <= 6 && s <= w; s++) {
		const uint64_t width = 1ull << (w - s);
		std::vector<std::vector<uint32_t>> lines(1u << s);
		bool fits = true;
		size_t i = 0;
		uint32_t cur = first;
		for (uint32_t k = 0; k < (1u << s) && fits; k++) {
			const uint64_t S = (uint64_t)base + k * width;
			auto &L = lines[k];
			L.assign(V6T_LW, 0xFFFFFFFFu);
			for (; i < cut.size() && (uint64_t)cut[i].first <= S; i++)
				cur = cut[i].second;
			L[V6T_NB] = outer;
			L[V6T_NB + 1] = cur;
			uint32_t n = 0;
			for (; i < cut.size() && (uint64_t)cut[i].first < S + width; i++) {
				if (n == V6T_NB) {
					fits = false;
					break;
				}
				L[n] = (uint32_t)cut[i].first - 1u;
				cur = cut[i].second;
				L[V6T_NB + 1 + ++n] = cur;
			}
			for (uint32_t j = n + 1; j <= V6T_NB; j++)
				L[V6T_NB + 1 + j] = cur;
		}
		if (!fits)
			continue;
		for (auto &L : lines)
			b.pool.insert(b.pool.end(), L.begin(), L.end());
		break;
	}
	if (s > 6 || s > w) {
		s = V6T_LONG;
		w = 32;
		base = 0;
		std::vector<uint32_t> h(V6T_LW, 0u);
		h[0] = (uint32_t)cut.size();
		h[V6T_NB] = first;
		b.pool.insert(b.pool.end(), h.begin(), h.end());
		for (auto &c : cut)
			b.pool.push_back((uint32_t)c.first - 1u);
		b.pool.push_back(first);
		for (auto &c : cut)
			b.pool.push_back(c.second);
		b.pool.resize((b.pool.size() + V6T_LW - 1) / V6T_LW * V6T_LW, 0u);
	}
	b.too_big |= line > V6T_LINE_MASK;
	return make_uint2(DIR_TAG_GROUP | (deep ? V6T_DEEP : 0u) | (uint32_t)line, base | (w - 9u) | s << 5);
}

/* the /64 record of prefixes longer than /64 (ps: one /64, rank order) */
static std::array<uint32_t, 8> v6t_rec64(V6Build &b, uint64_t top, const std::vector<const T6 *> &ps)
{
	Runs r((u128)1 << 64, V6T_FALL);
	for (const T6 *p : ps)
		r.paint(p->lo, (u128)p->lo + ((u128)1 << (128 - p->len)), p->enc);
	std::vector<std::pair<u128, uint32_t>> cut;
	uint32_t first;
	r.cuts(cut, first);
	std::array<uint32_t, 8> rec{(uint32_t)(top >> 32), (uint32_t)top, 0u, 0u, 0u, 0u, 0u, 0u};
	const bool inline1 = first == V6T_FALL && !cut.empty() && cut.size() <= 2 &&
			     (cut.size() == 1 || cut[1].second == V6T_FALL);
	if (inline1) {
		const uint64_t lo = (uint64_t)cut[0].first;
		const uint64_t hi = cut.size() == 2 ? (uint64_t)(cut[1].first - 1) : ~0ull;
		rec[2] = cut[0].second;
		rec[4] = (uint32_t)(lo >> 32);
		rec[5] = (uint32_t)lo;
		rec[6] = (uint32_t)(hi >> 32);
		rec[7] = (uint32_t)hi;
		return rec;
	}
	const uint32_t off = (uint32_t)(b.pool.size() / 4);
	b.pool.insert(b.pool.end(), {(uint32_t)cut.size(), 0u, 0u, 0u});
	for (auto &c : cut) {
		b.pool.push_back((uint32_t)((uint64_t)c.first >> 32));
		b.pool.push_back((uint32_t)(uint64_t)c.first);
	}
	b.pool.push_back(first);
	for (auto &c : cut)
		b.pool.push_back(c.second);
	while (b.pool.size() % 4)
		b.pool.push_back(0u);
	rec[2] = DIR_TAG_GROUP | off;
	return rec;
}

uint32_t h64_home(const std::array<uint32_t, 8> &r) { return mix32(r[0], r[1]); }

template <size_t W>
void hop_place(std::vector<std::array<uint32_t, W>> &tab, uint32_t &mask,
	       const std::vector<std::array<uint32_t, W>> &recs, uint32_t (*home_of)(const std::array<uint32_t, W> &));

/* Longest-prefix trie over (rank, len, address) candidates; see tables.h v6_lpm. */
void build_v6(std::vector<Rank6> cand, V6Build &b)
{
	b.any = !cand.empty();
	if (!b.any)
		return;
	b.vals.clear();
	std::vector<T6> ps;
	ps.reserve(cand.size());
	for (auto &c : cand) {
		uint64_t hi = 0, lo = 0;
		for (int i = 0; i < 8; i++) {
			hi = hi << 8 | c.addr[i];
			lo = lo << 8 | c.addr[8 + i];
		}
		ps.push_back(T6{hi, lo, c.len, c.rank, 0u});
	}
	/* address order, ties by rank: every range's prefixes are contiguous */
	std::vector<uint32_t> ord(ps.size());
	for (uint32_t i = 0; i < ord.size(); i++)
		ord[i] = i;
	std::stable_sort(ord.begin(), ord.end(), [&](uint32_t x, uint32_t y) { return cand[x].rank < cand[y].rank; });
	for (uint32_t i : ord) /* vals in rank order (as the DIR builds) */
		ps[i].enc = v6_encode(b.vals, cand[i].label);
	std::vector<T6> srt(ps);
	std::stable_sort(srt.begin(), srt.end(), [](const T6 &x, const T6 &y) {
		return x.hi != y.hi ? x.hi < y.hi : (x.lo != y.lo ? x.lo < y.lo : x.rank < y.rank);
	});
	auto by_rank = [](std::vector<const T6 *> &v) {
		std::stable_sort(v.begin(), v.end(), [](const T6 *x, const T6 *y) { return x->rank < y->rank; });
	};
	/* /0../16 */
	std::vector<const T6 *> shortp;
	for (auto &p : srt)
		if (p.len <= 16)
			shortp.push_back(&p);
	by_rank(shortp);
	b.root.assign(65536, 0u);
	for (const T6 *p : shortp) {
		const uint32_t cnt = 1u << (16 - p->len);
		const uint32_t base = p->len == 0 ? 0 : ((uint32_t)(p->hi >> 48) & ~(cnt - 1));
		std::fill(b.root.begin() + base, b.root.begin() + base + cnt, p->enc);
	}
	b.pool.assign(V6T_LW, 0xFFFFFFFFu); /* line 0 unused */
	b.b24.clear();
	b.b32.clear();
	std::vector<std::array<uint32_t, 8>> r64;
	size_t i = 0;
	while (i < srt.size()) {
		const uint32_t top16 = (uint32_t)(srt[i].hi >> 48);
		size_t j = i;
		while (j < srt.size() && (uint32_t)(srt[j].hi >> 48) == top16)
			j++;
		std::vector<const T6 *> g16;
		for (size_t k = i; k < j; k++)
			if (srt[k].len > 16)
				g16.push_back(&srt[k]);
		if (g16.empty()) {
			i = j;
			continue;
		}
		std::array<uint32_t, 256> e24;
		e24.fill(b.root[top16]);
		{
			std::vector<const T6 *> v;
			for (const T6 *p : g16)
				if (p->len <= 24)
					v.push_back(p);
			by_rank(v);
			for (const T6 *p : v) {
				const uint32_t cnt = 1u << (24 - p->len);
				const uint32_t base = (uint32_t)(p->hi >> 40) & 0xFFu & ~(cnt - 1);
				std::fill(e24.begin() + base, e24.begin() + base + cnt, p->enc);
			}
		}
		size_t k = 0;
		while (k < g16.size()) {
			const uint32_t x24 = (uint32_t)(g16[k]->hi >> 40) & 0xFFu;
			size_t l = k;
			std::vector<const T6 *> g24;
			for (; l < g16.size() && ((uint32_t)(g16[l]->hi >> 40) & 0xFFu) == x24; l++)
				if (g16[l]->len > 24)
					g24.push_back(g16[l]);
			if (g24.empty()) {
				k = l;
				continue;
			}
			std::array<uint32_t, 256> e32;
			e32.fill(e24[x24]);
			{
				std::vector<const T6 *> v;
				for (const T6 *p : g24)
					if (p->len <= 32)
						v.push_back(p);
				by_rank(v);
				for (const T6 *p : v) {
					const uint32_t cnt = 1u << (32 - p->len);
					const uint32_t base = (uint32_t)(p->hi >> 32) & 0xFFu & ~(cnt - 1);
					std::fill(e32.begin() + base, e32.begin() + base + cnt, p->enc);
				}
			}
			std::array<uint2, 256> n32;
			for (uint32_t x = 0; x < 256; x++)
				n32[x] = make_uint2(e32[x], 0u);
			size_t q = 0;
			while (q < g24.size()) {
				const uint32_t x32 = (uint32_t)(g24[q]->hi >> 32) & 0xFFu;
				size_t r = q;
				std::vector<const T6 *> g32, g64;
				for (; r < g24.size() && ((uint32_t)(g24[r]->hi >> 32) & 0xFFu) == x32; r++)
					if (g24[r]->len > 32)
						(g24[r]->len <= 64 ? g32 : g64).push_back(g24[r]);
				if (!g32.empty() || !g64.empty()) {
					by_rank(g32);
					n32[x32] = v6t_node32(b, g32, e32[x32], !g64.empty());
					/* /64 groups (address order within the /32) */
					size_t m = 0;
					while (m < g64.size()) {
						const uint64_t top = g64[m]->hi;
						std::vector<const T6 *> v;
						for (; m < g64.size() && g64[m]->hi == top; m++)
							v.push_back(g64[m]);
						by_rank(v);
						r64.push_back(v6t_rec64(b, top, v));
					}
				}
				q = r;
			}
			e24[x24] = DIR_TAG_GROUP | (uint32_t)(b.b32.size() / 2 / 256);
			for (auto &e : n32) {
				b.b32.push_back(e.x);
				b.b32.push_back(e.y);
			}
			k = l;
		}
		b.root[top16] = DIR_TAG_GROUP | (uint32_t)(b.b24.size() / 256);
		b.b24.insert(b.b24.end(), e24.begin(), e24.end());
		i = j;
	}
	hop_place<8>(b.h64, b.m64, r64, h64_home);
	/* the bloom of the /64s with records: ~2 records per 32-bit word (3
	 * bits each) keeps false positives near 1 % */
	{
		uint32_t nw = 16;
		while (nw < V6T_BLOOM_MAX_WORDS && nw * 2u < r64.size())
			nw <<= 1;
		b.bl64.assign(nw, 0u);
		for (const auto &r : r64) {
			const uint32_t h = mix32(r[0], r[1]);
			b.bl64[v6_bloom_word(h, nw - 1u)] |= v6_bloom_bits(h);
		}
	}
	/* a line past the last: a lane reads a whole line */
	b.pool.insert(b.pool.end(), V6T_LW, 0xFFFFFFFFu);
	/* LDS-staged forms */
	const uint32_t nb24 = (uint32_t)(b.b24.size() / 256), nb32 = (uint32_t)(b.b32.size() / 512);
	b.rbits.assign(V6T_RBITS_WORDS, 0u);
	uint32_t rank = 0;
	for (uint32_t wd = 0; wd < 2048; wd++) {
		b.rbits[2048 + wd / 2] |= rank << (16 * (wd & 1));
		for (uint32_t k = 0; k < 32; k++)
			if ((b.root[32 * wd + k] & DIR_TAG_MASK) == DIR_TAG_GROUP) {
				b.rbits[wd] |= 1u << k;
				rank++;
			}
	}
	b.b24_16.clear();
	if (nb32 <= 0x7FFFu) {
		b.b24_16.resize(b.b24.size());
		for (size_t x = 0; x < b.b24.size(); x++)
			b.b24_16[x] = (b.b24[x] & DIR_TAG_MASK) == DIR_TAG_GROUP
					      ? (uint16_t)(0x8000u | (b.b24[x] & DIR_PAYLOAD_MASK))
					      : (uint16_t)0u;
	}
	(void)nb24;
}

/* The device lookup (kernels.hip v6_lookup) restated over a V6Build on the
 * host: the trie builder's CPU test hook (cgpu_diag_ipc6_trie) */
static uint32_t v6t_host_lookup(const V6Build &b, const uint8_t *a)
{
	uint32_t w[4];
	for (int i = 0; i < 4; i++)
		w[i] = (uint32_t)a[4 * i] << 24 | (uint32_t)a[4 * i + 1] << 16 | (uint32_t)a[4 * i + 2] << 8 | a[4 * i + 3];
	auto grp = [](uint32_t e) { return (e & DIR_TAG_MASK) == DIR_TAG_GROUP; };
	uint32_t e = b.root[w[0] >> 16];
	if (grp(e))
		e = b.b24[(size_t)(e & DIR_PAYLOAD_MASK) * 256 + ((w[0] >> 8) & 0xFFu)];
	if (!grp(e))
		return e;
	const size_t bi = (size_t)(e & DIR_PAYLOAD_MASK) * 256 + (w[0] & 0xFFu);
	const uint32_t nx = b.b32[2 * bi], ny = b.b32[2 * bi + 1];
	if (!grp(nx))
		return nx;
	const uint32_t x = w[1], wb = (ny & 31u) + 9u, sc = (ny >> 5) & 7u, rel = x - (ny & ~511u);
	size_t line = nx & V6T_LINE_MASK;
	uint32_t lab;
	if (sc == V6T_LONG) {
		const uint32_t n = b.pool[V6T_LW * line];
		uint32_t c = 0;
		for (uint32_t i = 0; i < n; i++)
			c += b.pool[V6T_LW * (line + 1) + i] < x;
		lab = b.pool[V6T_LW * (line + 1) + n + c];
	} else {
		const bool out = wb < 32 && (rel >> wb) != 0;
		const uint32_t sh = wb - sc;
		line += out || sh >= 32 ? 0 : rel >> sh;
		uint32_t c = 0;
		for (uint32_t i = 0; i < V6T_NB; i++)
			c += b.pool[V6T_LW * line + i] < x;
		lab = out ? b.pool[V6T_LW * line + V6T_NB] : b.pool[V6T_LW * line + V6T_NB + 1 + c];
	}
	if (nx & V6T_DEEP) {
		const uint32_t home = mix32(w[0], w[1]) & b.m64;
		const uint32_t hop = b.h64[home][3] >> POL_HOP_SHIFT;
		for (uint32_t d = 0; d < POL_HOP; d++) {
			if (!(hop >> d & 1u))
				continue;
			const auto &r = b.h64[(home + d) & b.m64];
			if (r[0] != w[0] || r[1] != w[1])
				continue;
			const uint64_t xl = (uint64_t)w[2] << 32 | w[3];
			uint32_t v;
			if (grp(r[2])) {
				const uint32_t *p = &b.pool[4 * (size_t)(r[2] & DIR_PAYLOAD_MASK)];
				uint32_t c = 0;
				for (uint32_t i = 0; i < p[0]; i++)
					c += ((uint64_t)p[4 + 2 * i] << 32 | p[5 + 2 * i]) <= xl;
				v = p[4 + 2 * p[0] + c];
			} else {
				const uint64_t lo = (uint64_t)r[4] << 32 | r[5], hi = (uint64_t)r[6] << 32 | r[7];
				v = lo <= xl && xl <= hi ? r[2] : V6T_FALL;
			}
			if (v != V6T_FALL)
				lab = v;
			break;
		}
	}
	return lab;
}

/* ---- IPv6 any-match cover (tables.h cover6) ---- */
struct Cover6Build {
	std::vector<uint32_t> root, b24, b32, pool;
	std::vector<uint16_t> root16, b24_16; /* empty: not representable */
	std::vector<uint32_t> rbits;
	std::vector<std::array<uint32_t, 8>> h64;
	uint32_t m64 = 0;
	bool any = false;
	bool too_big = false; /* node lines past the 25-bit b32 field */
};

struct P6 {
	uint64_t hi, lo;
	uint32_t len;
	bool operator<(const P6 &o) const { return hi != o.hi ? hi < o.hi : lo < o.lo; }
};

/* sorted, merged (overlapping or adjacent) closed intervals */
template <typename T> std::vector<std::pair<T, T>> merge_iv(std::vector<std::pair<T, T>> v)
{
	std::sort(v.begin(), v.end());
	std::vector<std::pair<T, T>> out;
	for (auto &x : v) {
		if (!out.empty() && (x.first <= out.back().second ||
				     (out.back().second != (T)~(T)0 && x.first == out.back().second + 1)))
			out.back().second = std::max(out.back().second, x.second);
		else
			out.push_back(x);
	}
	return out;
}

/* /32 node (tables.h cover6 "node32"): the bits 32..63 range is split into
 * 2^s equal sub-ranges, s the least that fits every sub-range in one 128-B
 * line of 32 slots.  The line of sub-range [S, E] holds b - 1 for every
 * boundary b of the merged covered intervals with S <= b <= E, plus S - 1
 * when an odd number of boundaries lie below S (it counts for every x of
 * the sub-range), 0xFFFFFFFF past the last; a boundary at 0 becomes the
 * entry's flip bit instead.  x is covered iff (flip if x is in sub-range 0)
 * + #(slot < x) over its line is odd.  Parity needs no length, so the 8
 * lanes of an octet read the line with one load and treat their units alike
 * (c6_node32_coop).  Returns the b32 entry NODE << 30 | code << 25 | line,
 * code = flip | deep << 1 | s << 2 (deep: the /32 has h64 records, so an
 * uncovered x consults h64); s = 7 (COVER6_LONG) marks a node that even 64
 * sub-ranges do not fit: one header unit {nb, 0, 0, 0} and all boundaries,
 * scanned whole by its owner lane. */
uint32_t cover6_node32(Cover6Build &b, const std::vector<std::pair<uint32_t, uint32_t>> &iv, bool deep)
{
	std::vector<uint32_t> bnd; /* boundaries b > 0 */
	uint32_t flip = 0;
	for (auto &x : iv) {
		if (x.first)
			bnd.push_back(x.first);
		else
			flip = 1;
		if (x.second != 0xFFFFFFFFu)
			bnd.push_back(x.second + 1u);
	}
	std::sort(bnd.begin(), bnd.end());
	b.pool.resize((b.pool.size() + 31) / 32 * 32, 0u);
	const size_t line = b.pool.size() / 32;
	uint32_t s = 0;
	for (; s <= 6; s++) {
		const uint64_t width = 1ull << (32 - s);
		std::vector<std::vector<uint32_t>> sub(1u << s);
		bool fits = true;
		size_t i = 0;
		uint32_t below = flip; /* parity of the boundaries below S, flip included */
		for (uint32_t k = 0; k < (1u << s) && fits; k++) {
			const uint64_t S = k * width;
			auto &v = sub[k];
			if (k && (below & 1u))
				v.push_back((uint32_t)(S - 1));
			for (; i < bnd.size() && bnd[i] < S + width; i++, below ^= 1u)
				v.push_back(bnd[i] - 1u);
			fits = v.size() <= 32;
		}
		if (!fits)
			continue;
		for (auto &v : sub) {
			v.resize(32, 0xFFFFFFFFu);
			b.pool.insert(b.pool.end(), v.begin(), v.end());
		}
		break;
	}
	if (s > 6) {
		s = COVER6_LONG;
		b.pool.insert(b.pool.end(), {(uint32_t)bnd.size(), 0u, 0u, 0u});
		for (uint32_t x : bnd)
			b.pool.push_back(x - 1u);
		b.pool.resize((b.pool.size() + 31) / 32 * 32, 0xFFFFFFFFu);
	}
	b.too_big |= b.pool.size() / 32 > (1u << 25);
	return COVER6_NODE << 30 | (flip | (deep ? 2u : 0u) | s << 2) << 25 | (uint32_t)line;
}

uint32_t cover6_node64(Cover6Build &b, const std::vector<std::pair<uint64_t, uint64_t>> &iv)
{
	std::vector<uint64_t> bnd;
	for (auto &x : iv) {
		bnd.push_back(x.first);
		if (x.second != ~0ull)
			bnd.push_back(x.second + 1u);
	}
	const uint32_t off = (uint32_t)(b.pool.size() / 4);
	b.pool.insert(b.pool.end(), {(uint32_t)bnd.size(), 0u, 0u, 0u});
	for (uint64_t x : bnd) {
		b.pool.push_back((uint32_t)(x >> 32));
		b.pool.push_back((uint32_t)x);
	}
	while (b.pool.size() % 4)
		b.pool.push_back(0);
	return COVER6_NODE << 30 | off;
}

template <size_t W>
void hop_place(std::vector<std::array<uint32_t, W>> &tab, uint32_t &mask,
	       const std::vector<std::array<uint32_t, W>> &recs, uint32_t (*home_of)(const std::array<uint32_t, W> &))
{
	uint32_t nb = next_pow2(std::max<uint64_t>(64, 2 * recs.size()));
	for (;;) {
		tab.assign(nb, std::array<uint32_t, W>{});
		mask = nb - 1;
		bool ok = true;
		for (auto &r : recs) {
			const uint32_t home = home_of(r) & mask;
			uint32_t d = 0;
			while (d < POL_HOP && (tab[(home + d) & mask][3] & COVER6_USED))
				d++;
			if (d == POL_HOP) {
				ok = false;
				break;
			}
			auto &sl = tab[(home + d) & mask];
			const uint32_t hop = sl[3] & ~0xFFFFFFu;
			sl = r;
			sl[3] = hop | COVER6_USED;
			tab[home][3] |= 1u << (POL_HOP_SHIFT + d);
		}
		if (ok)
			return;
		nb *= 2;
	}
}

/* The /32 entry of the prefixes longer than /32 among ps[k, l) (one /32,
 * sorted; shorter ones are skipped): an interval node over bits 32..63
 * (/33../64) flagged deep when the /32 also has /64 records, or DEEP when only
 * /65+ prefixes exist; appends the /64 records to r64. */
uint32_t cover6_group32(Cover6Build &b, const std::vector<P6> &ps, size_t k, size_t l,
			std::vector<std::array<uint32_t, 8>> &r64)
{
	std::vector<std::pair<uint32_t, uint32_t>> s2;
	std::vector<uint32_t> pts; /* bits 32..63 of the /64s with an h64 record */
	for (size_t q = k; q < l; q++) {
		const P6 &p = ps[q];
		if (p.len <= 32)
			continue;
		if (p.len <= 64) {
			const uint32_t st = (uint32_t)p.hi;
			const uint32_t span = 64 - p.len;
			s2.push_back({st, span == 32 ? 0xFFFFFFFFu : st + ((1u << span) - 1u)});
		} else if (pts.empty() || pts.back() != (uint32_t)p.hi) {
			pts.push_back((uint32_t)p.hi);
		}
	}
	/* /64 groups */
	size_t m = k;
	while (m < l) {
		if (ps[m].len <= 64) {
			m++;
			continue;
		}
		const uint64_t top64 = ps[m].hi;
		std::vector<std::pair<uint64_t, uint64_t>> s3;
		size_t q = m;
		for (; q < l && ps[q].hi == top64; q++) {
			const P6 &p = ps[q];
			if (p.len > 64) {
				const uint32_t span = 128 - p.len;
				s3.push_back({p.lo, span == 64 ? ~0ull : p.lo + ((1ull << span) - 1ull)});
			}
		}
		auto iv = merge_iv(s3);
		std::array<uint32_t, 8> r{(uint32_t)(top64 >> 32), (uint32_t)top64, 0u, 0u, 0u, 0u, 0u, 0u};
		if (iv.size() == 1) {
			r[2] = COVER6_FULL << 30; /* inline [lo, hi] */
			r[4] = (uint32_t)(iv[0].first >> 32);
			r[5] = (uint32_t)iv[0].first;
			r[6] = (uint32_t)(iv[0].second >> 32);
			r[7] = (uint32_t)iv[0].second;
		} else {
			r[2] = cover6_node64(b, iv);
		}
		r64.push_back(r);
		m = q;
	}
	return s2.empty() ? COVER6_DEEP << 30 : cover6_node32(b, merge_iv(s2), !pts.empty());
}

/* Any-match cover of (len, address) prefixes, see tables.h cover6: /0../16
 * fill root entries, /17../24 fill entries of the /16's 256-entry b24 block,
 * /25../32 entries of the /24's b32 block (controlled prefix expansion: an
 * any-match set needs no priorities), longer prefixes become the node or
 * DEEP entry of their /32 unless a shorter prefix covers it whole. */
void build_cover6(const std::vector<Rank6> &cand, Cover6Build &b)
{
	b.any = !cand.empty();
	if (!b.any)
		return;
	std::vector<P6> ps;
	ps.reserve(cand.size());
	for (auto &c : cand) {
		uint64_t hi = 0, lo = 0;
		for (int i = 0; i < 8; i++) {
			hi = hi << 8 | c.addr[i];
			lo = lo << 8 | c.addr[8 + i];
		}
		ps.push_back(P6{hi, lo, c.len});
	}
	std::sort(ps.begin(), ps.end());
	/* line 0: all-ones, the line c6_node32_coop loads for a lane without
	 * a node line to read */
	b.pool.assign(32, 0xFFFFFFFFu);
	const uint32_t FULL = COVER6_FULL << 30, DEEP = COVER6_DEEP << 30;
	b.root.assign(65536, 0);
	b.b24.clear();
	b.b32.clear();
	for (auto &p : ps)
		if (p.len <= 16) {
			const uint32_t cnt = 1u << (16 - p.len);
			const uint32_t base = p.len == 0 ? 0 : ((uint32_t)(p.hi >> 48) & ~(cnt - 1));
			std::fill(b.root.begin() + base, b.root.begin() + base + cnt, FULL);
		}
	std::vector<std::array<uint32_t, 8>> r64;
	size_t i = 0;
	while (i < ps.size()) {
		const uint32_t top16 = (uint32_t)(ps[i].hi >> 48);
		size_t j = i;
		while (j < ps.size() && (uint32_t)(ps[j].hi >> 48) == top16)
			j++;
		bool below16 = false;
		for (size_t k = i; k < j; k++)
			below16 |= ps[k].len > 16;
		if (b.root[top16] == FULL || !below16) {
			i = j;
			continue;
		}
		/* the /16's b24 block: /17../24 prefixes */
		std::array<uint32_t, 256> e24{};
		for (size_t k = i; k < j; k++)
			if (ps[k].len > 16 && ps[k].len <= 24) {
				const uint32_t cnt = 1u << (24 - ps[k].len);
				const uint32_t base = (uint32_t)(ps[k].hi >> 40) & 0xFFu & ~(cnt - 1);
				std::fill(e24.begin() + base, e24.begin() + base + cnt, FULL);
			}
		/* /24 groups (contiguous in sorted order) */
		size_t k = i;
		while (k < j) {
			const uint32_t x24 = (uint32_t)(ps[k].hi >> 40) & 0xFFu;
			size_t l = k;
			while (l < j && ((uint32_t)(ps[l].hi >> 40) & 0xFFu) == x24)
				l++;
			bool below = false;
			for (size_t q = k; q < l; q++)
				below |= ps[q].len > 24;
			if (e24[x24] == FULL || !below) {
				k = l;
				continue;
			}
			std::array<uint32_t, 256> e32{};
			for (size_t q = k; q < l; q++)
				if (ps[q].len > 24 && ps[q].len <= 32) {
					const uint32_t cnt = 1u << (32 - ps[q].len);
					const uint32_t base = (uint32_t)(ps[q].hi >> 32) & 0xFFu & ~(cnt - 1);
					std::fill(e32.begin() + base, e32.begin() + base + cnt, FULL);
				}
			size_t q = k;
			while (q < l) {
				const uint32_t x32 = (uint32_t)(ps[q].hi >> 32) & 0xFFu;
				size_t r = q;
				while (r < l && ((uint32_t)(ps[r].hi >> 32) & 0xFFu) == x32)
					r++;
				bool below32 = false;
				for (size_t t = q; t < r; t++)
					below32 |= ps[t].len > 32;
				if (e32[x32] != FULL && below32)
					e32[x32] = cover6_group32(b, ps, q, r, r64);
				q = r;
			}
			e24[x24] = DEEP | (uint32_t)(b.b32.size() / 256);
			b.b32.insert(b.b32.end(), e32.begin(), e32.end());
			k = l;
		}
		b.root[top16] = DEEP | (uint32_t)(b.b24.size() / 256);
		b.b24.insert(b.b24.end(), e24.begin(), e24.end());
		i = j;
	}
	hop_place<8>(b.h64, b.m64, r64, h64_home);
	/* 8 zero units past the last node: the octet load of a node reads
	 * 128 B from its start whatever its length */
	b.pool.insert(b.pool.end(), 32, 0u);
	/* the LDS-staged forms (tables.h cover6) */
	auto u16e = [](uint32_t e) {
		return (uint16_t)((e >> 30) == COVER6_DEEP ? 2u + (e & 0x3FFFFFFFu)
							   : ((e >> 30) == COVER6_FULL ? 1u : 0u));
	};
	b.root16.clear();
	b.rbits.clear();
	b.b24_16.clear();
	if (b.b24.size() / 256 <= 0xFFFDu) {
		b.root16.resize(65536);
		for (uint32_t x = 0; x < 65536; x++)
			b.root16[x] = u16e(b.root[x]);
	}
	if (b.b32.size() / 256 <= 0xFFFDu && b.b24.size() / 256 <= 0xFFFFu) {
		b.rbits.assign(COVER6_RBITS_WORDS, 0u);
		uint32_t rank = 0;
		for (uint32_t w = 0; w < 2048; w++) {
			b.rbits[4096 + w / 2] |= rank << (16 * (w & 1));
			for (uint32_t k = 0; k < 32; k++) {
				const uint32_t e = b.root[32 * w + k];
				if ((e >> 30) == COVER6_DEEP) {
					b.rbits[w] |= 1u << k;
					rank++;
				} else if ((e >> 30) == COVER6_FULL) {
					b.rbits[2048 + w] |= 1u << k;
				}
			}
		}
		/* b24 blocks were appended in root order: block = rank */
		b.b24_16.resize(b.b24.size());
		for (size_t x = 0; x < b.b24.size(); x++)
			b.b24_16[x] = u16e(b.b24[x]);
	}
}

/* prefilter v6 any-match set (bpf_xdp.c:132-156): dyn6 (if
 * CIDR6_LPM_PREFILTER) + fix6 keys with prefixlen 128 (dyn keys canonical) */
std::vector<Rank6> pf6_candidates(const PfIn &in)
{
	std::vector<Rank6> cand;
	if (!in.fix6)
		return cand;
	if (in.dyn6)
		for (auto &k : in.dyn6k) {
			Rank6 r{k.prefixlen, k.prefixlen, {}, 1};
			memcpy(r.addr.data(), k.addr, 16);
			cand.push_back(r);
		}
	for (auto &k : in.fix6k) {
		if (k.prefixlen != 128)
			continue;
		Rank6 r{128, 128, {}, 1};
		memcpy(r.addr.data(), k.addr, 16);
		cand.push_back(r);
	}
	return cand;
}

/* ipcache -> v6 LPM for IPv6 lookups (ipcache_lookup6, eps.h:56-66): a
 * lookup key is {prefixlen 160, pad 0, family 2, ip6}; entries ending inside
 * the static part rank below /0, exactly as ipc4_candidate.  canon: the
 * mirror's masked key data. */
static const uint8_t kStaticV6[4] = {0, 0, 0, 2};
bool ipc6_candidate(const cgpu_ipcache_key &raw, const uint8_t *canon, uint32_t label, Rank6 *r)
{
	const uint32_t p = raw.prefixlen;
	if (!prefix_eq((const uint8_t *)&raw + 4, kStaticV6, std::min<uint32_t>(p, 32)))
		return false;
	*r = Rank6{p, 0, {}, label};
	if (p >= 32) {
		r->len = p - 32;
		memcpy(r->addr.data(), canon + 4, 16);
	}
	return true;
}

} // namespace

/* Test hook (not part of the drop-in boundary, no header): build the IPv6
 * ipcache trie of n ipcache keys / labels exactly as a commit does and look
 * up m addresses on the host.  out[j] = the matched sec_label, 0xFFFFFFFF
 * for no match; stats (8 words): /32 nodes, V6T_LONG nodes, h64 records, /64
 * lists, pool words, b24 blocks, b32 blocks, h64 slots. */
CGPU_EXPORT int cgpu_diag_ipc6_trie(const cgpu_ipcache_key *keys, const uint32_t *labels, size_t n,
				    const uint8_t *addrs, size_t m, uint32_t *out, uint32_t *stats)
{
	std::vector<Rank6> cand;
	for (size_t i = 0; i < n; i++) {
		uint8_t canon[20];
		memcpy(canon, (const uint8_t *)&keys[i] + 4, 20);
		const uint32_t p = std::min<uint32_t>(keys[i].prefixlen, 160);
		for (uint32_t bit = p; bit < 160; bit++)
			canon[bit / 8] &= (uint8_t) ~(0x80u >> (bit % 8));
		Rank6 r;
		if (ipc6_candidate(keys[i], canon, labels[i], &r))
			cand.push_back(r);
	}
	V6Build b;
	build_v6(cand, b);
	for (size_t j = 0; j < m; j++) {
		const uint32_t e = b.any ? v6t_host_lookup(b, addrs + 16 * j) : 0u;
		out[j] = !e ? 0xFFFFFFFFu
			    : ((e & DIR_TAG_MASK) == DIR_TAG_INDIRECT ? b.vals[e & DIR_PAYLOAD_MASK] : e & DIR_PAYLOAD_MASK);
	}
	if (stats) {
		uint32_t st[8] = {};
		for (size_t i = 0; i + 1 < b.b32.size(); i += 2)
			if ((b.b32[i] & DIR_TAG_MASK) == DIR_TAG_GROUP) {
				st[0]++;
				st[1] += ((b.b32[i + 1] >> 5) & 7u) == V6T_LONG;
			}
		for (auto &r : b.h64)
			if (r[3] & COVER6_USED) {
				st[2]++;
				st[3] += (r[2] & DIR_TAG_MASK) == DIR_TAG_GROUP;
			}
		st[4] = (uint32_t)b.pool.size();
		st[5] = (uint32_t)(b.b24.size() / 256);
		st[6] = (uint32_t)(b.b32.size() / 512);
		st[7] = (uint32_t)b.h64.size();
		memcpy(stats, st, sizeof(st));
	}
	return b.too_big ? -E2BIG : 0;
}

namespace {

/* Service map -> frontend hash + dense backend rows (tables.h lb_table).
 * Returns -E2BIG when sparse slave numbers would need more than
 * 4 * lb_max_entries + 65536 backend rows. */
struct LbBuild {
	std::vector<std::array<uint32_t, 4>> fe, be;
	std::vector<uint32_t> vip; /* tables.h lb_table.vip */
	uint32_t mask = 0, vip_mask = 0;
};

typedef std::vector<std::pair<uint64_t, cgpu_lb4_service>> LbIn; /* sorted by mkey */

int build_lb(const LbIn &lb, uint32_t lb_max_entries, LbBuild &b)
{
	std::vector<std::array<uint32_t, 4>> fes;
	const uint64_t cap = 4ull * lb_max_entries + 65536ull;
	for (auto it = lb.begin(); it != lb.end();) {
		const uint64_t fk = it->first >> 16;
		uint32_t mcount = 0, maxs = 0;
		const cgpu_lb4_service *master = nullptr;
		auto jt = it;
		for (; jt != lb.end() && (jt->first >> 16) == fk; ++jt) {
			const uint32_t s = (uint32_t)(jt->first & 0xFFFFu);
			if (s == 0) {
				mcount = jt->second.count;
				master = &jt->second;
			} else {
				maxs = s; /* ascending: the last is the largest */
			}
		}
		const uint64_t base = b.be.size();
		const uint32_t rows = maxs + (master ? 1u : 0u);
		if (base + rows > cap)
			return fail(-E2BIG, "lb4 backend rows exceed %llu (sparse slave numbers)",
				    (unsigned long long)cap);
		b.be.resize(base + rows, std::array<uint32_t, 4>{0, 0, 0, 0});
		auto row = [](const cgpu_lb4_service &v) {
			return std::array<uint32_t, 4>{v.target, (uint32_t)v.port | (uint32_t)v.count << 16,
						       (uint32_t)v.rev_nat_index | (uint32_t)v.weight << 16, 1u};
		};
		for (auto kt = it; kt != jt; ++kt) {
			const uint32_t s = (uint32_t)(kt->first & 0xFFFFu);
			if (s)
				b.be[base + s - 1] = row(kt->second);
		}
		if (master) /* LB_FE_MASTER: the slave-0 row after the slaves */
			b.be[base + maxs] = row(*master);
		fes.push_back({(uint32_t)(fk >> 16), (uint32_t)(fk & 0xFFFFu) | mcount << 16, (uint32_t)base,
			       maxs | (master ? LB_FE_MASTER : 0u)});
		it = jt;
	}
	/* frontend slots per frontend (power-of-two rounded); hopscotch insertion
	 * as the policy table's (PolBuild::insert): first-fit needed 16 slots per
	 * frontend for config 5's 1M frontends (a 256-MiB table, past the
	 * Infinity Cache) */
	uint32_t nb = next_pow2(std::max<uint64_t>(64, (uint64_t)CGPU_LB_SLOTS_PER_FE * fes.size()));
	for (;;) {
		b.fe.assign(nb, std::array<uint32_t, 4>{0, 0, 0, 0});
		b.mask = nb - 1;
		bool ok = true;
		auto used = [&](uint32_t i) { return (b.fe[i & b.mask][3] & LB_FE_USED) != 0u; };
		for (auto &f : fes) {
			const uint32_t home = lb_hash(f[0], f[1] & 0xFFFFu) & b.mask;
			uint32_t d = 0;
			const uint32_t limit = std::min<uint32_t>(b.mask + 1u, 4096u);
			while (d < limit && used(home + d))
				d++;
			while (ok && d < limit && d >= POL_HOP) {
				const uint32_t fr = (home + d) & b.mask;
				bool moved = false;
				for (uint32_t j = POL_HOP - 1; j >= 1 && !moved; j--) {
					const uint32_t h2 = (fr - j) & b.mask;
					const uint32_t hop2 = b.fe[h2][3] >> POL_HOP_SHIFT;
					for (uint32_t o = 0; o < j; o++) {
						if (!((hop2 >> o) & 1u))
							continue;
						auto &src = b.fe[(h2 + o) & b.mask], &dst = b.fe[fr];
						dst[0] = src[0];
						dst[1] = src[1];
						dst[2] = src[2];
						dst[3] = (dst[3] & 0xFF000000u) | (src[3] & 0xFFFFFFu);
						src[0] = src[1] = src[2] = 0;
						src[3] &= 0xFF000000u;
						b.fe[h2][3] = (b.fe[h2][3] & ~(1u << (POL_HOP_SHIFT + o))) | (1u << (POL_HOP_SHIFT + j));
						d -= j - o;
						moved = true;
						break;
					}
				}
				ok = moved;
			}
			if (!ok || d >= POL_HOP) {
				ok = false;
				break;
			}
			auto &sl = b.fe[(home + d) & b.mask];
			sl[0] = f[0];
			sl[1] = f[1];
			sl[2] = f[2];
			sl[3] = (sl[3] & ~0xFFFFFFu) | f[3] | LB_FE_USED;
			b.fe[home][3] |= 1u << (POL_HOP_SHIFT + d);
		}
		if (ok)
			break;
		nb *= 2;
	}
	if (b.be.empty())
		b.be.push_back({0, 0, 0, 0});
	/* 8 bits per frontend (config 5 at 4 / 8 / 16 / 32 / 64 bits per
	 * frontend: 22.6 / 22.5 / 22.3 / 22.0 / 21.7 Gpps, round 1) */
	const uint64_t bits = next_pow2(std::max<uint64_t>(1u << 15, 8ull * fes.size()));
	b.vip.assign(bits / 32, 0u);
	b.vip_mask = (uint32_t)(bits - 1);
	for (auto &f : fes) {
		const uint32_t k = lb_vip_bit(f[0]) & b.vip_mask;
		b.vip[k >> 5] |= 1u << (k & 31u);
	}
	return 0;
}

/* the lb6 mirror's key: address, dport (network order), then the slave
 * BIG-endian so a frontend's entries sort by slave number */
typedef std::array<uint8_t, 20> Lb6K;
typedef std::vector<std::pair<Lb6K, cgpu_lb6_service>> Lb6In; /* sorted by key */

static inline Lb6K lb6_mkey(const cgpu_lb6_key *k)
{
	Lb6K m;
	memcpy(m.data(), k, 18);
	m[18] = (uint8_t)(k->slave >> 8);
	m[19] = (uint8_t)k->slave;
	return m;
}

static inline cgpu_lb6_key lb6_unkey(const Lb6K &m)
{
	cgpu_lb6_key k;
	memcpy(&k, m.data(), 18);
	k.slave = (uint16_t)(m[18] << 8 | m[19]);
	return k;
}

struct Lb6Build {
	std::vector<std::array<uint32_t, 8>> fe, be;
	std::vector<uint32_t> vip;
	uint32_t mask = 0, vip_mask = 0;
};

/* cilium_lb6_services -> frontend hash + dense backend rows (tables.h
 * lb6_table): the build_lb scheme with 32-byte rows */
int build_lb6(const Lb6In &lb, uint32_t lb_max_entries, Lb6Build &b)
{
	struct Fe {
		uint32_t a[4], dport, mcount, base, nslaves;
	};
	std::vector<Fe> fes;
	const uint64_t cap = 4ull * lb_max_entries + 65536ull;
	for (auto it = lb.begin(); it != lb.end();) {
		auto jt = it;
		uint32_t mcount = 0, maxs = 0;
		const cgpu_lb6_service *master = nullptr;
		for (; jt != lb.end() && !memcmp(jt->first.data(), it->first.data(), 18); ++jt) {
			const uint32_t sl = (uint32_t)jt->first[18] << 8 | jt->first[19];
			if (sl == 0) {
				mcount = jt->second.count;
				master = &jt->second;
			} else {
				maxs = sl; /* ascending */
			}
		}
		const uint64_t base = b.be.size();
		const uint32_t rows = maxs + (master ? 1u : 0u);
		if (base + rows > cap)
			return fail(-E2BIG, "lb6 backend rows exceed %llu (sparse slave numbers)",
				    (unsigned long long)cap);
		b.be.resize(base + rows, std::array<uint32_t, 8>{});
		auto put = [&](uint64_t at, const cgpu_lb6_service &v) {
			auto &row = b.be[at];
			memcpy(row.data(), v.target, 16);
			row[4] = (uint32_t)v.port | (uint32_t)v.count << 16;
			row[5] = (uint32_t)v.rev_nat_index | (uint32_t)v.weight << 16;
			row[6] = 1u;
		};
		for (auto kt = it; kt != jt; ++kt) {
			const uint32_t sl = (uint32_t)kt->first[18] << 8 | kt->first[19];
			if (sl)
				put(base + sl - 1, kt->second);
		}
		if (master) /* LB_FE_MASTER: the slave-0 row after the slaves */
			put(base + maxs, *master);
		Fe f{};
		memcpy(f.a, it->first.data(), 16);
		uint16_t dp;
		memcpy(&dp, it->first.data() + 16, 2);
		f.dport = dp;
		f.mcount = mcount;
		f.base = (uint32_t)base;
		f.nslaves = maxs | (master ? LB_FE_MASTER : 0u);
		fes.push_back(f);
		it = jt;
	}
	uint32_t nb = next_pow2(std::max<uint64_t>(64, 2 * fes.size()));
	for (;;) {
		b.fe.assign(nb, std::array<uint32_t, 8>{});
		b.mask = nb - 1;
		bool ok = true;
		for (auto &f : fes) {
			const uint32_t home = lb6_hash(fold6(f.a[0], f.a[1], f.a[2], f.a[3]), f.dport) & b.mask;
			uint32_t d = 0;
			while (d < POL_HOP && (b.fe[(home + d) & b.mask][6] & LB_FE_USED))
				d++;
			if (d == POL_HOP) {
				ok = false;
				break;
			}
			auto &sl = b.fe[(home + d) & b.mask];
			memcpy(sl.data(), f.a, 16);
			sl[4] = f.dport | f.mcount << 16;
			sl[5] = f.base;
			sl[6] = (sl[6] & ~0xFFFFFFu) | f.nslaves | LB_FE_USED;
			b.fe[home][6] |= 1u << (POL_HOP_SHIFT + d);
		}
		if (ok)
			break;
		nb *= 2;
	}
	if (b.be.empty())
		b.be.push_back(std::array<uint32_t, 8>{});
	const uint64_t bits = next_pow2(std::max<uint64_t>(1u << 15, 8ull * fes.size()));
	b.vip.assign(bits / 32, 0u);
	b.vip_mask = (uint32_t)(bits - 1);
	for (auto &f : fes) {
		const uint32_t k = lb6_vip_bit(fold6(f.a[0], f.a[1], f.a[2], f.a[3])) & b.vip_mask;
		b.vip[k >> 5] |= 1u << (k & 31u);
	}
	return 0;
}

/* ---------------- device buffers, snapshots (epochs) ----------------
 * Every table group of a snapshot lives in one device buffer; a commit
 * uploads the groups that changed and shares the others with the previous
 * snapshot.  A buffer is freed stream-ordered on the context's retirement
 * stream (hipFreeAsync) once no snapshot references it, and only after that
 * stream has waited for the last launch of every snapshot that used it. */
enum { G_IPC = 0, G_POL, G_PF, G_EP, G_LB, G_LXC, G_LB6, G_N };

struct DevBuf {
	void *p = nullptr;
	size_t bytes = 0;
	int dev = -1;
	hipStream_t st = nullptr;
	uint64_t host_sum = 0; /* table_sum_word over the host image (verification) */
	size_t gather = 0;     /* bytes of the parts lookups gather from device memory
				  (not LDS-staged, not fallback-only); 0 = all (cgpu_table_bytes) */
	std::vector<std::pair<size_t, size_t>> parts; /* (offset, bytes) summed */
	~DevBuf()
	{
		if (p) {
			(void)hipSetDevice(dev);
			(void)hipFreeAsync(p, st); /* the context's retirement stream */
		}
	}
};
typedef std::shared_ptr<DevBuf> DevBufP;

struct Epoch;

/* host images kept between commits (guarded by cgpu_ctx::commit_mu) so that
 * small deltas patch them instead of recompiling everything */
struct BuildState {
	bool ipc4_ok = false;
	Dir248 dir;       /* ipcache v4 DIR-24-8 (host only) */
	Lpm16cBuild lc;   /* its compressed form (uploaded) */
	V6Build v6;
	bool pol_ok = false;
	PolBuild pol;
	PgBuild pg;
	uint64_t sum[G_N] = {};
};

/* One conntrack map (tables.h ct_table layout; CtK4 / CtK6 slots in
 * kernels.hip).  A host shadow serves the bpf(2)-style map calls; the device
 * copy is authoritative once a batch ran (dev_newer) and is refreshed from
 * the shadow before the next batch after host edits (host_newer). */
/* LRU mode's bloom filter of a batch's conntrack keys: 2^22 words (2^27 bits) */
#define CT_BLOOM_WORDS (1u << 22)

struct CtMap {
	bool v6 = false;
	uint32_t max = 0;               /* CT_MAP_SIZE */
	std::vector<uint4> keys, vals;  /* [sw() * nslots], [4 * nslots] */
	uint32_t mask = 0, live = 0, tombs = 0;
	bool dev_newer = false, host_newer = false;
	uint4 *d_keys = nullptr, *d_vals = nullptr;
	uint32_t *d_count = nullptr;
	/* the device compaction's second table (allocated at its first use) and
	 * the device GC's result word */
	uint4 *d_keys2 = nullptr, *d_vals2 = nullptr;
	uint32_t *d_gc = nullptr;
	uint32_t *d_bloom = nullptr; /* LRU mode: the batch's key filter */
	uint64_t compactions = 0;
	uint32_t sw() const { return v6 ? 4u : 1u; } /* uint4 key words per slot */
};

} // namespace

struct cgpu_ctx {
	cgpu_config cfg;
	int device = -1;
	/* lock order: commit_mu -> mu -> retire_mu; pub_mu and pk_mu are leaves */
	std::mutex mu;        /* host mirror */
	std::mutex commit_mu; /* one commit at a time; BuildState */
	std::mutex pub_mu;    /* the published snapshot */
	std::mutex pk_mu;     /* per-stream packed counter buffers */
	std::mutex retire_mu;

	/* ---- host mirror ---- */
	std::map<LpmKey<20>, IpcEntry> ipc;
	std::vector<std::map<uint64_t, PolEntry>> pol;
	size_t pol_total = 0;
	/* counter slots: hot class [0, hot_cap) for L3-only / wildcard keys,
	 * cold class [hot_cap, n_ctr_slots) for the rest.  A slot whose key a
	 * published snapshot holds is quarantined on delete until every
	 * snapshot up to that one has finished its launches. */
	std::vector<uint32_t> free_hot, free_cold;
	std::deque<std::pair<uint64_t, uint32_t>> quarantine; /* (snapshot id, slot) */
	uint32_t next_hot = 0, next_cold = 0, hot_cap = 0;
	std::vector<SlotInit> slot_inits;
	std::map<LpmKey<4>, cgpu_cidr_key> dyn4;
	std::map<LpmKey<16>, cgpu_cidr_key> dyn6;
	std::set<std::array<uint8_t, 8>> fix4;
	std::set<std::array<uint8_t, 20>> fix6;
	std::set<std::array<uint8_t, 20>> lxc;
	/* cilium_lb4_services, keyed address << 32 | dport << 16 | slave so that
	 * a frontend's entries are adjacent */
	std::map<uint64_t, cgpu_lb4_service> lb;
	std::map<Lb6K, cgpu_lb6_service> lb6;
	/* per-endpoint lxc_config.h identity (cgpu_lxc_update) */
	std::map<uint32_t, cgpu_lxc_info> lxcinfo;
	int64_t pf_revision = 1; /* PreFilter revision (pkg/policy/prefilter.go:283) */
	/* ---- change tracking since the last captured commit ---- */
	uint32_t dirty = 0;             /* 1 << G_* */
	bool ipc_full = true, pol_full = true;
	std::vector<LpmKey<20>> ipc_changes;
	std::vector<std::pair<uint32_t, uint64_t>> pol_changes; /* (ep, key) */
	uint64_t captured = 0;          /* id of the newest snapshot whose inputs were captured */
	uint64_t sum_ipc = 0, sum_pol = 0; /* order-independent content sums */
	uint64_t sum_slots = 0;            /* (ep, key, counter slot) of every policy key */

	/* ---- device ---- */
	hipStream_t ustream = nullptr;  /* uploads + counter slot init of commits */
	hipStream_t rstream = nullptr;  /* retirement: waits on launches, then frees */
	hipMemPool_t pool = nullptr;    /* snapshot buffers (stream-ordered) */
	BuildState b;
	std::shared_ptr<Epoch> cur;     /* published snapshot (pub_mu) */
	uint64_t epoch = 0;             /* id of the published snapshot */
	uint64_t checksum = 0;
	uint64_t slot_checksum = 0;     /* sum_slots of the published snapshot */
	/* snapshots unpublished but maybe still running: (id, done event on
	 * rstream); alive = ids not known complete (incl. the published one) */
	std::deque<std::pair<uint64_t, hipEvent_t>> retiring;
	std::set<uint64_t> alive;
	uint32_t n_ctr_slots = 0;
	uint64_t *d_totals = nullptr; /* [2*slots + METRICS] */
	uint64_t *d_delta_own = nullptr;
	uint64_t *d_delta = nullptr;  /* own or bound */
	uint64_t *d_verify = nullptr; /* [G_N + 1] device-side table sums of a commit / verify */
	/* [n_ctr_slots] packed counter accumulator per stream (zero between
	 * classify calls; one per stream keeps its exactness bound per call).
	 * At most kMaxPkStreams buffers: a new stream past that takes the least
	 * recently used one once that stream's last launch finished (`last`). */
	struct PkBuf {
		uint64_t *p = nullptr;
		hipEvent_t last = nullptr;
		uint64_t tick = 0;
	};
	std::map<void *, PkBuf> d_pk;
	uint64_t pk_tick = 0;

	/* ---- multi-GPU counter reduction (cgpu_comm_init) ---- */
	void *comm = nullptr; /* ncclComm_t */

	/* ---- conntrack maps cilium_ct4_global / cilium_ct6_global ---- */
	CtMap ct4, ct6;
	void *d_ct_scratch = nullptr;
	uint64_t *d_ct_pk = nullptr; /* the conntrack finish's packed counters (k_unpack re-zeroes) */
	/* host-resident batches (cgpu_classify_v4_host / _frames_host): device
	 * staging for up to HS_NBUF chunks (grown to the largest batch seen,
	 * freed by cgpu_host_stage_release), one stream per direction */
	std::mutex host_mu;
	struct {
		int nb = 0;
		void *d_in[16] = {}, *d_out[16] = {};
		hipStream_t h2d = nullptr, d2h = nullptr;
		hipEvent_t ev_in[16] = {}, ev_cls[16] = {}, ev_out[16] = {};
	} hs;
	size_t ct_scratch_cap = 0;
	hipStream_t ct_stream = nullptr; /* the conntrack path's internal stream */
	hipEvent_t ct_done = nullptr;
};

namespace {

/* One published snapshot.  Launches pin it (shared_ptr) while they enqueue,
 * wait on `ready` (its uploads) and record a per-stream event after their
 * kernels; when the last reference drops, the retirement stream waits on
 * those events before the buffers it alone held are freed, and `done` marks
 * when every launch of this snapshot has finished. */
struct Epoch {
	cgpu_ctx *c = nullptr;
	uint64_t id = 0;
	cgpu_snapshot snap{};
	DevBufP bufs[G_N];
	hipEvent_t ready = nullptr;
	std::mutex mu;
	std::vector<std::pair<hipStream_t, hipEvent_t>> used;
	~Epoch()
	{
		(void)hipSetDevice(c->device);
		for (auto &u : used) {
			(void)hipStreamWaitEvent(c->rstream, u.second, 0);
			(void)hipEventDestroy(u.second);
		}
		hipEvent_t done = nullptr;
		if (hipEventCreateWithFlags(&done, hipEventDisableTiming) == hipSuccess &&
		    hipEventRecord(done, c->rstream) == hipSuccess) {
			std::lock_guard<std::mutex> g(c->retire_mu);
			c->retiring.push_back({id, done});
		} else {
			(void)hipStreamSynchronize(c->rstream);
			if (done)
				(void)hipEventDestroy(done);
			std::lock_guard<std::mutex> g(c->retire_mu);
			c->alive.erase(id);
		}
		if (ready)
			(void)hipEventDestroy(ready);
		/* bufs release after this body: their hipFreeAsync follows the waits */
	}
};

/* snapshots whose launches finished leave `alive` (caller holds retire_mu) */
void poll_retired(cgpu_ctx *c)
{
	while (!c->retiring.empty()) {
		auto &f = c->retiring.front();
		if (hipEventQuery(f.second) != hipSuccess)
			break;
		(void)hipEventDestroy(f.second);
		c->alive.erase(f.first);
		c->retiring.pop_front();
	}
}

/* The oldest quarantined counter slot, once every snapshot that may count
 * into it has finished its launches (caller holds mu).  Slot assignment must
 * depend only on the sequence of map operations and commits, never on how far
 * the GPU got: replicas on other ranks apply the same sequence and their
 * delta buffers are summed slot by slot (cgpu_counters_allreduce).  So the
 * quarantine is used only after the free lists and the never-used slots, in
 * deletion order, and is WAITED for (not polled) when its snapshot is still
 * running.  A slot that the newest captured snapshot may still count into
 * cannot be reused before the next commit: -E2BIG, as a full map. */
int take_quarantined(cgpu_ctx *c, uint32_t *slot)
{
	if (c->quarantine.empty() || c->quarantine.front().first >= c->captured)
		return -E2BIG;
	const uint64_t need = c->quarantine.front().first;
	for (;;) {
		std::unique_lock<std::mutex> g(c->retire_mu);
		poll_retired(c);
		const uint64_t lowest = c->alive.empty() ? UINT64_MAX : *c->alive.begin();
		if (lowest > need)
			break;
		hipEvent_t ev = nullptr;
		for (auto &r : c->retiring)
			if (r.first == lowest)
				ev = r.second;
		if (ev) {
			if (hipEventSynchronize(ev) != hipSuccess)
				return -EIO;
		} else {
			/* still published (a commit in another thread is replacing it)
			 * or being retired right now */
			g.unlock();
			std::this_thread::yield();
		}
	}
	*slot = c->quarantine.front().second;
	c->quarantine.pop_front();
	return 0;
}

} // namespace

/* ======================================================================= */
/* config / context                                                          */
/* ======================================================================= */
CGPU_EXPORT void cgpu_config_default(cgpu_config *c)
{
	memset(c, 0, sizeof(*c));
	c->abi_version = CGPU_ABI_VERSION;
	c->ipcache_max = 512000;      /* pkg/maps/ipcache/ipcache.go:36 */
	c->policy_max_per_ep = 16384; /* pkg/maps/policymap/policymap.go:37 */
	c->policy_max_total = 1u << 20;
	c->max_endpoints = 65536;     /* ENDPOINTS_MAP_SIZE */
	c->cidr_dyn_max = 1u << 20;   /* > maxLKeys: device capacity, configurable */
	c->cidr_fix_max = 20u << 20;  /* maxHKeys (pkg/policy/prefilter.go:44) */
	c->endpoints_max = 65536;
	c->host_id = 1;
	c->world_id = 2;
	c->cluster_id = 3;
	c->health_id = 4;
	c->ipv4_cluster_mask = 0xff0000;  /* bpf/node_config.h:42 */
	c->ipv4_cluster_range = 0x100000; /* bpf/node_config.h:43 */
	c->ct_proto_gate = 1;             /* CONNTRACK (bpf/lxc_config.h:46) */
	c->ingress_secctx_world = 0;
	c->prefilter_fix4 = c->prefilter_dyn4 = 1; /* bpf/filter_config.h */
	c->prefilter_fix6 = c->prefilter_dyn6 = 1;
	c->ingress_src_identity = 0;
	/* as many as a kernel's LDS holds (each launcher caps it): with the
	 * popularity rebalance, config 2 1.692 / 1.657 / 1.645 ms at 12288 /
	 * 16384 / 17920 (the x4 kernel's cap), v6 2.805 / 2.759 / 2.725 at
	 * 12288 / 16384 / 24576 (profiles/r4_z/) */
	c->hot_counter_slots = 24576;
	c->lb_max_entries = 65536;        /* CILIUM_LB_MAP_MAX_ENTRIES, bpf/node_config.h:60 */
	c->ipv4_loopback = 0x1ffff50a;    /* IPV4_LOOPBACK, bpf/node_config.h:45 */
	c->lb_flags = CGPU_LB_L3 | CGPU_LB_L4; /* bpf/lxc_config.h:44-45 */
	static const uint8_t router[16] = {0xbe, 0xef, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0x1,
					   0x0, 0x1, 0x0, 0x0}; /* ROUTER_IP, bpf/node_config.h:30 */
	memcpy(c->ipv6_router_ip, router, 16);
	static const uint8_t node_mac[6] = {0xde, 0xad, 0xbe, 0xef, 0xc0, 0xde}; /* NODE_MAC, node_config.h:51 */
	memcpy(c->node_mac, node_mac, 6);
	c->ct_max = 1000000; /* CT_MAP_SIZE = MapNumEntriesGlobal, pkg/maps/ctmap/ctmap.go:101 */
}

CGPU_EXPORT const char *cgpu_last_error(void) { return g_last_error.c_str(); }
CGPU_EXPORT const char *cgpu_version(void) { return "cgpu 0.1 gfx950 abi1"; }

CGPU_EXPORT int cgpu_ctx_create(const cgpu_config *cfg, int device, cgpu_ctx **out)
{
	if (!cfg || !out)
		return fail(-EINVAL, "null argument");
	if (cfg->abi_version != CGPU_ABI_VERSION)
		return fail(-EINVAL, "abi_version %u != %u", cfg->abi_version, CGPU_ABI_VERSION);
	if (!cfg->max_endpoints || !cfg->policy_max_total)
		return fail(-EINVAL, "zero capacity");
	if (cfg->policy_max_total >= POL_CTR_EMPTY)
		return fail(-EINVAL, "policy_max_total %u >= 2^24 - 1", cfg->policy_max_total);
	if (!cfg->ct_max || cfg->ct_max > (1u << 28))
		return fail(-EINVAL, "ct_max %u out of range (1 .. 2^28)", cfg->ct_max);
	if (cfg->ct6_max > (1u << 27))
		return fail(-EINVAL, "ct6_max %u out of range (0 .. 2^27)", cfg->ct6_max);
	cgpu_ctx *c = new cgpu_ctx();
	c->cfg = *cfg;
	c->pol.resize(cfg->max_endpoints);
	c->n_ctr_slots = cfg->policy_max_total;
	c->hot_cap = std::min(cfg->hot_counter_slots, cfg->policy_max_total / 2);
	c->next_cold = c->hot_cap;
	c->dirty = (1u << G_N) - 1u; /* the first commit compiles every group */
	c->ct4.max = cfg->ct_max;
	c->ct6.v6 = true;
	c->ct6.max = cfg->ct6_max ? cfg->ct6_max : cfg->ct_max;
	if (device >= 0) {
		int ndev = 0, pools = 0;
		if (hipGetDeviceCount(&ndev) != hipSuccess || device >= ndev) {
			delete c;
			return fail(-ENODEV, "HIP device %d not present", device);
		}
		c->device = device;
		size_t words = (size_t)2 * c->n_ctr_slots + CGPU_METRICS_WORDS;
		if (hipSetDevice(device) != hipSuccess ||
		    hipDeviceGetAttribute(&pools, hipDeviceAttributeMemoryPoolsSupported, device) != hipSuccess ||
		    !pools) {
			delete c;
			return fail(-EIO, "device %d: no stream-ordered memory pools", device);
		}
		hipMemPoolProps pp{};
		pp.allocType = hipMemAllocationTypePinned;
		pp.location.type = hipMemLocationTypeDevice;
		pp.location.id = device;
		uint64_t keep = UINT64_MAX;
		int no = 0;
		if (hipStreamCreateWithFlags(&c->ustream, hipStreamNonBlocking) != hipSuccess ||
		    hipStreamCreateWithFlags(&c->rstream, hipStreamNonBlocking) != hipSuccess ||
		    hipMemPoolCreate(&c->pool, &pp) != hipSuccess ||
		    hipMemPoolSetAttribute(c->pool, hipMemPoolAttrReleaseThreshold, &keep) != hipSuccess ||
		    /* an upload never waits behind the retirement stream's waits */
		    hipMemPoolSetAttribute(c->pool, hipMemPoolReuseAllowInternalDependencies, &no) != hipSuccess ||
		    hipStreamCreateWithFlags(&c->ct_stream, hipStreamNonBlocking) != hipSuccess ||
		    hipEventCreateWithFlags(&c->ct_done, hipEventDisableTiming) != hipSuccess ||
		    hipMalloc((void **)&c->d_totals, words * 8) != hipSuccess ||
		    hipMalloc((void **)&c->d_delta_own, words * 8) != hipSuccess ||
		    hipMalloc((void **)&c->d_verify, (G_N + 1) * 8) != hipSuccess ||
		    hipMemset(c->d_totals, 0, words * 8) != hipSuccess ||
		    hipMemset(c->d_delta_own, 0, words * 8) != hipSuccess) {
			(void)hipFree(c->d_totals);
			(void)hipFree(c->d_delta_own);
			(void)hipFree(c->d_verify);
			if (c->ustream)
				(void)hipStreamDestroy(c->ustream);
			if (c->rstream)
				(void)hipStreamDestroy(c->rstream);
			if (c->pool)
				(void)hipMemPoolDestroy(c->pool);
			if (c->ct_stream)
				(void)hipStreamDestroy(c->ct_stream);
			if (c->ct_done)
				(void)hipEventDestroy(c->ct_done);
			delete c;
			return fail(-EIO, "device context allocation failed");
		}
		c->d_delta = c->d_delta_own;
	}
	*out = c;
	return 0;
}

static void comm_destroy(cgpu_ctx *c);

/* the host-batch staging (cgpu_classify_v4_host / _frames_host): waits for
 * every upload, classify and store queued on it, then frees it (the next host
 * call allocates again) */
static void host_stage_free(cgpu_ctx *c)
{
	auto &H = c->hs;
	if (H.h2d)
		(void)hipStreamSynchronize(H.h2d);
	if (H.d2h)
		(void)hipStreamSynchronize(H.d2h);
	for (int b = 0; b < H.nb; b++) {
		(void)hipEventSynchronize(H.ev_cls[b]);
		(void)hipFree(H.d_in[b]);
		(void)hipFree(H.d_out[b]);
		(void)hipEventDestroy(H.ev_in[b]);
		(void)hipEventDestroy(H.ev_cls[b]);
		(void)hipEventDestroy(H.ev_out[b]);
		H.d_in[b] = H.d_out[b] = nullptr;
		H.ev_in[b] = H.ev_cls[b] = H.ev_out[b] = nullptr;
	}
	H.nb = 0;
	if (H.h2d)
		(void)hipStreamDestroy(H.h2d);
	if (H.d2h)
		(void)hipStreamDestroy(H.d2h);
	H.h2d = H.d2h = nullptr;
}

CGPU_EXPORT void cgpu_ctx_destroy(cgpu_ctx *c)
{
	if (!c)
		return;
	if (c->device >= 0) {
		(void)hipSetDevice(c->device);
		(void)hipDeviceSynchronize();
		std::shared_ptr<Epoch> last;
		{
			std::lock_guard<std::mutex> g(c->pub_mu);
			last.swap(c->cur);
		}
		last.reset(); /* waits + frees enqueued on rstream */
		(void)hipStreamSynchronize(c->ustream);
		(void)hipStreamSynchronize(c->rstream);
		{
			std::lock_guard<std::mutex> g(c->retire_mu);
			for (auto &r : c->retiring)
				(void)hipEventDestroy(r.second);
			c->retiring.clear();
		}
		comm_destroy(c);
		(void)hipFree(c->d_totals);
		(void)hipFree(c->d_delta_own);
		(void)hipFree(c->d_verify);
		{
			std::lock_guard<std::mutex> g(c->pk_mu);
			for (auto &kv : c->d_pk) {
				(void)hipFree(kv.second.p);
				if (kv.second.last)
					(void)hipEventDestroy(kv.second.last);
			}
			c->d_pk.clear();
		}
		for (CtMap *m : {&c->ct4, &c->ct6}) {
			(void)hipFree(m->d_keys);
			(void)hipFree(m->d_vals);
			(void)hipFree(m->d_count);
			(void)hipFree(m->d_keys2);
			(void)hipFree(m->d_vals2);
			(void)hipFree(m->d_gc);
			(void)hipFree(m->d_bloom);
		}
		(void)hipFree(c->d_ct_scratch);
		(void)hipFree(c->d_ct_pk);
		host_stage_free(c);
		(void)hipEventDestroy(c->ct_done);
		(void)hipStreamDestroy(c->ct_stream);
		(void)hipStreamDestroy(c->ustream);
		(void)hipStreamDestroy(c->rstream);
		(void)hipMemPoolDestroy(c->pool);
	}
	delete c;
}

static int check_flags(uint64_t flags)
{
	return flags > CGPU_EXIST ? fail(-EINVAL, "bad update flags %llu", (unsigned long long)flags) : 0;
}

/* ======================================================================= */
/* change tracking (caller holds mu)                                         */
/* ======================================================================= */
/* more changes than this between commits: recompile the group instead */
static const size_t kMaxPatch = 4096;

static uint64_t ipc_hash(const LpmKey<20> &k, const cgpu_remote_endpoint_info &v)
{
	return fnv(fnv(1469598103934665603ull, &k, sizeof(k)), &v, 8);
}

/* over the map contents only (not the counter slot a key happened to get),
 * so replicas holding the same maps agree whatever their update history */
static uint64_t pol_hash_sum(uint32_t ep, uint64_t key, const PolEntry &e)
{
	const uint64_t h = fnv(1469598103934665603ull ^ ep, &key, 8);
	return fnv(h, &e.proxy_port, 2);
}

/* the counter slot a key holds (cgpu_counter_layout_checksum) */
static uint64_t slot_hash(uint32_t ep, uint64_t key, uint32_t slot)
{
	return fnv(fnv(0x51075107ull ^ ep, &key, 8), &slot, 4);
}

static void ipc_touch(cgpu_ctx *c, const LpmKey<20> &k)
{
	c->dirty |= 1u << G_IPC;
	if (c->ipc_full)
		return;
	if (c->ipc_changes.size() >= kMaxPatch) {
		c->ipc_full = true;
		c->ipc_changes.clear();
	} else {
		c->ipc_changes.push_back(k);
	}
}

static void pol_touch(cgpu_ctx *c, uint32_t ep, uint64_t key)
{
	c->dirty |= 1u << G_POL;
	if (c->pol_full)
		return;
	if (c->pol_changes.size() >= kMaxPatch) {
		c->pol_full = true;
		c->pol_changes.clear();
	} else {
		c->pol_changes.push_back({ep, key});
	}
}

/* ======================================================================= */
/* ipcache                                                                   */
/* ======================================================================= */
CGPU_EXPORT int cgpu_ipcache_update(cgpu_ctx *c, const cgpu_ipcache_key *key,
				    const cgpu_remote_endpoint_info *val, uint64_t flags)
{
	if (!c || !key || !val)
		return fail(-EINVAL, "null argument");
	if (int r = check_flags(flags))
		return r;
	if (key->prefixlen > 160) /* data is 20 bytes: lpm_trie max_prefixlen */
		return fail(-EINVAL, "ipcache prefixlen %u > 160", key->prefixlen);
	std::lock_guard<std::mutex> g(c->mu);
	auto k = lpm_canon<20>(key->prefixlen, (const uint8_t *)key + 4);
	auto it = c->ipc.find(k);
	if (it == c->ipc.end()) {
		if (flags == CGPU_EXIST)
			return fail(-ENOENT, "ipcache key not present");
		if (c->ipc.size() >= c->cfg.ipcache_max)
			return fail(-ENOSPC, "ipcache full (%u)", c->cfg.ipcache_max);
		c->ipc.emplace(k, IpcEntry{*key, *val});
	} else {
		if (flags == CGPU_NOEXIST)
			return fail(-EEXIST, "ipcache key exists");
		c->sum_ipc -= ipc_hash(k, it->second.val);
		it->second = IpcEntry{*key, *val};
	}
	c->sum_ipc += ipc_hash(k, *val);
	ipc_touch(c, k);
	return 0;
}

CGPU_EXPORT int cgpu_ipcache_delete(cgpu_ctx *c, const cgpu_ipcache_key *key)
{
	if (!c || !key)
		return fail(-EINVAL, "null argument");
	if (key->prefixlen > 160)
		return fail(-EINVAL, "ipcache prefixlen %u > 160", key->prefixlen);
	std::lock_guard<std::mutex> g(c->mu);
	const auto k = lpm_canon<20>(key->prefixlen, (const uint8_t *)key + 4);
	auto it = c->ipc.find(k);
	if (it == c->ipc.end())
		return fail(-ENOENT, "ipcache key not present");
	c->sum_ipc -= ipc_hash(k, it->second.val);
	c->ipc.erase(it);
	ipc_touch(c, k);
	return 0;
}

/* bpf(2) lookup on an LPM trie = longest prefix match of the given key */
CGPU_EXPORT int cgpu_ipcache_lookup(cgpu_ctx *c, const cgpu_ipcache_key *key,
				    cgpu_remote_endpoint_info *out)
{
	if (!c || !key || !out)
		return fail(-EINVAL, "null argument");
	std::lock_guard<std::mutex> g(c->mu);
	const uint8_t *q = (const uint8_t *)key + 4;
	uint32_t qlen = std::min<uint32_t>(key->prefixlen, 160);
	/* probe each shorter-or-equal prefix length, longest first */
	for (int64_t p = qlen; p >= 0; p--) {
		auto it = c->ipc.find(lpm_canon<20>((uint32_t)p, q));
		if (it != c->ipc.end()) {
			*out = it->second.val;
			return 0;
		}
	}
	return -ENOENT;
}

CGPU_EXPORT int cgpu_ipcache_get_next_key(cgpu_ctx *c, const cgpu_ipcache_key *key,
					  cgpu_ipcache_key *next)
{
	if (!c || !next)
		return fail(-EINVAL, "null argument");
	std::lock_guard<std::mutex> g(c->mu);
	auto it = c->ipc.begin();
	if (key) {
		auto k = lpm_canon<20>(std::min<uint32_t>(key->prefixlen, 160), (const uint8_t *)key + 4);
		it = c->ipc.upper_bound(k);
	}
	if (it == c->ipc.end())
		return -ENOENT;
	*next = it->second.raw;
	return 0;
}

CGPU_EXPORT size_t cgpu_ipcache_count(cgpu_ctx *c)
{
	std::lock_guard<std::mutex> g(c->mu);
	return c->ipc.size();
}

/* ======================================================================= */
/* policy                                                                    */
/* ======================================================================= */
static inline uint64_t pol_key64(const cgpu_policy_key *k)
{
	uint64_t x;
	memcpy(&x, k, 8);
	return x;
}

/* BPF_MAP_UPDATE_ELEM on an endpoint's policy map; caller holds c->mu and
 * has checked the flags and the endpoint index */
static int pol_update_locked(cgpu_ctx *c, uint32_t ep, const cgpu_policy_key *key,
			     const cgpu_policy_entry *e, uint64_t flags)
{
	auto &m = c->pol[ep];
	uint64_t k = pol_key64(key);
	auto it = m.find(k);
	uint32_t slot;
	if (it == m.end()) {
		if (flags == CGPU_EXIST)
			return fail(-ENOENT, "policy key not present");
		if (m.size() >= c->cfg.policy_max_per_ep)
			return fail(-E2BIG, "policy map of ep %u full (%u)", ep, c->cfg.policy_max_per_ep);
		/* L3-only {id, 0, 0, dir} and wildcard {0, port, proto, dir} keys
		 * absorb most hits: give them hot (LDS-accumulated) slots */
		bool hot = (key->dport == 0 && key->protocol == 0) || key->sec_label == 0;
		if (hot && !c->free_hot.empty()) {
			slot = c->free_hot.back();
			c->free_hot.pop_back();
		} else if (hot && c->next_hot < c->hot_cap) {
			slot = c->next_hot++;
		} else if (!c->free_cold.empty()) {
			slot = c->free_cold.back();
			c->free_cold.pop_back();
		} else if (c->next_cold < c->n_ctr_slots) {
			slot = c->next_cold++;
		} else if (int r = take_quarantined(c, &slot)) {
			return r == -EIO ? fail(-EIO, "waiting for a retired snapshot failed")
					 : fail(-E2BIG, "policy device slots exhausted (%u)", c->n_ctr_slots);
		}
		auto ins = m.emplace(k, PolEntry{e->proxy_port, slot, c->captured + 1}).first;
		c->pol_total++;
		c->sum_pol += pol_hash_sum(ep, k, ins->second);
		c->sum_slots += slot_hash(ep, k, slot);
	} else {
		if (flags == CGPU_NOEXIST)
			return fail(-EEXIST, "policy key exists");
		c->sum_pol -= pol_hash_sum(ep, k, it->second);
		it->second.proxy_port = e->proxy_port;
		slot = it->second.slot;
		c->sum_pol += pol_hash_sum(ep, k, it->second);
	}
	pol_touch(c, ep, k);
	/* kernel htab replaces the whole value: counters restart from it */
	c->slot_inits.push_back(SlotInit{slot, e->packets, e->bytes});
	return 0;
}

CGPU_EXPORT int cgpu_policy_update(cgpu_ctx *c, uint32_t ep, const cgpu_policy_key *key,
				   const cgpu_policy_entry *e, uint64_t flags)
{
	if (!c || !key || !e)
		return fail(-EINVAL, "null argument");
	if (int r = check_flags(flags))
		return r;
	if (ep >= c->cfg.max_endpoints)
		return fail(-EINVAL, "endpoint %u >= max_endpoints %u", ep, c->cfg.max_endpoints);
	std::lock_guard<std::mutex> g(c->mu);
	return pol_update_locked(c, ep, key, e, flags);
}

static void pol_erase(cgpu_ctx *c, uint32_t ep, std::map<uint64_t, PolEntry> &m,
		      std::map<uint64_t, PolEntry>::iterator it)
{
	const uint32_t slot = it->second.slot;
	if (it->second.first_epoch <= c->captured) /* a snapshot may count into it */
		c->quarantine.push_back({c->captured, slot});
	else
		(slot < c->hot_cap ? c->free_hot : c->free_cold).push_back(slot);
	c->sum_pol -= pol_hash_sum(ep, it->first, it->second);
	c->sum_slots -= slot_hash(ep, it->first, slot);
	pol_touch(c, ep, it->first);
	m.erase(it);
	c->pol_total--;
}

CGPU_EXPORT int cgpu_policy_delete(cgpu_ctx *c, uint32_t ep, const cgpu_policy_key *key)
{
	if (!c || !key)
		return fail(-EINVAL, "null argument");
	if (ep >= c->cfg.max_endpoints)
		return fail(-EINVAL, "endpoint %u out of range", ep);
	std::lock_guard<std::mutex> g(c->mu);
	auto &m = c->pol[ep];
	auto it = m.find(pol_key64(key));
	if (it == m.end())
		return fail(-ENOENT, "policy key not present");
	pol_erase(c, ep, m, it);
	return 0;
}

CGPU_EXPORT int cgpu_policy_flush(cgpu_ctx *c, uint32_t ep)
{
	if (!c || ep >= c->cfg.max_endpoints)
		return fail(-EINVAL, "bad argument");
	std::lock_guard<std::mutex> g(c->mu);
	auto &m = c->pol[ep];
	while (!m.empty())
		pol_erase(c, ep, m, m.begin());
	return 0;
}

static int read_counter_words(cgpu_ctx *c, size_t word, size_t nwords, uint64_t *out)
{
	/* totals + delta; pending launches complete first */
	std::vector<uint64_t> a(nwords), b(nwords);
	uint64_t *delta;
	{
		std::lock_guard<std::mutex> g(c->pk_mu);
		delta = c->d_delta;
	}
	HIP_OR_EIO(hipSetDevice(c->device));
	HIP_OR_EIO(hipDeviceSynchronize());
	HIP_OR_EIO(hipMemcpy(a.data(), c->d_totals + word, nwords * 8, hipMemcpyDeviceToHost));
	HIP_OR_EIO(hipMemcpy(b.data(), delta + word, nwords * 8, hipMemcpyDeviceToHost));
	for (size_t i = 0; i < nwords; i++)
		out[i] = a[i] + b[i];
	return 0;
}

CGPU_EXPORT int cgpu_policy_lookup(cgpu_ctx *c, uint32_t ep, const cgpu_policy_key *key,
				   cgpu_policy_entry *out)
{
	if (!c || !key || !out)
		return fail(-EINVAL, "null argument");
	if (ep >= c->cfg.max_endpoints)
		return fail(-EINVAL, "endpoint %u out of range", ep);
	std::lock_guard<std::mutex> g(c->mu);
	auto &m = c->pol[ep];
	auto it = m.find(pol_key64(key));
	if (it == m.end())
		return -ENOENT;
	memset(out, 0, sizeof(*out));
	out->proxy_port = it->second.proxy_port;
	/* the most recent update's counter values until the next commit */
	uint64_t pk = 0, by = 0;
	bool pending = false;
	for (auto s = c->slot_inits.rbegin(); s != c->slot_inits.rend(); ++s)
		if (s->slot == it->second.slot) {
			pk = s->packets;
			by = s->bytes;
			pending = true;
			break;
		}
	if (!pending && c->device >= 0 && c->captured) {
		uint64_t w[2];
		if (int r = read_counter_words(c, (size_t)2 * it->second.slot, 2, w))
			return r;
		pk = w[0];
		by = w[1];
	}
	out->packets = pk;
	out->bytes = by;
	return 0;
}

CGPU_EXPORT int cgpu_policy_get_next_key(cgpu_ctx *c, uint32_t ep, const cgpu_policy_key *key,
					 cgpu_policy_key *next)
{
	if (!c || !next || ep >= c->cfg.max_endpoints)
		return fail(-EINVAL, "bad argument");
	std::lock_guard<std::mutex> g(c->mu);
	auto &m = c->pol[ep];
	auto it = key ? m.upper_bound(pol_key64(key)) : m.begin();
	if (it == m.end())
		return -ENOENT;
	memcpy(next, &it->first, 8);
	return 0;
}

CGPU_EXPORT size_t cgpu_policy_count(cgpu_ctx *c, uint32_t ep)
{
	if (!c || ep >= c->cfg.max_endpoints)
		return 0;
	std::lock_guard<std::mutex> g(c->mu);
	return c->pol[ep].size();
}

/* ======================================================================= */
/* prefilter CIDR maps + endpoint map                                        */
/* ======================================================================= */
/* the map operations with mu held (cgpu_prefilter_* runs several under one lock) */
static int cidr_update_l(cgpu_ctx *c, int which, const cgpu_cidr_key *key, uint64_t flags)
{
	bool exists;
	switch (which) {
	case CGPU_CIDR_V4_DYN:
	case CGPU_CIDR_V6_DYN: {
		uint32_t maxp = which == CGPU_CIDR_V4_DYN ? 32 : 128;
		if (key->prefixlen > maxp)
			return fail(-EINVAL, "prefixlen %u > %u", key->prefixlen, maxp);
		if (which == CGPU_CIDR_V4_DYN) {
			auto k = lpm_canon<4>(key->prefixlen, key->addr);
			exists = c->dyn4.count(k);
			if (exists && flags == CGPU_NOEXIST) return fail(-EEXIST, "exists");
			if (!exists && flags == CGPU_EXIST) return fail(-ENOENT, "missing");
			if (!exists && c->dyn4.size() >= c->cfg.cidr_dyn_max) return fail(-ENOSPC, "dyn4 full");
			c->dyn4[k] = *key;
			c->dirty |= 1u << G_PF;
		} else {
			auto k = lpm_canon<16>(key->prefixlen, key->addr);
			exists = c->dyn6.count(k);
			if (exists && flags == CGPU_NOEXIST) return fail(-EEXIST, "exists");
			if (!exists && flags == CGPU_EXIST) return fail(-ENOENT, "missing");
			if (!exists && c->dyn6.size() >= c->cfg.cidr_dyn_max) return fail(-ENOSPC, "dyn6 full");
			c->dyn6[k] = *key;
			c->dirty |= 1u << G_PF;
		}
		return 0;
	}
	case CGPU_CIDR_V4_FIX: {
		std::array<uint8_t, 8> k;
		memcpy(k.data(), key, 8);
		exists = c->fix4.count(k);
		if (exists && flags == CGPU_NOEXIST) return fail(-EEXIST, "exists");
		if (!exists && flags == CGPU_EXIST) return fail(-ENOENT, "missing");
		if (!exists && c->fix4.size() >= c->cfg.cidr_fix_max) return fail(-E2BIG, "fix4 full");
		c->fix4.insert(k);
		c->dirty |= 1u << G_PF;
		return 0;
	}
	case CGPU_CIDR_V6_FIX: {
		std::array<uint8_t, 20> k;
		memcpy(k.data(), key, 20);
		exists = c->fix6.count(k);
		if (exists && flags == CGPU_NOEXIST) return fail(-EEXIST, "exists");
		if (!exists && flags == CGPU_EXIST) return fail(-ENOENT, "missing");
		if (!exists && c->fix6.size() >= c->cfg.cidr_fix_max) return fail(-E2BIG, "fix6 full");
		c->fix6.insert(k);
		c->dirty |= 1u << G_PF;
		return 0;
	}
	}
	return fail(-EINVAL, "bad cidr map %d", which);
}

CGPU_EXPORT int cgpu_cidr_update(cgpu_ctx *c, int which, const cgpu_cidr_key *key, uint64_t flags)
{
	if (!c || !key)
		return fail(-EINVAL, "null argument");
	if (int r = check_flags(flags))
		return r;
	std::lock_guard<std::mutex> g(c->mu);
	return cidr_update_l(c, which, key, flags);
}

static int cidr_delete_l(cgpu_ctx *c, int which, const cgpu_cidr_key *key)
{
	size_t n = 0;
	switch (which) {
	case CGPU_CIDR_V4_DYN:
		if (key->prefixlen > 32) return fail(-EINVAL, "prefixlen");
		n = c->dyn4.erase(lpm_canon<4>(key->prefixlen, key->addr));
		break;
	case CGPU_CIDR_V6_DYN:
		if (key->prefixlen > 128) return fail(-EINVAL, "prefixlen");
		n = c->dyn6.erase(lpm_canon<16>(key->prefixlen, key->addr));
		break;
	case CGPU_CIDR_V4_FIX: {
		std::array<uint8_t, 8> k;
		memcpy(k.data(), key, 8);
		n = c->fix4.erase(k);
		break;
	}
	case CGPU_CIDR_V6_FIX: {
		std::array<uint8_t, 20> k;
		memcpy(k.data(), key, 20);
		n = c->fix6.erase(k);
		break;
	}
	default:
		return fail(-EINVAL, "bad cidr map %d", which);
	}
	if (n)
		c->dirty |= 1u << G_PF;
	return n ? 0 : -ENOENT;
}

CGPU_EXPORT int cgpu_cidr_delete(cgpu_ctx *c, int which, const cgpu_cidr_key *key)
{
	if (!c || !key)
		return fail(-EINVAL, "null argument");
	std::lock_guard<std::mutex> g(c->mu);
	return cidr_delete_l(c, which, key);
}

static int cidr_lookup_l(cgpu_ctx *c, int which, const cgpu_cidr_key *key)
{
	switch (which) {
	case CGPU_CIDR_V4_DYN:
		for (int64_t p = std::min<uint32_t>(key->prefixlen, 32); p >= 0; p--)
			if (c->dyn4.count(lpm_canon<4>((uint32_t)p, key->addr)))
				return 0;
		return -ENOENT;
	case CGPU_CIDR_V6_DYN:
		for (int64_t p = std::min<uint32_t>(key->prefixlen, 128); p >= 0; p--)
			if (c->dyn6.count(lpm_canon<16>((uint32_t)p, key->addr)))
				return 0;
		return -ENOENT;
	case CGPU_CIDR_V4_FIX: {
		std::array<uint8_t, 8> k;
		memcpy(k.data(), key, 8);
		return c->fix4.count(k) ? 0 : -ENOENT;
	}
	case CGPU_CIDR_V6_FIX: {
		std::array<uint8_t, 20> k;
		memcpy(k.data(), key, 20);
		return c->fix6.count(k) ? 0 : -ENOENT;
	}
	}
	return fail(-EINVAL, "bad cidr map %d", which);
}

CGPU_EXPORT int cgpu_cidr_lookup(cgpu_ctx *c, int which, const cgpu_cidr_key *key)
{
	if (!c || !key)
		return fail(-EINVAL, "null argument");
	std::lock_guard<std::mutex> g(c->mu);
	return cidr_lookup_l(c, which, key);
}

/* ---- PreFilter (pkg/policy/prefilter.go:30-203) over the four maps ---- */
/* selectMap (prefilter.go:108-122): /32 and /128 to the exact maps, shorter
 * prefixes to the LPM maps; -1: no such map enabled (maps exist iff their
 * config switch is on, prefilter.go:206-250; the v6 exact map follows its
 * own switch, not fix4 as the reference's initOneMap does, :237) */
static int prefilter_select(const cgpu_ctx *c, const cgpu_prefix &p)
{
	int which;
	if (p.bits == 32)
		which = p.key.prefixlen == 32 ? CGPU_CIDR_V4_FIX : CGPU_CIDR_V4_DYN;
	else if (p.bits == 128)
		which = p.key.prefixlen == 128 ? CGPU_CIDR_V6_FIX : CGPU_CIDR_V6_DYN;
	else
		return -1;
	const bool on[4] = {c->cfg.prefilter_dyn4 != 0, c->cfg.prefilter_fix4 != 0,
			    c->cfg.prefilter_dyn6 != 0, c->cfg.prefilter_fix6 != 0};
	return on[which] ? which : -1;
}

CGPU_EXPORT int cgpu_prefilter_insert(cgpu_ctx *c, int64_t revision, const cgpu_prefix *cidrs, size_t n)
{
	if (!c || (n && !cidrs))
		return fail(-EINVAL, "null argument");
	std::lock_guard<std::mutex> g(c->mu);
	if (revision != 0 && c->pf_revision != revision)
		return fail(-ESTALE, "Latest revision is %lld not %lld", (long long)c->pf_revision,
			    (long long)revision);
	size_t done = 0;
	int rc = 0;
	for (; done < n; done++) {
		const int which = prefilter_select(c, cidrs[done]);
		if (which < 0) {
			rc = fail(-EOPNOTSUPP, "No map enabled for CIDR %zu", done);
			break;
		}
		if ((rc = cidr_update_l(c, which, &cidrs[done].key, CGPU_ANY)) != 0)
			break;
	}
	if (!rc) {
		c->pf_revision++;
		return 0;
	}
	const std::string msg = g_last_error;
	for (size_t i = 0; i < done; i++) /* undo (prefilter.go:152-156) */
		(void)cidr_delete_l(c, prefilter_select(c, cidrs[i]), &cidrs[i].key);
	g_last_error = msg;
	return rc;
}

CGPU_EXPORT int cgpu_prefilter_delete(cgpu_ctx *c, int64_t revision, const cgpu_prefix *cidrs, size_t n)
{
	if (!c || (n && !cidrs))
		return fail(-EINVAL, "null argument");
	std::lock_guard<std::mutex> g(c->mu);
	if (revision != 0 && c->pf_revision != revision)
		return fail(-ESTALE, "Latest revision is %lld not %lld", (long long)c->pf_revision,
			    (long long)revision);
	/* the obvious cases first, so nothing needs unrolling (prefilter.go:171-181):
	 * CIDRExists is a map lookup, longest-prefix on the LPM maps */
	for (size_t i = 0; i < n; i++) {
		const int which = prefilter_select(c, cidrs[i]);
		if (which < 0)
			return fail(-EOPNOTSUPP, "No map enabled for CIDR %zu", i);
		if (cidr_lookup_l(c, which, &cidrs[i].key) != 0)
			return fail(-ENOENT, "No map entry for CIDR %zu", i);
	}
	size_t done = 0;
	int rc = 0;
	for (; done < n; done++)
		if ((rc = cidr_delete_l(c, prefilter_select(c, cidrs[done]), &cidrs[done].key)) != 0) {
			rc = fail(rc, "Error deleting CIDR %zu", done);
			break;
		}
	if (!rc) {
		c->pf_revision++;
		return 0;
	}
	const std::string msg = g_last_error;
	for (size_t i = 0; i < done; i++) /* undo (prefilter.go:196-200) */
		(void)cidr_update_l(c, prefilter_select(c, cidrs[i]), &cidrs[i].key, CGPU_ANY);
	g_last_error = msg;
	return rc;
}

CGPU_EXPORT int cgpu_prefilter_revision(cgpu_ctx *c, int64_t *revision_out)
{
	if (!c || !revision_out)
		return fail(-EINVAL, "null argument");
	std::lock_guard<std::mutex> g(c->mu);
	*revision_out = c->pf_revision;
	return 0;
}

CGPU_EXPORT int cgpu_cidr_get_next_key(cgpu_ctx *c, int which, const cgpu_cidr_key *key,
				       cgpu_cidr_key *next)
{
	if (!c || !next)
		return fail(-EINVAL, "null argument");
	std::lock_guard<std::mutex> g(c->mu);
	memset(next, 0, sizeof(*next));
	switch (which) {
	case CGPU_CIDR_V4_DYN: {
		auto it = key ? c->dyn4.upper_bound(lpm_canon<4>(std::min<uint32_t>(key->prefixlen, 32), key->addr))
			      : c->dyn4.begin();
		if (it == c->dyn4.end()) return -ENOENT;
		*next = it->second;
		return 0;
	}
	case CGPU_CIDR_V6_DYN: {
		auto it = key ? c->dyn6.upper_bound(lpm_canon<16>(std::min<uint32_t>(key->prefixlen, 128), key->addr))
			      : c->dyn6.begin();
		if (it == c->dyn6.end()) return -ENOENT;
		*next = it->second;
		return 0;
	}
	case CGPU_CIDR_V4_FIX: {
		std::array<uint8_t, 8> k{};
		if (key) memcpy(k.data(), key, 8);
		auto it = key ? c->fix4.upper_bound(k) : c->fix4.begin();
		if (it == c->fix4.end()) return -ENOENT;
		memcpy(next, it->data(), 8);
		return 0;
	}
	case CGPU_CIDR_V6_FIX: {
		std::array<uint8_t, 20> k{};
		if (key) memcpy(k.data(), key, 20);
		auto it = key ? c->fix6.upper_bound(k) : c->fix6.begin();
		if (it == c->fix6.end()) return -ENOENT;
		memcpy(next, it->data(), 20);
		return 0;
	}
	}
	return fail(-EINVAL, "bad cidr map %d", which);
}

CGPU_EXPORT int cgpu_endpoint_update(cgpu_ctx *c, const cgpu_endpoint_key *key, uint64_t flags)
{
	if (!c || !key)
		return fail(-EINVAL, "null argument");
	if (int r = check_flags(flags))
		return r;
	std::array<uint8_t, 20> k;
	memcpy(k.data(), key, 20);
	std::lock_guard<std::mutex> g(c->mu);
	bool exists = c->lxc.count(k);
	if (exists && flags == CGPU_NOEXIST) return fail(-EEXIST, "exists");
	if (!exists && flags == CGPU_EXIST) return fail(-ENOENT, "missing");
	if (!exists && c->lxc.size() >= c->cfg.endpoints_max) return fail(-E2BIG, "endpoint map full");
	c->lxc.insert(k);
	c->dirty |= 1u << G_EP;
	return 0;
}

CGPU_EXPORT int cgpu_endpoint_delete(cgpu_ctx *c, const cgpu_endpoint_key *key)
{
	if (!c || !key)
		return fail(-EINVAL, "null argument");
	std::array<uint8_t, 20> k;
	memcpy(k.data(), key, 20);
	std::lock_guard<std::mutex> g(c->mu);
	if (!c->lxc.erase(k))
		return -ENOENT;
	c->dirty |= 1u << G_EP;
	return 0;
}

CGPU_EXPORT int cgpu_endpoint_lookup(cgpu_ctx *c, const cgpu_endpoint_key *key)
{
	if (!c || !key)
		return fail(-EINVAL, "null argument");
	std::array<uint8_t, 20> k;
	memcpy(k.data(), key, 20);
	std::lock_guard<std::mutex> g(c->mu);
	return c->lxc.count(k) ? 0 : -ENOENT;
}

/* per-endpoint identity of the endpoint program (lib/lxc.h:31-89) */
CGPU_EXPORT int cgpu_lxc_update(cgpu_ctx *c, uint32_t ep, const cgpu_lxc_info *info)
{
	if (!c || !info)
		return fail(-EINVAL, "null argument");
	if (ep >= 65536u)
		return fail(-EINVAL, "endpoint id beyond the u16 ep column");
	if (info->verify & ~(CGPU_VERIFY_SMAC | CGPU_VERIFY_DMAC | CGPU_VERIFY_SIP))
		return fail(-EINVAL, "unknown verify bits");
	std::lock_guard<std::mutex> g(c->mu);
	c->lxcinfo[ep] = *info;
	c->dirty |= 1u << G_LXC;
	return 0;
}

CGPU_EXPORT int cgpu_lxc_delete(cgpu_ctx *c, uint32_t ep)
{
	if (!c)
		return fail(-EINVAL, "null argument");
	std::lock_guard<std::mutex> g(c->mu);
	if (!c->lxcinfo.erase(ep))
		return -ENOENT;
	c->dirty |= 1u << G_LXC;
	return 0;
}

CGPU_EXPORT int cgpu_lxc_lookup(cgpu_ctx *c, uint32_t ep, cgpu_lxc_info *out)
{
	if (!c || !out)
		return fail(-EINVAL, "null argument");
	std::lock_guard<std::mutex> g(c->mu);
	auto it = c->lxcinfo.find(ep);
	if (it == c->lxcinfo.end())
		return -ENOENT;
	*out = it->second;
	return 0;
}

/* ======================================================================= */
/* service map (pkg/maps/lbmap; bpf(2) htab semantics, whole-key compare)    */
/* ======================================================================= */
static inline uint64_t lb_mkey(const cgpu_lb4_key *k)
{
	return (uint64_t)k->address << 32 | (uint64_t)k->dport << 16 | k->slave;
}

static inline cgpu_lb4_key lb_unkey(uint64_t m)
{
	cgpu_lb4_key k;
	k.address = (uint32_t)(m >> 32);
	k.dport = (uint16_t)(m >> 16);
	k.slave = (uint16_t)m;
	return k;
}

static int lb_put(cgpu_ctx *c, const cgpu_lb4_key *key, const cgpu_lb4_service *val, uint64_t flags)
{
	const uint64_t m = lb_mkey(key);
	auto it = c->lb.find(m);
	if (it == c->lb.end()) {
		if (flags == CGPU_EXIST)
			return fail(-ENOENT, "lb4 key not present");
		if (c->lb.size() >= c->cfg.lb_max_entries)
			return fail(-E2BIG, "lb4 service map full (%u)", c->cfg.lb_max_entries);
		c->lb.emplace(m, *val);
	} else {
		if (flags == CGPU_NOEXIST)
			return fail(-EEXIST, "lb4 key exists");
		it->second = *val;
	}
	c->dirty |= 1u << G_LB;
	return 0;
}

CGPU_EXPORT int cgpu_lb4_update(cgpu_ctx *c, const cgpu_lb4_key *key, const cgpu_lb4_service *val,
				uint64_t flags)
{
	if (!c || !key || !val)
		return fail(-EINVAL, "null argument");
	if (int r = check_flags(flags))
		return r;
	std::lock_guard<std::mutex> g(c->mu);
	return lb_put(c, key, val, flags);
}

CGPU_EXPORT int cgpu_lb4_update_batch(cgpu_ctx *c, const cgpu_lb4_key *keys,
				      const cgpu_lb4_service *vals, size_t n, uint64_t flags)
{
	if (!c || (n && (!keys || !vals)))
		return fail(-EINVAL, "null argument");
	if (int r = check_flags(flags))
		return r;
	std::lock_guard<std::mutex> g(c->mu);
	for (size_t i = 0; i < n; i++)
		if (int r = lb_put(c, &keys[i], &vals[i], flags))
			return r;
	return 0;
}

CGPU_EXPORT int cgpu_lb4_delete(cgpu_ctx *c, const cgpu_lb4_key *key)
{
	if (!c || !key)
		return fail(-EINVAL, "null argument");
	std::lock_guard<std::mutex> g(c->mu);
	if (!c->lb.erase(lb_mkey(key)))
		return -ENOENT;
	c->dirty |= 1u << G_LB;
	return 0;
}

CGPU_EXPORT int cgpu_lb4_lookup(cgpu_ctx *c, const cgpu_lb4_key *key, cgpu_lb4_service *out)
{
	if (!c || !key || !out)
		return fail(-EINVAL, "null argument");
	std::lock_guard<std::mutex> g(c->mu);
	auto it = c->lb.find(lb_mkey(key));
	if (it == c->lb.end())
		return -ENOENT;
	*out = it->second;
	return 0;
}

CGPU_EXPORT int cgpu_lb4_get_next_key(cgpu_ctx *c, const cgpu_lb4_key *key, cgpu_lb4_key *next)
{
	if (!c || !next)
		return fail(-EINVAL, "null argument");
	std::lock_guard<std::mutex> g(c->mu);
	auto it = key ? c->lb.upper_bound(lb_mkey(key)) : c->lb.begin();
	if (it == c->lb.end())
		return -ENOENT;
	*next = lb_unkey(it->first);
	return 0;
}

CGPU_EXPORT size_t cgpu_lb4_count(cgpu_ctx *c)
{
	if (!c)
		return 0;
	std::lock_guard<std::mutex> g(c->mu);
	return c->lb.size();
}

static int lb6_put(cgpu_ctx *c, const cgpu_lb6_key *key, const cgpu_lb6_service *val, uint64_t flags)
{
	const Lb6K m = lb6_mkey(key);
	auto it = c->lb6.find(m);
	if (it == c->lb6.end()) {
		if (flags == CGPU_EXIST)
			return fail(-ENOENT, "lb6 key not present");
		if (c->lb6.size() >= c->cfg.lb_max_entries)
			return fail(-E2BIG, "lb6 service map full (%u)", c->cfg.lb_max_entries);
		c->lb6.emplace(m, *val);
	} else {
		if (flags == CGPU_NOEXIST)
			return fail(-EEXIST, "lb6 key exists");
		it->second = *val;
	}
	c->dirty |= 1u << G_LB6;
	return 0;
}

CGPU_EXPORT int cgpu_lb6_update(cgpu_ctx *c, const cgpu_lb6_key *key, const cgpu_lb6_service *val,
				uint64_t flags)
{
	if (!c || !key || !val)
		return fail(-EINVAL, "null argument");
	if (int r = check_flags(flags))
		return r;
	std::lock_guard<std::mutex> g(c->mu);
	return lb6_put(c, key, val, flags);
}

CGPU_EXPORT int cgpu_lb6_update_batch(cgpu_ctx *c, const cgpu_lb6_key *keys,
				      const cgpu_lb6_service *vals, size_t n, uint64_t flags)
{
	if (!c || (n && (!keys || !vals)))
		return fail(-EINVAL, "null argument");
	if (int r = check_flags(flags))
		return r;
	std::lock_guard<std::mutex> g(c->mu);
	for (size_t i = 0; i < n; i++)
		if (int r = lb6_put(c, &keys[i], &vals[i], flags))
			return r;
	return 0;
}

CGPU_EXPORT int cgpu_lb6_delete(cgpu_ctx *c, const cgpu_lb6_key *key)
{
	if (!c || !key)
		return fail(-EINVAL, "null argument");
	std::lock_guard<std::mutex> g(c->mu);
	if (!c->lb6.erase(lb6_mkey(key)))
		return -ENOENT;
	c->dirty |= 1u << G_LB6;
	return 0;
}

CGPU_EXPORT int cgpu_lb6_lookup(cgpu_ctx *c, const cgpu_lb6_key *key, cgpu_lb6_service *out)
{
	if (!c || !key || !out)
		return fail(-EINVAL, "null argument");
	std::lock_guard<std::mutex> g(c->mu);
	auto it = c->lb6.find(lb6_mkey(key));
	if (it == c->lb6.end())
		return -ENOENT;
	*out = it->second;
	return 0;
}

CGPU_EXPORT int cgpu_lb6_get_next_key(cgpu_ctx *c, const cgpu_lb6_key *key, cgpu_lb6_key *next)
{
	if (!c || !next)
		return fail(-EINVAL, "null argument");
	std::lock_guard<std::mutex> g(c->mu);
	auto it = key ? c->lb6.upper_bound(lb6_mkey(key)) : c->lb6.begin();
	if (it == c->lb6.end())
		return -ENOENT;
	*next = lb6_unkey(it->first);
	return 0;
}

CGPU_EXPORT size_t cgpu_lb6_count(cgpu_ctx *c)
{
	if (!c)
		return 0;
	std::lock_guard<std::mutex> g(c->mu);
	return c->lb6.size();
}

CGPU_EXPORT uint32_t cgpu_flow_hash6(const uint8_t *saddr16, const uint8_t *daddr16, uint16_t sport,
				     uint16_t dport, uint8_t proto)
{
	uint32_t s[4] = {0, 0, 0, 0}, d[4] = {0, 0, 0, 0};
	if (saddr16)
		memcpy(s, saddr16, 16);
	if (daddr16)
		memcpy(d, daddr16, 16);
	return flow_hash(fold6(s[0], s[1], s[2], s[3]), fold6(d[0], d[1], d[2], d[3]), sport, dport, proto);
}


CGPU_EXPORT uint32_t cgpu_flow_hash(uint32_t saddr, uint32_t daddr, uint16_t sport, uint16_t dport,
				    uint8_t proto)
{
	return flow_hash(saddr, daddr, sport, dport, proto);
}


/* ======================================================================= */
/* commit: capture (mirror lock) -> compile (no lock) -> upload -> publish   */
/* ======================================================================= */
namespace {

struct PolChange {
	uint32_t ep;
	uint64_t key;
	bool present;
	PolEntry e;
};

/* everything a commit compiles, copied out of the mirror under mu */
struct CommitIn {
	uint64_t id = 0;
	uint32_t dirty = 0;
	cgpu_config cfg{};
	/* ipcache */
	bool ipc4_full = false, ipc6_build = false;
	std::vector<Rank4> ipc4_cand;
	std::vector<Ipc4Patch> ipc4_patches;
	std::vector<Rank6> ipc6_cand;
	/* policy */
	bool pol_full = false;
	std::vector<PolKey> pol_keys;
	std::vector<PolChange> pol_changes;
	uint32_t next_hot = 0, next_cold = 0;
	std::vector<SlotInit> inits;
	/* other groups (full copies when dirty) */
	PfIn pf{};
	std::vector<std::array<uint8_t, 20>> lxc;
	LbIn lb;
	Lb6In lb6;
	std::vector<std::pair<uint32_t, cgpu_lxc_info>> lxcinfo;
	uint64_t sum_ipc = 0, sum_pol = 0, sum_slots = 0;
};


static PolKey pol_key_of(uint32_t ep, uint64_t key, const PolEntry &e)
{
	return PolKey{(uint32_t)key, (uint32_t)(key >> 32), ep | (uint32_t)e.proxy_port << 16, e.slot};
}

/* every candidate of one family, in map order (static-part entries first) */
template <typename R, typename F>
static void ipc_family(const cgpu_ctx *c, const uint8_t *stat, std::vector<R> &out, F cand)
{
	uint8_t d[20] = {0};
	memcpy(d, stat, 4);
	for (uint32_t p = 0; p < 32; p++) {
		auto it = c->ipc.find(lpm_canon<20>(p, d));
		R r;
		if (it != c->ipc.end() && cand(it->second, it->first, &r))
			out.push_back(r);
	}
	LpmKey<20> lo = lpm_canon<20>(0, d);
	lo.data = {};
	memcpy(lo.data.data(), stat, 4);
	LpmKey<20> hi = lo;
	hi.data[3]++;
	for (auto it = c->ipc.lower_bound(lo); it != c->ipc.end() && it->first < hi; ++it) {
		R r;
		if (it->second.raw.prefixlen >= 32 && cand(it->second, it->first, &r))
			out.push_back(r);
	}
}

static void capture_ipc(cgpu_ctx *c, CommitIn &in, const BuildState &b)
{
	auto c4 = [](const IpcEntry &e, const LpmKey<20> &, Rank4 *r) {
		return ipc4_candidate(e.raw, e.val.sec_label, r);
	};
	auto c6 = [](const IpcEntry &e, const LpmKey<20> &k, Rank6 *r) {
		return ipc6_candidate(e.raw, k.data.data(), e.val.sec_label, r);
	};
	in.ipc4_full = c->ipc_full || !b.ipc4_ok || b.lc.bloated();
	in.ipc6_build = c->ipc_full || !b.ipc4_ok;
	std::set<LpmKey<20>> seen;
	for (const auto &k : c->ipc_changes) {
		if (in.ipc4_full && in.ipc6_build)
			break;
		if (!seen.insert(k).second)
			continue;
		const uint8_t *d = k.data.data();
		if (k.plen < 32) { /* a static-part entry: under every address */
			if (prefix_eq(d, kStaticV4, k.plen))
				in.ipc4_full = true;
			if (prefix_eq(d, kStaticV6, k.plen))
				in.ipc6_build = true;
			continue;
		}
		if (!memcmp(d, kStaticV6, 4)) {
			in.ipc6_build = true;
			continue;
		}
		if (memcmp(d, kStaticV4, 4) || k.plen > 64 || in.ipc4_full)
			continue; /* no IPv4 lookup reaches it */
		Ipc4Patch pt;
		pt.len = k.plen - 32;
		uint32_t a;
		memcpy(&a, d + 4, 4);
		pt.addr = bswap32(a);
		pt.has_cover = false;
		pt.cover_label = 0;
		for (int64_t l = (int64_t)pt.len - 1; l >= 0 && !pt.has_cover; l--) {
			auto it = c->ipc.find(lpm_canon<20>(32 + (uint32_t)l, d));
			if (it != c->ipc.end()) {
				pt.has_cover = true;
				pt.cover_label = it->second.val.sec_label;
			}
		}
		for (int64_t p = 31; p >= 0 && !pt.has_cover; p--) {
			auto it = c->ipc.find(lpm_canon<20>((uint32_t)p, d));
			if (it != c->ipc.end() && prefix_eq(it->first.data.data(), kStaticV4, (uint32_t)p)) {
				pt.has_cover = true;
				pt.cover_label = it->second.val.sec_label;
			}
		}
		/* every entry inside the range (this key included, if present) */
		LpmKey<20> lo{};
		lo.plen = 0;
		memcpy(lo.data.data(), d, 8);
		const uint32_t last = pt.len ? pt.addr + ((pt.len == 32 ? 1u : (1u << (32 - pt.len))) - 1u)
					     : 0xFFFFFFFFu;
		for (auto it = c->ipc.lower_bound(lo); it != c->ipc.end(); ++it) {
			const uint8_t *e = it->first.data.data();
			if (memcmp(e, kStaticV4, 4))
				break;
			uint32_t ea;
			memcpy(&ea, e + 4, 4);
			if (bswap32(ea) > last)
				break;
			Rank4 r;
			if (it->first.plen >= k.plen && it->first.plen <= 64 &&
			    ipc4_candidate(it->second.raw, it->second.val.sec_label, &r))
				pt.subs.push_back(r);
		}
		in.ipc4_patches.push_back(std::move(pt));
	}
	if (in.ipc4_full) {
		in.ipc4_patches.clear();
		ipc_family<Rank4>(c, kStaticV4, in.ipc4_cand, c4);
	}
	if (in.ipc6_build)
		ipc_family<Rank6>(c, kStaticV6, in.ipc6_cand, c6);
	c->ipc_changes.clear();
	c->ipc_full = false;
}

static void capture_pol(cgpu_ctx *c, CommitIn &in, const BuildState &b)
{
	in.pol_full = c->pol_full || !b.pol_ok;
	if (!in.pol_full) {
		std::set<std::pair<uint32_t, uint64_t>> seen;
		for (auto &ch : c->pol_changes) {
			if (!seen.insert(ch).second)
				continue;
			PolChange pc{ch.first, ch.second, false, PolEntry{0, 0, 0}};
			auto &m = c->pol[ch.first];
			auto it = m.find(ch.second);
			if (it != m.end()) {
				pc.present = true;
				pc.e = it->second;
			}
			in.pol_changes.push_back(pc);
		}
		if (b.pol.count + in.pol_changes.size() > b.pol.slots.size() / 2 ||
		    b.pg.count + in.pol_changes.size() > b.pg.slots.size() / 2)
			in.pol_full = true; /* could pass 50 % load: grow */
	}
	if (in.pol_full) {
		in.pol_changes.clear();
		in.pol_keys.reserve(c->pol_total);
		for (uint32_t ep = 0; ep < c->pol.size(); ep++)
			for (auto &kv : c->pol[ep])
				in.pol_keys.push_back(pol_key_of(ep, kv.first, kv.second));
	}
	c->pol_changes.clear();
	c->pol_full = false;
}

static void capture(cgpu_ctx *c, CommitIn &in, const BuildState &b)
{
	in.dirty = c->dirty;
	in.cfg = c->cfg;
	if (in.dirty & (1u << G_IPC))
		capture_ipc(c, in, b);
	if (in.dirty & (1u << G_POL))
		capture_pol(c, in, b);
	in.next_hot = c->next_hot;
	in.next_cold = c->next_cold;
	in.inits.swap(c->slot_inits);
	if (in.dirty & (1u << G_PF)) {
		in.pf.fix4 = c->cfg.prefilter_fix4;
		in.pf.dyn4 = c->cfg.prefilter_dyn4;
		in.pf.fix6 = c->cfg.prefilter_fix6;
		in.pf.dyn6 = c->cfg.prefilter_dyn6;
		for (auto &kv : c->dyn4) { /* canonical (masked) addresses */
			cgpu_cidr_key k{};
			k.prefixlen = kv.first.plen;
			memcpy(k.addr, kv.first.data.data(), 4);
			in.pf.dyn4k.push_back(k);
		}
		for (auto &kv : c->dyn6) {
			cgpu_cidr_key k{};
			k.prefixlen = kv.first.plen;
			memcpy(k.addr, kv.first.data.data(), 16);
			in.pf.dyn6k.push_back(k);
		}
		for (auto &x : c->fix4) {
			cgpu_cidr_key k{};
			memcpy(&k, x.data(), 8);
			in.pf.fix4k.push_back(k);
		}
		for (auto &x : c->fix6) {
			cgpu_cidr_key k{};
			memcpy(&k, x.data(), 20);
			in.pf.fix6k.push_back(k);
		}
	}
	if (in.dirty & (1u << G_EP))
		in.lxc.assign(c->lxc.begin(), c->lxc.end());
	if (in.dirty & (1u << G_LB))
		in.lb.assign(c->lb.begin(), c->lb.end());
	if (in.dirty & (1u << G_LB6))
		in.lb6.assign(c->lb6.begin(), c->lb6.end());
	if (in.dirty & (1u << G_LXC))
		in.lxcinfo.assign(c->lxcinfo.begin(), c->lxcinfo.end());
	in.sum_ipc = c->sum_ipc;
	in.sum_pol = c->sum_pol;
	in.sum_slots = c->sum_slots;
	c->dirty = 0;
	in.id = ++c->captured;
}

/* a failed commit leaves its groups to be recompiled whole next time */
static void uncapture(cgpu_ctx *c, const CommitIn &in)
{
	c->dirty |= in.dirty;
	if (in.dirty & (1u << G_IPC)) {
		c->ipc_full = true;
		c->ipc_changes.clear();
	}
	if (in.dirty & (1u << G_POL)) {
		c->pol_full = true;
		c->pol_changes.clear();
	}
	c->slot_inits.insert(c->slot_inits.begin(), in.inits.begin(), in.inits.end());
}

/* table_sum_word over words [a, b) of one part (its bytes at word w0) */
static uint64_t part_sum(const uint8_t *p, size_t bytes, size_t w0, size_t a, size_t b)
{
	uint64_t sum = 0;
	const size_t full = std::min(b, bytes / 8u);
	for (size_t j = a; j < full; j++) {
		uint64_t w;
		memcpy(&w, p + 8u * j, 8);
		sum += table_sum_word(w, w0 + j);
	}
	if (b > full && full * 8u < bytes) {
		uint64_t w = 0;
		memcpy(&w, p + 8u * full, bytes % 8u);
		sum += table_sum_word(w, w0 + full);
	}
	return sum;
}

/* table_sum_word over the arena's parts at their offsets (large arenas on
 * several threads: a commit waits for it) */
static uint64_t arena_sum(const Arena &ar)
{
	const size_t big = (size_t)1 << 20;
	uint64_t sum = 0;
	for (size_t i = 0; i < ar.parts.size(); i++) {
		const uint8_t *p = static_cast<const uint8_t *>(ar.parts[i].first);
		const size_t bytes = ar.parts[i].second, w0 = ar.offs[i] / 8u, nw = (bytes + 7u) / 8u;
		if (bytes < 4 * big) {
			sum += part_sum(p, bytes, w0, 0, nw);
			continue;
		}
		const size_t nt = std::min<size_t>(8, bytes / big);
		std::vector<uint64_t> sums(nt, 0);
		std::vector<std::thread> th;
		for (size_t t = 0; t < nt; t++)
			th.emplace_back([&, t] { sums[t] = part_sum(p, bytes, w0, nw * t / nt, nw * (t + 1) / nt); });
		for (auto &x : th)
			x.join();
		for (uint64_t x : sums)
			sum += x;
	}
	return sum;
}

/* Upload an arena as one group buffer (stream-ordered on ustream), and queue
 * the device-side sum of what landed into d_verify[slot]: cgpu_commit
 * compares it with the host image's sum before publishing (SURVEY §5:
 * a bad upload or a corrupted buffer is an -EIO, not silent wrong verdicts). */
static int upload(cgpu_ctx *c, const Arena &ar, DevBufP &out, int slot)
{
	auto b = std::make_shared<DevBuf>();
	b->dev = c->device;
	b->st = c->rstream;
	b->bytes = ar.total ? ar.total : 256;
	HIP_OR_EIO(hipMallocFromPoolAsync(&b->p, b->bytes, c->pool, c->ustream));
	for (size_t i = 0; i < ar.parts.size(); i++)
		if (ar.parts[i].second) {
			HIP_OR_EIO(hipMemcpyAsync((char *)b->p + ar.offs[i], ar.parts[i].first, ar.parts[i].second,
						  hipMemcpyHostToDevice, c->ustream));
			HIP_OR_EIO(launch_table_sum(b->p, ar.offs[i], ar.parts[i].second, c->d_verify + slot,
						    c->ustream));
			b->parts.push_back({ar.offs[i], ar.parts[i].second});
		}
	b->host_sum = arena_sum(ar); /* while the device copies and sums */
	out = b;
	return 0;
}

template <typename T> static const T *at(const DevBufP &b, size_t off)
{
	return reinterpret_cast<const T *>(static_cast<const char *>(b->p) + off);
}

/* group IPC: compressed ipcache v4 (+ DIR-24-8 leaves' vals) and v6 LPM */
static int commit_ipc(cgpu_ctx *c, CommitIn &in, cgpu_snapshot &s, DevBufP &buf)
{
	BuildState &b = c->b;
	if (in.ipc4_full) {
		build_dir(std::move(in.ipc4_cand), b.dir, false);
		b.lc.build(b.dir.tbl24, b.dir.tbl8);
		b.ipc4_ok = true;
	} else {
		for (auto &pt : in.ipc4_patches)
			apply_ipc4_patch(pt, b.dir, b.lc);
	}
	if (in.ipc6_build) {
		b.v6 = V6Build();
		build_v6(std::move(in.ipc6_cand), b.v6);
	}
	Arena ar;
	const size_t o_x = ar.add(b.lc.x16.data(), b.lc.x16.size() * 4);
	const size_t o_d = ar.add(b.lc.d16.data(), b.lc.d16.size() * 4);
	const size_t o_n = ar.add(b.lc.nodes.data(), b.lc.nodes.size() * 4);
	const size_t o_c = ar.add(b.lc.dict.data(), b.lc.dict.size() * 4);
	const size_t o_v = ar.add(b.dir.vals.data(), b.dir.vals.size() * 4);
	if (b.v6.too_big)
		return fail(-E2BIG, "ipcache v6 trie exceeds 2^29 node lines");
	size_t o6[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
	if (b.v6.any) {
		o6[0] = ar.add(b.v6.root.data(), b.v6.root.size() * 4);
		o6[1] = ar.add(b.v6.b24.data(), b.v6.b24.size() * 4);
		o6[2] = ar.add(b.v6.b32.data(), b.v6.b32.size() * 4);
		o6[3] = ar.add(b.v6.pool.data(), b.v6.pool.size() * 4);
		o6[4] = ar.add(b.v6.vals.data(), b.v6.vals.size() * 4);
		o6[5] = ar.add(b.v6.h64.data(), b.v6.h64.size() * 32);
		o6[6] = ar.add(b.v6.rbits.data(), b.v6.rbits.size() * 4);
		o6[7] = ar.add(b.v6.b24_16.data(), b.v6.b24_16.size() * 2);
		o6[8] = ar.add(b.v6.bl64.data(), b.v6.bl64.size() * 4);
	}
	if (int r = upload(c, ar, buf, G_IPC))
		return r;
	/* the x4 kernels read x16 and the overflow nodes (the leaf dictionary in
	 * LDS); the v6 pre-pass b32, the node lines, labels and h64 records (root
	 * and b24 LDS-staged when representable) */
	buf->gather = (b.lc.x16.size() + b.lc.nodes.size()) * 4;
	if (b.v6.any)
		buf->gather += (b.v6.b32.size() + b.v6.pool.size() + b.v6.vals.size()) * 4 + b.v6.h64.size() * 32 +
			       (b.v6.b24_16.empty() ? b.v6.b24.size() * 4 + b.v6.root.size() * 4 : 0);
	s.ipc4c = lpm16c{at<uint32_t>(buf, o_d), at<uint32_t>(buf, o_n), at<uint32_t>(buf, o_v),
			 at<uint32_t>(buf, o_x), at<uint32_t>(buf, o_c), (uint32_t)b.lc.nodes.size(),
			 (uint32_t)b.lc.dict.size()};
	s.ipc6 = v6_lpm{};
	if (b.v6.any)
		s.ipc6 = v6_lpm{at<uint32_t>(buf, o6[0]), at<uint32_t>(buf, o6[1]), at<uint2>(buf, o6[2]),
				at<uint32_t>(buf, o6[3]), at<uint32_t>(buf, o6[4]), at<uint4>(buf, o6[5]), b.v6.m64,
				at<uint32_t>(buf, o6[6]),
				b.v6.b24_16.empty() ? nullptr : at<uint16_t>(buf, o6[7]),
				(uint32_t)(b.v6.b24.size() / 256), at<uint32_t>(buf, o6[8]),
				(uint32_t)b.v6.bl64.size() - 1u};
	b.sum[G_IPC] = in.sum_ipc;
	return 0;
}

/* group POL: the policy hash and its groups */
static int commit_pol(cgpu_ctx *c, CommitIn &in, cgpu_snapshot &s, DevBufP &buf)
{
	BuildState &b = c->b;
	bool full = in.pol_full;
	if (!full) {
		for (auto &ch : in.pol_changes) {
			const uint32_t lo = (uint32_t)ch.key, hi = (uint32_t)(ch.key >> 32);
			b.pol.erase(lo, hi, ch.ep);
			const PolKey k = pol_key_of(ch.ep, ch.key, ch.e);
			if (!ch.present) {
				b.pg.remove(k);
			} else if (!b.pol.insert(k) || !b.pg.add(k) || b.pg.overloaded()) {
				full = true; /* a full neighbourhood: rebuild from the mirror */
				break;
			}
		}
	}
	if (full) {
		if (in.pol_keys.empty() && !in.pol_full) {
			std::lock_guard<std::mutex> g(c->mu);
			for (uint32_t ep = 0; ep < c->pol.size(); ep++)
				for (auto &kv : c->pol[ep])
					in.pol_keys.push_back(pol_key_of(ep, kv.first, kv.second));
		}
		b.pol.build(in.pol_keys);
		b.pg.build(in.pol_keys);
		b.pol_ok = true;
	}
	Arena ar;
	const size_t o_p = ar.add(b.pol.slots.data(), b.pol.slots.size() * sizeof(pol_slot));
	const size_t o_g = ar.add(b.pg.slots.data(), b.pg.slots.size() * sizeof(uint4));
	if (int r = upload(c, ar, buf, G_POL))
		return r;
	buf->gather = b.pol.slots.size() * sizeof(pol_slot) + b.pg.slots.size() * sizeof(uint4);
	s.pol = pol_table{at<pol_slot>(buf, o_p), b.pol.mask, 0};
	s.pg = pol_groups{at<uint4>(buf, o_g), b.pg.mask, 0};
	b.sum[G_POL] = in.sum_pol;
	return 0;
}

/* the any-match DIR-24-8 image of the v4 deny set as one boundary node per
 * /16 (tables.h PF4X_*) */
static void build_pf4x(const Dir248 &d, std::vector<uint4> &x)
{
	x.assign((size_t)65536 * 2, uint4{0, 0, 0, 0});
	std::vector<uint32_t> b;
	for (uint32_t p = 0; p < 65536; p++) {
		b.clear();
		bool cur = false, flip = false;
		for (uint32_t j = 0; j < 256 && b.size() <= 15; j++) {
			const uint32_t e = d.tbl24[(size_t)p * 256 + j];
			const bool grp = (e & DIR_TAG_MASK) == DIR_TAG_GROUP;
			for (uint32_t k = 0; k < (grp ? 256u : 1u); k++) {
				const bool v = (grp ? d.tbl8[(size_t)(e & DIR_PAYLOAD_MASK) * 256 + k] : e) != 0u;
				const uint32_t at = (j << 8) | k;
				if (at == 0)
					flip = cur = v;
				else if (v != cur) {
					b.push_back(at);
					cur = v;
				}
			}
		}
		uint16_t w[16];
		for (int i = 0; i < 16; i++)
			w[i] = 0xFFFFu;
		uint16_t h = flip ? 1u : 0u;
		if (b.size() > 15) {
			h |= PF4X_OVF;
		} else {
			if (b.size() > 7)
				h |= PF4X_TWO;
			for (size_t i = 0; i < b.size(); i++)
				w[1 + i] = (uint16_t)(b[i] - 1u);
		}
		w[0] = h;
		uint32_t u[8];
		for (int i = 0; i < 8; i++)
			u[i] = (uint32_t)w[2 * i] | ((uint32_t)w[2 * i + 1] << 16);
		x[2 * p] = uint4{u[0], u[1], u[2], u[3]};
		x[2 * p + 1] = uint4{u[4], u[5], u[6], u[7]};
	}
}

/* group PF: XDP prefilter any-match tables (v4 compressed like the ipcache,
 * v6 interval cover) */
static int commit_pf(cgpu_ctx *c, CommitIn &in, cgpu_snapshot &s, DevBufP &buf)
{
	std::vector<Rank4> c4 = pf4_candidates(in.pf);
	const bool have4 = !c4.empty();
	Dir248 d;
	Lpm16cBuild lc;
	std::vector<uint4> x4;
	if (have4) {
		build_dir(std::move(c4), d, true);
		lc.build(d.tbl24, d.tbl8);
		build_pf4x(d, x4);
		d.tbl24.clear();
		d.tbl24.shrink_to_fit();
		d.tbl8.clear();
		d.tbl8.shrink_to_fit();
	}
	Cover6Build pf6;
	build_cover6(pf6_candidates(in.pf), pf6);
	if (pf6.too_big)
		return fail(-E2BIG, "prefilter v6 cover exceeds 2^25 node lines");
	Arena ar;
	size_t o4[5] = {0, 0, 0, 0, 0}, o6[8] = {0, 0, 0, 0, 0, 0, 0, 0};
	if (have4) {
		o4[4] = ar.add(x4.data(), x4.size() * sizeof(uint4));
		o4[0] = ar.add(lc.x16.data(), lc.x16.size() * 4);
		o4[1] = ar.add(lc.d16.data(), lc.d16.size() * 4);
		o4[2] = ar.add(lc.nodes.data(), lc.nodes.size() * 4);
		o4[3] = ar.add(lc.dict.data(), lc.dict.size() * 4);
	}
	if (pf6.any) {
		o6[0] = ar.add(pf6.root.data(), pf6.root.size() * 4);
		o6[1] = ar.add(pf6.pool.data(), pf6.pool.size() * 4);
		o6[2] = ar.add(pf6.b24.data(), pf6.b24.size() * 4);
		o6[3] = ar.add(pf6.b32.data(), pf6.b32.size() * 4);
		o6[4] = ar.add(pf6.h64.data(), pf6.h64.size() * 32);
		o6[5] = ar.add(pf6.root16.data(), pf6.root16.size() * 2);
		o6[6] = ar.add(pf6.rbits.data(), pf6.rbits.size() * 4);
		o6[7] = ar.add(pf6.b24_16.data(), pf6.b24_16.size() * 2);
	}
	if (int r = upload(c, ar, buf, G_PF))
		return r;
	/* the cascade's lookups gather pf4x (and the nodes of overflowing /16s) */
	buf->gather = have4 ? x4.size() * sizeof(uint4) + lc.nodes.size() * 4 : 0;
	if (pf6.any)
		buf->gather += (pf6.b32.size() + pf6.pool.size()) * 4 + pf6.h64.size() * 32 +
			       (pf6.b24_16.empty() ? pf6.b24.size() * 4 : 0) +
			       (pf6.root16.empty() && pf6.rbits.empty() ? pf6.root.size() * 4 : 0);
	s.pf4c = lpm16c{};
	s.pf4x = have4 ? at<uint4>(buf, o4[4]) : nullptr;
	if (have4)
		s.pf4c = lpm16c{at<uint32_t>(buf, o4[1]), at<uint32_t>(buf, o4[2]), nullptr, at<uint32_t>(buf, o4[0]),
				at<uint32_t>(buf, o4[3]), (uint32_t)lc.nodes.size(), (uint32_t)lc.dict.size()};
	s.pf6 = cover6{};
	if (pf6.any)
		s.pf6 = cover6{at<uint32_t>(buf, o6[0]),
			       pf6.root16.empty() ? nullptr : at<uint16_t>(buf, o6[5]),
			       pf6.rbits.empty() ? nullptr : at<uint32_t>(buf, o6[6]),
			       pf6.rbits.empty() ? nullptr : at<uint16_t>(buf, o6[7]),
			       (uint32_t)(pf6.b24.size() / 256),
			       at<uint32_t>(buf, o6[2]), at<uint32_t>(buf, o6[3]), at<uint32_t>(buf, o6[1]),
			       at<uint4>(buf, o6[4]), pf6.m64};
	uint64_t sum = 0;
	for (auto &k : in.pf.dyn4k) sum += fnv(7, &k, 8);
	for (auto &k : in.pf.dyn6k) sum += fnv(11, &k, 20);
	for (auto &k : in.pf.fix4k) sum += fnv(13, &k, 8);
	for (auto &k : in.pf.fix6k) sum += fnv(17, &k, 20);
	c->b.sum[G_PF] = sum;
	return 0;
}

/* group EP: cilium_lxc endpoint sets */
static int commit_ep(cgpu_ctx *c, CommitIn &in, cgpu_snapshot &s, DevBufP &buf)
{
	std::vector<uint32_t> e4;
	std::vector<std::array<uint32_t, 6>> e6;
	uint64_t sum = 0;
	for (auto &k : in.lxc) {
		sum += fnv(19, k.data(), k.size());
		const cgpu_endpoint_key *ek = (const cgpu_endpoint_key *)k.data();
		if (ek->pad4 || ek->pad5)
			continue; /* lookup keys have zero padding: never matches */
		uint32_t w[4];
		memcpy(w, ek->ip, 16);
		if (ek->family == 1 && !w[1] && !w[2] && !w[3])
			e4.push_back(w[0]);
		else if (ek->family == 2)
			e6.push_back({w[0], w[1], w[2], w[3], 0, 0});
	}
	Set4Build ep4;
	Set16Build ep6;
	build_set4(e4, ep4);
	build_set16(e6, ep6, true); /* bucket = pfx6_hash(raw words, 0) */
	/* the v6 endpoint bloom filter (tables.h ep6_bloom): ~12 bits per key */
	const uint32_t nw = (uint32_t)std::min<uint64_t>(
		EP6_BLOOM_MAX_WORDS, next_pow2(std::max<uint64_t>(64, e6.size() * 12 / 32 + 1)));
	std::vector<uint32_t> bloom(nw, 0);
	for (auto &k : e6) {
		const uint32_t h = pfx6_hash(k[0], k[1], k[2], k[3], 0);
		bloom[v6_bloom_word(h, nw - 1)] |= v6_bloom_bits(h);
	}
	Arena ar;
	const size_t o4 = ar.add(ep4.slots.data(), ep4.slots.size() * sizeof(set4_slot));
	const size_t o6 = ar.add(ep6.slots.data(), ep6.slots.size() * sizeof(set16_slot));
	const size_t ob = ar.add(bloom.data(), bloom.size() * 4);
	if (int r = upload(c, ar, buf, G_EP))
		return r;
	s.ep4 = addr_set4{at<set4_slot>(buf, o4), ep4.mask, ep4.max_probe};
	s.ep6 = addr_set16{at<set16_slot>(buf, o6), ep6.mask, ep6.max_probe};
	s.ep6_bloom = at<uint32_t>(buf, ob);
	s.ep6_bloom_mask = nw - 1;
	c->b.sum[G_EP] = sum;
	return 0;
}

/* group LB: cilium_lb4_services frontends + backends */
static int commit_lb(cgpu_ctx *c, CommitIn &in, cgpu_snapshot &s, DevBufP &buf)
{
	LbBuild lbb;
	if (int r = build_lb(in.lb, in.cfg.lb_max_entries, lbb))
		return r;
	Arena ar;
	const size_t o_f = ar.add(lbb.fe.data(), lbb.fe.size() * 16);
	const size_t o_b = ar.add(lbb.be.data(), lbb.be.size() * 16);
	const size_t o_v = ar.add(lbb.vip.data(), lbb.vip.size() * 4);
	if (int r = upload(c, ar, buf, G_LB))
		return r;
	s.lb = lb_table{at<uint4>(buf, o_f), at<uint4>(buf, o_b), lbb.mask, (uint32_t)lbb.be.size(),
			at<uint32_t>(buf, o_v), lbb.vip_mask};
	uint64_t sum = 0;
	for (auto &kv : in.lb)
		sum += fnv(fnv(23, &kv.first, 8), &kv.second, sizeof(kv.second));
	c->b.sum[G_LB] = sum;
	return 0;
}

/* group LB6: cilium_lb6_services frontends + backends */
static int commit_lb6(cgpu_ctx *c, CommitIn &in, cgpu_snapshot &s, DevBufP &buf)
{
	Lb6Build b;
	if (int r = build_lb6(in.lb6, in.cfg.lb_max_entries, b))
		return r;
	Arena ar;
	const size_t o_f = ar.add(b.fe.data(), b.fe.size() * 32);
	const size_t o_b = ar.add(b.be.data(), b.be.size() * 32);
	const size_t o_v = ar.add(b.vip.data(), b.vip.size() * 4);
	if (int r = upload(c, ar, buf, G_LB6))
		return r;
	s.lb6 = lb6_table{at<uint4>(buf, o_f), at<uint4>(buf, o_b), b.mask, (uint32_t)b.be.size(),
			  at<uint32_t>(buf, o_v), b.vip_mask};
	uint64_t sum = 0;
	for (auto &kv : in.lb6)
		sum += fnv(fnv(31, kv.first.data(), 20), &kv.second, sizeof(kv.second));
	c->b.sum[G_LB6] = sum;
	return 0;
}

/* group LXC: dense per-endpoint lxc identity, 32 B each (absent: verify nothing) */
static int commit_lxc(cgpu_ctx *c, CommitIn &in, cgpu_snapshot &s, DevBufP &buf)
{
	static_assert(sizeof(cgpu_lxc_info) == 32, "cgpu_lxc_info is 2 x uint4");
	const uint32_t n = in.lxcinfo.empty() ? 0u : in.lxcinfo.back().first + 1u;
	std::vector<cgpu_lxc_info> v(n);
	if (n)
		memset(v.data(), 0, v.size() * sizeof(cgpu_lxc_info));
	uint64_t sum = 0;
	for (auto &kv : in.lxcinfo) {
		v[kv.first] = kv.second;
		sum += fnv(fnv(29, &kv.first, 4), &kv.second, sizeof(kv.second));
	}
	Arena ar;
	const size_t o = ar.add(v.data(), v.size() * sizeof(cgpu_lxc_info));
	if (int r = upload(c, ar, buf, G_LXC))
		return r;
	s.lxc = at<uint4>(buf, o);
	s.n_lxc = n;
	c->b.sum[G_LXC] = sum;
	return 0;
}

/* counter slots whose entry was (re)written: their totals restart from the
 * supplied packets/bytes (kernel htab update replaces the value); the newest
 * write of a slot wins */
static int commit_inits(cgpu_ctx *c, const CommitIn &in)
{
	if (in.inits.empty())
		return 0;
	std::vector<uint32_t> slot;
	std::vector<uint64_t> pk, by;
	std::vector<uint8_t> seen(c->n_ctr_slots, 0);
	for (auto it = in.inits.rbegin(); it != in.inits.rend(); ++it) {
		if (seen[it->slot])
			continue;
		seen[it->slot] = 1;
		slot.push_back(it->slot);
		pk.push_back(it->packets);
		by.push_back(it->bytes);
	}
	Arena ar;
	const size_t o_s = ar.add(slot.data(), slot.size() * 4);
	const size_t o_p = ar.add(pk.data(), pk.size() * 8);
	const size_t o_b = ar.add(by.data(), by.size() * 8);
	DevBufP buf;
	if (int r = upload(c, ar, buf, G_N))
		return r;
	HIP_OR_EIO(launch_slot_init(c->d_totals, c->d_delta, at<uint32_t>(buf, o_s), at<uint64_t>(buf, o_p),
				    at<uint64_t>(buf, o_b), (uint32_t)slot.size(), c->ustream));
	/* the scratch buffer's free (on rstream) must follow the init kernel */
	hipEvent_t ev;
	HIP_OR_EIO(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
	(void)hipEventRecord(ev, c->ustream);
	(void)hipStreamWaitEvent(c->rstream, ev, 0);
	(void)hipEventDestroy(ev);
	return 0;
}

} // namespace

static int commit_locked(cgpu_ctx *c, uint64_t *epoch_out);

CGPU_EXPORT int cgpu_commit(cgpu_ctx *c, uint64_t *epoch_out)
{
	if (!c)
		return fail(-EINVAL, "null argument");
	if (c->device < 0)
		return fail(-ENODEV, "context has no device");
	std::lock_guard<std::mutex> cg(c->commit_mu);
	return commit_locked(c, epoch_out);
}

/* the commit proper; caller holds commit_mu */
static int commit_locked(cgpu_ctx *c, uint64_t *epoch_out)
{
	CommitIn in;
	{
		std::lock_guard<std::mutex> g(c->mu);
		capture(c, in, c->b);
	}
	HIP_OR_EIO(hipSetDevice(c->device));
	std::shared_ptr<Epoch> prev;
	{
		std::lock_guard<std::mutex> g(c->pub_mu);
		prev = c->cur;
	}
	auto e = std::make_shared<Epoch>();
	e->c = c;
	e->id = in.id;
	if (prev) {
		e->snap = prev->snap;
		for (int k = 0; k < G_N; k++)
			e->bufs[k] = prev->bufs[k];
	}
	cgpu_snapshot &s = e->snap;
	int (*const step[G_N])(cgpu_ctx *, CommitIn &, cgpu_snapshot &, DevBufP &) = {
		commit_ipc, commit_pol, commit_pf, commit_ep, commit_lb, commit_lxc, commit_lb6};
	int rc = hipMemsetAsync(c->d_verify, 0, (G_N + 1) * 8, c->ustream) == hipSuccess
			 ? 0 : fail(-EIO, "commit: verify buffer reset failed");
	for (int k = 0; k < G_N && !rc; k++)
		if (in.dirty & (1u << k)) {
			rc = step[k](c, in, s, e->bufs[k]);
			/* a host image half-patched by a failed step is rebuilt */
			if (rc && k == G_IPC)
				c->b.ipc4_ok = false;
			if (rc && k == G_POL)
				c->b.pol_ok = false;
		}
	if (!rc)
		rc = commit_inits(c, in);
	hipError_t he = hipSuccess;
	if (!rc && ((he = hipEventCreateWithFlags(&e->ready, hipEventDisableTiming)) != hipSuccess ||
		    (he = hipEventRecord(e->ready, c->ustream)) != hipSuccess ||
		    (he = hipEventSynchronize(e->ready)) != hipSuccess))
		rc = fail(-EIO, "commit upload: %s", hipGetErrorString(he));
	if (!rc) { /* the device's sums of what it received == the host images' */
		uint64_t got[G_N + 1];
		if ((he = hipMemcpy(got, c->d_verify, sizeof(got), hipMemcpyDeviceToHost)) != hipSuccess)
			rc = fail(-EIO, "commit verify: %s", hipGetErrorString(he));
		for (int k = 0; k < G_N && !rc; k++)
			if ((in.dirty & (1u << k)) && e->bufs[k] && got[k] != e->bufs[k]->host_sum)
				rc = fail(-EIO, "device table group %d differs from the host image after upload", k);
	}
	if (rc) {
		std::string msg = g_last_error;
		{
			std::lock_guard<std::mutex> g(c->mu);
			uncapture(c, in);
		}
		{
			std::lock_guard<std::mutex> g(c->retire_mu);
			c->alive.insert(e->id); /* its destructor retires the id */
		}
		e.reset();
		g_last_error = msg;
		return rc;
	}
	const cgpu_config &cf = in.cfg;
	memcpy(s.router_ip64, cf.ipv6_router_ip, 8);
	memcpy(s.router_ip, cf.ipv6_router_ip, 16);
	s.pf4_enabled = cf.prefilter_fix4;
	s.pf6_enabled = cf.prefilter_fix6;
	s.world_id = cf.world_id;
	s.cluster_id = cf.cluster_id;
	s.host_id = cf.host_id;
	s.health_id = cf.health_id;
	s.ipv4_cluster_mask = cf.ipv4_cluster_mask;
	s.ipv4_cluster_range = cf.ipv4_cluster_range;
	s.ct_proto_gate = cf.ct_proto_gate;
	s.ingress_secctx_world = cf.ingress_secctx_world;
	s.ingress_src_identity = cf.ingress_src_identity;
	s.n_ctr_slots = c->n_ctr_slots;
	s.hot_slots = in.next_hot; /* LDS per workgroup: only the hot slots in use */
	s.cold_hi = in.next_cold;
	s.lb_flags = cf.lb_flags;
	s.ipv4_loopback = cf.ipv4_loopback;
	memcpy(&s.node_mac_lo, cf.node_mac, 4);
	s.node_mac_hi = (uint32_t)cf.node_mac[4] | ((uint32_t)cf.node_mac[5] << 8);
	s.schedule = cf.schedule;
	s.epoch = e->id;
	uint64_t sum = 0;
	for (int k = 0; k < G_N; k++)
		sum += c->b.sum[k];
	{
		std::lock_guard<std::mutex> g(c->retire_mu);
		c->alive.insert(e->id);
	}
	{
		std::lock_guard<std::mutex> g(c->pub_mu);
		c->cur.swap(e); /* e now holds the previous snapshot */
		c->epoch = s.epoch;
		c->checksum = sum;
		c->slot_checksum = in.sum_slots;
	}
	e.reset();
	prev.reset(); /* the last reference retires it (waits + frees on rstream) */
	if (epoch_out)
		*epoch_out = s.epoch;
	return 0;
}

CGPU_EXPORT int cgpu_table_checksum(cgpu_ctx *c, uint64_t *sum)
{
	if (!c || !sum)
		return fail(-EINVAL, "null argument");
	std::lock_guard<std::mutex> g(c->pub_mu);
	if (!c->cur)
		return fail(-ENOENT, "nothing committed");
	*sum = c->checksum;
	return 0;
}

CGPU_EXPORT int cgpu_table_bytes(cgpu_ctx *c, uint64_t *out)
{
	if (!c || !out)
		return fail(-EINVAL, "null argument");
	static_assert(G_N == CGPU_TBL_CT4, "table groups of cgpu.h");
	std::shared_ptr<Epoch> ep;
	{
		std::lock_guard<std::mutex> g(c->pub_mu);
		ep = c->cur;
	}
	for (int k = 0; k < G_N; k++) {
		const DevBuf *b = ep ? ep->bufs[k].get() : nullptr;
		out[k] = !b ? 0u : b->gather ? (uint64_t)b->gather : (uint64_t)b->bytes;
	}
	{
		/* ct_classify resizes the mirrors under mu */
		std::lock_guard<std::mutex> g(c->mu);
		out[CGPU_TBL_CT4] = (uint64_t)(c->ct4.keys.size() + c->ct4.vals.size()) * 16u;
		out[CGPU_TBL_CT6] = (uint64_t)(c->ct6.keys.size() + c->ct6.vals.size()) * 16u;
	}
	return 0;
}

/* Popularity-ordered counter slots.  Counter slots [0, hot_cap) accumulate
 * in LDS per workgroup (one flush per workgroup), the rest cost one global
 * atomic per hit that the workgroup's small LDS cache misses; slots are first
 * handed out by key class (L3-only / identity-wildcard keys hot).  This call
 * re-assigns them by measured traffic: the hot_cap keys with the most
 * packets so far take the hot slots (ties: hot class first, then endpoint and
 * key order, so replicas with the same folded totals choose alike), moved
 * keys carry their counters with them, and the policy tables are republished
 * (a commit).  Control-plane call: it synchronizes the device, folds the
 * delta buffer, and needs every map change committed (else -EBUSY); no batch
 * may be launched on the context while it runs. */
CGPU_EXPORT int cgpu_counters_rebalance(cgpu_ctx *c, uint64_t *moved_out)
{
	if (!c)
		return fail(-EINVAL, "null argument");
	if (c->device < 0)
		return fail(-ENODEV, "context has no device");
	std::lock_guard<std::mutex> cg(c->commit_mu);
	uint64_t moved = 0;
	{
		std::lock_guard<std::mutex> g(c->mu);
		if ((c->dirty & (1u << G_POL)) || !c->slot_inits.empty())
			return fail(-EBUSY, "uncommitted policy changes: commit first");
		const size_t words = (size_t)2 * c->n_ctr_slots + CGPU_METRICS_WORDS;
		uint64_t *delta;
		{
			std::lock_guard<std::mutex> pg(c->pk_mu);
			delta = c->d_delta;
		}
		HIP_OR_EIO(hipSetDevice(c->device));
		HIP_OR_EIO(hipDeviceSynchronize());
		HIP_OR_EIO(launch_fold(c->d_totals, delta, words, c->ustream));
		HIP_OR_EIO(hipStreamSynchronize(c->ustream));
		std::vector<uint64_t> tot(words);
		HIP_OR_EIO(hipMemcpy(tot.data(), c->d_totals, words * 8, hipMemcpyDeviceToHost));
		struct K {
			uint64_t pk;
			bool cls;
			uint32_t ep;
			uint64_t key;
			PolEntry *e;
		};
		std::vector<K> ks;
		ks.reserve(c->pol_total);
		for (uint32_t ep = 0; ep < c->pol.size(); ep++)
			for (auto &kv : c->pol[ep]) {
				cgpu_policy_key pkey;
				memcpy(&pkey, &kv.first, 8);
				const bool cls = (pkey.dport == 0 && pkey.protocol == 0) || pkey.sec_label == 0;
				ks.push_back(K{tot[2u * kv.second.slot], cls, ep, kv.first, &kv.second});
			}
		std::sort(ks.begin(), ks.end(), [](const K &a, const K &b) {
			if (a.pk != b.pk)
				return a.pk > b.pk;
			if (a.cls != b.cls)
				return a.cls;
			if (a.ep != b.ep)
				return a.ep < b.ep;
			return a.key < b.key;
		});
		const size_t H = std::min<size_t>(c->hot_cap, ks.size());
		std::vector<uint8_t> used(c->n_ctr_slots, 0);
		for (auto &k : ks)
			used[k.e->slot] = 1;
		/* target keys already hot stay; the others' hot slots are released */
		std::vector<uint8_t> keep(c->hot_cap, 0);
		for (size_t i = 0; i < H; i++)
			if (ks[i].e->slot < c->hot_cap)
				keep[ks[i].e->slot] = 1;
		std::vector<uint64_t> nt(tot.begin(), tot.begin() + 2 * (size_t)c->n_ctr_slots);
		std::vector<uint32_t> hot_free, cold_free;
		for (uint32_t sl = c->hot_cap; sl-- > 0;)
			if (!keep[sl])
				hot_free.push_back(sl); /* lowest last: handed out first */
		uint32_t next_cold = c->next_cold;
		for (uint32_t sl = c->n_ctr_slots; sl-- > c->hot_cap;)
			if (sl < next_cold && !used[sl])
				cold_free.push_back(sl);
		auto move = [&](PolEntry *e, uint32_t to) {
			nt[2u * to] = tot[2u * e->slot];
			nt[2u * to + 1u] = tot[2u * e->slot + 1u];
			e->slot = to;
			moved++;
		};
		/* evict non-target keys from hot slots first (their slots are in hot_free) */
		for (size_t i = H; i < ks.size(); i++) {
			PolEntry *e = ks[i].e;
			if (e->slot >= c->hot_cap)
				continue;
			uint32_t to;
			if (!cold_free.empty()) {
				to = cold_free.back();
				cold_free.pop_back();
			} else if (next_cold < c->n_ctr_slots) {
				to = next_cold++;
			} else {
				return fail(-E2BIG, "no cold counter slot left to rebalance into");
			}
			nt[2u * e->slot] = nt[2u * e->slot + 1u] = 0;
			move(e, to);
		}
		for (size_t i = 0; i < H; i++) {
			PolEntry *e = ks[i].e;
			if (e->slot < c->hot_cap)
				continue;
			const uint32_t from = e->slot;
			const uint32_t to = hot_free.back();
			hot_free.pop_back();
			move(e, to);
			nt[2u * from] = nt[2u * from + 1u] = 0;
			cold_free.push_back(from);
		}
		/* counters follow their keys; the layout sum is recomputed */
		HIP_OR_EIO(hipMemcpy(c->d_totals, nt.data(), nt.size() * 8, hipMemcpyHostToDevice));
		c->sum_slots = 0;
		for (auto &k : ks)
			c->sum_slots += slot_hash(k.ep, k.key, k.e->slot);
		/* hot slots in use end at next_hot; unused ones below it are free */
		std::vector<uint8_t> hot_used(c->hot_cap, 0);
		for (auto &k : ks)
			if (k.e->slot < c->hot_cap)
				hot_used[k.e->slot] = 1;
		uint32_t nh = 0;
		for (uint32_t sl = 0; sl < c->hot_cap; sl++)
			if (hot_used[sl])
				nh = sl + 1u;
		c->free_hot.clear();
		for (uint32_t sl = nh; sl-- > 0;)
			if (!hot_used[sl])
				c->free_hot.push_back(sl);
		std::sort(cold_free.begin(), cold_free.end(), std::greater<uint32_t>());
		c->free_cold.assign(cold_free.begin(), cold_free.end());
		c->quarantine.clear(); /* the device is idle: no snapshot counts any more */
		c->next_hot = nh;
		c->next_cold = next_cold;
		if (moved) {
			c->dirty |= 1u << G_POL;
			c->pol_full = true;
			c->pol_changes.clear();
		}
	}
	if (moved_out)
		*moved_out = moved;
	return moved ? commit_locked(c, nullptr) : 0;
}

/* SURVEY §5 failure detection: recompute every group buffer of the
 * published snapshot on the device and compare with the host image's sum */
CGPU_EXPORT int cgpu_table_verify(cgpu_ctx *c)
{
	if (!c)
		return fail(-EINVAL, "null argument");
	if (c->device < 0)
		return fail(-ENODEV, "context has no device");
	std::lock_guard<std::mutex> cg(c->commit_mu);
	std::shared_ptr<Epoch> e;
	{
		std::lock_guard<std::mutex> g(c->pub_mu);
		e = c->cur;
	}
	if (!e)
		return fail(-ENOENT, "nothing committed");
	HIP_OR_EIO(hipSetDevice(c->device));
	HIP_OR_EIO(hipMemsetAsync(c->d_verify, 0, (G_N + 1) * 8, c->ustream));
	for (int k = 0; k < G_N; k++)
		if (e->bufs[k])
			for (auto &pt : e->bufs[k]->parts)
				HIP_OR_EIO(launch_table_sum(e->bufs[k]->p, pt.first, pt.second, c->d_verify + k,
							    c->ustream));
	uint64_t got[G_N + 1];
	HIP_OR_EIO(hipMemcpyAsync(got, c->d_verify, sizeof(got), hipMemcpyDeviceToHost, c->ustream));
	HIP_OR_EIO(hipStreamSynchronize(c->ustream));
	static const char *names[G_N] = {"ipcache", "policy", "prefilter", "endpoints", "lb4", "lxc", "lb6"};
	for (int k = 0; k < G_N; k++)
		if (e->bufs[k] && got[k] != e->bufs[k]->host_sum)
			return fail(-EIO, "device %s tables differ from the host image (sum %016llx, expected %016llx)",
				    names[k], (unsigned long long)got[k], (unsigned long long)e->bufs[k]->host_sum);
	return 0;
}

/* TEST HOOK (not in cgpu.h): xor `mask` into byte `off` of group `group`'s
 * device buffer of the published snapshot, so that tests can show
 * cgpu_table_verify catching a corrupted table. */
CGPU_EXPORT int cgpu__test_corrupt(cgpu_ctx *c, int group, size_t off, uint8_t mask)
{
	if (!c || c->device < 0 || group < 0 || group >= G_N)
		return -EINVAL;
	std::shared_ptr<Epoch> e;
	{
		std::lock_guard<std::mutex> g(c->pub_mu);
		e = c->cur;
	}
	if (!e || !e->bufs[group] || off >= e->bufs[group]->bytes)
		return -EINVAL;
	uint8_t b;
	HIP_OR_EIO(hipSetDevice(c->device));
	HIP_OR_EIO(hipDeviceSynchronize());
	HIP_OR_EIO(hipMemcpy(&b, (char *)e->bufs[group]->p + off, 1, hipMemcpyDeviceToHost));
	b ^= mask;
	HIP_OR_EIO(hipMemcpy((char *)e->bufs[group]->p + off, &b, 1, hipMemcpyHostToDevice));
	return 0;
}

CGPU_EXPORT int cgpu_counter_layout_checksum(cgpu_ctx *c, uint64_t *sum)
{
	if (!c || !sum)
		return fail(-EINVAL, "null argument");
	std::lock_guard<std::mutex> g(c->pub_mu);
	if (!c->cur)
		return fail(-ENOENT, "nothing committed");
	*sum = c->slot_checksum;
	return 0;
}

/* ======================================================================= */
/* batch entry points                                                        */
/* ======================================================================= */
/* A launch pins the published snapshot for as long as it enqueues: the
 * stream first waits for the snapshot's uploads, and afterwards an event
 * recorded on it tells the snapshot's retirement when these kernels end.
 * Launches never take the mirror lock, so commits (and table updates) do
 * not block them. */
static const size_t kMaxPkStreams = 16;

struct Pinned {
	std::shared_ptr<Epoch> ep;
	cgpu_ctx *c = nullptr;
	hipStream_t st = nullptr;
	uint64_t *delta = nullptr, *pk = nullptr;
	const cgpu_snapshot &snap() const { return ep->snap; }
	~Pinned()
	{
		if (!ep)
			return;
		if (pk) { /* the stream's packed buffer is free again after this point */
			std::lock_guard<std::mutex> g(c->pk_mu);
			auto it = c->d_pk.find((void *)st);
			if (it != c->d_pk.end() && it->second.p == pk)
				(void)hipEventRecord(it->second.last, st);
		}
		std::lock_guard<std::mutex> g(ep->mu);
		hipEvent_t ev = nullptr;
		for (auto &u : ep->used)
			if (u.first == st)
				ev = u.second;
		if (!ev && hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess)
			ep->used.push_back({st, ev});
		if (ev)
			(void)hipEventRecord(ev, st);
	}
};

static int pin(cgpu_ctx *c, void *stream, Pinned &p, bool want_pk = false)
{
	if (!c)
		return fail(-EINVAL, "null context");
	if (c->device < 0)
		return fail(-ENODEV, "context has no device (host-only); no CPU classification path");
	{
		std::lock_guard<std::mutex> g(c->pub_mu);
		p.ep = c->cur;
	}
	if (!p.ep)
		return fail(-ENOENT, "no committed snapshot (call cgpu_commit)");
	p.st = (hipStream_t)stream;
	p.c = c;
	HIP_OR_EIO(hipSetDevice(c->device));
	HIP_OR_EIO(hipStreamWaitEvent(p.st, p.ep->ready, 0));
	std::lock_guard<std::mutex> g(c->pk_mu);
	p.delta = c->d_delta;
	if (want_pk) {
		auto it = c->d_pk.find(stream);
		if (it == c->d_pk.end()) {
			cgpu_ctx::PkBuf b;
			if (c->d_pk.size() >= kMaxPkStreams) {
				/* recycle the least recently used stream's buffer: zero again
				 * once that stream's last launch (its unpack) finished */
				auto lru = c->d_pk.begin();
				for (auto j = c->d_pk.begin(); j != c->d_pk.end(); ++j)
					if (j->second.tick < lru->second.tick)
						lru = j;
				HIP_OR_EIO(hipEventSynchronize(lru->second.last));
				b = lru->second;
				c->d_pk.erase(lru);
			} else {
				const size_t bytes = (size_t)c->n_ctr_slots * 8;
				HIP_OR_EIO(hipMalloc((void **)&b.p, bytes));
				if (hipMemset(b.p, 0, bytes) != hipSuccess ||
				    hipEventCreateWithFlags(&b.last, hipEventDisableTiming) != hipSuccess) {
					(void)hipFree(b.p);
					return fail(-EIO, "packed counter buffer init failed");
				}
			}
			it = c->d_pk.emplace(stream, b).first;
		}
		it->second.tick = ++c->pk_tick;
		p.pk = it->second.p;
	}
	return 0;
}

CGPU_EXPORT int cgpu_stream_release(cgpu_ctx *c, void *stream)
{
	if (!c)
		return fail(-EINVAL, "null context");
	if (c->device < 0)
		return 0;
	std::lock_guard<std::mutex> g(c->pk_mu);
	auto it = c->d_pk.find(stream);
	if (it == c->d_pk.end())
		return 0;
	HIP_OR_EIO(hipSetDevice(c->device));
	HIP_OR_EIO(hipEventSynchronize(it->second.last));
	(void)hipFree(it->second.p);
	(void)hipEventDestroy(it->second.last);
	c->d_pk.erase(it);
	return 0;
}

CGPU_EXPORT int cgpu_classify_v4(cgpu_ctx *c, const cgpu_tuples_v4 *t, size_t n, int32_t *verdict,
				 uint32_t *identity, uint8_t *stage, void *stream)
{
	Pinned P;
	if (int r = pin(c, stream, P, true))
		return r;
	const cgpu_snapshot &s = P.snap();
	uint64_t *delta = P.delta, *pk = P.pk;
	if (!t || (n && (!t->saddr || !t->daddr || !t->dport || !t->proto || !t->flags || !t->len ||
			 !t->ep || !verdict || !identity)))
		return fail(-EINVAL, "null tuple column or output");
	if (!n)
		return 0;
	classify_v4_args a{t->saddr, t->daddr, t->dport, t->proto, t->flags, t->len, t->ep,
			   verdict, identity, stage, delta, (uint64_t)n, pk, 0, nullptr, nullptr};
	HIP_OR_EIO(hipSetDevice(c->device));
	HIP_OR_EIO(launch_classify_v4(s, a, (hipStream_t)stream));
	return 0;
}

/* ---- host-resident batches (host or device pointers) ----
 * The batch streams through device staging buffers of one chunk each:
 * chunk k's columns go up on the h2d stream, its classify runs on the
 * caller's stream, its outputs come back on the d2h stream, so chunk k + 1's
 * upload and chunk k - 1's download overlap chunk k's classify. */
/* tuples per staging chunk: 8M (4M: tuples 2.45 -> 2.52 Gpps, frames 0.68 ->
 * 0.71, v6 1.10 -> 1.20; 16M 2.49, profiles/r6_m/host_ab_chunk*.log) */
#ifndef CGPU_HS_CHUNK_LOG2
#define CGPU_HS_CHUNK_LOG2 23
#endif
#define HS_CHUNK (1u << CGPU_HS_CHUNK_LOG2)
#define HS_NBUF 16
/* one staging pair holds HS_CHUNK v4 tuples (18 B in, 9 B out) in
 * 256-aligned columns; a wider tuple (frames) takes fewer per chunk */
#define HS_IN_BYTES ((size_t)HS_CHUNK * 18 + 8 * 256)
#define HS_OUT_BYTES ((size_t)HS_CHUNK * 9 + 4 * 256)
/* uploads of a batch whose columns are all narrower than this many bytes
 * per tuple go by the runtime's DMA copies, the others (64-byte frame
 * slots) by the CUs: tuples 2.15 -> 2.37 Gpps, v6 1.00 -> 1.08, pf6 1.56 ->
 * 1.64, frames 0.68 -> 0.59 with DMA uploads (profiles/r6_m/) */
#ifndef CGPU_HS_UP_DMA_BELOW
#define CGPU_HS_UP_DMA_BELOW 64
#endif
#ifndef CGPU_HS_STORE
#define CGPU_HS_STORE 1
#endif

/* a host batch: its input and output columns and their bytes per tuple */
struct hs_cols {
	int nin = 0, nout = 0;
	const uint8_t *in[8] = {};
	size_t in_el[8] = {};
	uint8_t *out[8] = {}; /* null: output not requested */
	size_t out_el[8] = {};
};

static size_t hs_off(const size_t *el, size_t m, int col)
{
	size_t o = 0;
	for (int k = 0; k < col; k++)
		o += (m * el[k] + 255) & ~(size_t)255;
	return o;
}

/* tuples per chunk: what one staging pair holds, a multiple of 4096 (so
 * every column of chunk k starts 16-byte aligned in the caller's buffers
 * whenever the column does) */
static size_t hs_chunk(const hs_cols &C)
{
	size_t pin = 0, pout = 0;
	for (int k = 0; k < C.nin; k++)
		pin += C.in_el[k];
	for (int k = 0; k < C.nout; k++)
		pout += C.out_el[k];
	size_t m = HS_CHUNK;
	m = std::min(m, (HS_IN_BYTES - (size_t)256 * C.nin) / std::max<size_t>(pin, 1));
	m = std::min(m, (HS_OUT_BYTES - (size_t)256 * C.nout) / std::max<size_t>(pout, 1));
	return m & ~(size_t)4095;
}

/* grow the staging to min(nch, HS_NBUF) buffers.  A failed allocation rolls
 * back that buffer; the call then runs on the buffers it has (any number >= 1
 * is correct: chunk k uses buffer k % nb). */
static int host_stage_init(cgpu_ctx *c, size_t nch)
{
	auto &H = c->hs;
	if (!H.h2d) {
		/* the copy streams in priority classes of their own, non-blocking:
		 * the runtime spreads plain streams over the process's few hardware
		 * queues round robin, and an upload stream that landed on the
		 * caller's queue serialised every chunk's classify behind all queued
		 * uploads (profiles/r4_ah); queues are pooled per priority */
		int least = 0, greatest = 0;
		HIP_OR_EIO(hipDeviceGetStreamPriorityRange(&least, &greatest));
		HIP_OR_EIO(hipStreamCreateWithPriority(&H.h2d, hipStreamNonBlocking, greatest));
		if (hipStreamCreateWithPriority(&H.d2h, hipStreamNonBlocking, least) != hipSuccess) {
			(void)hipGetLastError();
			(void)hipStreamDestroy(H.h2d);
			H.h2d = nullptr;
			return fail(-EIO, "host staging stream creation failed");
		}
	}
	const int want = (int)std::min<size_t>(nch, HS_NBUF);
	while (H.nb < want) {
		void *in = nullptr, *out = nullptr;
		hipEvent_t ev[3] = {};
		bool ok = hipMalloc(&in, HS_IN_BYTES) == hipSuccess && hipMalloc(&out, HS_OUT_BYTES) == hipSuccess;
		for (int k = 0; ok && k < 3; k++)
			ok = hipEventCreateWithFlags(&ev[k], hipEventDisableTiming) == hipSuccess;
		if (!ok) {
			(void)hipGetLastError();
			(void)hipFree(in);
			(void)hipFree(out);
			for (hipEvent_t e : ev)
				if (e)
					(void)hipEventDestroy(e);
			if (H.nb)
				break;
			return fail(-ENOMEM, "host staging allocation failed");
		}
		const int b = H.nb++;
		H.d_in[b] = in;
		H.d_out[b] = out;
		H.ev_in[b] = ev[0];
		H.ev_cls[b] = ev[1];
		H.ev_out[b] = ev[2];
	}
	return 0;
}

/* the device address of a page-locked host range [p, p + bytes), or null
 * when the range is not page-locked host memory the device maps (both ends
 * checked) */
static void *host_mapped(const void *p, size_t bytes)
{
	if (!p || !bytes)
		return nullptr;
	hipPointerAttribute_t a0{}, a1{};
	const char *last = static_cast<const char *>(p) + bytes - 1;
	if (hipPointerGetAttributes(&a0, p) != hipSuccess || hipPointerGetAttributes(&a1, last) != hipSuccess) {
		(void)hipGetLastError();
		return nullptr;
	}
	if (a0.type != hipMemoryTypeHost || a1.type != hipMemoryTypeHost || !a0.devicePointer ||
	    static_cast<char *>(a1.devicePointer) != static_cast<char *>(a0.devicePointer) + bytes - 1)
		return nullptr;
	return a0.devicePointer;
}

/* The pipeline of a host batch.  classify(m, din, dout) enqueues one chunk's
 * work on cs over device columns.  Page-locked, mapped output columns are
 * written by the CUs, all columns of a chunk in one launch (a DMA download
 * ran at a quarter of the link rate beside the uploads, profiles/r4_ah);
 * mapped input columns are read by the CUs too when one of them is a 64-byte
 * frame slot, else uploaded by the runtime's DMA copies (CGPU_HS_UP_DMA_BELOW);
 * columns that are not page-locked are copied by the runtime.
 * Called with host_mu held. */
template <typename F>
static int host_pipeline(cgpu_ctx *c, size_t n, const hs_cols &C, hipStream_t cs, F &&classify)
{
	auto &H = c->hs;
	const size_t chunk = hs_chunk(C);
	if (!chunk)
		return fail(-EINVAL, "tuple too wide for the host staging");
	const size_t nch = (n + chunk - 1) / chunk;
	if (int r = host_stage_init(c, nch))
		return r;
	const size_t nb = (size_t)H.nb;
	/* after an error past the first enqueue, every copy already queued still
	 * reads or writes the caller's buffers: wait for them before returning */
	struct Drain {
		cgpu_ctx *c;
		bool armed = false;
		~Drain()
		{
			if (armed) {
				(void)hipStreamSynchronize(c->hs.h2d);
				(void)hipStreamSynchronize(c->hs.d2h);
			}
		}
	} drain{c};
	const uint8_t *src_dev[8] = {};
	uint8_t *dst_dev[8] = {};
	for (int k = 0; k < C.nin; k++)
		src_dev[k] = static_cast<const uint8_t *>(host_mapped(C.in[k], n * C.in_el[k]));
	for (int k = 0; k < C.nout; k++)
		dst_dev[k] = C.out[k] ? static_cast<uint8_t *>(host_mapped(C.out[k], n * C.out_el[k])) : nullptr;
	auto aligned = [](const void *p) { return !(reinterpret_cast<uintptr_t>(p) & 15u); };
	size_t widest = 0;
	for (int k = 0; k < C.nin; k++)
		widest = std::max(widest, C.in_el[k]);
	const bool dma_up = widest < CGPU_HS_UP_DMA_BELOW;
	/* one launch for the mapped columns; the others (and, should the launch
	 * fail, those too) by the runtime's copy on the same stream */
	auto move = [&](hipStream_t st, hipMemcpyKind kind, int ncol, void *const *dst, const void *const *src,
			void *const *dst_mapped, const void *const *src_mapped, const size_t *bytes) -> int {
		copy_segs d{};
		int which[8];
		for (int col = 0; col < ncol; col++) {
			if (!bytes[col])
				continue;
			void *dd = dst_mapped ? dst_mapped[col] : dst[col];
			const void *ss = src_mapped ? src_mapped[col] : src[col];
			const bool by_cu = kind == hipMemcpyDeviceToHost || !dma_up;
			if (CGPU_HS_STORE && by_cu && dd && ss && aligned(dd) && aligned(ss)) {
				which[d.n] = col;
				d.seg[d.n++] = copy_seg{dd, ss, bytes[col]};
				continue;
			}
			HIP_OR_EIO(hipMemcpyAsync(dst[col], src[col], bytes[col], kind, st));
		}
		if (d.n && launch_copy_host_multi(d, st) != hipSuccess) {
			(void)hipGetLastError();
			for (uint32_t j = 0; j < d.n; j++)
				HIP_OR_EIO(hipMemcpyAsync(dst[which[j]], src[which[j]], bytes[which[j]], kind, st));
		}
		return 0;
	};
	/* chunk k's columns up on the h2d stream into buffer k % nb, free once
	 * that buffer's last classify ran (in this call or an earlier one; an
	 * event never recorded is no wait) */
	auto upload = [&](size_t k) -> int {
		const size_t off = k * chunk, m = std::min(chunk, n - off), b = k % nb;
		uint8_t *in = static_cast<uint8_t *>(H.d_in[b]);
		HIP_OR_EIO(hipStreamWaitEvent(H.h2d, H.ev_cls[b], 0));
		void *dst[8];
		const void *src[8], *src_m[8];
		size_t bytes[8];
		for (int col = 0; col < C.nin; col++) {
			dst[col] = in + hs_off(C.in_el, m, col);
			src[col] = C.in[col] + off * C.in_el[col];
			src_m[col] = src_dev[col] ? src_dev[col] + off * C.in_el[col] : nullptr;
			bytes[col] = m * C.in_el[col];
		}
		drain.armed = true;
		if (int r = move(H.h2d, hipMemcpyHostToDevice, C.nin, dst, src, nullptr, src_m, bytes))
			return r;
		HIP_OR_EIO(hipEventRecord(H.ev_in[b], H.h2d));
		return 0;
	};
	/* every upload that has a buffer of its own is queued first, so the
	 * h2d stream runs back to back (the runtime resolves a copy's wait on
	 * another stream's event on the issuing thread: an upload queued behind
	 * a download's wait on a classify stalled until that classify ended,
	 * profiles/r4_ah); past nb chunks, chunk k + nb goes up once chunk k's
	 * classify is queued */
	for (size_t k = 0; k < std::min(nch, nb); k++)
		if (int r = upload(k))
			return r;
	for (size_t k = 0; k < nch; k++) {
		const size_t off = k * chunk, m = std::min(chunk, n - off), b = k % nb;
		uint8_t *in = static_cast<uint8_t *>(H.d_in[b]), *out = static_cast<uint8_t *>(H.d_out[b]);
		/* classify on the caller's stream once the columns landed and the
		 * output buffer drained (its last download) */
		HIP_OR_EIO(hipStreamWaitEvent(cs, H.ev_in[b], 0));
		HIP_OR_EIO(hipStreamWaitEvent(cs, H.ev_out[b], 0));
		uint8_t *din[8], *dout[8];
		for (int col = 0; col < C.nin; col++)
			din[col] = in + hs_off(C.in_el, m, col);
		for (int col = 0; col < C.nout; col++)
			dout[col] = C.out[col] ? out + hs_off(C.out_el, m, col) : nullptr;
		if (int r = classify(m, din, dout))
			return r;
		HIP_OR_EIO(hipEventRecord(H.ev_cls[b], cs));
		if (k + nb < nch)
			if (int r = upload(k + nb))
				return r;
		HIP_OR_EIO(hipStreamWaitEvent(H.d2h, H.ev_cls[b], 0));
		void *dst[8], *dst_m[8];
		const void *src[8];
		size_t bytes[8];
		for (int col = 0; col < C.nout; col++) {
			dst[col] = C.out[col] ? C.out[col] + off * C.out_el[col] : nullptr;
			dst_m[col] = dst_dev[col] ? dst_dev[col] + off * C.out_el[col] : nullptr;
			src[col] = dout[col];
			bytes[col] = C.out[col] ? m * C.out_el[col] : 0;
		}
		if (int r = move(H.d2h, hipMemcpyDeviceToHost, C.nout, dst, src, dst_m, nullptr, bytes))
			return r;
		HIP_OR_EIO(hipEventRecord(H.ev_out[b], H.d2h));
	}
	/* the caller's stream completes once the last outputs are in host memory */
	for (size_t b = 0; b < nb && b < nch; b++)
		HIP_OR_EIO(hipStreamWaitEvent(cs, H.ev_out[b], 0));
	drain.armed = false;
	return 0;
}

/* the host-resident v4 paths: plain (lb 0), service-translated (lb 1) and
 * the XDP prefilter cascade (lb 1, xdp 1); the service paths upload the hash
 * column when there is one (it wins over sport in the kernel), else sport */
static int v4_host(cgpu_ctx *c, const cgpu_tuples_v4 *t, const uint16_t *sport, const uint32_t *hash, size_t n,
		   int32_t *verdict, uint32_t *identity, uint8_t *stage, void *stream, int lb, int xdp)
{
	if (!c)
		return fail(-EINVAL, "null context");
	if (!t || (n && (!t->saddr || !t->daddr || !t->dport || !t->proto || !t->flags || !t->len ||
			 !t->ep || !verdict || !identity)))
		return fail(-EINVAL, "null tuple column or output");
	if (lb && n && !hash && !sport)
		return fail(-EINVAL, "either a hash or an sport column is needed");
	if (c->device < 0)
		return fail(-ENODEV, "context has no device (host-only); no CPU path");
	if (!n)
		return 0;
	std::lock_guard<std::mutex> g(c->host_mu);
	/* ONE snapshot and one packed-counter buffer for the whole batch: a
	 * commit from another thread between chunks cannot split it */
	Pinned P;
	if (int r = pin(c, stream, P, true))
		return r;
	const cgpu_snapshot &s = P.snap();
	const hipStream_t cs = (hipStream_t)stream;
	hs_cols C;
	C.nin = 7;
	const void *cols[7] = {t->saddr, t->daddr, t->dport, t->proto, t->flags, t->len, t->ep};
	static const size_t el[7] = {4, 4, 2, 1, 1, 4, 2};
	for (int k = 0; k < 7; k++) {
		C.in[k] = static_cast<const uint8_t *>(cols[k]);
		C.in_el[k] = el[k];
	}
	if (lb) {
		C.in[7] = hash ? reinterpret_cast<const uint8_t *>(hash) : reinterpret_cast<const uint8_t *>(sport);
		C.in_el[7] = hash ? 4 : 2;
		C.nin = 8;
	}
	C.nout = 3;
	C.out[0] = reinterpret_cast<uint8_t *>(verdict);
	C.out[1] = reinterpret_cast<uint8_t *>(identity);
	C.out[2] = stage;
	C.out_el[0] = C.out_el[1] = 4;
	C.out_el[2] = 1;
	return host_pipeline(c, n, C, cs, [&](size_t m, uint8_t *const *di, uint8_t *const *dout) -> int {
		classify_v4_args a{reinterpret_cast<const uint32_t *>(di[0]), reinterpret_cast<const uint32_t *>(di[1]),
				   reinterpret_cast<const uint16_t *>(di[2]), di[3], di[4],
				   reinterpret_cast<const uint32_t *>(di[5]), reinterpret_cast<const uint16_t *>(di[6]),
				   reinterpret_cast<int32_t *>(dout[0]), reinterpret_cast<uint32_t *>(dout[1]), dout[2],
				   P.delta, (uint64_t)m, P.pk, 0, nullptr, nullptr};
		if (lb) {
			a.lb = 1;
			a.xdp = xdp;
			if (hash)
				a.hash = reinterpret_cast<const uint32_t *>(di[7]);
			else
				a.sport = reinterpret_cast<const uint16_t *>(di[7]);
		}
		HIP_OR_EIO(launch_classify_v4(s, a, cs));
		return 0;
	});
}

CGPU_EXPORT int cgpu_classify_v4_host(cgpu_ctx *c, const cgpu_tuples_v4 *t, size_t n, int32_t *verdict,
				      uint32_t *identity, uint8_t *stage, void *stream)
{
	return v4_host(c, t, nullptr, nullptr, n, verdict, identity, stage, stream, 0, 0);
}

CGPU_EXPORT int cgpu_classify_v4_lb_host(cgpu_ctx *c, const cgpu_tuples_v4 *t, const uint16_t *sport,
					 const uint32_t *hash, size_t n, int32_t *verdict, uint32_t *identity,
					 uint8_t *stage, void *stream)
{
	return v4_host(c, t, sport, hash, n, verdict, identity, stage, stream, 1, 0);
}

CGPU_EXPORT int cgpu_classify_v4_cascade_host(cgpu_ctx *c, const cgpu_tuples_v4 *t, const uint16_t *sport,
					      const uint32_t *hash, size_t n, int32_t *verdict, uint32_t *identity,
					      uint8_t *stage, void *stream)
{
	return v4_host(c, t, sport, hash, n, verdict, identity, stage, stream, 1, 1);
}

CGPU_EXPORT int cgpu_host_stage_release(cgpu_ctx *c)
{
	if (!c)
		return fail(-EINVAL, "null context");
	if (c->device < 0)
		return 0;
	std::lock_guard<std::mutex> g(c->host_mu);
	HIP_OR_EIO(hipSetDevice(c->device));
	host_stage_free(c);
	return 0;
}

CGPU_EXPORT size_t cgpu_host_stage_bytes(cgpu_ctx *c)
{
	if (!c)
		return 0;
	std::lock_guard<std::mutex> g(c->host_mu);
	return (size_t)c->hs.nb * (HS_IN_BYTES + HS_OUT_BYTES);
}

CGPU_EXPORT int cgpu_classify_v4_lb(cgpu_ctx *c, const cgpu_tuples_v4 *t, const uint16_t *sport,
				    const uint32_t *hash, size_t n, int32_t *verdict, uint32_t *identity,
				    uint8_t *stage, void *stream)
{
	Pinned P;
	if (int r = pin(c, stream, P, true))
		return r;
	const cgpu_snapshot &s = P.snap();
	uint64_t *delta = P.delta, *pk = P.pk;
	if (!t || (n && (!t->saddr || !t->daddr || !t->dport || !t->proto || !t->flags || !t->len ||
			 !t->ep || !verdict || !identity)))
		return fail(-EINVAL, "null tuple column or output");
	if (n && !hash && !sport)
		return fail(-EINVAL, "either a hash or an sport column is needed");
	if (!n)
		return 0;
	classify_v4_args a{t->saddr, t->daddr, t->dport, t->proto, t->flags, t->len, t->ep,
			   verdict, identity, stage, delta, (uint64_t)n, pk};
	a.lb = 1;
	a.sport = sport;
	a.hash = hash;
	HIP_OR_EIO(hipSetDevice(c->device));
	HIP_OR_EIO(launch_classify_v4(s, a, (hipStream_t)stream));
	return 0;
}

CGPU_EXPORT int cgpu_classify_v4_cascade(cgpu_ctx *c, const cgpu_tuples_v4 *t, const uint16_t *sport,
					 const uint32_t *hash, size_t n, int32_t *verdict, uint32_t *identity,
					 uint8_t *stage, void *stream)
{
	Pinned P;
	if (int r = pin(c, stream, P, true))
		return r;
	const cgpu_snapshot &s = P.snap();
	uint64_t *delta = P.delta, *pk = P.pk;
	if (!t || (n && (!t->saddr || !t->daddr || !t->dport || !t->proto || !t->flags || !t->len ||
			 !t->ep || !verdict || !identity)))
		return fail(-EINVAL, "null tuple column or output");
	if (n && !hash && !sport)
		return fail(-EINVAL, "either a hash or an sport column is needed");
	if (!n)
		return 0;
	classify_v4_args a{t->saddr, t->daddr, t->dport, t->proto, t->flags, t->len, t->ep,
			   verdict, identity, stage, delta, (uint64_t)n, pk};
	a.lb = 1;
	a.xdp = 1;
	a.sport = sport;
	a.hash = hash;
	HIP_OR_EIO(hipSetDevice(c->device));
	HIP_OR_EIO(launch_classify_v4(s, a, (hipStream_t)stream));
	return 0;
}

CGPU_EXPORT int cgpu_lb4_select(cgpu_ctx *c, int mode, const cgpu_lb4_tuples *t, size_t n,
				const cgpu_lb4_out *out, void *stream)
{
	Pinned P;
	if (int r = pin(c, stream, P))
		return r;
	const cgpu_snapshot &s = P.snap();
	if (mode != CGPU_LB_NETDEV && mode != CGPU_LB_LXC)
		return fail(-EINVAL, "bad lb mode %d", mode);
	if (!t || !out || (n && (!t->saddr || !t->daddr || !t->dport || !t->proto || !out->ret)))
		return fail(-EINVAL, "null tuple column or output");
	if (n && !t->hash && !t->sport)
		return fail(-EINVAL, "either a hash or an sport column is needed");
	if (!n)
		return 0;
	lb4_args a{t->saddr, t->daddr, t->sport, t->dport, t->proto, t->hash, out->ret, out->saddr,
		   out->daddr, out->dport, out->rev_nat, out->slave, (uint64_t)n, mode};
	HIP_OR_EIO(hipSetDevice(c->device));
	HIP_OR_EIO(launch_lb4(s, a, (hipStream_t)stream));
	return 0;
}

CGPU_EXPORT int cgpu_classify_v6(cgpu_ctx *c, const cgpu_tuples_v6 *t, size_t n, int32_t *verdict,
				 uint32_t *identity, uint8_t *stage, void *stream)
{
	Pinned P;
	if (int r = pin(c, stream, P, true))
		return r;
	const cgpu_snapshot &s = P.snap();
	uint64_t *delta = P.delta, *pk = P.pk;
	if (!t || (n && (!t->saddr || !t->daddr || !t->dport || !t->proto || !t->flags || !t->len ||
			 !t->ep || !verdict || !identity)))
		return fail(-EINVAL, "null tuple column or output");
	if (((uintptr_t)t->saddr | (uintptr_t)t->daddr) & 15)
		return fail(-EINVAL, "v6 address columns must be 16-byte aligned");
	if (!n)
		return 0;
	classify_v6_args a{t->saddr, t->daddr, t->dport, t->proto, t->flags, t->len, t->ep,
			   verdict, identity, stage, delta, (uint64_t)n, pk};
	HIP_OR_EIO(hipSetDevice(c->device));
	/* the x4 schedule's ipcache pre-pass: n entries of stream-ordered pool
	 * scratch */
	void *scr = nullptr;
	/* (the pre-pass folds the egress fallback identity into a DIRECT entry
	 * of cluster_id: its payload must hold it) */
	if (s.ipc6.root && !(s.schedule & (CGPU_SCHED_PER_LANE | CGPU_SCHED_GLOBAL_CTR)) &&
	    s.cluster_id && s.cluster_id <= DIR_PAYLOAD_MASK)
		HIP_OR_EIO(hipMallocFromPoolAsync(&scr, (size_t)n * 4u, c->pool, (hipStream_t)stream));
	a.ipc_e = static_cast<uint32_t *>(scr);
	const hipError_t le = launch_classify_v6(s, a, (hipStream_t)stream);
	if (scr)
		HIP_OR_EIO(hipFreeAsync(scr, (hipStream_t)stream));
	HIP_OR_EIO(le);
	return 0;
}

CGPU_EXPORT int cgpu_classify_v6_lb(cgpu_ctx *c, const cgpu_tuples_v6 *t, const uint16_t *sport,
				    const uint32_t *hash, size_t n, int32_t *verdict, uint32_t *identity,
				    uint8_t *stage, void *stream)
{
	Pinned P;
	if (int r = pin(c, stream, P, true))
		return r;
	const cgpu_snapshot &s = P.snap();
	uint64_t *delta = P.delta, *pk = P.pk;
	if (!t || (n && (!t->saddr || !t->daddr || !t->dport || !t->proto || !t->flags || !t->len ||
			 !t->ep || !verdict || !identity)))
		return fail(-EINVAL, "null tuple column or output");
	if (((uintptr_t)t->saddr | (uintptr_t)t->daddr) & 15)
		return fail(-EINVAL, "v6 address columns must be 16-byte aligned");
	if (n && !hash && !sport)
		return fail(-EINVAL, "either a hash or an sport column is needed");
	if (!n)
		return 0;
	classify_v6_args a{t->saddr, t->daddr, t->dport, t->proto, t->flags, t->len, t->ep,
			   verdict, identity, stage, delta, (uint64_t)n, pk};
	a.lb = 1;
	a.sport = sport;
	a.hash = hash;
	HIP_OR_EIO(hipSetDevice(c->device));
	HIP_OR_EIO(launch_classify_v6(s, a, (hipStream_t)stream));
	return 0;
}


/* the host-resident v6 paths (plain and service-translated): 42 B of
 * columns per tuple in, the x4 pre-pass scratch per chunk from the pool */
static int v6_host(cgpu_ctx *c, const cgpu_tuples_v6 *t, const uint16_t *sport, const uint32_t *hash, size_t n,
		   int32_t *verdict, uint32_t *identity, uint8_t *stage, void *stream, int lb)
{
	if (!c)
		return fail(-EINVAL, "null context");
	if (!t || (n && (!t->saddr || !t->daddr || !t->dport || !t->proto || !t->flags || !t->len ||
			 !t->ep || !verdict || !identity)))
		return fail(-EINVAL, "null tuple column or output");
	if (lb && n && !hash && !sport)
		return fail(-EINVAL, "either a hash or an sport column is needed");
	if (c->device < 0)
		return fail(-ENODEV, "context has no device (host-only); no CPU path");
	if (!n)
		return 0;
	std::lock_guard<std::mutex> g(c->host_mu);
	Pinned P;
	if (int r = pin(c, stream, P, true))
		return r;
	const cgpu_snapshot &s = P.snap();
	const hipStream_t cs = (hipStream_t)stream;
	hs_cols C;
	C.nin = 7;
	const void *cols[7] = {t->saddr, t->daddr, t->dport, t->proto, t->flags, t->len, t->ep};
	static const size_t el[7] = {16, 16, 2, 1, 1, 4, 2};
	for (int k = 0; k < 7; k++) {
		C.in[k] = static_cast<const uint8_t *>(cols[k]);
		C.in_el[k] = el[k];
	}
	if (lb) {
		C.in[7] = hash ? reinterpret_cast<const uint8_t *>(hash) : reinterpret_cast<const uint8_t *>(sport);
		C.in_el[7] = hash ? 4 : 2;
		C.nin = 8;
	}
	C.nout = 3;
	C.out[0] = reinterpret_cast<uint8_t *>(verdict);
	C.out[1] = reinterpret_cast<uint8_t *>(identity);
	C.out[2] = stage;
	C.out_el[0] = C.out_el[1] = 4;
	C.out_el[2] = 1;
	const bool pre = !lb && s.ipc6.root && !(s.schedule & (CGPU_SCHED_PER_LANE | CGPU_SCHED_GLOBAL_CTR)) &&
			 s.cluster_id && s.cluster_id <= DIR_PAYLOAD_MASK;
	return host_pipeline(c, n, C, cs, [&](size_t m, uint8_t *const *di, uint8_t *const *dout) -> int {
		classify_v6_args a{di[0], di[1], reinterpret_cast<const uint16_t *>(di[2]), di[3], di[4],
				   reinterpret_cast<const uint32_t *>(di[5]), reinterpret_cast<const uint16_t *>(di[6]),
				   reinterpret_cast<int32_t *>(dout[0]), reinterpret_cast<uint32_t *>(dout[1]), dout[2],
				   P.delta, (uint64_t)m, P.pk};
		if (lb) {
			a.lb = 1;
			if (hash)
				a.hash = reinterpret_cast<const uint32_t *>(di[7]);
			else
				a.sport = reinterpret_cast<const uint16_t *>(di[7]);
		}
		void *scr = nullptr;
		if (pre)
			HIP_OR_EIO(hipMallocFromPoolAsync(&scr, m * 4u, c->pool, cs));
		a.ipc_e = static_cast<uint32_t *>(scr);
		const hipError_t le = launch_classify_v6(s, a, cs);
		if (scr)
			HIP_OR_EIO(hipFreeAsync(scr, cs));
		HIP_OR_EIO(le);
		return 0;
	});
}

CGPU_EXPORT int cgpu_classify_v6_host(cgpu_ctx *c, const cgpu_tuples_v6 *t, size_t n, int32_t *verdict,
				      uint32_t *identity, uint8_t *stage, void *stream)
{
	return v6_host(c, t, nullptr, nullptr, n, verdict, identity, stage, stream, 0);
}

CGPU_EXPORT int cgpu_classify_v6_lb_host(cgpu_ctx *c, const cgpu_tuples_v6 *t, const uint16_t *sport,
					 const uint32_t *hash, size_t n, int32_t *verdict, uint32_t *identity,
					 uint8_t *stage, void *stream)
{
	return v6_host(c, t, sport, hash, n, verdict, identity, stage, stream, 1);
}


static int frames_check(cgpu_ctx *c, const cgpu_frames *f, size_t n)
{
	if (!f || (n && (!f->data || !f->len || !f->flags || !f->ep)))
		return fail(-EINVAL, "null frame column");
	if (f->stride < 64 || (f->stride & 15))
		return fail(-EINVAL, "frame stride must be a multiple of 16 and >= 64");
	if ((uintptr_t)f->data & 15)
		return fail(-EINVAL, "frame buffer must be 16-byte aligned");
	return 0;
}

CGPU_EXPORT int cgpu_frames_parse(cgpu_ctx *c, const cgpu_frames *f, size_t n,
				  const cgpu_frame_tuples *o, void *stream)
{
	Pinned P;
	if (int r = pin(c, stream, P))
		return r;
	const cgpu_snapshot &s = P.snap();
	if (int r = frames_check(c, f, n))
		return r;
	if (!o || (n && !o->status))
		return fail(-EINVAL, "null status output");
	if (!n)
		return 0;
	frames_args a{f->data, f->len, f->flags, f->ep, f->stride, (uint64_t)n,
		      o->status, o->family, o->saddr, o->daddr, o->dport, o->proto, o->flags,
		      nullptr, nullptr, nullptr, nullptr};
	HIP_OR_EIO(hipSetDevice(c->device));
	HIP_OR_EIO(launch_frames_parse(s, a, (hipStream_t)stream));
	return 0;
}

/* cgpu_classify_frames' launches on a pinned snapshot (device columns) */
static int frames_enqueue(cgpu_ctx *c, const cgpu_snapshot &s, uint64_t *delta, uint64_t *pk,
			  const cgpu_frames *f, size_t n, int32_t *verdict, uint32_t *identity, uint8_t *stage,
			  hipStream_t st)
{
	frames_args a{f->data, f->len, f->flags, f->ep, f->stride, (uint64_t)n,
		      nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
		      verdict, identity, stage, delta, pk};
	const bool x4 = !(s.schedule & (CGPU_SCHED_PER_LANE | CGPU_SCHED_GLOBAL_CTR)) &&
			!(((uintptr_t)f->len | (uintptr_t)verdict | (uintptr_t)identity) & 15) &&
			!((uintptr_t)f->ep & 7) && !((uintptr_t)stage & 3);
	if (!x4) {
		HIP_OR_EIO(launch_classify_frames(s, a, st));
		return 0;
	}
	/* the parsed columns: stream-ordered scratch from the context's memory
	 * pool (which keeps freed memory for the next call, cgpu_ctx_create) */
	void *scr = nullptr;
	HIP_OR_EIO(hipMallocFromPoolAsync(&scr, frames_x4_bytes(n), c->pool, st));
	const hipError_t e = launch_classify_frames_x4(s, a, frames_x4_carve(scr, n), st);
	HIP_OR_EIO(hipFreeAsync(scr, st));
	HIP_OR_EIO(e);
	return 0;
}

CGPU_EXPORT int cgpu_classify_frames(cgpu_ctx *c, const cgpu_frames *f, size_t n, int32_t *verdict,
				     uint32_t *identity, uint8_t *stage, void *stream)
{
	Pinned P;
	if (int r = pin(c, stream, P, true))
		return r;
	if (int r = frames_check(c, f, n))
		return r;
	if (n && (!verdict || !identity))
		return fail(-EINVAL, "null output");
	if (!n)
		return 0;
	HIP_OR_EIO(hipSetDevice(c->device));
	return frames_enqueue(c, P.snap(), P.delta, P.pk, f, n, verdict, identity, stage, (hipStream_t)stream);
}

CGPU_EXPORT int cgpu_classify_frames_host(cgpu_ctx *c, const cgpu_frames *f, size_t n, int32_t *verdict,
					  uint32_t *identity, uint8_t *stage, void *stream)
{
	if (!c)
		return fail(-EINVAL, "null context");
	if (int r = frames_check(c, f, n))
		return r;
	if (n && (!verdict || !identity))
		return fail(-EINVAL, "null output");
	if (c->device < 0)
		return fail(-ENODEV, "context has no device (host-only); no CPU path");
	if (!n)
		return 0;
	std::lock_guard<std::mutex> g(c->host_mu);
	Pinned P;
	if (int r = pin(c, stream, P, true))
		return r;
	const cgpu_snapshot &s = P.snap();
	const hipStream_t cs = (hipStream_t)stream;
	hs_cols C;
	C.nin = 4;
	C.in[0] = f->data;
	C.in_el[0] = f->stride;
	C.in[1] = reinterpret_cast<const uint8_t *>(f->len);
	C.in_el[1] = 4;
	C.in[2] = f->flags;
	C.in_el[2] = 1;
	C.in[3] = reinterpret_cast<const uint8_t *>(f->ep);
	C.in_el[3] = 2;
	C.nout = 3;
	C.out[0] = reinterpret_cast<uint8_t *>(verdict);
	C.out[1] = reinterpret_cast<uint8_t *>(identity);
	C.out[2] = stage;
	C.out_el[0] = C.out_el[1] = 4;
	C.out_el[2] = 1;
	return host_pipeline(c, n, C, cs, [&](size_t m, uint8_t *const *di, uint8_t *const *dout) -> int {
		const cgpu_frames df{di[0], reinterpret_cast<const uint32_t *>(di[1]), di[2],
				     reinterpret_cast<const uint16_t *>(di[3]), f->stride, 0};
		return frames_enqueue(c, s, P.delta, P.pk, &df, m, reinterpret_cast<int32_t *>(dout[0]),
				      reinterpret_cast<uint32_t *>(dout[1]), dout[2], cs);
	});
}

CGPU_EXPORT int cgpu_prefilter_v4(cgpu_ctx *c, const uint32_t *saddr, const uint32_t *daddr,
				  const uint8_t *flags, size_t n, uint8_t *verdict, void *stream)
{
	Pinned P;
	if (int r = pin(c, stream, P))
		return r;
	const cgpu_snapshot &s = P.snap();
	if (n && (!saddr || !daddr || !flags || !verdict))
		return fail(-EINVAL, "null column");
	if (!n)
		return 0;
	prefilter_args a{saddr, daddr, nullptr, nullptr, flags, verdict, (uint64_t)n};
	HIP_OR_EIO(hipSetDevice(c->device));
	HIP_OR_EIO(launch_prefilter_v4(s, a, (hipStream_t)stream));
	return 0;
}

CGPU_EXPORT int cgpu_prefilter_v6(cgpu_ctx *c, const uint8_t *saddr, const uint8_t *daddr,
				  const uint8_t *flags, size_t n, uint8_t *verdict, void *stream)
{
	Pinned P;
	if (int r = pin(c, stream, P))
		return r;
	const cgpu_snapshot &s = P.snap();
	if (n && (!saddr || !daddr || !flags || !verdict))
		return fail(-EINVAL, "null column");
	if (((uintptr_t)saddr | (uintptr_t)daddr) & 15)
		return fail(-EINVAL, "v6 address columns must be 16-byte aligned");
	if (!n)
		return 0;
	prefilter_args a{nullptr, nullptr, saddr, daddr, flags, verdict, (uint64_t)n};
	HIP_OR_EIO(hipSetDevice(c->device));
	HIP_OR_EIO(launch_prefilter_v6(s, a, (hipStream_t)stream));
	return 0;
}

/* the prefilters over host-resident columns (addresses, flags in; one
 * verdict byte out) */
static int prefilter_host(cgpu_ctx *c, const void *saddr, const void *daddr, const uint8_t *flags, size_t n,
			  uint8_t *verdict, void *stream, int v6)
{
	if (!c)
		return fail(-EINVAL, "null context");
	if (n && (!saddr || !daddr || !flags || !verdict))
		return fail(-EINVAL, "null column");
	if (c->device < 0)
		return fail(-ENODEV, "context has no device (host-only); no CPU path");
	if (!n)
		return 0;
	std::lock_guard<std::mutex> g(c->host_mu);
	Pinned P;
	if (int r = pin(c, stream, P))
		return r;
	const cgpu_snapshot &s = P.snap();
	const hipStream_t cs = (hipStream_t)stream;
	const size_t ael = v6 ? 16 : 4;
	hs_cols C;
	C.nin = 3;
	C.in[0] = static_cast<const uint8_t *>(saddr);
	C.in[1] = static_cast<const uint8_t *>(daddr);
	C.in[2] = flags;
	C.in_el[0] = C.in_el[1] = ael;
	C.in_el[2] = 1;
	C.nout = 1;
	C.out[0] = verdict;
	C.out_el[0] = 1;
	return host_pipeline(c, n, C, cs, [&](size_t m, uint8_t *const *di, uint8_t *const *dout) -> int {
		prefilter_args a{nullptr, nullptr, nullptr, nullptr, di[2], dout[0], (uint64_t)m};
		if (v6) {
			a.saddr16 = di[0];
			a.daddr16 = di[1];
			HIP_OR_EIO(launch_prefilter_v6(s, a, cs));
		} else {
			a.saddr4 = reinterpret_cast<const uint32_t *>(di[0]);
			a.daddr4 = reinterpret_cast<const uint32_t *>(di[1]);
			HIP_OR_EIO(launch_prefilter_v4(s, a, cs));
		}
		return 0;
	});
}

CGPU_EXPORT int cgpu_prefilter_v4_host(cgpu_ctx *c, const uint32_t *saddr, const uint32_t *daddr,
				       const uint8_t *flags, size_t n, uint8_t *verdict, void *stream)
{
	return prefilter_host(c, saddr, daddr, flags, n, verdict, stream, 0);
}

CGPU_EXPORT int cgpu_prefilter_v6_host(cgpu_ctx *c, const uint8_t *saddr, const uint8_t *daddr,
				       const uint8_t *flags, size_t n, uint8_t *verdict, void *stream)
{
	return prefilter_host(c, saddr, daddr, flags, n, verdict, stream, 1);
}

/* ======================================================================= */
/* counters                                                                  */
/* ======================================================================= */
CGPU_EXPORT size_t cgpu_counter_delta_bytes(cgpu_ctx *c)
{
	return c ? ((size_t)2 * c->n_ctr_slots + CGPU_METRICS_WORDS) * 8 : 0;
}

CGPU_EXPORT int cgpu_counter_bind(cgpu_ctx *c, void *buf, size_t bytes)
{
	if (!c)
		return fail(-EINVAL, "null context");
	if (c->device < 0)
		return fail(-ENODEV, "context has no device");
	std::lock_guard<std::mutex> g(c->pk_mu);
	if (!buf) {
		c->d_delta = c->d_delta_own;
		return 0;
	}
	if (bytes < cgpu_counter_delta_bytes(c))
		return fail(-EINVAL, "counter buffer %zu < %zu bytes", bytes, cgpu_counter_delta_bytes(c));
	if ((uintptr_t)buf & 7)
		return fail(-EINVAL, "counter buffer not 8-byte aligned");
	c->d_delta = (uint64_t *)buf;
	return 0;
}

CGPU_EXPORT int cgpu_counter_fold(cgpu_ctx *c, void *stream)
{
	if (!c)
		return fail(-EINVAL, "null context");
	if (c->device < 0)
		return fail(-ENODEV, "context has no device");
	HIP_OR_EIO(hipSetDevice(c->device));
	HIP_OR_EIO(launch_fold(c->d_totals, c->d_delta,
			       (uint64_t)2 * c->n_ctr_slots + CGPU_METRICS_WORDS, (hipStream_t)stream));
	return 0;
}

CGPU_EXPORT int cgpu_metrics_read(cgpu_ctx *c, uint64_t *out)
{
	if (!c || !out)
		return fail(-EINVAL, "null argument");
	if (c->device < 0)
		return fail(-ENODEV, "context has no device");
	std::lock_guard<std::mutex> g(c->mu);
	return read_counter_words(c, (size_t)2 * c->n_ctr_slots, CGPU_METRICS_WORDS, out);
}

CGPU_EXPORT int cgpu_counters_reset(cgpu_ctx *c)
{
	if (!c)
		return fail(-EINVAL, "null context");
	if (c->device < 0)
		return 0;
	std::lock_guard<std::mutex> g(c->mu);
	size_t bytes = cgpu_counter_delta_bytes(c);
	HIP_OR_EIO(hipSetDevice(c->device));
	HIP_OR_EIO(hipDeviceSynchronize());
	HIP_OR_EIO(hipMemset(c->d_totals, 0, bytes));
	HIP_OR_EIO(hipMemset(c->d_delta, 0, bytes));
	{
		std::lock_guard<std::mutex> pg(c->pk_mu);
		for (auto &kv : c->d_pk)
			HIP_OR_EIO(hipMemset(kv.second.p, 0, (size_t)c->n_ctr_slots * 8));
	}
	HIP_OR_EIO(hipDeviceSynchronize());
	return 0;
}

/* ======================================================================= */
/* batched map writes and counter reads (the same per-key semantics)         */
/* ======================================================================= */
CGPU_EXPORT int cgpu_ipcache_update_batch(cgpu_ctx *c, const cgpu_ipcache_key *keys,
					  const cgpu_remote_endpoint_info *vals, size_t n, uint64_t flags)
{
	if (!c || (n && (!keys || !vals)))
		return fail(-EINVAL, "null argument");
	for (size_t i = 0; i < n; i++)
		if (int r = cgpu_ipcache_update(c, &keys[i], &vals[i], flags))
			return r;
	return 0;
}

CGPU_EXPORT int cgpu_policy_update_batch(cgpu_ctx *c, const uint32_t *eps, const cgpu_policy_key *keys,
					 const cgpu_policy_entry *entries, size_t n, uint64_t flags)
{
	if (!c || (n && (!eps || !keys || !entries)))
		return fail(-EINVAL, "null argument");
	for (size_t i = 0; i < n; i++)
		if (int r = cgpu_policy_update(c, eps[i], &keys[i], &entries[i], flags))
			return r;
	return 0;
}

CGPU_EXPORT int cgpu_cidr_update_batch(cgpu_ctx *c, int which, const cgpu_cidr_key *keys, size_t n,
				       uint64_t flags)
{
	if (!c || (n && !keys))
		return fail(-EINVAL, "null argument");
	for (size_t i = 0; i < n; i++)
		if (int r = cgpu_cidr_update(c, which, &keys[i], flags))
			return r;
	return 0;
}

/* entries of n (ep, key) pairs with ONE read of the device counters */
static int policy_fill(cgpu_ctx *c, const std::vector<std::pair<const PolEntry *, size_t>> &hit,
		       cgpu_policy_entry *out)
{
	std::vector<uint64_t> w;
	const bool dev = c->device >= 0 && c->captured;
	if (dev && !hit.empty()) {
		w.resize((size_t)2 * c->n_ctr_slots);
		if (int r = read_counter_words(c, 0, w.size(), w.data()))
			return r;
	}
	std::unordered_map<uint32_t, const SlotInit *> pending;
	for (auto &s : c->slot_inits)
		pending[s.slot] = &s; /* the most recent write of a slot wins */
	for (auto &h : hit) {
		cgpu_policy_entry &o = out[h.second];
		memset(&o, 0, sizeof(o));
		o.proxy_port = h.first->proxy_port;
		auto it = pending.find(h.first->slot);
		if (it != pending.end()) {
			o.packets = it->second->packets;
			o.bytes = it->second->bytes;
		} else if (dev) {
			o.packets = w[2u * h.first->slot];
			o.bytes = w[2u * h.first->slot + 1u];
		}
	}
	return 0;
}

CGPU_EXPORT int cgpu_policy_lookup_batch(cgpu_ctx *c, const uint32_t *eps, const cgpu_policy_key *keys,
					 size_t n, cgpu_policy_entry *out, int32_t *rc_out)
{
	if (!c || (n && (!eps || !keys || !out || !rc_out)))
		return fail(-EINVAL, "null argument");
	std::lock_guard<std::mutex> g(c->mu);
	std::vector<std::pair<const PolEntry *, size_t>> hit;
	for (size_t i = 0; i < n; i++) {
		rc_out[i] = -ENOENT;
		if (eps[i] >= c->cfg.max_endpoints) {
			rc_out[i] = -EINVAL;
			continue;
		}
		auto &m = c->pol[eps[i]];
		auto it = m.find(pol_key64(&keys[i]));
		if (it != m.end()) {
			rc_out[i] = 0;
			hit.push_back({&it->second, i});
		} else {
			memset(&out[i], 0, sizeof(out[i]));
		}
	}
	return policy_fill(c, hit, out);
}

CGPU_EXPORT int cgpu_policy_dump(cgpu_ctx *c, uint32_t ep, cgpu_policy_key *keys, cgpu_policy_entry *entries,
				 size_t cap, size_t *n_out)
{
	if (!c || !n_out || (cap && (!keys || !entries)) || ep >= (c ? c->cfg.max_endpoints : 0))
		return fail(-EINVAL, "bad argument");
	std::lock_guard<std::mutex> g(c->mu);
	auto &m = c->pol[ep];
	*n_out = m.size();
	if (m.size() > cap)
		return fail(-ENOSPC, "policy map of ep %u holds %zu keys > %zu", ep, m.size(), cap);
	std::vector<std::pair<const PolEntry *, size_t>> hit;
	size_t i = 0;
	for (auto &kv : m) {
		memcpy(&keys[i], &kv.first, 8);
		hit.push_back({&kv.second, i});
		i++;
	}
	return policy_fill(c, hit, entries);
}

/* ======================================================================= */
/* multi-GPU counter reduction: RCCL over xGMI                  */
/* ======================================================================= */
static_assert(CGPU_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "ncclUniqueId size");

static void comm_destroy(cgpu_ctx *c)
{
	if (c->comm) {
		(void)ncclCommDestroy((ncclComm_t)c->comm);
		c->comm = nullptr;
	}
}

CGPU_EXPORT int cgpu_comm_id_create(uint8_t *id_out)
{
	if (!id_out)
		return fail(-EINVAL, "null argument");
	ncclUniqueId id;
	const ncclResult_t r = ncclGetUniqueId(&id);
	if (r != ncclSuccess)
		return fail(-EIO, "ncclGetUniqueId: %s", ncclGetErrorString(r));
	memcpy(id_out, &id, sizeof(id));
	return 0;
}

CGPU_EXPORT int cgpu_comm_init(cgpu_ctx *c, const uint8_t *id, int nranks, int rank)
{
	if (!c || !id || nranks < 1 || rank < 0 || rank >= nranks)
		return fail(-EINVAL, "bad argument");
	if (c->device < 0)
		return fail(-ENODEV, "context has no device");
	std::lock_guard<std::mutex> g(c->pk_mu);
	if (c->comm)
		return fail(-EEXIST, "context already has a communicator");
	ncclUniqueId uid;
	memcpy(&uid, id, sizeof(uid));
	HIP_OR_EIO(hipSetDevice(c->device));
	ncclComm_t comm = nullptr;
	const ncclResult_t r = ncclCommInitRank(&comm, nranks, uid, rank);
	if (r != ncclSuccess)
		return fail(-EIO, "ncclCommInitRank(%d of %d): %s", rank, nranks, ncclGetErrorString(r));
	c->comm = comm;
	return 0;
}

CGPU_EXPORT int cgpu_counters_allreduce(cgpu_ctx *c, void *stream)
{
	if (!c)
		return fail(-EINVAL, "null context");
	if (c->device < 0)
		return fail(-ENODEV, "context has no device");
	uint64_t *delta;
	void *comm;
	{
		std::lock_guard<std::mutex> g(c->pk_mu);
		delta = c->d_delta;
		comm = c->comm;
	}
	if (!comm)
		return fail(-ENOENT, "no communicator (cgpu_comm_init)");
	HIP_OR_EIO(hipSetDevice(c->device));
	const size_t words = (size_t)2 * c->n_ctr_slots + CGPU_METRICS_WORDS;
	/* u64 SUM: order-independent, so every rank ends with the same bits */
	const ncclResult_t r = ncclAllReduce(delta, delta, words, ncclUint64, ncclSum, (ncclComm_t)comm,
					     (hipStream_t)stream);
	if (r != ncclSuccess)
		return fail(-EIO, "ncclAllReduce: %s", ncclGetErrorString(r));
	return 0;
}

/* ======================================================================= */
/* conntrack maps cilium_ct4_global / cilium_ct6_global   */
/* ======================================================================= */
static_assert(sizeof(cgpu_ct4_tuple) == 14, "ipv4_ct_tuple layout");
static_assert(sizeof(cgpu_ct6_tuple) == 38, "ipv6_ct_tuple layout");
static_assert(sizeof(cgpu_ct_entry) == 56, "ct_entry layout");

/* a key in slot format (CtK4 / CtK6 of kernels.hip), tag bits zero */
struct CtKey {
	uint4 w[3];
};

static inline CtKey ct_key4(const cgpu_ct4_tuple *k)
{
	CtKey r{};
	r.w[0] = uint4{k->daddr, k->saddr, (uint32_t)k->dport | ((uint32_t)k->sport << 16),
		       (uint32_t)k->nexthdr | ((uint32_t)k->flags << 8)};
	return r;
}

static inline CtKey ct_key6(const cgpu_ct6_tuple *k)
{
	CtKey r{};
	r.w[0] = uint4{(uint32_t)k->dport | ((uint32_t)k->sport << 16),
		       (uint32_t)k->nexthdr | ((uint32_t)k->flags << 8), 0u, 0u};
	memcpy(&r.w[1], k->daddr, 16);
	memcpy(&r.w[2], k->saddr, 16);
	return r;
}

static inline uint32_t ctm_meta(const CtMap &m, uint32_t h)
{
	return m.v6 ? m.keys[4u * h].y : m.keys[h].w;
}

static inline uint32_t ctm_tag(const CtMap &m, uint32_t h) { return ctm_meta(m, h) >> 16; }

static inline uint32_t ctm_hash(const CtMap &m, const CtKey &k)
{
	if (!m.v6)
		return ct_hash(k.w[0].x, k.w[0].y, k.w[0].z, k.w[0].w);
	const uint4 d = k.w[1], s = k.w[2];
	return ct_hash(fold6(d.x, d.y, d.z, d.w), fold6(s.x, s.y, s.z, s.w), k.w[0].x, k.w[0].y);
}

static inline bool eq4(uint4 a, uint4 b) { return a.x == b.x && a.y == b.y && a.z == b.z && a.w == b.w; }

static inline bool ctm_same(const CtMap &m, uint32_t h, const CtKey &k)
{
	if (!m.v6) {
		const uint4 s = m.keys[h];
		return s.x == k.w[0].x && s.y == k.w[0].y && s.z == k.w[0].z &&
		       (s.w & 0xFFFFu) == (k.w[0].w & 0xFFFFu);
	}
	const uint4 *s = &m.keys[4u * h];
	return s[0].x == k.w[0].x && (s[0].y & 0xFFFFu) == (k.w[0].y & 0xFFFFu) && eq4(s[1], k.w[1]) &&
	       eq4(s[2], k.w[2]);
}

static inline void ctm_set(CtMap &m, uint32_t h, const CtKey &k, uint32_t tag)
{
	if (!m.v6) {
		m.keys[h] = uint4{k.w[0].x, k.w[0].y, k.w[0].z, (k.w[0].w & 0xFFFFu) | (tag << 16)};
		return;
	}
	m.keys[4u * h] = uint4{k.w[0].x, (k.w[0].y & 0xFFFFu) | (tag << 16), 0u, 0u};
	m.keys[4u * h + 1u] = k.w[1];
	m.keys[4u * h + 2u] = k.w[2];
	m.keys[4u * h + 3u] = uint4{0u, 0u, 0u, 0u};
}

static inline CtKey ctm_key_at(const CtMap &m, uint32_t h)
{
	CtKey k{};
	if (!m.v6) {
		k.w[0] = m.keys[h];
		k.w[0].w &= 0xFFFFu;
	} else {
		k.w[0] = m.keys[4u * h];
		k.w[0].y &= 0xFFFFu;
		k.w[1] = m.keys[4u * h + 1u];
		k.w[2] = m.keys[4u * h + 2u];
	}
	return k;
}

static void ct_alloc_shadow(CtMap &m)
{
	if (!m.keys.empty())
		return;
	const uint32_t nslots = next_pow2((uint64_t)m.max * 2u);
	m.mask = nslots - 1u;
	m.keys.assign((size_t)nslots * m.sw(), uint4{0, 0, 0, 0});
	m.vals.assign((size_t)nslots * 4u, uint4{0, 0, 0, 0});
}

/* the probe of k_ct_walk's ct_find, on the shadow */
static int ct_h_find(const CtMap &m, const CtKey &k, uint32_t *free_at)
{
	uint32_t h = ctm_hash(m, k) & m.mask;
	uint32_t ff = UINT32_MAX;
	for (uint32_t probe = 0; probe <= m.mask; probe++) {
		const uint32_t tag = ctm_tag(m, h);
		if (tag == CT_TAG_EMPTY) {
			*free_at = ff != UINT32_MAX ? ff : h;
			return -1;
		}
		if (tag == CT_TAG_LIVE && ctm_same(m, h, k))
			return (int)h;
		if (tag == CT_TAG_TOMB && ff == UINT32_MAX)
			ff = h;
		h = (h + 1u) & m.mask;
	}
	*free_at = ff;
	return -1;
}

/* re-insert the live entries into clean arrays (drops tombstones) */
static void ct_rebuild(CtMap &m)
{
	std::vector<uint4> ok(m.keys.size(), uint4{0, 0, 0, 0}), ov(m.vals.size(), uint4{0, 0, 0, 0});
	ok.swap(m.keys);
	ov.swap(m.vals);
	CtMap old;
	old.v6 = m.v6;
	old.keys.swap(ok);
	for (uint32_t i = 0; i <= m.mask; i++) {
		if (ctm_tag(old, i) != CT_TAG_LIVE)
			continue;
		const CtKey k = ctm_key_at(old, i);
		uint32_t h = ctm_hash(m, k) & m.mask;
		while (ctm_tag(m, h) != CT_TAG_EMPTY)
			h = (h + 1u) & m.mask;
		ctm_set(m, h, k, CT_TAG_LIVE);
		for (int j = 0; j < 4; j++)
			m.vals[4u * h + j] = ov[4u * i + j];
	}
	m.tombs = 0;
}

/* device -> shadow after batches ran */
static int ct_pull(cgpu_ctx *c, CtMap &m)
{
	ct_alloc_shadow(m);
	if (c->device < 0 || !m.dev_newer)
		return 0;
	uint32_t cnt[2];
	HIP_OR_EIO(hipSetDevice(c->device));
	HIP_OR_EIO(hipDeviceSynchronize());
	HIP_OR_EIO(hipMemcpy(m.keys.data(), m.d_keys, m.keys.size() * 16, hipMemcpyDeviceToHost));
	HIP_OR_EIO(hipMemcpy(m.vals.data(), m.d_vals, m.vals.size() * 16, hipMemcpyDeviceToHost));
	HIP_OR_EIO(hipMemcpy(cnt, m.d_count, 8, hipMemcpyDeviceToHost));
	m.live = cnt[0];
	m.tombs = cnt[1];
	m.dev_newer = false;
	return 0;
}

/* shadow -> device before a batch (allocates the device map on first use) */
static int ct_push(CtMap &m)
{
	ct_alloc_shadow(m);
	if (!m.d_keys) {
		HIP_OR_EIO(hipMalloc((void **)&m.d_keys, m.keys.size() * 16));
		HIP_OR_EIO(hipMalloc((void **)&m.d_vals, m.vals.size() * 16));
		HIP_OR_EIO(hipMalloc((void **)&m.d_count, 8));
		m.host_newer = true;
	}
	if (!m.host_newer)
		return 0;
	const uint32_t cnt[2] = {m.live, m.tombs};
	HIP_OR_EIO(hipMemcpy(m.d_keys, m.keys.data(), m.keys.size() * 16, hipMemcpyHostToDevice));
	HIP_OR_EIO(hipMemcpy(m.d_vals, m.vals.data(), m.vals.size() * 16, hipMemcpyHostToDevice));
	HIP_OR_EIO(hipMemcpy(m.d_count, cnt, 8, hipMemcpyHostToDevice));
	m.host_newer = false;
	return 0;
}

static int ct_update_l(cgpu_ctx *c, CtMap &m, const CtKey &k, const cgpu_ct_entry *val, uint64_t flags)
{
	if (!val)
		return fail(-EINVAL, "null value");
	if (int r = check_flags(flags))
		return r;
	std::lock_guard<std::mutex> g(c->mu);
	if (int r = ct_pull(c, m))
		return r;
	uint32_t free_at;
	int slot = ct_h_find(m, k, &free_at);
	if (slot >= 0 && flags == CGPU_NOEXIST)
		return fail(-EEXIST, "conntrack entry exists");
	if (slot < 0) {
		if (flags == CGPU_EXIST)
			return fail(-ENOENT, "no such conntrack entry");
		if (m.live >= m.max)
			return fail(-E2BIG, "conntrack map full (%u entries)", m.max);
		if (free_at == UINT32_MAX) {
			ct_rebuild(m);
			(void)ct_h_find(m, k, &free_at);
		}
		if (ctm_tag(m, free_at) == CT_TAG_TOMB)
			m.tombs--;
		slot = (int)free_at;
		ctm_set(m, (uint32_t)slot, k, CT_TAG_LIVE);
		m.live++;
	}
	uint4 row[4] = {};
	memcpy(row, val, sizeof(*val));
	for (int j = 0; j < 4; j++)
		m.vals[4u * slot + j] = row[j];
	m.host_newer = true;
	return 0;
}

static int ct_delete_l(cgpu_ctx *c, CtMap &m, const CtKey &k)
{
	std::lock_guard<std::mutex> g(c->mu);
	if (int r = ct_pull(c, m))
		return r;
	uint32_t free_at;
	const int slot = ct_h_find(m, k, &free_at);
	if (slot < 0)
		return fail(-ENOENT, "no such conntrack entry");
	ctm_set(m, (uint32_t)slot, CtKey{}, CT_TAG_TOMB);
	for (int j = 0; j < 4; j++)
		m.vals[4u * slot + j] = uint4{0, 0, 0, 0};
	m.live--;
	m.tombs++;
	if (m.tombs > (m.mask + 1u) / 4u)
		ct_rebuild(m);
	m.host_newer = true;
	return 0;
}

static int ct_lookup_l(cgpu_ctx *c, CtMap &m, const CtKey &k, cgpu_ct_entry *val_out)
{
	std::lock_guard<std::mutex> g(c->mu);
	if (int r = ct_pull(c, m))
		return r;
	uint32_t free_at;
	const int slot = ct_h_find(m, k, &free_at);
	if (slot < 0)
		return fail(-ENOENT, "no such conntrack entry");
	if (val_out)
		memcpy(val_out, &m.vals[4u * slot], sizeof(*val_out));
	return 0;
}

/* GetNextKey in slot order (a missing key restarts from the first): the
 * live key after `k` (or the first when k is null), in slot format */
static int ct_next_l(cgpu_ctx *c, CtMap &m, const CtKey *k, CtKey *next)
{
	std::lock_guard<std::mutex> g(c->mu);
	if (int r = ct_pull(c, m))
		return r;
	uint32_t from = 0;
	if (k) {
		uint32_t free_at;
		const int slot = ct_h_find(m, *k, &free_at);
		if (slot >= 0)
			from = (uint32_t)slot + 1u;
	}
	for (uint64_t i = from; i <= m.mask; i++)
		if (ctm_tag(m, (uint32_t)i) == CT_TAG_LIVE) {
			*next = ctm_key_at(m, (uint32_t)i);
			return 0;
		}
	return -ENOENT;
}

static size_t ct_count_l(cgpu_ctx *c, CtMap &m)
{
	std::lock_guard<std::mutex> g(c->mu);
	if (ct_pull(c, m))
		return 0;
	return m.live;
}

/* compaction on the device (caller holds mu; the map is current on the
 * device): every live entry re-inserted into the second table on the
 * conntrack stream, then the two swap */
static int ct_rehash_dev(cgpu_ctx *c, CtMap &m, hipStream_t cs)
{
	const size_t kb = m.keys.size() * 16, vb = m.vals.size() * 16;
	if (!m.d_keys2) {
		HIP_OR_EIO(hipMalloc((void **)&m.d_keys2, kb));
		HIP_OR_EIO(hipMalloc((void **)&m.d_vals2, vb));
	}
	HIP_OR_EIO(hipMemsetAsync(m.d_keys2, 0, kb, cs));
	const ct_table src{m.d_keys, m.d_vals, m.mask, m.max, m.d_count, 1u};
	const ct_table dst{m.d_keys2, m.d_vals2, m.mask, m.max, m.d_count, 1u};
	HIP_OR_EIO(launch_ct_rehash(src, dst, m.v6, cs));
	HIP_OR_EIO(hipMemsetAsync(m.d_count + 1, 0, 4, cs));
	std::swap(m.d_keys, m.d_keys2);
	std::swap(m.d_vals, m.d_vals2);
	m.tombs = 0;
	m.compactions++;
	(void)c;
	return 0;
}

static int ct_gc_l(cgpu_ctx *c, CtMap &m, uint32_t time, uint64_t *deleted_out)
{
	std::lock_guard<std::mutex> g(c->mu);
	if (c->device >= 0 && m.d_keys && !m.host_newer) {
		/* the device map is current: filter it in place, ordered behind
		 * the batches on the conntrack stream; one read of the result */
		HIP_OR_EIO(hipSetDevice(c->device));
		const hipStream_t cs = c->ct_stream;
		if (!m.d_gc)
			HIP_OR_EIO(hipMalloc((void **)&m.d_gc, 4));
		HIP_OR_EIO(hipMemsetAsync(m.d_gc, 0, 4, cs));
		const ct_table T{m.d_keys, m.d_vals, m.mask, m.max, m.d_count, 1u};
		HIP_OR_EIO(launch_ct_gc(T, m.v6, time, m.d_gc, cs));
		uint32_t r[3];
		HIP_OR_EIO(hipMemcpyAsync(r, m.d_gc, 4, hipMemcpyDeviceToHost, cs));
		HIP_OR_EIO(hipMemcpyAsync(r + 1, m.d_count, 8, hipMemcpyDeviceToHost, cs));
		HIP_OR_EIO(hipStreamSynchronize(cs));
		m.live = r[1];
		m.tombs = r[2];
		m.dev_newer = true;
		if (deleted_out)
			*deleted_out = r[0];
		return 0;
	}
	if (int r = ct_pull(c, m))
		return r;
	uint64_t del = 0;
	for (uint32_t i = 0; i <= m.mask; i++) {
		if (ctm_tag(m, i) != CT_TAG_LIVE)
			continue;
		const uint32_t lifetime = m.vals[4u * i + 2u].x;
		if (lifetime < time) { /* doFiltering: RemoveExpired && Lifetime < Time */
			ctm_set(m, i, CtKey{}, CT_TAG_TOMB);
			for (int j = 0; j < 4; j++)
				m.vals[4u * i + j] = uint4{0, 0, 0, 0};
			m.live--;
			del++;
		}
	}
	ct_rebuild(m);
	m.host_newer = true;
	if (deleted_out)
		*deleted_out = del;
	return 0;
}

static int ct_flush_l(cgpu_ctx *c, CtMap &m)
{
	std::lock_guard<std::mutex> g(c->mu);
	ct_alloc_shadow(m);
	m.live = m.tombs = 0;
	if (c->device >= 0 && m.d_keys) {
		/* empty the device map in place, ordered on the conntrack stream
		 * behind every batch before it (tags and counts; rows are
		 * rewritten whole by every insert): no device-wide wait.  The host
		 * shadow is then stale and re-read before any host access
		 * (ct_pull), so it is not cleared here either. */
		HIP_OR_EIO(hipSetDevice(c->device));
		HIP_OR_EIO(hipMemsetAsync(m.d_keys, 0, m.keys.size() * 16, c->ct_stream));
		HIP_OR_EIO(hipMemsetAsync(m.d_count, 0, 8, c->ct_stream));
		m.dev_newer = true;
		m.host_newer = false;
		return 0;
	}
	std::fill(m.keys.begin(), m.keys.end(), uint4{0, 0, 0, 0});
	std::fill(m.vals.begin(), m.vals.end(), uint4{0, 0, 0, 0});
	m.dev_newer = false;
	m.host_newer = true;
	return 0;
}

static cgpu_ct4_tuple ct_unkey4(const CtKey &k)
{
	cgpu_ct4_tuple t;
	t.daddr = k.w[0].x;
	t.saddr = k.w[0].y;
	t.dport = (uint16_t)k.w[0].z;
	t.sport = (uint16_t)(k.w[0].z >> 16);
	t.nexthdr = (uint8_t)k.w[0].w;
	t.flags = (uint8_t)(k.w[0].w >> 8);
	return t;
}

static cgpu_ct6_tuple ct_unkey6(const CtKey &k)
{
	cgpu_ct6_tuple t;
	memcpy(t.daddr, &k.w[1], 16);
	memcpy(t.saddr, &k.w[2], 16);
	t.dport = (uint16_t)k.w[0].x;
	t.sport = (uint16_t)(k.w[0].x >> 16);
	t.nexthdr = (uint8_t)k.w[0].y;
	t.flags = (uint8_t)(k.w[0].y >> 8);
	return t;
}

/* ---- cilium_ct4_global ---- */
CGPU_EXPORT int cgpu_ct4_update(cgpu_ctx *c, const cgpu_ct4_tuple *key, const cgpu_ct_entry *val,
				uint64_t flags)
{
	if (!c || !key)
		return fail(-EINVAL, "null argument");
	return ct_update_l(c, c->ct4, ct_key4(key), val, flags);
}

CGPU_EXPORT int cgpu_ct4_delete(cgpu_ctx *c, const cgpu_ct4_tuple *key)
{
	if (!c || !key)
		return fail(-EINVAL, "null argument");
	return ct_delete_l(c, c->ct4, ct_key4(key));
}

CGPU_EXPORT int cgpu_ct4_lookup(cgpu_ctx *c, const cgpu_ct4_tuple *key, cgpu_ct_entry *val_out)
{
	if (!c || !key)
		return fail(-EINVAL, "null argument");
	return ct_lookup_l(c, c->ct4, ct_key4(key), val_out);
}

CGPU_EXPORT int cgpu_ct4_get_next_key(cgpu_ctx *c, const cgpu_ct4_tuple *key, cgpu_ct4_tuple *next_out)
{
	if (!c || !next_out)
		return fail(-EINVAL, "null argument");
	CtKey k = key ? ct_key4(key) : CtKey{}, nk;
	const int r = ct_next_l(c, c->ct4, key ? &k : nullptr, &nk);
	if (!r)
		*next_out = ct_unkey4(nk);
	return r;
}

CGPU_EXPORT size_t cgpu_ct4_count(cgpu_ctx *c) { return c ? ct_count_l(c, c->ct4) : 0; }

CGPU_EXPORT int cgpu_ct4_gc(cgpu_ctx *c, uint32_t time, uint64_t *deleted_out)
{
	if (!c)
		return fail(-EINVAL, "null context");
	return ct_gc_l(c, c->ct4, time, deleted_out);
}

CGPU_EXPORT int cgpu_ct_stats(cgpu_ctx *c, int v6, uint64_t *out)
{
	if (!c || !out)
		return fail(-EINVAL, "null argument");
	CtMap &m = v6 ? c->ct6 : c->ct4;
	std::lock_guard<std::mutex> g(c->mu);
	uint32_t live = m.live, tombs = m.tombs;
	if (c->device >= 0 && m.d_count && m.dev_newer) {
		uint32_t cnt[2];
		HIP_OR_EIO(hipSetDevice(c->device));
		HIP_OR_EIO(hipMemcpyAsync(cnt, m.d_count, 8, hipMemcpyDeviceToHost, c->ct_stream));
		HIP_OR_EIO(hipStreamSynchronize(c->ct_stream));
		live = cnt[0];
		tombs = cnt[1];
	}
	out[0] = live;
	out[1] = tombs;
	out[2] = m.compactions;
	return 0;
}

CGPU_EXPORT int cgpu_ct4_flush(cgpu_ctx *c)
{
	if (!c)
		return fail(-EINVAL, "null context");
	return ct_flush_l(c, c->ct4);
}

/* ---- cilium_ct6_global ---- */
CGPU_EXPORT int cgpu_ct6_update(cgpu_ctx *c, const cgpu_ct6_tuple *key, const cgpu_ct_entry *val,
				uint64_t flags)
{
	if (!c || !key)
		return fail(-EINVAL, "null argument");
	return ct_update_l(c, c->ct6, ct_key6(key), val, flags);
}

CGPU_EXPORT int cgpu_ct6_delete(cgpu_ctx *c, const cgpu_ct6_tuple *key)
{
	if (!c || !key)
		return fail(-EINVAL, "null argument");
	return ct_delete_l(c, c->ct6, ct_key6(key));
}

CGPU_EXPORT int cgpu_ct6_lookup(cgpu_ctx *c, const cgpu_ct6_tuple *key, cgpu_ct_entry *val_out)
{
	if (!c || !key)
		return fail(-EINVAL, "null argument");
	return ct_lookup_l(c, c->ct6, ct_key6(key), val_out);
}

CGPU_EXPORT int cgpu_ct6_get_next_key(cgpu_ctx *c, const cgpu_ct6_tuple *key, cgpu_ct6_tuple *next_out)
{
	if (!c || !next_out)
		return fail(-EINVAL, "null argument");
	CtKey k = key ? ct_key6(key) : CtKey{}, nk;
	const int r = ct_next_l(c, c->ct6, key ? &k : nullptr, &nk);
	if (!r)
		*next_out = ct_unkey6(nk);
	return r;
}

CGPU_EXPORT size_t cgpu_ct6_count(cgpu_ctx *c) { return c ? ct_count_l(c, c->ct6) : 0; }

CGPU_EXPORT int cgpu_ct6_gc(cgpu_ctx *c, uint32_t time, uint64_t *deleted_out)
{
	if (!c)
		return fail(-EINVAL, "null context");
	return ct_gc_l(c, c->ct6, time, deleted_out);
}

CGPU_EXPORT int cgpu_ct6_flush(cgpu_ctx *c)
{
	if (!c)
		return fail(-EINVAL, "null context");
	return ct_flush_l(c, c->ct6);
}

/* scratch of one cgpu_classify_v{4,6}_ct launch over n packets */
struct CtScratch {
	size_t rec, gkey, gkey_sorted, idx, idx_sorted, heads, n_heads, heads_pos, head,
		temp, temp_bytes, svc_out, ctl, flags2, pcls, total;
};

static CtScratch ct_scratch_layout(uint64_t n, size_t rec_bytes, bool svc, bool v6)
{
	CtScratch L{};
	auto take = [&](size_t bytes) {
		size_t off = L.total;
		L.total += (bytes + 255) & ~(size_t)255;
		return off;
	};
	L.rec = take(n * rec_bytes);
	L.gkey = take(n * 4);
	L.gkey_sorted = take(n * 4);
	L.idx = take(n * 4);
	L.idx_sorted = take(n * 4);
	L.heads = take(n * 4);
	L.n_heads = take(4);
	L.heads_pos = take(n * 4);
	L.head = take(n);
	L.temp_bytes = ct_temp_bytes(n);
	L.temp = take(L.temp_bytes);
	L.flags2 = take((svc ? 4 : 2) * n); /* phase-2 candidates */
	if (svc) {
		L.svc_out = take(n * (v6 ? 32 : 16));
		L.ctl = take(16);
		L.pcls = take(n);
	}
	return L;
}

/* one stateful batch on map m: columns already validated by the caller */
static int ct_classify(cgpu_ctx *c, const cgpu_snapshot &s, uint64_t *delta, CtMap &m, ct_launch a,
		       void *stream, bool svc = false)
{
	/* One conntrack map, one scratch: every batch runs on the context's
	 * conntrack stream, after the caller's stream reaches this call (its
	 * inputs), and the caller's stream then waits for the batch. */
	std::lock_guard<std::mutex> g(c->mu);
	HIP_OR_EIO(hipSetDevice(c->device));
	const hipStream_t cs = c->ct_stream;
	HIP_OR_EIO(hipEventRecord(c->ct_done, (hipStream_t)stream));
	HIP_OR_EIO(hipStreamWaitEvent(cs, c->ct_done, 0));
	uint32_t live = m.live;
	if (m.d_count && !m.host_newer) {
		/* tombstones left by the device's deletes: compact before they
		 * lengthen every probe chain (the host reads the count after the
		 * previous batch: the one host synchronisation of this call) */
		uint32_t cnt[2];
		HIP_OR_EIO(hipMemcpyAsync(cnt, m.d_count, 8, hipMemcpyDeviceToHost, cs));
		HIP_OR_EIO(hipStreamSynchronize(cs));
		live = cnt[0];
		if (cnt[1] > (m.mask + 1u) / 4u) {
			if (int r = ct_rehash_dev(c, m, cs))
				return r;
		}
	}
	if (int r = ct_push(m))
		return r;
	const CtScratch L = ct_scratch_layout(a.n, m.v6 ? 64 : svc ? 48 : 32, svc, m.v6);
	if (L.total > c->ct_scratch_cap) {
		HIP_OR_EIO(hipStreamSynchronize(cs));
		(void)hipFree(c->d_ct_scratch);
		c->d_ct_scratch = nullptr;
		c->ct_scratch_cap = 0;
		HIP_OR_EIO(hipMalloc(&c->d_ct_scratch, L.total));
		c->ct_scratch_cap = L.total;
	}
	if (!c->d_ct_pk) {
		HIP_OR_EIO(hipMalloc((void **)&c->d_ct_pk, (size_t)c->n_ctr_slots * 8u));
		HIP_OR_EIO(hipMemsetAsync(c->d_ct_pk, 0, (size_t)c->n_ctr_slots * 8u, cs));
	}
	uint8_t *b = static_cast<uint8_t *>(c->d_ct_scratch);
	/* every walker wave (2048 x 4) holding a chunk stays under a quarter
	 * of the headroom */
	const uint32_t headroom = m.max > live ? m.max - live : 0u;
	const uint32_t chunk = std::min<uint32_t>(256u, std::max<uint32_t>(1u, headroom / 32768u));
	ct_table T{m.d_keys, m.d_vals, m.mask, m.max, m.d_count, chunk};
	/* LRU mode (the plain paths; the service paths keep failing creates
	 * closed): the batch's key filter, 16 MiB */
	if (c->cfg.ct_lru && !svc) {
		if (!m.d_bloom)
			HIP_OR_EIO(hipMalloc((void **)&m.d_bloom, (size_t)CT_BLOOM_WORDS * 4u));
		T.bloom = m.d_bloom;
		T.bloom_mask = CT_BLOOM_WORDS - 1u;
		T.lru = 1;
	}
	a.delta = delta;
	a.rec = reinterpret_cast<uint4 *>(b + L.rec);
	a.gkey = reinterpret_cast<uint32_t *>(b + L.gkey);
	a.gkey_sorted = reinterpret_cast<uint32_t *>(b + L.gkey_sorted);
	a.idx = reinterpret_cast<uint32_t *>(b + L.idx);
	a.idx_sorted = reinterpret_cast<uint32_t *>(b + L.idx_sorted);
	a.head = b + L.head;
	a.heads = reinterpret_cast<uint32_t *>(b + L.heads);
	a.n_heads = reinterpret_cast<uint32_t *>(b + L.n_heads);
	a.heads_pos = reinterpret_cast<uint32_t *>(b + L.heads_pos);
	a.temp = b + L.temp;
	a.temp_bytes = L.temp_bytes;
	a.flags2 = b + L.flags2;
	a.pk = c->d_ct_pk;
	a.dflt = 1u; /* group-default results (kernels.hip CT_DFLT; the launchers clear it where a prep stores every result) */
	hipError_t le;
	if (svc) {
		a.svc_out = reinterpret_cast<uint4 *>(b + L.svc_out);
		a.ctl = reinterpret_cast<uint32_t *>(b + L.ctl);
		a.pcls = b + L.pcls;
		le = m.v6 ? launch_classify_v6_ctlb(s, T, a, cs) : launch_classify_v4_ctlb(s, T, a, cs);
	} else {
		le = m.v6 ? launch_classify_v6_ct(s, T, a, cs) : launch_classify_v4_ct(s, T, a, cs);
	}
	if (le != hipSuccess) {
		/* pk is shared by every conntrack call and only k_unpack zeroes it:
		 * a finish whose unpack never ran must not leak into the next call */
		(void)hipMemsetAsync(c->d_ct_pk, 0, (size_t)c->n_ctr_slots * 8u, cs);
		return fail(-EIO, "conntrack launch: %s", hipGetErrorString(le));
	}
	HIP_OR_EIO(hipEventRecord(c->ct_done, cs));
	HIP_OR_EIO(hipStreamWaitEvent((hipStream_t)stream, c->ct_done, 0));
	m.dev_newer = true;
	return 0;
}

CGPU_EXPORT int cgpu_classify_v4_ct(cgpu_ctx *c, const cgpu_tuples_v4_ct *t, size_t n, uint32_t now,
				    int32_t *verdict, uint8_t *ct_ret, uint32_t *identity,
				    uint8_t *stage, void *stream)
{
	Pinned P;
	if (int r = pin(c, stream, P))
		return r;
	if (!t || (n && (!t->saddr || !t->daddr || !t->sport || !t->dport || !t->proto || !t->l4 ||
			 !t->flags || !t->len || !t->ep || !verdict || !ct_ret || !identity)))
		return fail(-EINVAL, "null tuple column or output");
	if (n > (size_t)INT32_MAX)
		return fail(-EINVAL, "batch of %zu packets exceeds 2^31 - 1", n);
	if (!n)
		return 0;
	ct_launch a{};
	a.saddr = t->saddr;
	a.daddr = t->daddr;
	a.sport = t->sport;
	a.dport = t->dport;
	a.proto = t->proto;
	a.l4 = t->l4;
	a.flags = t->flags;
	a.len = t->len;
	a.ep = t->ep;
	a.verdict = verdict;
	a.ct_ret = ct_ret;
	a.identity = identity;
	a.stage = stage;
	a.n = n;
	a.now = now;
	return ct_classify(c, P.snap(), P.delta, c->ct4, a, stream);
}

CGPU_EXPORT int cgpu_classify_v4_ctlb(cgpu_ctx *c, const cgpu_tuples_v4_ct *t, const uint32_t *hash,
				      size_t n, uint32_t now, const cgpu_ctlb_out *out, void *stream)
{
	Pinned P;
	if (int r = pin(c, stream, P))
		return r;
	if (!t || !out || (n && (!t->saddr || !t->daddr || !t->sport || !t->dport || !t->proto || !t->l4 ||
				 !t->flags || !t->len || !t->ep || !out->verdict || !out->ct_ret ||
				 !out->identity)))
		return fail(-EINVAL, "null tuple column or output");
	if (n > (size_t)INT32_MAX / 2)
		return fail(-EINVAL, "batch of %zu packets exceeds 2^30 - 1", n);
	if (!n)
		return 0;
	ct_launch a{};
	a.saddr = t->saddr;
	a.daddr = t->daddr;
	a.sport = t->sport;
	a.dport = t->dport;
	a.proto = t->proto;
	a.l4 = t->l4;
	a.flags = t->flags;
	a.len = t->len;
	a.ep = t->ep;
	a.verdict = out->verdict;
	a.ct_ret = out->ct_ret;
	a.identity = out->identity;
	a.stage = out->stage;
	a.xdaddr = out->daddr;
	a.xdport = out->dport;
	a.hash = hash;
	a.n = n;
	a.now = now;
	return ct_classify(c, P.snap(), P.delta, c->ct4, a, stream, true);
}

CGPU_EXPORT int cgpu_classify_v6_ctlb(cgpu_ctx *c, const cgpu_tuples_v6_ct *t, const uint32_t *hash,
				      size_t n, uint32_t now, const cgpu_ctlb6_out *out, void *stream)
{
	Pinned P;
	if (int r = pin(c, stream, P))
		return r;
	if (!t || !out || (n && (!t->saddr || !t->daddr || !t->sport || !t->dport || !t->proto || !t->l4 ||
				 !t->flags || !t->len || !t->ep || !out->verdict || !out->ct_ret ||
				 !out->identity)))
		return fail(-EINVAL, "null tuple column or output");
	if (n && (((uintptr_t)t->saddr | (uintptr_t)t->daddr | (uintptr_t)out->daddr) & 15))
		return fail(-EINVAL, "IPv6 address columns must be 16-byte aligned");
	if (n > (size_t)INT32_MAX / 2)
		return fail(-EINVAL, "batch of %zu packets exceeds 2^30 - 1", n);
	if (!n)
		return 0;
	ct_launch a{};
	a.saddr = t->saddr;
	a.daddr = t->daddr;
	a.sport = t->sport;
	a.dport = t->dport;
	a.proto = t->proto;
	a.l4 = t->l4;
	a.flags = t->flags;
	a.len = t->len;
	a.ep = t->ep;
	a.verdict = out->verdict;
	a.ct_ret = out->ct_ret;
	a.identity = out->identity;
	a.stage = out->stage;
	a.xdaddr = out->daddr;
	a.xdport = out->dport;
	a.hash = hash;
	a.n = n;
	a.now = now;
	return ct_classify(c, P.snap(), P.delta, c->ct6, a, stream, true);
}

CGPU_EXPORT int cgpu_classify_v6_ct(cgpu_ctx *c, const cgpu_tuples_v6_ct *t, size_t n, uint32_t now,
				    int32_t *verdict, uint8_t *ct_ret, uint32_t *identity,
				    uint8_t *stage, void *stream)
{
	Pinned P;
	if (int r = pin(c, stream, P))
		return r;
	if (!t || (n && (!t->saddr || !t->daddr || !t->sport || !t->dport || !t->proto || !t->l4 ||
			 !t->flags || !t->len || !t->ep || !verdict || !ct_ret || !identity)))
		return fail(-EINVAL, "null tuple column or output");
	if (n && (((uintptr_t)t->saddr | (uintptr_t)t->daddr) & 15))
		return fail(-EINVAL, "IPv6 address columns must be 16-byte aligned");
	if (n > (size_t)INT32_MAX)
		return fail(-EINVAL, "batch of %zu packets exceeds 2^31 - 1", n);
	if (!n)
		return 0;
	ct_launch a{};
	a.saddr = t->saddr;
	a.daddr = t->daddr;
	a.sport = t->sport;
	a.dport = t->dport;
	a.proto = t->proto;
	a.l4 = t->l4;
	a.flags = t->flags;
	a.len = t->len;
	a.ep = t->ep;
	a.verdict = verdict;
	a.ct_ret = ct_ret;
	a.identity = identity;
	a.stage = stage;
	a.n = n;
	a.now = now;
	return ct_classify(c, P.snap(), P.delta, c->ct6, a, stream);
}

/* ======================================================================= */
/* host mirror snapshot / restore (SURVEY §5 checkpoint / resume)            */
/* ======================================================================= */
/* The reference keeps its maps pinned in bpffs across agent restarts and
 * replays the ipcache into new listeners (pkg/ipcache/ipcache.go:328-338
 * DumpToListenerLocked).  The engine's authoritative state is the host
 * mirror (plus the device-side counters and conntrack maps), so a checkpoint
 * is the mirror serialized, and a restore replays it through the same map
 * calls the agent uses.  File: "CGPUMIR1", u32 version, u32 section count,
 * sections {u32 tag, u32 record bytes, u64 count, records}, then the FNV-1a
 * hash of everything before it. */
enum { MIR_IPC = 1, MIR_POL, MIR_CIDR, MIR_EP, MIR_LB4, MIR_LB6, MIR_LXC, MIR_REV, MIR_CT4, MIR_CT6 };

struct MirOut {
	std::vector<uint8_t> buf;
	void put(const void *p, size_t n)
	{
		const uint8_t *b = static_cast<const uint8_t *>(p);
		buf.insert(buf.end(), b, b + n);
	}
	template <typename T> void put(const T &v) { put(&v, sizeof(v)); }
	size_t section(uint32_t tag, uint32_t rec)
	{
		put(tag);
		put(rec);
		const size_t at = buf.size();
		put((uint64_t)0);
		return at;
	}
	void count(size_t at, uint64_t n) { memcpy(&buf[at], &n, 8); }
};

static void mir_ct(MirOut &o, uint32_t tag, const CtMap &m, uint32_t ksz)
{
	const size_t at = o.section(tag, ksz + 56);
	uint64_t n = 0;
	for (uint32_t h = 0; h <= m.mask && !m.keys.empty(); h++) {
		if (ctm_tag(m, h) != CT_TAG_LIVE)
			continue;
		const CtKey k = ctm_key_at(m, h);
		if (m.v6) {
			const cgpu_ct6_tuple t = ct_unkey6(k);
			o.put(&t, ksz);
		} else {
			const cgpu_ct4_tuple t = ct_unkey4(k);
			o.put(&t, ksz);
		}
		o.put(&m.vals[4u * h], 56);
		n++;
	}
	o.count(at, n);
}

CGPU_EXPORT int cgpu_mirror_save(cgpu_ctx *c, const char *path)
{
	if (!c || !path)
		return fail(-EINVAL, "null argument");
	MirOut o;
	o.put("CGPUMIR1", 8);
	o.put((uint32_t)1);
	o.put((uint32_t)10);
	{
		std::lock_guard<std::mutex> g(c->mu);
		/* device-side state the mirror does not hold: per-entry counters
		 * (as cgpu_policy_lookup reports them) and the conntrack maps */
		std::vector<std::pair<const PolEntry *, size_t>> hit;
		for (uint32_t ep = 0; ep < c->pol.size(); ep++)
			for (auto &kv : c->pol[ep])
				hit.push_back({&kv.second, hit.size()});
		std::vector<cgpu_policy_entry> ents(hit.size());
		if (int r = policy_fill(c, hit, ents.data()))
			return r;
		if (int r = ct_pull(c, c->ct4))
			return r;
		if (int r = ct_pull(c, c->ct6))
			return r;
		size_t at = o.section(MIR_IPC, 32);
		for (auto &kv : c->ipc) {
			o.put(kv.second.raw);
			o.put(kv.second.val);
		}
		o.count(at, c->ipc.size());
		at = o.section(MIR_POL, 36);
		uint64_t n = 0;
		for (uint32_t ep = 0; ep < c->pol.size(); ep++)
			for (auto &kv : c->pol[ep]) {
				o.put(ep);
				o.put(&kv.first, 8);
				o.put(ents[n]);
				n++;
			}
		o.count(at, n);
		at = o.section(MIR_CIDR, 24);
		n = 0;
		auto cidr = [&](uint32_t which, const cgpu_cidr_key &k) {
			o.put(which);
			o.put(k);
			n++;
		};
		for (auto &kv : c->dyn4)
			cidr(CGPU_CIDR_V4_DYN, kv.second);
		for (auto &kv : c->dyn6)
			cidr(CGPU_CIDR_V6_DYN, kv.second);
		for (auto &x : c->fix4) {
			cgpu_cidr_key k{};
			memcpy(&k, x.data(), x.size());
			cidr(CGPU_CIDR_V4_FIX, k);
		}
		for (auto &x : c->fix6) {
			cgpu_cidr_key k{};
			memcpy(&k, x.data(), x.size());
			cidr(CGPU_CIDR_V6_FIX, k);
		}
		o.count(at, n);
		at = o.section(MIR_EP, 20);
		for (auto &x : c->lxc)
			o.put(x.data(), 20);
		o.count(at, c->lxc.size());
		at = o.section(MIR_LB4, 20);
		for (auto &kv : c->lb) {
			const cgpu_lb4_key k = lb_unkey(kv.first);
			o.put(k);
			o.put(kv.second);
		}
		o.count(at, c->lb.size());
		at = o.section(MIR_LB6, 44);
		for (auto &kv : c->lb6) {
			const cgpu_lb6_key k = lb6_unkey(kv.first);
			o.put(k);
			o.put(kv.second);
		}
		o.count(at, c->lb6.size());
		at = o.section(MIR_LXC, 36);
		for (auto &kv : c->lxcinfo) {
			o.put(kv.first);
			o.put(kv.second);
		}
		o.count(at, c->lxcinfo.size());
		at = o.section(MIR_REV, 8);
		o.put(c->pf_revision);
		o.count(at, 1);
		mir_ct(o, MIR_CT4, c->ct4, 14);
		mir_ct(o, MIR_CT6, c->ct6, 38);
	}
	o.put(fnv(1469598103934665603ull, o.buf.data(), o.buf.size()));
	const std::string tmp = std::string(path) + ".tmp";
	FILE *f = fopen(tmp.c_str(), "wb");
	if (!f)
		return fail(-errno, "cannot create %s", tmp.c_str());
	const bool ok = fwrite(o.buf.data(), 1, o.buf.size(), f) == o.buf.size();
	if (fclose(f) != 0 || !ok || rename(tmp.c_str(), path) != 0) {
		remove(tmp.c_str());
		return fail(-EIO, "cannot write %s", path);
	}
	return 0;
}

struct MirSec {
	uint32_t tag, rec;
	uint64_t n;
	size_t off;
};

struct CgpuConfigCaps {
	uint64_t ipcache, policy_per_ep, endpoints, lb, ct4, ct6;
};

static CgpuConfigCaps config_caps(const cgpu_ctx *c)
{
	return CgpuConfigCaps{c->cfg.ipcache_max, c->cfg.policy_max_per_ep, c->cfg.endpoints_max,
			      c->cfg.lb_max_entries, c->ct4.max, c->ct6.max};
}

/* undo a partial replay: delete, newest first, every record of sections
 * [0, si) and records [0, upto) of section si (each was a NOEXIST insert
 * into the empty context), and put the prefilter revision back */
static void mirror_rollback(cgpu_ctx *c, const std::vector<uint8_t> &buf, const std::vector<MirSec> &secs,
			    size_t si, uint64_t upto, int64_t rev0)
{
	for (size_t k = si + 1; k-- > 0;) {
		const MirSec &s_ = secs[k];
		const uint64_t n = k == si ? upto : s_.n;
		for (uint64_t i = n; i-- > 0;) {
			const uint8_t *r = &buf[s_.off + i * s_.rec];
			switch (s_.tag) {
			case MIR_IPC: {
				cgpu_ipcache_key key;
				memcpy(&key, r, 24);
				cgpu_ipcache_delete(c, &key);
				break;
			}
			case MIR_POL: {
				uint32_t ep;
				cgpu_policy_key key;
				memcpy(&ep, r, 4);
				memcpy(&key, r + 4, 8);
				cgpu_policy_delete(c, ep, &key);
				break;
			}
			case MIR_CIDR: {
				uint32_t which;
				cgpu_cidr_key key;
				memcpy(&which, r, 4);
				memcpy(&key, r + 4, 20);
				cgpu_cidr_delete(c, (int)which, &key);
				break;
			}
			case MIR_EP: {
				cgpu_endpoint_key key;
				memcpy(&key, r, 20);
				cgpu_endpoint_delete(c, &key);
				break;
			}
			case MIR_LB4: {
				cgpu_lb4_key key;
				memcpy(&key, r, 8);
				cgpu_lb4_delete(c, &key);
				break;
			}
			case MIR_LB6: {
				cgpu_lb6_key key;
				memcpy(&key, r, 20);
				cgpu_lb6_delete(c, &key);
				break;
			}
			case MIR_LXC: {
				uint32_t ep;
				memcpy(&ep, r, 4);
				cgpu_lxc_delete(c, ep);
				break;
			}
			case MIR_REV: {
				std::lock_guard<std::mutex> g(c->mu);
				c->pf_revision = rev0;
				break;
			}
			case MIR_CT4: {
				cgpu_ct4_tuple key;
				memcpy(&key, r, 14);
				cgpu_ct4_delete(c, &key);
				break;
			}
			case MIR_CT6: {
				cgpu_ct6_tuple key;
				memcpy(&key, r, 38);
				cgpu_ct6_delete(c, &key);
				break;
			}
			}
		}
	}
}

CGPU_EXPORT int cgpu_mirror_restore(cgpu_ctx *c, const char *path)
{
	if (!c || !path)
		return fail(-EINVAL, "null argument");
	std::vector<uint8_t> buf;
	{
		FILE *f = fopen(path, "rb");
		if (!f)
			return fail(-ENOENT, "cannot open %s", path);
		uint8_t chunk[1 << 16];
		size_t got;
		while ((got = fread(chunk, 1, sizeof(chunk), f)) > 0)
			buf.insert(buf.end(), chunk, chunk + got);
		fclose(f);
	}
	if (buf.size() < 24 || memcmp(buf.data(), "CGPUMIR1", 8))
		return fail(-EINVAL, "%s is not a cgpu mirror snapshot", path);
	uint64_t want;
	memcpy(&want, &buf[buf.size() - 8], 8);
	if (fnv(1469598103934665603ull, buf.data(), buf.size() - 8) != want)
		return fail(-EINVAL, "%s: checksum mismatch (truncated or corrupted)", path);
	uint32_t version, nsec;
	memcpy(&version, &buf[8], 4);
	memcpy(&nsec, &buf[12], 4);
	if (version != 1)
		return fail(-EINVAL, "%s: snapshot version %u", path, version);
	{
		std::lock_guard<std::mutex> g(c->mu);
		bool empty = c->ipc.empty() && !c->pol_total && c->dyn4.empty() && c->dyn6.empty() &&
			     c->fix4.empty() && c->fix6.empty() && c->lxc.empty() && c->lb.empty() &&
			     c->lb6.empty() && c->lxcinfo.empty();
		for (CtMap *m : {&c->ct4, &c->ct6}) {
			if (int r = ct_pull(c, *m))
				return r;
			empty = empty && !m->live;
		}
		if (!empty)
			return fail(-EEXIST, "restore needs an empty context");
	}
	/* validate the section structure before applying anything */
	typedef MirSec Sec;
	std::vector<Sec> secs;
	size_t off = 16;
	const size_t end = buf.size() - 8;
	static const uint32_t recsz[] = {0, 32, 36, 24, 20, 20, 44, 36, 8, 70, 94};
	for (uint32_t i = 0; i < nsec; i++) {
		Sec s_;
		if (off + 16 > end)
			return fail(-EINVAL, "%s: truncated section header", path);
		memcpy(&s_.tag, &buf[off], 4);
		memcpy(&s_.rec, &buf[off + 4], 4);
		memcpy(&s_.n, &buf[off + 8], 8);
		s_.off = off + 16;
		if (s_.tag < MIR_IPC || s_.tag > MIR_CT6 || s_.rec != recsz[s_.tag] ||
		    s_.n > (end - s_.off) / s_.rec)
			return fail(-EINVAL, "%s: bad section %u", path, s_.tag);
		off = s_.off + s_.n * s_.rec;
		secs.push_back(s_);
	}
	if (off != end)
		return fail(-EINVAL, "%s: trailing bytes", path);
	/* capacities of this context against the snapshot's record counts: a
	 * context configured smaller than the one that saved the file is refused
	 * before anything is applied */
	{
		uint64_t cnt[MIR_CT6 + 1] = {};
		std::map<uint32_t, uint64_t> per_ep;
		for (const Sec &s_ : secs) {
			cnt[s_.tag] += s_.n;
			if (s_.tag == MIR_POL)
				for (uint64_t i = 0; i < s_.n; i++) {
					uint32_t ep;
					memcpy(&ep, &buf[s_.off + i * s_.rec], 4);
					per_ep[ep]++;
				}
		}
		const CgpuConfigCaps cap = config_caps(c);
		const struct {
			int tag;
			uint64_t max;
			const char *what;
		} lim[] = {{MIR_IPC, cap.ipcache, "ipcache_max"},   {MIR_EP, cap.endpoints, "endpoints_max"},
			   {MIR_LB4, cap.lb, "lb_max_entries (lb4)"}, {MIR_LB6, cap.lb, "lb_max_entries (lb6)"},
			   {MIR_CT4, cap.ct4, "ct_max"},              {MIR_CT6, cap.ct6, "ct6_max"}};
		for (const auto &l : lim)
			if (cnt[l.tag] > l.max)
				return fail(-E2BIG, "%s: %llu records exceed this context's %s (%llu)", path,
					    (unsigned long long)cnt[l.tag], l.what, (unsigned long long)l.max);
		for (const auto &kv : per_ep)
			if (kv.second > cap.policy_per_ep)
				return fail(-E2BIG, "%s: %llu policy keys of endpoint %u exceed policy_max_per_ep (%llu)",
					    path, (unsigned long long)kv.second, kv.first,
					    (unsigned long long)cap.policy_per_ep);
	}
	/* replay through the map calls (the listeners' path); a record that
	 * still fails (a per-family limit, a bad key) rolls every applied record
	 * back, so the context is empty again and the restore can be retried */
	int64_t rev0;
	{
		std::lock_guard<std::mutex> g(c->mu);
		rev0 = c->pf_revision;
	}
	for (size_t si = 0; si < secs.size(); si++) {
		const Sec &s_ = secs[si];
		for (uint64_t i = 0; i < s_.n; i++) {
			const uint8_t *r = &buf[s_.off + i * s_.rec];
			int rc = 0;
			switch (s_.tag) {
			case MIR_IPC: {
				cgpu_ipcache_key k;
				cgpu_remote_endpoint_info v;
				memcpy(&k, r, 24);
				memcpy(&v, r + 24, 8);
				rc = cgpu_ipcache_update(c, &k, &v, CGPU_NOEXIST);
				break;
			}
			case MIR_POL: {
				uint32_t ep;
				cgpu_policy_key k;
				cgpu_policy_entry e;
				memcpy(&ep, r, 4);
				memcpy(&k, r + 4, 8);
				memcpy(&e, r + 12, 24);
				rc = cgpu_policy_update(c, ep, &k, &e, CGPU_NOEXIST);
				break;
			}
			case MIR_CIDR: {
				uint32_t which;
				cgpu_cidr_key k;
				memcpy(&which, r, 4);
				memcpy(&k, r + 4, 20);
				rc = cgpu_cidr_update(c, (int)which, &k, CGPU_NOEXIST);
				break;
			}
			case MIR_EP: {
				cgpu_endpoint_key k;
				memcpy(&k, r, 20);
				rc = cgpu_endpoint_update(c, &k, CGPU_NOEXIST);
				break;
			}
			case MIR_LB4: {
				cgpu_lb4_key k;
				cgpu_lb4_service v;
				memcpy(&k, r, 8);
				memcpy(&v, r + 8, 12);
				rc = cgpu_lb4_update(c, &k, &v, CGPU_NOEXIST);
				break;
			}
			case MIR_LB6: {
				cgpu_lb6_key k;
				cgpu_lb6_service v;
				memcpy(&k, r, 20);
				memcpy(&v, r + 20, 24);
				rc = cgpu_lb6_update(c, &k, &v, CGPU_NOEXIST);
				break;
			}
			case MIR_LXC: {
				uint32_t ep;
				cgpu_lxc_info v;
				memcpy(&ep, r, 4);
				memcpy(&v, r + 4, 32);
				rc = cgpu_lxc_update(c, ep, &v);
				break;
			}
			case MIR_REV: {
				std::lock_guard<std::mutex> g(c->mu);
				memcpy(&c->pf_revision, r, 8);
				break;
			}
			case MIR_CT4: {
				cgpu_ct4_tuple k;
				cgpu_ct_entry v;
				memcpy(&k, r, 14);
				memcpy(&v, r + 14, 56);
				rc = cgpu_ct4_update(c, &k, &v, CGPU_NOEXIST);
				break;
			}
			case MIR_CT6: {
				cgpu_ct6_tuple k;
				cgpu_ct_entry v;
				memcpy(&k, r, 38);
				memcpy(&v, r + 38, 56);
				rc = cgpu_ct6_update(c, &k, &v, CGPU_NOEXIST);
				break;
			}
			}
			if (rc) {
				mirror_rollback(c, buf, secs, si, i, rev0);
				return rc;
			}
		}
	}
	return 0;
}

/* ======================================================================= */
/* L3 MapState compilation                               */
/* ======================================================================= */
/* validate a program + label sets (+ a MapState spec), upload them, run
 * the selector kernels and copy back allow bytes [ne][ni] and, with a spec,
 * the L4 identity bitmaps [n_filters][ceil(ni / 64)] */
static int l3_run(cgpu_ctx *c, const cgpu_l3_program *p, const cgpu_label_sets *eps,
		  const cgpu_label_sets *ids, uint32_t flags, const cgpu_mapstate_spec *ms,
		  uint8_t *allow_out, uint64_t *l4_out)
{
	if (c->device < 0)
		return fail(-ENODEV, "context has no device (host-only); no CPU path");
	if (!p->rule_clauses || !eps->offsets || !ids->offsets)
		return fail(-EINVAL, "null offsets");
	/* validate every index the kernels follow */
	for (uint32_t r = 0; r < p->n_rules; r++)
		if (p->rule_subject[r] >= p->n_selectors || p->rule_clauses[r] > p->rule_clauses[r + 1])
			return fail(-EINVAL, "rule %u out of range", r);
	if (p->rule_clauses[p->n_rules] > p->n_clauses)
		return fail(-EINVAL, "clause offsets past n_clauses");
	for (uint32_t k = 0; k < p->n_clauses; k++)
		if (p->clauses[k].selector >= p->n_selectors || p->clauses[k].dir > 1 || p->clauses[k].kind > 1)
			return fail(-EINVAL, "clause %u out of range", k);
	for (uint32_t k = 0; k < p->n_selectors; k++)
		if ((uint64_t)p->selectors[k].reqs_off + p->selectors[k].n_reqs > p->n_reqs)
			return fail(-EINVAL, "selector %u out of range", k);
	for (uint32_t k = 0; k < p->n_reqs; k++)
		if ((uint64_t)p->reqs[k].values_off + p->reqs[k].n_values > p->n_values || p->reqs[k].op > 3)
			return fail(-EINVAL, "requirement %u out of range", k);
	const uint32_t ne = eps->n_sets, ni = ids->n_sets;
	for (uint32_t k = 0; k < ne; k++)
		if (eps->offsets[k] > eps->offsets[k + 1])
			return fail(-EINVAL, "endpoint label offsets not monotone");
	for (uint32_t k = 0; k < ni; k++)
		if (ids->offsets[k] > ids->offsets[k + 1])
			return fail(-EINVAL, "identity label offsets not monotone");
	const uint32_t nf = ms ? ms->n_filters : 0;
	for (uint32_t k = 0; k < nf; k++) {
		const cgpu_l4_filter &F = ms->filters[k];
		if (F.endpoint >= ne || F.dir > 1 || (uint64_t)F.sels_off + F.n_sels > ms->n_filter_sels)
			return fail(-EINVAL, "filter %u out of range", k);
	}
	for (uint32_t k = 0; ms && k < ms->n_filter_sels; k++)
		if (ms->filter_sels[k] >= p->n_selectors)
			return fail(-EINVAL, "filter selector %u out of range", k);
	if (!ne || !ni)
		return 0;
	const size_t nel = eps->offsets[ne], nil = ids->offsets[ni];
	const size_t nw = ((size_t)ni + 63) / 64;
	/* one device buffer: program, label sets, subject bits, results */
	size_t off = 0;
	auto take = [&](size_t b) { size_t o = off; off += (b + 255) & ~(size_t)255; return o; };
	const size_t o_sel = take(sizeof(cgpu_selector) * p->n_selectors);
	const size_t o_req = take(sizeof(cgpu_requirement) * p->n_reqs);
	const size_t o_val = take(4ull * p->n_values);
	const size_t o_rs = take(4ull * p->n_rules);
	const size_t o_rc = take(4ull * (p->n_rules + 1));
	const size_t o_cl = take(sizeof(cgpu_l3_clause) * p->n_clauses);
	const size_t o_eo = take(4ull * (ne + 1)), o_io = take(4ull * (ni + 1));
	const size_t o_el = take(sizeof(cgpu_label) * nel), o_il = take(sizeof(cgpu_label) * nil);
	const size_t o_subj = take((size_t)ne * p->n_rules), o_allow = take((size_t)ne * ni);
	const size_t o_ef = take(ms ? 4ull * ne : 0), o_ft = take(sizeof(cgpu_l4_filter) * nf);
	const size_t o_fs = take(ms ? 4ull * ms->n_filter_sels : 0), o_l4 = take(8ull * nf * nw);
	std::lock_guard<std::mutex> g(c->mu);
	HIP_OR_EIO(hipSetDevice(c->device));
	uint8_t *d = nullptr;
	HIP_OR_EIO(hipMalloc((void **)&d, off));
	auto up = [&](size_t o, const void *src, size_t b) {
		return b ? hipMemcpy(d + o, src, b, hipMemcpyHostToDevice) : hipSuccess;
	};
	hipError_t e = hipSuccess;
	if ((e = up(o_sel, p->selectors, sizeof(cgpu_selector) * p->n_selectors)) == hipSuccess &&
	    (e = up(o_req, p->reqs, sizeof(cgpu_requirement) * p->n_reqs)) == hipSuccess &&
	    (e = up(o_val, p->values, 4ull * p->n_values)) == hipSuccess &&
	    (e = up(o_rs, p->rule_subject, 4ull * p->n_rules)) == hipSuccess &&
	    (e = up(o_rc, p->rule_clauses, 4ull * (p->n_rules + 1))) == hipSuccess &&
	    (e = up(o_cl, p->clauses, sizeof(cgpu_l3_clause) * p->n_clauses)) == hipSuccess &&
	    (e = up(o_eo, eps->offsets, 4ull * (ne + 1))) == hipSuccess &&
	    (e = up(o_io, ids->offsets, 4ull * (ni + 1))) == hipSuccess &&
	    (e = up(o_el, eps->labels, sizeof(cgpu_label) * nel)) == hipSuccess &&
	    (e = up(o_il, ids->labels, sizeof(cgpu_label) * nil)) == hipSuccess &&
	    (!ms || ((e = up(o_ef, ms->ep_flags, 4ull * ne)) == hipSuccess &&
		     (e = up(o_ft, ms->filters, sizeof(cgpu_l4_filter) * nf)) == hipSuccess &&
		     (e = up(o_fs, ms->filter_sels, 4ull * ms->n_filter_sels)) == hipSuccess))) {
		l3_launch L{reinterpret_cast<const cgpu_selector *>(d + o_sel),
			    reinterpret_cast<const cgpu_requirement *>(d + o_req),
			    reinterpret_cast<const uint32_t *>(d + o_val),
			    reinterpret_cast<const uint32_t *>(d + o_rs),
			    reinterpret_cast<const uint32_t *>(d + o_rc), p->n_rules,
			    reinterpret_cast<const cgpu_l3_clause *>(d + o_cl),
			    reinterpret_cast<const uint32_t *>(d + o_eo), reinterpret_cast<const uint32_t *>(d + o_io),
			    reinterpret_cast<const cgpu_label *>(d + o_el), reinterpret_cast<const cgpu_label *>(d + o_il),
			    ne, ni, flags, d + o_subj, d + o_allow,
			    ms ? reinterpret_cast<const uint32_t *>(d + o_ef) : nullptr,
			    reinterpret_cast<const cgpu_l4_filter *>(d + o_ft),
			    reinterpret_cast<const uint32_t *>(d + o_fs), nf,
			    nf ? reinterpret_cast<uint64_t *>(d + o_l4) : nullptr};
		if ((e = launch_l3_compile(L, nullptr)) == hipSuccess && (e = hipDeviceSynchronize()) == hipSuccess &&
		    (e = hipMemcpy(allow_out, d + o_allow, (size_t)ne * ni, hipMemcpyDeviceToHost)) == hipSuccess &&
		    nf)
			e = hipMemcpy(l4_out, d + o_l4, 8ull * nf * nw, hipMemcpyDeviceToHost);
	}
	(void)hipFree(d);
	if (e != hipSuccess)
		return fail(-EIO, "L3/L4 selector kernels: %s", hipGetErrorString(e));
	return 0;
}

CGPU_EXPORT int cgpu_l3_compile(cgpu_ctx *c, const cgpu_l3_program *p, const cgpu_label_sets *eps,
				const cgpu_label_sets *ids, uint32_t flags, uint8_t *allow_out)
{
	if (!c || !p || !eps || !ids || (!allow_out && eps->n_sets && ids->n_sets))
		return fail(-EINVAL, "null argument");
	return l3_run(c, p, eps, ids, flags, nullptr, allow_out, nullptr);
}

static inline uint64_t ms_key(uint32_t id, uint16_t dport_host, uint8_t proto, uint8_t dir)
{
	cgpu_policy_key k{id, __builtin_bswap16(dport_host), proto, dir};
	return pol_key64(&k);
}

CGPU_EXPORT int cgpu_mapstate_sync(cgpu_ctx *c, const cgpu_l3_program *p, const cgpu_label_sets *eps,
				   const cgpu_label_sets *ids, const cgpu_mapstate_spec *ms,
				   cgpu_mapstate_stats *stats)
{
	if (!c || !p || !eps || !ids || !ms)
		return fail(-EINVAL, "null argument");
	const uint32_t ne = eps->n_sets, ni = ids->n_sets;
	if (ne && (!ms->ep_map || !ms->ep_flags))
		return fail(-EINVAL, "null endpoint arrays");
	if (ni && !ms->identity)
		return fail(-EINVAL, "null identity array");
	if ((ms->n_filters && !ms->filters) || (ms->n_filter_sels && !ms->filter_sels))
		return fail(-EINVAL, "null filter arrays");
	for (uint32_t k = 0; k < ne; k++)
		if (ms->ep_map[k] >= c->cfg.max_endpoints)
			return fail(-EINVAL, "endpoint row %u: map %u >= max_endpoints", k, ms->ep_map[k]);
	const size_t nw = ((size_t)ni + 63) / 64;
	std::vector<uint8_t> allow((size_t)ne * ni);
	std::vector<uint64_t> l4((size_t)ms->n_filters * nw);
	if (int r = l3_run(c, p, eps, ids, 0, ms, allow.data(), l4.data()))
		return r;
	std::vector<std::vector<uint32_t>> ep_filters(ne);
	for (uint32_t f = 0; f < ms->n_filters; f++)
		ep_filters[ms->filters[f].endpoint].push_back(f);
	cgpu_mapstate_stats st{};
	int first_err = 0;
	std::map<uint64_t, uint16_t> want; /* key -> proxy port (network order) */
	std::vector<uint64_t> drop;
	for (uint32_t e = 0; e < ne; e++) {
		/* computeDesiredPolicyMapState (policy.go:273-280), in its order */
		want.clear();
		for (uint32_t f : ep_filters[e]) {
			const cgpu_l4_filter &F = ms->filters[f];
			if (F.redirect && F.proxy_port == 0)
				continue;
			const uint64_t *bits = &l4[(size_t)f * nw];
			for (size_t w = 0; w < nw; w++)
				for (uint64_t b = bits[w]; b; b &= b - 1) {
					const size_t i = w * 64 + (size_t)__builtin_ctzll(b);
					want[ms_key(ms->identity[i], F.port, F.proto, F.dir)] =
						F.redirect ? __builtin_bswap16(F.proxy_port) : (uint16_t)0;
				}
		}
		const uint32_t fl = ms->ep_flags[e];
		if (fl & CGPU_MS_ALLOW_LOCALHOST) {
			want[ms_key(1 /* HOST_ID */, 0, 0, 0)] = 0;
			if (fl & CGPU_MS_HOST_ALLOWS_WORLD)
				want[ms_key(2 /* WORLD_ID */, 0, 0, 0)] = 0;
		}
		const uint8_t *row = &allow[(size_t)e * ni];
		for (uint32_t i = 0; i < ni; i++) {
			if (row[i] & 1)
				want[ms_key(ms->identity[i], 0, 0, 0)] = 0;
			if (row[i] & 2)
				want[ms_key(ms->identity[i], 0, 0, 1)] = 0;
		}
		st.desired += want.size();
		/* syncPolicyMap (endpoint.go:2572-2652): deletes first, then adds */
		const uint32_t m = ms->ep_map[e];
		std::lock_guard<std::mutex> g(c->mu);
		auto &cur = c->pol[m];
		drop.clear();
		for (auto &kv : cur)
			if (!want.count(kv.first))
				drop.push_back(kv.first);
		for (uint64_t k : drop) {
			pol_erase(c, m, cur, cur.find(k));
			st.deleted++;
		}
		for (auto &kv : want) {
			auto it = cur.find(kv.first);
			if (it != cur.end() && it->second.proxy_port == kv.second) {
				st.unchanged++;
				continue;
			}
			const bool had = it != cur.end();
			cgpu_policy_key k;
			memcpy(&k, &kv.first, 8);
			cgpu_policy_entry v{};
			v.proxy_port = kv.second;
			if (int r = pol_update_locked(c, m, &k, &v, CGPU_ANY)) {
				st.failed++;
				if (!first_err)
					first_err = r;
			} else {
				(had ? st.updated : st.added)++;
			}
		}
	}
	if (stats)
		*stats = st;
	return first_err;
}
