/*
 * Device-resident table layouts (HBM) shared by the host compiler
 * (host.cpp) and the gfx950 kernels (kernels.hip).  See DESIGN.md §3.
 *
 * All tables of one committed snapshot live in ONE hipMalloc'd arena; the
 * snapshot descriptor below holds device pointers into it and is passed to
 * kernels by value (kernarg), so a launch never dereferences host memory.
 */
#ifndef CGPU_TABLES_H
#define CGPU_TABLES_H

#include <stdint.h>

/* ---- DIR-24-8 entry encoding (host.cpp builds a DIR-24-8 image per LPM
 * table and compiles it into the compressed lpm16c form below) ----
 * tbl24[addr >> 8] (2^24 u32 = 64 MiB) and 256-entry tbl8 groups for
 * prefixes longer than /24.  Entry encoding (u32):
 *   0                      no match (NULL from map_lookup_elem)
 *   0b01 << 30 | label     match, sec_label < 2^30 stored inline
 *   0b10 << 30 | group     descend into tbl8[group * 256 + (addr & 255)]
 *   0b11 << 30 | idx       match, sec_label = vals[idx] (labels >= 2^30)
 * tbl8 entries never hold the group form.  A tombstone (sec_label 0) is a
 * match (0x40000000): it shadows shorter prefixes exactly as the kernel LPM
 * trie does (pkg/maps/ipcache/ipcache.go:182-194). */
#define DIR_TAG_SHIFT 30u
#define DIR_TAG_MASK (3u << DIR_TAG_SHIFT)
#define DIR_TAG_DIRECT (1u << DIR_TAG_SHIFT)
#define DIR_TAG_GROUP (2u << DIR_TAG_SHIFT)
#define DIR_TAG_INDIRECT (3u << DIR_TAG_SHIFT)
#define DIR_PAYLOAD_MASK ((1u << DIR_TAG_SHIFT) - 1u)
#define DIR_TBL24_ENTRIES (1u << 24)

/* ---- compressed IPv4 longest-prefix table (L2-resident ipcache) ----
 * The same function as a DIR-24-8 image (it is compiled FROM one), in ~1/50 of the
 * bytes, so that it stays in every XCD's 4 MiB L2 instead of being served
 * from the Infinity Cache.  d16[addr >> 16] holds a DIR entry (0 / direct /
 * indirect leaf, DIR encoding) or a GROUP reference
 *   bits 28..29 kind, bits 0..27 offset in 16-byte units into `nodes`:
 *   kind 0/1/2: a run node of 16 / 32 / 64 bytes over the low 16 bits (or,
 *               below an array, the low 8 bits) x of the address:
 *               NB = 1 / 2 / 5 words of u16 run starts b_1 < .. < b_2NB
 *               (unused ones 0xFFFF, whose value repeats the last), then
 *               2NB + 1 u32 leaf values; result = value[#{i : b_i <= x}]
 *   kind 3:     an array of 256 u32 entries indexed by the next address
 *               byte; an entry is a leaf, a run node (kind 0..2) over the
 *               last byte, or (below d16 only) another kind-3 array of 256
 *               leaves (the last byte, like a tbl8 group).
 * Leaves use the DIR entry encoding and share its `vals`. */
#define LPMC_KIND_SHIFT 28u
#define LPMC_OFF_MASK ((1u << LPMC_KIND_SHIFT) - 1u)
#define LPMC_MAX_RUN_BOUNDS 10u

/* x16[addr >> 16]: a 16-byte INLINE run node per /16, so that most lookups
 * are ONE 16-byte gather from a 1 MiB table:
 *   words 0..1: u16 run starts b_1..b_4 (unused 0xFFFF, value repeats)
 *   words 2..3: u64 V, code_i = (V >> 12 i) & 0xFFF for i = 0..4, the
 *               leaf of run i as an index into `dict` (kept in LDS);
 *               bit 63 set = overflow: word 0 is then a d16-style entry
 *               (leaf, or GROUP reference into `nodes`).
 * A /16 goes inline when it has <= 4 run starts and every leaf has a code
 * (the LPMC_DICT most frequent leaves get one). */
#define LPMC_DICT 4095u
#define LPMC_OVERFLOW (1u << 31)

typedef struct lpm16c {
	const uint32_t *d16;   /* 65536 entries; NULL = not compiled */
	const uint32_t *nodes; /* 16-byte aligned */
	const uint32_t *vals;
	const uint32_t *x16;   /* 65536 x 4 words (inline run nodes) */
	const uint32_t *dict;  /* leaf per code */
	uint32_t n_node_words;
	uint32_t n_dict;
} lpm16c;

/* 32-bit mixer of two words (hash tables below) */
static inline __host__ __device__ uint32_t mix32(uint32_t a, uint32_t b)
{
	uint64_t h = ((uint64_t)b << 32 | a) * 0x9E3779B97F4A7C15ull;
	h ^= h >> 29;
	h *= 0xbf58476d1ce4e5b9ull;
	h ^= h >> 32;
	return (uint32_t)h;
}

/* ---- policy hash: one open-addressing table for all endpoints ----
 * 16-byte slots {x = sec_label, y = dport | proto << 16 | egress_pad << 24,
 * z = ep | proxy_port << 16, w = counter slot | hop << 24}.  (x, y) is the
 * raw 8-byte policy_key, compared whole like the kernel htab memcmp (pad
 * bits included).  Neighbourhood ("hop") hashing: a key lives within
 * POL_HOP slots of its home slot h = pol_hash(key, ep) & mask; w bits 0..23
 * hold the counter slot (POL_CTR_EMPTY = empty slot) and bit 24 + j of home
 * slot h says "slot h + j holds a key whose home is h".  A lookup loads the
 * home slot (one 16-byte gather): hop == 0 is a miss, bit 0 + key match a
 * hit; only other set bits cost further loads.  Kept at <= 50 % load; a
 * commit patches keys in place (host.cpp pol_patch) or rebuilds. */
#define POL_HOP 8u
#define POL_HOP_SHIFT 24u
#define POL_CTR_MASK 0x00FFFFFFu
#define POL_CTR_EMPTY POL_CTR_MASK

typedef struct pol_slot {
	uint32_t key_lo;  /* sec_label */
	uint32_t key_hi;  /* dport | protocol << 16 | egress_pad << 24 */
	uint32_t ep_proxy;/* ep | proxy_port << 16 */
	uint32_t ctr;     /* counter slot | hop << 24 (POL_CTR_EMPTY: free) */
} pol_slot;

typedef struct pol_table {
	const pol_slot *slots; /* bucket_mask + 1 slots */
	uint32_t bucket_mask;
	uint32_t pad_;
} pol_table;

/* ---- policy groups: one 16-B slot per (endpoint, identity, direction) ----
 * The reference's cascade (bpf/lib/policy.h:46-110) keys probe 1 and probe 2
 * on the same {identity, direction} of one endpoint's map: probe 2 is the
 * L3-only key {id, 0, 0, dir}, probe 1 the exact {id, dport, proto, dir}.
 * A group slot answers probe 2 directly (the L3 key's counter slot) and
 * filters probe 1 with a bloom over the (dport, proto) of the group's keys,
 * so the exact-key table is gathered only when a key may exist:
 *   x = sec_label, y = ep | egress << 16 | PG_USED | hop << 24,
 *   z = counter slot of the L3 key (POL_CTR_EMPTY: none), w = bloom.
 * Neighbourhood hashing as the policy table.  Only keys with pad bits 0 are
 * grouped (a datapath lookup key always has pad 0).  A bloom bit is never
 * cleared by a delete (a stale bit costs one exact probe, never a verdict);
 * a full rebuild recomputes them. */
#define PG_EGRESS (1u << 16)
#define PG_USED (1u << 17)

typedef struct pol_groups {
	const uint4 *slots; /* mask + 1 slots */
	uint32_t mask;
	uint32_t pad_;
} pol_groups;

static inline __host__ __device__ uint32_t pg_hash(uint32_t id, uint32_t ep_dir)
{
	return mix32(id, ep_dir ^ 0x6a09e667u);
}

/* the two bloom bits of a (network-order dport, proto) pair */
static inline __host__ __device__ uint32_t pg_bloom(uint32_t dport, uint32_t proto)
{
	const uint32_t h = mix32(dport | proto << 16, 0x3c6ef372u);
	return (1u << (h & 31u)) | (1u << ((h >> 8) & 31u));
}

static inline __host__ __device__ uint32_t pol_hash(uint32_t key_lo, uint32_t key_hi, uint32_t ep)
{
	uint64_t h = ((uint64_t)key_hi << 32 | key_lo) ^ ((uint64_t)ep * 0x9E3779B97F4A7C15ull);
	h ^= h >> 33;
	h *= 0xff51afd7ed558ccdull;
	h ^= h >> 33;
	h *= 0xc4ceb9fe1a85ec53ull;
	h ^= h >> 33;
	return (uint32_t)h;
}

/* ---- exact address sets (cilium_lxc endpoints) ----
 * v4: 64-byte buckets of 8 x {addr_be, used}; v6: 64-byte buckets of
 * 2 x {addr[16], used, pad[3]} (32-byte slots). */
typedef struct set4_slot {
	uint32_t addr;
	uint32_t used;
} set4_slot;

typedef struct set16_slot {
	uint32_t a[4];
	uint32_t used; /* bit0 used; bits 8..15 = prefix length for prefix sets */
	uint32_t pad[3];
} set16_slot;

typedef struct addr_set4 {
	const set4_slot *slots; /* n_buckets * 8 */
	uint32_t bucket_mask;
	uint32_t max_probe;
} addr_set4;

typedef struct addr_set16 {
	const set16_slot *slots; /* n_buckets * 2 */
	uint32_t bucket_mask;
	uint32_t max_probe;
} addr_set16;

static inline __host__ __device__ uint32_t hash16(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3,
						  uint32_t salt)
{
	return mix32(mix32(a0, a1) ^ salt, mix32(a2, a3));
}

/* ---- IPv6 prefix keys of v6_lpm ----
 * A prefix is keyed by its address as four host-order words (w0 = address
 * bits 0..31), masked to its length, plus the length.  The hash is a
 * multiply-sum over the words and the length with one 32-bit finalizer, so a
 * lookup trying many lengths of one address recomputes only the word the
 * length cuts (kernels.hip v6_next) instead of a full 16-byte hash. */
#define PFX6_C0 0x9E3779B1u
#define PFX6_C1 0x85EBCA77u
#define PFX6_C2 0xC2B2AE3Du
#define PFX6_C3 0x27D4EB2Fu
#define PFX6_CL 0x165667B1u

static inline __host__ __device__ uint32_t fmix32(uint32_t h)
{
	h ^= h >> 16;
	h *= 0x85ebca6bu;
	h ^= h >> 13;
	h *= 0xc2b2ae35u;
	h ^= h >> 16;
	return h;
}

static inline __host__ __device__ uint32_t pfx6_hash(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3,
						     uint32_t len)
{
	return fmix32(w0 * PFX6_C0 + w1 * PFX6_C1 + w2 * PFX6_C2 + w3 * PFX6_C3 + len * PFX6_CL);
}

/* ---- IPv6 longest-prefix trie (ipcache v6, ipcache_lookup6 eps.h:56-66) ----
 * Strides 16 / 8 / 8 over address bits 0..31, labelled interval lines over
 * bits 32..63, hashed /64 records for the prefixes longer than /64.  The
 * entries use the DIR encoding: a leaf (0 / DIRECT / INDIRECT) is the
 * highest-ranked prefix covering the entry's whole range, by controlled prefix
 * expansion in rank order; GROUP descends.
 *   root[bits 0..15], b24[blk * 256 + bits 16..23]: u32, leaf or GROUP | blk;
 *   b32[blk * 256 + bits 24..31]: uint2, {leaf, 0} or the /32's node
 *     {GROUP | deep << 29 | line, base | (w - 9) | s << 5}.
 * A node is the /32's labelled intervals over x = bits 32..63 (prefixes /33..
 * /64, the /32's own leaf where none covers x): every boundary (a point where
 * the label changes) lies in the window [base, base + 2^w), w >= 9, outside
 * of which the label is the line's `outer`; the window is cut into 2^s equal
 * sub-ranges (the least s that fits), one 128-B line each:
 *   slots 0..14  b - 1 for each boundary b inside the sub-range (not at its
 *                start), ascending, 0xFFFFFFFF past the last
 *   slot 15      outer
 *   slots 16..31 label of region r = #{slot i < x, i < 15}
 * so a lookup reads one line: four 16-B loads and one label word.
 * s = 7 (V6T_LONG: even 64 sub-ranges do not fit): line {n, .., slot 15 =
 * outer} then n boundaries (b - 1) and n + 1 labels from the next line on,
 * binary-searched (no window).
 * deep: the /32 holds prefixes longer than /64, in h64, a hop hash over the
 * /64 (home = mix32(w0, w1), 32-B slots {w0, w1, lbl, used | hop << 24, lo.hi,
 * lo.lo, hi.hi, hi.lo}): lbl a leaf = the label of low-64 x in [lo, hi];
 * lbl = GROUP | off: a list at pool[4 * off] {n, 0, 0, 0}, n boundaries (hi,
 * lo words), n + 1 labels.  V6T_FALL where no /65+ prefix covers x: the node's
 * label stands. */
#define V6T_LONG 7u
#ifndef CGPU_V6T_NB
#define CGPU_V6T_NB 15
#endif
/* boundaries per node line (15: 128-B lines as above; 7: 64-B lines of 7
 * boundaries, outer, 8 labels: the label is in the registers the count
 * read) */
#define V6T_NB ((uint32_t)CGPU_V6T_NB)
#define V6T_LW (2u * (V6T_NB + 1u)) /* line words */
#define V6T_FALL DIR_TAG_GROUP
#define V6T_RBITS_WORDS (2048u + 1024u) /* GROUP bitmap of the root, u16 ranks */
#define V6T_DEEP (1u << 29)
#define V6T_LINE_MASK (V6T_DEEP - 1u)

typedef struct v6_lpm {
	const uint32_t *root;  /* 65536 entries; NULL = empty table */
	const uint32_t *b24;
	const uint2 *b32;
	const uint32_t *pool;  /* 128-B lines (node32) and 16-B units (lists) */
	const uint32_t *vals;  /* indirect labels (>= 2^30) */
	const uint4 *h64;      /* (m64 + 1) x 2 uint4 */
	uint32_t m64;
	/* LDS-staged forms (k_classify_x4): rbits = the root's GROUP bitmap
	 * (2048 words) and u16 ranks (GROUP entries before word k: the b24
	 * block, blocks being appended in root order); b24_16 = every b24 entry
	 * as u16: 0x8000 | b32 block for GROUP, 0 for a leaf (read b24);
	 * NULL when not representable */
	const uint32_t *rbits;
	const uint16_t *b24_16;
	uint32_t n_b24;        /* b24 blocks */
	/* blocked bloom filter of the /64s that hold h64 records (v6_bloom_word /
	 * v6_bloom_bits over mix32 of the /64's words), staged in LDS by the
	 * lookup pre-pass: a lookup whose /64 misses it skips the h64 probe */
	const uint32_t *bl64;
	uint32_t bl64_mask;    /* words - 1 */
} v6_lpm;

#define V6T_BLOOM_MAX_WORDS 16384u /* 64 KiB */

#define EP6_BLOOM_MAX_WORDS 8192u /* 32 KiB: staged in LDS by k_prefilter_v6_q */

static inline __host__ __device__ uint32_t v6_bloom_word(uint32_t h, uint32_t mask) { return (h >> 16) & mask; }
static inline __host__ __device__ uint32_t v6_bloom_bits(uint32_t h)
{
	const uint32_t g = h * 0x2545F491u;
	return (1u << ((g >> 17) & 31u)) | (1u << ((g >> 22) & 31u)) | (1u << (g >> 27));
}

/* ---- service map (cilium_lb4_services, bpf/lib/lb.h:70-76) ----
 * Grouped by frontend {address, dport}: one 16-byte frontend slot per
 * frontend in a single-slot neighbourhood hash (POL_HOP scheme, hop bits
 * 24..31 of w), and the frontend's backends in a dense array:
 *   fe: x = address, y = dport | master_count << 16, z = base (index in `be`
 *       of slave 1), w = nslaves (bits 0..15) | LB_FE_USED | hop << 24.
 *       master_count = count of the slave-0 entry, 0 when there is none:
 *       slave 0 is only ever read by lb4_lookup_service, which treats count
 *       0 and "no entry" alike (lb.h:613-629).
 *   be[base + s - 1], s = 1..nslaves: {target, port | count << 16,
 *       rev_nat_index | weight << 16, present}.
 * A service lookup is one 16-byte gather (the frontend slot, usually its
 * home slot) and a backend lookup one more, dependent, 16-byte gather. */
#define LB_FE_USED (1u << 16)
/* the frontend has a slave-0 (master) entry, stored as a full row at
 * be[base + nslaves]: read only by the stateful service step, where a stored
 * CT_SERVICE entry may name slave 0 (lb4_lookup_slave, lb.h:637-651) */
#define LB_FE_MASTER (1u << 17)

typedef struct lb_table {
	const uint4 *fe; /* fe_mask + 1 slots, never NULL once committed */
	const uint4 *be;
	uint32_t fe_mask;
	uint32_t n_be;
	/* presence bitmap over the frontend ADDRESSES (bit lb_vip_bit(addr) &
	 * vip_mask set for every frontend, any dport): a clear bit proves both
	 * the L4 and the L3 key of that daddr are absent, so a tuple aimed at no
	 * service skips its frontend probes.  ~8 bits per frontend (1 MiB at 1M
	 * services) so it mostly stays in L2 while the 32-MiB frontend table
	 * does not. */
	const uint32_t *vip;
	uint32_t vip_mask;
} lb_table;

static inline __host__ __device__ uint32_t lb_vip_bit(uint32_t addr)
{
	return mix32(addr, 0x5f1b7e11u);
}

static inline __host__ __device__ uint32_t lb_hash(uint32_t addr, uint32_t dport)
{
	return mix32(addr, dport ^ 0x1b5e0000u);
}

/* cgpu_flow_hash (include/cgpu.h): murmur3 finalizer over the stored
 * 5-tuple, = cilium_amd/shard.py flowhash_np */
static inline __host__ __device__ uint32_t flow_hash(uint32_t saddr, uint32_t daddr, uint32_t sport,
						     uint32_t dport, uint32_t proto)
{
	uint32_t h = saddr * 0x9E3779B1u;
	h ^= daddr;
	h *= 0x85EBCA77u;
	h ^= (sport << 16) | dport;
	h *= 0xC2B2AE3Du;
	h ^= proto;
	h ^= h >> 16;
	h *= 0x85EBCA6Bu;
	h ^= h >> 13;
	h *= 0xC2B2AE35u;
	h ^= h >> 16;
	return h;
}

/* ---- IPv6 service map (cilium_lb6_services, bpf/lib/lb.h:46-52) ----
 * The lb4 scheme with 32-byte rows: frontend slot = 2 x uint4
 *   {address (raw words)}, {dport | master_count << 16, base, nslaves | LB_FE_USED | hop << 24, 0}
 * backend row = 2 x uint4 {target (raw words)}, {port | count << 16, rev_nat | weight << 16, present, 0}.
 * A service lookup is one 32-byte gather (the home slot), a backend one more. */
typedef struct lb6_table {
	const uint4 *fe; /* (fe_mask + 1) x 2 */
	const uint4 *be; /* n_be x 2 */
	uint32_t fe_mask;
	uint32_t n_be;
	const uint32_t *vip; /* presence bitmap over frontend addresses (lb6_vip_bit) */
	uint32_t vip_mask;
} lb6_table;

/* 16 address bytes (as four little-endian words) -> 32 bits */
static inline __host__ __device__ uint32_t fold6(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3)
{
	return fmix32(w0 ^ fmix32(w1 ^ fmix32(w2 ^ fmix32(w3 ^ 0x6B43A9B5u))));
}

static inline __host__ __device__ uint32_t lb6_hash(uint32_t f, uint32_t dport)
{
	return mix32(f, dport ^ 0x6d5e0000u);
}

static inline __host__ __device__ uint32_t lb6_vip_bit(uint32_t f)
{
	return mix32(f, 0x2f6b1e17u);
}

/* ---- IPv6 any-match cover (XDP prefilter v6) ----
 * The prefilter only asks "does ANY deny prefix cover saddr" (bpf_xdp.c:
 * 142-152: both the dyn LPM and the fix /128 hash lead to XDP_DROP), so the
 * union of the prefixes is compiled into a multibit trie of strides
 * 16 / 8 / 8 with covered intervals below /32:
 *   root[bits 0..15] -> b24[block * 256 + bits 16..23] -> b32[block * 256 +
 *   bits 24..31]: direct-indexed u32 entries; prefixes of /17../32 are
 *   expanded into the entries they cover (an any-match set has no
 *   priorities, so expansion is exact).  b32 entries of /32s holding
 *   longer prefixes are NODEs (node32, host.cpp cover6_node32): 2^s
 *   128-B lines, one per equal sub-range of bits 32..63, each 32 slots of
 *   b - 1 for the boundaries b of the merged covered intervals in its
 *   sub-range (plus S - 1 when an odd number lie below its start S),
 *   0xFFFFFFFF past the last; x is covered iff (flip, in sub-range 0) +
 *   #(slot < x) over x's line is odd.  The b32 entry carries code << 25 |
 *   line, code = flip | deep << 1 | s << 2 (s = COVER6_LONG: a header unit
 *   {nb, 0, 0, 0} + every boundary, scanned whole); deep: the /32 has h64
 *   records, so an uncovered x consults h64.
 *   h64: hop-hashed 32-B slots {top64.hi, top64.lo, entry, used | hop << 24,
 *        lo.hi, lo.lo, hi.hi, hi.lo} for the /64s holding prefixes longer
 *        than /64 (an INLINE FULL entry covers [lo, hi] of the low 64 bits).
 * entry: tag << 30 | payload, tag COVER6_NONE / _FULL / _DEEP (root, b24:
 * payload = the next level's block; b32: consult h64) / _NODE (payload =
 * code << 25 | 128-B line of `pool`; in h64 records: offset in 16-B units).
 * Typical config-3 packet: root, b24, b32 (768 KiB together, L2-resident) +
 * one 128-B node + rarely one h64 slot. */
#define COVER6_NONE 0u
#define COVER6_FULL 1u
#define COVER6_DEEP 2u
#define COVER6_NODE 3u
#define COVER6_USED (1u << 16)
#define COVER6_LONG 7u /* node32 split code: header + boundaries, no split fits */
#define COVER6_RBITS_WORDS (2048u * 2u + 1024u) /* DEEP, FULL bitmaps + u16 ranks */

typedef struct cover6 {
	const uint32_t *root; /* 65536 entries; NULL = empty set */
	/* LDS-staged forms (k_prefilter_v6_q picks the deepest that fits):
	 * root16: the root as 65536 u16 (0 NONE, 1 FULL, 2 + b24 block);
	 * rbits + b24_16: the root as bitmaps {DEEP[2048], FULL[2048] words,
	 * rank[2048] u16 = DEEP bits before word k} and every b24 block as u16
	 * entries (0 NONE, 1 FULL, 2 + b32 block); NULL when not representable */
	const uint16_t *root16;
	const uint32_t *rbits;
	const uint16_t *b24_16;
	uint32_t n_b24;
	const uint32_t *b24;  /* 256-entry blocks */
	const uint32_t *b32;  /* 256-entry blocks */
	const uint32_t *pool; /* 16-B aligned nodes */
	const uint4 *h64;     /* (m64 + 1) x 2 uint4 */
	uint32_t m64;
} cover6;

/* ---- IPv4 any-match /16 nodes (the XDP deny set, cgpu_classify_v4_cascade) ----
 * pf4x[2 p], pf4x[2 p + 1]: the /16 p as the addresses x (its low 16 bits)
 * where coverage changes, b_1 < .. < b_k in [1, 0xFFFF], stored as b_i - 1
 * (u16, pad 0xFFFF): x is covered iff flip + #{i : b_i - 1 < x} is odd.
 *   u16 0 of the first uint4: header (PF4X_OVF: more than 15 boundaries,
 *         look the address up in pf4c; PF4X_TWO: slots 7..14 are used;
 *         bit 0: flip = coverage at x = 0)
 *   u16 1..7: slots 0..6;  the second uint4: slots 7..14.
 * A lookup is one 16-byte gather for a /16 of <= 7 boundaries (three /32s),
 * a second in the same line for <= 15. */
#define PF4X_OVF 0x8000u
#define PF4X_TWO 0x4000u

/* ---- one committed snapshot ---- */
typedef struct cgpu_snapshot {
	lpm16c ipc4c;    /* ipcache, IPv4 lookups (compiled from a host DIR-24-8) */
	pol_table pol;   /* every policy key (probe 1 / 3 gathers) */
	pol_groups pg;   /* per (ep, identity, dir): probe 2 + probe 1 filter */
	lpm16c pf4c;     /* any-match: dyn4 (if enabled) + fix4 /32; leaves 0 / 1 */
	const uint4 *pf4x; /* the same set as one 32-byte boundary node per /16 (PF4X_*), or NULL */
	addr_set4 ep4;   /* cilium_lxc IPv4 keys */
	addr_set16 ep6;  /* cilium_lxc IPv6 keys (bucket: pfx6_hash(raw words, 0)) */
	/* bloom filter over ep6 keys (v6_bloom_word / v6_bloom_bits of the same
	 * hash), staged in LDS by k_prefilter_v6_q: a daddr it rules out is no
	 * endpoint without a bucket read */
	const uint32_t *ep6_bloom;
	uint32_t ep6_bloom_mask;
	cover6 pf6;      /* any-match: dyn6 (if enabled) + fix6 /128 */
	v6_lpm ipc6;     /* ipcache, IPv6 lookups */
	uint32_t pf4_enabled; /* CIDR4_FILTER */
	uint32_t pf6_enabled; /* CIDR6_FILTER */
	/* config */
	uint32_t world_id, cluster_id, host_id, health_id;
	uint32_t ipv4_cluster_mask, ipv4_cluster_range;
	uint32_t router_ip64[2]; /* first 8 bytes of ROUTER_IP (ipv6_match_prefix_64) */
	uint32_t router_ip[4];   /* ROUTER_IP whole (handle_ipv6's ICMPv6 responders) */
	uint32_t ct_proto_gate, ingress_secctx_world, ingress_src_identity;
	uint32_t n_ctr_slots;
	uint32_t hot_slots;      /* counter slots [0, hot_slots) may live in LDS */
	uint32_t cold_hi;        /* counter slots >= cold_hi are unassigned */
	lb_table lb;
	lb6_table lb6;
	uint32_t lb_flags;       /* CGPU_LB_L3 | CGPU_LB_L4 */
	uint32_t ipv4_loopback;  /* IPV4_LOOPBACK, network order */
	/* per-endpoint lxc_config.h identity (cgpu_lxc_info, 32 B = 2 x uint4
	 * per endpoint id, dense over [0, n_lxc)) and NODE_MAC */
	const uint4 *lxc;
	uint32_t n_lxc;
	uint32_t node_mac_lo, node_mac_hi; /* bytes 0-3, 4-5 of NODE_MAC (LE words) */
	uint32_t schedule;       /* cgpu_config.schedule (CGPU_SCHED_*) */
	uint64_t epoch;
} cgpu_snapshot;

/* ---- conntrack map cilium_ct4_global ----
 * Open addressing with linear probing over nslots = 2^k >= 2 * max slots.
 * keys[slot] (16 B, one gather per probe) = the 14-byte struct ipv4_ct_tuple
 * (bpf/lib/common.h:359-366) plus a 16-bit slot tag in the top half of .w:
 *   .x daddr  .y saddr  .z dport | sport << 16  .w nexthdr | flags << 8 | tag << 16
 *   tag 0 empty, CT_TAG_LIVE occupied, CT_TAG_CLAIM being written, CT_TAG_TOMB
 *   deleted (probe chains run through it; inserts reuse it).
 * vals[slot] (64 B = 4 x uint4, one row per slot) = struct ct_entry
 * (common.h:380-408, 56 B) in its own byte layout, then 8 spare bytes.
 * The device table is authoritative after a batch: the walker kernel
 * inserts, updates and deletes entries in place. */
#define CT_TAG_EMPTY 0u
#define CT_TAG_LIVE 1u
#define CT_TAG_CLAIM 0xFFFEu
#define CT_TAG_TOMB 0xFFFFu

typedef struct ct_table {
	uint4 *keys;
	uint4 *vals;
	uint32_t mask;      /* nslots - 1 */
	uint32_t max;       /* CT_MAP_SIZE: live entries allowed */
	uint32_t *count;    /* [0] live entries, [1] tombstones */
	uint32_t res_chunk; /* capacity a workgroup reserves at a time (headroom-sized) */
	/* LRU mode (cgpu_config.ct_lru): a create that finds the map full evicts
	 * an entry none of the batch's packets can touch -- the batch's keys are
	 * in this bloom filter (bloom_mask + 1 words) -- instead of failing */
	const uint32_t *bloom;
	uint32_t bloom_mask;
	uint32_t lru;
} ct_table;

#if defined(__HIPCC__)
#define CT_HD __host__ __device__ __forceinline__
#else
#define CT_HD static inline
#endif

CT_HD uint32_t ct_fmix(uint32_t h)
{
	h ^= h >> 16;
	h *= 0x85ebca6bu;
	h ^= h >> 13;
	h *= 0xc2b2ae35u;
	h ^= h >> 16;
	return h;
}

/* home slot hash of a 14-byte tuple (tag bits excluded) */
CT_HD uint32_t ct_hash(uint32_t x, uint32_t y, uint32_t z, uint32_t w)
{
	uint32_t h = ct_fmix(x ^ 0x7f4a7c15u);
	h = ct_fmix(h ^ y);
	h = ct_fmix(h ^ z);
	return ct_fmix(h ^ (w & 0xFFFFu));
}

/* the conntrack group of a packet: every map key its ct_lookup4 /
 * ct_create4 / ct_delete4 touch has the same unordered address pair */
CT_HD uint32_t ct_group(uint32_t a, uint32_t b)
{
	const uint32_t lo = a < b ? a : b, hi = a < b ? b : a;
	return ct_fmix(ct_fmix(lo ^ 0x2545f491u) ^ hi);
}

/* the phase-1 conntrack group of a TCP / UDP packet on the plain path: its
 * connection (unordered address pair, unordered ports, protocol).  Every
 * key its ct_lookup / ct_create / ct_delete touch but the ICMP entry of
 * ct_create carries the connection; that entry is owed to phase 2, which
 * groups by address pair.  z = sport | dport << 16 of either direction. */
CT_HD uint32_t ct_conn_group(uint32_t pair_group, uint32_t z, uint32_t proto)
{
	const uint32_t a = z & 0xFFFFu, b = z >> 16;
	const uint32_t ports = a < b ? (a | b << 16) : (b | a << 16);
	return ct_fmix(pair_group ^ ct_fmix(ports ^ (proto << 24) ^ 0x68e31da4u));
}

/* Table verification sum (SURVEY §5 failure detection): over the 8-byte
 * words of every part of an uploaded group buffer, sum of word x an odd
 * multiplier that depends on the word's index in the buffer (a changed word
 * always changes the sum: odd multipliers are invertible mod 2^64).  The
 * host computes it over its image before the upload, the device over the
 * buffer it holds. */
CT_HD uint64_t table_sum_word(uint64_t w, uint64_t i)
{
	return w * ((i * 0x9E3779B97F4A7C15ull) | 1ull);
}

/* counters: u64 {packets, bytes} per policy slot, then metrics */
#define CGPU_METRICS_WORDS (256u * 4u * 2u)

#endif
