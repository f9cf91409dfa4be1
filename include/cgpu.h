/*
 * cgpu.h — C ABI of the MI355X flow-classification engine.
 *
 * Drop-in for the kernel-map boundary the reference's Go agent programs
 * through bpf(2) (pkg/bpf/bpf.go:153-245 UpdateElement / LookupElement /
 * DeleteElement / GetNextKey) and for the per-packet BPF datapath functions
 * that read those maps (bpf/lib/policy.h, bpf/lib/eps.h, bpf/bpf_xdp.c).
 * A Go package pkg/datapath/gpu binds this header through cgo (see
 * INTEGRATION.md); keys and values are the reference byte layouts so the Go
 * side passes unsafe.Pointer through unchanged, exactly as it does today.
 *
 * Conventions (mirroring bpf(2) as wrapped by pkg/bpf):
 *   - every function returns 0 or a negative errno:
 *       -ENOENT missing key, -EEXIST / -ENOENT for BPF_NOEXIST / BPF_EXIST,
 *       -E2BIG hash map full, -ENOSPC LPM map full, -EINVAL bad argument
 *       (prefixlen, family, flags), -ENODEV no GPU bound to the context,
 *       -EIO device error (details: cgpu_last_error()).
 *   - the caller owns every key/value/tuple buffer; the library copies.
 *   - table updates are thread-safe (one mutex on the host mirror) and become
 *     visible to classification only at cgpu_commit(), which publishes a new
 *     immutable device snapshot (epoch).  Classification launches read the
 *     latest published snapshot and never take the mirror lock: they run
 *     concurrently with updates and with commits (a launch pins the snapshot
 *     it started on; its buffers are freed only after its kernels finish).
 *     Like the reference (pkg/endpoint/bpf.go:459-465), a set of updates is
 *     not atomic unless it is committed at once.
 *   - batch entry points take DEVICE pointers (HBM-resident SoA columns) and
 *     a hipStream_t (passed as void*; NULL = the null stream).  They enqueue
 *     and return; results are ready when the stream reaches that point.
 *     There is no CPU execution path: without a device they fail -ENODEV.
 */
#ifndef CGPU_H
#define CGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CGPU_ABI_VERSION 2u

/* bpf(2) update flags (include/uapi/linux/bpf.h) */
#define CGPU_ANY 0u
#define CGPU_NOEXIST 1u
#define CGPU_EXIST 2u

/* ------------------------------------------------------------------ */
/* Reference byte layouts                                              */
/* ------------------------------------------------------------------ */

/* struct policy_key, bpf/lib/common.h:180-186; Go PolicyKey
 * (pkg/maps/policymap/policymap.go:63-68).  dport in network order.
 * egress_pad holds the bitfield byte {egress:1, pad:7}: bit 0 = egress. */
typedef struct cgpu_policy_key {
	uint32_t sec_label;
	uint16_t dport;
	uint8_t protocol;
	uint8_t egress_pad;
} cgpu_policy_key;

/* struct policy_entry, bpf/lib/common.h:188-193 (proxy_port network order) */
typedef struct cgpu_policy_entry {
	uint16_t proxy_port;
	uint16_t pad[3];
	uint64_t packets;
	uint64_t bytes;
} cgpu_policy_entry;

/* struct ipcache_key, bpf/lib/maps.h:135-148 (24 B, packed).  prefixlen
 * counts the 32 static bits {pad[3], family} plus the IP bits
 * (bpf/lib/eps.h:48-52; Go pkg/maps/ipcache/ipcache.go:72-98). */
typedef struct cgpu_ipcache_key {
	uint32_t prefixlen;
	uint8_t pad[3];
	uint8_t family; /* ENDPOINT_KEY_IPV4 = 1, ENDPOINT_KEY_IPV6 = 2 */
	uint8_t ip[16];
} cgpu_ipcache_key;

/* struct remote_endpoint_info, bpf/lib/common.h:175-178 */
typedef struct cgpu_remote_endpoint_info {
	uint32_t sec_label;
	uint32_t tunnel_endpoint;
} cgpu_remote_endpoint_info;

/* struct lpm_v4_key / lpm_v6_key, bpf/lib/xdp.h:23-31 (Go cidrKey,
 * pkg/maps/cidrmap/cidrmap.go:49-52, truncated to 4 + AddrSize bytes).
 * Only the first 4 (v4) or 16 (v6) bytes of addr are used. */
typedef struct cgpu_cidr_key {
	uint32_t prefixlen;
	uint8_t addr[16];
} cgpu_cidr_key;

/* struct endpoint_key, bpf/lib/common.h:147-160 (20 B, packed) */
typedef struct cgpu_endpoint_key {
	uint8_t ip[16];
	uint8_t family;
	uint8_t pad4;
	uint16_t pad5;
} cgpu_endpoint_key;

/* prefilter maps: pkg/policy/prefilter.go:33-39 preFilterMapType */
enum cgpu_cidr_map {
	CGPU_CIDR_V4_DYN = 0, /* LPM, bpf_xdp.c CIDR4_LMAP_NAME */
	CGPU_CIDR_V4_FIX = 1, /* exact hash, CIDR4_HMAP_NAME */
	CGPU_CIDR_V6_DYN = 2,
	CGPU_CIDR_V6_FIX = 3,
};

/* ------------------------------------------------------------------ */
/* Configuration: the compile-time #defines the agent writes into      */
/* node_config.h / lxc_config.h / filter_config.h become runtime fields */
/* ------------------------------------------------------------------ */
typedef struct cgpu_config {
	uint32_t abi_version;       /* = CGPU_ABI_VERSION */
	/* capacities (max_elem of the reference maps; device sizing) */
	uint32_t ipcache_max;       /* IPCACHE_MAP_SIZE 512000 (node_config.h:63) */
	uint32_t policy_max_per_ep; /* POLICY_MAP_SIZE 16384 (policymap.go:37) */
	uint32_t policy_max_total;  /* device slots across all endpoints */
	uint32_t max_endpoints;     /* policy maps = endpoint ids [0, max) */
	uint32_t cidr_dyn_max;      /* maxLKeys 64k (prefilter.go:43) */
	uint32_t cidr_fix_max;      /* maxHKeys 20M (prefilter.go:44) */
	uint32_t endpoints_max;     /* ENDPOINTS_MAP_SIZE 65536 */
	/* reserved identities (node_config.h:34-37) */
	uint32_t host_id, world_id, cluster_id, health_id;
	/* IPV4_CLUSTER_MASK / IPV4_CLUSTER_RANGE, network-order u32 as the
	 * agent writes them (daemon/daemon.go:919-920) */
	uint32_t ipv4_cluster_mask, ipv4_cluster_range;
	uint8_t ipv6_router_ip[16]; /* ROUTER_IP, ipv6_match_prefix_64 */
	/* CONNTRACK protocol gate: non ICMP/TCP/UDP -> DROP_CT_UNKNOWN_PROTO
	 * before policy (bpf/lib/conntrack.h:526-528) */
	uint8_t ct_proto_gate;
	/* ingress label: 0 -> secctx = resolved source identity (FROM_HOST
	 * form, bpf_netdev.c:403); 1 -> WORLD_ID (derive_ipv4_sec_ctx,
	 * bpf_netdev.c:278-290) */
	uint8_t ingress_secctx_world;
	/* prefilter: CIDR4_FILTER/CIDR4_LPM_PREFILTER/... (prefilter.go:65-89) */
	uint8_t prefilter_fix4, prefilter_dyn4, prefilter_fix6, prefilter_dyn6;
	uint8_t reserved0[2];
	/* identity handed to handle_ipv4 on ingress (from_netdev: 0) */
	uint32_t ingress_src_identity;
	/* counter slots [0, hot_counter_slots) are reserved for L3-only and
	 * identity-wildcard policy keys (the entries most tuples hit) and are
	 * accumulated in LDS per workgroup before one flush to HBM */
	uint32_t hot_counter_slots;
	/* service map cilium_lb4_services: max_elem (CILIUM_LB_MAP_MAX_ENTRIES,
	 * bpf/node_config.h:60; raise it for the 1M-service config) */
	uint32_t lb_max_entries;
	/* IPV4_LOOPBACK (bpf/node_config.h:45), network-order u32 as written */
	uint32_t ipv4_loopback;
	/* CGPU_LB_L3 | CGPU_LB_L4: the LB_L3 / LB_L4 build switches of lib/lb.h
	 * (bpf/lxc_config.h:44-45 and bpf/init.sh:352 set both) */
	uint32_t lb_flags;
	/* NODE_MAC (bpf/node_config.h:51): the gateway MAC an endpoint's egress
	 * frames must be addressed to (is_valid_gw_dst_mac, lib/lxc.h:77-90) */
	uint8_t node_mac[6];
	uint8_t reserved1[2];
	/* CT_MAP_SIZE of cilium_ct4_global: live conntrack entries the map
	 * holds (MapNumEntriesGlobal 1000000, pkg/maps/ctmap/ctmap.go:101);
	 * device slots are 2x this, rounded up to a power of two */
	uint32_t ct_max;
	/* schedule overrides, CGPU_SCHED_* (0 = the tuned default).  Every
	 * schedule computes the same results; they exist for the parity tests of
	 * the fallback kernels and for A/B timing, and are fixed per context (no
	 * behaviour is read from the environment). */
	uint32_t schedule;
	/* CT_MAP_SIZE of cilium_ct6_global (0 = ct_max) */
	uint32_t ct6_max;
	/* 1: the conntrack maps behave as BPF_MAP_TYPE_LRU_HASH, which the
	 * reference builds CT_MAP4 / CT_MAP6 as on every kernel with LRU maps
	 * (bpf/bpf_lxc.c:53-75, probe bpf/probes/raw_lru_map.t): a create that
	 * finds the map full evicts an entry instead of failing.  The victim is
	 * the engine's own choice, not the kernel's per-CPU LRU list: a live
	 * entry none of the batch's packets can look up or create (a key filter
	 * built before the walk; the scan covers CT_EVICT_SCAN = 4096 slots from
	 * a hashed start), so every packet of a batch gets the result the map it
	 * started from gives it.  cgpu_classify_v{4,6}_ct only: the service paths
	 * keep failing the create (DROP_NO_SERVICE / DROP_CT_CREATE_FAILED).
	 * 0 (default): the non-LRU build, CT_MAP_SIZE enforced as -E2BIG. */
	uint32_t ct_lru;
	uint32_t reserved[1];
} cgpu_config;

#define CGPU_SCHED_PER_LANE 1u   /* classify: one tuple per lane (k_classify) instead of x4 */
#define CGPU_SCHED_GLOBAL_CTR 2u /* classify: per-lane kernel, one global atomic per hit */
#define CGPU_SCHED_NO_CCACHE 4u  /* x4 classify without the LDS cold-slot cache */
#define CGPU_SCHED_FRAMES_SPLIT 8u /* classify_frames, 64-byte slots: a header pass writes tuple columns, then the classify pass (default: one fused kernel) */
/* bits 4-5: v6 prefilter LDS staging mode + 1 (0 = the deepest that fits) */
#define CGPU_SCHED_PF6_LDS(mode) ((((uint32_t)(mode)) + 1u) << 4)
/* bits 8-13: conntrack group-key radix sort bits (8..32; 0 = 24) */
#define CGPU_SCHED_CT_SORT_BITS(b) (((uint32_t)(b)) << 8)

#define CGPU_LB_L3 1u
#define CGPU_LB_L4 2u

typedef struct cgpu_ctx cgpu_ctx;

void cgpu_config_default(cgpu_config *cfg);
/* device: HIP device ordinal, or -1 for a host-only context (table
 * management and dumps work; batch entry points return -ENODEV). */
int cgpu_ctx_create(const cgpu_config *cfg, int device, cgpu_ctx **out);
void cgpu_ctx_destroy(cgpu_ctx *ctx);
const char *cgpu_last_error(void);
const char *cgpu_version(void);

/* ------------------------------------------------------------------ */
/* ipcache: pkg/maps/ipcache (Map.Update/Delete, LPM semantics of       */
/* kernel/bpf/lpm_trie.c; lookup is longest-prefix like bpf(2) lookup)  */
/* ------------------------------------------------------------------ */
int cgpu_ipcache_update(cgpu_ctx *ctx, const cgpu_ipcache_key *key,
			const cgpu_remote_endpoint_info *val, uint64_t flags);
int cgpu_ipcache_delete(cgpu_ctx *ctx, const cgpu_ipcache_key *key);
int cgpu_ipcache_lookup(cgpu_ctx *ctx, const cgpu_ipcache_key *key,
			cgpu_remote_endpoint_info *val_out);
/* GetNextKey: key == NULL returns the first key; -ENOENT after the last */
int cgpu_ipcache_get_next_key(cgpu_ctx *ctx, const cgpu_ipcache_key *key,
			      cgpu_ipcache_key *next_out);
size_t cgpu_ipcache_count(cgpu_ctx *ctx);
/* n updates in order; stops at the first failure (its -errno is returned,
 * the updates before it stay applied): the listener's sequence of
 * OnIPIdentityCacheChange writes in one call */
int cgpu_ipcache_update_batch(cgpu_ctx *ctx, const cgpu_ipcache_key *keys,
			      const cgpu_remote_endpoint_info *vals, size_t n, uint64_t flags);

/* ------------------------------------------------------------------ */
/* policy maps: pkg/maps/policymap (AllowKey/DeleteKey/DumpToSlice/     */
/* Flush), one map per endpoint id                                      */
/* ------------------------------------------------------------------ */
int cgpu_policy_update(cgpu_ctx *ctx, uint32_t ep, const cgpu_policy_key *key,
		       const cgpu_policy_entry *entry, uint64_t flags);
int cgpu_policy_delete(cgpu_ctx *ctx, uint32_t ep, const cgpu_policy_key *key);
/* entry_out.packets/bytes include every committed-and-classified batch */
int cgpu_policy_lookup(cgpu_ctx *ctx, uint32_t ep, const cgpu_policy_key *key,
		       cgpu_policy_entry *entry_out);
int cgpu_policy_get_next_key(cgpu_ctx *ctx, uint32_t ep, const cgpu_policy_key *key,
			     cgpu_policy_key *next_out);
int cgpu_policy_flush(cgpu_ctx *ctx, uint32_t ep);
size_t cgpu_policy_count(cgpu_ctx *ctx, uint32_t ep);
/* AllowKey for n (ep, key) pairs in order (stops at the first failure) */
int cgpu_policy_update_batch(cgpu_ctx *ctx, const uint32_t *eps, const cgpu_policy_key *keys,
			     const cgpu_policy_entry *entries, size_t n, uint64_t flags);
/* cgpu_policy_lookup of n (ep, key) pairs with one read of the device
 * counters: rc_out[i] = 0 or -ENOENT (-EINVAL for an ep out of range) */
int cgpu_policy_lookup_batch(cgpu_ctx *ctx, const uint32_t *eps, const cgpu_policy_key *keys,
			     size_t n, cgpu_policy_entry *entries_out, int32_t *rc_out);
/* DumpToSlice (pkg/maps/policymap/policymap.go:208-240): every key of ep's
 * map with its entry, in GetNextKey order; *n_out = the key count
 * (-ENOSPC when it exceeds cap, nothing written) */
int cgpu_policy_dump(cgpu_ctx *ctx, uint32_t ep, cgpu_policy_key *keys_out,
		     cgpu_policy_entry *entries_out, size_t cap, size_t *n_out);

/* ------------------------------------------------------------------ */
/* prefilter CIDR maps: pkg/maps/cidrmap (InsertCIDR/DeleteCIDR/        */
/* CIDRExists/CIDRDump) and the endpoint map cilium_lxc (lxcmap)        */
/* ------------------------------------------------------------------ */
int cgpu_cidr_update(cgpu_ctx *ctx, int which, const cgpu_cidr_key *key, uint64_t flags);
int cgpu_cidr_delete(cgpu_ctx *ctx, int which, const cgpu_cidr_key *key);
/* exact key presence (CIDRExists semantics for fix; LPM lookup for dyn) */
int cgpu_cidr_lookup(cgpu_ctx *ctx, int which, const cgpu_cidr_key *key);
int cgpu_cidr_get_next_key(cgpu_ctx *ctx, int which, const cgpu_cidr_key *key,
			   cgpu_cidr_key *next_out);
/* n InsertCIDR writes in order (stops at the first failure) */
int cgpu_cidr_update_batch(cgpu_ctx *ctx, int which, const cgpu_cidr_key *keys, size_t n,
			   uint64_t flags);
/* PreFilter (pkg/policy/prefilter.go:30-203): the revisioned CIDR set the
 * agent's PATCH/DELETE /prefilter handlers drive (daemon/prefilter.go).
 * A prefix carries its address family as the mask size of net.IPNet
 * (bits 32 / 128).  selectMap (prefilter.go:108-122) routes /32 and /128 to
 * the exact ("fix") maps and shorter prefixes to the LPM ("dyn") maps; a map
 * whose cgpu_config switch is off does not exist (-EOPNOTSUPP, "No map
 * enabled").  revision != 0 must equal the current revision (else -ESTALE,
 * "Latest revision is ..."); it starts at 1 and each successful call adds 1.
 * insert: every prefix or none -- on the first failure the prefixes already
 * inserted are deleted again (prefilter.go:124-159).  delete: every prefix
 * must exist first (a map lookup: longest-prefix on the LPM maps, -ENOENT
 * before anything changed); a later failure re-inserts the deleted ones
 * (:161-203).  The map contents reach the device at cgpu_commit. */
typedef struct cgpu_prefix {
	uint32_t bits; /* 32: IPv4, 128: IPv6 */
	cgpu_cidr_key key;
} cgpu_prefix;
int cgpu_prefilter_insert(cgpu_ctx *ctx, int64_t revision, const cgpu_prefix *cidrs, size_t n);
int cgpu_prefilter_delete(cgpu_ctx *ctx, int64_t revision, const cgpu_prefix *cidrs, size_t n);
int cgpu_prefilter_revision(cgpu_ctx *ctx, int64_t *revision_out);

int cgpu_endpoint_update(cgpu_ctx *ctx, const cgpu_endpoint_key *key, uint64_t flags);
int cgpu_endpoint_delete(cgpu_ctx *ctx, const cgpu_endpoint_key *key);
int cgpu_endpoint_lookup(cgpu_ctx *ctx, const cgpu_endpoint_key *key);

/* ------------------------------------------------------------------ */
/* service map cilium_lb4_services: pkg/maps/lbmap (UpdateService /     */
/* DeleteService, lbmap.go:341-429), bpf/lib/lb.h:70-76                  */
/* ------------------------------------------------------------------ */
/* struct lb4_key, bpf/lib/common.h:427-431: address and dport in network
 * order, slave host order (Go Service4Key.ToNetwork, lbmap/ipv4.go:99-104) */
typedef struct cgpu_lb4_key {
	uint32_t address;
	uint16_t dport;
	uint16_t slave; /* 0 = the service ("master"), 1.. = backends */
} cgpu_lb4_key;

/* struct lb4_service, bpf/lib/common.h:433-439: target, port, rev_nat_index,
 * weight in network order; count host order (lbmap/ipv4.go:135-181) */
typedef struct cgpu_lb4_service {
	uint32_t target;
	uint16_t port;
	uint16_t count;
	uint16_t rev_nat_index;
	uint16_t weight;
} cgpu_lb4_service;

int cgpu_lb4_update(cgpu_ctx *ctx, const cgpu_lb4_key *key, const cgpu_lb4_service *val,
		    uint64_t flags);
/* n updates in order; stops at the first failure (its -errno is returned,
 * the entries before it stay applied).  The Go writer issues one bpf(2)
 * call per entry; this is the same sequence in one call. */
int cgpu_lb4_update_batch(cgpu_ctx *ctx, const cgpu_lb4_key *keys, const cgpu_lb4_service *vals,
			  size_t n, uint64_t flags);
int cgpu_lb4_delete(cgpu_ctx *ctx, const cgpu_lb4_key *key);
int cgpu_lb4_lookup(cgpu_ctx *ctx, const cgpu_lb4_key *key, cgpu_lb4_service *val_out);
int cgpu_lb4_get_next_key(cgpu_ctx *ctx, const cgpu_lb4_key *key, cgpu_lb4_key *next_out);
size_t cgpu_lb4_count(cgpu_ctx *ctx);

/* struct lb6_key, bpf/lib/common.h:408-412 (packed, 20 B): address and dport
 * in network order, slave host order */
typedef struct cgpu_lb6_key {
	uint8_t address[16];
	uint16_t dport;
	uint16_t slave;
} cgpu_lb6_key;

/* struct lb6_service, bpf/lib/common.h:414-420 (packed, 24 B) */
typedef struct cgpu_lb6_service {
	uint8_t target[16];
	uint16_t port;
	uint16_t count;
	uint16_t rev_nat_index;
	uint16_t weight;
} cgpu_lb6_service;

/* cilium_lb6_services (lb.h:46-52), the map lbmap writes for IPv6
 * frontends (pkg/maps/lbmap/ipv6.go); same semantics as the lb4 calls.
 * Shares lb_max_entries with the lb4 map as a per-map capacity. */
int cgpu_lb6_update(cgpu_ctx *ctx, const cgpu_lb6_key *key, const cgpu_lb6_service *val,
		    uint64_t flags);
int cgpu_lb6_update_batch(cgpu_ctx *ctx, const cgpu_lb6_key *keys, const cgpu_lb6_service *vals,
			  size_t n, uint64_t flags);
int cgpu_lb6_delete(cgpu_ctx *ctx, const cgpu_lb6_key *key);
int cgpu_lb6_lookup(cgpu_ctx *ctx, const cgpu_lb6_key *key, cgpu_lb6_service *val_out);
int cgpu_lb6_get_next_key(cgpu_ctx *ctx, const cgpu_lb6_key *key, cgpu_lb6_key *next_out);
size_t cgpu_lb6_count(cgpu_ctx *ctx);

/* The flow hash the batch entry points use when no hash column is given
 * (skb->hash comes from the kernel's flow dissector, which the reference
 * does not contain: SURVEY §8c).  Over the stored (network-order) fields. */
uint32_t cgpu_flow_hash(uint32_t saddr, uint32_t daddr, uint16_t sport, uint16_t dport,
			uint8_t proto);
/* IPv6: cgpu_flow_hash over the two addresses folded to 32 bits each
 * (tables.h fold6: the 16 bytes as four little-endian words, murmur3-mixed) */
uint32_t cgpu_flow_hash6(const uint8_t *saddr16, const uint8_t *daddr16, uint16_t sport,
			 uint16_t dport, uint8_t proto);

/* ------------------------------------------------------------------ */
/* per-endpoint identity of the endpoint program (lxc_config.h)         */
/* ------------------------------------------------------------------ */
/* The #defines the agent writes per endpoint into lxc_config.h and that the
 * from-container program checks on every frame (bpf/lib/lxc.h:31-89):
 * LXC_MAC, LXC_IPV4, LXC_IP, and which checks are compiled in (the absence
 * of DISABLE_SMAC_VERIFICATION / DISABLE_DMAC_VERIFICATION /
 * DISABLE_SIP_VERIFICATION).  An endpoint without an entry verifies nothing. */
#define CGPU_VERIFY_SMAC 1u /* h_source == LXC_MAC      -> else DROP_INVALID_SMAC (-130) */
#define CGPU_VERIFY_DMAC 2u /* h_dest == NODE_MAC       -> else DROP_INVALID_DMAC (-131) */
#define CGPU_VERIFY_SIP 4u  /* saddr == LXC_IPV4/LXC_IP -> else DROP_INVALID_SIP (-132) */

typedef struct cgpu_lxc_info {
	uint8_t mac[6];   /* LXC_MAC */
	uint8_t verify;   /* CGPU_VERIFY_* */
	uint8_t pad;
	uint32_t ipv4;    /* LXC_IPV4: raw u32 compared with ip4->saddr (lxc.h:55-62) */
	uint8_t ipv6[16]; /* LXC_IP, network order */
	uint32_t sec_label; /* SECLABEL: src_sec_id of the entries the endpoint's egress
			       creates (bpf_lxc.c:517, conntrack.h:705) */
} cgpu_lxc_info;

int cgpu_lxc_update(cgpu_ctx *ctx, uint32_t ep, const cgpu_lxc_info *info);
int cgpu_lxc_delete(cgpu_ctx *ctx, uint32_t ep);
int cgpu_lxc_lookup(cgpu_ctx *ctx, uint32_t ep, cgpu_lxc_info *info_out);

/* ------------------------------------------------------------------ */
/* publication                                                          */
/* ------------------------------------------------------------------ */
/* Compile the host mirror into device tables and publish them as the new
 * snapshot read by later batch launches.  *epoch_out (optional) receives
 * the snapshot number.  Only the table groups that changed since the last
 * commit are uploaded (the rest is shared with the previous snapshot); a
 * few ipcache / policy changes patch the previous tables instead of
 * recompiling them, the way the reference writes each map key in place
 * (pkg/endpoint/endpoint.go:2572-2652 syncPolicyMap,
 * pkg/datapath/ipcache/listener.go:78-127).  Returns once the upload (on the
 * context's own stream) is complete; launches in flight on the previous
 * snapshot are never waited for.  Counter values supplied with a rewritten
 * policy entry reach the device here; hits that launches still running on
 * the previous snapshot add to that entry may land before or after. */
int cgpu_commit(cgpu_ctx *ctx, uint64_t *epoch_out);
/* order-independent checksum of the committed table contents; replicas on
 * different GPUs/ranks holding the same tables report the same value */
int cgpu_table_checksum(cgpu_ctx *ctx, uint64_t *sum_out);
/* Device bytes a lookup into each table group of the published snapshot
 * gathers from (0 for a group never committed; parts staged in LDS or read
 * only by fallback schedules excluded), and of the conntrack maps: bench.py
 * prices each map's lookups at the measured gather ceiling of the cache tier
 * a table of that size lives in. */
enum {
	CGPU_TBL_IPCACHE = 0, CGPU_TBL_POLICY, CGPU_TBL_PREFILTER, CGPU_TBL_ENDPOINT, CGPU_TBL_LB4,
	CGPU_TBL_LXC, CGPU_TBL_LB6, CGPU_TBL_CT4, CGPU_TBL_CT6, CGPU_TBL_N
};
int cgpu_table_bytes(cgpu_ctx *ctx, uint64_t *bytes_out /* [CGPU_TBL_N] */);
/* Failure detection: every group buffer a commit uploads is
 * summed on the device and compared with the host image's sum before the
 * snapshot is published (a mismatch fails the commit with -EIO).  This call
 * re-sums every buffer of the published snapshot on the device and returns
 * -EIO (naming the table group) when one no longer matches its host image;
 * a caller recovers by committing again from the authoritative host mirror. */
int cgpu_table_verify(cgpu_ctx *ctx);
/* checksum of which counter slot every committed policy key holds.  Slot
 * assignment is a function of the sequence of map operations and commits
 * only (never of GPU progress), so replicas that applied the same sequence
 * agree; ranks compare it before cgpu_counters_allreduce, which sums the
 * delta buffers slot by slot. */
int cgpu_counter_layout_checksum(cgpu_ctx *ctx, uint64_t *sum_out);

/* ------------------------------------------------------------------ */
/* batch classification (device pointers)                              */
/* ------------------------------------------------------------------ */
/* Tuple flag bits */
#define CGPU_F_EGRESS 1u   /* from-container (bpf_lxc.c handle_ipv4_from_lxc) */
#define CGPU_F_FRAGMENT 2u /* ipv4_is_fragment (bpf/lib/ipv4.h:50-61) */

typedef struct cgpu_tuples_v4 {
	const uint32_t *saddr; /* network order */
	const uint32_t *daddr; /* network order */
	const uint16_t *dport; /* network order (policy port, conntrack.h:471-524) */
	const uint8_t *proto;
	const uint8_t *flags;  /* CGPU_F_* */
	const uint32_t *len;   /* skb->len */
	const uint16_t *ep;    /* endpoint id: selects the policy map */
} cgpu_tuples_v4;

/*
 * For every tuple: ipcache LPM of the remote address, identity fallback,
 * the three-probe policy cascade of __policy_can_access (policy.h:46-110),
 * the per-entry packets/bytes counters and the {reason, dir} metrics.
 *   verdict[i]  : proxy port (raw be16 as int, e.g. 4000 -> 40975), 0 allow,
 *                 DROP_POLICY (-133), DROP_CT_UNKNOWN_PROTO (-137)
 *   identity[i] : label given to policy (dstID on egress, secctx on ingress)
 *   stage[i]    : optional (NULL ok): 1 exact, 2 L3-only, 3 identity-wildcard
 *                 L4, 0 miss, 4 protocol-gated (6: service drop, _lb only)
 */
int cgpu_classify_v4(cgpu_ctx *ctx, const cgpu_tuples_v4 *t, size_t n, int32_t *verdict,
		     uint32_t *identity, uint8_t *stage, void *stream);

/*
 * cgpu_classify_v4 over a HOST-resident batch (the reference
 * classifies each packet as the NIC hands it over, bpf_xdp.c:181-184 /
 * bpf_netdev.c:470; the engine takes batches that arrive in host memory
 * too): every column of t and the outputs are host pointers.  The batch
 * streams through device staging (up to 16 chunks of 8M tuples): uploads,
 * the classify of each chunk on `stream` and the stores of its outputs
 * overlap on queues of their own.  Returns once enqueued; the outputs are
 * complete when `stream` is (page-locked outputs are written by the CUs,
 * page-locked inputs uploaded by DMA, or read by the CUs for 64-byte frame
 * slots; pageable buffers are copied by the runtime and serialise).  Same results, counters
 * and metrics as cgpu_classify_v4 of the same tuples.  -ENODEV on a
 * host-only context, -EINVAL for a null column or output.
 */
int cgpu_classify_v4_host(cgpu_ctx *ctx, const cgpu_tuples_v4 *t, size_t n, int32_t *verdict,
			  uint32_t *identity, uint8_t *stage, void *stream);
/*
 * A host call pins ONE snapshot for its whole batch: a cgpu_commit from
 * another thread while the chunks are queued does not split the batch.  On
 * an error after the first chunk was queued, the call waits for every copy
 * it queued (they read and write the caller's buffers) before returning.
 * The staging (up to 16 x ~227 MB of device memory) stays allocated for the
 * next host call: cgpu_host_stage_bytes reports it, cgpu_host_stage_release
 * waits for the host calls queued on it and frees it (cgpu_ctx_destroy does
 * too).
 */
int cgpu_host_stage_release(cgpu_ctx *ctx);
size_t cgpu_host_stage_bytes(cgpu_ctx *ctx);

typedef struct cgpu_tuples_v6 {
	const uint8_t *saddr;  /* 16 bytes per tuple, network order */
	const uint8_t *daddr;  /* 16 bytes per tuple */
	const uint16_t *dport; /* network order */
	const uint8_t *proto;  /* nexthdr */
	const uint8_t *flags;  /* CGPU_F_EGRESS (fragments: IPv6 passes false) */
	const uint32_t *len;
	const uint16_t *ep;
} cgpu_tuples_v6;

/*
 * IPv6 form of cgpu_classify_v4: ipcache_lookup6 (eps.h:56-66), egress
 * fallback CLUSTER_ID when ipv6_match_prefix_64(daddr, ROUTER_IP)
 * (bpf_lxc.c:170-191), ingress identity without the HOST_ID exception
 * (bpf_netdev.c:203-211), protocol gate ICMPv6/TCP/UDP (conntrack.h:330-378).
 * The ingress label is the resolved source identity (FROM_HOST form).
 */
int cgpu_classify_v6(cgpu_ctx *ctx, const cgpu_tuples_v6 *t, size_t n, int32_t *verdict,
		     uint32_t *identity, uint8_t *stage, void *stream);

/*
 * cgpu_classify_v4 with the egress service step of handle_ipv4_from_lxc in
 * front (bpf_lxc.c:444-469; BASELINE config 5): every egress tuple is first
 * translated by lb4_local (stateless: conntrack empty, CT_NEW), ipcache then
 * resolves the translated tuple.daddr and policy sees the rewritten dport.
 * A DROP_NO_SERVICE (-158) ends the tuple: identity 0, stage 6, metrics
 * reason 158 egress (bpf_lxc.c:659-666).  Ingress tuples are as in
 * cgpu_classify_v4.  hash: skb->hash per tuple, or NULL for cgpu_flow_hash
 * over (saddr, daddr, sport, dport, proto); sport may be NULL when hash is
 * given.
 */
int cgpu_classify_v4_lb(cgpu_ctx *ctx, const cgpu_tuples_v4 *t, const uint16_t *sport,
			const uint32_t *hash, size_t n, int32_t *verdict, uint32_t *identity,
			uint8_t *stage, void *stream);

/*
 * BASELINE config 5 whole ("prefilter -> ipcache identity -> policy verdict ->
 * LB"): cgpu_classify_v4_lb with the netdev's XDP prefilter in front of every
 * INGRESS tuple, as a packet meets xdp_start -> check_filters -> check_v4
 * (bpf_xdp.c:97-121, :158-184) before from_netdev (bpf_netdev.c:470):
 *   saddr in the dyn4 LPM (CIDR4_LPM_PREFILTER) or a fix4 /32 (CIDR4_FILTER;
 *   both per cgpu_config.prefilter_*) -> XDP_DROP; else daddr must be a key
 *   of the endpoint map (check_v4_endpoint :88-95) -> XDP_PASS, else XDP_DROP.
 * An XDP_DROP ends the tuple: verdict CGPU_VERDICT_XDP_DROP, identity 0,
 * stage 8, no policy counters and no metrics (the XDP program notifies
 * nothing).  A passed ingress tuple and every egress tuple are classified
 * exactly as cgpu_classify_v4_lb (egress: lb4_local, then ipcache / policy).
 * Replaces, for a pre-parsed batch, the XDP program + bpf_netdev.c +
 * bpf_lxc.c sequence the kernel runs per packet.
 */
#define CGPU_VERDICT_XDP_DROP (-4097)
#define CGPU_STAGE_XDP_DROP 8
int cgpu_classify_v4_cascade(cgpu_ctx *ctx, const cgpu_tuples_v4 *t, const uint16_t *sport,
			     const uint32_t *hash, size_t n, int32_t *verdict, uint32_t *identity,
			     uint8_t *stage, void *stream);

/*
 * cgpu_classify_v6 with the egress service step of ipv6_l3_from_lxc in front
 * (bpf_lxc.c:108-139): lb6_extract_key, lb6_lookup_service and lb6_local
 * (lb.h:334-483) with an empty conntrack table (CT_NEW); ipcache then
 * resolves the translated tuple->daddr and policy sees the dport ct_lookup6
 * reloads from the rewritten packet.  IPv6 has no loopback case.  A
 * DROP_NO_SERVICE (-158) ends the tuple: identity 0, stage 6, metrics reason
 * 158 egress.  hash: skb->hash per tuple or NULL for cgpu_flow_hash6 (then
 * sport is required).
 */
int cgpu_classify_v6_lb(cgpu_ctx *ctx, const cgpu_tuples_v6 *t, const uint16_t *sport,
			const uint32_t *hash, size_t n, int32_t *verdict, uint32_t *identity,
			uint8_t *stage, void *stream);

/*
 * The HOST-resident forms of the service, cascade and IPv6 paths: the same
 * arguments, results, counters and metrics as the device call of the same
 * name without _host, with every column and output a host pointer, streamed
 * through the staging of cgpu_classify_v4_host (same snapshot pinning, same
 * error drain, same completion on `stream`).  The service forms upload the
 * hash column when one is given (it wins over sport, as on the device), else
 * sport.  The v6 address columns need no alignment here (the staging is
 * aligned).  -ENODEV on a host-only context.
 */
int cgpu_classify_v4_lb_host(cgpu_ctx *ctx, const cgpu_tuples_v4 *t, const uint16_t *sport,
			     const uint32_t *hash, size_t n, int32_t *verdict, uint32_t *identity,
			     uint8_t *stage, void *stream);
int cgpu_classify_v4_cascade_host(cgpu_ctx *ctx, const cgpu_tuples_v4 *t, const uint16_t *sport,
				  const uint32_t *hash, size_t n, int32_t *verdict, uint32_t *identity,
				  uint8_t *stage, void *stream);
int cgpu_classify_v6_host(cgpu_ctx *ctx, const cgpu_tuples_v6 *t, size_t n, int32_t *verdict,
			  uint32_t *identity, uint8_t *stage, void *stream);
int cgpu_classify_v6_lb_host(cgpu_ctx *ctx, const cgpu_tuples_v6 *t, const uint16_t *sport,
			     const uint32_t *hash, size_t n, int32_t *verdict, uint32_t *identity,
			     uint8_t *stage, void *stream);

/* Service translation alone (device pointers). */
#define CGPU_LB_NETDEV 0 /* bpf_lb.c handle_ipv4 (bpf_lb.c:118-170) */
#define CGPU_LB_LXC 1    /* lb4_local on the endpoint egress path (bpf_lxc.c:444-460) */
/* ret codes of CGPU_LB_LXC (CGPU_LB_NETDEV returns TC_ACT_OK 0 when the
 * packet is not load-balanced, TC_ACT_REDIRECT 7 when it is) */
#define CGPU_LB_NONE 0
#define CGPU_LB_XLATED 1
#define CGPU_LB_XLATED_LOOPBACK 2 /* source NAT to IPV4_LOOPBACK, lb.h:753-767 */
#define CGPU_DROP_NO_SERVICE (-158)

typedef struct cgpu_lb4_tuples {
	const uint32_t *saddr, *daddr; /* network order */
	const uint16_t *sport, *dport; /* network order; sport only for the default hash */
	const uint8_t *proto;
	const uint32_t *hash;          /* NULL: cgpu_flow_hash */
} cgpu_lb4_tuples;

/* outputs (device pointers; all but ret may be NULL): the packet's saddr /
 * daddr / dport after lb4_xlate, the chosen entry's rev_nat_index and slave */
typedef struct cgpu_lb4_out {
	int32_t *ret;
	uint32_t *saddr, *daddr;
	uint16_t *dport, *rev_nat, *slave;
} cgpu_lb4_out;

int cgpu_lb4_select(cgpu_ctx *ctx, int mode, const cgpu_lb4_tuples *t, size_t n,
		    const cgpu_lb4_out *out, void *stream);

/* XDP prefilter over pre-parsed packets (bpf_xdp.c:88-184).
 * flags: 0 IP packet of this family, 1 truncated (-> XDP_DROP),
 *        2 not IPv4/IPv6 (-> XDP_PASS).  verdict: XDP_DROP 1 / XDP_PASS 2. */
#define CGPU_PKT_OK 0u
#define CGPU_PKT_TRUNCATED 1u
#define CGPU_PKT_NOT_IP 2u
int cgpu_prefilter_v4(cgpu_ctx *ctx, const uint32_t *saddr, const uint32_t *daddr,
		      const uint8_t *flags, size_t n, uint8_t *verdict, void *stream);
/* saddr/daddr: 16 bytes per packet, contiguous */
int cgpu_prefilter_v6(cgpu_ctx *ctx, const uint8_t *saddr, const uint8_t *daddr,
		      const uint8_t *flags, size_t n, uint8_t *verdict, void *stream);
/* the prefilters over host-resident columns (as cgpu_classify_v4_host) */
int cgpu_prefilter_v4_host(cgpu_ctx *ctx, const uint32_t *saddr, const uint32_t *daddr,
			   const uint8_t *flags, size_t n, uint8_t *verdict, void *stream);
int cgpu_prefilter_v6_host(cgpu_ctx *ctx, const uint8_t *saddr, const uint8_t *daddr,
			   const uint8_t *flags, size_t n, uint8_t *verdict, void *stream);

/* ------------------------------------------------------------------ */
/* raw Ethernet frames                               */
/* ------------------------------------------------------------------ */
/*
 * A batch of frames in one device buffer: frame i is the first
 * min(len[i], stride) bytes at data + i * stride (a fixed-size receive ring
 * slot; the rest of the slot is ignored).  stride is a multiple of 16 and
 * >= 64; data is 16-byte aligned.  len[i] is the wire length (skb->len), the
 * bound of every header read as in skb_load_bytes / revalidate_data.
 * flags[i]: CGPU_F_EGRESS = from-container (the endpoint's egress program),
 * else to-container (ingress); other bits are ignored.  ep[i] selects the
 * policy map and the cgpu_lxc_info of the endpoint.
 */
typedef struct cgpu_frames {
	const uint8_t *data;
	const uint32_t *len;
	const uint8_t *flags;
	const uint16_t *ep;
	uint32_t stride;
	uint32_t reserved;
} cgpu_frames;

/* frame status / verdict values beyond the reference's DROP_* codes */
#define CGPU_FRAME_NOT_CLASSIFIED 1 /* egress ARP (tail call to the ARP responder,
				       bpf_lxc.c:703-706), an egress ICMPv6 frame the
				       ICMPv6 responders take (bpf_lxc.c:377-386) or
				       ingress non-IP (passed to the stack,
				       bpf_netdev.c:518-520) */
#define CGPU_DROP_SNAPLEN (-4096)   /* a header the reference would read lies past
				       the stored slot (stride < len): re-submit
				       with a larger stride */

/* The policy tuple a frame reaches the ipcache / policy step with. */
typedef struct cgpu_frame_tuples {
	int32_t *status;   /* 0 reached policy; CGPU_FRAME_NOT_CLASSIFIED; or the
			      DROP_* / -errno the program returned before policy */
	uint8_t *family;   /* 4, 6, or 0 (not IP) */
	uint8_t *saddr;    /* 16 bytes per frame (IPv4: first 4, rest zero) */
	uint8_t *daddr;    /* 16 bytes per frame */
	uint16_t *dport;   /* tuple.dport after ct_lookup (network order; 0 without
			      CONNTRACK, i.e. ct_proto_gate = 0) */
	uint8_t *proto;    /* tuple.nexthdr (after the IPv6 extension-header walk) */
	uint8_t *flags;    /* CGPU_F_EGRESS | CGPU_F_FRAGMENT (ingress IPv4 only) */
} cgpu_frame_tuples;

/*
 * Per frame, the steps of the endpoint programs before the ipcache lookup
 * (stateless: conntrack empty, every packet CT_NEW):
 *   egress : skb->protocol dispatch (bpf_lxc.c:683-711; other than IPv4,
 *            IPv6, ARP -> DROP_UNKNOWN_L3 -139), revalidate_data (-134),
 *            handle_ipv6's ICMPv6 responders (bpf_lxc.c:364-389: an ICMPv6
 *            frame shorter than its icmp6hdr -134; a neighbour solicitation
 *            for another target DROP_UNKNOWN_TARGET -150, for ROUTER_IP -134
 *            without its ND option, else -- and an echo request to ROUTER_IP
 *            -- handed to the responder: CGPU_FRAME_NOT_CLASSIFIED), the
 *            SMAC / DMAC / SIP checks (-130 / -131 / -132), ipv6_hdrlen
 *            (-156, -157, -134), extract_l4_port of lb{4,6}_extract_key
 *            (TCP/UDP dport past len -> -14, -EFAULT of skb_load_bytes),
 *            ct_lookup{4,6} port extraction (-135 truncated L4, -137 other
 *            than ICMP/ICMPv6/TCP/UDP; with ct_proto_gate = 0 the
 *            non-CONNTRACK stubs: no port load, no gate)
 *   ingress: bpf_netdev.c dispatch (non-IP passed), ipv4_policy /
 *            ipv6_policy up to ct_lookup (bpf_lxc.c:876-897, :731-773)
 * All outputs are device pointers; any but status may be NULL.
 */
int cgpu_frames_parse(cgpu_ctx *ctx, const cgpu_frames *f, size_t n,
		      const cgpu_frame_tuples *out, void *stream);

/*
 * Raw frames to verdicts in one pass: cgpu_frames_parse, then for frames
 * that reach policy the decision of cgpu_classify_v4 / cgpu_classify_v6 on
 * that tuple (mixed IPv4 / IPv6 batches).  Frames that end before policy get
 * verdict = their status, identity 0 and stage 5 (DROP_CT_UNKNOWN_PROTO keeps
 * stage 4 as in cgpu_classify_v4; NOT_CLASSIFIED: verdict 0, stage 7, not
 * counted in the metrics).  Metrics count every other frame
 * once at {reason = -verdict (u8) or 0, dir}; SNAPLEN frames are not counted.
 */
int cgpu_classify_frames(cgpu_ctx *ctx, const cgpu_frames *f, size_t n, int32_t *verdict,
			 uint32_t *identity, uint8_t *stage, void *stream);

/*
 * cgpu_classify_frames over a HOST-resident batch (the frames as the NIC's
 * receive ring holds them, bpf_xdp.c:181-184 / bpf_netdev.c:470): f's data,
 * len, flags and ep and the outputs are host pointers; the batch streams
 * through the staging of cgpu_classify_v4_host (~1M 64-byte slots per
 * chunk), with its snapshot, error and completion rules.  Same results,
 * counters and metrics as cgpu_classify_frames of the same frames.
 */
int cgpu_classify_frames_host(cgpu_ctx *ctx, const cgpu_frames *f, size_t n, int32_t *verdict,
			      uint32_t *identity, uint8_t *stage, void *stream);

/* ------------------------------------------------------------------ */
/* conntrack: the map cilium_ct4_global               */
/* ------------------------------------------------------------------ */
/* struct ipv4_ct_tuple (bpf/lib/common.h:359-366), packed, 14 B */
#pragma pack(push, 1)
typedef struct cgpu_ct4_tuple {
	uint32_t daddr;  /* network order */
	uint32_t saddr;
	uint16_t dport;  /* network order */
	uint16_t sport;
	uint8_t nexthdr;
	uint8_t flags;   /* TUPLE_F_OUT 0 / TUPLE_F_IN 1 | TUPLE_F_RELATED 2 */
} cgpu_ct4_tuple;
#pragma pack(pop)

/* struct ct_entry (bpf/lib/common.h:380-408), 56 B */
typedef struct cgpu_ct_entry {
	uint64_t rx_packets, rx_bytes, tx_packets, tx_bytes;
	uint32_t lifetime;
	uint16_t bits;   /* rx_closing:1 tx_closing:1 nat46:1 lb_loopback:1 seen_non_syn:1 */
	uint16_t rev_nat_index;
	uint16_t slave;
	uint8_t tx_flags_seen, rx_flags_seen;
	uint32_t src_sec_id;
	uint32_t last_tx_report, last_rx_report;
} cgpu_ct_entry;

/*
 * Map operations with the bpf(2) semantics the agent's ctmap package uses
 * (pkg/maps/ctmap/ctmap.go, pkg/bpf/bpf.go:153-245): update with
 * CGPU_ANY/NOEXIST/EXIST (-EEXIST / -ENOENT), -E2BIG for a new key past
 * ct_max; delete / lookup -ENOENT; get_next_key (NULL key = first) walks the
 * map in slot order.  The device table is authoritative once a batch ran:
 * these calls synchronize with it (they are control-plane operations).
 */
int cgpu_ct4_update(cgpu_ctx *ctx, const cgpu_ct4_tuple *key, const cgpu_ct_entry *val,
		    uint64_t flags);
int cgpu_ct4_delete(cgpu_ctx *ctx, const cgpu_ct4_tuple *key);
int cgpu_ct4_lookup(cgpu_ctx *ctx, const cgpu_ct4_tuple *key, cgpu_ct_entry *val_out);
int cgpu_ct4_get_next_key(cgpu_ctx *ctx, const cgpu_ct4_tuple *key, cgpu_ct4_tuple *next_out);
size_t cgpu_ct4_count(cgpu_ctx *ctx);
/* ctmap.GC with RemoveExpired (ctmap.go:306-310, :345-357): delete every
 * entry whose lifetime < time; *deleted_out (optional) = how many */
int cgpu_ct4_gc(cgpu_ctx *ctx, uint32_t time, uint64_t *deleted_out);
/* ctmap Flush (ctmap.go:361-367): delete every entry */
int cgpu_ct4_flush(cgpu_ctx *ctx);
/* (new, diagnostic) the map's slot statistics after everything queued on it:
 * out[0] live entries, out[1] tombstones, out[2] compactions so far (a batch
 * that finds more than a quarter of the slots tombstones first re-inserts the
 * live entries into a clean table, on the device).  v6: cilium_ct6_global. */
int cgpu_ct_stats(cgpu_ctx *ctx, int v6, uint64_t *out);

/* A batch of IPv4 packets for the stateful path (device pointers). */
typedef struct cgpu_tuples_v4_ct {
	const uint32_t *saddr; /* network order */
	const uint32_t *daddr;
	const uint16_t *sport; /* L4 header ports as on the wire (TCP/UDP) */
	const uint16_t *dport;
	const uint8_t *proto;
	const uint16_t *l4;    /* TCP: header bytes 12-13 as loaded (byte 12 in the
				  low half: doff/NS, byte 13 in the high half: flags);
				  ICMP: the type in the low byte; else ignored */
	const uint8_t *flags;  /* CGPU_F_EGRESS | CGPU_F_FRAGMENT */
	const uint32_t *len;
	const uint16_t *ep;
} cgpu_tuples_v4_ct;

/* ct_lookup4 results (bpf/lib/common.h:331-336) as reported in ct_ret[] */
#define CGPU_CT_NEW 0
#define CGPU_CT_ESTABLISHED 1
#define CGPU_CT_REPLY 2
#define CGPU_CT_RELATED 3
#define CGPU_CT_NONE 255 /* ct_lookup4 failed (DROP_CT_UNKNOWN_PROTO) */
#define CGPU_DROP_CT_CREATE_FAILED (-155)

/*
 * The stateful decision of the endpoint programs for n packets, with the
 * result of processing them IN ORDER (packet i sees every conntrack change
 * of packets < i, as the reference's programs do for a packet sequence):
 *   ct_lookup4 (bpf/lib/conntrack.h:441-561): the reply-direction tuple,
 *     then the forward one; on a hit the entry's timeout / TCP flags /
 *     closing bits / rx|tx counters are updated (:198-259);
 *   identity as cgpu_classify_v4; policy on the tuple as ct_lookup4 left it
 *     (the reply tuple's dport for CT_REPLY / CT_RELATED);
 *   CT_REPLY / CT_RELATED pass whatever policy says; otherwise a denied
 *     packet is dropped (DROP_POLICY) and, if CT_ESTABLISHED, its entry
 *     deleted; an allowed CT_NEW creates the forward entry and its ICMP
 *     related entry (ct_create4, :653-744; src_sec_id = the endpoint's
 *     SECLABEL on egress, the source identity on ingress), or fails with
 *     DROP_CT_CREATE_FAILED when the map is full;
 *   bpf_lxc.c:506-576 (egress), :918-950 (ingress).
 *   verdict[i]: DROP_* (-133, -137, -155), the proxy port (egress: any
 *               ct state; ingress: CT_NEW / CT_ESTABLISHED), else 0
 *   ct_ret[i] : CGPU_CT_*; identity[i], stage[i] as cgpu_classify_v4
 *               (stage may be NULL)
 * now = bpf_ktime_get_sec() for the batch.  Packets of one address pair are
 * resolved in order by one lane; pairs are independent.  The one departure
 * from a sequential run: which creates fail when the map fills up DURING a
 * batch depends on the order lanes reach the capacity check.
 * The context has ONE conntrack map: batches of every caller run in order
 * on the context's internal conntrack stream (after `stream` reaches the
 * call; `stream` then waits for the batch).  The host reads the map's
 * tombstone count once per call, which waits for the previous batch.
 */
int cgpu_classify_v4_ct(cgpu_ctx *ctx, const cgpu_tuples_v4_ct *t, size_t n, uint32_t now,
			int32_t *verdict, uint8_t *ct_ret, uint32_t *identity, uint8_t *stage,
			void *stream);

/* outputs of cgpu_classify_v4_ctlb (device pointers; stage, daddr, dport
 * may be NULL) */
typedef struct cgpu_ctlb_out {
	int32_t *verdict;   /* as cgpu_classify_v4_ct, plus DROP_NO_SERVICE (-158) */
	uint8_t *ct_ret;    /* the CT_EGRESS / CT_INGRESS lookup; CGPU_CT_NONE for a
			       service drop or DROP_CT_UNKNOWN_PROTO */
	uint32_t *identity; /* 0 for a service drop */
	uint8_t *stage;     /* as cgpu_classify_v4_ct; 6 = service drop */
	uint32_t *daddr;    /* the frame's daddr after the service step (lb4_xlate) */
	uint16_t *dport;    /* the frame's dport after it (network order) */
} cgpu_ctlb_out;

/*
 * cgpu_classify_v4_ct with the STATEFUL service step of handle_ipv4_from_lxc
 * in front (bpf_lxc.c:444-469; lb4_local with CONNTRACK, lib/lb.h:700-775),
 * packets processed in order as the reference's programs would:
 *   egress packets whose {daddr, dport} (or {daddr, 0}) is a service
 *   (lb4_extract_key / lb4_lookup_service, lb.h:590-635) look up their
 *   CT_SERVICE entry (ct_lookup4 with TUPLE_F_SERVICE, no forward lookup):
 *   CT_NEW selects slave = hash % count + 1 and creates the entry and its
 *   ICMP entry (src_sec_id 0) -- a failed create drops the packet with
 *   DROP_NO_SERVICE (fail closed); a hit reuses the stored slave (and
 *   lb_loopback).  A slave whose backend is gone falls back to
 *   lb4_lookup_service with key.slave kept, re-selects from that entry's
 *   count and rewrites the entry's slave (ct_update4_slave); no service ->
 *   DROP_NO_SERVICE.  Loopback (saddr == target): source NAT to
 *   IPV4_LOOPBACK and tuple.daddr keeps the service address.
 *   Then the egress conntrack path of cgpu_classify_v4_ct on the translated
 *   tuple: ipcache of tuple.daddr, policy on the rewritten dport, and an
 *   allowed CT_NEW creates its entry with the service's rev_nat_index,
 *   slave and lb_loopback, the address entry of ct_create4 (tuple->daddr :=
 *   backend or IPV4_LOOPBACK; conntrack.h:697-725) and the ICMP entry.
 *   A hit entry's reverse NAT goes through the empty cilium_lb4_reverse_nat
 *   map (a no-op, lb.h:562-576).  Ingress packets are as cgpu_classify_v4_ct.
 * hash: skb->hash per packet (NULL: cgpu_flow_hash over the 5-tuple).
 * Service drops: verdict -158, ct_ret CGPU_CT_NONE, identity 0, stage 6,
 * metrics reason 158 egress.  Ordering, streams and the capacity caveat as
 * cgpu_classify_v4_ct (an address entry's capacity is taken when its create
 * runs).  n < 2^30.
 */
int cgpu_classify_v4_ctlb(cgpu_ctx *ctx, const cgpu_tuples_v4_ct *t, const uint32_t *hash, size_t n,
			  uint32_t now, const cgpu_ctlb_out *out, void *stream);

/* ------------------------------------------------------------------ */
/* conntrack, IPv6: the map cilium_ct6_global (CT_MAP6, bpf_lxc.c:53-63) */
/* ------------------------------------------------------------------ */
/* struct ipv6_ct_tuple (bpf/lib/common.h:338-346), packed, 38 B */
#pragma pack(push, 1)
typedef struct cgpu_ct6_tuple {
	uint8_t daddr[16]; /* network order */
	uint8_t saddr[16];
	uint16_t dport;    /* network order */
	uint16_t sport;
	uint8_t nexthdr;
	uint8_t flags;     /* TUPLE_F_OUT 0 / TUPLE_F_IN 1 | TUPLE_F_RELATED 2 */
} cgpu_ct6_tuple;
#pragma pack(pop)

/* The cgpu_ct4_* map operations on cilium_ct6_global (capacity
 * cgpu_config.ct6_max, default ct_max). */
int cgpu_ct6_update(cgpu_ctx *ctx, const cgpu_ct6_tuple *key, const cgpu_ct_entry *val,
		    uint64_t flags);
int cgpu_ct6_delete(cgpu_ctx *ctx, const cgpu_ct6_tuple *key);
int cgpu_ct6_lookup(cgpu_ctx *ctx, const cgpu_ct6_tuple *key, cgpu_ct_entry *val_out);
int cgpu_ct6_get_next_key(cgpu_ctx *ctx, const cgpu_ct6_tuple *key, cgpu_ct6_tuple *next_out);
size_t cgpu_ct6_count(cgpu_ctx *ctx);
int cgpu_ct6_gc(cgpu_ctx *ctx, uint32_t time, uint64_t *deleted_out);
int cgpu_ct6_flush(cgpu_ctx *ctx);

/* A batch of IPv6 packets for the stateful path (device pointers). */
typedef struct cgpu_tuples_v6_ct {
	const uint8_t *saddr;  /* 16 bytes per packet, network order; 16-byte aligned */
	const uint8_t *daddr;
	const uint16_t *sport; /* L4 header ports as on the wire (TCP/UDP) */
	const uint16_t *dport;
	const uint8_t *proto;  /* nexthdr after the extension headers */
	const uint16_t *l4;    /* TCP: header bytes 12-13 as loaded; ICMPv6: the type
				  in the low byte; else ignored */
	const uint8_t *flags;  /* CGPU_F_EGRESS (IPv6 has no fragment flag) */
	const uint32_t *len;
	const uint16_t *ep;
} cgpu_tuples_v6_ct;

/*
 * cgpu_classify_v4_ct for IPv6 over cilium_ct6_global, in the order of
 * ipv6_l3_from_lxc (egress, bpf_lxc.c:108-203) and ipv6_policy (ingress,
 * :731-800): ct_lookup6 (conntrack.h:288-412; ICMPv6 errors 1-4 RELATED,
 * echo request / reply ports 128), identity as cgpu_classify_v6, policy on
 * the tuple ct_lookup6 left, ct_delete6 of a denied ESTABLISHED entry,
 * ct_create6 (:588-639, with its ICMPv6 related entry) of an allowed CT_NEW
 * packet.  An ingress entry is created with rev_nat_index =
 * daddr.s6_addr32[3] & 0xFFFF (bpf_lxc.c:748); a hit entry's reverse NAT
 * goes through the empty cilium_lb6_reverse_nat map (a no-op, lib/lb.h:
 * 305-317).  Outputs, ordering and the capacity caveat as cgpu_classify_v4_ct.
 */
int cgpu_classify_v6_ct(cgpu_ctx *ctx, const cgpu_tuples_v6_ct *t, size_t n, uint32_t now,
			int32_t *verdict, uint8_t *ct_ret, uint32_t *identity, uint8_t *stage,
			void *stream);

/* cgpu_classify_v6_ctlb's outputs: as cgpu_ctlb_out with the frame's daddr
 * 16 bytes per packet (16-byte aligned) */
typedef struct cgpu_ctlb6_out {
	int32_t *verdict;
	uint8_t *ct_ret;
	uint32_t *identity;
	uint8_t *stage;
	uint8_t *daddr;     /* [n][16]: the frame's daddr after lb6_xlate */
	uint16_t *dport;
} cgpu_ctlb6_out;

/*
 * cgpu_classify_v6_ct with the stateful service step of ipv6_l3_from_lxc in
 * front (bpf_lxc.c:122-146; lb6_local with CONNTRACK, lib/lb.h:426-483):
 * egress packets whose {daddr, dport} (or {daddr, 0}) is an IPv6 service
 * (lb6_extract_key / lb6_lookup_service, lb.h:327-365) look up their
 * CT_SERVICE entry in cilium_ct6_global; CT_NEW selects slave = hash % count
 * + 1 and creates it (ct_create6 with its ICMPv6 entry; a failed create
 * drops with DROP_NO_SERVICE), a hit reuses the stored slave; a slave whose
 * backend is gone falls back to lb6_lookup_service with key.slave kept and
 * ct_update6_slave; no service -> DROP_NO_SERVICE.  lb6_xlate rewrites the
 * frame's daddr (and the dport for TCP / UDP under CGPU_LB_L4); the tuple's
 * daddr becomes the backend, its dport the rewritten one.  Then the egress
 * conntrack path of cgpu_classify_v6_ct on that tuple, identity from the
 * ipcache of the backend, CT_NEW creates the entry with the service's
 * rev_nat_index and slave (ct_create6 writes no address entry).  Outputs as
 * cgpu_classify_v4_ctlb.  n < 2^30; address columns 16-byte aligned.
 */
int cgpu_classify_v6_ctlb(cgpu_ctx *ctx, const cgpu_tuples_v6_ct *t, const uint32_t *hash, size_t n,
			  uint32_t now, const cgpu_ctlb6_out *out, void *stream);

/* ------------------------------------------------------------------ */
/* checkpoint / resume                                      */
/* ------------------------------------------------------------------ */
/* The host mirror is authoritative (the device is rebuilt from it at any
 * commit), so a checkpoint is the mirror written to a file: every ipcache,
 * policy (with each entry's packets / bytes counters), prefilter CIDR,
 * endpoint, lb4 / lb6 and lxc entry, the PreFilter revision, and both
 * conntrack maps.  The reference's counterpart is its maps pinned in bpffs
 * plus the ipcache replay into listeners (pkg/ipcache/ipcache.go:328-338).
 * save: atomic (written to path.tmp, then renamed).  restore: into a context
 * whose maps are all empty (else -EEXIST); the file is validated whole
 * (-EINVAL on a bad header, section or checksum) and replayed through the
 * map calls with BPF_NOEXIST (capacity errors are returned as those calls
 * return them).  The tables reach the device at the next cgpu_commit.  The
 * {reason, dir} metrics are not part of a checkpoint (they restart at 0). */
int cgpu_mirror_save(cgpu_ctx *ctx, const char *path);
int cgpu_mirror_restore(cgpu_ctx *ctx, const char *path);

/* ------------------------------------------------------------------ */
/* L3 MapState compilation                           */
/* ------------------------------------------------------------------ */
/* The label decision computeDesiredL3PolicyMapEntries asks of the policy
 * repository for every (endpoint, identity) pair (pkg/endpoint/policy.go:
 * 317-390): Repository.AllowsIngressLabelAccess / AllowsEgressLabelAccess
 * (pkg/policy/repository.go:80-130, :443-490) over rule.canReachIngress /
 * canReachEgress (pkg/policy/rule.go:323-405).  Strings are interned by the
 * caller (cilium_amd/policy.py); every id below is such an interned id. */
#define CGPU_SEL_IN 0         /* In / = / ==: Has(key) && Get(key) in values */
#define CGPU_SEL_NOT_IN 1     /* NotIn / !=: !Has(key) || Get(key) not in values */
#define CGPU_SEL_EXISTS 2
#define CGPU_SEL_NOT_EXISTS 3 /* DoesNotExist */

/* a label of a LabelArray: ids of its key, of "source.key" and of its value */
typedef struct cgpu_label {
	uint32_t key, ext_key, value;
} cgpu_label;

/* labels.Requirement: any_source -> key is a key id matched against every
 * label's key (LabelArray.Has/Get with source "any", pkg/labels/array.go:
 * 92-130); else key is an ext_key id matched against "source.key" */
typedef struct cgpu_requirement {
	uint32_t any_source, key, op, values_off, n_values;
} cgpu_requirement;

/* EndpointSelector: requirements [reqs_off, +n_reqs), all must match;
 * match_all = matchLabels holds "reserved.all" (selector.go:290-294) */
typedef struct cgpu_selector {
	uint32_t reqs_off, n_reqs, match_all;
} cgpu_selector;

#define CGPU_L3_INGRESS 0
#define CGPU_L3_EGRESS 1
#define CGPU_L3_REQUIRES 0 /* FromRequires / ToRequires: must match, else Denied */
#define CGPU_L3_ALLOWS 1   /* FromEndpoints / ToEndpoints: match without ToPorts -> Allowed */
typedef struct cgpu_l3_clause {
	uint32_t dir, kind, selector, has_ports;
} cgpu_l3_clause;

typedef struct cgpu_l3_program {
	const cgpu_selector *selectors;
	uint32_t n_selectors;
	const cgpu_requirement *reqs;
	uint32_t n_reqs;
	const uint32_t *values;
	uint32_t n_values;
	const uint32_t *rule_subject; /* per rule: its EndpointSelector */
	const uint32_t *rule_clauses; /* n_rules + 1 offsets into clauses */
	uint32_t n_rules;
	const cgpu_l3_clause *clauses;
	uint32_t n_clauses;
} cgpu_l3_program;

/* label arrays: set i = labels[offsets[i] .. offsets[i + 1]) in array order */
typedef struct cgpu_label_sets {
	const uint32_t *offsets;
	const cgpu_label *labels;
	uint32_t n_sets;
} cgpu_label_sets;

#define CGPU_L3_INGRESS_ENFORCED 1u /* else ingress allows all (policy.go:351-360) */
#define CGPU_L3_EGRESS_ENFORCED 2u
/*
 * allow_out[e * n_identities + i] (host memory) = bit 0: ingress from
 * identity i to endpoint e is Allowed; bit 1: egress from e to i is Allowed.
 * All inputs are host pointers (a control-plane call: it uploads, evaluates
 * every pair on the device, one lane per pair, and copies the result back).
 */
int cgpu_l3_compile(cgpu_ctx *ctx, const cgpu_l3_program *prog, const cgpu_label_sets *endpoints,
		    const cgpu_label_sets *identities, uint32_t flags, uint8_t *allow_out);

/* ------------------------------------------------------------------ */
/* full MapState: L4 + localhost/world + L3 keys, synced into the maps  */
/* (pkg/endpoint/policy.go:143-390, endpoint.go:2572)   */
/* ------------------------------------------------------------------ */
/* One L4Filter of an endpoint's resolved L4 policy (pkg/policy/l4.go:83-103),
 * as Repository.ResolveL4{Ingress,Egress}Policy (repository.go:240-329) left
 * it, wildcardL3L4Rules included; the caller (cilium_amd/policy.py) resolves
 * the filters, which is O(rules) per endpoint.  Its Endpoints selectors are
 * ids into the program's selector table. */
typedef struct cgpu_l4_filter {
	uint32_t endpoint;         /* row of the endpoint label sets */
	uint32_t sels_off, n_sels; /* selectors filter_sels[sels_off, +n_sels) */
	uint16_t port;             /* L4Filter.Port, host order */
	uint8_t proto;             /* L4Filter.U8Proto */
	uint8_t dir;               /* CGPU_L3_INGRESS / CGPU_L3_EGRESS */
	uint16_t proxy_port;       /* realizedRedirects[ProxyID] (host order) of a redirect */
	uint8_t redirect;          /* L7Parser != "": no keys while proxy_port is 0 (policy.go:158-166) */
	uint8_t pad;
} cgpu_l4_filter;

#define CGPU_MS_ALLOW_LOCALHOST 4u   /* AlwaysAllowLocalhost() || DesiredL4Policy.HasRedirect() */
#define CGPU_MS_HOST_ALLOWS_WORLD 8u /* option HostAllowsWorld (policy.go:305-315) */
typedef struct cgpu_mapstate_spec {
	const cgpu_l4_filter *filters;
	uint32_t n_filters;
	const uint32_t *filter_sels;
	uint32_t n_filter_sels;
	const uint32_t *ep_map;   /* [n_endpoints] the policy-map index (`ep`) of each endpoint row */
	const uint32_t *ep_flags; /* [n_endpoints] CGPU_L3_*_ENFORCED | CGPU_MS_* */
	const uint32_t *identity; /* [n_identities] NumericIdentity of each identity row */
} cgpu_mapstate_spec;

typedef struct cgpu_mapstate_stats {
	uint64_t desired;   /* keys in the desired MapStates */
	uint64_t added;     /* AllowKey of a key the map did not hold */
	uint64_t updated;   /* AllowKey of a held key with another proxy port (counters restart) */
	uint64_t deleted;   /* DeleteKey of a held key no longer desired */
	uint64_t unchanged; /* desired keys already held with the same proxy port */
	uint64_t failed;    /* AllowKey / DeleteKey errors (e.g. -E2BIG) */
} cgpu_mapstate_stats;

/*
 * computeDesiredPolicyMapState for every endpoint row, then syncPolicyMap
 * into that endpoint's policy map:
 *   1. L4 keys {identity, port, proto, dir} -> proxy_port for every identity
 *      any of a filter's selectors matches (computeDesiredL4PolicyMapEntries,
 *      policy.go:143-192); one wave per (filter, 64 identities) on the device;
 *   2. {HOST_ID, 0, 0, ingress} if CGPU_MS_ALLOW_LOCALHOST, then
 *      {WORLD_ID, 0, 0, ingress} if also CGPU_MS_HOST_ALLOWS_WORLD
 *      (determineAllowLocalhost / determineAllowFromWorld, policy.go:284-315);
 *   3. the L3 keys of cgpu_l3_compile under the endpoint's enforcement bits
 *      (policy.go:317-390).
 * Sync (endpoint.go:2572-2652): held keys not desired are deleted; desired
 * keys absent or held with another proxy port are written (the value, and
 * with it the counters, restart); the rest are left alone.  Like the
 * reference, a failing key does not stop the others: the first error is
 * returned after all keys were tried.  Changes go to the host mirror and
 * become visible to classify at the next cgpu_commit (a small delta patches
 * the device tables in place).  All inputs are host pointers.
 */
int cgpu_mapstate_sync(cgpu_ctx *ctx, const cgpu_l3_program *prog, const cgpu_label_sets *endpoints,
		       const cgpu_label_sets *identities, const cgpu_mapstate_spec *spec,
		       cgpu_mapstate_stats *stats);

/* ------------------------------------------------------------------ */
/* counters                                                             */
/* ------------------------------------------------------------------ */
/*
 * Batch launches accumulate into a DELTA buffer of cgpu_counter_delta_bytes()
 * bytes: u64 {packets, bytes} per policy slot, then u64 {count, bytes} per
 * {reason 0..255, dir 0..3} metrics key.  By default the context owns it;
 * cgpu_counter_bind() points launches at a caller-owned device buffer (e.g.
 * a torch tensor that is all-reduced over RCCL across ranks holding the same
 * committed tables).  cgpu_counter_fold() adds the delta into the
 * totals reported by cgpu_policy_lookup / cgpu_metrics_read and zeroes it.
 */
size_t cgpu_counter_delta_bytes(cgpu_ctx *ctx);
int cgpu_counter_bind(cgpu_ctx *ctx, void *device_buf, size_t bytes);
int cgpu_counter_fold(cgpu_ctx *ctx, void *stream);
/* out: [256][4][2] u64 {count, bytes} (folds and synchronizes first) */
int cgpu_metrics_read(cgpu_ctx *ctx, uint64_t *out);
int cgpu_counters_reset(cgpu_ctx *ctx);
/* Popularity-ordered counter slots: hot slots [0, hot_counter_slots)
 * accumulate in LDS (one flush per workgroup), the others cost a global
 * atomic per hit.  Slots start out by key class (L3-only / identity-wildcard
 * keys hot); this re-assigns them by measured traffic: the keys with the most
 * packets so far take the hot slots (ties: class, endpoint, key -- replicas
 * with the same folded totals choose alike), counters move with their keys,
 * and the policy tables are republished.  A control-plane call: it
 * synchronizes the device and folds the delta buffer; every map change must be
 * committed (else -EBUSY) and no batch may run on the context meanwhile.
 * *moved_out (optional) = keys whose slot changed. */
int cgpu_counters_rebalance(cgpu_ctx *ctx, uint64_t *moved_out);
/* Classify launches keep a packed counter accumulator of 8 B per policy
 * slot (policy_max_total x 8 B of HBM) for each stream they ran on, at most
 * 16 of them; a 17th stream recycles the least recently used one after that
 * stream's last launch finished.  A caller that is done with a stream (e.g.
 * before hipStreamDestroy) releases its buffer here; waits for the stream's
 * last launch of this context. */
int cgpu_stream_release(cgpu_ctx *ctx, void *stream);

/* ------------------------------------------------------------------ */
/* multi-GPU counter reduction (consumer: the agent's      */
/* metrics export, pkg/maps/metricsmap/metricsmap.go:170 SyncMetricsMap)*/
/* ------------------------------------------------------------------ */
/* One process (or context) per GPU holds the same committed tables and
 * classifies its own shard of the stream.  Rank 0 creates a communicator id
 * and hands it to every rank out of band (the agent's own channel); each
 * rank then joins with cgpu_comm_init (collective: blocks until all
 * nranks joined).  cgpu_counters_allreduce enqueues the RCCL SUM (over
 * xGMI) of the delta buffer on `stream`; after it every rank's delta holds
 * the counts of all ranks, and cgpu_counter_fold adds them to the totals
 * (integer sums: bit-exact against one GPU classifying the whole stream). */
#define CGPU_COMM_ID_BYTES 128
int cgpu_comm_id_create(uint8_t *id_out /* [CGPU_COMM_ID_BYTES] */);
int cgpu_comm_init(cgpu_ctx *ctx, const uint8_t *id, int nranks, int rank);
int cgpu_counters_allreduce(cgpu_ctx *ctx, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* CGPU_H */
