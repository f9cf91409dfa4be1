/* Internal interface between host.cpp (C ABI, table compiler) and
 * kernels.hip (gfx950 kernels).  Not exported. */
#ifndef CGPU_LAUNCH_H
#define CGPU_LAUNCH_H

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "tables.h"
#include "../../include/cgpu.h"

struct classify_v4_args {
	const uint32_t *saddr, *daddr;
	const uint16_t *dport;
	const uint8_t *proto, *flags;
	const uint32_t *len;
	const uint16_t *ep;
	int32_t *verdict;
	uint32_t *identity;
	uint8_t *stage;
	uint64_t *delta; /* [2 * n_ctr_slots] policy + [CGPU_METRICS_WORDS] metrics */
	uint64_t n;
	uint64_t *pk;    /* [n_ctr_slots] packed cold-slot accumulator, zero between calls */
	/* egress service step first (cgpu_classify_v4_lb) */
	int lb;
	const uint16_t *sport;
	const uint32_t *hash; /* NULL: flow_hash(saddr, daddr, sport, dport, proto) */
	/* with lb: the XDP prefilter before every ingress tuple (cgpu_classify_v4_cascade) */
	int xdp;
};

hipError_t launch_classify_v4(const cgpu_snapshot &s, const classify_v4_args &a, hipStream_t st);

struct classify_v6_args {
	const uint8_t *saddr16, *daddr16;
	const uint16_t *dport;
	const uint8_t *proto, *flags;
	const uint32_t *len;
	const uint16_t *ep;
	int32_t *verdict;
	uint32_t *identity;
	uint8_t *stage;
	uint64_t *delta;
	uint64_t n;
	uint64_t *pk; /* packed cold-slot accumulator (per stream) */
	/* egress service step first (cgpu_classify_v6_lb) */
	int lb;
	const uint16_t *sport;
	const uint32_t *hash; /* NULL: flow_hash(fold6(saddr), fold6(daddr), sport, dport, proto) */
	/* scratch of n u32 (optional): the x4 schedule's ipcache pre-pass
	 * (k_ipc6_pre) writes every tuple's trie entry there */
	uint32_t *ipc_e;
};

hipError_t launch_classify_v6(const cgpu_snapshot &s, const classify_v6_args &a, hipStream_t st);

struct prefilter_args {
	const uint32_t *saddr4, *daddr4;
	const uint8_t *saddr16, *daddr16;
	const uint8_t *flags;
	uint8_t *verdict;
	uint64_t n;
};

hipError_t launch_prefilter_v4(const cgpu_snapshot &s, const prefilter_args &a, hipStream_t st);
hipError_t launch_prefilter_v6(const cgpu_snapshot &s, const prefilter_args &a, hipStream_t st);

struct lb4_args {
	const uint32_t *saddr, *daddr;
	const uint16_t *sport, *dport;
	const uint8_t *proto;
	const uint32_t *hash;
	int32_t *ret;
	uint32_t *saddr_out, *daddr_out;
	uint16_t *dport_out, *rev_nat_out, *slave_out;
	uint64_t n;
	int mode; /* CGPU_LB_NETDEV / CGPU_LB_LXC */
};

hipError_t launch_lb4(const cgpu_snapshot &s, const lb4_args &a, hipStream_t st);

/* raw frames (cgpu_frames_parse / cgpu_classify_frames) */
struct frames_args {
	const uint8_t *data;
	const uint32_t *len;
	const uint8_t *flags;
	const uint16_t *ep;
	uint32_t stride;
	uint64_t n;
	/* parse outputs (any but status may be NULL) */
	int32_t *status;
	uint8_t *family, *saddr16, *daddr16;
	uint16_t *dport;
	uint8_t *proto, *tflags;
	/* classify outputs */
	int32_t *verdict;
	uint32_t *identity;
	uint8_t *stage;
	uint64_t *delta;
	uint64_t *pk; /* the stream's packed cold-slot accumulator (classify) */
};

hipError_t launch_frames_parse(const cgpu_snapshot &s, const frames_args &a, hipStream_t st);

/* scratch of the frames x4 schedule (launch_classify_frames_x4): the IPv4
 * policy-tuple columns [n] and the compacted IPv6 ones [n] with their
 * results; every column 16-byte aligned */
struct frames_x4 {
	uint32_t *sa4, *da4;
	uint16_t *dport;
	uint8_t *proto, *fl;
	uint4 *sa6, *da6;
	uint16_t *dport6;
	uint8_t *proto6, *fl6;
	uint32_t *len6;
	uint16_t *ep6;
	uint32_t *idx6;
	int32_t *v6;
	uint32_t *id6;
	uint8_t *st6;
	uint32_t *n6;
};
/* bytes of that scratch for n frames, and its carving */
size_t frames_x4_bytes(uint64_t n);
frames_x4 frames_x4_carve(void *base, uint64_t n);
hipError_t launch_classify_frames_x4(const cgpu_snapshot &s, const frames_args &a, const frames_x4 &c,
				     hipStream_t st);
hipError_t launch_classify_frames(const cgpu_snapshot &s, const frames_args &a, hipStream_t st);

/* stateful classification (cgpu_classify_v4_ct): packet columns, outputs,
 * and the caller-allocated scratch (ct_scratch_layout in host.cpp) */
struct ct_launch {
	const void *saddr, *daddr; /* IPv4: u32 per packet; IPv6: 16 bytes (16-byte aligned) */
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
	uint4 *rec; /* [2n] IPv4, [4n] IPv6 */
	uint32_t *gkey, *gkey_sorted, *idx, *idx_sorted;
	uint8_t *head;
	uint32_t *heads, *n_heads;
	uint32_t *heads_pos; /* [n] scratch for the longest-first group sort */
	void *temp;
	size_t temp_bytes;
	/* the stateful service step (cgpu_classify_v4_ctlb); rec is [3n] */
	const uint32_t *hash; /* NULL: cgpu_flow_hash */
	uint4 *svc_out;       /* [n] */
	uint32_t *ctl;        /* [4] */
	uint8_t *flags2;      /* [2n] plain path, [4n] service path: phase-2 candidates */
	uint8_t *pcls;        /* [n] service path: each packet's phase-2 class (k_ct_prep) */
	uint64_t *pk;         /* [n_ctr_slots] packed counters, zero between calls */
	void *xdaddr;         /* [n] optional (IPv6: 16 bytes each) */
	uint16_t *xdport;     /* [n] optional */
	uint32_t dflt;        /* nonzero: group-default results (CGPU_CT_DFLT) */
};

size_t ct_temp_bytes(uint64_t n);
/* ctmap.GC RemoveExpired on the device map; compaction into an empty table */
hipError_t launch_ct_gc(const ct_table &T, bool v6, uint32_t time, uint32_t *deleted, hipStream_t st);
hipError_t launch_ct_rehash(const ct_table &src, const ct_table &dst, bool v6, hipStream_t st);

hipError_t launch_classify_v4_ct(const cgpu_snapshot &s, const ct_table &T, const ct_launch &L,
				 hipStream_t st);
/* the same over cilium_ct6_global (tables.h CtK6 slots), rec [4n] */
hipError_t launch_classify_v6_ct(const cgpu_snapshot &s, const ct_table &T, const ct_launch &L,
				 hipStream_t st);

/* behind the IPv6 stateful service step (cilium_ct6_global, rec [4n],
 * svc_out [2n], xdaddr 16 bytes per packet) */
hipError_t launch_classify_v6_ctlb(const cgpu_snapshot &s, const ct_table &T, const ct_launch &L,
				   hipStream_t st);
/* the same behind the stateful service step (cilium_ct4_global, rec [3n]) */
hipError_t launch_classify_v4_ctlb(const cgpu_snapshot &s, const ct_table &T, const ct_launch &L,
				   hipStream_t st);

/* L3 MapState compilation (cgpu_l3_compile): device copies of the program */
struct l3_launch {
	const cgpu_selector *sel;
	const cgpu_requirement *req;
	const uint32_t *val;
	const uint32_t *rule_subject, *rule_clauses;
	uint32_t n_rules;
	const cgpu_l3_clause *cl;
	const uint32_t *ep_off, *id_off;
	const cgpu_label *ep_lab, *id_lab;
	uint32_t n_ep, n_id, flags;
	uint8_t *subj, *allow;
	/* cgpu_mapstate_sync only (nullptr / 0 for cgpu_l3_compile) */
	const uint32_t *ep_flags; /* per endpoint: replaces `flags` */
	const cgpu_l4_filter *flt;
	const uint32_t *flt_sels;
	uint32_t n_flt;
	uint64_t *l4bits; /* [n_flt][ceil(n_id / 64)] identity bitmaps */
};

hipError_t launch_l3_compile(const l3_launch &L, hipStream_t st);

/* *out += sum of table_sum_word over `bytes` bytes of buf from byte `off`
 * (a multiple of 8) */
hipError_t launch_table_sum(const void *buf, size_t off, size_t bytes, uint64_t *out, hipStream_t st);

/* totals[i] += delta[i]; delta[i] = 0 over n u64 words */
hipError_t launch_fold(uint64_t *totals, uint64_t *delta, uint64_t n, hipStream_t st);
/* a copy by the CUs between device memory and a device-visible page-locked
 * host range (either way); hipErrorInvalidValue unless dst and src are
 * 16-byte aligned */
hipError_t launch_copy_host(void *dst, const void *src, uint64_t bytes, hipStream_t st);
/* up to 8 such copies in one launch (every segment 16-byte aligned) */
struct copy_seg {
	void *dst;
	const void *src;
	uint64_t bytes;
};
struct copy_segs {
	copy_seg seg[8];
	uint32_t n;
};
hipError_t launch_copy_host_multi(const copy_segs &d, hipStream_t st);
/* totals[2*slot[i]] = pk[i]; totals[2*slot[i]+1] = by[i]; delta[..] = 0 */
hipError_t launch_slot_init(uint64_t *totals, uint64_t *delta, const uint32_t *slot,
			    const uint64_t *pk, const uint64_t *by, uint32_t n, hipStream_t st);

#endif
