/*
 * TEST INFRASTRUCTURE — the reference oracle for the STATEFUL service step
 * of the endpoint's egress path (VERDICT r2 "next" 7; SURVEY §8f rows 1 + 3).
 * Built ONLY in the development container into oracle/_ref/libref_ctlb.so
 * (oracle/Makefile); run only by oracle/gen_golden.py.
 *
 * Compiles the reference's bpf/lib/{lb,conntrack,policy,eps}.h as host C
 * under node_config.h + lxc_config.h (LB_L3, LB_L4, CONNTRACK,
 * CONNTRACK_ACCOUNTING; loopback LB on) with -DSKIP_DEBUG, unmodified, and
 * drives, per packet and in order, over ONE conntrack map:
 *   egress  handle_ipv4_from_lxc (bpf_lxc.c:429-537): lb4_extract_key,
 *           lb4_lookup_service, lb4_local (lb.h:700-775: ct_lookup4 with
 *           CT_SERVICE, slave select + ct_create4 of the service entry on
 *           CT_NEW -- DROP_NO_SERVICE when that create fails --, the stored
 *           slave otherwise, re-selection + ct_update4_slave when the backend
 *           is gone, lb4_xlate of the frame), then ct_lookup4(CT_EGRESS) on
 *           the translated tuple, dstID from ipcache(orig_dip), policy on the
 *           rewritten dport, the reply/related skip, ct_delete4 of a denied
 *           ESTABLISHED entry, ct_create4(CT_EGRESS) with the service's
 *           ct_state (rev_nat_index, slave, loopback, the address entry);
 *           a hit entry's reverse NAT goes through the empty
 *           cilium_lb4_reverse_nat map (lb.h lb4_rev_nat: a no-op).
 *   ingress ipv4_policy (bpf_lxc.c:862-950) as harness_ct.c.
 * IPv6 (ref_ctlb_classify_v6): ipv6_l3_from_lxc (bpf_lxc.c:108-215):
 *           lb6_extract_key, lb6_lookup_service, lb6_local (lb.h:426-483:
 *           CT_SERVICE entries in CT_MAP6, the stored slave, fallback +
 *           ct_update6_slave, fail closed), lb6_xlate, then ct_lookup6
 *           (CT_EGRESS), dstID from ipcache6(orig_dip) else CLUSTER_ID when
 *           the frame's daddr matches ROUTER_IP /64, policy_can_egress6,
 *           ct_create6 with the service's ct_state (no address entry on
 *           IPv6); ingress ipv6_policy as harness_ct.c.
 * Mocks: the CT map is a kernel htab with max_elem (-E2BIG); the service map
 * a hash; get_hash_recalc returns the injected skb->hash; the frame (Ethernet
 * + IPv4 without options + a 20-byte L4 header built from the tuple columns)
 * lives in a MAP_32BIT buffer that skb_load_bytes / skb_store_bytes read and
 * write; checksum helpers return 0; ktime_get_ns the batch clock.
 */
#include <stdio.h>
#include <string.h>
#include <stdint.h>
#include <sys/mman.h>

#include "lib/utils.h"
#include "node_config.h"
#include "lxc_config.h"
#undef DROP_NOTIFY
#undef TRACE_NOTIFY
#undef DEBUG
#include "lib/common.h"
#include "lib/maps.h"
#include "lib/ipv4.h"
#include "lib/l4.h"
#include "lib/policy.h"
#include "lib/eps.h"
#include "lib/lb.h"

#include "mockmap.h"

#define REF_MAX_EP 64

static int ct_map4, ct_map6;
static struct mockmap ct, ct6, svc_m, svc6_m, ipcache, policy_maps[REF_MAX_EP];
static size_t ct_max = 1u << 20, ct6_max = 1u << 20;
static int cur_ep, inited, pol_probes, pol_hit_probe;
static uint64_t now_ns;
static uint32_t inj_hash;
static unsigned char *frame_buf;
static uint32_t frame_len;

static void *mock_lookup(void *map, const void *key)
{
	if (map == &POLICY_MAP) {
		void *v;
		pol_probes++;
		v = mockmap_lookup(&policy_maps[cur_ep], key);
		if (v)
			pol_hit_probe = pol_probes;
		return v;
	}
	if (map == &cilium_ipcache)
		return mockmap_lookup(&ipcache, key);
	if (map == &ct_map4)
		return mockmap_lookup(&ct, key);
	if (map == &cilium_lb4_services)
		return mockmap_lookup(&svc_m, key);
	if (map == &cilium_lb4_reverse_nat)
		return NULL;
	if (map == &ct_map6)
		return mockmap_lookup(&ct6, key);
	if (map == &cilium_lb6_services)
		return mockmap_lookup(&svc6_m, key);
	if (map == &cilium_lb6_reverse_nat)
		return NULL;
	fprintf(stderr, "ctlb harness: lookup on unexpected map %p\n", map);
	return NULL;
}

static int mock_update(void *map, const void *key, const void *val, uint32_t flags)
{
	if (map == &ct_map6) {
		if (!mockmap_lookup(&ct6, key) && ct6.n >= ct6_max)
			return -7; /* -E2BIG */
		mockmap_update(&ct6, key, val);
		return 0;
	}
	if (map != &ct_map4)
		return -1;
	if (!mockmap_lookup(&ct, key) && ct.n >= ct_max)
		return -7; /* -E2BIG */
	mockmap_update(&ct, key, val);
	return 0;
}

static int mock_delete(void *map, const void *key)
{
	if (map == &ct_map6)
		return mockmap_delete(&ct6, key) ? 0 : -2;
	if (map != &ct_map4)
		return -1;
	return mockmap_delete(&ct, key) ? 0 : -2;
}

static uint64_t mock_ktime(void) { return now_ns; }

static int mock_load(struct __sk_buff *skb, uint32_t off, void *to, uint32_t len)
{
	if ((uint64_t)off + len > frame_len)
		return -14;
	memcpy(to, frame_buf + off, len);
	return 0;
}

static int mock_store(struct __sk_buff *skb, uint32_t off, const void *from, uint32_t len,
		      uint32_t flags)
{
	if ((uint64_t)off + len > frame_len)
		return -14;
	memcpy(frame_buf + off, from, len);
	return 0;
}

static uint32_t mock_hash(struct __sk_buff *skb) { return inj_hash; }
static uint32_t mock_hash_invalid(struct __sk_buff *skb) { return 0; }
static int mock_csum_diff(void *from, uint32_t fs, void *to, uint32_t ts, uint32_t seed) { return 0; }
static int mock_csum_replace(struct __sk_buff *skb, uint32_t off, uint32_t from, uint32_t to,
			     uint32_t flags) { return 0; }

static int ensure_init(void)
{
	if (inited)
		return 0;
	for (int i = 0; i < REF_MAX_EP; i++)
		mockmap_init(&policy_maps[i], MOCK_HASH, sizeof(struct policy_key),
			     sizeof(struct policy_entry));
	mockmap_init(&ipcache, MOCK_LPM, sizeof(struct ipcache_key),
		     sizeof(struct remote_endpoint_info));
	mockmap_init(&ct, MOCK_HASH, sizeof(struct ipv4_ct_tuple), sizeof(struct ct_entry));
	mockmap_init(&svc_m, MOCK_HASH, sizeof(struct lb4_key), sizeof(struct lb4_service));
	mockmap_init(&ct6, MOCK_HASH, sizeof(struct ipv6_ct_tuple), sizeof(struct ct_entry));
	mockmap_init(&svc6_m, MOCK_HASH, sizeof(struct lb6_key), sizeof(struct lb6_service));
	frame_buf = mmap(NULL, 1 << 12, PROT_READ | PROT_WRITE,
			 MAP_PRIVATE | MAP_ANONYMOUS | MAP_32BIT, -1, 0);
	if (frame_buf == MAP_FAILED)
		return -1;
	map_lookup_elem = mock_lookup;
	map_update_elem = mock_update;
	map_delete_elem = mock_delete;
	ktime_get_ns = mock_ktime;
	get_hash_recalc = mock_hash;
	set_hash_invalid = mock_hash_invalid;
	skb_load_bytes = mock_load;
	skb_store_bytes = mock_store;
	csum_diff = mock_csum_diff;
	l3_csum_replace = mock_csum_replace;
	l4_csum_replace = mock_csum_replace;
	inited = 1;
	return 0;
}

void ref_ctlb_reset(size_t max_elem)
{
	ensure_init();
	for (int i = 0; i < REF_MAX_EP; i++)
		mockmap_clear(&policy_maps[i]);
	mockmap_clear(&ipcache);
	mockmap_clear(&ct);
	mockmap_clear(&svc_m);
	mockmap_clear(&ct6);
	mockmap_clear(&svc6_m);
	ct_max = ct6_max = max_elem;
}

void ref_ctlb_set_now(uint32_t sec) { now_ns = (uint64_t)sec * NSEC_PER_SEC; }
int ref_ctlb_policy_update(int ep, const void *key, const void *entry)
{
	ensure_init();
	return (ep < 0 || ep >= REF_MAX_EP) ? -1 : mockmap_update(&policy_maps[ep], key, entry);
}
int ref_ctlb_policy_read(int ep, const void *key, void *entry_out)
{
	void *v = mockmap_lookup(&policy_maps[ep], key);
	if (!v)
		return -1;
	memcpy(entry_out, v, sizeof(struct policy_entry));
	return 0;
}
int ref_ctlb_policy_delete(int ep, const void *key)
{
	return (ep < 0 || ep >= REF_MAX_EP) ? -1 : (mockmap_delete(&policy_maps[ep], key) ? 0 : -2);
}
/* a conntrack entry installed by the agent (bpf(2) BPF_ANY) */
int ref_ctlb_ct_update(const void *key, const void *val) { ensure_init(); return mock_update(&ct_map4, key, val, 0); }
int ref_ctlb_ipcache_update(const void *key, const void *info) { ensure_init(); return mockmap_update(&ipcache, key, info); }
int ref_ctlb_svc_update(const void *key, const void *val) { ensure_init(); return mockmap_update(&svc_m, key, val); }
int ref_ctlb_svc_delete(const void *key) { ensure_init(); return mockmap_delete(&svc_m, key) ? 0 : -2; }
size_t ref_ctlb_count(void) { return ct.n; }
int ref_ctlb_svc6_update(const void *key, const void *val) { ensure_init(); return mockmap_update(&svc6_m, key, val); }
int ref_ctlb_svc6_delete(const void *key) { ensure_init(); return mockmap_delete(&svc6_m, key) ? 0 : -2; }
int ref_ctlb_ct6_update(const void *key, const void *val) { ensure_init(); return mock_update(&ct_map6, key, val, 0); }
size_t ref_ctlb6_count(void) { return ct6.n; }
int ref_ctlb6_entry(size_t i, void *key_out, void *val_out)
{
	if (i >= ct6.n)
		return -1;
	memcpy(key_out, ct6.keys + i * ct6.ksz, ct6.ksz);
	memcpy(val_out, ct6.vals + i * ct6.vsz, ct6.vsz);
	return 0;
}
int ref_ctlb_entry(size_t i, void *key_out, void *val_out)
{
	if (i >= ct.n)
		return -1;
	memcpy(key_out, ct.keys + i * ct.ksz, ct.ksz);
	memcpy(val_out, ct.vals + i * ct.vsz, ct.vsz);
	return 0;
}

/* Ethernet + IPv4 (ihl 5) + a 20-byte L4 header from the tuple columns */
static void build_frame(uint32_t saddr, uint32_t daddr, uint16_t sport, uint16_t dport, uint8_t proto,
			uint16_t l4w, uint32_t len)
{
	memset(frame_buf, 0, 64);
	frame_buf[12] = 0x08;
	frame_buf[13] = 0x00;
	struct iphdr *ip4 = (struct iphdr *)(frame_buf + ETH_HLEN);
	ip4->ihl = 5;
	ip4->version = 4;
	ip4->tot_len = bpf_htons(40);
	ip4->protocol = proto;
	ip4->saddr = saddr;
	ip4->daddr = daddr;
	uint8_t *l4 = frame_buf + ETH_HLEN + 20;
	if (proto == IPPROTO_ICMP) {
		l4[0] = (uint8_t)l4w;
	} else {
		memcpy(l4, &sport, 2);
		memcpy(l4 + 2, &dport, 2);
		if (proto == IPPROTO_TCP) {
			l4[12] = (uint8_t)l4w;
			l4[13] = (uint8_t)(l4w >> 8);
		}
	}
	frame_len = ETH_HLEN + 40;
	(void)len;
}

/*
 * One packet through the stateful service step + conntrack + ipcache +
 * policy, in order.  Outputs as ref_ct_classify_v4, plus the translated
 * daddr / dport of the frame (egress) and whether a service matched.
 */
int ref_ctlb_classify_v4(uint32_t saddr_be, uint32_t daddr_be, uint16_t sport_be, uint16_t dport_be,
			 uint8_t proto, uint16_t l4w, uint8_t flags, uint32_t len, int ep,
			 uint32_t seclabel, uint32_t hash, uint32_t cfg_src_identity, int *ct_ret,
			 uint32_t *identity_out, int *stage_out, uint32_t *xdaddr, uint16_t *xdport,
			 int *svc_hit)
{
	struct ipv4_ct_tuple tuple = {};
	struct ct_state ct_state = {}, ct_state_new = {};
	struct csum_offset csum_off = {};
	struct lb4_key key = {};
	struct lb4_service *svc;
	struct __sk_buff skb;
	struct remote_endpoint_info *info;
	bool monitor = false;
	int egress = flags & 1, frag = (flags >> 1) & 1;
	int ret, verdict, l4_off = ETH_HLEN + 20;
	uint32_t id;
	__be32 orig_dip;

	if (ensure_init())
		return -1;
	build_frame(saddr_be, daddr_be, sport_be, dport_be, proto, l4w, len);
	memset(&skb, 0, sizeof(skb));
	skb.data = (uint32_t)(unsigned long)frame_buf;
	skb.data_end = (uint32_t)(unsigned long)(frame_buf + frame_len);
	skb.len = len;
	skb.protocol = bpf_htons(ETH_P_IP);
	inj_hash = hash;
	cur_ep = ep;
	pol_probes = pol_hit_probe = 0;
	*identity_out = 0;
	*stage_out = 0;
	*svc_hit = 0;
	*ct_ret = 255;
	tuple.nexthdr = proto;
	tuple.daddr = daddr_be;
	tuple.saddr = saddr_be;

	if (egress) {
		ret = lb4_extract_key(&skb, &tuple, l4_off, &key, &csum_off, CT_EGRESS);
		if (IS_ERR(ret)) {
			if (ret == DROP_UNKNOWN_L4)
				goto skip_service_lookup;
			*stage_out = 5;
			return ret;
		}
		ct_state_new.orig_dport = key.dport;
		if ((svc = lb4_lookup_service(&skb, &key)) != NULL) {
			*svc_hit = 1;
			ret = lb4_local(&ct_map4, &skb, ETH_HLEN, l4_off, &csum_off, &key, &tuple, svc,
					&ct_state_new, saddr_be);
			if (IS_ERR(ret)) {
				*stage_out = 6;
				memcpy(xdaddr, frame_buf + ETH_HLEN + 16, 4);
				memcpy(xdport, frame_buf + l4_off + 2, 2);
				return ret;
			}
		}
skip_service_lookup:
		orig_dip = tuple.daddr;
		memcpy(xdaddr, frame_buf + ETH_HLEN + 16, 4);
		memcpy(xdport, frame_buf + l4_off + 2, 2);
		ret = ct_lookup4(&ct_map4, &tuple, &skb, l4_off, CT_EGRESS, &ct_state, &monitor);
		*ct_ret = ret;
		if (ret < 0) {
			*stage_out = ret == DROP_CT_UNKNOWN_PROTO ? 4 : 5;
			return ret;
		}
		info = ipcache_lookup4(&cilium_ipcache, orig_dip, V4_CACHE_KEY_LEN);
		if (info && info->sec_label)
			id = info->sec_label;
		else if ((orig_dip & IPV4_CLUSTER_MASK) == IPV4_CLUSTER_RANGE)
			id = CLUSTER_ID;
		else
			id = WORLD_ID;
		verdict = policy_can_egress4(&skb, &tuple, id, ipv4_ct_tuple_get_daddr(&tuple));
		*identity_out = id;
		*stage_out = pol_hit_probe;
		if (ret != CT_REPLY && ret != CT_RELATED && verdict < 0) {
			if (ret == CT_ESTABLISHED)
				ct_delete4(&ct_map4, &tuple, &skb);
			return verdict;
		}
		if (ret == CT_NEW) {
			ct_state_new.src_sec_id = seclabel;
			ret = ct_create4(&ct_map4, &tuple, &skb, CT_EGRESS, &ct_state_new);
			if (IS_ERR(ret))
				return ret;
		} else if ((ret == CT_REPLY || ret == CT_RELATED) && ct_state.rev_nat_index) {
			ret = lb4_rev_nat(&skb, ETH_HLEN, l4_off, &csum_off, &ct_state, &tuple, 0);
			if (IS_ERR(ret))
				return ret;
		}
		return verdict > 0 ? verdict : 0;
	}

	/* ingress: bpf_netdev.c:374-404 identity, then ipv4_policy */
	memcpy(xdaddr, &daddr_be, 4);
	memcpy(xdport, &dport_be, 2);
	ret = ct_lookup4(&ct_map4, &tuple, &skb, l4_off, CT_INGRESS, &ct_state, &monitor);
	*ct_ret = ret;
	if (ret < 0) {
		*stage_out = ret == DROP_CT_UNKNOWN_PROTO ? 4 : 5;
		return ret;
	}
	{
		uint32_t src = cfg_src_identity;
		if (identity_is_reserved(src)) {
			info = ipcache_lookup4(&cilium_ipcache, saddr_be, V4_CACHE_KEY_LEN);
			if (info && info->sec_label && info->sec_label != CLUSTER_ID &&
			    info->sec_label != HOST_ID)
				src = info->sec_label;
		}
		id = src;
	}
	if (ret == CT_REPLY && ct_state.rev_nat_index && !ct_state.loopback) {
		int r2 = lb4_rev_nat(&skb, ETH_HLEN, l4_off, &csum_off, &ct_state, &tuple,
				     REV_NAT_F_TUPLE_SADDR);
		if (IS_ERR(r2))
			return r2;
	}
	verdict = policy_can_access_ingress(&skb, id, tuple.dport, tuple.nexthdr, 4, &saddr_be,
					    frag ? true : false);
	*identity_out = id;
	*stage_out = pol_hit_probe ? (frag ? 2 : pol_hit_probe) : 0;
	if (ret != CT_REPLY && ret != CT_RELATED && verdict < 0) {
		if (ret == CT_ESTABLISHED)
			ct_delete4(&ct_map4, &tuple, &skb);
		return DROP_POLICY;
	}
	if (ret == CT_NEW) {
		ct_state_new.orig_dport = tuple.dport;
		ct_state_new.src_sec_id = id;
		ret = ct_create4(&ct_map4, &tuple, &skb, CT_INGRESS, &ct_state_new);
		if (IS_ERR(ret))
			return ret;
	}
	if (verdict > 0 && (ret == CT_NEW || ret == CT_ESTABLISHED))
		return verdict;
	return 0;
}

/* Ethernet + IPv6 (no extension headers) + a 20-byte L4 header */
static void build_frame6(const uint8_t *sa16, const uint8_t *da16, uint16_t sport, uint16_t dport,
			 uint8_t proto, uint16_t l4w)
{
	memset(frame_buf, 0, 96);
	frame_buf[12] = 0x86;
	frame_buf[13] = 0xDD;
	struct ipv6hdr *ip6 = (struct ipv6hdr *)(frame_buf + ETH_HLEN);
	ip6->version = 6;
	ip6->nexthdr = proto;
	ip6->payload_len = bpf_htons(20);
	ip6->hop_limit = 64;
	memcpy(&ip6->saddr, sa16, 16);
	memcpy(&ip6->daddr, da16, 16);
	uint8_t *l4 = frame_buf + ETH_HLEN + 40;
	if (proto == IPPROTO_ICMPV6) {
		l4[0] = (uint8_t)l4w;
	} else {
		memcpy(l4, &sport, 2);
		memcpy(l4 + 2, &dport, 2);
		if (proto == IPPROTO_TCP) {
			l4[12] = (uint8_t)l4w;
			l4[13] = (uint8_t)(l4w >> 8);
		}
	}
	frame_len = ETH_HLEN + 60;
}

/*
 * One IPv6 packet through the stateful service step + conntrack + ipcache6
 * + policy, in order (see the header).  Outputs as ref_ctlb_classify_v4;
 * xdaddr16 / xdport: the frame's daddr / L4 bytes 2-3 after the service step.
 */
int ref_ctlb_classify_v6(const uint8_t *saddr16, const uint8_t *daddr16, uint16_t sport_be, uint16_t dport_be,
			 uint8_t proto, uint16_t l4w, uint8_t flags, uint32_t len, int ep, uint32_t seclabel,
			 uint32_t hash, uint32_t cfg_src_identity, int *ct_ret, uint32_t *identity_out,
			 int *stage_out, uint8_t *xdaddr16, uint16_t *xdport, int *svc_hit)
{
	struct ipv6_ct_tuple tuple = {};
	struct ct_state ct_state = {}, ct_state_new = {};
	struct csum_offset csum_off = {};
	struct lb6_key key = {};
	struct lb6_service *svc;
	struct __sk_buff skb;
	struct remote_endpoint_info *info;
	union v6addr sa, da, orig_dip, fdaddr, router_ip;
	bool monitor = false;
	int egress = flags & 1;
	int ret, verdict, l4_off = ETH_HLEN + 40;
	uint32_t id;
	BPF_V6(router_ip, ROUTER_IP);

	if (ensure_init())
		return -1;
	build_frame6(saddr16, daddr16, sport_be, dport_be, proto, l4w);
	memset(&skb, 0, sizeof(skb));
	skb.data = (uint32_t)(unsigned long)frame_buf;
	skb.data_end = (uint32_t)(unsigned long)(frame_buf + frame_len);
	skb.len = len;
	skb.protocol = bpf_htons(ETH_P_IPV6);
	inj_hash = hash;
	cur_ep = ep;
	pol_probes = pol_hit_probe = 0;
	*identity_out = 0;
	*stage_out = 0;
	*svc_hit = 0;
	*ct_ret = 255;
	memcpy(&sa, saddr16, 16);
	memcpy(&da, daddr16, 16);
	tuple.nexthdr = proto;
	ipv6_addr_copy(&tuple.daddr, &da);
	ipv6_addr_copy(&tuple.saddr, &sa);

	if (egress) {
		ret = lb6_extract_key(&skb, &tuple, l4_off, &key, &csum_off, CT_EGRESS);
		if (IS_ERR(ret)) {
			if (ret == DROP_UNKNOWN_L4)
				goto skip_service_lookup;
			*stage_out = 5;
			return ret;
		}
		ct_state_new.orig_dport = key.dport;
		if ((svc = lb6_lookup_service(&skb, &key)) != NULL) {
			*svc_hit = 1;
			ret = lb6_local(&ct_map6, &skb, ETH_HLEN, l4_off, &csum_off, &key, &tuple, svc,
					&ct_state_new);
			if (IS_ERR(ret)) {
				*stage_out = 6;
				memcpy(xdaddr16, frame_buf + ETH_HLEN + 24, 16);
				memcpy(xdport, frame_buf + l4_off + 2, 2);
				return ret;
			}
		}
skip_service_lookup:
		ipv6_addr_copy(&orig_dip, &tuple.daddr);
		memcpy(xdaddr16, frame_buf + ETH_HLEN + 24, 16);
		memcpy(xdport, frame_buf + l4_off + 2, 2);
		ret = ct_lookup6(&ct_map6, &tuple, &skb, l4_off, CT_EGRESS, &ct_state, &monitor);
		*ct_ret = ret;
		if (ret < 0) {
			*stage_out = ret == DROP_CT_UNKNOWN_PROTO ? 4 : 5;
			return ret;
		}
		memcpy(&fdaddr, frame_buf + ETH_HLEN + 24, 16); /* ip6->daddr after revalidate */
		info = ipcache_lookup6(&cilium_ipcache, &orig_dip, V6_CACHE_KEY_LEN);
		if (info && info->sec_label)
			id = info->sec_label;
		else if (ipv6_match_prefix_64(&fdaddr, &router_ip))
			id = CLUSTER_ID;
		else
			id = WORLD_ID;
		verdict = policy_can_egress6(&skb, &tuple, id, ipv6_ct_tuple_get_daddr(&tuple));
		*identity_out = id;
		*stage_out = pol_hit_probe;
		if (ret != CT_REPLY && ret != CT_RELATED && verdict < 0) {
			if (ret == CT_ESTABLISHED)
				ct_delete6(&ct_map6, &tuple, &skb);
			return verdict;
		}
		if (ret == CT_NEW) {
			ct_state_new.src_sec_id = seclabel;
			ret = ct_create6(&ct_map6, &tuple, &skb, CT_EGRESS, &ct_state_new);
			if (IS_ERR(ret))
				return ret;
		}
		/* CT_REPLY / CT_RELATED with rev_nat_index: lb6_rev_nat through the
		 * empty cilium_lb6_reverse_nat map, a no-op (lb.h:305-317) */
		return verdict > 0 ? verdict : 0;
	}

	/* ingress: ipv6_policy as harness_ct.c ref_ct_classify_v6 */
	memcpy(xdaddr16, daddr16, 16);
	memcpy(xdport, &dport_be, 2);
	{
		uint32_t w3;
		memcpy(&w3, daddr16 + 12, 4);
		ct_state_new.rev_nat_index = w3 & 0xFFFF;
	}
	ret = ct_lookup6(&ct_map6, &tuple, &skb, l4_off, CT_INGRESS, &ct_state, &monitor);
	*ct_ret = ret;
	if (ret < 0) {
		*stage_out = ret == DROP_CT_UNKNOWN_PROTO ? 4 : 5;
		return ret;
	}
	{
		uint32_t src = cfg_src_identity;
		if (identity_is_reserved(src)) {
			info = ipcache_lookup6(&cilium_ipcache, &sa, V6_CACHE_KEY_LEN);
			if (info && info->sec_label && info->sec_label != CLUSTER_ID)
				src = info->sec_label;
		}
		id = src;
	}
	verdict = policy_can_access_ingress(&skb, id, tuple.dport, tuple.nexthdr, sizeof(tuple.saddr),
					    &tuple.saddr, false);
	*identity_out = id;
	*stage_out = pol_hit_probe;
	if (ret != CT_REPLY && ret != CT_RELATED && verdict < 0) {
		if (ret == CT_ESTABLISHED)
			ct_delete6(&ct_map6, &tuple, &skb);
		return DROP_POLICY;
	}
	if (ret == CT_NEW) {
		ct_state_new.orig_dport = tuple.dport;
		ct_state_new.src_sec_id = id;
		ret = ct_create6(&ct_map6, &tuple, &skb, CT_INGRESS, &ct_state_new);
		if (IS_ERR(ret))
			return ret;
	}
	if (verdict > 0 && (ret == CT_NEW || ret == CT_ESTABLISHED))
		return verdict;
	return 0;
}
