/*
 * TEST INFRASTRUCTURE — the reference oracle for stateful conntrack on the
 * classification path.  Built ONLY in the development
 * container into oracle/_ref/libref_ct.so (oracle/Makefile); run only by
 * oracle/gen_golden.py.
 *
 * Compiles the reference's bpf/lib/{conntrack,policy,eps}.h as host C under
 * node_config.h + lxc_config.h (CONNTRACK, CONNTRACK_ACCOUNTING, and
 * NEEDS_TIMEOUT from lib/common.h:33), unmodified, and drives, per packet and
 * in order, the conntrack / policy part of the endpoint programs:
 *   egress  handle_ipv4_from_lxc (bpf_lxc.c:465-537): ct_lookup4(CT_EGRESS),
 *           dstID from ipcache(orig_dip) (:484-500), policy_can_egress4,
 *           "ret != CT_REPLY && ret != CT_RELATED && verdict < 0" -> delete
 *           the entry if CT_ESTABLISHED and return the verdict, CT_NEW ->
 *           ct_create4(CT_EGRESS) with src_sec_id = SECLABEL, then
 *           redirect_to_proxy(verdict) (:576) — every direction of ct.
 *   ingress ipv4_policy (bpf_lxc.c:893-950): ct_lookup4(CT_INGRESS),
 *           policy_can_access_ingress(src_label, tuple.dport, ...), the same
 *           reply/related skip and delete, CT_NEW -> ct_create4(CT_INGRESS)
 *           with src_sec_id = src_label, proxy redirect only for CT_NEW /
 *           CT_ESTABLISHED (:944).
 * The service lookup in front of egress (bpf_lxc.c:444-460) runs over an
 * empty service map (no translation, ct_state.addr = 0); no entry carries a
 * rev_nat_index, so lb4_rev_nat never runs.  The program's end result is
 * reported as: the DROP_* it returns, the proxy port it redirects to, or 0
 * (forwarded).
 *
 * IPv6 (ref_ct_classify_v6): the same for ct_lookup6 / ct_create6 /
 * ct_delete6 over CT_MAP6 (bpf_lxc.c:53-63), in the order of
 * ipv6_l3_from_lxc (bpf_lxc.c:108-203: dstID from ipcache6(orig_dip), else
 * CLUSTER_ID when ipv6_match_prefix_64(daddr, ROUTER_IP), else WORLD_ID) and
 * ipv6_policy (:731-800: the reverse NAT index of the created entry is
 * daddr.s6_addr32[3] & 0xFFFF, :748; a hit entry's rev_nat_index sends the
 * packet through lb6_rev_nat, which is a no-op over the empty
 * cilium_lb6_reverse_nat map, lib/lb.h:305-317; is_fragment false).  Ingress
 * identity as bpf_netdev.c:203-211 (no HOST_ID exception on IPv6), the label
 * the resolved source (FROM_HOST form).
 *
 * Mocks (writable helper pointers, bpf/include/bpf/api.h:101-118): the CT map
 * is a kernel htab (whole-key memcmp) with max_elem (new keys past it fail as
 * htab_map_update_elem does, -E2BIG); map_delete_elem removes; the policy map
 * and ipcache are the mockmap.c hash / LPM; ktime_get_ns returns the batch
 * clock set by ref_ct_set_now (seconds * 1e9); skb_load_bytes reads a 20-byte
 * L4 header built from the tuple columns (sport, dport, TCP header bytes
 * 12-13 or the ICMP type).
 */
#include <stdio.h>
#include <string.h>
#include <stdint.h>

#include "lib/utils.h"
#include "node_config.h"
#include "lxc_config.h"
#undef DROP_NOTIFY
#undef TRACE_NOTIFY
#undef DEBUG
#include "lib/common.h"
#include "lib/policy.h"
#include "lib/eps.h"
#include "lib/conntrack.h"

#include "mockmap.h"

#define REF_MAX_EP 64

/* stand in for the endpoint's CT_MAP4 (bpf_lxc.c:64-75) and CT_MAP6 (:53-63) */
static int ct_map4, ct_map6;
static struct mockmap ct, ct6;
static size_t ct_max = 1u << 20, ct6_max = 1u << 20;
static struct mockmap policy_maps[REF_MAX_EP];
static struct mockmap ipcache;
static int cur_ep, inited;
static int pol_probes, pol_hit_probe;
static uint64_t now_ns;
static uint8_t l4buf[20];

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
	if (map == &ct_map6)
		return mockmap_lookup(&ct6, key);
	fprintf(stderr, "ct harness: lookup on unexpected map %p\n", map);
	return NULL;
}

static int mock_update(void *map, const void *key, const void *val, uint32_t flags)
{
	struct mockmap *m = map == &ct_map4 ? &ct : map == &ct_map6 ? &ct6 : NULL;
	size_t max = map == &ct_map4 ? ct_max : ct6_max;
	if (!m)
		return -1;
	if (!mockmap_lookup(m, key) && m->n >= max)
		return -7; /* -E2BIG */
	mockmap_update(m, key, val);
	return 0;
}

static int mock_delete(void *map, const void *key)
{
	struct mockmap *m = map == &ct_map4 ? &ct : map == &ct_map6 ? &ct6 : NULL;
	if (!m)
		return -1;
	return mockmap_delete(m, key) ? 0 : -2;
}

static uint64_t mock_ktime(void) { return now_ns; }

static int mock_load(struct __sk_buff *skb, uint32_t off, void *to, uint32_t len)
{
	if ((uint64_t)off + len > sizeof(l4buf))
		return -14;
	memcpy(to, l4buf + off, len);
	return 0;
}

static void ensure_init(void)
{
	if (inited)
		return;
	for (int i = 0; i < REF_MAX_EP; i++)
		mockmap_init(&policy_maps[i], MOCK_HASH, sizeof(struct policy_key),
			     sizeof(struct policy_entry));
	mockmap_init(&ipcache, MOCK_LPM, sizeof(struct ipcache_key),
		     sizeof(struct remote_endpoint_info));
	mockmap_init(&ct, MOCK_HASH, sizeof(struct ipv4_ct_tuple), sizeof(struct ct_entry));
	mockmap_init(&ct6, MOCK_HASH, sizeof(struct ipv6_ct_tuple), sizeof(struct ct_entry));
	map_lookup_elem = mock_lookup;
	map_update_elem = mock_update;
	map_delete_elem = mock_delete;
	ktime_get_ns = mock_ktime;
	skb_load_bytes = mock_load;
	inited = 1;
}

void ref_ct_reset(size_t max_elem)
{
	ensure_init();
	for (int i = 0; i < REF_MAX_EP; i++)
		mockmap_clear(&policy_maps[i]);
	mockmap_clear(&ipcache);
	mockmap_clear(&ct);
	mockmap_clear(&ct6);
	ct_max = max_elem;
	ct6_max = max_elem;
}

int ref_ct_sizes(int *tuple_sz, int *entry_sz, int *tuple6_sz)
{
	*tuple_sz = sizeof(struct ipv4_ct_tuple);
	*entry_sz = sizeof(struct ct_entry);
	*tuple6_sz = sizeof(struct ipv6_ct_tuple);
	return 0;
}

void ref_ct_set_now(uint32_t sec) { now_ns = (uint64_t)sec * NSEC_PER_SEC; }

int ref_ct_policy_update(int ep, const void *key, const void *entry)
{
	ensure_init();
	if (ep < 0 || ep >= REF_MAX_EP)
		return -1;
	return mockmap_update(&policy_maps[ep], key, entry);
}

int ref_ct_policy_read(int ep, const void *key, void *entry_out)
{
	void *v;
	ensure_init();
	v = mockmap_lookup(&policy_maps[ep], key);
	if (!v)
		return -1;
	memcpy(entry_out, v, sizeof(struct policy_entry));
	return 0;
}

int ref_ct_policy_delete(int ep, const void *key)
{
	ensure_init();
	return mockmap_delete(&policy_maps[ep], key) ? 0 : -1;
}

int ref_ct_ipcache_update(const void *key, const void *info)
{
	ensure_init();
	return mockmap_update(&ipcache, key, info);
}

/* raw 14-byte ipv4_ct_tuple / 56-byte ct_entry, as bpf(2) copies them */
int ref_ct_update(const void *key, const void *val) { ensure_init(); return mock_update(&ct_map4, key, val, 0); }
int ref_ct_delete(const void *key) { ensure_init(); return mock_delete(&ct_map4, key); }
size_t ref_ct_count(void) { return ct.n; }
/* entry i of the map (any order): 0, or -1 past the end */
int ref_ct_entry(size_t i, void *key_out, void *val_out)
{
	if (i >= ct.n)
		return -1;
	memcpy(key_out, ct.keys + i * ct.ksz, ct.ksz);
	memcpy(val_out, ct.vals + i * ct.vsz, ct.vsz);
	return 0;
}

/* raw 38-byte ipv6_ct_tuple / 56-byte ct_entry of CT_MAP6 */
int ref_ct6_update(const void *key, const void *val) { ensure_init(); return mock_update(&ct_map6, key, val, 0); }
int ref_ct6_delete(const void *key) { ensure_init(); return mock_delete(&ct_map6, key); }
size_t ref_ct6_count(void) { return ct6.n; }
int ref_ct6_entry(size_t i, void *key_out, void *val_out)
{
	if (i >= ct6.n)
		return -1;
	memcpy(key_out, ct6.keys + i * ct6.ksz, ct6.ksz);
	memcpy(val_out, ct6.vals + i * ct6.vsz, ct6.vsz);
	return 0;
}

static void l4_header(uint8_t proto, uint16_t sport_be, uint16_t dport_be, uint16_t l4w)
{
	memset(l4buf, 0, sizeof(l4buf));
	if (proto == IPPROTO_ICMP || proto == IPPROTO_ICMPV6) {
		l4buf[0] = (uint8_t)l4w; /* icmphdr.type */
	} else {
		memcpy(l4buf, &sport_be, 2);
		memcpy(l4buf + 2, &dport_be, 2);
		if (proto == IPPROTO_TCP) {
			l4buf[12] = (uint8_t)l4w;        /* doff << 4 | reserved (bit 0: NS) */
			l4buf[13] = (uint8_t)(l4w >> 8); /* FIN 0x01 SYN 0x02 RST 0x04 PSH ACK ... */
		}
	}
}

/*
 * One IPv4 packet through conntrack + ipcache + policy, in order.
 * flags bit0 = egress (from-container), bit1 = is_fragment (ingress).
 * Outputs: the program's end result (return), *ct_ret = ct_lookup4's result
 * (CT_NEW 0 / ESTABLISHED 1 / REPLY 2 / RELATED 3, or its negative error),
 * *identity_out = label given to policy, *stage_out = policy probe that hit
 * (1 exact, 2 L3-only, 3 wildcard, 0 miss; 4 protocol gate).
 */
int ref_ct_classify_v4(uint32_t saddr_be, uint32_t daddr_be, uint16_t sport_be,
		       uint16_t dport_be, uint8_t proto, uint16_t l4w, uint8_t flags,
		       uint32_t len, int ep, uint32_t seclabel, uint32_t cfg_src_identity,
		       int cfg_secctx_world, int *ct_ret, uint32_t *identity_out,
		       int *stage_out)
{
	struct ipv4_ct_tuple tuple = {};
	struct ct_state ct_state = {}, ct_state_new = {};
	struct __sk_buff skb;
	bool monitor = false;
	int egress = flags & 1, frag = (flags >> 1) & 1;
	int ret, verdict;
	uint32_t label = 0, id;
	struct remote_endpoint_info *info;

	ensure_init();
	memset(&skb, 0, sizeof(skb));
	skb.len = len;
	cur_ep = ep;
	pol_probes = pol_hit_probe = 0;
	*identity_out = 0;
	*stage_out = 0;
	l4_header(proto, sport_be, dport_be, l4w);

	tuple.nexthdr = proto;
	tuple.daddr = daddr_be;
	tuple.saddr = saddr_be;
	ret = ct_lookup4(&ct_map4, &tuple, &skb, 0, egress ? CT_EGRESS : CT_INGRESS,
			 &ct_state, &monitor);
	*ct_ret = ret;
	if (ret < 0) {
		*stage_out = ret == DROP_CT_UNKNOWN_PROTO ? 4 : 5;
		return ret;
	}

	if (egress) {
		/* bpf_lxc.c:484-500, orig_dip = the packet's daddr */
		info = ipcache_lookup4(&cilium_ipcache, daddr_be, V4_CACHE_KEY_LEN);
		if (info && info->sec_label)
			id = info->sec_label;
		else if ((daddr_be & IPV4_CLUSTER_MASK) == IPV4_CLUSTER_RANGE)
			id = CLUSTER_ID;
		else
			id = WORLD_ID;
		verdict = policy_can_egress4(&skb, &tuple, id, ipv4_ct_tuple_get_daddr(&tuple));
	} else {
		/* bpf_netdev.c:374-404 (identity), then ipv4_policy */
		uint32_t src = cfg_src_identity;
		if (identity_is_reserved(src)) {
			info = ipcache_lookup4(&cilium_ipcache, saddr_be, V4_CACHE_KEY_LEN);
			if (info && info->sec_label && info->sec_label != CLUSTER_ID &&
			    info->sec_label != HOST_ID)
				src = info->sec_label;
		}
		id = cfg_secctx_world ? WORLD_ID : src;
		verdict = policy_can_access_ingress(&skb, id, tuple.dport, tuple.nexthdr, 0, NULL,
						    frag ? true : false);
	}
	*identity_out = id;
	*stage_out = pol_hit_probe ? (frag && !egress ? 2 : pol_hit_probe) : 0;
	(void)label;

	if (ret != CT_REPLY && ret != CT_RELATED && verdict < 0) {
		if (ret == CT_ESTABLISHED)
			ct_delete4(&ct_map4, &tuple, &skb);
		return egress ? verdict : DROP_POLICY;
	}
	if (ret == CT_NEW) {
		ct_state_new.orig_dport = tuple.dport;
		ct_state_new.src_sec_id = egress ? seclabel : id;
		ret = ct_create4(&ct_map4, &tuple, &skb, egress ? CT_EGRESS : CT_INGRESS,
				 &ct_state_new);
		if (IS_ERR(ret))
			return ret;
	}
	if (verdict > 0 && (egress || ret == CT_NEW || ret == CT_ESTABLISHED))
		return verdict; /* redirect_to_proxy: the proxy port */
	return 0;
}

/*
 * One IPv6 packet through conntrack + ipcache + policy, in order (the v6
 * endpoint programs, see the header).  Arguments and outputs as
 * ref_ct_classify_v4; addresses are 16 network-order bytes.
 */
int ref_ct_classify_v6(const uint8_t *saddr16, const uint8_t *daddr16, uint16_t sport_be,
		       uint16_t dport_be, uint8_t proto, uint16_t l4w, uint8_t flags, uint32_t len,
		       int ep, uint32_t seclabel, uint32_t cfg_src_identity, int *ct_ret,
		       uint32_t *identity_out, int *stage_out)
{
	struct ipv6_ct_tuple tuple = {};
	struct ct_state ct_state = {}, ct_state_new = {};
	struct __sk_buff skb;
	bool monitor = false;
	int egress = flags & 1;
	int ret, verdict;
	uint32_t id;
	union v6addr sa, da, router_ip;
	struct remote_endpoint_info *info;
	BPF_V6(router_ip, ROUTER_IP);

	ensure_init();
	memset(&skb, 0, sizeof(skb));
	skb.len = len;
	cur_ep = ep;
	pol_probes = pol_hit_probe = 0;
	*identity_out = 0;
	*stage_out = 0;
	l4_header(proto, sport_be, dport_be, l4w);
	memcpy(&sa, saddr16, 16);
	memcpy(&da, daddr16, 16);

	tuple.nexthdr = proto;
	ipv6_addr_copy(&tuple.daddr, &da);
	ipv6_addr_copy(&tuple.saddr, &sa);
	if (!egress) {
		/* ipv6_policy: ct_state_new.rev_nat_index = ip6->daddr.s6_addr32[3] & 0xFFFF */
		uint32_t w3;
		memcpy(&w3, daddr16 + 12, 4);
		ct_state_new.rev_nat_index = w3 & 0xFFFF;
	}
	ret = ct_lookup6(&ct_map6, &tuple, &skb, 0, egress ? CT_EGRESS : CT_INGRESS, &ct_state,
			 &monitor);
	*ct_ret = ret;
	if (ret < 0) {
		*stage_out = ret == DROP_CT_UNKNOWN_PROTO ? 4 : 5;
		return ret;
	}

	if (egress) {
		info = ipcache_lookup6(&cilium_ipcache, &da, V6_CACHE_KEY_LEN);
		if (info && info->sec_label)
			id = info->sec_label;
		else if (ipv6_match_prefix_64(&da, &router_ip))
			id = CLUSTER_ID;
		else
			id = WORLD_ID;
		verdict = policy_can_egress6(&skb, &tuple, id, ipv6_ct_tuple_get_daddr(&tuple));
	} else {
		uint32_t src = cfg_src_identity;
		if (identity_is_reserved(src)) {
			info = ipcache_lookup6(&cilium_ipcache, &sa, V6_CACHE_KEY_LEN);
			if (info && info->sec_label && info->sec_label != CLUSTER_ID)
				src = info->sec_label;
		}
		id = src;
		verdict = policy_can_access_ingress(&skb, id, tuple.dport, tuple.nexthdr,
						    sizeof(tuple.saddr), &tuple.saddr, false);
	}
	*identity_out = id;
	*stage_out = pol_hit_probe;

	if (ret != CT_REPLY && ret != CT_RELATED && verdict < 0) {
		if (ret == CT_ESTABLISHED)
			ct_delete6(&ct_map6, &tuple, &skb);
		return egress ? verdict : DROP_POLICY;
	}
	if (ret == CT_NEW) {
		ct_state_new.orig_dport = tuple.dport;
		ct_state_new.src_sec_id = egress ? seclabel : id;
		ret = ct_create6(&ct_map6, &tuple, &skb, egress ? CT_EGRESS : CT_INGRESS,
				 &ct_state_new);
		if (IS_ERR(ret))
			return ret;
	}
	if (verdict > 0 && (egress || ret == CT_NEW || ret == CT_ESTABLISHED))
		return verdict;
	return 0;
}

/* Constants the restatement must agree with. */
int ref_ct_constants(uint32_t *out, int n)
{
	uint32_t c[] = { CT_LIFETIME_TCP, CT_LIFETIME_NONTCP, CT_SYN_TIMEOUT, CT_CLOSE_TIMEOUT,
			 CT_REPORT_INTERVAL, TUPLE_F_OUT, TUPLE_F_IN, TUPLE_F_RELATED,
			 (uint32_t)DROP_CT_CREATE_FAILED, CT_MAP_SIZE };
	int k = (int)(sizeof(c) / sizeof(c[0]));
	for (int i = 0; i < n && i < k; i++)
		out[i] = c[i];
	return k;
}
