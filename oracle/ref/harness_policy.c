/*
 * TEST INFRASTRUCTURE — the reference oracle.  Built ONLY in the development
 * container (it #includes /root/reference/bpf, which never travels to the
 * GPU box) into oracle/_ref/libref_policy.so by oracle/Makefile.  It is run
 * solely by oracle/gen_golden.py to emit tests/golden/* fixtures.
 *
 * It compiles the reference's own datapath C as host C, unmodified:
 *   - __policy_can_access / policy_can_access_ingress / policy_can_egress
 *     (bpf/lib/policy.h:46-177)
 *   - ipcache_lookup4 / ipcache_lookup6 (bpf/lib/eps.h:56-80)
 *   - identity_is_reserved (bpf/lib/policy.h:41-44)
 * with map_lookup_elem pointed at the mock map store (mockmap.c), because
 * the map implementations live in the Linux kernel, not in the reference.
 * The metrics the reference keeps (cilium_metrics, bpf/lib/maps.h:35-41)
 * come from its own call sites: send_drop_notify on a drop
 * (bpf/lib/drop.h:113-118 -> update_metrics, metrics.h:41-59) and
 * send_trace_notify at the forwarding observation point
 * (bpf/lib/trace.h:163-186: TRACE_TO_LXC ingress, TRACE_TO_STACK egress,
 * TRACE_TO_PROXY nothing), with map_update_elem pointed at the mock too.
 *
 * The per-tuple composition (which address feeds ipcache, the identity
 * fallback, the protocol gate) is glue restated from the reference's
 * callers, each line citing the caller it follows.
 */
#include <stdio.h>
#include <string.h>
#include <stdint.h>

#include "lib/utils.h"
#include "node_config.h"
#include "lxc_config.h"
/* Notification/debug paths emit perf events through helpers the harness
 * does not mock; they do not influence verdicts or map contents. */
#undef DROP_NOTIFY
#undef TRACE_NOTIFY
#undef DEBUG
#include "lib/common.h"
#include "lib/policy.h"
#include "lib/eps.h"
#include "lib/drop.h"
#include "lib/trace.h"

#include "mockmap.h"

#define REF_MAX_EP 64

static struct mockmap policy_maps[REF_MAX_EP];
static struct mockmap ipcache;
static struct mockmap metrics; /* cilium_metrics (one CPU: a plain hash) */
static void fresh_skb(struct __sk_buff *skb, uint32_t len);
static int cur_ep;
static int inited;
/* probe accounting: index (1-based) of the policy probe that hit, and count */
static int pol_probes, pol_hit_probe;

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
	if (map == &cilium_metrics)
		return mockmap_lookup(&metrics, key);
	fprintf(stderr, "ref harness: lookup on unexpected map %p\n", map);
	return NULL;
}

static int mock_update(void *map, const void *key, const void *val, __u32 flags)
{
	(void)flags;
	if (map == &cilium_metrics)
		return mockmap_update(&metrics, key, val) < 0 ? -1 : 0;
	fprintf(stderr, "ref harness: update on unexpected map %p\n", map);
	return -1;
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
	mockmap_init(&metrics, MOCK_HASH, sizeof(struct metrics_key), sizeof(struct metrics_value));
	map_lookup_elem = mock_lookup;
	map_update_elem = mock_update;
	inited = 1;
}

void ref_reset(void)
{
	ensure_init();
	for (int i = 0; i < REF_MAX_EP; i++)
		mockmap_clear(&policy_maps[i]);
	mockmap_clear(&ipcache);
	mockmap_clear(&metrics);
}

/* cilium_metrics as [reason 256][dir 4][count, bytes] (u64) */
void ref_metrics_read(uint64_t *out)
{
	ensure_init();
	memset(out, 0, 256 * 4 * 2 * sizeof(uint64_t));
	for (size_t i = 0; i < metrics.n; i++) {
		const struct metrics_key *k = (const void *)(metrics.keys + i * metrics.ksz);
		const struct metrics_value *v = (const void *)(metrics.vals + i * metrics.vsz);
		out[(k->reason * 4 + k->dir) * 2] += v->count;
		out[(k->reason * 4 + k->dir) * 2 + 1] += v->bytes;
	}
}

/* The metrics of one packet whose program ended with `ret` (bpf_lxc.c):
 * a drop is reported by the tail-call wrapper with send_drop_notify
 * (egress tail_handle_ipv4 :659-666 / tail_handle_ipv6, ingress
 * tail_ipv4_policy :980-988 / tail_ipv6_policy); a proxy redirect traces
 * TRACE_TO_PROXY in ipv4_redirect_to_host_port (lib/lxc.h:115-117); any
 * other egress packet leaves through TRACE_TO_STACK (:652) or local
 * delivery (lib/l3.h:128, an egress forward as well); an allowed ingress
 * packet traces TRACE_TO_LXC (:969). */
void ref_metrics_packet(int ret, uint32_t len, int egress)
{
	struct __sk_buff skb;
	ensure_init();
	fresh_skb(&skb, len);
	if (ret < 0)
		send_drop_notify(&skb, 0, 0, 0, 0, ret, TC_ACT_SHOT, egress ? METRIC_EGRESS : METRIC_INGRESS);
	else if (ret > 0)
		send_trace_notify(&skb, TRACE_TO_PROXY, 0, 0, 0, 0, 0, false);
	else
		send_trace_notify(&skb, egress ? TRACE_TO_STACK : TRACE_TO_LXC, 0, 0, 0, 0, 0, false);
}

int ref_sizes(int *policy_key_sz, int *policy_entry_sz, int *ipcache_key_sz,
	      int *remote_info_sz)
{
	*policy_key_sz = sizeof(struct policy_key);
	*policy_entry_sz = sizeof(struct policy_entry);
	*ipcache_key_sz = sizeof(struct ipcache_key);
	*remote_info_sz = sizeof(struct remote_endpoint_info);
	return 0;
}

/* Raw 8-byte policy_key / 24-byte policy_entry, as bpf(2) would copy them. */
int ref_policy_update(int ep, const void *key, const void *entry)
{
	ensure_init();
	if (ep < 0 || ep >= REF_MAX_EP)
		return -1;
	return mockmap_update(&policy_maps[ep], key, entry);
}

int ref_policy_read(int ep, const void *key, void *entry_out)
{
	void *v;
	ensure_init();
	v = mockmap_lookup(&policy_maps[ep], key);
	if (!v)
		return -1;
	memcpy(entry_out, v, sizeof(struct policy_entry));
	return 0;
}

/* Raw 24-byte ipcache_key / 8-byte remote_endpoint_info. */
int ref_ipcache_update(const void *key, const void *info)
{
	ensure_init();
	return mockmap_update(&ipcache, key, info);
}

/* ipcache_lookup4 (bpf/lib/eps.h:70-80) at V4_CACHE_KEY_LEN, the
 * HAVE_LPM_MAP_TYPE form used by the datapath (eps.h:111-114). */
int ref_ipcache_lookup4(uint32_t addr_be, uint32_t *sec_label, uint32_t *tunnel)
{
	struct remote_endpoint_info *info;
	ensure_init();
	info = ipcache_lookup4(&cilium_ipcache, addr_be, V4_CACHE_KEY_LEN);
	if (!info)
		return 0;
	*sec_label = info->sec_label;
	*tunnel = info->tunnel_endpoint;
	return 1;
}

/* ipcache_lookup6 (bpf/lib/eps.h:56-66) at V6_CACHE_KEY_LEN. */
int ref_ipcache_lookup6(const uint8_t *addr16, uint32_t *sec_label, uint32_t *tunnel)
{
	struct remote_endpoint_info *info;
	union v6addr a;
	ensure_init();
	memcpy(&a, addr16, 16);
	info = ipcache_lookup6(&cilium_ipcache, &a, V6_CACHE_KEY_LEN);
	if (!info)
		return 0;
	*sec_label = info->sec_label;
	*tunnel = info->tunnel_endpoint;
	return 1;
}

static void fresh_skb(struct __sk_buff *skb, uint32_t len)
{
	memset(skb, 0, sizeof(*skb));
	skb->len = len; /* cb[CB_POLICY] == 0: no CT reply/proxy skip mark */
}

/* policy_can_access_ingress (bpf/lib/policy.h:126-146). */
int ref_policy_ingress(int ep, uint32_t identity, uint16_t dport_be, uint8_t proto,
		       int is_fragment, uint32_t len, int *nprobes, int *hit_probe)
{
	struct __sk_buff skb;
	int ret;
	ensure_init();
	fresh_skb(&skb, len);
	cur_ep = ep;
	pol_probes = pol_hit_probe = 0;
	ret = policy_can_access_ingress(&skb, identity, dport_be, proto, 0, NULL,
					is_fragment ? true : false);
	*nprobes = pol_probes;
	*hit_probe = pol_hit_probe;
	return ret;
}

/* policy_can_egress (bpf/lib/policy.h:150-163). */
int ref_policy_egress(int ep, uint32_t identity, uint16_t dport_be, uint8_t proto,
		      uint32_t len, int *nprobes, int *hit_probe)
{
	struct __sk_buff skb;
	int ret;
	ensure_init();
	fresh_skb(&skb, len);
	cur_ep = ep;
	pol_probes = pol_hit_probe = 0;
	ret = policy_can_egress(&skb, identity, dport_be, proto);
	*nprobes = pol_probes;
	*hit_probe = pol_hit_probe;
	return ret;
}

/* Raw __policy_can_access (bpf/lib/policy.h:46-110), to pin the
 * un-collapsed DROP_FRAG_NOSUPPORT (-157) path. */
int ref_policy_raw(int ep, uint32_t identity, uint16_t dport_be, uint8_t proto,
		   int dir, int is_fragment, uint32_t len, int *nprobes, int *hit_probe)
{
	struct __sk_buff skb;
	int ret;
	ensure_init();
	fresh_skb(&skb, len);
	cur_ep = ep;
	pol_probes = pol_hit_probe = 0;
	ret = __policy_can_access(&POLICY_MAP, &skb, identity, dport_be, proto, 0,
				  NULL, dir, is_fragment ? true : false);
	*nprobes = pol_probes;
	*hit_probe = pol_hit_probe;
	return ret;
}

/*
 * One stateless IPv4 tuple through the reference's decision (CT_NEW, no
 * CB_POLICY mark).  Glue, each step restated from the caller it follows:
 *
 *  flags bit0 = egress (from-container), bit1 = is_fragment.
 *  cfg_gate: CONNTRACK's protocol gate — ct_lookup4 returns
 *    DROP_CT_UNKNOWN_PROTO for anything but ICMP/TCP/UDP before any policy
 *    (bpf/lib/conntrack.h:470-528; callers bpf_lxc.c:477-481, :895-897).
 *  Egress (bpf_lxc.c:484-505): dstID = ipcache(daddr) sec_label if nonzero,
 *    else CLUSTER_ID if (daddr & IPV4_CLUSTER_MASK) == IPV4_CLUSTER_RANGE,
 *    else WORLD_ID; verdict = policy_can_egress4(dstID, dport, proto).
 *  Ingress (bpf_netdev.c:374-398 then bpf_lxc.c:893-926): src starts at
 *    cfg_src_identity; if identity_is_reserved(src), ipcache(saddr) replaces
 *    it when sec_label is nonzero and not CLUSTER_ID/HOST_ID.  The policy
 *    label is secctx: src (FROM_HOST form, :403) or, with cfg_secctx_world,
 *    derive_ipv4_sec_ctx() == WORLD_ID (non-FROM_HOST form, :278-290,371).
 *    verdict = policy_can_access_ingress(label, dport, proto, is_fragment).
 *
 * Outputs: verdict, identity (label given to policy), stage (1 exact,
 * 2 L3-only, 3 identity-wildcard L4, 0 miss, 4 protocol-gated), probes.
 */
int ref_classify_v4(uint32_t saddr_be, uint32_t daddr_be, uint16_t dport_be,
		    uint8_t proto, uint8_t flags, uint32_t len, int ep,
		    int cfg_gate, uint32_t cfg_src_identity, int cfg_secctx_world,
		    uint32_t *identity_out, int *stage_out, int *nprobes_out,
		    int *naddr_out)
{
	int egress = flags & 1, frag = (flags >> 1) & 1;
	int ret, probes = 0, hit = 0;
	uint32_t label, tun;

	*naddr_out = 0;
	if (cfg_gate && proto != IPPROTO_ICMP && proto != IPPROTO_TCP &&
	    proto != IPPROTO_UDP) {
		*identity_out = 0;
		*stage_out = 4;
		*nprobes_out = 0;
		ref_metrics_packet(DROP_CT_UNKNOWN_PROTO, len, egress);
		return DROP_CT_UNKNOWN_PROTO;
	}
	if (egress) {
		uint32_t dst_id;
		*naddr_out = 1;
		if (ref_ipcache_lookup4(daddr_be, &label, &tun) && label)
			dst_id = label;
		else if ((daddr_be & IPV4_CLUSTER_MASK) == IPV4_CLUSTER_RANGE)
			dst_id = CLUSTER_ID;
		else
			dst_id = WORLD_ID;
		ret = ref_policy_egress(ep, dst_id, dport_be, proto, len, &probes, &hit);
		*identity_out = dst_id;
	} else {
		uint32_t src = cfg_src_identity, secctx;
		if (identity_is_reserved(src)) {
			*naddr_out = 1;
			if (ref_ipcache_lookup4(saddr_be, &label, &tun) && label &&
			    label != CLUSTER_ID && label != HOST_ID)
				src = label;
		}
		secctx = cfg_secctx_world ? WORLD_ID : src;
		ret = ref_policy_ingress(ep, secctx, dport_be, proto, frag, len,
					 &probes, &hit);
		*identity_out = secctx;
	}
	*nprobes_out = probes;
	*stage_out = hit ? (frag && !egress ? 2 : hit) : 0;
	ref_metrics_packet(ret, len, egress);
	return ret;
}

/* Constants the restatement must agree with (node_config.h, common.h). */
int ref_constants(uint32_t *out, int n)
{
	uint32_t c[] = { HOST_ID, WORLD_ID, CLUSTER_ID, HEALTH_ID, INIT_ID,
			 IPV4_CLUSTER_MASK, IPV4_CLUSTER_RANGE,
			 (uint32_t)DROP_POLICY, (uint32_t)DROP_FRAG_NOSUPPORT,
			 (uint32_t)DROP_CT_UNKNOWN_PROTO, CT_EGRESS, CT_INGRESS };
	int k = (int)(sizeof(c) / sizeof(c[0]));
	for (int i = 0; i < n && i < k; i++)
		out[i] = c[i];
	return k;
}

/*
 * One stateless IPv6 tuple.  Glue restated from the callers:
 *  gate: ct_lookup6 accepts ICMPv6/TCP/UDP only (bpf/lib/conntrack.h:330-378).
 *  Egress (bpf_lxc.c:170-191): dstID = ipcache6(daddr) sec_label if nonzero,
 *    else CLUSTER_ID if ipv6_match_prefix_64(daddr, ROUTER_IP), else WORLD_ID;
 *    verdict = policy_can_egress6(dstID, dport, nexthdr).
 *  Ingress (bpf_netdev.c:203-211, then bpf_lxc.c:787-789): if
 *    identity_is_reserved(src), ipcache6(saddr) replaces it when sec_label
 *    is nonzero and not CLUSTER_ID (no HOST_ID exception on v6); the label
 *    is the resolved src (FROM_HOST form, :222); IPv6 passes is_fragment =
 *    false.
 */
int ref_classify_v6(const uint8_t *saddr16, const uint8_t *daddr16, uint16_t dport_be,
		    uint8_t proto, uint8_t flags, uint32_t len, int ep, int cfg_gate,
		    uint32_t cfg_src_identity, uint32_t *identity_out, int *stage_out,
		    int *nprobes_out, int *naddr_out)
{
	int egress = flags & 1;
	int ret, probes = 0, hit = 0;
	uint32_t label, tun;
	union v6addr sa, da;
	union v6addr router_ip;
	BPF_V6(router_ip, ROUTER_IP);

	memcpy(&sa, saddr16, 16);
	memcpy(&da, daddr16, 16);
	*naddr_out = 0;
	if (cfg_gate && proto != IPPROTO_ICMPV6 && proto != IPPROTO_TCP &&
	    proto != IPPROTO_UDP) {
		*identity_out = 0;
		*stage_out = 4;
		*nprobes_out = 0;
		ref_metrics_packet(DROP_CT_UNKNOWN_PROTO, len, egress);
		return DROP_CT_UNKNOWN_PROTO;
	}
	if (egress) {
		uint32_t dst_id;
		*naddr_out = 1;
		if (ref_ipcache_lookup6(daddr16, &label, &tun) && label)
			dst_id = label;
		else if (ipv6_match_prefix_64(&da, &router_ip))
			dst_id = CLUSTER_ID;
		else
			dst_id = WORLD_ID;
		ret = ref_policy_egress(ep, dst_id, dport_be, proto, len, &probes, &hit);
		*identity_out = dst_id;
	} else {
		uint32_t src = cfg_src_identity;
		if (identity_is_reserved(src)) {
			*naddr_out = 1;
			if (ref_ipcache_lookup6(saddr16, &label, &tun) && label &&
			    label != CLUSTER_ID)
				src = label;
		}
		ret = ref_policy_ingress(ep, src, dport_be, proto, 0, len, &probes, &hit);
		*identity_out = src;
	}
	*nprobes_out = probes;
	*stage_out = hit;
	ref_metrics_packet(ret, len, egress);
	return ret;
}

void ref_router_ip(uint8_t *out16)
{
	union v6addr router_ip;
	BPF_V6(router_ip, ROUTER_IP);
	memcpy(out16, &router_ip, 16);
}
