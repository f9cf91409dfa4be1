/*
 * TEST INFRASTRUCTURE — the reference oracle for raw-frame -> policy-tuple
 * extraction.  Built ONLY in the development container
 * into oracle/_ref/libref_frame{,_noct,_nover}.so (oracle/Makefile); run only
 * by oracle/gen_golden.py.
 *
 * Compiles the reference's bpf/lib/{ipv4,ipv6,lxc,lb,conntrack}.h as host C
 * under node_config.h + lxc_config.h (LB_L3, LB_L4, CONNTRACK, LXC_MAC,
 * LXC_IP, LXC_IPV4) and runs, per Ethernet frame, the steps of the endpoint
 * programs that come BEFORE the ipcache / policy decision:
 *   egress  (from-container): handle_ingress dispatch (bpf_lxc.c:683-711),
 *           handle_ipv4_from_lxc (bpf_lxc.c:426-481) / handle_ipv6's
 *           ICMPv6 responders (bpf_lxc.c:364-389, lib/icmp6.h) and
 *           ipv6_l3_from_lxc (bpf_lxc.c:82-163): revalidate_data, SMAC / DMAC / SIP checks,
 *           ipv{4,6}_hdrlen, lb{4,6}_extract_key + lb{4,6}_lookup_service
 *           over an EMPTY service map, ct_lookup{4,6}(CT_EGRESS)
 *   ingress (to-container): bpf_netdev.c handle_netdev dispatch (:494-521,
 *           non-IP -> TC_ACT_OK to the stack), ipv4_policy (bpf_lxc.c:
 *           876-897) / ipv6_policy (bpf_lxc.c:731-773): revalidate_data,
 *           ipv{4,6}_hdrlen, ipv4_is_fragment, ct_lookup{4,6}(CT_INGRESS)
 * with an EMPTY conntrack map (every packet CT_NEW: the stateless scope of
 * SURVEY §8a row a8).  Its outputs are the tuple the policy step then sees:
 * (saddr, daddr, tuple.dport, tuple.nexthdr, is_fragment).
 *
 * Variants: -DHARNESS_NO_CONNTRACK (conntrack.h's stubs: ports never loaded,
 * no protocol gate); -DDISABLE_SMAC_VERIFICATION -DDISABLE_DMAC_VERIFICATION
 * -DDISABLE_SIP_VERIFICATION (lib/lxc.h:31-89).
 *
 * Mocks (writable helper pointers, bpf/include/bpf/api.h:101-112): every map
 * lookup misses; skb_load_bytes reads the frame buffer bounded by skb->len
 * (-EFAULT past it, as the kernel helper); debug helpers are inert.
 */
#include <setjmp.h>
#include <stdio.h>
#include <string.h>
#include <sys/mman.h>

#include "lib/utils.h"
#include "node_config.h"
#include "lxc_config.h"
#undef DROP_NOTIFY
#undef TRACE_NOTIFY
#undef DEBUG
#ifdef HARNESS_NO_CONNTRACK
#undef CONNTRACK
#undef ENABLE_NAT46
#endif
#include "lib/common.h"
#include "lib/maps.h"
#include "lib/ipv4.h"
#include "lib/ipv6.h"
#include "lib/l4.h"
#include "lib/lb.h"
#include "lib/lxc.h"
#include "lib/icmp6.h"

/* stand in for the endpoint's CT_MAP4 / CT_MAP6 (bpf_lxc.c:53-75) */
static int ct_map4, ct_map6;

static int inited;
static unsigned char *frame_buf;
static uint32_t frame_len;

/* BPF_LD_ABS (api.h:228-235: load_byte / load_half / load_word are these
 * LLVM BPF intrinsics), used by icmp6_load_type */
unsigned long long harness_fr_ld_abs_b(void *skb, unsigned long long off) __asm__("llvm.bpf.load.byte");
unsigned long long harness_fr_ld_abs_b(void *skb, unsigned long long off) { return frame_buf[off]; }
unsigned long long harness_fr_ld_abs_h(void *skb, unsigned long long off) __asm__("llvm.bpf.load.half");
unsigned long long harness_fr_ld_abs_h(void *skb, unsigned long long off)
{
	return (unsigned long long)frame_buf[off] << 8 | frame_buf[off + 1];
}
unsigned long long harness_fr_ld_abs_w(void *skb, unsigned long long off) __asm__("llvm.bpf.load.word");
unsigned long long harness_fr_ld_abs_w(void *skb, unsigned long long off)
{
	return (unsigned long long)frame_buf[off] << 24 | (unsigned long long)frame_buf[off + 1] << 16 |
	       (unsigned long long)frame_buf[off + 2] << 8 | frame_buf[off + 3];
}

/* the ICMPv6 responders of handle_ipv6 (bpf_lxc.c:377-386) are tail calls
 * that end the program: the mocked tail call runs the responder's body and
 * returns its outcome to frame_v6 */
static jmp_buf icmp6_env;
static int icmp6_ret;

static void *mock_lookup(void *map, const void *key) { return NULL; }
static int mock_update(void *map, const void *key, const void *val, uint32_t flags) { return 0; }
static int mock_delete(void *map, const void *key) { return 0; }
static uint64_t mock_ktime(void) { return 0; }

static int mock_load(struct __sk_buff *skb, uint32_t off, void *to, uint32_t len)
{
	if ((uint64_t)off + len > frame_len)
		return -14; /* -EFAULT, bpf_skb_load_bytes */
	memcpy(to, frame_buf + off, len);
	return 0;
}

static int mock_store(struct __sk_buff *skb, uint32_t off, const void *from, uint32_t len, uint32_t flags)
{
	if ((uint64_t)off + len > frame_len)
		return -14;
	memcpy(frame_buf + off, from, len);
	return 0;
}

static int mock_csum_diff(void *from, uint32_t fs, void *to, uint32_t ts, uint32_t seed) { return 0; }
static int mock_csum_replace(struct __sk_buff *skb, uint32_t off, uint32_t from, uint32_t to, uint32_t flags)
{
	return 0;
}
static int mock_redirect(int ifindex, uint32_t flags) { return TC_ACT_REDIRECT; }

/* a responder's outcome: its drop, or 1 (the frame left the classification
 * path, as an ARP request does) */
static void mock_tail_call(struct __sk_buff *skb, void *map, uint32_t index)
{
	int r;
	if (index == CILIUM_CALL_HANDLE_ICMP6_NS)
		r = __icmp6_handle_ns(skb, skb->cb[0]);
	else if (index == CILIUM_CALL_SEND_ICMP6_ECHO_REPLY)
		r = __icmp6_send_echo_reply(skb, skb->cb[0]);
	else
		return;
	icmp6_ret = IS_ERR(r) ? r : 1;
	longjmp(icmp6_env, 1);
}

static int ensure_init(void)
{
	if (inited)
		return 0;
	frame_buf = mmap(NULL, 1 << 16, PROT_READ | PROT_WRITE,
			 MAP_PRIVATE | MAP_ANONYMOUS | MAP_32BIT, -1, 0);
	if (frame_buf == MAP_FAILED)
		return -1;
	map_lookup_elem = mock_lookup;
	map_update_elem = mock_update;
	map_delete_elem = mock_delete;
	ktime_get_ns = mock_ktime;
	skb_load_bytes = mock_load;
	skb_store_bytes = mock_store;
	csum_diff = mock_csum_diff;
	l3_csum_replace = mock_csum_replace;
	l4_csum_replace = mock_csum_replace;
	redirect = mock_redirect;
	tail_call = mock_tail_call;
	inited = 1;
	return 0;
}

struct frame_out {
	uint8_t saddr[16], daddr[16];
	uint16_t dport;
	uint8_t proto;
	uint8_t is_fragment;
};

/* handle_ipv4_from_lxc up to ct_lookup4 (bpf_lxc.c:426-481), or
 * ipv4_policy up to ct_lookup4 (bpf_lxc.c:876-897) */
static int frame_v4(struct __sk_buff *skb, int egress, struct frame_out *o)
{
	struct ipv4_ct_tuple tuple = {};
	struct ct_state ct_state = {};
	void *data, *data_end;
	struct iphdr *ip4;
	bool monitor = false;
	int ret, l4_off;

	if (!revalidate_data(skb, &data, &data_end, &ip4))
		return DROP_INVALID;
	tuple.nexthdr = ip4->protocol;
	if (egress) {
		struct ethhdr *eth = data;
		if (unlikely(!is_valid_lxc_src_mac(eth)))
			return DROP_INVALID_SMAC;
		else if (unlikely(!is_valid_gw_dst_mac(eth)))
			return DROP_INVALID_DMAC;
		else if (unlikely(!is_valid_lxc_src_ipv4(ip4)))
			return DROP_INVALID_SIP;
	}
	tuple.daddr = ip4->daddr;
	tuple.saddr = ip4->saddr;
	memcpy(o->saddr, &ip4->saddr, 4);
	memcpy(o->daddr, &ip4->daddr, 4);
	l4_off = ETH_HLEN + ipv4_hdrlen(ip4);
	if (egress) {
		struct csum_offset csum_off = {};
		struct lb4_key key = {};
		ret = lb4_extract_key(skb, &tuple, l4_off, &key, &csum_off, CT_EGRESS);
		if (IS_ERR(ret)) {
			if (ret != DROP_UNKNOWN_L4)
				return ret;
		} else {
			(void)lb4_lookup_service(skb, &key); /* empty service map */
		}
		o->is_fragment = 0; /* policy_can_egress4 passes false */
	} else {
		o->is_fragment = ipv4_is_fragment(ip4) ? 1 : 0;
	}
	ret = ct_lookup4(&ct_map4, &tuple, skb, l4_off, egress ? CT_EGRESS : CT_INGRESS,
			 &ct_state, &monitor);
	if (ret < 0)
		return ret;
	o->dport = tuple.dport;
	o->proto = tuple.nexthdr;
	return 0;
}

/* ipv6_l3_from_lxc up to ct_lookup6 (bpf_lxc.c:82-163), or ipv6_policy up
 * to ct_lookup6 (bpf_lxc.c:731-773; its rev-NAT daddr rewrite does not
 * reach the policy tuple) */
static int frame_v6(struct __sk_buff *skb, int egress, struct frame_out *o)
{
	struct ipv6_ct_tuple tuple = {};
	struct ct_state ct_state = {};
	void *data, *data_end;
	struct ipv6hdr *ip6;
	bool monitor = false;
	int ret, l4_off, hdrlen;

	if (!revalidate_data(skb, &data, &data_end, &ip6))
		return DROP_INVALID;
	if (egress && ip6->nexthdr == IPPROTO_ICMPV6) {
		/* handle_ipv6 (bpf_lxc.c:364-389): special ICMPv6 messages before
		 * ipv6_l3_from_lxc -- neighbour solicitations and echo requests
		 * to the router go to the responders (icmp6_handle,
		 * lib/icmp6.h:390-412) */
		if (data + sizeof(*ip6) + ETH_HLEN + sizeof(struct icmp6hdr) > data_end)
			return DROP_INVALID;
		if (setjmp(icmp6_env))
			return icmp6_ret;
		ret = icmp6_handle(skb, ETH_HLEN, ip6, METRIC_EGRESS);
		if (IS_ERR(ret))
			return ret;
	}
	tuple.nexthdr = ip6->nexthdr;
	if (egress) {
		struct ethhdr *eth = data;
		if (unlikely(!is_valid_lxc_src_mac(eth)))
			return DROP_INVALID_SMAC;
		else if (unlikely(!is_valid_gw_dst_mac(eth)))
			return DROP_INVALID_DMAC;
		else if (unlikely(!is_valid_lxc_src_ip(ip6)))
			return DROP_INVALID_SIP;
	}
	ipv6_addr_copy(&tuple.daddr, (union v6addr *)&ip6->daddr);
	ipv6_addr_copy(&tuple.saddr, (union v6addr *)&ip6->saddr);
	memcpy(o->saddr, &ip6->saddr, 16);
	memcpy(o->daddr, &ip6->daddr, 16);
	hdrlen = ipv6_hdrlen(skb, ETH_HLEN, &tuple.nexthdr);
	if (hdrlen < 0)
		return hdrlen;
	l4_off = ETH_HLEN + hdrlen;
	if (egress) {
		struct csum_offset csum_off = {};
		struct lb6_key key = {};
		ret = lb6_extract_key(skb, &tuple, l4_off, &key, &csum_off, CT_EGRESS);
		if (IS_ERR(ret)) {
			if (ret != DROP_UNKNOWN_L4)
				return ret;
		} else {
			(void)lb6_lookup_service(skb, &key); /* empty service map */
		}
	}
	o->is_fragment = 0; /* IPv6 passes is_fragment = false (bpf_lxc.c:787-789) */
	ret = ct_lookup6(&ct_map6, &tuple, skb, l4_off, egress ? CT_EGRESS : CT_INGRESS,
			 &ct_state, &monitor);
	if (ret < 0)
		return ret;
	o->dport = tuple.dport;
	o->proto = tuple.nexthdr;
	return 0;
}

/*
 * One frame.  Returns 0 when the frame reaches the ipcache / policy step
 * (then *family is 4 or 6 and the tuple fields are set), 1 when it is not
 * classified (egress ARP: tail call to the ARP responder, bpf_lxc.c:703-706;
 * ingress non-IP: TC_ACT_OK to the stack, bpf_netdev.c:518-520), or the
 * negative DROP_* / -errno the program returns.
 */
int ref_frame_parse(const uint8_t *frame, uint32_t len, int egress, int *family,
		    uint8_t *saddr16, uint8_t *daddr16, uint16_t *dport, uint8_t *proto,
		    uint8_t *is_fragment)
{
	struct __sk_buff skb;
	struct frame_out o;
	uint16_t eth_proto;
	int ret;

	if (ensure_init() || len > (1 << 16) || len < ETH_HLEN)
		return -1;
	memcpy(frame_buf, frame, len);
	frame_len = len;
	memset(&skb, 0, sizeof(skb));
	memset(&o, 0, sizeof(o));
	skb.data = (uint32_t)(unsigned long)frame_buf;
	skb.data_end = (uint32_t)(unsigned long)(frame_buf + len);
	skb.len = len;
	memcpy(&eth_proto, frame_buf + 12, 2);
	skb.protocol = eth_proto; /* skb->protocol: the frame's ethertype */
	*family = 0;
	switch (skb.protocol) {
	case bpf_htons(ETH_P_IP):
		ret = frame_v4(&skb, egress, &o);
		*family = 4;
		break;
	case bpf_htons(ETH_P_IPV6):
		ret = frame_v6(&skb, egress, &o);
		*family = 6;
		break;
	case bpf_htons(ETH_P_ARP):
		return 1;
	default:
		return egress ? DROP_UNKNOWN_L3 : 1;
	}
	memcpy(saddr16, o.saddr, 16);
	memcpy(daddr16, o.daddr, 16);
	*dport = o.dport;
	*proto = o.proto;
	*is_fragment = o.is_fragment;
	return ret;
}

/* The endpoint / node identity the variant was compiled with:
 * out = LXC_MAC[6] NODE_MAC[6] LXC_IPV4[4] LXC_IP[16] verify-bits[1] */
void ref_frame_config(uint8_t *out)
{
	union macaddr lmac = LXC_MAC, nmac = NODE_MAC;
	union v6addr lip = {};
	uint32_t l4 = LXC_IPV4;
	uint8_t verify = 0;
	BPF_V6(lip, LXC_IP);
	memcpy(out, lmac.addr, 6);
	memcpy(out + 6, nmac.addr, 6);
	memcpy(out + 12, &l4, 4);
	memcpy(out + 16, lip.addr, 16);
#ifndef DISABLE_SMAC_VERIFICATION
	verify |= 1;
#endif
#ifndef DISABLE_DMAC_VERIFICATION
	verify |= 2;
#endif
#ifndef DISABLE_SIP_VERIFICATION
	verify |= 4;
#endif
	out[32] = verify;
}
