/*
 * TEST INFRASTRUCTURE — the reference's host-device program compiled whole,
 * so that the ingress source identity the endpoint's policy program receives
 * comes from the reference's own code rather than the restatement in
 * harness_lxc.c (ref_lxc_src_identity).  Built
 * ONLY in the development container into oracle/_ref/libref_netdev.so
 * (oracle/Makefile); run only by tests/test_composition.py.
 *
 * #includes bpf/bpf_netdev.c under the reference's own node_config.h and
 * netdev_config.h (the cilium_host build: FROM_HOST, ENCAP_IFINDEX,
 * HANDLE_NS), -DSKIP_DEBUG.  Per packet it runs the program's IPv4 entry
 * tail_handle_ipv4 (bpf_netdev.c:457-466: handle_ipv4, :357-452) with
 * skb->cb[CB_SRC_IDENTITY] = the identity from_netdev would hand over, or
 * handle_ipv6 (:173-236 and its local delivery) directly, as from_netdev
 * does.  The destination is a local endpoint (cilium_lxc answers every
 * lookup with one non-host endpoint), so the program ends in
 * ipv{4,6}_local_delivery's tail call into the endpoint's policy program
 * (lib/l3.h:103-131); the mocked tail_call reads skb->cb[CB_SRC_LABEL] there
 * -- the source identity the endpoint's ipv4_policy / ipv6_policy receive --
 * and returns to the harness (longjmp: a BPF tail call does not return).
 *
 * Mocks (writable helper pointers, bpf/include/bpf/api.h): the ipcache is
 * mockmap.c's longest-prefix map; cilium_lxc returns the endpoint; the proxy,
 * tunnel and metrics maps are empty / accept updates; skb_load_bytes /
 * skb_store_bytes act on a MAP_32BIT frame buffer; checksum helpers return 0.
 */
#include <setjmp.h>
#include <stdio.h>
#include <string.h>
#include <stdint.h>
#include <sys/mman.h>

#include "bpf_netdev.c"

#include "mockmap.h"

static struct mockmap ipcache;
static int inited;
static unsigned char *frame_buf;
static uint32_t frame_len;
static jmp_buf tail_env;
static uint32_t tail_label;
static struct endpoint_info local_ep = {.ifindex = 11, .lxc_id = 7};

unsigned long long harness_nd_ld_abs_b(void *skb, unsigned long long off) __asm__("llvm.bpf.load.byte");
unsigned long long harness_nd_ld_abs_b(void *skb, unsigned long long off) { return frame_buf[off]; }
unsigned long long harness_nd_ld_abs_h(void *skb, unsigned long long off) __asm__("llvm.bpf.load.half");
unsigned long long harness_nd_ld_abs_h(void *skb, unsigned long long off)
{
	return (unsigned long long)frame_buf[off] << 8 | frame_buf[off + 1];
}
unsigned long long harness_nd_ld_abs_w(void *skb, unsigned long long off) __asm__("llvm.bpf.load.word");
unsigned long long harness_nd_ld_abs_w(void *skb, unsigned long long off)
{
	return (unsigned long long)frame_buf[off] << 24 | (unsigned long long)frame_buf[off + 1] << 16 |
	       (unsigned long long)frame_buf[off + 2] << 8 | frame_buf[off + 3];
}

static void *mock_lookup(void *map, const void *key)
{
	if (map == &cilium_ipcache)
		return mockmap_lookup(&ipcache, key);
	if (map == &cilium_lxc)
		return &local_ep;
	return NULL; /* proxy maps, tunnel map, metrics */
}

static int mock_update(void *map, const void *key, const void *val, uint32_t flags) { return 0; }
static int mock_delete(void *map, const void *key) { return -2; }
static uint64_t mock_ktime(void) { return 0; }

static int mock_load(struct __sk_buff *skb, uint32_t off, void *to, uint32_t len)
{
	if ((uint64_t)off + len > frame_len)
		return -14;
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
static int mock_tunnel_key(struct __sk_buff *skb, const struct bpf_tunnel_key *from, uint32_t size,
			   uint32_t flags)
{
	return 0;
}

static void mock_tail_call(struct __sk_buff *skb, void *map, uint32_t index)
{
	if (map == &cilium_policy) {
		tail_label = skb->cb[CB_SRC_LABEL];
		longjmp(tail_env, 1);
	}
}

static int mock_event_output(struct __sk_buff *skb, void *map, uint64_t index, const void *data, uint32_t size)
{
	return 0;
}

static uint32_t mock_cpu(void) { return 0; }

static int ensure_init(void)
{
	if (inited)
		return 0;
	mockmap_init(&ipcache, MOCK_LPM, sizeof(struct ipcache_key), sizeof(struct remote_endpoint_info));
	frame_buf = mmap(NULL, 1 << 12, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_32BIT, -1, 0);
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
	skb_event_output = mock_event_output;
	skb_set_tunnel_key = mock_tunnel_key;
	get_smp_processor_id = mock_cpu;
	inited = 1;
	return 0;
}

void ref_netdev_reset(void)
{
	ensure_init();
	mockmap_clear(&ipcache);
}

int ref_netdev_ipcache_update(const void *key, const void *info)
{
	ensure_init();
	return mockmap_update(&ipcache, key, info);
}

/* The program on one frame; *label = the source identity handed to the
 * endpoint's policy program, or the program's return code when it ended
 * before the tail call (returns 1 then, 0 on the tail call). */
static int run(int v6, uint32_t src_identity, uint32_t *label)
{
	struct __sk_buff skb;
	volatile int ret = 0;
	memset(&skb, 0, sizeof(skb));
	skb.data = (uint32_t)(unsigned long)frame_buf;
	skb.data_end = (uint32_t)(unsigned long)(frame_buf + frame_len);
	skb.len = frame_len;
	skb.protocol = v6 ? bpf_htons(ETH_P_IPV6) : bpf_htons(ETH_P_IP);
	if (setjmp(tail_env)) {
		*label = tail_label;
		return 0;
	}
	if (v6) {
		ret = handle_ipv6(&skb, src_identity);
	} else {
		skb.cb[CB_SRC_IDENTITY] = src_identity;
		ret = tail_handle_ipv4(&skb);
	}
	*label = (uint32_t)ret;
	return 1;
}

/* Ethernet + IPv4 (ihl 5, ttl 64) + 20 zero bytes of L4 */
int ref_netdev_v4(uint32_t saddr_be, uint32_t daddr_be, uint8_t proto, uint32_t src_identity, uint32_t *label)
{
	if (ensure_init())
		return -1;
	memset(frame_buf, 0, 128);
	frame_buf[12] = 0x08;
	struct iphdr *ip4 = (struct iphdr *)(frame_buf + ETH_HLEN);
	ip4->ihl = 5;
	ip4->version = 4;
	ip4->ttl = 64;
	ip4->tot_len = bpf_htons(40);
	ip4->protocol = proto;
	ip4->saddr = saddr_be;
	ip4->daddr = daddr_be;
	frame_len = ETH_HLEN + 40;
	return run(0, src_identity, label);
}

/* Ethernet + IPv6 (no extension header, hop limit 64) + 20 zero bytes */
int ref_netdev_v6(const uint8_t *saddr16, const uint8_t *daddr16, uint8_t proto, uint32_t src_identity,
		  uint32_t *label)
{
	if (ensure_init())
		return -1;
	memset(frame_buf, 0, 128);
	frame_buf[12] = 0x86;
	frame_buf[13] = 0xDD;
	struct ipv6hdr *ip6 = (struct ipv6hdr *)(frame_buf + ETH_HLEN);
	ip6->version = 6;
	ip6->nexthdr = proto;
	ip6->payload_len = bpf_htons(20);
	ip6->hop_limit = 64;
	memcpy(&ip6->saddr, saddr16, 16);
	memcpy(&ip6->daddr, daddr16, 16);
	frame_len = ETH_HLEN + 60;
	return run(1, src_identity, label);
}
