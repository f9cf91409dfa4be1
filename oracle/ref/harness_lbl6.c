/*
 * TEST INFRASTRUCTURE — the reference oracle for the IPv6 service step of the
 * endpoint egress path (widened to IPv6).  Built ONLY in the
 * development container into oracle/_ref/libref_lbl6{,_noct}.so
 * (oracle/Makefile); run only by oracle/gen_golden.py.
 *
 * Compiles the reference's bpf/lib/lb.h + bpf/lib/conntrack.h + bpf/lib/ipv6.h
 * as host C under node_config.h + lxc_config.h (LB_L3, LB_L4, CONNTRACK) with
 * -DSKIP_DEBUG, and runs the service step of ipv6_l3_from_lxc
 * (bpf_lxc.c:108-139): ipv6_hdrlen -> lb6_extract_key -> lb6_lookup_service
 * -> lb6_local (lb.h:334-483), whose ct_lookup6 / ct_create6
 * (conntrack.h:288-403, :588-650) see an EMPTY conntrack map: every packet is
 * CT_NEW, the stateless scope of SURVEY §8a row a8.
 *
 * Mocks as harness_lbl.c: the lb6 service map is a mock hash map, the CT map
 * misses every lookup and accepts every create, get_hash_recalc returns the
 * injected hash, packet bytes live in a MAP_32BIT frame buffer, checksum
 * helpers return 0.
 */
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
#include "lib/ipv6.h"
#include "lib/l4.h"
#include "lib/lb.h"

#include "mockmap.h"

/* stands for the endpoint's CT_MAP6 (bpf_lxc.c:53-75): only its address is used */
static int ct_map6;

static struct mockmap svc_m;
static int inited;
static unsigned char *frame_buf;
static uint32_t frame_len, inj_hash;
static uint64_t lookups;

static void *mock_lookup(void *map, const void *key)
{
	if (map == &cilium_lb6_services) {
		lookups++;
		return mockmap_lookup(&svc_m, key);
	}
	if (map == &ct_map6)
		return NULL;
	fprintf(stderr, "ref lbl6 harness: lookup on unexpected map %p\n", map);
	return NULL;
}

static int mock_update(void *map, const void *key, const void *val, uint32_t flags)
{
	return map == &ct_map6 ? 0 : -1;
}

static int mock_delete(void *map, const void *key) { return 0; }
static uint64_t mock_ktime(void) { return 0; }

static int mock_load(struct __sk_buff *skb, uint32_t off, void *to, uint32_t len)
{
	if (off + len > frame_len)
		return -14;
	memcpy(to, frame_buf + off, len);
	return 0;
}

static int mock_store(struct __sk_buff *skb, uint32_t off, const void *from, uint32_t len,
		      uint32_t flags)
{
	if (off + len > frame_len)
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
	mockmap_init(&svc_m, MOCK_HASH, sizeof(struct lb6_key), sizeof(struct lb6_service));
	frame_buf = mmap(NULL, 1 << 16, PROT_READ | PROT_WRITE,
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

void ref_lbl6_reset(void)
{
	ensure_init();
	mockmap_clear(&svc_m);
}

int ref_lbl6_update(const void *key, const void *val)
{
	if (ensure_init())
		return -1;
	return mockmap_update(&svc_m, key, val);
}

/*
 * The service step of ipv6_l3_from_lxc over one Ethernet + IPv6 frame (glue
 * restated from bpf_lxc.c:108-139 and handle_ipv6's tuple.nexthdr =
 * ip6->nexthdr).  Returns a negative DROP_* the step produced, else 0.
 * *svc_hit: lb6_lookup_service found a service; tuple_daddr (16 B):
 * tuple->daddr afterwards (orig_dip, the address the ipcache lookup of
 * bpf_lxc.c:175-185 resolves); rev_nat / slave: the ct_state lb6_local
 * filled; *l4_off: the L4 offset ipv6_hdrlen found.  The frame is rewritten
 * in place (the dport the egress ct_lookup6 reloads for policy).
 */
int ref_lbl6_run(uint8_t *frame, uint32_t len, uint32_t hash, int *svc_hit, uint8_t *tuple_daddr,
		 uint16_t *rev_nat, uint16_t *slave, int *l4_off_out, uint64_t *nlookups)
{
	struct __sk_buff skb;
	struct ipv6_ct_tuple tuple = {};
	struct csum_offset csum_off = {};
	struct lb6_key key = {};
	struct ct_state ct_state_new = {};
	struct lb6_service *svc;
	void *data, *data_end;
	struct ipv6hdr *ip6;
	int ret = 0, l3_off = ETH_HLEN, l4_off = 0, hdrlen;

	if (ensure_init() || len > (1 << 16))
		return -1;
	memcpy(frame_buf, frame, len);
	frame_len = len;
	inj_hash = hash;
	memset(&skb, 0, sizeof(skb));
	skb.data = (uint32_t)(unsigned long)frame_buf;
	skb.data_end = (uint32_t)(unsigned long)(frame_buf + len);
	skb.len = len;
	skb.protocol = bpf_htons(ETH_P_IPV6);
	lookups = 0;
	*svc_hit = 0;
	memset(tuple_daddr, 0, 16);
	if (!revalidate_data(&skb, &data, &data_end, &ip6)) {
		ret = DROP_INVALID;
		goto out;
	}
	tuple.nexthdr = ip6->nexthdr;
	ipv6_addr_copy(&tuple.daddr, (union v6addr *)&ip6->daddr);
	ipv6_addr_copy(&tuple.saddr, (union v6addr *)&ip6->saddr);
	hdrlen = ipv6_hdrlen(&skb, l3_off, &tuple.nexthdr);
	if (hdrlen < 0) {
		ret = hdrlen;
		goto out;
	}
	l4_off = l3_off + hdrlen;
	ret = lb6_extract_key(&skb, &tuple, l4_off, &key, &csum_off, CT_EGRESS);
	if (IS_ERR(ret)) {
		if (ret == DROP_UNKNOWN_L4)
			ret = 0; /* skip_service_lookup */
		goto out;
	}
	ct_state_new.orig_dport = key.dport;
	if ((svc = lb6_lookup_service(&skb, &key)) != NULL) {
		*svc_hit = 1;
		ret = lb6_local(&ct_map6, &skb, l3_off, l4_off, &csum_off, &key, &tuple, svc,
				&ct_state_new);
		if (!IS_ERR(ret))
			ret = 0;
	}
out:
	memcpy(tuple_daddr, &tuple.daddr, 16);
	*rev_nat = ct_state_new.rev_nat_index;
	*slave = ct_state_new.slave;
	*l4_off_out = l4_off;
	memcpy(frame, frame_buf, len);
	*nlookups = lookups;
	return ret;
}
