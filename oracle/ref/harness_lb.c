/*
 * TEST INFRASTRUCTURE — the reference oracle for the standalone service load
 * balancer.  Built ONLY in the development container into
 * oracle/_ref/libref_lb.so by oracle/Makefile; run only by
 * oracle/gen_golden.py.
 *
 * Compiles the reference's bpf/bpf_lb.c as host C (-DSKIP_DEBUG, so the
 * perf-event debug paths compile out; LB_L3 / LB_L4 as bpf/Makefile:42-44 and
 * bpf/init.sh:352 build it) and runs its handle_ipv4 (bpf_lb.c:118-170):
 * extract_l4_port -> lb4_lookup_service -> lb4_select_slave ->
 * lb4_lookup_slave -> lb4_xlate (bpf/lib/lb.h:158-697).
 *
 * Kernel helpers are mocked through the writable helper pointers of
 * bpf/include/bpf/api.h:101-112:
 *   map_lookup_elem         mock hash map (mockmap.c, whole-key memcmp)
 *   get_hash_recalc         returns the hash the caller injects: skb->hash is
 *                           kernel-internal, so LB parity is pinned with the
 *                           hash as an input
 *   skb_load/store_bytes    read / write the frame buffer
 *   csum_diff, l3/l4_csum_replace   return 0 (checksums are not part of the
 *                           compared outputs)
 * The frame lives in a MAP_32BIT buffer because __sk_buff.data/data_end are
 * __u32 in the reference's uapi header.
 */
#include <stdio.h>
#include <string.h>
#include <sys/mman.h>

#include "bpf_lb.c"

#include "mockmap.h"

static struct mockmap svc_m;
static int inited;
static unsigned char *frame_buf;
static uint32_t frame_len, inj_hash;
static uint64_t lookups;

static void *mock_lookup(void *map, const void *key)
{
	if (map == &cilium_lb4_services) {
		lookups++;
		return mockmap_lookup(&svc_m, key);
	}
	fprintf(stderr, "ref lb harness: lookup on unexpected map %p\n", map);
	return NULL;
}

static int mock_load(struct __sk_buff *skb, uint32_t off, void *to, uint32_t len)
{
	if (off + len > frame_len)
		return -14; /* -EFAULT: the kernel helper fails past the data */
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
	mockmap_init(&svc_m, MOCK_HASH, sizeof(struct lb4_key), sizeof(struct lb4_service));
	frame_buf = mmap(NULL, 1 << 16, PROT_READ | PROT_WRITE,
			 MAP_PRIVATE | MAP_ANONYMOUS | MAP_32BIT, -1, 0);
	if (frame_buf == MAP_FAILED)
		return -1;
	map_lookup_elem = mock_lookup;
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

void ref_lb_reset(void)
{
	ensure_init();
	mockmap_clear(&svc_m);
}

/* raw struct lb4_key (8 B) / struct lb4_service (12 B), bpf/lib/common.h:427-439 */
int ref_lb_update(const void *key, const void *val)
{
	if (ensure_init())
		return -1;
	return mockmap_update(&svc_m, key, val);
}

int ref_lb_sizes(int *key_sz, int *val_sz)
{
	*key_sz = sizeof(struct lb4_key);
	*val_sz = sizeof(struct lb4_service);
	return DROP_NO_SERVICE;
}

/* handle_ipv4 of bpf_lb.c over one Ethernet + IPv4 frame; the frame is
 * rewritten in place (daddr / dport), as the program rewrites the skb. */
int ref_lb_netdev(uint8_t *frame, uint32_t len, uint32_t hash, uint64_t *nlookups)
{
	struct __sk_buff skb;
	int ret;
	if (ensure_init() || len > (1 << 16))
		return -1;
	memcpy(frame_buf, frame, len);
	frame_len = len;
	inj_hash = hash;
	memset(&skb, 0, sizeof(skb));
	skb.data = (uint32_t)(unsigned long)frame_buf;
	skb.data_end = (uint32_t)(unsigned long)(frame_buf + len);
	skb.len = len;
	skb.protocol = bpf_htons(ETH_P_IP);
	lookups = 0;
	ret = handle_ipv4(&skb);
	memcpy(frame, frame_buf, len);
	*nlookups = lookups;
	return ret;
}
