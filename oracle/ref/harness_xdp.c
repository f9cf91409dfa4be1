/*
 * TEST INFRASTRUCTURE — the reference oracle for the XDP CIDR prefilter.
 * Built ONLY in the development container into oracle/_ref/libref_xdp.so
 * (see oracle/Makefile); run only by oracle/gen_golden.py.
 *
 * Compiles the reference's bpf/bpf_xdp.c (xdp_start -> check_filters ->
 * check_v4/check_v6 -> lookup_ip{4,6}_endpoint, bpf_xdp.c:88-184) as host C
 * with the shipped filter_config.h (all four CIDR maps enabled) and
 * HAVE_LPM_MAP_TYPE.  Frames are copied into a MAP_32BIT buffer because
 * xdp_md.data/data_end are __u32 in the reference's uapi header.
 */
#include <stdio.h>
#include <string.h>
#include <sys/mman.h>

#include "bpf_xdp.c"

#include "mockmap.h"

static struct mockmap v4_dyn_m, v4_fix_m, v6_dyn_m, v6_fix_m, lxc_m;
static uint64_t probes;
static int inited;
static unsigned char *frame_buf;

static void *mock_lookup(void *map, const void *key)
{
	probes++;
	if (map == &CIDR4_LMAP_NAME)
		return mockmap_lookup(&v4_dyn_m, key);
	if (map == &CIDR4_HMAP_NAME)
		return mockmap_lookup(&v4_fix_m, key);
	if (map == &CIDR6_LMAP_NAME)
		return mockmap_lookup(&v6_dyn_m, key);
	if (map == &CIDR6_HMAP_NAME)
		return mockmap_lookup(&v6_fix_m, key);
	if (map == &cilium_lxc)
		return mockmap_lookup(&lxc_m, key);
	fprintf(stderr, "ref xdp harness: lookup on unexpected map %p\n", map);
	return NULL;
}

static int ensure_init(void)
{
	if (inited)
		return 0;
	mockmap_init(&v4_dyn_m, MOCK_LPM, sizeof(struct lpm_v4_key), sizeof(struct lpm_val));
	mockmap_init(&v4_fix_m, MOCK_HASH, sizeof(struct lpm_v4_key), sizeof(struct lpm_val));
	mockmap_init(&v6_dyn_m, MOCK_LPM, sizeof(struct lpm_v6_key), sizeof(struct lpm_val));
	mockmap_init(&v6_fix_m, MOCK_HASH, sizeof(struct lpm_v6_key), sizeof(struct lpm_val));
	mockmap_init(&lxc_m, MOCK_HASH, sizeof(struct endpoint_key), sizeof(struct endpoint_info));
	frame_buf = mmap(NULL, 1 << 16, PROT_READ | PROT_WRITE,
			 MAP_PRIVATE | MAP_ANONYMOUS | MAP_32BIT, -1, 0);
	if (frame_buf == MAP_FAILED)
		return -1;
	map_lookup_elem = mock_lookup;
	inited = 1;
	return 0;
}

void ref_xdp_reset(void)
{
	ensure_init();
	mockmap_clear(&v4_dyn_m);
	mockmap_clear(&v4_fix_m);
	mockmap_clear(&v6_dyn_m);
	mockmap_clear(&v6_fix_m);
	mockmap_clear(&lxc_m);
}

/* which: 0 = v4 dyn (LPM), 1 = v4 fix (hash), 2 = v6 dyn, 3 = v6 fix.
 * key = raw lpm_v4_key (8 B) / lpm_v6_key (20 B), bpf/lib/xdp.h:23-31. */
int ref_xdp_cidr_update(int which, const void *key)
{
	struct lpm_val v = { 0 };
	struct mockmap *m[] = { &v4_dyn_m, &v4_fix_m, &v6_dyn_m, &v6_fix_m };
	if (ensure_init() || which < 0 || which > 3)
		return -1;
	return mockmap_update(m[which], key, &v);
}

/* raw endpoint_key (20 B, bpf/lib/common.h:147-160) into cilium_lxc. */
int ref_xdp_endpoint_update(const void *key)
{
	struct endpoint_info info;
	if (ensure_init())
		return -1;
	memset(&info, 0, sizeof(info));
	return mockmap_update(&lxc_m, key, &info);
}

/* Run xdp_start over one frame; returns XDP_DROP (1) / XDP_PASS (2). */
int ref_xdp_run(const uint8_t *frame, uint32_t len, uint64_t *nprobes)
{
	struct xdp_md x;
	int ret;
	if (ensure_init() || len > (1 << 16))
		return -1;
	memcpy(frame_buf, frame, len);
	memset(&x, 0, sizeof(x));
	x.data = (uint32_t)(unsigned long)frame_buf;
	x.data_end = (uint32_t)(unsigned long)(frame_buf + len);
	probes = 0;
	ret = xdp_start(&x);
	*nprobes = probes;
	return ret;
}

int ref_xdp_sizes(int *v4key, int *v6key, int *epkey)
{
	*v4key = sizeof(struct lpm_v4_key);
	*v6key = sizeof(struct lpm_v6_key);
	*epkey = sizeof(struct endpoint_key);
	return XDP_DROP * 16 + XDP_PASS;
}
