/*
 * Sanitizer driver (SURVEY §5 race detection / sanitizers): the C ABI of
 * libcgpu on host-only contexts (device = -1: every table, PreFilter,
 * conntrack, checkpoint call; no device), linked against a build of the
 * library whose host code carries -fsanitize=address,undefined (mode
 * "asan") or -fsanitize=thread (mode "tsan": the same calls from several
 * threads on one context, the mirror lock's contract).  Any report aborts
 * with a nonzero exit; tests/test_sanitizers.py builds and runs it.
 */
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "cgpu.h"

#define CHECK(x)                                                                              \
	do {                                                                                   \
		if (!(x)) {                                                                    \
			fprintf(stderr, "%s:%d: CHECK(%s) failed: %s\n", __FILE__, __LINE__, #x, \
				cgpu_last_error());                                            \
			exit(2);                                                               \
		}                                                                              \
	} while (0)

static bool g_concurrent; /* tsan mode: other threads change the maps between calls */

static cgpu_ctx *make(uint32_t ct_max = 4096)
{
	cgpu_config cfg;
	cgpu_config_default(&cfg);
	cfg.ct_max = ct_max;
	cfg.ct6_max = ct_max / 2;
	cfg.policy_max_per_ep = 512;
	cfg.max_endpoints = 16;
	cfg.lb_max_entries = 2048;
	cgpu_ctx *c = nullptr;
	CHECK(cgpu_ctx_create(&cfg, -1, &c) == 0);
	return c;
}

static void tables(cgpu_ctx *c, std::mt19937 &rng, int rounds)
{
	for (int i = 0; i < rounds; i++) {
		cgpu_ipcache_key k{};
		const bool v6 = rng() & 1;
		k.family = v6 ? 2 : 1;
		k.prefixlen = 32 + (uint32_t)(rng() % (v6 ? 129 : 33));
		for (auto &b : k.ip)
			b = (uint8_t)rng();
		cgpu_remote_endpoint_info v{(uint32_t)rng() % 70000, (uint32_t)rng()};
		const int r = cgpu_ipcache_update(c, &k, &v, rng() % 3);
		CHECK(r == 0 || r == -EEXIST || r == -ENOENT || r == -ENOSPC);
		cgpu_remote_endpoint_info o;
		(void)cgpu_ipcache_lookup(c, &k, &o);
		if (rng() % 4 == 0)
			(void)cgpu_ipcache_delete(c, &k);
		k.prefixlen = 161 + (uint32_t)(rng() % 8);
		CHECK(cgpu_ipcache_update(c, &k, &v, 0) == -EINVAL);

		const uint32_t ep = rng() % 20; /* some out of range */
		cgpu_policy_key pk{(uint32_t)rng() % 300, (uint16_t)(rng() % 4), (uint8_t)(rng() % 3 ? 6 : 0),
				   (uint8_t)(rng() & 1)};
		cgpu_policy_entry pe{};
		pe.proxy_port = (uint16_t)(rng() % 3 ? 0 : rng());
		pe.packets = rng() % 10;
		const int pr = cgpu_policy_update(c, ep, &pk, &pe, rng() % 3);
		CHECK(pr == 0 || pr == -EEXIST || pr == -ENOENT || pr == -E2BIG || pr == -EINVAL);
		if (rng() % 5 == 0)
			(void)cgpu_policy_delete(c, ep, &pk);
		if (rng() % 97 == 0)
			(void)cgpu_policy_flush(c, ep % 16);

		cgpu_cidr_key ck{};
		const int which = (int)(rng() % 4);
		ck.prefixlen = (uint32_t)(rng() % 140);
		for (auto &b : ck.addr)
			b = (uint8_t)rng();
		const int cr = cgpu_cidr_update(c, which, &ck, 0);
		CHECK(cr == 0 || cr == -EINVAL || cr == -E2BIG || cr == -ENOSPC);
		(void)cgpu_cidr_lookup(c, which, &ck);

		cgpu_endpoint_key ek{};
		ek.family = 1 + (rng() & 1);
		ek.ip[15] = (uint8_t)rng();
		(void)cgpu_endpoint_update(c, &ek, 0);

		cgpu_lb4_key lk{(uint32_t)rng() % 64, (uint16_t)(rng() % 3), (uint16_t)(rng() % 4)};
		cgpu_lb4_service ls{(uint32_t)rng(), 80, (uint16_t)(rng() % 4), 1, 0};
		(void)cgpu_lb4_update(c, &lk, &ls, 0);
		cgpu_lb6_key l6{};
		l6.address[0] = (uint8_t)(rng() % 16);
		l6.slave = (uint16_t)(rng() % 3);
		cgpu_lb6_service s6{};
		s6.count = 2;
		(void)cgpu_lb6_update(c, &l6, &s6, 0);
		if (rng() % 7 == 0)
			(void)cgpu_lb4_delete(c, &lk);

		cgpu_lxc_info li{};
		li.sec_label = (uint32_t)rng();
		(void)cgpu_lxc_update(c, rng() % 8, &li);

		cgpu_ct4_tuple t4{(uint32_t)rng() % 500, 1, 80, (uint16_t)rng(), 6, (uint8_t)(rng() % 4)};
		cgpu_ct_entry ce{};
		ce.lifetime = (uint32_t)(rng() % 1000);
		const int r4 = cgpu_ct4_update(c, &t4, &ce, 0);
		CHECK(r4 == 0 || r4 == -E2BIG);
		cgpu_ct6_tuple t6{};
		t6.daddr[15] = (uint8_t)rng();
		t6.daddr[3] = (uint8_t)rng();
		t6.nexthdr = 58;
		const int r6 = cgpu_ct6_update(c, &t6, &ce, 0);
		CHECK(r6 == 0 || r6 == -E2BIG);
		if (rng() % 3 == 0)
			(void)cgpu_ct6_delete(c, &t6);
		if (rng() % 3 == 0)
			(void)cgpu_ct4_delete(c, &t4);
		cgpu_ct_entry got;
		(void)cgpu_ct4_lookup(c, &t4, &got);
	}
}

static void walks(cgpu_ctx *c)
{
	cgpu_ipcache_key k, n;
	const cgpu_ipcache_key *p = nullptr;
	while (cgpu_ipcache_get_next_key(c, p, &n) == 0) {
		k = n;
		p = &k;
	}
	for (uint32_t ep = 0; ep < 16; ep++) {
		size_t cnt = 0;
		(void)cgpu_policy_dump(c, ep, nullptr, nullptr, 0, &cnt);
		std::vector<cgpu_policy_key> keys(cnt + 1);
		std::vector<cgpu_policy_entry> ents(cnt + 1);
		const int r = cgpu_policy_dump(c, ep, keys.data(), ents.data(), keys.size(), &cnt);
		CHECK(r == 0 || (g_concurrent && r == -ENOSPC));
		if (!g_concurrent && cnt > 1)
			CHECK(cgpu_policy_dump(c, ep, keys.data(), ents.data(), cnt - 1, &cnt) == -ENOSPC);
	}
	for (int w = 0; w < 4; w++) {
		cgpu_cidr_key a, b;
		const cgpu_cidr_key *q = nullptr;
		while (cgpu_cidr_get_next_key(c, w, q, &b) == 0) {
			a = b;
			q = &a;
		}
	}
	cgpu_ct4_tuple a4, b4;
	const cgpu_ct4_tuple *q4 = nullptr;
	while (cgpu_ct4_get_next_key(c, q4, &b4) == 0) {
		a4 = b4;
		q4 = &a4;
	}
	cgpu_ct6_tuple a6, b6;
	const cgpu_ct6_tuple *q6 = nullptr;
	while (cgpu_ct6_get_next_key(c, q6, &b6) == 0) {
		a6 = b6;
		q6 = &a6;
	}
	cgpu_lb4_key l4, m4;
	const cgpu_lb4_key *r4 = nullptr;
	while (cgpu_lb4_get_next_key(c, r4, &m4) == 0) {
		l4 = m4;
		r4 = &l4;
	}
	(void)cgpu_ipcache_count(c);
	(void)cgpu_ct4_count(c);
	(void)cgpu_ct6_count(c);
	(void)cgpu_lb6_count(c);
}

static void prefilter(cgpu_ctx *c)
{
	int64_t rev;
	CHECK(cgpu_prefilter_revision(c, &rev) == 0);
	cgpu_prefix p[3] = {};
	p[0].bits = 32;
	p[0].key.prefixlen = 24;
	p[0].key.addr[0] = 10;
	p[1].bits = 128;
	p[1].key.prefixlen = 128;
	p[1].key.addr[0] = 0xfe;
	p[2] = p[0]; /* duplicate: the insert fails and is undone */
	(void)cgpu_prefilter_insert(c, rev, p, 3);
	(void)cgpu_prefilter_insert(c, rev, p, 2);
	CHECK(g_concurrent || cgpu_prefilter_insert(c, rev, p, 2) == -ESTALE);
	CHECK(cgpu_prefilter_revision(c, &rev) == 0);
	(void)cgpu_prefilter_delete(c, rev, p, 2);
}

static void checkpoint(cgpu_ctx *c, const std::string &dir)
{
	const std::string path = dir + "/mirror.bin";
	CHECK(cgpu_mirror_save(c, path.c_str()) == 0);
	cgpu_ctx *d = make();
	CHECK(cgpu_mirror_restore(d, path.c_str()) == 0);
	CHECK(cgpu_ipcache_count(d) == cgpu_ipcache_count(c));
	CHECK(cgpu_ct4_count(d) == cgpu_ct4_count(c));
	CHECK(cgpu_ct6_count(d) == cgpu_ct6_count(c));
	CHECK(cgpu_mirror_restore(d, path.c_str()) == -EEXIST);
	cgpu_ctx_destroy(d);
	/* a corrupted copy is rejected whole */
	FILE *f = fopen(path.c_str(), "r+b");
	CHECK(f);
	fseek(f, 40, SEEK_SET);
	fputc(0x5a, f);
	fclose(f);
	d = make();
	CHECK(cgpu_mirror_restore(d, path.c_str()) == -EINVAL);
	CHECK(cgpu_ipcache_count(d) == 0);
	cgpu_ctx_destroy(d);
}

int main(int argc, char **argv)
{
	const std::string mode = argc > 1 ? argv[1] : "asan";
	const std::string dir = argc > 2 ? argv[2] : "/tmp";
	std::mt19937 rng(12345);
	cgpu_ctx *c = make();
	if (mode == "tsan") {
		g_concurrent = true;
		std::vector<std::thread> th;
		for (int t = 0; t < 4; t++)
			th.emplace_back([c, t] {
				std::mt19937 r(7 + t);
				tables(c, r, 1500);
				walks(c);
			});
		th.emplace_back([c] {
			for (int i = 0; i < 20; i++) {
				walks(c);
				prefilter(c);
				uint64_t del;
				(void)cgpu_ct4_gc(c, 500, &del);
				(void)cgpu_ct6_gc(c, 500, &del);
			}
		});
		th.emplace_back([c, dir] {
			for (int i = 0; i < 5; i++)
				CHECK(cgpu_mirror_save(c, (dir + "/mirror_t.bin").c_str()) == 0);
		});
		for (auto &x : th)
			x.join();
	} else {
		tables(c, rng, 6000);
		walks(c);
		prefilter(c);
		uint64_t del = 0;
		CHECK(cgpu_ct4_gc(c, 500, &del) == 0);
		CHECK(cgpu_ct6_gc(c, 500, &del) == 0);
		CHECK(cgpu_ct4_flush(c) == 0);
		tables(c, rng, 2000);
		checkpoint(c, dir);
		/* device-only calls fail cleanly on a host-only context */
		CHECK(cgpu_commit(c, nullptr) == -ENODEV);
		CHECK(cgpu_table_verify(c) == -ENODEV);
		CHECK(cgpu_classify_v4(c, nullptr, 0, nullptr, nullptr, nullptr, nullptr) == -ENODEV);
		(void)cgpu_flow_hash(1, 2, 3, 4, 6);
		uint8_t a[16] = {1}, b[16] = {2};
		(void)cgpu_flow_hash6(a, b, 3, 4, 17);
	}
	cgpu_ctx_destroy(c);
	printf("sanitizer driver (%s) ok\n", mode.c_str());
	return 0;
}
