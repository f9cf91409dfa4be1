/*
 * TEST INFRASTRUCTURE — the "optimized CPU" ipcache lookups of BASELINE.md
 * §2 (a DIR-24-8 for IPv4 and a multibit trie for IPv6), so that the GPU is
 * not compared only against the kernel-like binary trie.  Part of the CPU
 * restatement (included by cgpu_oracle.c only), selected by or_set_fast();
 * it answers every lookup exactly as lpm_lookup() on the same ipcache does
 * (pinned by the same golden tests, tests/test_oracle_golden.py), which is
 * the longest-prefix semantics of the reference's ipcache_lookup4 / 6
 * (bpf/lib/eps.h:56-80) over kernel/bpf/lpm_trie.c.
 *
 * The ipcache key is {pad[3], family, ip[16]} with the prefix length counted
 * over all of it: a v4 lookup is a /64 key (32 static bits + 32), a v6 one
 * /160.  An entry that ends inside the static 32 bits and agrees with the
 * lookup's {pad, family} matches every address of that family, below any
 * real prefix (the per-family default here); an entry longer than the
 * lookup key never matches it.
 *
 * IPv4: tbl24[2^24] entries, tbl8 groups of 256 for the /25-/32 parts; an
 *   entry is a value index + 1 (0: none -> the default), or bit 31 + a group.
 * IPv6: a root of 2^16 entries, then 8-bit strides down to bit 64 (levels at
 *   16, 24, ..., 56), values pushed to the leaves (controlled prefix
 *   expansion); a /64 entry that holds longer prefixes carries bit 30 and
 *   the /64's own value, and its longer prefixes sit in a per-/64 list
 *   (open-addressed by the /64, longest first) probed after the trie.
 */
#ifndef ORACLE_FAST_LPM_H
#define ORACLE_FAST_LPM_H

#define FL_CHILD 0x80000000u
#define FL_DEEP 0x40000000u
#define FL_IDX 0x3FFFFFFFu

struct fl_deep {            /* one prefix longer than /64 */
	uint64_t lo;        /* address bits 64..127 (host order, MSB first) */
	uint32_t len;       /* 65..128 */
	uint32_t val;       /* value index + 1 */
};

struct fast_lpm {
	const uint8_t **vals; /* value index -> the trie's value bytes */
	size_t n_vals, cap_vals;
	uint32_t def4, def6;  /* value index + 1 of the per-family defaults */
	uint32_t *tbl24, *tbl8;
	size_t n8, cap8;
	uint32_t *root6;      /* 65536 entries */
	uint32_t *nodes6;     /* 256-entry nodes */
	size_t nn6, capn6;
	/* /64 -> its longer prefixes: open addressing over (hi, start, count) */
	uint64_t *dk;         /* the /64 (host order), 0 = empty slot (with dused) */
	uint32_t *dstart, *dcount;
	uint8_t *dused;
	size_t dmask;
	struct fl_deep *deep;
	size_t ndeep;
};

static uint32_t fl_val(struct fast_lpm *f, const uint8_t *v)
{
	if (f->n_vals == f->cap_vals) {
		f->cap_vals = f->cap_vals ? 2 * f->cap_vals : 1024;
		f->vals = realloc(f->vals, f->cap_vals * sizeof(*f->vals));
	}
	f->vals[f->n_vals] = v;
	return (uint32_t)++f->n_vals;
}

static void fl_free(struct fast_lpm *f)
{
	if (!f)
		return;
	free(f->vals);
	free(f->tbl24);
	free(f->tbl8);
	free(f->root6);
	free(f->nodes6);
	free(f->dk);
	free(f->dstart);
	free(f->dcount);
	free(f->dused);
	free(f->deep);
	free(f);
}

struct fl_pfx {
	const uint8_t *data; /* the key's 20 data bytes */
	uint32_t plen;       /* over the whole key */
	const uint8_t *val;
};

static void fl_collect(const struct lpm_node *n, struct fl_pfx **out, size_t *cnt, size_t *cap)
{
	if (!n)
		return;
	if (!(n->flags & LPM_IM)) {
		if (*cnt == *cap) {
			*cap = *cap ? 2 * *cap : 4096;
			*out = realloc(*out, *cap * sizeof(**out));
		}
		(*out)[(*cnt)++] = (struct fl_pfx){n->data, n->prefixlen, n->val};
	}
	fl_collect(n->child[0], out, cnt, cap);
	fl_collect(n->child[1], out, cnt, cap);
}

static int fl_cmp_len(const void *a, const void *b)
{
	const struct fl_pfx *x = a, *y = b;
	return x->plen < y->plen ? -1 : x->plen > y->plen;
}

/* do the first `bits` bits of the key data equal the static header
 * {0, 0, 0, family}? */
static int fl_header_match(const uint8_t *data, uint32_t bits, uint8_t family)
{
	const uint8_t hdr[4] = {0, 0, 0, family};
	for (uint32_t i = 0; i < bits; i++)
		if (lpm_bit(data, i) != lpm_bit(hdr, i))
			return 0;
	return 1;
}

static uint64_t fl_be64(const uint8_t *p)
{
	uint64_t x = 0;
	for (int i = 0; i < 8; i++)
		x = x << 8 | p[i];
	return x;
}

/* a new 256-entry v6 node filled with `fill` */
static uint32_t fl_node6(struct fast_lpm *f, uint32_t fill)
{
	if (f->nn6 == f->capn6) {
		f->capn6 = f->capn6 ? 2 * f->capn6 : 4096;
		f->nodes6 = realloc(f->nodes6, f->capn6 * 256 * sizeof(uint32_t));
	}
	uint32_t *e = f->nodes6 + f->nn6 * 256;
	for (int i = 0; i < 256; i++)
		e[i] = fill;
	return (uint32_t)f->nn6++;
}

/* the entry slot for address bits [0, 16 + 8 * level) of a (host-order
 * bytes), creating the nodes above it (leaf-pushing their entries) */
static uint32_t *fl_slot6(struct fast_lpm *f, const uint8_t *a, int level)
{
	uint32_t *e = &f->root6[(uint32_t)a[0] << 8 | a[1]];
	for (int l = 1; l <= level; l++) {
		if (!(*e & FL_CHILD)) {
			const uint32_t node = fl_node6(f, *e & ~FL_DEEP);
			e = &f->root6[(uint32_t)a[0] << 8 | a[1]]; /* nodes6 may have moved: re-walk */
			for (int k = 1; k < l; k++)
				e = &f->nodes6[(size_t)(*e & FL_IDX) * 256 + a[k + 1]];
			*e = FL_CHILD | node;
		}
		e = &f->nodes6[(size_t)(*e & FL_IDX) * 256 + a[l + 1]];
	}
	return e;
}

static size_t fl_dslot(const struct fast_lpm *f, uint64_t hi)
{
	uint64_t h = hi * 0x9E3779B97F4A7C15ull;
	size_t j = (size_t)(h >> 29) & f->dmask;
	while (f->dused[j] && f->dk[j] != hi)
		j = (j + 1) & f->dmask;
	return j;
}

struct fl_deep_tmp {
	uint64_t hi;
	struct fl_deep d;
};

static int fl_cmp_deep_tmp(const void *a, const void *b)
{
	const struct fl_deep_tmp *x = a, *y = b;
	if (x->hi != y->hi)
		return x->hi < y->hi ? -1 : 1;
	return x->d.len > y->d.len ? -1 : x->d.len < y->d.len; /* longest first */
}

/* hdr: the ipcache layout ({pad[3], family, ip[16]}, prefix lengths over the
 * whole key); else a plain address trie (the XDP prefilter's lpm_v4_key /
 * lpm_v6_key data: the address alone, family by its size) */
static struct fast_lpm *fl_build(const struct lpm_trie *t, int hdr)
{
	struct fast_lpm *f = calloc(1, sizeof(*f));
	struct fl_pfx *p = NULL;
	size_t np = 0, cap = 0;
	struct fl_deep_tmp *dt = NULL;
	size_t ndt = 0;
	fl_collect(t->root, &p, &np, &cap);
	qsort(p, np, sizeof(*p), fl_cmp_len);
	f->tbl24 = calloc((size_t)1 << 24, sizeof(uint32_t));
	f->root6 = calloc(65536, sizeof(uint32_t));
	dt = malloc((np ? np : 1) * sizeof(*dt));
	for (size_t i = 0; i < np; i++) {
		const struct fl_pfx *x = &p[i];
		if (!hdr) {
			/* the plain trie in the ipcache form of its family (a
			 * buffer this iteration alone reads) */
			static __thread uint8_t d[20];
			memset(d, 0, sizeof(d));
			d[3] = t->data_size == 4 ? 1 : 2;
			memcpy(d + 4, x->data, t->data_size);
			p[i] = (struct fl_pfx){d, x->plen + 32, x->val};
			x = &p[i];
		}
		if (x->plen < 32) {
			/* ends inside the static header: a per-family default (the
			 * longest wins: ascending order) */
			if (fl_header_match(x->data, x->plen, 1))
				f->def4 = fl_val(f, x->val);
			if (fl_header_match(x->data, x->plen, 2))
				f->def6 = fl_val(f, x->val);
			continue;
		}
		if (!fl_header_match(x->data, 32, x->data[3]) || (x->data[3] != 1 && x->data[3] != 2))
			continue; /* a header no lookup key carries */
		const uint32_t q = x->plen - 32;
		if (x->data[3] == 1) {
			if (q > 32)
				continue; /* longer than the v4 lookup key: never matches */
			const uint32_t a = (uint32_t)x->data[4] << 24 | (uint32_t)x->data[5] << 16 |
					   (uint32_t)x->data[6] << 8 | x->data[7];
			const uint32_t v = fl_val(f, x->val);
			if (q <= 24) {
				const uint32_t lo = q ? (a >> 8) & ~((1u << (24 - q)) - 1u) : 0u;
				const uint32_t hi = lo + (1u << (24 - q));
				for (uint32_t k = lo; k < hi; k++)
					f->tbl24[k] = v;
			} else {
				uint32_t *e = &f->tbl24[a >> 8];
				if (!(*e & FL_CHILD)) {
					if (f->n8 == f->cap8) {
						f->cap8 = f->cap8 ? 2 * f->cap8 : 1024;
						f->tbl8 = realloc(f->tbl8, f->cap8 * 256 * sizeof(uint32_t));
					}
					for (int k = 0; k < 256; k++)
						f->tbl8[f->n8 * 256 + k] = *e;
					*e = FL_CHILD | (uint32_t)f->n8++;
				}
				uint32_t *g = f->tbl8 + (size_t)(*e & FL_IDX) * 256;
				const uint32_t lo = (a & 0xFFu) & ~((1u << (32 - q)) - 1u);
				for (uint32_t k = lo; k < lo + (1u << (32 - q)); k++)
					g[k] = v;
			}
			continue;
		}
		/* IPv6 */
		const uint8_t *a = x->data + 4;
		const uint32_t v = fl_val(f, x->val);
		if (q > 64) {
			uint32_t *e = fl_slot6(f, a, 6);
			*e |= FL_DEEP;
			dt[ndt].hi = fl_be64(a);
			dt[ndt].d.lo = fl_be64(a + 8) & (q == 128 ? ~0ull : ~(~0ull >> (q - 64)));
			dt[ndt].d.len = q;
			dt[ndt].d.val = v;
			ndt++;
			continue;
		}
		/* levels: root covers bits 0..15, level l bits 16 + 8 (l - 1) .. */
		const int level = q <= 16 ? 0 : (int)((q - 16 + 7) / 8);
		const uint32_t span = level ? 16u + 8u * (uint32_t)level : 16u;
		const uint32_t free_bits = span - q; /* expanded bits of the last stride */
		uint32_t *e = level ? fl_slot6(f, a, level) : &f->root6[(uint32_t)a[0] << 8 | a[1]];
		/* e is the entry of the prefix's first expansion; its node / root
		 * holds the 2^free_bits entries from the aligned start */
		uint32_t *base;
		uint32_t idx;
		if (level == 0) {
			base = f->root6;
			idx = ((uint32_t)a[0] << 8 | a[1]) & ~((1u << free_bits) - 1u);
		} else {
			base = e - a[level + 1];
			idx = (uint32_t)a[level + 1] & ~((1u << free_bits) - 1u);
		}
		for (uint32_t k = idx; k < idx + (1u << free_bits); k++) {
			/* no child exists below a stride a shorter prefix fills
			 * (ascending order); keep a /64's deep bit (set by none yet) */
			base[k] = (base[k] & FL_DEEP) | v;
		}
	}
	/* the per-/64 lists, longest first */
	qsort(dt, ndt, sizeof(*dt), fl_cmp_deep_tmp);
	f->deep = malloc((ndt ? ndt : 1) * sizeof(*f->deep));
	f->ndeep = ndt;
	size_t slots = 64;
	while (slots < 2 * ndt)
		slots <<= 1;
	f->dmask = slots - 1;
	f->dk = calloc(slots, sizeof(uint64_t));
	f->dstart = calloc(slots, sizeof(uint32_t));
	f->dcount = calloc(slots, sizeof(uint32_t));
	f->dused = calloc(slots, 1);
	for (size_t i = 0; i < ndt; i++) {
		f->deep[i] = dt[i].d;
		const size_t j = fl_dslot(f, dt[i].hi);
		if (!f->dused[j]) {
			f->dused[j] = 1;
			f->dk[j] = dt[i].hi;
			f->dstart[j] = (uint32_t)i;
		}
		f->dcount[j]++;
	}
	free(dt);
	free(p);
	return f;
}

static const uint8_t *fl_lookup4(const struct fast_lpm *f, uint32_t addr_be)
{
	const uint32_t a = __builtin_bswap32(addr_be);
	uint32_t e = f->tbl24[a >> 8];
	if (e & FL_CHILD)
		e = f->tbl8[(size_t)(e & FL_IDX) * 256 + (a & 0xFFu)];
	e = e ? e : f->def4;
	return e ? f->vals[e - 1] : NULL;
}

static const uint8_t *fl_lookup6(const struct fast_lpm *f, const uint8_t *a)
{
	uint32_t e = f->root6[(uint32_t)a[0] << 8 | a[1]];
	for (int l = 2; (e & FL_CHILD) && l < 8; l++)
		e = f->nodes6[(size_t)(e & FL_IDX) * 256 + a[l]];
	if (e & FL_DEEP) {
		const uint64_t hi = fl_be64(a), lo = fl_be64(a + 8);
		const size_t j = fl_dslot(f, hi);
		if (f->dused[j]) {
			const struct fl_deep *d = f->deep + f->dstart[j];
			for (uint32_t k = 0; k < f->dcount[j]; k++) {
				const uint64_t m = d[k].len == 128 ? ~0ull : ~(~0ull >> (d[k].len - 64));
				if ((lo & m) == d[k].lo)
					return f->vals[d[k].val - 1];
			}
		}
	}
	e &= FL_IDX;
	e = e ? e : f->def6;
	return e ? f->vals[e - 1] : NULL;
}

#endif
