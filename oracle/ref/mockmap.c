/* TEST INFRASTRUCTURE — see mockmap.h. */
#include "mockmap.h"

#include <stdlib.h>
#include <string.h>

void mockmap_init(struct mockmap *m, int kind, size_t ksz, size_t vsz)
{
	memset(m, 0, sizeof(*m));
	m->kind = kind;
	m->ksz = ksz;
	m->vsz = vsz;
}

void mockmap_clear(struct mockmap *m)
{
	m->n = 0;
	m->lookups = 0;
}

void mockmap_free(struct mockmap *m)
{
	free(m->keys);
	free(m->vals);
	m->keys = m->vals = NULL;
	m->n = m->cap = 0;
}

/* Bit i of an LPM key's data, MSB first within each byte. */
static int lpm_bit(const uint8_t *data, uint32_t i)
{
	return (data[i / 8] >> (7 - (i % 8))) & 1;
}

/* Do the first `bits` bits of a and b agree? */
static int lpm_prefix_eq(const uint8_t *a, const uint8_t *b, uint32_t bits)
{
	for (uint32_t i = 0; i < bits; i++)
		if (lpm_bit(a, i) != lpm_bit(b, i))
			return 0;
	return 1;
}

/* Kernel lpm_trie identifies an element by (prefixlen, first prefixlen
 * bits); trailing bits of the stored key are whatever the last update
 * wrote (trie_update_elem replaces the node with a copy of the new key). */
static long find_same(const struct mockmap *m, const void *key)
{
	for (size_t i = 0; i < m->n; i++) {
		const uint8_t *k = m->keys + i * m->ksz;
		if (m->kind == MOCK_HASH) {
			if (!memcmp(k, key, m->ksz))
				return (long)i;
		} else {
			uint32_t pa, pb;
			memcpy(&pa, k, 4);
			memcpy(&pb, key, 4);
			if (pa == pb && lpm_prefix_eq(k + 4, (const uint8_t *)key + 4, pa))
				return (long)i;
		}
	}
	return -1;
}

int mockmap_update(struct mockmap *m, const void *key, const void *val)
{
	long i = find_same(m, key);
	if (i >= 0) {
		memcpy(m->keys + i * m->ksz, key, m->ksz);
		memcpy(m->vals + i * m->vsz, val, m->vsz);
		return 1;
	}
	if (m->n == m->cap) {
		m->cap = m->cap ? 2 * m->cap : 64;
		m->keys = realloc(m->keys, m->cap * m->ksz);
		m->vals = realloc(m->vals, m->cap * m->vsz);
	}
	memcpy(m->keys + m->n * m->ksz, key, m->ksz);
	memcpy(m->vals + m->n * m->vsz, val, m->vsz);
	m->n++;
	return 0;
}

void *mockmap_lookup(struct mockmap *m, const void *key)
{
	m->lookups++;
	if (m->kind == MOCK_HASH) {
		long i = find_same(m, key);
		return i < 0 ? NULL : m->vals + i * m->vsz;
	}
	uint32_t qlen;
	memcpy(&qlen, key, 4);
	long best = -1;
	uint32_t best_len = 0;
	for (size_t i = 0; i < m->n; i++) {
		const uint8_t *k = m->keys + i * m->ksz;
		uint32_t plen;
		memcpy(&plen, k, 4);
		if (plen > qlen)
			continue;
		if (best >= 0 && plen <= best_len)
			continue;
		if (lpm_prefix_eq(k + 4, (const uint8_t *)key + 4, plen)) {
			best = (long)i;
			best_len = plen;
		}
	}
	return best < 0 ? NULL : m->vals + best * m->vsz;
}

int mockmap_delete(struct mockmap *m, const void *key)
{
	long i = find_same(m, key);
	if (i < 0)
		return 0;
	m->n--;
	if ((size_t)i != m->n) {
		memmove(m->keys + i * m->ksz, m->keys + (i + 1) * m->ksz, (m->n - i) * m->ksz);
		memmove(m->vals + i * m->vsz, m->vals + (i + 1) * m->vsz, (m->n - i) * m->vsz);
	}
	return 1;
}
