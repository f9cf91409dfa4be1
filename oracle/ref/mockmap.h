/*
 * TEST INFRASTRUCTURE — part of the oracle, never part of the product.
 *
 * Mock BPF map store for the reference harness (oracle/ref/harness_*.c).
 * The reference BPF C (/root/reference/bpf) calls map_lookup_elem() through a
 * writable helper pointer (bpf/include/bpf/api.h:101-112); the harness points
 * it at mockmap_lookup(), which supplies the kernel map semantics the
 * reference relies on but does not vendor:
 *   - BPF_MAP_TYPE_HASH: exact match, memcmp over the whole key including
 *     padding (kernel/bpf/hashtab.c htab_map_lookup_elem).
 *   - BPF_MAP_TYPE_LPM_TRIE: longest prefix match over key->data, MSB first
 *     within each byte, candidates restricted to entry.prefixlen <=
 *     query.prefixlen (kernel/bpf/lpm_trie.c trie_lookup_elem, Linux >= 4.11).
 * Linear scans: the harness only runs golden-vector sized cases.
 */
#ifndef ORACLE_REF_MOCKMAP_H
#define ORACLE_REF_MOCKMAP_H

#include <stddef.h>
#include <stdint.h>

enum { MOCK_HASH = 0, MOCK_LPM = 1 };

struct mockmap {
	int kind;
	size_t ksz, vsz;
	size_t n, cap;
	uint8_t *keys;
	uint8_t *vals;
	uint64_t lookups; /* number of lookups served (probe accounting) */
};

void mockmap_init(struct mockmap *m, int kind, size_t ksz, size_t vsz);
void mockmap_clear(struct mockmap *m);
void mockmap_free(struct mockmap *m);
/* returns 0 on insert, 1 on replace */
int mockmap_update(struct mockmap *m, const void *key, const void *val);
void *mockmap_lookup(struct mockmap *m, const void *key);
/* exact-key removal (kernel htab_map_delete_elem); returns 1 if removed */
int mockmap_delete(struct mockmap *m, const void *key);

#endif
