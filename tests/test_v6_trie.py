"""CPU parity of the IPv6 ipcache trie (tables.h v6_lpm, host.cpp build_v6;
VERDICT r2 next 4): the library builds the trie from ipcache keys exactly as
a commit does and answers lookups with its host restatement of the device
walk (cgpu_diag_ipc6_trie, a test hook outside include/cgpu.h); the answers
must equal the restatement's ipcache LPM (oracle/cgpu_oracle.c
or_ipcache_lookup, pinned by tests/golden/classify_v6.npz), address by
address.  The GPU tests (test_gpu_parity / test_gpu_fullsize v6 cases) check
the device walk itself.  Shapes: the config-v6 table, a /32 too dense for
64 sub-range lines (the binary-searched long node), boundaries at both ends
of a /32 (a window of the whole range), /64s with several nested or disjoint
/65+ prefixes (lists), static-part entries and ::/0 under everything, /17../32
expansion under longer prefixes, tombstones."""
import ctypes as C

import numpy as np
import pytest

from cilium_amd import _abi, layouts as L, synth

V6T_LONG = 7


def trie(keys, labels, addrs):
    f = _abi.lib().cgpu_diag_ipc6_trie
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p]
    keys = np.ascontiguousarray(keys)
    labels = np.ascontiguousarray(labels, np.uint32)
    addrs = np.ascontiguousarray(addrs, np.uint8)
    out = np.empty(len(addrs), np.uint32)
    st = np.zeros(8, np.uint32)
    rc = f(keys.ctypes.data, labels.ctypes.data, len(keys), addrs.ctypes.data, len(addrs),
           out.ctypes.data, st.ctypes.data)
    assert rc == 0
    return out, dict(zip(("nodes", "long", "h64", "lists", "pool", "b24", "b32", "slots"), st.tolist()))


def oracle_labels(keys, labels, addrs):
    from oracle import Oracle
    o = Oracle()
    v = np.zeros(len(keys), L.REMOTE_ENDPOINT_INFO)
    v["sec_label"] = labels
    for k, x in zip(keys, v):
        assert o.ipcache_update(k, x) == 0
    q = np.zeros((), L.IPCACHE_KEY)
    q["prefixlen"] = L.IPCACHE_STATIC_PREFIX + 128
    q["family"] = L.ENDPOINT_KEY_IPV6
    out = np.empty(len(addrs), np.uint32)
    for i, a in enumerate(addrs):
        q["ip"] = a
        r, raw = o.ipcache_lookup(q)
        out[i] = np.frombuffer(raw, L.REMOTE_ENDPOINT_INFO)[0]["sec_label"] if r == 0 else 0xFFFFFFFF
    return out


def keys_of(addr, plen, static=False):
    k = np.zeros(len(plen), L.IPCACHE_KEY)
    k["family"] = L.ENDPOINT_KEY_IPV6
    k["prefixlen"] = np.asarray(plen) + (0 if static else L.IPCACHE_STATIC_PREFIX)
    k["ip"] = addr
    return k


def probes(addr, plen, rng, n_rand):
    """Every prefix's first and last address and their outside neighbours,
    random addresses inside prefixes and under their /16s."""
    a = np.asarray(addr, np.uint8)
    m = synth.MASK6[np.asarray(plen)]
    lo, hi = a & m, (a & m) | ~m
    out = [lo, hi]
    M = (1 << 128) - 1
    for x, d in ((lo, -1), (hi, 1)):
        v = [((int.from_bytes(r.tobytes(), "big") + d) & M).to_bytes(16, "big") for r in x]
        out.append(np.frombuffer(b"".join(v), np.uint8).reshape(-1, 16))
    pi = rng.integers(0, len(a), n_rand)
    r = rng.integers(0, 256, (n_rand, 16), dtype=np.uint8)
    out.append((a[pi] & m[pi]) | (r & ~m[pi]))
    r2 = rng.integers(0, 256, (n_rand, 16), dtype=np.uint8)
    r2[:, :2] = a[pi, :2]
    out.append(r2)
    return np.concatenate(out)


def check(keys, labels, addrs):
    got, st = trie(keys, labels, addrs)
    exp = oracle_labels(keys, labels, addrs)
    bad = np.flatnonzero(got != exp)
    assert len(bad) == 0, (len(bad), addrs[bad[:3]], got[bad[:3]], exp[bad[:3]])
    return st


def test_trie_config_v6_table():
    T = synth.make_tables6(n_prefixes=20_000, n_identities=500, n_endpoints=2, keys_per_ep=100)
    rng = np.random.Generator(np.random.PCG64(61))
    pick = rng.choice(len(T.pfx_len), 3000, replace=False)
    addrs = probes(T.pfx_addr[pick], T.pfx_len[pick], rng, 5000)
    addrs = np.concatenate([addrs, synth.make_tuples6(T, 5000)["daddr"]])
    st = check(T.ipc_keys, T.ipc_vals["sec_label"], addrs)
    assert st["nodes"] > 100 and st["h64"] > 1000


def edge_table():
    rng = np.random.Generator(np.random.PCG64(62))
    addr, plen, lab = [], [], []

    def put(a, n, lb):
        a = np.array(a, np.uint8)
        addr.append(a & synth.MASK6[n])
        plen.append(n)
        lab.append(lb)
    base = np.zeros(16, np.uint8)
    # a /32 too dense for 64 sub-range lines: 1500 /64s (3000 boundaries)
    d = base.copy()
    d[:4] = [0x20, 0x01, 0x0d, 0xb8]
    put(d, 32, 1001)
    for i in range(1500):
        x = d.copy()
        x[4:8] = rng.integers(0, 256, 4, dtype=np.uint8)
        put(x, 64, 2000 + i)
    # boundaries at both ends of a /32, nested inside a /24 and a /20
    e = base.copy()
    e[:4] = [0x20, 0x01, 0x0e, 0x77]
    put(e, 20, 1101)
    put(e, 24, 1102)
    lo = e.copy()
    put(lo, 48, 1103)
    hi = e.copy()
    hi[4:8] = 0xFF
    put(hi, 64, 1104)
    mid = e.copy()
    mid[4:6] = [0x80, 0x00]
    put(mid, 33, 1105)
    put(mid, 40, 1106)
    # /64s with nested and disjoint /65+ prefixes (lists) and one inline
    for j in range(40):
        s = base.copy()
        s[:8] = [0x20, 0x01, 0x0f, 0x00, 0x00, j, 0x12, 0x34]
        put(s, 64, 3000 + j)
        t = s.copy()
        t[8:] = rng.integers(0, 256, 8, dtype=np.uint8)
        put(t, 96, 3100 + j)
        put(t, 112, 3200 + j)
        put(t, 128, 3300 + j)
        if j % 2:
            u = s.copy()
            u[8:] = rng.integers(0, 256, 8, dtype=np.uint8)
            put(u, 128, 3400 + j)
            put(u, 65, 3500 + j)
        if j % 5 == 0:
            v = s.copy()
            v[8:] = 0xFF
            put(v, 128, 3600 + j)  # ends at the /64's last address
    inl = base.copy()
    inl[:8] = [0x20, 0x01, 0x0f, 0x01, 0, 0, 0, 1]
    put(inl, 100, 3700)  # a /64 whose only /65+ prefix is inline
    # /65+ only under a /32 (no /33../64): a deep node of one line
    o = base.copy()
    o[:4] = [0x20, 0x01, 0x0f, 0x02]
    o[8:] = rng.integers(0, 256, 8, dtype=np.uint8)
    put(o, 128, 3800)
    # /17../32 expansion around a /48, tombstones
    f = base.copy()
    f[:6] = [0x20, 0x01, 0x0a, 0x0b, 0x0c, 0x0d]
    put(f, 17, 4001)
    put(f, 23, 4002)
    put(f, 29, 0)  # tombstone (sec_label 0: a match that shadows)
    put(f, 31, 4004)
    put(f, 48, 4005)
    put(f, 56, 0)
    # ::/0 and two static-part entries (rank below /0)
    put(base, 0, 2)
    keys = keys_of(np.array(addr), plen)
    st_keys = np.zeros(2, L.IPCACHE_KEY)
    st_keys["family"] = L.ENDPOINT_KEY_IPV6
    st_keys["prefixlen"] = [0, 31]
    return (np.concatenate([keys, st_keys]), np.array(lab + [7, 8], np.uint32),
            np.array(addr), np.array(plen), rng)


def test_trie_edge_shapes():
    keys, labels, addr, plen, rng = edge_table()
    addrs = probes(addr, plen, rng, 20_000)
    st = check(keys, labels, addrs)
    assert st["long"] >= 1           # the dense /32
    assert st["lists"] >= 20         # nested / disjoint /65+ in one /64
    assert st["h64"] > st["lists"]   # and inline records


def test_trie_static_only_and_empty():
    # only static-part entries: no trie levels below the root
    k = np.zeros(1, L.IPCACHE_KEY)
    k["family"] = L.ENDPOINT_KEY_IPV6
    k["prefixlen"] = 20
    addrs = np.random.Generator(np.random.PCG64(3)).integers(0, 256, (100, 16), dtype=np.uint8)
    check(k, np.array([9], np.uint32), addrs)
    got, _ = trie(np.zeros(0, L.IPCACHE_KEY), np.zeros(0, np.uint32), addrs)
    assert (got == 0xFFFFFFFF).all()


@pytest.mark.parametrize("seed", [1, 2])
def test_trie_random_nested(seed):
    """Random nested prefix sets: every length 0..128 under a few /16 roots."""
    rng = np.random.Generator(np.random.PCG64(100 + seed))
    roots = rng.integers(0, 256, (4, 2), dtype=np.uint8)
    n = 4000
    a = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    a[:, :2] = roots[rng.integers(0, 4, n)]
    # cluster: half the prefixes share longer stems so they nest
    stem = a[rng.integers(0, 64, n)]
    keep = rng.integers(2, 14, n)
    for i in range(n // 2):
        a[i, :keep[i]] = stem[i, :keep[i]]
    plen = rng.integers(0, 129, n)
    a &= synth.MASK6[plen]
    keys = keys_of(a, plen)
    canon = np.zeros(n, np.dtype([("l", "u4"), ("a", "u1", (16,))]))
    canon["l"], canon["a"] = plen, a
    _, first = np.unique(canon.view(np.dtype((np.void, 20))), return_index=True)
    keys, a, plen = keys[first], a[first], plen[first]
    labels = rng.integers(1, 1 << 31, len(keys)).astype(np.uint32)  # indirect labels too
    addrs = probes(a, plen, rng, 10_000)
    check(keys, labels, addrs)
