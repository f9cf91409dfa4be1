"""Seeded synthetic workloads of SURVEY §8d / BASELINE.md §3.

Config 1 ("cpu"):  1k identities, 10k IPv4 ipcache prefixes + reserved
                   entries, ~16k MapState keys on one endpoint, 1M tuples.
Config 2 ("gpu"):  100k prefixes, 64k policy entries (4 endpoints x 16k),
                   64M-tuple batches.
Tables are seeded identically on every rank (replicated); tuple streams are
seeded per GPU (seed 0xC1110000 + gpu_id, PCG64).

Distributions: prefix lengths {8:2%, 16:8%, 20:10%, 24:55%,
28:10%, 32:15%}; reserved 0.0.0.0/0 -> WORLD, cluster /16 -> CLUSTER, 4 host
/32 -> HOST, 0.5% tombstones (identity 0); MapState 45% L4 exact (dport
Zipf(1.1) over 64 ports, TCP 85% / UDP 15%), 45% L3-only, 10% identity-0 L4,
5% with a proxy port; tuples 80% inside installed prefixes, 20% uniform,
50/50 direction, 0.5% fragments, len uniform 64..1500.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import layouts as L

SEED = 0xC1110000
PORTS64 = np.array([80, 443, 8080, 53, 22, 8443, 3306, 5432, 6379, 9090, 9092, 2379, 2380,
                    11211, 27017, 5672, 15672, 8000, 8001, 8888, 9200, 9300, 5601, 3000,
                    4000, 6443, 10250, 10255, 30000, 30001, 30002, 30003, 7000, 7001, 7199,
                    9042, 9160, 50051, 50052, 1883, 8883, 5222, 5269, 6000, 6001, 6002, 25,
                    110, 143, 465, 587, 993, 995, 389, 636, 123, 161, 162, 514, 873, 2049,
                    111, 135, 445], np.uint16)
assert len(PORTS64) == 64

CONFIGS = {
    "cpu": dict(n_prefixes=10_000, n_identities=1000, n_endpoints=1, keys_per_ep=16_000,
                n_tuples=1 << 20),
    "gpu": dict(n_prefixes=100_000, n_identities=1000, n_endpoints=4, keys_per_ep=16_000,
                n_tuples=64 << 20),
    # config 5: config-2 tables + 1M IPv4 services in front
    "cascade": dict(n_prefixes=100_000, n_identities=1000, n_endpoints=4, keys_per_ep=16_000,
                    n_tuples=64 << 20, n_services=1_000_000),
    # IPv6 classify at config-2 size (make_tables6)
    "v6": dict(n_prefixes=100_000, n_identities=1000, n_endpoints=4, keys_per_ep=16_000,
               n_tuples=64 << 20),
}

# cluster CIDR 10.0.0.0/8 expressed like node_config.h's IPV4_CLUSTER_MASK /
# IPV4_CLUSTER_RANGE (network-order u32 constants, daemon/daemon.go:919-920)
CLUSTER_MASK = L.ip4_be(0xFF000000)
CLUSTER_RANGE = L.ip4_be(0x0A000000)
CLUSTER_V4 = 0x0A000000


def zipf_ports(rng, n, s=1.1):
    w = 1.0 / np.arange(1, 65) ** s
    return PORTS64[rng.choice(64, n, p=w / w.sum())]


@dataclass
class Tables:
    ipc_keys: np.ndarray      # IPCACHE_KEY
    ipc_vals: np.ndarray      # REMOTE_ENDPOINT_INFO
    pfx_addr: np.ndarray      # host-order base address per non-reserved prefix
    pfx_len: np.ndarray
    pol_keys: np.ndarray      # POLICY_KEY
    pol_entries: np.ndarray   # POLICY_ENTRY
    pol_ep: np.ndarray        # uint16
    n_endpoints: int
    cluster_mask: int = CLUSTER_MASK
    cluster_range: int = CLUSTER_RANGE

    def engine_config(self):
        return dict(ipv4_cluster_mask=self.cluster_mask, ipv4_cluster_range=self.cluster_range,
                    policy_max_total=max(1 << 16, 2 * len(self.pol_keys)),
                    max_endpoints=max(64, self.n_endpoints))

    def oracle_config(self):
        return dict(ipv4_cluster_mask=self.cluster_mask, ipv4_cluster_range=self.cluster_range)


def make_tables(n_prefixes=10_000, n_identities=1000, n_endpoints=1, keys_per_ep=16_000,
                seed=SEED, **_):
    rng = np.random.Generator(np.random.PCG64(seed))
    idents = np.arange(256, 256 + n_identities, dtype=np.uint32)
    lens_c = np.array([8, 16, 20, 24, 28, 32])
    lens_p = np.array([0.02, 0.08, 0.10, 0.55, 0.10, 0.15])
    # draw extra, dedupe on (len, masked address), keep n_prefixes
    m = int(n_prefixes * 1.3) + 64
    ln = rng.choice(lens_c, m, p=lens_p).astype(np.uint64)
    addr = rng.integers(0, 2**32, m, dtype=np.uint64)
    # keep most prefixes outside the cluster /8 so fallbacks stay meaningful
    mask = np.where(ln == 0, 0, ((np.uint64(0xFFFFFFFF) << (np.uint64(32) - ln)) &
                                 np.uint64(0xFFFFFFFF)))
    addr = addr & mask
    uniq, first = np.unique((ln << np.uint64(32)) | addr, return_index=True)
    first = np.sort(first)[:n_prefixes]
    ln, addr = ln[first].astype(np.int64), addr[first].astype(np.uint32)
    labels = rng.choice(idents, len(ln)).astype(np.uint32)
    labels[rng.random(len(ln)) < 0.005] = 0  # tombstones

    recs = []  # (cidr base host-order, len, label)
    recs.append((0, 0, L.WORLD_ID))                          # 0.0.0.0/0 -> world
    recs.append((CLUSTER_V4 | (7 << 16), 16, L.CLUSTER_ID))  # cluster /16
    for h in range(4):
        recs.append((CLUSTER_V4 | (0xFF << 8) | (h + 1), 32, L.HOST_ID))
    n_res = len(recs)
    keys = np.zeros(n_res + len(ln), L.IPCACHE_KEY)
    vals = np.zeros(n_res + len(ln), L.REMOTE_ENDPOINT_INFO)
    all_addr = np.concatenate([np.array([r[0] for r in recs], np.uint32), addr])
    all_len = np.concatenate([np.array([r[1] for r in recs], np.int64), ln])
    all_lab = np.concatenate([np.array([r[2] for r in recs], np.uint32), labels])
    keys["prefixlen"] = L.IPCACHE_STATIC_PREFIX + all_len
    keys["family"] = L.ENDPOINT_KEY_IPV4
    keys["ip"][:, :4] = all_addr.astype(">u4").view(np.uint8).reshape(-1, 4)
    vals["sec_label"] = all_lab
    vals["tunnel_endpoint"] = rng.integers(0, 2**32, len(vals), dtype=np.uint64).astype(np.uint32)
    # dedupe reserved vs random collisions (keep the reserved entry)
    canon = (keys["prefixlen"].astype(np.uint64) << np.uint64(32)) | all_addr.astype(np.uint64)
    _, keep = np.unique(canon, return_index=True)
    keep = np.sort(keep)
    keys, vals = keys[keep], vals[keep]
    all_addr, all_len = all_addr[keep], all_len[keep]

    # policy MapState per endpoint
    pk, pe, pep = [], [], []
    for ep in range(n_endpoints):
        mm = int(keys_per_ep * 1.6) + 64
        kind = rng.choice(3, mm, p=[0.45, 0.45, 0.10])
        idn = rng.choice(idents, mm).astype(np.uint32)
        idn[kind == 2] = 0
        port = zipf_ports(rng, mm)
        proto = np.where(rng.random(mm) < 0.85, L.PROTO_TCP, L.PROTO_UDP).astype(np.uint8)
        port = np.where(kind == 1, 0, port).astype(np.uint16)
        proto = np.where(kind == 1, 0, proto).astype(np.uint8)
        egress = rng.integers(0, 2, mm).astype(np.uint8)
        k = np.zeros(mm, L.POLICY_KEY)
        k["sec_label"] = idn
        k["dport"] = port.byteswap()
        k["protocol"] = proto
        k["egress"] = egress
        # L3-only / wildcard keys saturate (2 x identities / 256 distinct):
        # top up with L4-exact keys until the endpoint holds keys_per_ep
        while True:
            _, idx = np.unique(k.view(np.uint64), return_index=True)
            if len(idx) >= keys_per_ep:
                break
            x = np.zeros(keys_per_ep, L.POLICY_KEY)
            x["sec_label"] = rng.choice(idents, keys_per_ep)
            x["dport"] = zipf_ports(rng, keys_per_ep).byteswap()
            x["protocol"] = np.where(rng.random(keys_per_ep) < 0.85, L.PROTO_TCP, L.PROTO_UDP)
            x["egress"] = rng.integers(0, 2, keys_per_ep)
            k = np.concatenate([k, x])
        idx = np.sort(idx)[:keys_per_ep]
        k = k[idx]
        e = np.zeros(len(k), L.POLICY_ENTRY)
        proxied = rng.random(len(k)) < 0.05
        e["proxy_port"] = np.where(proxied, rng.integers(10000, 20000, len(k)), 0).astype(
            np.uint16).byteswap()
        pk.append(k)
        pe.append(e)
        pep.append(np.full(len(k), ep, np.uint16))
    return Tables(keys, vals, all_addr, all_len, np.concatenate(pk), np.concatenate(pe),
                  np.concatenate(pep), n_endpoints)


def make_tuples(tables: Tables, n: int, seed=SEED, gpu_id: int = 0):
    """SoA tuple batch (numpy).  Addresses/dport in network byte order."""
    rng = np.random.Generator(np.random.PCG64(seed + gpu_id))
    npfx = len(tables.pfx_addr)

    def addrs():
        inside = rng.random(n) < 0.8
        pi = rng.integers(0, npfx, n)
        base = tables.pfx_addr[pi].astype(np.uint64)
        ln = tables.pfx_len[pi].astype(np.uint64)
        host = rng.integers(0, 2**32, n, dtype=np.uint64)
        hmask = (np.uint64(1) << (np.uint64(32) - ln)) - np.uint64(1)
        a = np.where(inside, base | (host & hmask), host).astype(np.uint32)
        return a.byteswap()  # host order -> network-order u32 as stored

    sa = addrs()
    da = addrs()
    egress = (rng.random(n) < 0.5).astype(np.uint8)
    frag = ((rng.random(n) < 0.005) & (egress == 0)).astype(np.uint8)
    # ports: mostly the MapState port set, some random
    port = np.where(rng.random(n) < 0.9, zipf_ports(rng, n),
                    rng.integers(1, 65536, n)).astype(np.uint16)
    proto = np.where(rng.random(n) < 0.85, L.PROTO_TCP, L.PROTO_UDP).astype(np.uint8)
    return {
        "saddr": sa,
        "daddr": da,
        "dport": port.byteswap(),
        "proto": proto,
        "flags": (egress | (frag << 1)).astype(np.uint8),
        "len": rng.integers(64, 1501, n).astype(np.uint32),
        "ep": rng.integers(0, tables.n_endpoints, n).astype(np.uint16),
    }


def load_engine(engine, t: Tables):
    rc = engine.ipcache_update_batch(t.ipc_keys, t.ipc_vals)
    assert rc == 0, rc
    rc = engine.policy_update_batch(t.pol_ep, t.pol_keys, t.pol_entries)
    assert rc == 0, rc


def load_oracle(oracle, t: Tables):
    for k, v in zip(t.ipc_keys, t.ipc_vals):
        assert oracle.ipcache_update(k, v) == 0
    for k, e, ep in zip(t.pol_keys, t.pol_entries, t.pol_ep):
        assert oracle.policy_update(int(ep), k, e) == 0


TUPLE_DTYPES = {"saddr": np.uint32, "daddr": np.uint32, "dport": np.uint16, "proto": np.uint8,
                "flags": np.uint8, "len": np.uint32, "ep": np.uint16, "sport": np.uint16,
                "hash": np.uint32, "l4b": np.uint16}


def to_device(t: dict, device="cuda"):
    """numpy SoA -> torch device tensors (bit-identical views).  IPv6
    address columns ((n, 16) uint8) stay uint8."""
    import torch
    view = {np.uint32: np.int32, np.uint16: np.int16, np.uint8: np.uint8}
    out = {}
    for k, dt in TUPLE_DTYPES.items():
        if k not in t:
            continue
        if k in ("saddr", "daddr") and np.asarray(t[k]).ndim == 2:
            a = np.ascontiguousarray(t[k], np.uint8)
        else:
            a = np.ascontiguousarray(t[k], dt).view(view[dt])
        out[k] = torch.from_numpy(a).to(device, non_blocking=False)
    return out


# ---------------------------------------------------------------------------
# services: VIPs in 100.64.0.0/10, 90% L4 (Zipf port
# set) / 10% L3 (dport 0) frontends, backends per service ~Geom(p=0.3) capped
# at 16, backend targets inside installed ipcache prefixes (so the post-DNAT
# identity is meaningful), 30% of backends on a different target port.
# Written as lbmap.UpdateService writes them: slave 0 = {count}, 1..n = backends.
# ---------------------------------------------------------------------------
@dataclass
class Services:
    keys: np.ndarray   # LB4_KEY
    vals: np.ndarray   # LB4_SERVICE
    vip: np.ndarray    # network-order u32 per service
    port: np.ndarray   # network-order u16 per service (0 = L3 service)


def make_services(tables: Tables, n_services: int, seed=SEED, max_backends=16, p=0.3,
                  l3_frac=0.1) -> Services:
    rng = np.random.Generator(np.random.PCG64(seed + 0x5E))
    host = rng.choice(1 << 22, n_services, replace=False).astype(np.uint32)
    vip = (np.uint32(0x64400000) | host).byteswap()        # 100.64.0.0/10
    port = np.where(rng.random(n_services) < l3_frac, 0,
                    zipf_ports(rng, n_services)).astype(np.uint16).byteswap()
    nb = np.minimum(rng.geometric(p, n_services), max_backends).astype(np.int64)
    nbt = int(nb.sum())
    keys = np.zeros(n_services + nbt, L.LB4_KEY)
    vals = np.zeros(n_services + nbt, L.LB4_SERVICE)
    keys["address"][:n_services] = vip
    keys["dport"][:n_services] = port
    vals["count"][:n_services] = nb
    svc = np.repeat(np.arange(n_services), nb)
    first = np.repeat(np.cumsum(nb) - nb, nb)
    slave = np.arange(nbt) - first + 1
    kb, vb = keys[n_services:], vals[n_services:]
    kb["address"] = vip[svc]
    kb["dport"] = port[svc]
    kb["slave"] = slave
    pi = rng.integers(0, len(tables.pfx_addr), nbt)
    ln = tables.pfx_len[pi].astype(np.uint64)
    hmask = (np.uint64(1) << (np.uint64(32) - ln)) - np.uint64(1)
    tgt = (tables.pfx_addr[pi].astype(np.uint64) |
           (rng.integers(0, 2**32, nbt, dtype=np.uint64) & hmask)).astype(np.uint32)
    vb["target"] = tgt.byteswap()
    svc_port = port[svc]
    other = rng.integers(1024, 65536, nbt).astype(np.uint16).byteswap()
    vb["port"] = np.where(rng.random(nbt) < 0.3, other, svc_port)
    vb["rev_nat_index"] = ((svc % 65535) + 1).astype(np.uint16).byteswap()
    vb["weight"] = np.uint16(1).byteswap()
    return Services(keys, vals, vip, port)


def add_service_traffic(t: dict, svcs: Services, frac=0.3, seed=SEED, gpu_id: int = 0):
    """sport + hash columns, and `frac` of the egress tuples aimed at a
    service (daddr = VIP, dport = its port, or any port for L3 services)."""
    from .shard import flowhash_np
    rng = np.random.Generator(np.random.PCG64(seed + 0x77 + gpu_id))
    n = len(t["saddr"])
    t = dict(t)
    t["sport"] = rng.integers(1024, 65536, n).astype(np.uint16).byteswap()
    hit = ((t["flags"] & 1) == 1) & (rng.random(n) < frac)
    si = rng.integers(0, len(svcs.vip), n)
    t["daddr"] = np.where(hit, svcs.vip[si], t["daddr"]).astype(np.uint32)
    t["dport"] = np.where(hit & (svcs.port[si] != 0), svcs.port[si], t["dport"]).astype(np.uint16)
    t["hash"] = flowhash_np(t["saddr"], t["daddr"], t["sport"], t["dport"], t["proto"])
    return t


def load_services(target, svcs: Services):
    """Engine (cgpu_lb4_update_batch) or Oracle (or_lb_update_many)."""
    if hasattr(target, "lb4_update_batch"):
        rc = target.lb4_update_batch(svcs.keys, svcs.vals)
    else:
        rc = target.lb_update_batch(svcs.keys, svcs.vals)
    assert rc == 0, rc


# ---------------------------------------------------------------------------
# config 5's first stage (BASELINE "prefilter -> ipcache -> policy -> LB"):
# the netdev's XDP CIDR prefilter (bpf_xdp.c check_v4) over an IPv4 deny set
# -- dyn4 LPM prefixes /16../28 (pkg/policy/prefilter.go maxLKeys 64k: 16k
# here) and fix4 /32s (maxHKeys 20M: 200k here), 5 % of each drawn inside
# installed ipcache prefixes (part of a remote identity's range denied), the
# rest uniform -- and the node's local endpoints in cilium_lxc (one IPv4 address
# per endpoint id, in the cluster range 10.0.0.0/8), which check_v4_endpoint
# requires of every ingress daddr.
# ---------------------------------------------------------------------------
@dataclass
class Prefilter4:
    dyn4: np.ndarray     # LPM_V4_KEY
    fix4: np.ndarray     # LPM_V4_KEY, prefixlen 32
    ep_addr: np.ndarray  # network-order u32 per endpoint id
    ep_keys: np.ndarray  # ENDPOINT_KEY (cilium_lxc)


def _lpm4_keys(addr_host, plen):
    k = np.zeros(len(addr_host), L.LPM_V4_KEY)
    k["prefixlen"] = plen
    k["addr"] = addr_host.astype(">u4").view(np.uint8).reshape(-1, 4)
    return k


def make_prefilter4(tables: Tables, n_dyn=16_000, n_fix=200_000, seed=SEED) -> Prefilter4:
    rng = np.random.Generator(np.random.PCG64(seed + 0x9F4))
    npfx = len(tables.pfx_addr)

    def draw(n, lens):
        # a deny prefix inside an installed ipcache prefix is no wider than
        # it (lens raised in place), so it blocks part of one identity's range
        inside = rng.random(n) < 0.05
        pi = rng.integers(0, npfx, n)
        ln = tables.pfx_len[pi].astype(np.uint64)
        hmask = (np.uint64(1) << (np.uint64(32) - ln)) - np.uint64(1)
        a = np.where(inside, tables.pfx_addr[pi].astype(np.uint64) |
                     (rng.integers(0, 2**32, n, dtype=np.uint64) & hmask),
                     rng.integers(0, 2**32, n, dtype=np.uint64))
        lens[:] = np.where(inside, np.maximum(lens, ln.astype(lens.dtype)), lens)
        m = ((np.uint64(0xFFFFFFFF) << (np.uint64(32) - lens.astype(np.uint64))) & np.uint64(0xFFFFFFFF))
        return (a & m).astype(np.uint32)

    # keep the cluster /8 (the endpoints' range) out of the deny set
    lens = rng.choice(np.array([16, 20, 24, 28]), int(n_dyn * 1.2) + 16, p=[0.05, 0.15, 0.6, 0.2])
    da = draw(len(lens), lens)
    ok = (da >> 24) != (CLUSTER_V4 >> 24)
    key = (lens.astype(np.uint64) << np.uint64(32)) | da.astype(np.uint64)
    _, first = np.unique(key, return_index=True)
    first = np.sort(first[ok[first]])[:n_dyn]
    dyn = _lpm4_keys(da[first], lens[first])
    fa = draw(int(n_fix * 1.2) + 16, np.full(int(n_fix * 1.2) + 16, 32))
    fa = fa[(fa >> 24) != (CLUSTER_V4 >> 24)]
    _, first = np.unique(fa, return_index=True)
    fa = fa[np.sort(first)][:n_fix]
    fix = _lpm4_keys(fa, 32)
    ep_host = (CLUSTER_V4 | (0x42 << 16) | (np.arange(max(tables.n_endpoints, 1)) + 2)).astype(np.uint32)
    ep_keys = np.zeros(len(ep_host), L.ENDPOINT_KEY)
    ep_keys["ip"][:, :4] = ep_host.astype(">u4").view(np.uint8).reshape(-1, 4)
    ep_keys["family"] = L.ENDPOINT_KEY_IPV4
    return Prefilter4(dyn, fix, ep_host.byteswap(), ep_keys)


def add_prefilter_traffic(t: dict, P: Prefilter4, seed=SEED, gpu_id: int = 0, deny_frac=0.05,
                          stray_frac=0.01):
    """Ingress tuples as the netdev hands them to XDP: daddr = the address
    of the endpoint whose policy map (ep) classifies them, except
    `stray_frac` aimed at no local endpoint (check_v4_endpoint drops them);
    `deny_frac` of them come from a deny-set address (half a dyn4 prefix,
    half a fix4 /32).  Egress tuples are left as they are."""
    rng = np.random.Generator(np.random.PCG64(seed + 0xD4 + gpu_id))
    n = len(t["saddr"])
    t = dict(t)
    ing = (t["flags"] & 1) == 0
    stray = rng.random(n) < stray_frac
    t["daddr"] = np.where(ing & ~stray, P.ep_addr[t["ep"] % len(P.ep_addr)], t["daddr"]).astype(np.uint32)
    deny = ing & (rng.random(n) < deny_frac)
    use_dyn = rng.random(n) < 0.5
    di = rng.integers(0, len(P.dyn4), n)
    dbase = P.dyn4["addr"][di].copy().view(">u4").ravel().astype(np.uint64)
    dlen = P.dyn4["prefixlen"][di].astype(np.uint64)
    dhost = rng.integers(0, 2**32, n, dtype=np.uint64) & ((np.uint64(1) << (np.uint64(32) - dlen)) - np.uint64(1))
    fi = rng.integers(0, len(P.fix4), n)
    fbase = P.fix4["addr"][fi].copy().view(">u4").ravel().astype(np.uint64)
    src = np.where(use_dyn, dbase | dhost, fbase).astype(np.uint32).byteswap()
    t["saddr"] = np.where(deny, src, t["saddr"]).astype(np.uint32)
    if "hash" in t:
        from .shard import flowhash_np
        t["hash"] = flowhash_np(t["saddr"], t["daddr"], t["sport"], t["dport"], t["proto"])
    return t


def load_prefilter4(target, P: Prefilter4):
    """Engine or Oracle: dyn4 / fix4 CIDR maps (pkg/maps/cidrmap) + cilium_lxc."""
    for which, keys in ((0, P.dyn4), (1, P.fix4)):
        if hasattr(target, "cidr_update_batch"):
            rc = target.cidr_update_batch(which, keys)
            assert rc == 0, rc
            continue
        for k in keys:
            rc = target.cidr_update(which, k)
            assert rc == 0, rc
    for k in P.ep_keys:
        rc = target.endpoint_update(k)
        assert rc == 0, rc


def make_services6(tables, n_services: int, seed=SEED, max_backends=16, p=0.3, l3_frac=0.1):
    """make_services for cilium_lb6_services: VIPs in fd00:96::/32, backend
    targets inside the installed IPv6 ipcache prefixes (tables: Tables6).
    -> Services with LB6_KEY / LB6_SERVICE records and vip (n, 16) uint8."""
    rng = np.random.Generator(np.random.PCG64(seed + 0x5F))
    vip = rng.integers(0, 256, (n_services, 16), dtype=np.uint8)
    vip[:, :4] = [0xFD, 0x00, 0x00, 0x96]
    vip[:, 4:8] = np.arange(n_services, dtype=np.uint32).view(np.uint8).reshape(-1, 4)  # distinct
    port = np.where(rng.random(n_services) < l3_frac, 0,
                    zipf_ports(rng, n_services)).astype(np.uint16).byteswap()
    nb = np.minimum(rng.geometric(p, n_services), max_backends).astype(np.int64)
    nbt = int(nb.sum())
    keys = np.zeros(n_services + nbt, L.LB6_KEY)
    vals = np.zeros(n_services + nbt, L.LB6_SERVICE)
    keys["address"][:n_services] = vip
    keys["dport"][:n_services] = port
    vals["count"][:n_services] = nb
    svc = np.repeat(np.arange(n_services), nb)
    first = np.repeat(np.cumsum(nb) - nb, nb)
    kb, vb = keys[n_services:], vals[n_services:]
    kb["address"] = vip[svc]
    kb["dport"] = port[svc]
    kb["slave"] = np.arange(nbt) - first + 1
    pi = rng.integers(0, len(tables.pfx_len), nbt)
    mk = MASK6[tables.pfx_len[pi]]
    vb["target"] = (tables.pfx_addr[pi] & mk) | (rng.integers(0, 256, (nbt, 16), dtype=np.uint8) & ~mk)
    other = rng.integers(1024, 65536, nbt).astype(np.uint16).byteswap()
    vb["port"] = np.where(rng.random(nbt) < 0.3, other, port[svc])
    vb["rev_nat_index"] = ((svc % 65535) + 1).astype(np.uint16).byteswap()
    vb["weight"] = np.uint16(1).byteswap()
    return Services(keys, vals, vip, port)


def add_service_traffic6(t: dict, svcs: Services, frac=0.3, seed=SEED, gpu_id: int = 0):
    """add_service_traffic for IPv6 tuples (hash = cgpu_flow_hash6)."""
    from .shard import flowhash6_np
    rng = np.random.Generator(np.random.PCG64(seed + 0x78 + gpu_id))
    n = len(t["flags"])
    t = dict(t)
    t["sport"] = rng.integers(1024, 65536, n).astype(np.uint16).byteswap()
    hit = ((t["flags"] & 1) == 1) & (rng.random(n) < frac)
    si = rng.integers(0, len(svcs.vip), n)
    t["daddr"] = np.where(hit[:, None], svcs.vip[si], t["daddr"]).astype(np.uint8)
    t["dport"] = np.where(hit & (svcs.port[si] != 0), svcs.port[si], t["dport"]).astype(np.uint16)
    t["hash"] = flowhash6_np(t["saddr"], t["daddr"], t["sport"], t["dport"], t["proto"])
    return t


def load_services6(target, svcs: Services):
    """Engine (cgpu_lb6_update_batch) or Oracle (or_lb6_update)."""
    rc = target.lb6_update_batch(svcs.keys, svcs.vals)
    assert rc == 0, rc


# ---------------------------------------------------------------------------
# IPv6 classify at config-2 size (ipcache_lookup6 of
# bpf/lib/eps.h:56-66 behind bpf_lxc.c:170-187 / bpf_netdev.c:203-211):
# 100k IPv6 ipcache prefixes laid out like a dual-stack cluster's ipcache --
# 1024 /48 sites under 64 /16 roots; /128 40% (pod and node addresses), /64
# 30% (node pod CIDRs), /56 10%, /48 7%, /96 5%, /112 5%, /32 3% (CIDR
# policy) -- plus ::/0 -> WORLD and 4 HOST /128s, and the config-2 MapState
# (4 endpoints x 16k keys).  Tuples: 80% inside an installed prefix, 20%
# random under a root; the rest as make_tuples.
# ---------------------------------------------------------------------------
V6_LENS = np.array([32, 48, 56, 64, 96, 112, 128])
V6_LENS_P = np.array([0.03, 0.07, 0.10, 0.30, 0.05, 0.05, 0.40])
# MASK6[L] = the 16 network-order bytes of a /L netmask
MASK6 = np.packbits((np.arange(128)[None, :] < np.arange(129)[:, None]).astype(np.uint8), axis=1)


@dataclass
class Tables6:
    ipc_keys: np.ndarray      # IPCACHE_KEY (family 2)
    ipc_vals: np.ndarray
    pfx_addr: np.ndarray      # (n, 16) uint8 masked base of every non-reserved prefix
    pfx_len: np.ndarray
    roots: np.ndarray         # (n_roots, 2) uint8
    router: bytes             # ROUTER_IP (16 bytes; its /64 is the cluster test)
    pol_keys: np.ndarray
    pol_entries: np.ndarray
    pol_ep: np.ndarray
    n_endpoints: int

    def engine_config(self):
        return dict(ipv6_router_ip=self.router,
                    policy_max_total=max(1 << 16, 2 * len(self.pol_keys)),
                    max_endpoints=max(64, self.n_endpoints))

    def oracle_config(self):
        return dict(router_ip=self.router)


def make_tables6(n_prefixes=100_000, n_identities=1000, n_endpoints=4, keys_per_ep=16_000,
                 seed=SEED, n_roots=64, n_sites=1024, **_):
    T = make_tables(n_prefixes=16, n_identities=n_identities, n_endpoints=n_endpoints,
                    keys_per_ep=keys_per_ep, seed=seed)  # the MapState (same as config 2)
    rng = np.random.Generator(np.random.PCG64(seed + 0x6C))
    idents = np.arange(256, 256 + n_identities, dtype=np.uint32)
    roots = rng.integers(0, 256, (n_roots, 2), dtype=np.uint8)
    sites = rng.integers(0, 256, (n_sites, 16), dtype=np.uint8)
    sites[:, :2] = roots[rng.integers(0, n_roots, n_sites)]
    m = int(n_prefixes * 1.2) + 64
    ln = rng.choice(V6_LENS, m, p=V6_LENS_P)
    a = rng.integers(0, 256, (m, 16), dtype=np.uint8)
    a[:, :6] = sites[rng.integers(0, n_sites, m), :6]
    a &= MASK6[ln]
    rec = np.zeros(m, np.dtype([("len", "u1"), ("a", "u1", (16,))]))
    rec["len"], rec["a"] = ln, a
    _, first = np.unique(rec.view(np.dtype((np.void, 17))), return_index=True)
    first = np.sort(first)[:n_prefixes]
    ln, a = ln[first], a[first]
    labels = rng.choice(idents, len(ln)).astype(np.uint32)
    labels[rng.random(len(ln)) < 0.005] = 0  # tombstones
    hosts = sites[:4].copy()
    hosts[:, 8:] = rng.integers(0, 256, (4, 8), dtype=np.uint8)
    r_addr = np.concatenate([np.zeros((1, 16), np.uint8), hosts])
    r_len = np.array([0, 128, 128, 128, 128])
    r_lab = np.array([L.WORLD_ID] + [L.HOST_ID] * 4, np.uint32)
    keys = np.zeros(len(r_len) + len(ln), L.IPCACHE_KEY)
    vals = np.zeros(len(keys), L.REMOTE_ENDPOINT_INFO)
    keys["family"] = L.ENDPOINT_KEY_IPV6
    keys["prefixlen"] = L.IPCACHE_STATIC_PREFIX + np.concatenate([r_len, ln])
    keys["ip"] = np.concatenate([r_addr, a])
    vals["sec_label"] = np.concatenate([r_lab, labels])
    vals["tunnel_endpoint"] = rng.integers(0, 2**32, len(vals), dtype=np.uint64).astype(np.uint32)
    canon = np.zeros(len(keys), np.dtype([("len", "u1"), ("a", "u1", (16,))]))
    canon["len"], canon["a"] = keys["prefixlen"], keys["ip"]
    _, keep = np.unique(canon.view(np.dtype((np.void, 17))), return_index=True)
    keep = np.sort(keep)
    keys, vals = keys[keep], vals[keep]
    router = bytes(sites[5, :8]) + bytes(rng.integers(0, 256, 8, dtype=np.uint8))
    return Tables6(keys, vals, a, ln, roots, router, T.pol_keys, T.pol_entries, T.pol_ep,
                   n_endpoints)


def make_tuples6(tables: Tables6, n: int, seed=SEED, gpu_id: int = 0, chunk=1 << 22):
    """SoA IPv6 tuple batch: saddr / daddr (n, 16) uint8, the rest as make_tuples."""
    rng = np.random.Generator(np.random.PCG64(seed + 0x600 + gpu_id))
    npfx = len(tables.pfx_len)

    def addrs(m):
        inside = rng.random(m) < 0.8
        pi = rng.integers(0, npfx, m)
        mk = MASK6[tables.pfx_len[pi]]
        r = rng.integers(0, 256, (m, 16), dtype=np.uint8)
        out = (tables.pfx_addr[pi] & mk) | (r & ~mk)
        rr = ~inside
        out[rr] = r[rr]
        out[rr, :2] = tables.roots[rng.integers(0, len(tables.roots), int(rr.sum()))]
        return out

    sa = np.empty((n, 16), np.uint8)
    da = np.empty((n, 16), np.uint8)
    for lo in range(0, n, chunk):
        hi = min(n, lo + chunk)
        sa[lo:hi] = addrs(hi - lo)
        da[lo:hi] = addrs(hi - lo)
    egress = (rng.random(n) < 0.5).astype(np.uint8)
    port = np.where(rng.random(n) < 0.9, zipf_ports(rng, n),
                    rng.integers(1, 65536, n)).astype(np.uint16)
    proto = np.where(rng.random(n) < 0.85, L.PROTO_TCP, L.PROTO_UDP).astype(np.uint8)
    return {
        "saddr": sa, "daddr": da, "dport": port.byteswap(), "proto": proto,
        "flags": egress, "len": rng.integers(64, 1501, n).astype(np.uint32),
        "ep": rng.integers(0, tables.n_endpoints, n).astype(np.uint16),
    }


# ---------------------------------------------------------------------------
# config 3: XDP IPv6 prefilter, 1M deny prefixes with lengths
# /32 5%, /48 45%, /56 20%, /64 20%, /128 10% (the /128s go to the "fix" hash,
# the rest to the "dyn" LPM), under 256 random /24 roots; 4k local endpoint
# IPs; packets 50% sourced inside a deny prefix, 30% addressed to an endpoint.
# ---------------------------------------------------------------------------
PF6_CONFIG = dict(n_prefixes=1_000_000, n_roots=256, n_endpoints=4096)


@dataclass
class Prefilter6:
    dyn6: np.ndarray    # LPM_V6_KEY
    fix6: np.ndarray    # LPM_V6_KEY, prefixlen 128
    ep6: np.ndarray     # ENDPOINT_KEY (family 2)
    roots: np.ndarray   # (n_roots, 3) uint8

    def engine_config(self):
        return dict(cidr_dyn_max=max(1 << 20, len(self.dyn6)),
                    cidr_fix_max=max(1 << 20, len(self.fix6)),
                    endpoints_max=max(65536, len(self.ep6)))

    def oracle_config(self):
        return {}


def make_prefilter6(n_prefixes=1_000_000, n_roots=256, n_endpoints=4096, seed=SEED, **_):
    rng = np.random.Generator(np.random.PCG64(seed + 0x36))
    roots = rng.integers(0, 256, (n_roots, 3), dtype=np.uint8)
    m = int(n_prefixes * 1.05) + 16
    ln = rng.choice(np.array([32, 48, 56, 64, 128]), m, p=[0.05, 0.45, 0.20, 0.20, 0.10])
    a = rng.integers(0, 256, (m, 16), dtype=np.uint8)
    a[:, :3] = roots[rng.integers(0, n_roots, m)]
    # canonical (masked) prefixes, deduplicated on (len, masked address)
    bits = np.unpackbits(a, axis=1)
    bits[np.arange(128)[None, :] >= ln[:, None]] = 0
    a = np.packbits(bits, axis=1)
    rec = np.zeros(m, np.dtype([("len", "u1"), ("a", "u1", (16,))]))
    rec["len"], rec["a"] = ln, a
    _, first = np.unique(rec.view(np.dtype((np.void, 17))), return_index=True)
    first = np.sort(first)[:n_prefixes]
    ln, a = ln[first], a[first]
    keys = np.zeros(len(ln), L.LPM_V6_KEY)
    keys["prefixlen"] = ln
    keys["addr"] = a
    fix = ln == 128
    ep_a = rng.integers(0, 256, (n_endpoints, 16), dtype=np.uint8)
    ep_a[:, :3] = roots[rng.integers(0, n_roots, n_endpoints)]
    ep = np.zeros(n_endpoints, L.ENDPOINT_KEY)
    ep["ip"] = ep_a
    ep["family"] = L.ENDPOINT_KEY_IPV6
    return Prefilter6(keys[~fix], keys[fix], ep, roots)


def make_packets6(P: Prefilter6, n: int, seed=SEED, gpu_id: int = 0, chunk=1 << 22):
    rng = np.random.Generator(np.random.PCG64(seed + 0x66 + gpu_id))
    allk = np.concatenate([P.dyn6, P.fix6])
    sa = np.empty((n, 16), np.uint8)
    da = np.empty((n, 16), np.uint8)
    for lo in range(0, n, chunk):
        hi = min(n, lo + chunk)
        m = hi - lo
        s = rng.integers(0, 256, (m, 16), dtype=np.uint8)
        inside = rng.random(m) < 0.5
        k = allk[rng.integers(0, len(allk), m)]
        bits = np.unpackbits(s, axis=1)
        kb = np.unpackbits(np.ascontiguousarray(k["addr"]), axis=1)
        keep = np.arange(128)[None, :] < k["prefixlen"][:, None].astype(np.int64)
        bits = np.where(inside[:, None] & keep, kb, bits)
        s = np.packbits(bits, axis=1)
        outside = ~inside
        s[outside, :3] = P.roots[rng.integers(0, len(P.roots), int(outside.sum()))]
        sa[lo:hi] = s
        d = rng.integers(0, 256, (m, 16), dtype=np.uint8)
        to_ep = rng.random(m) < 0.3
        d[to_ep] = P.ep6["ip"][rng.integers(0, len(P.ep6), int(to_ep.sum()))]
        da[lo:hi] = d
    return {"saddr": sa, "daddr": da, "flags": np.zeros(n, np.uint8)}


def load_prefilter6(target, P: Prefilter6):
    """Engine or Oracle: dyn6 / fix6 CIDR maps (pkg/maps/cidrmap) + cilium_lxc."""
    for which, keys in ((2, P.dyn6), (3, P.fix6)):
        if hasattr(target, "cidr_update_batch"):
            rc = target.cidr_update_batch(which, keys)
            assert rc == 0, rc
            continue
        for k in keys:
            rc = target.cidr_update(which, k)
            assert rc == 0, rc
    for k in P.ep6:
        rc = target.endpoint_update(k)
        assert rc == 0, rc


def packets6_to_device(p: dict, device="cuda"):
    import torch
    return {k: torch.from_numpy(np.ascontiguousarray(v, np.uint8)).to(device)
            for k, v in p.items()}


# ---------------------------------------------------------------------------
# raw Ethernet frames
# ---------------------------------------------------------------------------
# The endpoint identity of the reference's bpf/lxc_config.h (LXC_MAC, LXC_IPV4
# as the raw u32 the program compares, LXC_IP) -- what the golden harness is
# compiled with, and what the tests install through cgpu_lxc_update.
LXC_MAC = bytes([0xaa, 0xbb, 0xcc, 0xdd, 0xee, 0xff])
LXC_IPV4_RAW = 0x10203040
LXC_IP6 = bytes([0xbe, 0xef, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0x1, 0x1, 0x65, 0x82, 0xbc])

ICMP4_TYPES = np.array([0, 8, 8, 3, 11, 12, 5, 13, 0, 8], np.uint8)
ICMP6_TYPES = np.array([128, 128, 129, 1, 2, 3, 4, 135, 136, 128], np.uint8)
V4_PROTOS = np.array([6, 6, 6, 6, 17, 17, 17, 1, 1, 58, 132, 47, 0], np.uint8)
V6_PROTOS = np.array([6, 6, 6, 17, 17, 58, 58, 132, 47], np.uint8)
FRAG_OFFS = np.array([0, 0, 0, 0, 0, 0, 0x4000, 0x4000, 0x2000, 0x0001, 0x8000, 0xC000,
                      0x4001, 0x1fff], np.uint16)
EXT_TYPES = np.array([0, 43, 60, 51, 0, 43, 60, 51, 44, 59], np.uint8)


def _put(D, rows, off, vals):
    """D[rows, off + j] = vals[:, j] for variable per-row offsets (clipped to
    the buffer width: bytes past the slot are not stored)."""
    if len(rows) == 0:
        return
    vals = np.asarray(vals, np.uint8).reshape(len(rows), -1)
    cols = np.asarray(off, np.int64).reshape(-1, 1) + np.arange(vals.shape[1])
    ok = cols < D.shape[1]
    r = np.broadcast_to(np.asarray(rows).reshape(-1, 1), cols.shape)
    D[r[ok], cols[ok]] = vals[ok]


def _be16(x):
    x = np.asarray(x, np.uint16)
    return np.stack([x >> 8, x & 0xff], 1).astype(np.uint8)


# ROUTER_IP of the endpoint programs' build (bpf/node_config.h:30), the
# engine's and the restatement's default
ROUTER_IP6 = bytes([0xbe, 0xef, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 0, 1, 0, 0])


def make_frames(rng, n: int, width: int = 256, n_ep: int = 5, addr4=None, edge: bool = True):
    """Diverse Ethernet frames for the frame-path parity tests (vectorized).

    Mix: IPv4 (options, ihl < 5, every frag_off class, TCP/UDP/ICMP/other,
    ICMP types), IPv6 (0-5 extension headers incl. FRAGMENT / NONE / AUTH),
    ARP, other ethertypes; egress frames mostly carry the endpoint's MAC /
    address (LXC_* above) with some corrupted; 20% truncated at a random
    length (edge=True also makes frames shorter than an Ethernet header).
    Returns dict data (n, width) u8, len u32, flags u8 (egress bit), ep u16;
    len may exceed what a narrower slot stores.  addr4: optional pool of
    network-order u32 addresses to draw v4 addresses from.
    """
    D = rng.integers(0, 256, (n, width), dtype=np.uint8)
    egress = rng.random(n) < 0.5
    p = [0.58, 0.28, 0.07, 0.07] if edge else [0.8, 0.2, 0.0, 0.0]
    kind = rng.choice(4, n, p=p)
    full = np.zeros(n, np.int64)
    # Ethernet: egress frames address the gateway from the endpoint's MAC
    ok_d = egress & (rng.random(n) < 0.95)
    ok_s = egress & (rng.random(n) < 0.95)
    D[ok_d, 0:6] = np.frombuffer(L.NODE_MAC, np.uint8)
    D[ok_s, 6:12] = np.frombuffer(LXC_MAC, np.uint8)
    other = np.array([0x88cc, 0x8100, 0x0000, 0x86dc, 0x0801, 0xdd86], np.uint16)
    et = np.select([kind == 0, kind == 1, kind == 2], [0x0800, 0x86DD, 0x0806],
                   rng.choice(other, n).astype(np.int64)).astype(np.uint16)
    D[:, 12:14] = _be16(et)
    full[kind >= 2] = 14 + 28

    def addr4_draw(m):
        if addr4 is not None and len(addr4):
            a = rng.choice(np.asarray(addr4, np.uint32), m)
            return np.where(rng.random(m) < 0.8, a, rng.integers(0, 2**32, m, dtype=np.uint64)
                            ).astype(np.uint32)
        return rng.integers(0, 2**32, m, dtype=np.uint64).astype(np.uint32)

    def l4(rows, off, proto, v6):
        """TCP 20 / UDP 8 / ICMP 8 / other 8 bytes at `off`; returns the length."""
        m = len(rows)
        ln = np.full(m, 8, np.int64)
        sport = rng.integers(1, 65536, m).astype(np.uint16)
        dport = np.where(rng.random(m) < 0.8, rng.choice(PORTS64, m),
                         rng.integers(0, 65536, m)).astype(np.uint16)
        hdr = rng.integers(0, 256, (m, 20), dtype=np.uint8)
        tcpudp = (proto == 6) | (proto == 17)
        hdr[tcpudp, 0:2] = _be16(sport[tcpudp])
        hdr[tcpudp, 2:4] = _be16(dport[tcpudp])
        icmp = proto == (58 if v6 else 1)
        hdr[icmp, 0] = rng.choice(ICMP6_TYPES if v6 else ICMP4_TYPES, int(icmp.sum()))
        ln[proto == 6] = 20
        _put(D, rows, off, hdr)
        return ln

    # ---- IPv4
    r4 = np.flatnonzero(kind == 0)
    m = len(r4)
    ihl = np.where(rng.random(m) < 0.82, 5, np.where(rng.random(m) < 0.6,
                                                      rng.integers(6, 16, m), rng.integers(0, 5, m)))
    proto = rng.choice(V4_PROTOS, m)
    sa = addr4_draw(m)
    lxc_src = egress[r4] & (rng.random(m) < 0.9)
    sa = np.where(lxc_src, np.uint32(LXC_IPV4_RAW), sa).astype(np.uint32)  # stored (raw) u32
    da = addr4_draw(m)
    D[r4, 14] = (0x40 | ihl).astype(np.uint8)
    D[r4, 20:22] = _be16(rng.choice(FRAG_OFFS, m))
    D[r4, 23] = proto
    D[r4, 26:30] = sa.view(np.uint8).reshape(m, 4)
    D[r4, 30:34] = da.view(np.uint8).reshape(m, 4)
    off = 14 + 4 * ihl
    has_l4 = ihl >= 5  # shorter headers leave the reference reading the IP header as L4
    ln = np.full(m, 8, np.int64)
    ln[has_l4] = l4(r4[has_l4], off[has_l4], proto[has_l4], False)
    full[r4] = np.maximum(off, 34) + ln

    # ---- IPv6
    r6 = np.flatnonzero(kind == 1)
    m = len(r6)
    proto = rng.choice(V6_PROTOS, m)
    next_chain = np.where(rng.random(m) < 0.6, 0, rng.integers(1, 6, m))
    chain = rng.choice(EXT_TYPES, (m, 6))
    D[r6, 14] = 0x60
    sa6 = rng.integers(0, 256, (m, 16), dtype=np.uint8)
    sa6[egress[r6] & (rng.random(m) < 0.9)] = np.frombuffer(LXC_IP6, np.uint8)
    D[r6, 22:38] = sa6
    first = np.where(next_chain > 0, chain[:, 0], proto)
    D[r6, 20] = first
    off = np.full(m, 54, np.int64)
    cur = first.copy()
    live = next_chain > 0
    for j in range(6):
        rows = np.flatnonzero(live)
        if len(rows) == 0:
            break
        nxt = np.where(j + 1 < next_chain[rows], chain[rows, min(j + 1, 5)], proto[rows])
        hl = rng.integers(0, 3, len(rows))
        _put(D, r6[rows], off[rows], np.stack([nxt, hl], 1))
        # advance as ipv6_hdrlen does (the AUTH rule keys on the NEXT header)
        step = np.where(nxt == 51, (hl + 2) << 2, (hl + 1) << 3)
        stop = (cur[rows] == 44) | (cur[rows] == 59)
        off[rows] += np.where(stop, 0, step)
        cur[rows] = nxt
        live[rows] = (j + 1 < next_chain[rows]) & ~stop
    ln = l4(r6, off, proto, True)
    full[r6] = off + ln

    full += rng.integers(0, 24, n)  # payload
    lens = np.minimum(full, 65535)
    trunc = rng.random(n) < 0.2
    lo = np.where(edge, 0, 14)
    lens[trunc] = rng.integers(lo, np.maximum(full[trunc], lo + 1))
    ep = rng.integers(0, n_ep, n).astype(np.uint16)
    # handle_ipv6's ICMPv6 responders (bpf_lxc.c:364-389, lib/icmp6.h):
    # neighbour solicitations for the router and for other targets, echo
    # requests to the router, at lengths around the responders' reads
    # (icmp6hdr 62, ND target 78, ND option 86); drawn last, so the frames
    # above stay as they were
    icmp6 = r6[(next_chain == 0) & (proto == 58)]
    pick = icmp6[rng.random(len(icmp6)) < 0.5]
    m = len(pick)
    ns = rng.random(m) < 0.6
    D[pick[ns], 54] = 135
    tgt = rng.integers(0, 256, (int(ns.sum()), 16), dtype=np.uint8)
    tgt[rng.random(int(ns.sum())) < 0.5] = np.frombuffer(ROUTER_IP6, np.uint8)
    if width >= 78:
        D[pick[ns], 62:78] = tgt
    D[pick[~ns], 54] = 128
    D[pick[~ns], 38:54] = np.frombuffer(ROUTER_IP6, np.uint8)
    lens[pick] = rng.integers(56, 100, m)
    return {"data": D, "len": lens.astype(np.uint32), "flags": egress.astype(np.uint8), "ep": ep}


def frames_from_tuples(t: dict, stride: int = 64, seed=SEED):
    """The IPv4 tuples of make_tuples as Ethernet frames: IPv4 without
    options, TCP (20 B) / UDP (8 B) header, MF set on fragments, the tuple's
    len as the wire length.  Every frame reaches policy with the tuple it
    came from (classify_frames == classify_v4 on TCP/UDP tuples)."""
    n = len(t["saddr"])
    rng = np.random.Generator(np.random.PCG64(seed ^ 0xF4A3E))
    D = np.zeros((n, stride), np.uint8)
    D[:, 0:6] = np.frombuffer(L.NODE_MAC, np.uint8)
    D[:, 6:12] = np.frombuffer(LXC_MAC, np.uint8)
    D[:, 12] = 0x08
    D[:, 14] = 0x45
    frag = (np.asarray(t["flags"]) >> 1) & 1
    D[:, 20] = np.where(frag == 1, 0x20, 0x00)
    D[:, 22] = 64
    D[:, 23] = t["proto"]
    D[:, 26:30] = np.ascontiguousarray(t["saddr"], np.uint32).view(np.uint8).reshape(n, 4)
    D[:, 30:34] = np.ascontiguousarray(t["daddr"], np.uint32).view(np.uint8).reshape(n, 4)
    D[:, 34:36] = _be16(rng.integers(1024, 65536, n))
    D[:, 36:38] = np.ascontiguousarray(t["dport"], np.uint16).view(np.uint8).reshape(n, 2)
    tcp = np.asarray(t["proto"]) == 6
    D[tcp, 46] = 0x50
    D[tcp, 47] = 0x10
    return {"data": D, "len": np.asarray(t["len"], np.uint32).copy(),
            "flags": (np.asarray(t["flags"]) & 1).astype(np.uint8),
            "ep": np.asarray(t["ep"], np.uint16).copy()}


def frames_to_device(f: dict, device="cuda"):
    import torch
    return {"data": torch.from_numpy(np.ascontiguousarray(f["data"])).to(device),
            "len": torch.from_numpy(np.ascontiguousarray(f["len"], np.uint32).view(np.int32)).to(device),
            "flags": torch.from_numpy(np.ascontiguousarray(f["flags"], np.uint8)).to(device),
            "ep": torch.from_numpy(np.ascontiguousarray(f["ep"], np.uint16).view(np.int16)).to(device)}


# ---------------------------------------------------------------- conntrack
def make_ct_stream(rng, n_conn: int, locals_be: np.ndarray, remotes_be: np.ndarray,
                   mean_pkts: float = 8.0, span: float = 0.02, frag_frac: float = 0.005,
                   icmp_err_frac: float = 0.03, other_frac: float = 0.01, pair_ok=None):
    """A packet stream of n_conn connections for the stateful path (SURVEY §8f
    row 3), vectorized.  Each connection is between a local endpoint address
    (locals_be[ep], network order) and a remote address, opened from either
    side, with ~Geom(1/mean_pkts) packets that alternate direction: TCP with
    SYN / SYN-ACK / ACK / PSH-ACK and a closing FIN or RST, UDP, ICMP echo
    (request, reply) and, in the reply direction, ICMP errors (types 3, 11,
    12) that conntrack relates to the connection; a few packets of an
    untracked protocol.  Connections overlap in time (start uniform in
    [0, 1), lifetime ~span), so packets of one connection are interleaved
    with others but stay in order.  Columns as cgpu_classify_v4_ct takes
    them: saddr, daddr, sport, dport (network order), proto, l4b (TCP header
    bytes 12-13 as a little-endian u16, or the ICMP type), flags (CGPU_F_EGRESS | CGPU_F_FRAGMENT), len, ep."""
    v6 = np.asarray(locals_be).ndim == 2  # (n, 16) uint8 addresses: IPv6 / ICMPv6
    adt = np.uint8 if v6 else np.uint32
    E = len(locals_be)
    ep = rng.integers(0, E, n_conn)
    loc = np.asarray(locals_be, adt)[ep]
    rem = np.asarray(remotes_be, adt)[rng.integers(0, len(remotes_be), n_conn)]
    if pair_ok is not None:  # e.g. this rank's conntrack shard: redraw the others
        bad = ~pair_ok(loc, rem)
        while bad.any():
            rem[bad] = np.asarray(remotes_be, adt)[rng.integers(0, len(remotes_be), int(bad.sum()))]
            bad[bad] = ~pair_ok(loc[bad], rem[bad])
    icmp = 58 if v6 else 1
    u = rng.random(n_conn)
    cproto = np.select([u < 0.70, u < 0.90, u < 1.0 - other_frac], [6, 17, icmp], 47).astype(np.uint8)
    init_eg = rng.random(n_conn) < 0.6
    eph = rng.integers(1024, 65536, n_conn)
    well = zipf_ports(rng, n_conn)
    lport = np.where(init_eg, eph, well).astype(np.uint16)
    rport = np.where(init_eg, well, eph).astype(np.uint16)
    k = rng.geometric(1.0 / mean_pkts, n_conn).astype(np.int64)
    total = int(k.sum())
    conn = np.repeat(np.arange(n_conn), k)
    first = np.cumsum(k) - k
    j = np.arange(total) - np.repeat(first, k)
    last = j == k[conn] - 1
    orig = (j == 0) | (rng.random(total) < 0.55)
    egress = np.where(orig, init_eg[conn], ~init_eg[conn])
    proto = cproto[conn].copy()
    r = rng.random(total)
    # TCP flags byte (tcphdr byte 13)
    tcpf = np.where(j == 0, L.TCP_SYN, np.where((j == 1) & ~orig, L.TCP_SYN | L.TCP_ACK,
                    np.where(r < 0.5, L.TCP_ACK, L.TCP_ACK | L.TCP_PSH)))
    r2 = rng.random(total)
    tcpf = np.where(last & (j > 0) & (r2 < 0.3), L.TCP_FIN | L.TCP_ACK, tcpf)
    tcpf = np.where(last & (j > 0) & (r2 > 0.95), L.TCP_RST, tcpf)
    # ICMP: echo request (8, some timestamp 13) one way, echo reply (0) back;
    # ICMPv6: echo request 128 (some 133, a router solicitation), reply 129
    if v6:
        icmpt = np.where(orig, np.where(r < 0.9, 128, 133), 129)
        errt = np.array([1, 2, 3, 4])  # DEST_UNREACH, PKT_TOOBIG, TIME_EXCEED, PARAMPROB
    else:
        icmpt = np.where(orig, np.where(r < 0.9, 8, 13), 0)
        errt = np.array([3, 11, 12])
    # errors related to any connection, in the reply direction
    err = ~orig & (rng.random(total) < icmp_err_frac)
    proto = np.where(err, icmp, proto).astype(np.uint8)
    icmpt = np.where(err, rng.choice(errt, total), icmpt)
    # TCP: header bytes 12-13 as loaded (doff << 4, NS bit sometimes set | flags << 8)
    ns = (rng.random(total) < 0.02).astype(np.int64)
    tcpw = (5 << 4) | ns | (tcpf.astype(np.int64) << 8)
    l4b = np.where(proto == 6, tcpw, np.where(proto == icmp, icmpt, 0)).astype(np.uint16)
    lc, rc = loc[conn], rem[conn]
    eg = egress[:, None] if v6 else egress
    saddr = np.where(eg, lc, rc).astype(adt)
    daddr = np.where(eg, rc, lc).astype(adt)
    lp, rp = lport[conn].byteswap(), rport[conn].byteswap()
    sport = np.where(egress, lp, rp).astype(np.uint16)
    dport = np.where(egress, rp, lp).astype(np.uint16)
    frag = (~egress) & (rng.random(total) < frag_frac) & (not v6)
    # interleave: connection start + in-connection gaps, stable by time
    t = rng.random(n_conn)[conn] + span * (j + rng.random(total)) / k[conn]
    order = np.argsort(t, kind="stable")
    out = {
        "saddr": saddr, "daddr": daddr, "sport": sport, "dport": dport, "proto": proto,
        "l4b": l4b, "flags": (egress.astype(np.uint8) | (frag.astype(np.uint8) << 1)),
        "len": rng.integers(64, 1501, total).astype(np.uint32), "ep": ep[conn].astype(np.uint16),
    }
    return {key: np.ascontiguousarray(v[order]) for key, v in out.items()}


def ct_endpoints(n_endpoints: int):
    """Local endpoint addresses (network order, inside the cluster /8) and
    their SECLABELs (lxc_config.h) for the stateful workloads."""
    locals_be = np.array([L.ip4_be(CLUSTER_V4 | (200 << 16) | (ep + 1)) for ep in range(n_endpoints)],
                         np.uint32)
    seclabels = (np.arange(n_endpoints, dtype=np.uint32) * 7 + 5000).astype(np.uint32)
    return locals_be, seclabels


def make_ct_workload(tables: Tables, n_conn: int, seed=SEED, gpu_id: int = 0, n_remote=None,
                     mean_pkts: float = 8.0, span: float = 0.02, world: int = 1):
    """The stateful stream over `tables`: n_conn connections
    between the tables' endpoints and remote addresses (80% inside installed
    ipcache prefixes), seeded per GPU like make_tuples.  With world > 1 every
    connection's address pair belongs to rank gpu_id's conntrack shard
    (shard.pairhash_np % world), so the rank streams are shards of one
    stream and no conntrack state is shared between ranks."""
    rng = np.random.Generator(np.random.PCG64(seed + 0xC7000 + gpu_id))
    locals_be, seclabels = ct_endpoints(tables.n_endpoints)
    nr = n_remote or max(16, n_conn // 4)
    pi = rng.integers(0, len(tables.pfx_addr), nr)
    base = tables.pfx_addr[pi].astype(np.uint64)
    ln = tables.pfx_len[pi].astype(np.uint64)
    host = rng.integers(0, 2**32, nr, dtype=np.uint64)
    hmask = (np.uint64(1) << (np.uint64(32) - ln)) - np.uint64(1)
    rem = np.where(rng.random(nr) < 0.8, base | (host & hmask), host).astype(np.uint32).byteswap()
    ok = None
    if world > 1:
        from .shard import pairhash_np
        ok = lambda a, b: (pairhash_np(a, b) % np.uint32(world)) == gpu_id  # noqa: E731
    t = make_ct_stream(rng, n_conn, locals_be, rem, mean_pkts=mean_pkts, span=span, pair_ok=ok)
    return t, locals_be, seclabels


def make_ctlb_workload(tables: Tables, svcs: Services, n_conn: int, seed=SEED, gpu_id: int = 0,
                       vip_frac: float = 0.4, mean_pkts: float = 8.0, span: float = 0.02,
                       loop_frac: float = 0.02, world: int = 1):
    """The stateful stream behind the service step (cgpu_classify_v4_ctlb):
    make_ct_workload where `vip_frac` of the connections' remotes are service
    addresses.  Egress packets to a service carry its port (L4 services);
    replies come from the service address or, for 2/3 of the connections,
    from the backend the connection's local port picks (the reverse NAT map
    is empty, so both occur on the wire).  `loop_frac` of the backends are
    the endpoints themselves (lb4_local's loopback source NAT).  hash =
    skb->hash: the flow hash of the connection's egress direction, redrawn
    for 5 % of the packets.  Returns (t, locals_be, seclabels, services)."""
    from .shard import flowhash_np, pairhash_np
    rng = np.random.Generator(np.random.PCG64(seed + 0xCB000 + gpu_id))
    locals_be, seclabels = ct_endpoints(tables.n_endpoints)
    ns = len(svcs.vip)
    vals = svcs.vals.copy()
    nb = vals["count"][:ns].astype(np.int64)
    loop = rng.random(len(vals) - ns) < loop_frac
    vals["target"][ns:] = np.where(loop, locals_be[rng.integers(0, len(locals_be), len(loop))],
                                   vals["target"][ns:])
    svcs = Services(svcs.keys, vals, svcs.vip, svcs.port)
    nr = max(16, n_conn // 4)
    pi = rng.integers(0, len(tables.pfx_addr), nr)
    base = tables.pfx_addr[pi].astype(np.uint64)
    ln = tables.pfx_len[pi].astype(np.uint64)
    host = rng.integers(0, 2**32, nr, dtype=np.uint64)
    hmask = (np.uint64(1) << (np.uint64(32) - ln)) - np.uint64(1)
    rem = np.where(rng.random(nr) < 0.8, base | (host & hmask), host).astype(np.uint32).byteswap()
    nv = int(nr * vip_frac / (1.0 - vip_frac))
    rem = np.concatenate([rem, svcs.vip[rng.integers(0, ns, nv)]]).astype(np.uint32)
    ok = None
    if world > 1:
        ok = lambda a, b: (pairhash_np(a, b) % np.uint32(world)) == gpu_id  # noqa: E731
    t = make_ct_stream(rng, n_conn, locals_be, rem, mean_pkts=mean_pkts, span=span, pair_ok=ok)
    order = np.argsort(svcs.vip, kind="stable")
    sv = svcs.vip[order]
    eg = (t["flags"] & 1).astype(bool)
    remote = np.where(eg, t["daddr"], t["saddr"])
    pos = np.minimum(np.searchsorted(sv, remote), ns - 1)
    isv = sv[pos] == remote
    si = order[pos]
    port = svcs.port[si]
    l4 = np.isin(t["proto"], [6, 17])
    setp = isv & (port != 0) & l4
    t["dport"] = np.where(eg & setp, port, t["dport"]).astype(np.uint16)
    t["sport"] = np.where(~eg & setp, port, t["sport"]).astype(np.uint16)
    # replies from a backend: the one the connection's local port picks
    lport = np.where(eg, t["sport"], t["dport"]).astype(np.int64)
    first = (ns + np.cumsum(nb) - nb)[si]
    bi = first + lport % np.maximum(nb[si], 1)
    fromb = ~eg & isv & (nb[si] > 0) & (lport % 3 != 0)
    bi = np.where(fromb, bi, 0)
    t["saddr"] = np.where(fromb, vals["target"][bi], t["saddr"]).astype(np.uint32)
    bport = vals["port"][bi]
    t["sport"] = np.where(fromb & l4 & (bport != 0), bport, t["sport"]).astype(np.uint16)
    loc = np.where(eg, t["saddr"], t["daddr"])
    rmt = np.where(eg, t["daddr"], t["saddr"])
    lp = np.where(eg, t["sport"], t["dport"])
    rp = np.where(eg, t["dport"], t["sport"])
    h = flowhash_np(loc, rmt, lp, rp, t["proto"])
    redraw = rng.random(len(h)) < 0.05
    h[redraw] = rng.integers(0, 2**32, int(redraw.sum()), dtype=np.uint64).astype(np.uint32)
    t["hash"] = h.astype(np.uint32)
    return t, locals_be, seclabels, svcs


def ct6_endpoints(tables, n_endpoints: int):
    """Local IPv6 endpoint addresses (inside ROUTER_IP's /64, the cluster
    range) and their SECLABELs for the IPv6 stateful workloads."""
    loc = np.tile(np.frombuffer(tables.router, np.uint8), (n_endpoints, 1))
    loc[:, 8:12] = [0xC0, 0xA8, 0, 0]
    loc[:, 12:14] = 0
    loc[:, 14] = (np.arange(n_endpoints) >> 8) & 0xFF
    loc[:, 15] = (np.arange(n_endpoints) + 1) & 0xFF
    seclabels = (np.arange(n_endpoints, dtype=np.uint32) * 7 + 6000).astype(np.uint32)
    return loc.astype(np.uint8), seclabels


def make_ct6_workload(tables, n_conn: int, seed=SEED, gpu_id: int = 0, n_remote=None,
                      mean_pkts: float = 8.0, span: float = 0.02, world: int = 1):
    """make_ct_workload over Tables6 (the IPv6 stateful path): remotes 80%
    inside installed IPv6 ipcache prefixes; with world > 1 every pair belongs
    to rank gpu_id's shard (shard.pairhash6_np % world)."""
    rng = np.random.Generator(np.random.PCG64(seed + 0xC6000 + gpu_id))
    loc, seclabels = ct6_endpoints(tables, tables.n_endpoints)
    nr = n_remote or max(16, n_conn // 4)
    pi = rng.integers(0, len(tables.pfx_addr), nr)
    host = rng.integers(0, 256, (nr, 16), dtype=np.uint8)
    m = MASK6[tables.pfx_len[pi]]
    inside = tables.pfx_addr[pi] | (host & ~m)
    rem = np.where((rng.random(nr) < 0.8)[:, None], inside, host).astype(np.uint8)
    ok = None
    if world > 1:
        from .shard import pairhash6_np
        ok = lambda a, b: (pairhash6_np(a, b) % np.uint32(world)) == gpu_id  # noqa: E731
    t = make_ct_stream(rng, n_conn, loc, rem, mean_pkts=mean_pkts, span=span, pair_ok=ok)
    return t, loc, seclabels


def make_ctlb6_workload(tables, svcs: Services, n_conn: int, seed=SEED, gpu_id: int = 0,
                        vip_frac: float = 0.4, mean_pkts: float = 8.0, span: float = 0.02,
                        loop_frac: float = 0.02, world: int = 1):
    """make_ctlb_workload for IPv6 (cgpu_classify_v6_ctlb) over Tables6 and
    make_services6: `vip_frac` of the remotes are service addresses, replies
    from the service address or (2/3 of the connections) the backend,
    `loop_frac` of the backends are the endpoints themselves, hash = the
    egress direction's cgpu_flow_hash6, redrawn for 5 % of the packets.
    Returns (t, locals, seclabels, services)."""
    from .shard import flowhash6_np, pairhash6_np
    rng = np.random.Generator(np.random.PCG64(seed + 0xCB600 + gpu_id))
    loc, seclabels = ct6_endpoints(tables, tables.n_endpoints)
    ns = len(svcs.vip)
    vals = svcs.vals.copy()
    nb = vals["count"][:ns].astype(np.int64)
    loop = rng.random(len(vals) - ns) < loop_frac
    vals["target"][ns:] = np.where(loop[:, None], loc[rng.integers(0, len(loc), len(loop))],
                                   vals["target"][ns:])
    svcs = Services(svcs.keys, vals, svcs.vip, svcs.port)
    nr = max(16, n_conn // 4)
    pi = rng.integers(0, len(tables.pfx_addr), nr)
    host = rng.integers(0, 256, (nr, 16), dtype=np.uint8)
    m = MASK6[tables.pfx_len[pi]]
    rem = np.where((rng.random(nr) < 0.8)[:, None], tables.pfx_addr[pi] | (host & ~m), host)
    nv = int(nr * vip_frac / (1.0 - vip_frac))
    rem = np.concatenate([rem, svcs.vip[rng.integers(0, ns, nv)]]).astype(np.uint8)
    ok = None
    if world > 1:
        ok = lambda a, b: (pairhash6_np(a, b) % np.uint32(world)) == gpu_id  # noqa: E731
    t = make_ct_stream(rng, n_conn, loc, rem, mean_pkts=mean_pkts, span=span, pair_ok=ok)
    eg = (t["flags"] & 1).astype(bool)
    remote = np.where(eg[:, None], t["daddr"], t["saddr"])
    # make_services6 VIPs: fd00:96:<index>:...; match the index, then the row
    si = np.ascontiguousarray(remote[:, 4:8]).view(np.uint32)[:, 0].astype(np.int64)
    isv = (remote[:, :4] == [0xFD, 0x00, 0x00, 0x96]).all(axis=1) & (si < ns)
    si = np.where(isv, si, 0)
    isv &= (svcs.vip[si] == remote).all(axis=1)
    port = svcs.port[si]
    l4 = np.isin(t["proto"], [6, 17])
    setp = isv & (port != 0) & l4
    t["dport"] = np.where(eg & setp, port, t["dport"]).astype(np.uint16)
    t["sport"] = np.where(~eg & setp, port, t["sport"]).astype(np.uint16)
    lport = np.where(eg, t["sport"], t["dport"]).astype(np.int64)
    first = (ns + np.cumsum(nb) - nb)[si]
    bi = first + lport % np.maximum(nb[si], 1)
    fromb = ~eg & isv & (nb[si] > 0) & (lport % 3 != 0)
    bi = np.where(fromb, bi, 0)
    t["saddr"] = np.where(fromb[:, None], vals["target"][bi], t["saddr"]).astype(np.uint8)
    bport = vals["port"][bi]
    t["sport"] = np.where(fromb & l4 & (bport != 0), bport, t["sport"]).astype(np.uint16)
    lo = np.where(eg[:, None], t["saddr"], t["daddr"])
    rm = np.where(eg[:, None], t["daddr"], t["saddr"])
    lp = np.where(eg, t["sport"], t["dport"])
    rp = np.where(eg, t["dport"], t["sport"])
    h = flowhash6_np(lo, rm, lp, rp, t["proto"])
    redraw = rng.random(len(h)) < 0.05
    h[redraw] = rng.integers(0, 2**32, int(redraw.sum()), dtype=np.uint64).astype(np.uint32)
    t["hash"] = h.astype(np.uint32)
    return t, loc, seclabels, svcs


def load_lxc(target, seclabels):
    """cgpu_lxc_update / or_lxc_update: the SECLABEL of every endpoint."""
    for ep, sl in enumerate(seclabels):
        rc = target.lxc_update(ep, L.lxc_info(b"\0" * 6, 0, b"\0" * 16, 0, int(sl)))
        assert rc == 0, rc


# --------------------------------------------------- L3 MapState compilation
def make_l3_workload(n_rules=1000, n_endpoints=100, n_identities=65536, seed=SEED, n_keys=16,
                     n_vals=8, requires_frac=0.03):
    """A policy repository and label sets for cgpu_l3_compile (SURVEY §8f
    row 4): rules whose subject / peer selectors mix matchLabels over three
    sources ("k8s", "container", "any") with In / NotIn / Exists /
    DoesNotExist expressions, some FromRequires and L4-restricted blocks, a
    few "reserved.all" selectors; endpoints and identities carry 1-5 labels."""
    from . import policy as P
    rng = np.random.Generator(np.random.PCG64(seed + 0x13))
    keys = [f"k{i}" for i in range(n_keys)]
    srcs = ["k8s", "container", "any"]

    def sel(lo=0):
        ml = {}
        for _ in range(rng.integers(lo, 3)):
            ml[f"{rng.choice(srcs)}.{rng.choice(keys)}"] = f"v{rng.integers(0, n_vals)}"
        ex = []
        for _ in range(rng.integers(0, 2)):
            op = str(rng.choice(["In", "NotIn", "Exists", "DoesNotExist"]))
            vals = [f"v{x}" for x in rng.integers(0, n_vals, rng.integers(1, 3))] if op in (
                "In", "NotIn") else []
            ex.append((f"{rng.choice(srcs)}.{rng.choice(keys)}", op, vals))
        if rng.random() < 0.02:
            ml["reserved.all"] = ""
        return P.EndpointSelector(ml, ex)

    repo = P.Repository()
    for _ in range(n_rules):
        ing = [P.IngressRule([sel(1) for _ in range(1 if rng.random() < requires_frac else 0)],
                             [sel(1) for _ in range(rng.integers(0, 3))], bool(rng.random() < 0.2))
               for _ in range(rng.integers(0, 3))]
        eg = [P.EgressRule([sel(1) for _ in range(1 if rng.random() < requires_frac else 0)],
                           [sel(1) for _ in range(rng.integers(0, 3))], bool(rng.random() < 0.2))
              for _ in range(rng.integers(0, 3))]
        repo.add(P.Rule(sel(1), ing, eg))

    def sets(n):
        nl = rng.integers(1, 6, n)
        src = rng.choice(np.array(srcs[:2]), int(nl.sum()))
        key = rng.integers(0, n_keys, int(nl.sum()))
        val = rng.integers(0, n_vals, int(nl.sum()))
        out, o = [], 0
        for c in nl:
            out.append([P.Label(str(src[o + j]), keys[key[o + j]], f"v{val[o + j]}") for j in range(c)])
            o += c
        return out

    return repo, sets(n_endpoints), sets(n_identities)


# ------------------------------------------- full MapState (L4 + L3 + CIDR)
def make_mapstate_workload(n_rules=120, n_endpoints=16, n_identities=400, seed=SEED, n_keys=8,
                           n_vals=4):
    """A repository exercising every input of computeDesiredPolicyMapState:
    FromEndpoints / FromRequires / FromEntities / FromCIDR / FromCIDRSet (and
    the To* forms), ToPorts over TCP / UDP / ANY with HTTP or Kafka L7 rules on
    some ports (one L7 kind per port, so merges never conflict), L3-only
    blocks that wildcardL3L4Rules folds into L7 filters; identities with label
    sets, the reserved identities and CIDR identities
    (labels/cidr.GetCIDRLabels); endpoints with mixed enforcement and some
    redirects left unallocated (proxy port 0).
    -> (repo, [EndpointPolicy], [(identity, [Label])])"""
    from . import policy as P
    rng = np.random.Generator(np.random.PCG64(seed + 0x14))
    keys = [f"k{i}" for i in range(n_keys)]
    srcs = ["k8s", "container", "any"]
    l7_of = {"80": "http", "8080": "http", "9092": "kafka", "53": None, "443": None, "5000": None}
    ports = list(l7_of)
    cidrs = ["10.0.0.0/8", "10.1.0.0/16", "192.168.0.0/16", "0.0.0.0/0", "172.16.5.0/24"]

    def sel(lo=0):
        ml = {}
        for _ in range(rng.integers(lo, 3)):
            ml[f"{rng.choice(srcs)}.{rng.choice(keys)}"] = f"v{rng.integers(0, n_vals)}"
        ex = []
        if rng.random() < 0.3:
            op = str(rng.choice(["In", "NotIn", "Exists", "DoesNotExist"]))
            vals = [f"v{x}" for x in rng.integers(0, n_vals, rng.integers(1, 3))] if op in (
                "In", "NotIn") else []
            ex.append((f"{rng.choice(srcs)}.{rng.choice(keys)}", op, vals))
        if rng.random() < 0.01:
            ml["reserved.all"] = ""
        return P.EndpointSelector(ml, ex)

    def port_rules():
        out = []
        for _ in range(rng.integers(1, 3)):
            ps = [(str(p), str(rng.choice(["TCP", "TCP", "UDP", "ANY"])))
                  for p in rng.choice(ports, rng.integers(1, 3), replace=False)]
            pr = P.PortRule(ps)
            kinds = {l7_of[p] for p, _ in ps} - {None}
            if len(kinds) == 1 and rng.random() < 0.6:
                kind = kinds.pop()
                if kind == "http":
                    pr.http = [("GET", "/")]
                else:
                    pr.kafka = [("produce",)]
                pr.ports = [(p, pr_) for p, pr_ in ps if l7_of[p] == kind]
            out.append(pr)
        return out

    def block(ingress):
        kw = {}
        has_ports = rng.random() < 0.5
        kind = rng.choice(["ep", "ep", "ep", "ent", "cidr", "cidrset", "none"])
        pre = "from_" if ingress else "to_"
        if kind == "ep":
            kw[pre + "endpoints"] = [sel(0) for _ in range(rng.integers(1, 3))]
        elif kind == "ent":
            kw[pre + "entities"] = list(rng.choice(["world", "host", "cluster", "all", "init"],
                                                   rng.integers(1, 3), replace=False))
        elif kind == "cidr" and (not ingress or not has_ports):  # Sanitize: no FromCIDR + ToPorts
            kw[pre + "cidr"] = list(rng.choice(cidrs, rng.integers(1, 3), replace=False))
        elif kind == "cidrset" and (not ingress or not has_ports):
            kw[pre + "cidr_set"] = [("10.0.0.0/8", ["10.96.0.0/12", "10.1.2.0/24"])]
        if rng.random() < 0.04 and kind == "ep":
            kw[pre + "requires"] = [sel(1)]
        if has_ports:
            kw["to_ports"] = port_rules()
        return (P.IngressRule if ingress else P.EgressRule)(**kw)

    repo = P.Repository()
    for _ in range(n_rules):
        repo.add(P.Rule(sel(1), [block(True) for _ in range(rng.integers(0, 3))],
                        [block(False) for _ in range(rng.integers(0, 3))]))

    def labels_of():
        nl = rng.integers(1, 5)
        return [P.Label(str(rng.choice(srcs[:2])), keys[rng.integers(0, n_keys)],
                        f"v{rng.integers(0, n_vals)}") for _ in range(nl)]

    ids = [(1, [P.parse_label("reserved:host")]), (2, [P.parse_label("reserved:world")]),
           (3, [P.parse_label("reserved:cluster")]), (5, [P.parse_label("reserved:init")])]
    cidr_ids = ["10.1.2.0/24", "10.1.0.0/16", "10.97.0.0/16", "192.168.4.0/24", "8.8.8.8/32",
                "172.16.5.7/32", "10.200.0.0/16"]
    for k, c in enumerate(cidr_ids):
        ids.append(((1 << 24) + 1 + k, P.cidr_identity_labels(c, "10.0.0.0/8")))
    while len(ids) < n_identities:
        ids.append((256 + len(ids), labels_of()))
    eps = []
    for i in range(n_endpoints):
        red = {}
        for ing in (True, False):
            for p in ("80", "8080", "9092"):
                if rng.random() < 0.8:
                    red[(ing, "TCP", int(p))] = int(10000 + 100 * i + int(p) % 97)
        eps.append(P.EndpointPolicy(labels_of(), i, bool(rng.random() < 0.85),
                                    bool(rng.random() < 0.85), red))
    return repo, eps, ids
