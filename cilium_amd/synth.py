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
    for k, v in zip(t.ipc_keys, t.ipc_vals):
        rc = engine.ipcache_update(k, v)
        assert rc == 0, rc
    for k, e, ep in zip(t.pol_keys, t.pol_entries, t.pol_ep):
        rc = engine.policy_update(int(ep), k, e)
        assert rc == 0, rc


def load_oracle(oracle, t: Tables):
    for k, v in zip(t.ipc_keys, t.ipc_vals):
        assert oracle.ipcache_update(k, v) == 0
    for k, e, ep in zip(t.pol_keys, t.pol_entries, t.pol_ep):
        assert oracle.policy_update(int(ep), k, e) == 0


TUPLE_DTYPES = {"saddr": np.uint32, "daddr": np.uint32, "dport": np.uint16, "proto": np.uint8,
                "flags": np.uint8, "len": np.uint32, "ep": np.uint16}


def to_device(t: dict, device="cuda"):
    """numpy SoA -> torch device tensors (bit-identical views).  IPv6
    address columns ((n, 16) uint8) stay uint8."""
    import torch
    view = {np.uint32: np.int32, np.uint16: np.int16, np.uint8: np.uint8}
    out = {}
    for k, dt in TUPLE_DTYPES.items():
        if k in ("saddr", "daddr") and np.asarray(t[k]).ndim == 2:
            a = np.ascontiguousarray(t[k], np.uint8)
        else:
            a = np.ascontiguousarray(t[k], dt).view(view[dt])
        out[k] = torch.from_numpy(a).to(device, non_blocking=False)
    return out
