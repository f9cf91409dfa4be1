"""TEST INFRASTRUCTURE — emit golden fixtures from the reference's own BPF C.

Run in the development container only (needs /root/reference):

    make -C oracle ref && python oracle/gen_golden.py

It loads oracle/_ref/libref_{policy,xdp,lb_*,lbl}.so — the reference's
bpf/lib/policy.h, bpf/lib/eps.h, bpf/bpf_xdp.c, bpf/bpf_lb.c and bpf/lib/lb.h
(+ conntrack.h) compiled as host C with mocked kernel maps and helpers
(oracle/ref/) — feeds them seeded scenarios, and writes
inputs + reference outputs as small .npz files (plain arrays, no pickles)
under tests/golden/, plus tests/golden/MANIFEST.json.  The fixtures are data;
nothing from the reference's sources is stored.
"""
from __future__ import annotations

import ctypes as C
import hashlib
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

from cilium_amd import layouts as L  # noqa: E402
from cilium_amd import shard  # noqa: E402
from cilium_amd import synth  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")
SEED = 0xC1110000


def load_ref():
    subprocess.run(["make", "-s", "-C", HERE, "ref", "_ref/unit-test"], check=True)
    pol = C.CDLL(os.path.join(HERE, "_ref", "libref_policy.so"))
    xdp = C.CDLL(os.path.join(HERE, "_ref", "libref_xdp.so"))
    u32p = C.POINTER(C.c_uint32)
    ip = C.POINTER(C.c_int)
    pol.ref_reset.restype = None
    pol.ref_policy_update.argtypes = [C.c_int, C.c_void_p, C.c_void_p]
    pol.ref_policy_read.argtypes = [C.c_int, C.c_void_p, C.c_void_p]
    pol.ref_ipcache_update.argtypes = [C.c_void_p, C.c_void_p]
    pol.ref_ipcache_lookup4.argtypes = [C.c_uint32, u32p, u32p]
    pol.ref_ipcache_lookup6.argtypes = [C.c_void_p, u32p, u32p]
    pol.ref_policy_ingress.argtypes = [C.c_int, C.c_uint32, C.c_uint16, C.c_uint8, C.c_int,
                                       C.c_uint32, ip, ip]
    pol.ref_policy_egress.argtypes = [C.c_int, C.c_uint32, C.c_uint16, C.c_uint8, C.c_uint32,
                                      ip, ip]
    pol.ref_policy_raw.argtypes = [C.c_int, C.c_uint32, C.c_uint16, C.c_uint8, C.c_int, C.c_int,
                                   C.c_uint32, ip, ip]
    pol.ref_classify_v4.argtypes = [C.c_uint32, C.c_uint32, C.c_uint16, C.c_uint8, C.c_uint8,
                                    C.c_uint32, C.c_int, C.c_int, C.c_uint32, C.c_int, u32p, ip,
                                    ip, ip]
    pol.ref_constants.argtypes = [u32p, C.c_int]
    pol.ref_classify_v6.argtypes = [C.c_void_p, C.c_void_p, C.c_uint16, C.c_uint8, C.c_uint8,
                                    C.c_uint32, C.c_int, C.c_int, C.c_uint32, u32p, ip, ip, ip]
    pol.ref_metrics_read.argtypes = [C.c_void_p]
    pol.ref_metrics_read.restype = None
    pol.ref_metrics_packet.argtypes = [C.c_int, C.c_uint32, C.c_int]
    pol.ref_metrics_packet.restype = None
    pol.ref_router_ip.argtypes = [C.c_void_p]
    pol.ref_router_ip.restype = None
    xdp.ref_xdp_reset.restype = None
    xdp.ref_xdp_cidr_update.argtypes = [C.c_int, C.c_void_p]
    xdp.ref_xdp_endpoint_update.argtypes = [C.c_void_p]
    xdp.ref_xdp_run.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(C.c_uint64)]
    return pol, xdp


def ref_metrics(pol):
    """cilium_metrics as the reference's update_metrics call sites left it
    (send_drop_notify / send_trace_notify, oracle/ref/harness_policy.c)."""
    m = np.zeros((256, 4, 2), np.uint64)
    pol.ref_metrics_read(m.ctypes.data)
    return m


def b(x):
    return np.ascontiguousarray(x).tobytes()


# ------------------------------------------------------------------ policy
IDENTS = np.array([0, 1, 2, 3, 4, 5, 256, 257, 300, 1000, 65535, 70000, 0xFFFFFFFF], np.uint32)
PORTS = np.array([0, 22, 53, 80, 443, 8080, 65535, 4000, 8, 0x0800], np.uint16)
PROTOS = np.array([0, 1, 6, 17, 132], np.uint8)


def gen_policy_keys(rng, n_ep, per_ep):
    keys, entries, eps = [], [], []
    for ep in range(n_ep):
        seen = set()
        while len([e for e in eps if e == ep]) < per_ep:
            kind = rng.integers(0, 3)
            ident = int(rng.choice(IDENTS))
            port = int(rng.choice(PORTS))
            proto = int(rng.choice(PROTOS))
            egress = int(rng.integers(0, 2))
            if kind == 1:
                port, proto = 0, 0
            elif kind == 2:
                ident = 0
            pad = int(rng.integers(1, 128)) if rng.random() < 0.05 else 0
            k = L.policy_key(ident, port, proto, egress, pad)
            kb = b(k)
            if kb in seen:
                continue
            seen.add(kb)
            proxy = int(rng.integers(1, 65536)) if rng.random() < 0.15 else 0
            keys.append(k)
            entries.append(L.policy_entry(proxy))
            eps.append(ep)
    return (np.array(keys, L.POLICY_KEY), np.array(entries, L.POLICY_ENTRY),
            np.array(eps, np.uint16))


def gen_policy_fixture(pol, rng):
    pol.ref_reset()
    keys, entries, eps = gen_policy_keys(rng, 4, 60)
    for k, e, ep in zip(keys, entries, eps):
        pol.ref_policy_update(int(ep), b(k), b(e))
    n = 4000
    q = {
        "ep": rng.integers(0, 5, n).astype(np.uint16),  # ep 4 has an empty map
        "identity": np.where(rng.random(n) < 0.8, rng.choice(IDENTS, n),
                             rng.integers(0, 2**32, n, dtype=np.uint64)).astype(np.uint32),
        "dport": np.array([L.htons(int(p)) for p in
                           np.where(rng.random(n) < 0.85, rng.choice(PORTS, n),
                                    rng.integers(0, 65536, n))], np.uint16),
        "proto": np.where(rng.random(n) < 0.9, rng.choice(PROTOS, n),
                          rng.integers(0, 256, n)).astype(np.uint8),
        "kind": rng.integers(0, 3, n).astype(np.uint8),  # 0 ingress, 1 egress, 2 raw
        "dir": rng.integers(0, 2, n).astype(np.uint8),   # CT_EGRESS 0 / CT_INGRESS 1 (raw)
        "frag": (rng.random(n) < 0.15).astype(np.uint8),
        "len": rng.integers(0, 70000, n).astype(np.uint32),
    }
    ret = np.empty(n, np.int32)
    nprobes = np.empty(n, np.int32)
    hit = np.empty(n, np.int32)
    a, h = C.c_int(), C.c_int()
    for i in range(n):
        ep, ident, dp, pr = int(q["ep"][i]), int(q["identity"][i]), int(q["dport"][i]), int(q["proto"][i])
        ln, fr = int(q["len"][i]), int(q["frag"][i])
        if q["kind"][i] == 0:
            r = pol.ref_policy_ingress(ep, ident, dp, pr, fr, ln, C.byref(a), C.byref(h))
        elif q["kind"][i] == 1:
            r = pol.ref_policy_egress(ep, ident, dp, pr, ln, C.byref(a), C.byref(h))
        else:
            r = pol.ref_policy_raw(ep, ident, dp, pr, int(q["dir"][i]), fr, ln, C.byref(a),
                                   C.byref(h))
        ret[i], nprobes[i], hit[i] = r, a.value, h.value
    final = np.zeros(len(keys), L.POLICY_ENTRY)
    for i, (k, ep) in enumerate(zip(keys, eps)):
        buf = C.create_string_buffer(24)
        assert pol.ref_policy_read(int(ep), b(k), buf) == 0
        final[i] = np.frombuffer(buf.raw, L.POLICY_ENTRY)[0]
    return dict(keys=keys, entries=entries, key_ep=eps, **{"q_" + k: v for k, v in q.items()},
                ret=ret, nprobes=nprobes, hit_probe=hit, final_entries=final)


# ----------------------------------------------------------------- ipcache
def rand_v4_prefixes(rng, n, lens, weights):
    lens = rng.choice(lens, n, p=np.array(weights) / np.sum(weights))
    addrs = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    # cluster prefixes in a few /8s so they overlap
    top = rng.choice(np.array([10, 172, 192, 100, 16], np.uint32), n)
    addrs = np.where(rng.random(n) < 0.7, (addrs & 0x00FFFFFF) | (top << 24), addrs)
    return addrs.astype(np.uint32), lens.astype(np.int64)


def v4_str(h):
    h = int(h)
    return f"{h >> 24}.{(h >> 16) & 255}.{(h >> 8) & 255}.{h & 255}"


def gen_ipcache_entries(rng, n4, n6, static=True):
    keys, vals = [], []
    addrs, lens = rand_v4_prefixes(rng, n4, [1, 2, 7, 8, 12, 16, 20, 23, 24, 25, 28, 31, 32],
                                   [1, 1, 2, 5, 5, 10, 10, 5, 30, 5, 10, 3, 15])
    for a, ln in zip(addrs, lens):
        k = L.ipcache_key(f"{v4_str(a)}/{ln}")
        if rng.random() < 0.3:  # keep host bits beyond the prefix (kernel ignores them)
            k["ip"][:4] = np.frombuffer(int(a).to_bytes(4, "big"), np.uint8)
        label = 0 if rng.random() < 0.05 else int(rng.choice(
            [1, 2, 3, 4, 5, int(rng.integers(256, 70000)), int(rng.integers(0, 2**32))]))
        keys.append(k)
        vals.append(L.remote_info(label, int(rng.integers(0, 2**32))))
    for _ in range(n6):
        ln = int(rng.choice([3, 8, 16, 32, 48, 56, 64, 65, 96, 112, 127, 128]))
        raw = bytearray(rng.integers(0, 256, 16, dtype=np.uint8).tobytes())
        if rng.random() < 0.7:
            raw[0:4] = bytes([0xf0, 0x0d, 0, int(rng.integers(0, 4))])
        k = np.zeros((), L.IPCACHE_KEY)
        k["family"] = L.ENDPOINT_KEY_IPV6
        k["prefixlen"] = 32 + ln
        k["ip"][:] = np.frombuffer(bytes(raw), np.uint8)
        label = 0 if rng.random() < 0.05 else int(rng.integers(1, 2**32))
        keys.append(k)
        vals.append(L.remote_info(label, int(rng.integers(0, 2**32))))
    # entries whose prefixlen stops inside the static {pad, family} part
    for plen, fam, pad in () if not static else ((0, 0, 0), (20, 0, 0), (30, 1, 0), (31, 2, 0), (31, 1, 0),
                           (24, 0, 5), (32, 1, 7)):
        k = np.zeros((), L.IPCACHE_KEY)
        k["prefixlen"] = plen
        k["family"] = fam
        k["pad"][2] = pad
        keys.append(k)
        vals.append(L.remote_info(0xABC00000 + plen, plen))
    return np.array(keys, L.IPCACHE_KEY), np.array(vals, L.REMOTE_ENDPOINT_INFO)


def v4_queries_near(rng, keys, n):
    v4 = keys[keys["family"] == L.ENDPOINT_KEY_IPV4]
    base = v4["ip"][:, :4].copy().view(">u4").ravel().astype(np.uint64)
    pick = base[rng.integers(0, len(base), n)]
    noise = rng.integers(0, 2**32, n, dtype=np.uint64) & rng.choice(
        np.array([0, 0xFF, 0xFFFF, 0xFFFFFF, 0xFFFFFFFF], np.uint64), n)
    h = np.where(rng.random(n) < 0.8, pick ^ noise, rng.integers(0, 2**32, n, dtype=np.uint64))
    return np.array([L.ip4_be(int(x)) for x in h.astype(np.uint32)], np.uint32)


def v6_queries_near(rng, keys, n):
    v6 = keys[keys["family"] == L.ENDPOINT_KEY_IPV6]["ip"]
    out = np.empty((n, 16), np.uint8)
    for i in range(n):
        if rng.random() < 0.8 and len(v6):
            a = v6[rng.integers(0, len(v6))].copy()
            cut = int(rng.integers(0, 17))
            a[cut:] = rng.integers(0, 256, 16 - cut, dtype=np.uint8)
        else:
            a = rng.integers(0, 256, 16, dtype=np.uint8)
        out[i] = a
    return out


def gen_ipcache_fixture(pol, rng):
    pol.ref_reset()
    keys, vals = gen_ipcache_entries(rng, 400, 300, static=True)
    n_static = 7  # the last 7 entries stop inside the static {pad, family} bits
    q4 = v4_queries_near(rng, keys, 4000)
    q6 = v6_queries_near(rng, keys, 3000)
    lab, tun = C.c_uint32(), C.c_uint32()
    out = dict(keys=keys, vals=vals, n_static=np.array(n_static), q4=q4, q6=q6)
    # phase a: without the static-part entries (misses occur); phase b: all
    for phase, upto in (("a", len(keys) - n_static), ("b", len(keys))):
        pol.ref_reset()
        for k, v in zip(keys[:upto], vals[:upto]):
            pol.ref_ipcache_update(b(k), b(v))
        r4 = np.zeros((len(q4), 3), np.uint32)
        for i, a in enumerate(q4):
            f = pol.ref_ipcache_lookup4(int(a), C.byref(lab), C.byref(tun))
            r4[i] = (f, lab.value if f else 0, tun.value if f else 0)
        r6 = np.zeros((len(q6), 3), np.uint32)
        for i, a in enumerate(q6):
            f = pol.ref_ipcache_lookup6(a.tobytes(), C.byref(lab), C.byref(tun))
            r6[i] = (f, lab.value if f else 0, tun.value if f else 0)
        out["r4" + phase], out["r6" + phase] = r4, r6
    return out


# ---------------------------------------------------------------- classify
CONFIGS = [  # (ct_proto_gate, ingress_src_identity, ingress_secctx_world)
    (1, 0, 0), (0, 2, 0), (1, 0, 1), (1, 256, 0), (1, 3, 0)]


def gen_classify_fixture(pol, rng):
    ikeys, ivals = gen_ipcache_entries(rng, 500, 0, static=False)
    keep = ikeys["prefixlen"] > 32 + 4  # no catch-all: exercise the cluster/world fallback
    ikeys, ivals = ikeys[keep], ivals[keep]
    # the agent's reserved entries (daemon/daemon.go:957-1013), minus 0.0.0.0/0
    extra = [("0.0.16.0/24", 3), ("10.0.0.1/32", 1), ("10.0.0.2/32", 1), ("172.16.0.0/12", 0)]
    ek = np.array([L.ipcache_key(c) for c, _ in extra], L.IPCACHE_KEY)
    ev = np.array([L.remote_info(i) for _, i in extra], L.REMOTE_ENDPOINT_INFO)
    ikeys = np.concatenate([ek, ikeys])
    ivals = np.concatenate([ev, ivals])
    hot = rng.choice(len(ikeys), 40, replace=False)
    labels = np.unique(ivals["sec_label"][hot])
    # policy keys drawn from the identities the ipcache resolves to
    pk, pe, pep = [], [], []
    for ep in range(4):
        seen = set()
        for _ in range(120):
            kind = rng.integers(0, 3)
            ident = int(rng.choice(labels)) if rng.random() < 0.8 else int(rng.choice(IDENTS))
            port = int(rng.choice(PORTS))
            proto = int(rng.choice(np.array([6, 17, 1, 6, 6, 132], np.uint8)))
            port = int(rng.choice(PORTS[1:6])) if kind != 1 and rng.random() < 0.7 else port
            egress = int(rng.integers(0, 2))
            if kind == 1:
                port, proto = 0, 0
            elif kind == 2:
                ident = 0
            k = L.policy_key(ident, port, proto, egress)
            if b(k) in seen:
                continue
            seen.add(b(k))
            pk.append(k)
            pe.append(L.policy_entry(int(rng.integers(1, 65536)) if rng.random() < 0.1 else 0))
            pep.append(ep)
    pk = np.array(pk, L.POLICY_KEY)
    pe = np.array(pe, L.POLICY_ENTRY)
    pep = np.array(pep, np.uint16)

    n = 6000
    hk = ikeys[hot]
    q4s = np.where(rng.random(n) < 0.5, v4_queries_near(rng, hk, n), v4_queries_near(rng, ikeys, n))
    q4d = np.where(rng.random(n) < 0.5, v4_queries_near(rng, hk, n), v4_queries_near(rng, ikeys, n))
    t = {
        "saddr": q4s, "daddr": q4d,
        "dport": np.array([L.htons(int(p)) for p in np.where(
            rng.random(n) < 0.9, rng.choice(PORTS[:6], n), rng.integers(0, 65536, n))], np.uint16),
        "proto": rng.choice(np.array([6, 6, 6, 6, 17, 17, 17, 1, 1, 47, 132, 0], np.uint8), n),
        "flags": ((rng.random(n) < 0.5).astype(np.uint8) |
                  ((rng.random(n) < 0.08).astype(np.uint8) << 1)),
        "len": rng.integers(0, 70000, n).astype(np.uint32),
        "ep": rng.integers(0, 5, n).astype(np.uint16),
    }
    out = {}
    for ci, (gate, src, sw) in enumerate(CONFIGS):
        pol.ref_reset()
        for k, v in zip(ikeys, ivals):
            pol.ref_ipcache_update(b(k), b(v))
        for k, e, ep in zip(pk, pe, pep):
            pol.ref_policy_update(int(ep), b(k), b(e))
        verdict = np.empty(n, np.int32)
        ident = np.empty(n, np.uint32)
        stage = np.empty(n, np.uint8)
        nprobes = np.empty(n, np.int32)
        naddr = np.empty(n, np.int32)
        idv, st, npb, na = C.c_uint32(), C.c_int(), C.c_int(), C.c_int()
        for i in range(n):
            verdict[i] = pol.ref_classify_v4(
                int(t["saddr"][i]), int(t["daddr"][i]), int(t["dport"][i]), int(t["proto"][i]),
                int(t["flags"][i]), int(t["len"][i]), int(t["ep"][i]), gate, src, sw,
                C.byref(idv), C.byref(st), C.byref(npb), C.byref(na))
            ident[i], stage[i], nprobes[i], naddr[i] = idv.value, st.value, npb.value, na.value
        final = np.zeros(len(pk), L.POLICY_ENTRY)
        for i, (k, ep) in enumerate(zip(pk, pep)):
            buf = C.create_string_buffer(24)
            assert pol.ref_policy_read(int(ep), b(k), buf) == 0
            final[i] = np.frombuffer(buf.raw, L.POLICY_ENTRY)[0]
        out[f"c{ci}_verdict"] = verdict
        out[f"c{ci}_identity"] = ident
        out[f"c{ci}_stage"] = stage
        out[f"c{ci}_nprobes"] = nprobes
        out[f"c{ci}_naddr"] = naddr
        out[f"c{ci}_final_entries"] = final
        out[f"c{ci}_metrics"] = ref_metrics(pol)
    return dict(ipc_keys=ikeys, ipc_vals=ivals, pol_keys=pk, pol_entries=pe, pol_ep=pep,
                configs=np.array(CONFIGS, np.int64), **{"t_" + k: v for k, v in t.items()}, **out)


# ------------------------------------------------------------- classify v6
CONFIGS6 = [(1, 0), (0, 2), (1, 256), (1, 3)]  # (ct_proto_gate, ingress_src_identity)


def gen_classify_v6_fixture(pol, rng):
    router = C.create_string_buffer(16)
    pol.ref_router_ip(router)
    router = np.frombuffer(router.raw, np.uint8).copy()
    ikeys, ivals = gen_ipcache_entries(rng, 60, 500, static=False)
    keep = ikeys["prefixlen"] > 32 + 4
    ikeys, ivals = ikeys[keep], ivals[keep]
    # entries inside the router's /64 (cluster range) and the router itself
    extra_k, extra_v = [], []
    for ln, lab in ((64, 0), (96, 3), (112, 5000), (128, 1)):
        k = np.zeros((), L.IPCACHE_KEY)
        k["family"] = L.ENDPOINT_KEY_IPV6
        k["prefixlen"] = 32 + ln
        a = router.copy()
        a[12:] = rng.integers(0, 256, 4, dtype=np.uint8)
        k["ip"][:] = a
        extra_k.append(k)
        extra_v.append(L.remote_info(lab))
    ikeys = np.concatenate([np.array(extra_k, L.IPCACHE_KEY), ikeys])
    ivals = np.concatenate([np.array(extra_v, L.REMOTE_ENDPOINT_INFO), ivals])
    v6 = ikeys["family"] == L.ENDPOINT_KEY_IPV6
    hot = rng.choice(np.nonzero(v6)[0], 40, replace=False)
    labels = np.unique(ivals["sec_label"][hot])
    pk, pe, pep = [], [], []
    for ep in range(3):
        seen = set()
        for _ in range(120):
            kind = rng.integers(0, 3)
            ident = int(rng.choice(labels)) if rng.random() < 0.8 else int(rng.choice(IDENTS))
            port = int(rng.choice(PORTS[1:6])) if rng.random() < 0.7 else int(rng.choice(PORTS))
            proto = int(rng.choice(np.array([6, 17, 58, 6, 6, 132], np.uint8)))
            egress = int(rng.integers(0, 2))
            if kind == 1:
                port, proto = 0, 0
            elif kind == 2:
                ident = 0
            k = L.policy_key(ident, port, proto, egress)
            if b(k) in seen:
                continue
            seen.add(b(k))
            pk.append(k)
            pe.append(L.policy_entry(int(rng.integers(1, 65536)) if rng.random() < 0.1 else 0))
            pep.append(ep)
    pk, pe, pep = (np.array(pk, L.POLICY_KEY), np.array(pe, L.POLICY_ENTRY),
                   np.array(pep, np.uint16))
    n = 5000

    def addrs():
        a = np.where(rng.random((n, 1)) < 0.5, v6_queries_near(rng, ikeys[hot], n),
                     v6_queries_near(rng, ikeys, n))
        inr = rng.random(n) < 0.1
        r = np.tile(router, (n, 1))
        r[:, 8:] = rng.integers(0, 256, (n, 8), dtype=np.uint8)
        a[inr] = r[inr]
        return a.astype(np.uint8)

    t = {
        "saddr": addrs(), "daddr": addrs(),
        "dport": np.array([L.htons(int(p)) for p in np.where(
            rng.random(n) < 0.9, rng.choice(PORTS[:6], n), rng.integers(0, 65536, n))], np.uint16),
        "proto": rng.choice(np.array([6, 6, 6, 6, 17, 17, 58, 58, 1, 47, 0], np.uint8), n),
        "flags": ((rng.random(n) < 0.5).astype(np.uint8) |
                  ((rng.random(n) < 0.08).astype(np.uint8) << 1)),
        "len": rng.integers(0, 70000, n).astype(np.uint32),
        "ep": rng.integers(0, 4, n).astype(np.uint16),
    }
    out = {}
    for ci, (gate, src) in enumerate(CONFIGS6):
        pol.ref_reset()
        for k, v in zip(ikeys, ivals):
            pol.ref_ipcache_update(b(k), b(v))
        for k, e, ep in zip(pk, pe, pep):
            pol.ref_policy_update(int(ep), b(k), b(e))
        verdict = np.empty(n, np.int32)
        ident = np.empty(n, np.uint32)
        stage = np.empty(n, np.uint8)
        nprobes = np.empty(n, np.int32)
        naddr = np.empty(n, np.int32)
        idv, st, npb, na = C.c_uint32(), C.c_int(), C.c_int(), C.c_int()
        for i in range(n):
            verdict[i] = pol.ref_classify_v6(
                t["saddr"][i].tobytes(), t["daddr"][i].tobytes(), int(t["dport"][i]),
                int(t["proto"][i]), int(t["flags"][i]), int(t["len"][i]), int(t["ep"][i]),
                gate, src, C.byref(idv), C.byref(st), C.byref(npb), C.byref(na))
            ident[i], stage[i], nprobes[i], naddr[i] = idv.value, st.value, npb.value, na.value
        final = np.zeros(len(pk), L.POLICY_ENTRY)
        for i, (k, ep) in enumerate(zip(pk, pep)):
            buf = C.create_string_buffer(24)
            assert pol.ref_policy_read(int(ep), b(k), buf) == 0
            final[i] = np.frombuffer(buf.raw, L.POLICY_ENTRY)[0]
        out[f"c{ci}_verdict"] = verdict
        out[f"c{ci}_identity"] = ident
        out[f"c{ci}_stage"] = stage
        out[f"c{ci}_nprobes"] = nprobes
        out[f"c{ci}_naddr"] = naddr
        out[f"c{ci}_final_entries"] = final
        out[f"c{ci}_metrics"] = ref_metrics(pol)
    return dict(router_ip=router, ipc_keys=ikeys, ipc_vals=ivals, pol_keys=pk, pol_entries=pe,
                pol_ep=pep, configs=np.array(CONFIGS6, np.int64),
                **{"t_" + k: v for k, v in t.items()}, **out)


# --------------------------------------------------------------------- xdp
def eth(ethertype, payload):
    return bytes(6) + bytes([2, 0, 0, 0, 0, 1]) + ethertype.to_bytes(2, "big") + payload


def ip4hdr(saddr_be, daddr_be):
    h = bytearray(20)
    h[0] = 0x45
    h[9] = 6
    h[12:16] = int(saddr_be).to_bytes(4, "little")
    h[16:20] = int(daddr_be).to_bytes(4, "little")
    return bytes(h)


def ip6hdr(s16, d16):
    h = bytearray(40)
    h[0] = 0x60
    h[6] = 17
    h[8:24] = bytes(s16)
    h[24:40] = bytes(d16)
    return bytes(h)


def gen_xdp_fixture(xdp, rng):
    xdp.ref_xdp_reset()
    dyn4, fix4, dyn6, fix6, eps = [], [], [], [], []
    a4, l4 = rand_v4_prefixes(rng, 150, [4, 8, 12, 16, 20, 24, 28, 31, 32], [1, 3, 3, 5, 5, 10, 3, 1, 2])
    for a, ln in zip(a4, l4):
        k = np.zeros((), L.LPM_V4_KEY)
        k["prefixlen"] = ln
        k["addr"][:] = np.frombuffer(int(a).to_bytes(4, "big"), np.uint8)
        dyn4.append(k)
    a4f, _ = rand_v4_prefixes(rng, 150, [32], [1])
    for i, a in enumerate(a4f):
        k = np.zeros((), L.LPM_V4_KEY)
        k["prefixlen"] = 32 if i % 25 else 24  # a hash key with prefixlen != 32 never matches
        k["addr"][:] = np.frombuffer(int(a).to_bytes(4, "big"), np.uint8)
        fix4.append(k)
    for i in range(150):
        k = np.zeros((), L.LPM_V6_KEY)
        k["prefixlen"] = int(rng.choice([16, 32, 48, 56, 64, 100, 128]))
        raw = bytearray(rng.integers(0, 256, 16, dtype=np.uint8).tobytes())
        raw[0:3] = bytes([0x20, 0x01, int(rng.integers(0, 4))])
        k["addr"][:] = np.frombuffer(bytes(raw), np.uint8)
        dyn6.append(k)
    for i in range(150):
        k = np.zeros((), L.LPM_V6_KEY)
        k["prefixlen"] = 128 if i % 25 else 64
        raw = bytearray(rng.integers(0, 256, 16, dtype=np.uint8).tobytes())
        raw[0:3] = bytes([0x20, 0x01, int(rng.integers(0, 4))])
        k["addr"][:] = np.frombuffer(bytes(raw), np.uint8)
        fix6.append(k)
    ep4 = rng.integers(0, 2**32, 60, dtype=np.uint64).astype(np.uint32)
    ep6 = rng.integers(0, 256, (60, 16), dtype=np.uint8)
    for i in range(60):
        k = np.zeros((), L.ENDPOINT_KEY)
        k["ip"][:4] = np.frombuffer(int(ep4[i]).to_bytes(4, "little"), np.uint8)
        k["family"] = 1
        if i % 20 == 19:
            k["pad4"] = 1  # never matches a lookup key
        eps.append(k)
        k6 = np.zeros((), L.ENDPOINT_KEY)
        k6["ip"][:] = ep6[i]
        k6["family"] = 2
        eps.append(k6)
    dyn4, fix4 = np.array(dyn4, L.LPM_V4_KEY), np.array(fix4, L.LPM_V4_KEY)
    dyn6, fix6 = np.array(dyn6, L.LPM_V6_KEY), np.array(fix6, L.LPM_V6_KEY)
    eps = np.array(eps, L.ENDPOINT_KEY)
    for w, arr in enumerate((dyn4, fix4, dyn6, fix6)):
        for k in arr:
            xdp.ref_xdp_cidr_update(w, b(k))
    for k in eps:
        xdp.ref_xdp_endpoint_update(b(k))

    def pick4(src):
        r = rng.random()
        if r < 0.35:
            base = int.from_bytes(bytes(src[rng.integers(0, len(src))]["addr"]), "big")
            return L.ip4_be(base ^ int(rng.integers(0, 256)) if rng.random() < 0.5 else base)
        return int(rng.integers(0, 2**32))

    frames, s4l, d4l, f4l, s6l, d6l, f6l, fam = [], [], [], [], [], [], [], []
    n = 2500
    for i in range(n):
        s = pick4(dyn4 if rng.random() < 0.5 else fix4)
        d = int(ep4[rng.integers(0, 60)]) if rng.random() < 0.6 else int(rng.integers(0, 2**32))
        fr = eth(0x0800, ip4hdr(s, d))
        if rng.random() < 0.03:
            fr = fr[: int(rng.integers(0, 34))]
        frames.append(fr)
    for i in range(n):
        src = dyn6 if rng.random() < 0.5 else fix6
        a = bytearray(bytes(src[rng.integers(0, len(src))]["addr"]))
        if rng.random() < 0.6:
            cut = int(rng.integers(2, 17))
            a[cut:] = rng.integers(0, 256, 16 - cut, dtype=np.uint8).tobytes()
        if rng.random() < 0.3:
            a = bytearray(rng.integers(0, 256, 16, dtype=np.uint8).tobytes())
        d = ep6[rng.integers(0, 60)].tobytes() if rng.random() < 0.6 else \
            rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
        fr = eth(0x86DD, ip6hdr(a, d))
        if rng.random() < 0.03:
            fr = fr[: int(rng.integers(0, 54))]
        frames.append(fr)
    for i in range(100):  # other ethertypes and runts
        et = int(rng.choice([0x0806, 0x8100, 0x88CC, 0x0000, 0xFFFF]))
        frames.append(eth(et, bytes(40))[: int(rng.integers(0, 60))])
    verdict = np.empty(len(frames), np.uint8)
    probes = np.empty(len(frames), np.uint64)
    pc = C.c_uint64()
    for i, fr in enumerate(frames):
        verdict[i] = xdp.ref_xdp_run(fr, len(fr), C.byref(pc))
        probes[i] = pc.value
    lens = np.array([len(f) for f in frames], np.uint32)
    blob = np.frombuffer(b"".join(frames), np.uint8)
    return dict(dyn4=dyn4, fix4=fix4, dyn6=dyn6, fix6=fix6, endpoints=eps,
                frame_bytes=blob, frame_len=lens, verdict=verdict, probes=probes)


# ---------------------------------------------------------------------- lb
def load_ref_lb():
    variants = {}
    for v in ("both", "l3", "l4"):
        L_ = C.CDLL(os.path.join(HERE, "_ref", f"libref_lb_{v}.so"))
        L_.ref_lb_reset.restype = None
        L_.ref_lb_update.argtypes = [C.c_void_p, C.c_void_p]
        L_.ref_lb_netdev.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint64)]
        variants[v] = L_
    lbls = {}
    for v, f in ((1, "libref_lbl.so"), (0, "libref_lbl_noct.so")):
        lbl = C.CDLL(os.path.join(HERE, "_ref", f))
        lbl.ref_lbl_reset.restype = None
        lbl.ref_lbl_update.argtypes = [C.c_void_p, C.c_void_p]
        u16p = C.POINTER(C.c_uint16)
        lbl.ref_lbl_run.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(C.c_int),
                                    C.POINTER(C.c_uint32), u16p, u16p, C.POINTER(C.c_int),
                                    C.POINTER(C.c_uint64)]
        lbls[v] = lbl
    return variants, lbls  # lbls[1]: CONNTRACK build, lbls[0]: without


LB_PROTOS = np.array([6, 6, 6, 6, 6, 17, 17, 17, 1, 1, 58, 47, 132, 0], np.uint8)


def gen_lb_services(rng, n_vip, targets, clients):
    """Service map contents as lbmap.UpdateService writes them (lbmap.go:350-428:
    slave 0 = master {count, weight}, slaves 1..count = backends), plus the
    irregular contents the map can also hold: a master with count 0, a master
    whose count exceeds its backends, backends with a nonzero count (reached by
    lb4_local's fallback), and sparse slave numbers."""
    keys, vals = [], []
    vips = []

    def put(addr_be, dport_be, slave, target_be, port_be, count, rev, weight):
        k = np.zeros((), L.LB4_KEY)
        k["address"], k["dport"], k["slave"] = addr_be, dport_be, slave
        v = np.zeros((), L.LB4_SERVICE)
        v["target"], v["port"], v["count"] = target_be, port_be, count
        v["rev_nat_index"], v["weight"] = rev, weight
        keys.append(k)
        vals.append(v)

    for i in range(n_vip):
        vip = L.ip4_be(0x0A600000 | int(rng.integers(1, 1 << 20)))  # 10.96.0.0/12
        vips.append(vip)
        kinds = ["l4"] if rng.random() < 0.5 else (["l3"] if rng.random() < 0.4 else ["l4", "l3"])
        for kind in kinds:
            dport = L.htons(int(rng.choice(PORTS[1:6]))) if kind == "l4" else 0
            nb = int(rng.integers(1, 6))
            rev = int(rng.integers(1, 65536))
            count = nb
            r = rng.random()
            if r < 0.08:
                count = 0          # a master with count 0 is not a service
            elif r < 0.2:
                count = nb + 1     # one selectable slave has no backend entry
            put(vip, dport, 0, 0, 0, count, 0, int(rng.integers(0, 3)))
            slaves = list(range(1, nb + 1))
            if rng.random() < 0.1:
                slaves[-1] = int(rng.integers(nb + 1, 40))  # sparse slave number
            for s in slaves:
                tgt = int(rng.choice(clients)) if rng.random() < 0.25 else int(rng.choice(targets))
                pr = rng.random()
                port = 0 if pr < 0.3 else (dport if pr < 0.5 else L.htons(int(rng.integers(1, 65536))))
                bc = int(rng.integers(1, 4)) if (kind == "l3" and rng.random() < 0.5) else 0
                put(vip, dport, s, tgt, port, bc, rev, int(rng.integers(0, 65536)))
    return (np.array(keys, L.LB4_KEY), np.array(vals, L.LB4_SERVICE),
            np.array(vips, np.uint32))


def l4_frame(saddr_be, daddr_be, sport_be, dport_be, proto, opts=False):
    """Ethernet + IPv4 (optionally with 4 option bytes) + an L4 header
    carrying the ports at offsets 0 / 2 (TCP, UDP) or an ICMP echo."""
    h = bytearray(24 if opts else 20)
    h[0] = 0x46 if opts else 0x45
    h[9] = proto
    h[12:16] = int(saddr_be).to_bytes(4, "little")
    h[16:20] = int(daddr_be).to_bytes(4, "little")
    if proto == 1:
        l4 = bytes([8, 0]) + bytes(6)
    else:
        l4 = int(sport_be).to_bytes(2, "little") + int(dport_be).to_bytes(2, "little") + \
             bytes(16 if proto == 6 else 4)
    return bytearray(eth(0x0800, bytes(h) + l4)), 14 + len(h)


def lb_tuples(rng, n, keys, vips, clients):
    fe = {}
    for k in keys:
        fe.setdefault(int(k["address"]), set()).add(int(k["dport"]))
    vsel = vips[rng.integers(0, len(vips), n)]
    daddr = np.where(rng.random(n) < 0.75, vsel,
                     rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)).astype(np.uint32)
    dport = np.empty(n, np.uint16)
    for i in range(n):
        ports = [p for p in fe.get(int(daddr[i]), ()) if p]
        dport[i] = int(rng.choice(ports)) if ports and rng.random() < 0.8 else \
            L.htons(int(rng.choice(PORTS)) if rng.random() < 0.5 else int(rng.integers(0, 65536)))
    saddr = np.where(rng.random(n) < 0.3, rng.choice(clients, n),
                     rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)).astype(np.uint32)
    h = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    h[:8] = [0, 1, 2, 0xFFFFFFFF, 0x7FFFFFFF, 65535, 65536, 0x80000000]
    return {"saddr": saddr, "daddr": daddr,
            "sport": rng.integers(0, 65536, n).astype(np.uint16), "dport": dport,
            "proto": rng.choice(LB_PROTOS, n), "hash": h,
            "opts": (rng.random(n) < 0.1).astype(np.uint8)}


def run_lb_netdev(lbv, keys, vals, t):
    lbv.ref_lb_reset()
    for k, v in zip(keys, vals):
        lbv.ref_lb_update(b(k), b(v))
    n = len(t["daddr"])
    ret = np.empty(n, np.int32)
    daddr = np.empty(n, np.uint32)
    dport = np.empty(n, np.uint16)
    lookups = np.empty(n, np.uint32)
    cnt = C.c_uint64()
    for i in range(n):
        fr, l4 = l4_frame(t["saddr"][i], t["daddr"][i], t["sport"][i], t["dport"][i],
                          int(t["proto"][i]), bool(t["opts"][i]))
        buf = (C.c_uint8 * len(fr)).from_buffer(fr)
        ret[i] = lbv.ref_lb_netdev(buf, len(fr), int(t["hash"][i]), C.byref(cnt))
        daddr[i] = int.from_bytes(bytes(fr[30:34]), "little")
        dport[i] = int.from_bytes(bytes(fr[l4 + 2:l4 + 4]), "little") \
            if int(t["proto"][i]) in (6, 17) else t["dport"][i]
        lookups[i] = cnt.value
    return ret, daddr, dport, lookups


def run_lb_lxc(lbl, keys, vals, t):
    lbl.ref_lbl_reset()
    for k, v in zip(keys, vals):
        lbl.ref_lbl_update(b(k), b(v))
    n = len(t["daddr"])
    out = {k: np.empty(n, dt) for k, dt in (
        ("ret", np.int32), ("svc_hit", np.uint8), ("tdaddr", np.uint32), ("rev_nat", np.uint16),
        ("slave", np.uint16), ("loopback", np.uint8), ("saddr", np.uint32), ("daddr", np.uint32),
        ("dport", np.uint16), ("lookups", np.uint32))}
    hit, td, lo, cnt = C.c_int(), C.c_uint32(), C.c_int(), C.c_uint64()
    rn, sl = C.c_uint16(), C.c_uint16()
    for i in range(n):
        fr, l4 = l4_frame(t["saddr"][i], t["daddr"][i], t["sport"][i], t["dport"][i],
                          int(t["proto"][i]), bool(t["opts"][i]))
        buf = (C.c_uint8 * len(fr)).from_buffer(fr)
        r = lbl.ref_lbl_run(buf, len(fr), int(t["hash"][i]), C.byref(hit), C.byref(td),
                            C.byref(rn), C.byref(sl), C.byref(lo), C.byref(cnt))
        out["ret"][i], out["svc_hit"][i], out["tdaddr"][i] = r, hit.value, td.value
        out["rev_nat"][i], out["slave"][i], out["loopback"][i] = rn.value, sl.value, lo.value
        out["saddr"][i] = int.from_bytes(bytes(fr[26:30]), "little")
        out["daddr"][i] = int.from_bytes(bytes(fr[30:34]), "little")
        out["dport"][i] = int.from_bytes(bytes(fr[l4 + 2:l4 + 4]), "little") \
            if int(t["proto"][i]) in (6, 17) else t["dport"][i]
        out["lookups"][i] = cnt.value
    return out


def gen_lb_fixture(lbvars, lbls, rng):
    targets = rng.integers(0, 2**32, 200, dtype=np.uint64).astype(np.uint32)
    clients = rng.integers(0, 2**32, 4, dtype=np.uint64).astype(np.uint32)
    keys, vals, vips = gen_lb_services(rng, 70, targets, clients)
    t = lb_tuples(rng, 5000, keys, vips, clients)
    out = dict(keys=keys, vals=vals, **{"t_" + k: v for k, v in t.items()})
    for name, lbv in lbvars.items():
        r, d, p, nl = run_lb_netdev(lbv, keys, vals, t)
        out.update({f"nd_{name}_ret": r, f"nd_{name}_daddr": d, f"nd_{name}_dport": p,
                    f"nd_{name}_lookups": nl})
    for ct, lbl in lbls.items():
        lx = run_lb_lxc(lbl, keys, vals, t)
        out.update({("lx_" if ct else "lxnoct_") + k: v for k, v in lx.items()})
    return out


def gen_classify_lb_fixture(pol, lbls, rng):
    """The egress path of BASELINE config 5 composed from the reference's own
    steps in bpf_lxc.c order: the service step (libref_lbl, bpf_lxc.c:444-469),
    then ipcache on tuple.daddr and policy on the rewritten dport (libref_policy
    ref_classify_v4 = bpf_lxc.c:484-505).  DROP_NO_SERVICE ends the packet
    before conntrack (bpf_lxc.c:455-458) and is counted by send_drop_notify with
    METRIC_EGRESS (:659-666).  Ingress tuples run the unchanged ingress path."""
    base = gen_classify_fixture(pol, rng)
    ikeys, ivals = base["ipc_keys"], base["ipc_vals"]
    pk, pe, pep = base["pol_keys"], base["pol_entries"], base["pol_ep"]
    v4 = ikeys["prefixlen"] >= 32
    pfx = ikeys[v4]["ip"][:, :4].copy().view("<u4").ravel()
    targets = pfx[rng.integers(0, len(pfx), 200)]
    clients = rng.integers(0, 2**32, 4, dtype=np.uint64).astype(np.uint32)
    keys, vals, vips = gen_lb_services(rng, 60, targets, clients)
    n = 5000
    lt = lb_tuples(rng, n, keys, vips, clients)
    t = {"saddr": lt["saddr"], "daddr": lt["daddr"], "sport": lt["sport"], "dport": lt["dport"],
         "proto": lt["proto"], "hash": lt["hash"],
         "flags": ((rng.random(n) < 0.7).astype(np.uint8) |
                   ((rng.random(n) < 0.05).astype(np.uint8) << 1)),
         "len": rng.integers(0, 70000, n).astype(np.uint32),
         "ep": rng.integers(0, 5, n).astype(np.uint16), "opts": lt["opts"]}
    out = {}
    idv, st, npb, na = C.c_uint32(), C.c_int(), C.c_int(), C.c_int()
    for ci, (gate, src, sw) in enumerate(CONFIGS[:2]):
        # the CONNTRACK switch decides both the policy protocol gate and
        # lb4_local's conntrack step
        lx = run_lb_lxc(lbls[gate], keys, vals, t)
        pol.ref_reset()
        for k, v in zip(ikeys, ivals):
            pol.ref_ipcache_update(b(k), b(v))
        for k, e, ep in zip(pk, pe, pep):
            pol.ref_policy_update(int(ep), b(k), b(e))
        verdict = np.empty(n, np.int32)
        ident = np.empty(n, np.uint32)
        stage = np.empty(n, np.uint8)
        nprobes = np.empty(n, np.int32)
        for i in range(n):
            eg = int(t["flags"][i]) & 1
            if eg and lx["ret"][i] < 0:
                verdict[i], ident[i], stage[i], nprobes[i] = lx["ret"][i], 0, 6, lx["lookups"][i]
                pol.ref_metrics_packet(int(lx["ret"][i]), int(t["len"][i]), 1)
                continue
            da = int(lx["tdaddr"][i]) if eg else int(t["daddr"][i])
            dp = int(lx["dport"][i]) if eg else int(t["dport"][i])
            verdict[i] = pol.ref_classify_v4(
                int(t["saddr"][i]), da, dp, int(t["proto"][i]), int(t["flags"][i]),
                int(t["len"][i]), int(t["ep"][i]), gate, src, sw,
                C.byref(idv), C.byref(st), C.byref(npb), C.byref(na))
            ident[i], stage[i] = idv.value, st.value
            nprobes[i] = npb.value + na.value + (int(lx["lookups"][i]) if eg else 0)
        final = np.zeros(len(pk), L.POLICY_ENTRY)
        for i, (k, ep) in enumerate(zip(pk, pep)):
            buf = C.create_string_buffer(24)
            assert pol.ref_policy_read(int(ep), b(k), buf) == 0
            final[i] = np.frombuffer(buf.raw, L.POLICY_ENTRY)[0]
        out[f"c{ci}_verdict"], out[f"c{ci}_identity"] = verdict, ident
        out[f"c{ci}_stage"], out[f"c{ci}_nprobes"] = stage, nprobes
        out[f"c{ci}_final_entries"] = final
        out[f"c{ci}_metrics"] = ref_metrics(pol)
    return dict(ipc_keys=ikeys, ipc_vals=ivals, pol_keys=pk, pol_entries=pe, pol_ep=pep,
                lb_keys=keys, lb_vals=vals, configs=np.array(CONFIGS[:2], np.int64),
                **{"t_" + k: v for k, v in t.items()}, **out)


def gen_cascade_fixture(pol, xdp, lbls, rng):
    """BASELINE config 5 whole, composed from the reference's own programs in
    the order a packet meets them: an INGRESS packet first runs the netdev's
    XDP program (libref_xdp = bpf_xdp.c xdp_start, :180-184, over a frame
    built from the tuple: check_v4's dyn LPM / fix hash on saddr, then
    check_v4_endpoint on daddr); XDP_DROP ends it (no counter, no metric:
    the XDP program notifies nothing), XDP_PASS hands it to the ingress
    identity + policy (libref_policy ref_classify_v4 = bpf_netdev.c +
    ipv4_policy).  An EGRESS packet takes the service step (libref_lbl)
    then ipcache / policy, as classify_v4_lb.npz."""
    base = gen_classify_fixture(pol, rng)
    ikeys, ivals = base["ipc_keys"], base["ipc_vals"]
    pk, pe, pep = base["pol_keys"], base["pol_entries"], base["pol_ep"]
    v4 = ikeys["prefixlen"] >= 32
    pfx = ikeys[v4]["ip"][:, :4].copy().view("<u4").ravel()
    targets = pfx[rng.integers(0, len(pfx), 200)]
    clients = rng.integers(0, 2**32, 4, dtype=np.uint64).astype(np.uint32)
    keys, vals, vips = gen_lb_services(rng, 60, targets, clients)
    # the deny set: dyn4 prefixes of every length class, fix4 /32s (and a few
    # prefixlen-24 hash keys, which a /32 lookup key never matches), many of
    # them over installed ipcache ranges; the local endpoints (a few keys
    # with a nonzero pad, which no lookup key matches)
    dyn4, fix4, eps = [], [], []
    a4, l4 = rand_v4_prefixes(rng, 120, [8, 12, 16, 20, 24, 28, 31, 32], [1, 2, 4, 5, 10, 3, 1, 2])
    for i, (a, ln) in enumerate(zip(a4, l4)):
        if i % 3 == 0:
            a = int(pfx[rng.integers(0, len(pfx))].byteswap())
        k = np.zeros((), L.LPM_V4_KEY)
        k["prefixlen"] = ln
        m = (0xFFFFFFFF << (32 - int(ln))) & 0xFFFFFFFF
        k["addr"][:] = np.frombuffer((int(a) & m).to_bytes(4, "big"), np.uint8)
        dyn4.append(k)
    a4f, _ = rand_v4_prefixes(rng, 150, [32], [1])
    for i, a in enumerate(a4f):
        if i % 2 == 0:
            a = int(pfx[rng.integers(0, len(pfx))].byteswap()) ^ int(rng.integers(0, 256))
        k = np.zeros((), L.LPM_V4_KEY)
        k["prefixlen"] = 32 if i % 25 else 24
        k["addr"][:] = np.frombuffer(int(a).to_bytes(4, "big"), np.uint8)
        fix4.append(k)
    ep4 = rng.integers(0, 2**32, 24, dtype=np.uint64).astype(np.uint32)
    for i in range(24):
        k = np.zeros((), L.ENDPOINT_KEY)
        k["ip"][:4] = np.frombuffer(int(ep4[i]).to_bytes(4, "little"), np.uint8)
        k["family"] = L.ENDPOINT_KEY_IPV4
        if i % 12 == 11:
            k["pad4"] = 1
        eps.append(k)
    dyn4, fix4, eps = (np.array(dyn4, L.LPM_V4_KEY), np.array(fix4, L.LPM_V4_KEY),
                       np.array(eps, L.ENDPOINT_KEY))
    xdp.ref_xdp_reset()
    for w, arr in ((0, dyn4), (1, fix4)):
        for k in arr:
            xdp.ref_xdp_cidr_update(w, b(k))
    for k in eps:
        xdp.ref_xdp_endpoint_update(b(k))
    n = 6000
    lt = lb_tuples(rng, n, keys, vips, clients)
    eg = (rng.random(n) < 0.5).astype(np.uint8)
    # ingress: daddr a local endpoint (or a stray address); saddr from the
    # deny set (inside a dyn prefix, on or next to a fix /32) or anywhere
    daddr = np.where(rng.random(n) < 0.8, ep4[rng.integers(0, 24, n)],
                     rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)).astype(np.uint32)
    dsrc = []
    for i in range(n):
        r = rng.random()
        if r < 0.2:
            k = dyn4[rng.integers(0, len(dyn4))]
            base_ = int.from_bytes(bytes(k["addr"]), "big")
            host = int(rng.integers(0, 2**32)) & ((1 << (32 - int(k["prefixlen"]))) - 1)
            dsrc.append(L.ip4_be(base_ | host))
        elif r < 0.35:
            base_ = int.from_bytes(bytes(fix4[rng.integers(0, len(fix4))]["addr"]), "big")
            dsrc.append(L.ip4_be(base_ ^ (int(rng.integers(0, 4)) if rng.random() < 0.3 else 0)))
        else:
            dsrc.append(int(lt["saddr"][i]))
    dsrc = np.array(dsrc, np.uint32)
    t = {"saddr": np.where(eg == 1, lt["saddr"], dsrc).astype(np.uint32),
         "daddr": np.where(eg == 1, lt["daddr"], daddr).astype(np.uint32),
         "sport": lt["sport"], "dport": lt["dport"], "proto": lt["proto"], "hash": lt["hash"],
         "flags": (eg | (((rng.random(n) < 0.05) & (eg == 0)).astype(np.uint8) << 1)).astype(np.uint8),
         "len": rng.integers(0, 70000, n).astype(np.uint32),
         "ep": rng.integers(0, 5, n).astype(np.uint16), "opts": lt["opts"]}
    xv = np.zeros(n, np.uint8)
    xp = np.zeros(n, np.uint64)
    pc = C.c_uint64()
    for i in range(n):
        if eg[i]:
            continue
        fr = eth(0x0800, ip4hdr(t["saddr"][i], t["daddr"][i]))
        xv[i] = xdp.ref_xdp_run(fr, len(fr), C.byref(pc))
        xp[i] = pc.value
    out = {"xdp_verdict": xv, "xdp_probes": xp}
    idv, st, npb, na = C.c_uint32(), C.c_int(), C.c_int(), C.c_int()
    for ci, (gate, src, sw) in enumerate(CONFIGS[:2]):
        lx = run_lb_lxc(lbls[gate], keys, vals, t)
        pol.ref_reset()
        for k, v in zip(ikeys, ivals):
            pol.ref_ipcache_update(b(k), b(v))
        for k, e, ep in zip(pk, pe, pep):
            pol.ref_policy_update(int(ep), b(k), b(e))
        verdict = np.empty(n, np.int32)
        ident = np.empty(n, np.uint32)
        stage = np.empty(n, np.uint8)
        nprobes = np.empty(n, np.int64)
        for i in range(n):
            if not eg[i] and xv[i] == L.XDP_DROP:
                verdict[i], ident[i], stage[i], nprobes[i] = L.VERDICT_XDP_DROP, 0, L.STAGE_XDP_DROP, xp[i]
                continue
            if eg[i] and lx["ret"][i] < 0:
                verdict[i], ident[i], stage[i], nprobes[i] = lx["ret"][i], 0, 6, lx["lookups"][i]
                pol.ref_metrics_packet(int(lx["ret"][i]), int(t["len"][i]), 1)
                continue
            da = int(lx["tdaddr"][i]) if eg[i] else int(t["daddr"][i])
            dp = int(lx["dport"][i]) if eg[i] else int(t["dport"][i])
            verdict[i] = pol.ref_classify_v4(
                int(t["saddr"][i]), da, dp, int(t["proto"][i]), int(t["flags"][i]),
                int(t["len"][i]), int(t["ep"][i]), gate, src, sw,
                C.byref(idv), C.byref(st), C.byref(npb), C.byref(na))
            ident[i], stage[i] = idv.value, st.value
            nprobes[i] = npb.value + na.value + (int(lx["lookups"][i]) if eg[i] else int(xp[i]))
        final = np.zeros(len(pk), L.POLICY_ENTRY)
        for i, (k, ep) in enumerate(zip(pk, pep)):
            buf = C.create_string_buffer(24)
            assert pol.ref_policy_read(int(ep), b(k), buf) == 0
            final[i] = np.frombuffer(buf.raw, L.POLICY_ENTRY)[0]
        out[f"c{ci}_verdict"], out[f"c{ci}_identity"] = verdict, ident
        out[f"c{ci}_stage"], out[f"c{ci}_nprobes"] = stage, nprobes
        out[f"c{ci}_final_entries"] = final
        out[f"c{ci}_metrics"] = ref_metrics(pol)
    return dict(ipc_keys=ikeys, ipc_vals=ivals, pol_keys=pk, pol_entries=pe, pol_ep=pep,
                lb_keys=keys, lb_vals=vals, dyn4=dyn4, fix4=fix4, endpoints=eps,
                configs=np.array(CONFIGS[:2], np.int64),
                **{"t_" + k: v for k, v in t.items()}, **out)


# ------------------------------------------------ IPv6 service translation
def load_ref_lbl6():
    libs = {}
    for v, f in ((1, "libref_lbl6.so"), (0, "libref_lbl6_noct.so")):
        lib = C.CDLL(os.path.join(HERE, "_ref", f))
        lib.ref_lbl6_reset.restype = None
        lib.ref_lbl6_update.argtypes = [C.c_void_p, C.c_void_p]
        u16p = C.POINTER(C.c_uint16)
        lib.ref_lbl6_run.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(C.c_int),
                                     C.c_void_p, u16p, u16p, C.POINTER(C.c_int),
                                     C.POINTER(C.c_uint64)]
        libs[v] = lib
    return libs  # [1]: CONNTRACK build, [0]: without


def gen_lb6_services(rng, n_vip, targets):
    """cilium_lb6_services contents (lbmap.UpdateService's layout, plus the
    irregular contents gen_lb_services also covers: count-0 masters, masters
    counting more slaves than exist, backends with a count, sparse slaves)."""
    keys, vals, vips = [], [], []

    def put(addr, dport_be, slave, target, port_be, count, rev, weight):
        k = np.zeros((), L.LB6_KEY)
        k["address"][:] = addr
        k["dport"], k["slave"] = dport_be, slave
        v = np.zeros((), L.LB6_SERVICE)
        v["target"][:] = target
        v["port"], v["count"], v["rev_nat_index"], v["weight"] = port_be, count, rev, weight
        keys.append(k)
        vals.append(v)

    for _ in range(n_vip):
        vip = np.zeros(16, np.uint8)
        vip[:6] = [0xFD, 0x00, 0x00, 0x96, 0, 0]
        vip[6:] = rng.integers(0, 256, 10, dtype=np.uint8)
        vips.append(vip)
        kinds = ["l4"] if rng.random() < 0.5 else (["l3"] if rng.random() < 0.4 else ["l4", "l3"])
        for kind in kinds:
            dport = L.htons(int(rng.choice(PORTS[1:6]))) if kind == "l4" else 0
            nb = int(rng.integers(1, 6))
            rev = int(rng.integers(1, 65536))
            count = nb
            r = rng.random()
            if r < 0.08:
                count = 0
            elif r < 0.2:
                count = nb + 1
            put(vip, dport, 0, np.zeros(16, np.uint8), 0, count, 0, int(rng.integers(0, 3)))
            slaves = list(range(1, nb + 1))
            if rng.random() < 0.1:
                slaves[-1] = int(rng.integers(nb + 1, 40))
            for sl in slaves:
                tgt = targets[int(rng.integers(0, len(targets)))]
                pr = rng.random()
                port = 0 if pr < 0.3 else (dport if pr < 0.5 else L.htons(int(rng.integers(1, 65536))))
                bc = int(rng.integers(1, 4)) if (kind == "l3" and rng.random() < 0.5) else 0
                put(vip, dport, sl, tgt, port, bc, rev, int(rng.integers(0, 65536)))
    return np.array(keys, L.LB6_KEY), np.array(vals, L.LB6_SERVICE), np.array(vips, np.uint8)


def l4_frame6(s16, d16, sport_be, dport_be, proto):
    """Ethernet + IPv6 (nexthdr = proto) + an L4 header carrying the ports at
    offsets 0 / 2 (TCP, UDP) or an ICMPv6 echo request."""
    if proto == 58:
        l4 = bytes([128, 0]) + bytes(6)
    else:
        l4 = int(sport_be).to_bytes(2, "little") + int(dport_be).to_bytes(2, "little") + \
            bytes(16 if proto == 6 else 4)
    h = bytearray(40)
    h[0] = 0x60
    h[4:6] = len(l4).to_bytes(2, "big")
    h[6] = proto
    h[8:24] = bytes(s16)
    h[24:40] = bytes(d16)
    return bytearray(eth(0x86DD, bytes(h) + l4)), 54


def gen_classify_v6_lb_fixture(pol, lbl6s, rng):
    """The IPv6 egress path with the service step, composed from the
    reference's own steps in ipv6_l3_from_lxc order: lb6_local
    (libref_lbl6, bpf_lxc.c:108-139), then ipcache on tuple->daddr and policy
    on the dport ct_lookup6 reloads from the rewritten packet (libref_policy
    ref_classify_v6 = bpf_lxc.c:158-203).  DROP_NO_SERVICE ends the packet
    before conntrack (bpf_lxc.c:136-138), counted with METRIC_EGRESS."""
    base = gen_classify_v6_fixture(pol, rng)
    ikeys, ivals = base["ipc_keys"], base["ipc_vals"]
    pk, pe, pep = base["pol_keys"], base["pol_entries"], base["pol_ep"]
    v6 = ikeys["family"] == L.ENDPOINT_KEY_IPV6
    targets = ikeys[v6]["ip"][rng.integers(0, int(v6.sum()), 200)].astype(np.uint8)
    keys, vals, vips = gen_lb6_services(rng, 60, targets)
    n = 5000
    fe = {}
    for k in keys:
        fe.setdefault(k["address"].tobytes(), set()).add(int(k["dport"]))
    vsel = vips[rng.integers(0, len(vips), n)]
    daddr = np.where(rng.random((n, 1)) < 0.75, vsel, base["t_daddr"]).astype(np.uint8)
    dport = np.empty(n, np.uint16)
    for i in range(n):
        ports = [p for p in fe.get(daddr[i].tobytes(), ()) if p]
        dport[i] = int(rng.choice(ports)) if ports and rng.random() < 0.8 else base["t_dport"][i]
    h = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    h[:8] = [0, 1, 2, 0xFFFFFFFF, 0x7FFFFFFF, 65535, 65536, 0x80000000]
    t = {"saddr": base["t_saddr"], "daddr": daddr, "sport": rng.integers(0, 65536, n).astype(np.uint16),
         # final L4 protocols only: the frame carries no extension header, so
         # an extension-header number (0 = hop-by-hop ...) is not a tuple protocol
         "dport": dport, "proto": rng.choice(np.array([6, 6, 6, 6, 17, 17, 58, 58, 1, 47, 132], np.uint8), n),
         "hash": h, "flags": (rng.random(n) < 0.7).astype(np.uint8),
         "len": rng.integers(0, 70000, n).astype(np.uint32), "ep": rng.integers(0, 4, n).astype(np.uint16)}
    out = {}
    idv, st, npb, na = C.c_uint32(), C.c_int(), C.c_int(), C.c_int()
    hit, rn, sl, l4o, cnt = C.c_int(), C.c_uint16(), C.c_uint16(), C.c_int(), C.c_uint64()
    td = C.create_string_buffer(16)
    for ci, (gate, src) in enumerate(CONFIGS6[:2]):
        lib = lbl6s[gate]
        lib.ref_lbl6_reset()
        for k, v in zip(keys, vals):
            lib.ref_lbl6_update(b(k), b(v))
        pol.ref_reset()
        for k, v in zip(ikeys, ivals):
            pol.ref_ipcache_update(b(k), b(v))
        for k, e, ep in zip(pk, pe, pep):
            pol.ref_policy_update(int(ep), b(k), b(e))
        verdict = np.empty(n, np.int32)
        ident = np.empty(n, np.uint32)
        stage = np.empty(n, np.uint8)
        nprobes = np.empty(n, np.int32)
        lbret = np.zeros(n, np.int32)
        tdaddr = np.array(t["daddr"], np.uint8)
        for i in range(n):
            eg = int(t["flags"][i]) & 1
            da, dp, nl = t["daddr"][i].tobytes(), int(t["dport"][i]), 0
            if eg:
                fr, l4 = l4_frame6(t["saddr"][i], t["daddr"][i], t["sport"][i], t["dport"][i],
                                   int(t["proto"][i]))
                buf = (C.c_uint8 * len(fr)).from_buffer(fr)
                r = lib.ref_lbl6_run(buf, len(fr), int(t["hash"][i]), C.byref(hit), td, C.byref(rn),
                                     C.byref(sl), C.byref(l4o), C.byref(cnt))
                lbret[i], nl = r, cnt.value
                if r < 0:
                    verdict[i], ident[i], stage[i], nprobes[i] = r, 0, 6, nl
                    pol.ref_metrics_packet(int(r), int(t["len"][i]), 1)
                    continue
                da = td.raw
                tdaddr[i] = np.frombuffer(da, np.uint8)
                if int(t["proto"][i]) in (6, 17):
                    dp = int.from_bytes(bytes(fr[l4 + 2:l4 + 4]), "little")
            verdict[i] = pol.ref_classify_v6(
                t["saddr"][i].tobytes(), da, dp, int(t["proto"][i]), int(t["flags"][i]),
                int(t["len"][i]), int(t["ep"][i]), gate, src, C.byref(idv), C.byref(st),
                C.byref(npb), C.byref(na))
            ident[i], stage[i] = idv.value, st.value
            nprobes[i] = npb.value + na.value + nl
        final = np.zeros(len(pk), L.POLICY_ENTRY)
        for i, (k, ep) in enumerate(zip(pk, pep)):
            buf = C.create_string_buffer(24)
            assert pol.ref_policy_read(int(ep), b(k), buf) == 0
            final[i] = np.frombuffer(buf.raw, L.POLICY_ENTRY)[0]
        out[f"c{ci}_verdict"], out[f"c{ci}_identity"] = verdict, ident
        out[f"c{ci}_stage"], out[f"c{ci}_nprobes"] = stage, nprobes
        out[f"c{ci}_lbret"], out[f"c{ci}_tdaddr"] = lbret, tdaddr
        out[f"c{ci}_final_entries"] = final
        out[f"c{ci}_metrics"] = ref_metrics(pol)
    return dict(router_ip=base["router_ip"], ipc_keys=ikeys, ipc_vals=ivals, pol_keys=pk,
                pol_entries=pe, pol_ep=pep, lb_keys=keys, lb_vals=vals,
                configs=np.array(CONFIGS6[:2], np.int64), **{"t_" + k: v for k, v in t.items()}, **out)


# ------------------------------------------------------------- raw frames
FRAME_VARIANTS = ("_ct", "_noct", "_nover")  # oracle/Makefile FRAME_VARIANTS


def load_ref_frame():
    libs = {}
    for v in FRAME_VARIANTS:
        lib = C.CDLL(os.path.join(HERE, "_ref", f"libref_frame{v}.so"))
        lib.ref_frame_parse.argtypes = [C.c_void_p, C.c_uint32, C.c_int, C.POINTER(C.c_int),
                                        C.c_void_p, C.c_void_p, C.POINTER(C.c_uint16),
                                        C.POINTER(C.c_uint8), C.POINTER(C.c_uint8)]
        lib.ref_frame_config.argtypes = [C.c_void_p]
        lib.ref_frame_config.restype = None
        libs[v] = lib
    return libs


def gen_frames_fixture(libs, rng, n=6000):
    """Frames (synth.make_frames: every header class and truncation point)
    through the reference's endpoint-program steps before ipcache, under the
    endpoint config as written, without CONNTRACK, and without the
    SMAC/DMAC/SIP checks (harness_frame.c)."""
    from cilium_amd import synth
    f = synth.make_frames(rng, n, width=256)
    f["len"] = np.maximum(f["len"], 14).astype(np.uint32)  # the skb always holds an Ethernet header
    out = {"data": f["data"], "len": f["len"], "flags": f["flags"], "ep": f["ep"]}
    fam, dp, pr, fg = C.c_int(), C.c_uint16(), C.c_uint8(), C.c_uint8()
    sa, da = C.create_string_buffer(16), C.create_string_buffer(16)
    for v, lib in libs.items():
        cfg = C.create_string_buffer(33)
        lib.ref_frame_config(cfg)
        out[f"{v[1:]}_config"] = np.frombuffer(cfg.raw, np.uint8).copy()
        res = {k: np.zeros(n, dt) for k, dt in (("status", np.int32), ("family", np.uint8),
                                                ("dport", np.uint16), ("proto", np.uint8),
                                                ("frag", np.uint8))}
        res["saddr"] = np.zeros((n, 16), np.uint8)
        res["daddr"] = np.zeros((n, 16), np.uint8)
        for i in range(n):
            ln = int(f["len"][i])
            buf = f["data"][i].tobytes()[:ln].ljust(ln, b"\0")
            r = lib.ref_frame_parse(buf, ln, int(f["flags"][i]), C.byref(fam), sa, da,
                                    C.byref(dp), C.byref(pr), C.byref(fg))
            res["status"][i] = r
            if r == 0:
                res["family"][i], res["dport"][i] = fam.value, dp.value
                res["proto"][i], res["frag"][i] = pr.value, fg.value
                res["saddr"][i] = np.frombuffer(sa.raw, np.uint8)
                res["daddr"][i] = np.frombuffer(da.raw, np.uint8)
        for k, a in res.items():
            out[f"{v[1:]}_{k}"] = a
    return out


# ------------------------------------------------------------- conntrack
def load_ref_ct():
    lib = C.CDLL(os.path.join(HERE, "_ref", "libref_ct.so"))
    ip, u32p = C.POINTER(C.c_int), C.POINTER(C.c_uint32)
    lib.ref_ct_reset.argtypes = [C.c_size_t]
    lib.ref_ct_reset.restype = None
    lib.ref_ct_set_now.argtypes = [C.c_uint32]
    lib.ref_ct_set_now.restype = None
    lib.ref_ct_policy_update.argtypes = [C.c_int, C.c_void_p, C.c_void_p]
    lib.ref_ct_policy_read.argtypes = [C.c_int, C.c_void_p, C.c_void_p]
    lib.ref_ct_policy_delete.argtypes = [C.c_int, C.c_void_p]
    lib.ref_ct_ipcache_update.argtypes = [C.c_void_p, C.c_void_p]
    lib.ref_ct_update.argtypes = [C.c_void_p, C.c_void_p]
    lib.ref_ct_delete.argtypes = [C.c_void_p]
    lib.ref_ct_count.restype = C.c_size_t
    lib.ref_ct_entry.argtypes = [C.c_size_t, C.c_void_p, C.c_void_p]
    lib.ref_ct_classify_v4.argtypes = [C.c_uint32, C.c_uint32, C.c_uint16, C.c_uint16, C.c_uint8,
                                       C.c_uint16, C.c_uint8, C.c_uint32, C.c_int, C.c_uint32,
                                       C.c_uint32, C.c_int, ip, u32p, ip]
    lib.ref_ct_constants.argtypes = [u32p, C.c_int]
    lib.ref_ct6_update.argtypes = [C.c_void_p, C.c_void_p]
    lib.ref_ct6_delete.argtypes = [C.c_void_p]
    lib.ref_ct6_count.restype = C.c_size_t
    lib.ref_ct6_entry.argtypes = [C.c_size_t, C.c_void_p, C.c_void_p]
    lib.ref_ct_classify_v6.argtypes = [C.c_char_p, C.c_char_p, C.c_uint16, C.c_uint16, C.c_uint8,
                                       C.c_uint16, C.c_uint8, C.c_uint32, C.c_int, C.c_uint32,
                                       C.c_uint32, ip, u32p, ip]
    return lib


def ref_ct_dump(lib):
    n = lib.ref_ct_count()
    keys = np.zeros(n, L.CT4_TUPLE)
    vals = np.zeros(n, L.CT_ENTRY)
    kb, vb = C.create_string_buffer(14), C.create_string_buffer(56)
    for i in range(n):
        assert lib.ref_ct_entry(i, kb, vb) == 0
        keys[i] = np.frombuffer(kb.raw, L.CT4_TUPLE)[0]
        vals[i] = np.frombuffer(vb.raw, L.CT_ENTRY)[0]
    return L.ct_sorted(keys, vals)


def ct_tables(rng):
    ikeys, ivals = gen_ipcache_entries(rng, 300, 0, static=False)
    keep = ikeys["prefixlen"] > 32 + 4  # no catch-all: exercise the cluster/world fallback
    ikeys, ivals = ikeys[keep], ivals[keep]
    locals_be = np.array([L.ip4_be(0x0A010001 + i) for i in range(4)], np.uint32)
    remotes = np.concatenate([v4_queries_near(rng, ikeys, 80),
                              np.array([L.ip4_be(0x0A000000 | int(x)) for x in
                                        rng.integers(0, 1 << 24, 8)], np.uint32)])
    labels = np.unique(ivals["sec_label"])
    labels = labels[labels != 0]
    pk, pe, pep = [], [], []
    for ep in range(4):
        seen = set()
        for _ in range(160):
            kind = rng.integers(0, 4)
            ident = int(rng.choice(labels)) if rng.random() < 0.85 else int(rng.choice([2, 3, 0]))
            egress = int(rng.integers(0, 2))
            if kind == 0:  # L3-only
                port, proto = 0, 0
            elif kind == 3:  # ICMP echo keys (raw dport 8 or 0)
                port, proto = int(rng.choice([0, L.ntohs(8)])), 1
            else:
                port = int(rng.choice(synth.PORTS64[:12]))
                proto = int(rng.choice([6, 6, 17]))
                if kind == 2:
                    ident = 0
            k = L.policy_key(ident, port, proto, egress)
            if b(k) in seen:
                continue
            seen.add(b(k))
            pk.append(k)
            pe.append(L.policy_entry(int(rng.integers(1, 65536)) if rng.random() < 0.1 else 0))
            pep.append(ep)
    return (ikeys, ivals, locals_be, remotes, np.array(pk, L.POLICY_KEY),
            np.array(pe, L.POLICY_ENTRY), np.array(pep, np.uint16))


def ref_ct_run(lib, t, now, seclabels, src_identity=0, secctx_world=0):
    n = len(t["saddr"])
    out = {"verdict": np.empty(n, np.int32), "ct_ret": np.empty(n, np.uint8),
           "identity": np.empty(n, np.uint32), "stage": np.empty(n, np.uint8)}
    cr, idv, st = C.c_int(), C.c_uint32(), C.c_int()
    lib.ref_ct_set_now(now)
    for i in range(n):
        ep = int(t["ep"][i])
        out["verdict"][i] = lib.ref_ct_classify_v4(
            int(t["saddr"][i]), int(t["daddr"][i]), int(t["sport"][i]), int(t["dport"][i]),
            int(t["proto"][i]), int(t["l4b"][i]), int(t["flags"][i]), int(t["len"][i]), ep,
            int(seclabels[ep]), src_identity, secctx_world, C.byref(cr), C.byref(idv), C.byref(st))
        out["ct_ret"][i] = cr.value if cr.value >= 0 else L.CT_NONE
        out["identity"][i], out["stage"][i] = idv.value, st.value
    return out


def gen_ct_fixture(lib, rng):
    """Stateful path: a connection stream cut into 4
    batches run in order through the reference's conntrack + policy, with
    CT entries installed beforehand (some closing), a quarter of the policy
    keys deleted between batches 1 and 2 (denied ESTABLISHED flows lose
    their entry), and a second run at a small CT_MAP_SIZE (create failures)."""
    ikeys, ivals, locals_be, remotes, pk, pe, pep = ct_tables(rng)
    seclabels = np.array([5000 + 7 * i for i in range(4)], np.uint32)
    t = synth.make_ct_stream(rng, 700, locals_be, remotes, mean_pkts=6.0, span=0.05)
    n = len(t["saddr"])
    cuts = np.array([0, n // 5, n // 2, (3 * n) // 4, n])
    nows = np.array([100, 103, 250, 40000], np.uint32)
    # pre-installed entries: the forward key of some connections' first packets
    pre_i = rng.choice(n, 40, replace=False)
    pre_k = np.zeros(50, L.CT4_TUPLE)
    eg = (t["flags"][pre_i] & 1).astype(bool)
    pre_k["daddr"][:40] = t["saddr"][pre_i]
    pre_k["saddr"][:40] = t["daddr"][pre_i]
    pre_k["dport"][:40] = np.where(t["proto"][pre_i] == 1, 0, t["dport"][pre_i])
    pre_k["sport"][:40] = np.where(t["proto"][pre_i] == 1, 0, t["sport"][pre_i])
    pre_k["nexthdr"][:40] = t["proto"][pre_i]
    pre_k["flags"][:40] = np.where(eg, L.TUPLE_F_OUT, L.TUPLE_F_IN)
    pre_k["daddr"][40:] = rng.integers(0, 2**32, 10, dtype=np.uint64).astype(np.uint32)
    pre_k["saddr"][40:] = rng.integers(0, 2**32, 10, dtype=np.uint64).astype(np.uint32)
    pre_k["nexthdr"][40:] = 6
    pre_v = np.zeros(50, L.CT_ENTRY)
    for f in ("rx_packets", "rx_bytes", "tx_packets", "tx_bytes"):
        pre_v[f] = rng.integers(0, 1000, 50)
    pre_v["lifetime"] = rng.integers(0, 500, 50)
    pre_v["bits"] = rng.choice(np.array([0, 1, 2, 3, 16, 19], np.uint16), 50)
    pre_v["tx_flags_seen"] = rng.integers(0, 256, 50)
    pre_v["rx_flags_seen"] = rng.integers(0, 256, 50)
    pre_v["src_sec_id"] = rng.integers(0, 70000, 50)
    pre_v["last_tx_report"] = rng.integers(0, 120, 50)
    pre_v["last_rx_report"] = rng.integers(0, 120, 50)
    pol_del = rng.choice(len(pk), len(pk) // 4, replace=False)

    def load(ct_max):
        lib.ref_ct_reset(ct_max)
        for k, v in zip(ikeys, ivals):
            lib.ref_ct_ipcache_update(b(k), b(v))
        for k, e, ep in zip(pk, pe, pep):
            lib.ref_ct_policy_update(int(ep), b(k), b(e))

    load(1 << 20)
    for k, v in zip(pre_k, pre_v):
        assert lib.ref_ct_update(b(k), b(v)) == 0
    outs, dumps = [], []
    for bi in range(4):
        if bi == 2:
            for d in pol_del:  # PolicyMap.DeleteKey between batches
                assert lib.ref_ct_policy_delete(int(pep[d]), b(pk[d])) == 0
        tb = {k: v[cuts[bi]:cuts[bi + 1]] for k, v in t.items()}
        outs.append(ref_ct_run(lib, tb, int(nows[bi]), seclabels))
        dumps.append(ref_ct_dump(lib))
    res = {f"b_{f}": np.concatenate([o[f] for o in outs]) for f in outs[0]}
    res["dump_n"] = np.array([len(d[0]) for d in dumps], np.int64)
    res["dump_keys"] = np.concatenate([d[0] for d in dumps])
    res["dump_vals"] = np.concatenate([d[1] for d in dumps])
    final = np.zeros(len(pk), L.POLICY_ENTRY)
    buf = C.create_string_buffer(24)
    for i, (k, ep) in enumerate(zip(pk, pep)):
        if lib.ref_ct_policy_read(int(ep), b(k), buf) == 0:
            final[i] = np.frombuffer(buf.raw, L.POLICY_ENTRY)[0]
    res["final_entries"] = final  # deleted keys: zero

    # a small CT map: ct_create4 failures (DROP_CT_CREATE_FAILED)
    t2 = synth.make_ct_stream(rng, 200, locals_be, remotes, mean_pkts=3.0, span=0.05)
    load(64)
    o2 = ref_ct_run(lib, t2, 500, seclabels)
    d2 = ref_ct_dump(lib)
    res.update({f"s_{f}": v for f, v in o2.items()})
    res["s_dump_keys"], res["s_dump_vals"] = d2
    return dict(ipc_keys=ikeys, ipc_vals=ivals, pol_keys=pk, pol_entries=pe, pol_ep=pep,
                seclabels=seclabels, cuts=cuts, nows=nows, pre_keys=pre_k, pre_vals=pre_v,
                pol_del=np.sort(pol_del), **{"t_" + k: v for k, v in t.items()},
                **{"t2_" + k: v for k, v in t2.items()}, **res)


# ------------------------------------------------------- conntrack, IPv6
def ref_ct6_dump(lib):
    n = lib.ref_ct6_count()
    keys = np.zeros(n, L.CT6_TUPLE)
    vals = np.zeros(n, L.CT_ENTRY)
    kb, vb = C.create_string_buffer(38), C.create_string_buffer(56)
    for i in range(n):
        assert lib.ref_ct6_entry(i, kb, vb) == 0
        keys[i] = np.frombuffer(kb.raw, L.CT6_TUPLE)[0]
        vals[i] = np.frombuffer(vb.raw, L.CT_ENTRY)[0]
    return L.ct_sorted(keys, vals)


def ref_ct6_run(lib, t, now, seclabels, src_identity=0):
    n = len(t["saddr"])
    out = {"verdict": np.empty(n, np.int32), "ct_ret": np.empty(n, np.uint8),
           "identity": np.empty(n, np.uint32), "stage": np.empty(n, np.uint8)}
    cr, idv, st = C.c_int(), C.c_uint32(), C.c_int()
    lib.ref_ct_set_now(now)
    for i in range(n):
        ep = int(t["ep"][i])
        out["verdict"][i] = lib.ref_ct_classify_v6(
            t["saddr"][i].tobytes(), t["daddr"][i].tobytes(), int(t["sport"][i]),
            int(t["dport"][i]), int(t["proto"][i]), int(t["l4b"][i]), int(t["flags"][i]),
            int(t["len"][i]), ep, int(seclabels[ep]), src_identity, C.byref(cr), C.byref(idv),
            C.byref(st))
        out["ct_ret"][i] = cr.value if cr.value >= 0 else L.CT_NONE
        out["identity"][i], out["stage"][i] = idv.value, st.value
    return out


def ct6_tables(pol, rng):
    """The IPv6 stateful fixtures' tables: ipcache6 prefixes, 4 local
    endpoints (two inside ROUTER_IP's /64), remotes, per-endpoint policy."""
    router = C.create_string_buffer(16)
    pol.ref_router_ip(router)
    router = np.frombuffer(router.raw, np.uint8).copy()
    ikeys, ivals = gen_ipcache_entries(rng, 0, 260, static=False)
    keep = ikeys["prefixlen"] > 32 + 4
    ikeys, ivals = ikeys[keep], ivals[keep]
    # local endpoints: two inside the router's /64 (cluster), two outside
    locals6 = np.zeros((4, 16), np.uint8)
    for i in range(4):
        a = router.copy() if i < 2 else v6_queries_near(rng, ikeys, 1)[0]
        a[12:] = rng.integers(0, 256, 4, dtype=np.uint8)
        if i == 3:
            a[12:14] = 0  # ingress to it: reverse-NAT index 0
        locals6[i] = a
    rem = v6_queries_near(rng, ikeys, 80)
    inr = np.tile(router, (8, 1))
    inr[:, 8:] = rng.integers(0, 256, (8, 8), dtype=np.uint8)
    remotes6 = np.concatenate([rem, inr])
    labels = np.unique(ivals["sec_label"])
    labels = labels[(labels != 0) & (labels < 2**24)]
    pk, pe, pep = [], [], []
    for ep in range(4):
        seen = set()
        for _ in range(160):
            kind = rng.integers(0, 4)
            ident = int(rng.choice(labels)) if rng.random() < 0.85 else int(rng.choice([2, 3, 0]))
            egress = int(rng.integers(0, 2))
            if kind == 0:  # L3-only
                port, proto = 0, 0
            elif kind == 3:  # ICMPv6 echo keys (raw dport 128 or 0)
                port, proto = int(rng.choice([0, L.ntohs(128)])), 58
            else:
                port = int(rng.choice(synth.PORTS64[:12]))
                proto = int(rng.choice([6, 6, 17]))
                if kind == 2:
                    ident = 0
            k = L.policy_key(ident, port, proto, egress)
            if b(k) in seen:
                continue
            seen.add(b(k))
            pk.append(k)
            pe.append(L.policy_entry(int(rng.integers(1, 65536)) if rng.random() < 0.1 else 0))
            pep.append(ep)
    pk, pe, pep = (np.array(pk, L.POLICY_KEY), np.array(pe, L.POLICY_ENTRY),
                   np.array(pep, np.uint16))
    return router, ikeys, ivals, locals6, remotes6, pk, pe, pep


def gen_ct6_fixture(lib, pol, rng):
    """IPv6 stateful path (CT_MAP6): as gen_ct_fixture over
    ct_lookup6 / ct_create6 / ct_delete6 in the v6 endpoint programs' order:
    ICMPv6 echo / errors, the ingress reverse-NAT index taken from the
    destination address, ROUTER_IP /64 cluster fallback; 4 batches with
    pre-installed entries and policy deletions, a small-map run, and a run
    with a reserved ingress source identity (ipcache-resolved sources)."""
    router, ikeys, ivals, locals6, remotes6, pk, pe, pep = ct6_tables(pol, rng)
    seclabels = np.array([6000 + 11 * i for i in range(4)], np.uint32)
    t = synth.make_ct_stream(rng, 700, locals6, remotes6, mean_pkts=6.0, span=0.05)
    n = len(t["saddr"])
    cuts = np.array([0, n // 5, n // 2, (3 * n) // 4, n])
    nows = np.array([100, 103, 250, 40000], np.uint32)
    pre_i = rng.choice(n, 40, replace=False)
    pre_k = np.zeros(50, L.CT6_TUPLE)
    eg = (t["flags"][pre_i] & 1).astype(bool)
    pre_k["daddr"][:40] = t["saddr"][pre_i]
    pre_k["saddr"][:40] = t["daddr"][pre_i]
    pre_k["dport"][:40] = np.where(t["proto"][pre_i] == 58, 0, t["dport"][pre_i])
    pre_k["sport"][:40] = np.where(t["proto"][pre_i] == 58, 0, t["sport"][pre_i])
    pre_k["nexthdr"][:40] = t["proto"][pre_i]
    pre_k["flags"][:40] = np.where(eg, L.TUPLE_F_OUT, L.TUPLE_F_IN)
    pre_k["daddr"][40:] = rng.integers(0, 256, (10, 16), dtype=np.uint8)
    pre_k["saddr"][40:] = rng.integers(0, 256, (10, 16), dtype=np.uint8)
    pre_k["nexthdr"][40:] = 6
    pre_v = np.zeros(50, L.CT_ENTRY)
    for f in ("rx_packets", "rx_bytes", "tx_packets", "tx_bytes"):
        pre_v[f] = rng.integers(0, 1000, 50)
    pre_v["lifetime"] = rng.integers(0, 500, 50)
    pre_v["bits"] = rng.choice(np.array([0, 1, 2, 3, 16, 19], np.uint16), 50)
    pre_v["rev_nat_index"] = rng.integers(0, 3, 50)
    pre_v["tx_flags_seen"] = rng.integers(0, 256, 50)
    pre_v["rx_flags_seen"] = rng.integers(0, 256, 50)
    pre_v["src_sec_id"] = rng.integers(0, 70000, 50)
    pre_v["last_tx_report"] = rng.integers(0, 120, 50)
    pre_v["last_rx_report"] = rng.integers(0, 120, 50)
    pol_del = rng.choice(len(pk), len(pk) // 4, replace=False)

    def load(ct_max):
        lib.ref_ct_reset(ct_max)
        for k, v in zip(ikeys, ivals):
            lib.ref_ct_ipcache_update(b(k), b(v))
        for k, e, ep in zip(pk, pe, pep):
            lib.ref_ct_policy_update(int(ep), b(k), b(e))

    load(1 << 20)
    for k, v in zip(pre_k, pre_v):
        assert lib.ref_ct6_update(b(k), b(v)) == 0
    outs, dumps = [], []
    for bi in range(4):
        if bi == 2:
            for d in pol_del:
                assert lib.ref_ct_policy_delete(int(pep[d]), b(pk[d])) == 0
        tb = {k: v[cuts[bi]:cuts[bi + 1]] for k, v in t.items()}
        outs.append(ref_ct6_run(lib, tb, int(nows[bi]), seclabels))
        dumps.append(ref_ct6_dump(lib))
    res = {f"b_{f}": np.concatenate([o[f] for o in outs]) for f in outs[0]}
    res["dump_n"] = np.array([len(d[0]) for d in dumps], np.int64)
    res["dump_keys"] = np.concatenate([d[0] for d in dumps])
    res["dump_vals"] = np.concatenate([d[1] for d in dumps])
    final = np.zeros(len(pk), L.POLICY_ENTRY)
    buf = C.create_string_buffer(24)
    for i, (k, ep) in enumerate(zip(pk, pep)):
        if lib.ref_ct_policy_read(int(ep), b(k), buf) == 0:
            final[i] = np.frombuffer(buf.raw, L.POLICY_ENTRY)[0]
    res["final_entries"] = final
    # a small CT map (DROP_CT_CREATE_FAILED), with a reserved ingress source
    # identity: ingress sources resolve through ipcache6 (bpf_netdev.c:203-211)
    t2 = synth.make_ct_stream(rng, 200, locals6, remotes6, mean_pkts=3.0, span=0.05)
    load(64)
    o2 = ref_ct6_run(lib, t2, 500, seclabels, src_identity=2)
    d2 = ref_ct6_dump(lib)
    res.update({f"s_{f}": v for f, v in o2.items()})
    res["s_dump_keys"], res["s_dump_vals"] = d2
    return dict(ipc_keys=ikeys, ipc_vals=ivals, pol_keys=pk, pol_entries=pe, pol_ep=pep,
                router_ip=router, locals=locals6, seclabels=seclabels, cuts=cuts, nows=nows,
                pre_keys=pre_k, pre_vals=pre_v, pol_del=np.sort(pol_del),
                **{"t_" + k: v for k, v in t.items()}, **{"t2_" + k: v for k, v in t2.items()},
                **res)


# ----------------------------------- stateful service step (lb4_local + CT)
def load_ref_ctlb():
    lib = C.CDLL(os.path.join(HERE, "_ref", "libref_ctlb.so"))
    ip, u32p, u16p = C.POINTER(C.c_int), C.POINTER(C.c_uint32), C.POINTER(C.c_uint16)
    lib.ref_ctlb_reset.argtypes = [C.c_size_t]
    lib.ref_ctlb_reset.restype = None
    lib.ref_ctlb_set_now.argtypes = [C.c_uint32]
    lib.ref_ctlb_set_now.restype = None
    lib.ref_ctlb_policy_update.argtypes = [C.c_int, C.c_void_p, C.c_void_p]
    lib.ref_ctlb_policy_read.argtypes = [C.c_int, C.c_void_p, C.c_void_p]
    lib.ref_ctlb_ipcache_update.argtypes = [C.c_void_p, C.c_void_p]
    lib.ref_ctlb_svc_update.argtypes = [C.c_void_p, C.c_void_p]
    lib.ref_ctlb_svc_delete.argtypes = [C.c_void_p]
    lib.ref_ctlb_policy_delete.argtypes = [C.c_int, C.c_void_p]
    lib.ref_ctlb_ct_update.argtypes = [C.c_void_p, C.c_void_p]
    lib.ref_ctlb_svc6_update.argtypes = [C.c_void_p, C.c_void_p]
    lib.ref_ctlb_svc6_delete.argtypes = [C.c_void_p]
    lib.ref_ctlb_ct6_update.argtypes = [C.c_void_p, C.c_void_p]
    lib.ref_ctlb6_count.restype = C.c_size_t
    lib.ref_ctlb6_entry.argtypes = [C.c_size_t, C.c_void_p, C.c_void_p]
    lib.ref_ctlb_classify_v6.argtypes = [C.c_char_p, C.c_char_p, C.c_uint16, C.c_uint16, C.c_uint8,
                                         C.c_uint16, C.c_uint8, C.c_uint32, C.c_int, C.c_uint32,
                                         C.c_uint32, C.c_uint32, C.POINTER(C.c_int),
                                         C.POINTER(C.c_uint32), C.POINTER(C.c_int), C.c_char_p,
                                         C.POINTER(C.c_uint16), C.POINTER(C.c_int)]
    lib.ref_ctlb_count.restype = C.c_size_t
    lib.ref_ctlb_entry.argtypes = [C.c_size_t, C.c_void_p, C.c_void_p]
    lib.ref_ctlb_classify_v4.argtypes = [C.c_uint32, C.c_uint32, C.c_uint16, C.c_uint16, C.c_uint8,
                                         C.c_uint16, C.c_uint8, C.c_uint32, C.c_int, C.c_uint32,
                                         C.c_uint32, C.c_uint32, ip, u32p, ip, u32p, u16p, ip]
    return lib


def ref_ctlb_dump(lib):
    n = lib.ref_ctlb_count()
    keys = np.zeros(n, L.CT4_TUPLE)
    vals = np.zeros(n, L.CT_ENTRY)
    kb, vb = C.create_string_buffer(14), C.create_string_buffer(56)
    for i in range(n):
        assert lib.ref_ctlb_entry(i, kb, vb) == 0
        keys[i] = np.frombuffer(kb.raw, L.CT4_TUPLE)[0]
        vals[i] = np.frombuffer(vb.raw, L.CT_ENTRY)[0]
    return L.ct_sorted(keys, vals)


def ref_ctlb_run(lib, t, now, seclabels):
    n = len(t["saddr"])
    out = {"verdict": np.empty(n, np.int32), "ct_ret": np.empty(n, np.uint8),
           "identity": np.empty(n, np.uint32), "stage": np.empty(n, np.uint8),
           "xdaddr": np.empty(n, np.uint32), "xdport": np.empty(n, np.uint16),
           "svc_hit": np.empty(n, np.uint8)}
    cr, idv, st, xd, xp, sh = (C.c_int(), C.c_uint32(), C.c_int(), C.c_uint32(), C.c_uint16(),
                               C.c_int())
    lib.ref_ctlb_set_now(now)
    for i in range(n):
        ep = int(t["ep"][i])
        out["verdict"][i] = lib.ref_ctlb_classify_v4(
            int(t["saddr"][i]), int(t["daddr"][i]), int(t["sport"][i]), int(t["dport"][i]),
            int(t["proto"][i]), int(t["l4b"][i]), int(t["flags"][i]), int(t["len"][i]), ep,
            int(seclabels[ep]), int(t["hash"][i]), 0, C.byref(cr), C.byref(idv), C.byref(st),
            C.byref(xd), C.byref(xp), C.byref(sh))
        out["ct_ret"][i] = cr.value if 0 <= cr.value < 255 else L.CT_NONE
        out["identity"][i], out["stage"][i] = idv.value, st.value
        out["xdaddr"][i], out["xdport"][i], out["svc_hit"][i] = xd.value, xp.value, sh.value
    return out


def ctlb_stream(rng, n_conn, locals_be, remotes, lb_keys, lb_vals, vips):
    """A connection stream (synth.make_ct_stream) where a third of the
    remotes are service VIPs: egress packets to a VIP carry one of its
    service ports; replies come back from the VIP or from one of its
    backends (the reverse NAT map is empty, so both occur on the wire).
    hash = skb->hash: the flow hash of the connection's egress direction,
    re-drawn for 10 % of the packets."""
    rem = np.concatenate([remotes, np.repeat(vips, 4)]).astype(np.uint32)
    t = synth.make_ct_stream(rng, n_conn, locals_be, rem, mean_pkts=6.0, span=0.05)
    ports, backs = {}, {}
    for k, v in zip(lb_keys, lb_vals):
        a = int(k["address"])
        if int(k["dport"]):
            ports.setdefault(a, set()).add(int(k["dport"]))
        if int(k["slave"]) and int(v["target"]):
            backs.setdefault(a, []).append((int(v["target"]), int(v["port"])))
    vipset = set(int(x) for x in vips)
    eg = (t["flags"] & 1).astype(bool)
    for i in range(len(t["saddr"])):
        vip = int(t["daddr"][i]) if eg[i] else int(t["saddr"][i])
        if vip not in vipset:
            continue
        rp = int(t["dport"][i]) if eg[i] else int(t["sport"][i])
        ps = sorted(ports.get(vip, ()))
        if ps and (rp * 2654435761) % 7 != 0:  # same mapping for a connection's packets
            rp = ps[(rp * 40503) % len(ps)]
        if eg[i]:
            t["dport"][i] = rp
        else:
            t["sport"][i] = rp
            bl = backs.get(vip, [])
            if bl and (int(t["dport"][i]) * 2246822519) % 3 != 0:
                tg, tp = bl[int(t["dport"][i]) % len(bl)]
                t["saddr"][i] = tg
                if tp and t["proto"][i] in (6, 17):
                    t["sport"][i] = tp
    loc = np.where(eg, t["saddr"], t["daddr"])
    rmt = np.where(eg, t["daddr"], t["saddr"])
    lp = np.where(eg, t["sport"], t["dport"])
    rp = np.where(eg, t["dport"], t["sport"])
    h = shard.flowhash_np(loc, rmt, lp, rp, t["proto"])
    redraw = rng.random(len(h)) < 0.1
    h[redraw] = rng.integers(0, 2**32, int(redraw.sum()), dtype=np.uint64).astype(np.uint32)
    h[:6] = [0, 1, 0xFFFFFFFF, 0x7FFFFFFF, 65536, 0x80000000]
    t["hash"] = h.astype(np.uint32)
    return t


def gen_ctlb_fixture(lib, rng):
    """The stateful service step (SURVEY §8f rows 1 + 3):
    lb4_local with CONNTRACK (CT_SERVICE entries, stored slaves, the
    vanished-backend fallback with ct_update4_slave, fail-closed
    DROP_NO_SERVICE, loopback) composed with the egress conntrack path in
    bpf_lxc.c order, over 4 batches with service backends deleted and
    re-added and policy keys deleted between them, CT entries (including
    CT_SERVICE ones with odd slaves / loopback bits) installed beforehand,
    and a small-map run (service creates failing -> DROP_NO_SERVICE)."""
    ikeys, ivals, locals_be, remotes, pk, pe, pep = ct_tables(rng)
    seclabels = np.array([7000 + 13 * i for i in range(4)], np.uint32)
    targets = np.concatenate([remotes[:40], locals_be]).astype(np.uint32)
    keys, vals, vips = gen_lb_services(rng, 24, targets, locals_be)
    t = ctlb_stream(rng, 700, locals_be, remotes, keys, vals, vips)
    n = len(t["saddr"])
    cuts = np.array([0, n // 5, n // 2, (3 * n) // 4, n])
    nows = np.array([100, 103, 250, 40000], np.uint32)
    # pre-installed entries: forward keys of some packets, CT_SERVICE keys of
    # some service-bound packets (slave 0 / past the backends / loopback bit)
    eg = (t["flags"] & 1).astype(bool)
    pre_i = rng.choice(n, 30, replace=False)
    tovip = np.flatnonzero(eg & np.isin(t["daddr"], vips) & np.isin(t["proto"], [6, 17]))
    svc_i = rng.choice(tovip, min(20, len(tovip)), replace=False)
    pre_k = np.zeros(30 + len(svc_i), L.CT4_TUPLE)
    pe_ = eg[pre_i]
    pre_k["daddr"][:30] = t["saddr"][pre_i]
    pre_k["saddr"][:30] = t["daddr"][pre_i]
    pre_k["dport"][:30] = np.where(t["proto"][pre_i] == 1, 0, t["dport"][pre_i])
    pre_k["sport"][:30] = np.where(t["proto"][pre_i] == 1, 0, t["sport"][pre_i])
    pre_k["nexthdr"][:30] = t["proto"][pre_i]
    pre_k["flags"][:30] = np.where(pe_, L.TUPLE_F_OUT, L.TUPLE_F_IN)
    pre_k["daddr"][30:] = t["daddr"][svc_i]
    pre_k["saddr"][30:] = t["saddr"][svc_i]
    pre_k["dport"][30:] = t["sport"][svc_i]  # ct_lookup4's load: dport <- the L4 sport
    pre_k["sport"][30:] = t["dport"][svc_i]
    pre_k["nexthdr"][30:] = t["proto"][svc_i]
    pre_k["flags"][30:] = 4  # TUPLE_F_SERVICE
    m = len(pre_k)
    pre_v = np.zeros(m, L.CT_ENTRY)
    for f in ("rx_packets", "rx_bytes", "tx_packets", "tx_bytes"):
        pre_v[f] = rng.integers(0, 1000, m)
    pre_v["lifetime"] = rng.integers(0, 500, m)
    pre_v["bits"] = rng.choice(np.array([0, 1, 2, 3, 8, 16, 19, 24], np.uint16), m)
    pre_v["rev_nat_index"] = rng.integers(0, 3, m)
    pre_v["slave"] = rng.choice(np.array([0, 1, 2, 3, 7, 40], np.uint16), m)
    pre_v["tx_flags_seen"] = rng.integers(0, 256, m)
    pre_v["rx_flags_seen"] = rng.integers(0, 256, m)
    pre_v["src_sec_id"] = rng.integers(0, 70000, m)
    pre_v["last_tx_report"] = rng.integers(0, 120, m)
    pre_v["last_rx_report"] = rng.integers(0, 120, m)
    pol_del = rng.choice(len(pk), len(pk) // 4, replace=False)
    slaves = np.flatnonzero(keys["slave"] != 0)
    svc_del = rng.choice(slaves, len(slaves) // 3, replace=False)  # before batch 2
    svc_readd = svc_del[: len(svc_del) // 2]                        # before batch 3
    readd_vals = vals[svc_readd].copy()
    readd_vals["target"] = targets[rng.integers(0, len(targets), len(svc_readd))]
    readd_vals["port"] = np.where(rng.random(len(svc_readd)) < 0.5, 0,
                                  rng.integers(1, 65536, len(svc_readd)))

    def load(ct_max):
        lib.ref_ctlb_reset(ct_max)
        for k, v in zip(ikeys, ivals):
            lib.ref_ctlb_ipcache_update(b(k), b(v))
        for k, e, ep in zip(pk, pe, pep):
            lib.ref_ctlb_policy_update(int(ep), b(k), b(e))
        for k, v in zip(keys, vals):
            lib.ref_ctlb_svc_update(b(k), b(v))

    load(1 << 20)
    for k, v in zip(pre_k, pre_v):
        assert lib.ref_ctlb_ct_update(b(k), b(v)) == 0
    outs, dumps = [], []
    for bi in range(4):
        if bi == 2:
            for d in pol_del:  # PolicyMap.DeleteKey between batches
                assert lib.ref_ctlb_policy_delete(int(pep[d]), b(pk[d])) == 0
            for d in svc_del:
                assert lib.ref_ctlb_svc_delete(b(keys[d])) == 0
        if bi == 3:
            for d, v in zip(svc_readd, readd_vals):
                lib.ref_ctlb_svc_update(b(keys[d]), b(v))
        tb = {k: v[cuts[bi]:cuts[bi + 1]] for k, v in t.items()}
        outs.append(ref_ctlb_run(lib, tb, int(nows[bi]), seclabels))
        dumps.append(ref_ctlb_dump(lib))
    res = {f"b_{f}": np.concatenate([o[f] for o in outs]) for f in outs[0]}
    res["dump_n"] = np.array([len(d[0]) for d in dumps], np.int64)
    res["dump_keys"] = np.concatenate([d[0] for d in dumps])
    res["dump_vals"] = np.concatenate([d[1] for d in dumps])
    final = np.zeros(len(pk), L.POLICY_ENTRY)
    buf = C.create_string_buffer(24)
    for i, (k, ep) in enumerate(zip(pk, pep)):
        if lib.ref_ctlb_policy_read(int(ep), b(k), buf) == 0:
            final[i] = np.frombuffer(buf.raw, L.POLICY_ENTRY)[0]
    res["final_entries"] = final
    # a small CT map: service creates fail (DROP_NO_SERVICE), egress /
    # ingress creates fail (DROP_CT_CREATE_FAILED)
    t2 = ctlb_stream(rng, 200, locals_be, remotes, keys, vals, vips)
    load(48)
    o2 = ref_ctlb_run(lib, t2, 500, seclabels)
    d2 = ref_ctlb_dump(lib)
    res.update({f"s_{f}": v for f, v in o2.items()})
    res["s_dump_keys"], res["s_dump_vals"] = d2
    return dict(ipc_keys=ikeys, ipc_vals=ivals, pol_keys=pk, pol_entries=pe, pol_ep=pep,
                lb_keys=keys, lb_vals=vals, vips=vips, svc_del=svc_del, svc_readd=svc_readd,
                readd_vals=readd_vals, locals=locals_be,
                seclabels=seclabels, cuts=cuts, nows=nows, pre_keys=pre_k, pre_vals=pre_v,
                pol_del=np.sort(pol_del), **{"t_" + k: v for k, v in t.items()},
                **{"t2_" + k: v for k, v in t2.items()}, **res)


def ref_ctlb6_dump(lib):
    n = lib.ref_ctlb6_count()
    keys = np.zeros(n, L.CT6_TUPLE)
    vals = np.zeros(n, L.CT_ENTRY)
    kb, vb = C.create_string_buffer(38), C.create_string_buffer(56)
    for i in range(n):
        assert lib.ref_ctlb6_entry(i, kb, vb) == 0
        keys[i] = np.frombuffer(kb.raw, L.CT6_TUPLE)[0]
        vals[i] = np.frombuffer(vb.raw, L.CT_ENTRY)[0]
    return L.ct_sorted(keys, vals)


def ref_ctlb6_run(lib, t, now, seclabels):
    n = len(t["saddr"])
    out = {"verdict": np.empty(n, np.int32), "ct_ret": np.empty(n, np.uint8),
           "identity": np.empty(n, np.uint32), "stage": np.empty(n, np.uint8),
           "xdaddr": np.empty((n, 16), np.uint8), "xdport": np.empty(n, np.uint16),
           "svc_hit": np.empty(n, np.uint8)}
    cr, idv, st, xp, sh = C.c_int(), C.c_uint32(), C.c_int(), C.c_uint16(), C.c_int()
    xd = C.create_string_buffer(16)
    lib.ref_ctlb_set_now(now)
    for i in range(n):
        ep = int(t["ep"][i])
        out["verdict"][i] = lib.ref_ctlb_classify_v6(
            t["saddr"][i].tobytes(), t["daddr"][i].tobytes(), int(t["sport"][i]), int(t["dport"][i]),
            int(t["proto"][i]), int(t["l4b"][i]), int(t["flags"][i]), int(t["len"][i]), ep,
            int(seclabels[ep]), int(t["hash"][i]), 0, C.byref(cr), C.byref(idv), C.byref(st), xd,
            C.byref(xp), C.byref(sh))
        out["ct_ret"][i] = cr.value if 0 <= cr.value < 255 else L.CT_NONE
        out["identity"][i], out["stage"][i] = idv.value, st.value
        out["xdaddr"][i] = np.frombuffer(xd.raw, np.uint8)
        out["xdport"][i], out["svc_hit"][i] = xp.value, sh.value
    return out


def ctlb6_stream(rng, n_conn, locals6, remotes6, lb_keys, lb_vals, vips):
    """ctlb_stream over IPv6 addresses ((n, 16) uint8)."""
    rem = np.concatenate([remotes6, np.repeat(vips, 4, axis=0)]).astype(np.uint8)
    t = synth.make_ct_stream(rng, n_conn, locals6, rem, mean_pkts=6.0, span=0.05)
    ports, backs = {}, {}
    for k, v in zip(lb_keys, lb_vals):
        a = k["address"].tobytes()
        if int(k["dport"]):
            ports.setdefault(a, set()).add(int(k["dport"]))
        if int(k["slave"]) and v["target"].any():
            backs.setdefault(a, []).append((v["target"].copy(), int(v["port"])))
    vipset = set(v.tobytes() for v in vips)
    eg = (t["flags"] & 1).astype(bool)
    for i in range(len(t["saddr"])):
        vip = (t["daddr"][i] if eg[i] else t["saddr"][i]).tobytes()
        if vip not in vipset:
            continue
        rp = int(t["dport"][i]) if eg[i] else int(t["sport"][i])
        ps = sorted(ports.get(vip, ()))
        if ps and (rp * 2654435761) % 7 != 0:
            rp = ps[(rp * 40503) % len(ps)]
        if eg[i]:
            t["dport"][i] = rp
        else:
            t["sport"][i] = rp
            bl = backs.get(vip, [])
            if bl and (int(t["dport"][i]) * 2246822519) % 3 != 0:
                tg, tp = bl[int(t["dport"][i]) % len(bl)]
                t["saddr"][i] = tg
                if tp and t["proto"][i] in (6, 17):
                    t["sport"][i] = tp
    loc = np.where(eg[:, None], t["saddr"], t["daddr"])
    rmt = np.where(eg[:, None], t["daddr"], t["saddr"])
    lp = np.where(eg, t["sport"], t["dport"])
    rp = np.where(eg, t["dport"], t["sport"])
    h = shard.flowhash_np(shard.fold6_np(loc), shard.fold6_np(rmt), lp, rp, t["proto"])
    redraw = rng.random(len(h)) < 0.1
    h[redraw] = rng.integers(0, 2**32, int(redraw.sum()), dtype=np.uint64).astype(np.uint32)
    h[:6] = [0, 1, 0xFFFFFFFF, 0x7FFFFFFF, 65536, 0x80000000]
    t["hash"] = h.astype(np.uint32)
    return t


def gen_ctlb6_fixture(lib, pol, rng):
    """The IPv6 stateful service step (lb6_local with CONNTRACK, lb.h:426-483)
    composed with the v6 egress conntrack path in ipv6_l3_from_lxc order, as
    gen_ctlb_fixture: 4 batches with backends deleted / re-added and policy
    keys deleted, CT_SERVICE entries installed beforehand (slave 0 / past the
    backends / lb_loopback), a small-map run."""
    router, ikeys, ivals, locals6, remotes6, pk, pe, pep = ct6_tables(pol, rng)
    seclabels = np.array([8000 + 17 * i for i in range(4)], np.uint32)
    targets = np.concatenate([remotes6[:40], locals6]).astype(np.uint8)
    keys, vals, vips = gen_lb6_services(rng, 24, targets)
    t = ctlb6_stream(rng, 700, locals6, remotes6, keys, vals, vips)
    n = len(t["saddr"])
    cuts = np.array([0, n // 5, n // 2, (3 * n) // 4, n])
    nows = np.array([100, 103, 250, 40000], np.uint32)
    eg = (t["flags"] & 1).astype(bool)
    pre_i = rng.choice(n, 30, replace=False)
    vipset = set(v.tobytes() for v in vips)
    tovip = np.flatnonzero(eg & np.array([d.tobytes() in vipset for d in t["daddr"]]) &
                           np.isin(t["proto"], [6, 17]))
    svc_i = rng.choice(tovip, min(20, len(tovip)), replace=False)
    pre_k = np.zeros(30 + len(svc_i), L.CT6_TUPLE)
    pe_ = eg[pre_i]
    pre_k["daddr"][:30] = t["saddr"][pre_i]
    pre_k["saddr"][:30] = t["daddr"][pre_i]
    pre_k["dport"][:30] = np.where(t["proto"][pre_i] == 58, 0, t["dport"][pre_i])
    pre_k["sport"][:30] = np.where(t["proto"][pre_i] == 58, 0, t["sport"][pre_i])
    pre_k["nexthdr"][:30] = t["proto"][pre_i]
    pre_k["flags"][:30] = np.where(pe_, L.TUPLE_F_OUT, L.TUPLE_F_IN)
    pre_k["daddr"][30:] = t["daddr"][svc_i]
    pre_k["saddr"][30:] = t["saddr"][svc_i]
    pre_k["dport"][30:] = t["sport"][svc_i]
    pre_k["sport"][30:] = t["dport"][svc_i]
    pre_k["nexthdr"][30:] = t["proto"][svc_i]
    pre_k["flags"][30:] = 4  # TUPLE_F_SERVICE
    m = len(pre_k)
    pre_v = np.zeros(m, L.CT_ENTRY)
    for f in ("rx_packets", "rx_bytes", "tx_packets", "tx_bytes"):
        pre_v[f] = rng.integers(0, 1000, m)
    pre_v["lifetime"] = rng.integers(0, 500, m)
    pre_v["bits"] = rng.choice(np.array([0, 1, 2, 3, 8, 16, 19, 24], np.uint16), m)
    pre_v["rev_nat_index"] = rng.integers(0, 3, m)
    pre_v["slave"] = rng.choice(np.array([0, 1, 2, 3, 7, 40], np.uint16), m)
    pre_v["tx_flags_seen"] = rng.integers(0, 256, m)
    pre_v["rx_flags_seen"] = rng.integers(0, 256, m)
    pre_v["src_sec_id"] = rng.integers(0, 70000, m)
    pre_v["last_tx_report"] = rng.integers(0, 120, m)
    pre_v["last_rx_report"] = rng.integers(0, 120, m)
    pol_del = rng.choice(len(pk), len(pk) // 4, replace=False)
    slaves = np.flatnonzero(keys["slave"] != 0)
    svc_del = rng.choice(slaves, len(slaves) // 3, replace=False)
    svc_readd = svc_del[: len(svc_del) // 2]
    readd_vals = vals[svc_readd].copy()
    readd_vals["target"] = targets[rng.integers(0, len(targets), len(svc_readd))]
    readd_vals["port"] = np.where(rng.random(len(svc_readd)) < 0.5, 0,
                                  rng.integers(1, 65536, len(svc_readd)))

    def load(ct_max):
        lib.ref_ctlb_reset(ct_max)
        for k, v in zip(ikeys, ivals):
            lib.ref_ctlb_ipcache_update(b(k), b(v))
        for k, e, ep in zip(pk, pe, pep):
            lib.ref_ctlb_policy_update(int(ep), b(k), b(e))
        for k, v in zip(keys, vals):
            lib.ref_ctlb_svc6_update(b(k), b(v))

    load(1 << 20)
    for k, v in zip(pre_k, pre_v):
        assert lib.ref_ctlb_ct6_update(b(k), b(v)) == 0
    outs, dumps = [], []
    for bi in range(4):
        if bi == 2:
            for d in pol_del:
                assert lib.ref_ctlb_policy_delete(int(pep[d]), b(pk[d])) == 0
            for d in svc_del:
                assert lib.ref_ctlb_svc6_delete(b(keys[d])) == 0
        if bi == 3:
            for d, v in zip(svc_readd, readd_vals):
                lib.ref_ctlb_svc6_update(b(keys[d]), b(v))
        tb = {k: v[cuts[bi]:cuts[bi + 1]] for k, v in t.items()}
        outs.append(ref_ctlb6_run(lib, tb, int(nows[bi]), seclabels))
        dumps.append(ref_ctlb6_dump(lib))
    res = {f"b_{f}": np.concatenate([o[f] for o in outs]) for f in outs[0]}
    res["dump_n"] = np.array([len(d[0]) for d in dumps], np.int64)
    res["dump_keys"] = np.concatenate([d[0] for d in dumps])
    res["dump_vals"] = np.concatenate([d[1] for d in dumps])
    final = np.zeros(len(pk), L.POLICY_ENTRY)
    buf = C.create_string_buffer(24)
    for i, (k, ep) in enumerate(zip(pk, pep)):
        if lib.ref_ctlb_policy_read(int(ep), b(k), buf) == 0:
            final[i] = np.frombuffer(buf.raw, L.POLICY_ENTRY)[0]
    res["final_entries"] = final
    t2 = ctlb6_stream(rng, 200, locals6, remotes6, keys, vals, vips)
    load(48)
    o2 = ref_ctlb6_run(lib, t2, 500, seclabels)
    d2 = ref_ctlb6_dump(lib)
    res.update({f"s_{f}": v for f, v in o2.items()})
    res["s_dump_keys"], res["s_dump_vals"] = d2
    return dict(ipc_keys=ikeys, ipc_vals=ivals, pol_keys=pk, pol_entries=pe, pol_ep=pep,
                router_ip=router, locals=locals6, lb_keys=keys, lb_vals=vals, vips=vips,
                svc_del=svc_del, svc_readd=svc_readd, readd_vals=readd_vals,
                seclabels=seclabels, cuts=cuts, nows=nows, pre_keys=pre_k, pre_vals=pre_v,
                pol_del=np.sort(pol_del), **{"t_" + k: v for k, v in t.items()},
                **{"t2_" + k: v for k, v in t2.items()}, **res)


def save(name, d):
    path = os.path.join(OUT, name)
    np.savez_compressed(path, **d)
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def main():
    os.makedirs(OUT, exist_ok=True)
    pol, xdp = load_ref()
    # the reference's own host unit test (test/bpf/unit-test.c) must pass as built
    subprocess.run([os.path.join(HERE, "_ref", "unit-test")], check=True)
    consts = (C.c_uint32 * 16)()
    k = pol.ref_constants(consts, 16)
    manifest = {"generator": "oracle/gen_golden.py", "seed": SEED,
                "reference": "sunxiaojun2014/cilium @ VERSION 1.2.90 (bpf/ compiled as host C)",
                "constants": [int(consts[i]) for i in range(k)], "files": {}}
    rng = np.random.Generator(np.random.PCG64(SEED))
    manifest["files"]["policy_cascade.npz"] = save("policy_cascade.npz", gen_policy_fixture(pol, rng))
    manifest["files"]["ipcache_lpm.npz"] = save("ipcache_lpm.npz", gen_ipcache_fixture(pol, rng))
    manifest["files"]["classify_v4.npz"] = save("classify_v4.npz", gen_classify_fixture(pol, rng))
    manifest["files"]["xdp_prefilter.npz"] = save("xdp_prefilter.npz", gen_xdp_fixture(xdp, rng))
    manifest["files"]["classify_v6.npz"] = save("classify_v6.npz", gen_classify_v6_fixture(pol, rng))
    # service load balancer; a separate stream keeps the
    # fixtures above byte-identical to earlier generations
    lbvars, lbls = load_ref_lb()
    rng_lb = np.random.Generator(np.random.PCG64(SEED + 0x1B))
    manifest["files"]["lb4.npz"] = save("lb4.npz", gen_lb_fixture(lbvars, lbls, rng_lb))
    manifest["files"]["classify_v4_lb.npz"] = save(
        "classify_v4_lb.npz", gen_classify_lb_fixture(pol, lbls, rng_lb))
    # raw frames, its own stream
    rng_fr = np.random.Generator(np.random.PCG64(SEED + 0xF2))
    manifest["files"]["frames.npz"] = save("frames.npz", gen_frames_fixture(load_ref_frame(), rng_fr))
    # conntrack, its own stream
    rng_ct = np.random.Generator(np.random.PCG64(SEED + 0xC7))
    manifest["files"]["ct4.npz"] = save("ct4.npz", gen_ct_fixture(load_ref_ct(), rng_ct))
    # IPv6 service translation (SURVEY §8f row 1 widened to IPv6), its own stream
    rng_lb6 = np.random.Generator(np.random.PCG64(SEED + 0x6B))
    manifest["files"]["classify_v6_lb.npz"] = save(
        "classify_v6_lb.npz", gen_classify_v6_lb_fixture(pol, load_ref_lbl6(), rng_lb6))
    # IPv6 conntrack (CT_MAP6), its own stream
    rng_ct6 = np.random.Generator(np.random.PCG64(SEED + 0xC6))
    manifest["files"]["ct6.npz"] = save("ct6.npz", gen_ct6_fixture(load_ref_ct(), pol, rng_ct6))
    # the stateful service step (lb4_local with CONNTRACK), its own stream
    rng_ctlb = np.random.Generator(np.random.PCG64(SEED + 0xCB))
    manifest["files"]["ctlb4.npz"] = save("ctlb4.npz", gen_ctlb_fixture(load_ref_ctlb(), rng_ctlb))
    # the IPv6 stateful service step (lb6_local with CONNTRACK), its own stream
    rng_ctlb6 = np.random.Generator(np.random.PCG64(SEED + 0xCC))
    manifest["files"]["ctlb6.npz"] = save("ctlb6.npz", gen_ctlb6_fixture(load_ref_ctlb(), pol, rng_ctlb6))
    # config 5 whole (the XDP prefilter in front of the ingress tuples), its own stream
    rng_cas = np.random.Generator(np.random.PCG64(SEED + 0xCA))
    manifest["files"]["cascade_v4.npz"] = save("cascade_v4.npz", gen_cascade_fixture(pol, xdp, lbls, rng_cas))
    with open(os.path.join(OUT, "MANIFEST.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(json.dumps(manifest, indent=1))


if __name__ == "__main__":
    main()
