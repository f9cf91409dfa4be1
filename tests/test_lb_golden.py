"""Pin the CPU restatement of the service load balancer (oracle/cgpu_oracle.c
or_lb4 / or_classify_v4_lb) to the reference.

tests/golden/lb4.npz and classify_v4_lb.npz were produced by the reference's
own bpf/bpf_lb.c (handle_ipv4, built with LB_L3+LB_L4, LB_L3 only and LB_L4
only) and bpf/lib/lb.h lb4_local under the endpoint config, compiled as host
C with mocked maps and helpers (oracle/ref/harness_lb*.c).  skb->hash is an
input column (the kernel's flow hash is not in the reference: SURVEY §8c).
Every check is bit-exact.
"""
import numpy as np
import pytest

from cilium_amd import layouts as L
from oracle import Oracle

VARIANTS = {"both": (1, 1), "l3": (1, 0), "l4": (0, 1)}


def _lb_oracle(g, l3=1, l4=1, prefix=""):
    o = Oracle(lb_l3=l3, lb_l4=l4)
    for k, v in zip(g[prefix + "keys"], g[prefix + "vals"]):
        assert o.lb_update(k, v) == 0
    return o


def _tuples(g):
    return {k[2:]: g[k] for k in g.files if k.startswith("t_")}


@pytest.mark.parametrize("variant", sorted(VARIANTS))
def test_lb_netdev_vs_reference(golden, variant):
    g = golden("lb4.npz")
    o = _lb_oracle(g, *VARIANTS[variant])
    out, probes = o.lb4(_tuples(g), L.LB_NETDEV)
    np.testing.assert_array_equal(out["ret"], g[f"nd_{variant}_ret"])
    np.testing.assert_array_equal(out["daddr"], g[f"nd_{variant}_daddr"])
    np.testing.assert_array_equal(out["dport"], g[f"nd_{variant}_dport"])
    assert probes == int(g[f"nd_{variant}_lookups"].sum())
    # every outcome occurs in the fixture
    assert {L.TC_ACT_OK, L.TC_ACT_REDIRECT, L.DROP_NO_SERVICE} <= set(out["ret"].tolist())


@pytest.mark.parametrize("ct", [1, 0])
def test_lb_lxc_vs_reference(golden, ct):
    """lb4_local with CONNTRACK (its CT_SERVICE lookup rejects protocols other
    than ICMP/TCP/UDP as DROP_NO_SERVICE) and without (conntrack.h stubs)."""
    g = golden("lb4.npz")
    o = _lb_oracle(g)
    o.configure(ct_proto_gate=ct)
    out, probes = o.lb4(_tuples(g), L.LB_LXC)
    px = "lx_" if ct else "lxnoct_"
    g = {k[len(px):] if k.startswith(px) else k: g[k] for k in g.files if not k.startswith("lx")
         or k.startswith(px)}
    g = {("lx_" + k if k in ("ret", "svc_hit", "loopback", "tdaddr", "saddr", "daddr", "dport",
                             "rev_nat", "slave", "lookups") else k): v for k, v in g.items()}
    ref = np.where(g["lx_ret"] < 0, g["lx_ret"],
                   np.where(g["lx_svc_hit"] == 1, 1 + g["lx_loopback"].astype(np.int32), 0))
    np.testing.assert_array_equal(out["ret"], ref)
    np.testing.assert_array_equal(out["tdaddr"], g["lx_tdaddr"])
    np.testing.assert_array_equal(out["saddr"], g["lx_saddr"])
    np.testing.assert_array_equal(out["daddr"], g["lx_daddr"])
    np.testing.assert_array_equal(out["dport"], g["lx_dport"])
    ok = g["lx_ret"] >= 0
    np.testing.assert_array_equal(out["rev_nat"][ok], g["lx_rev_nat"][ok])
    np.testing.assert_array_equal(out["slave"][ok], g["lx_slave"][ok])
    assert probes == int(g["lx_lookups"].sum())
    # the fixture reaches lb4_local's fallback (4 lookups) and the loopback NAT
    assert (g["lx_lookups"] == 4).any() and (ref == L.LB_XLATED_LOOPBACK).any()


def test_flow_hash_matches_sharder():
    from cilium_amd.shard import flowhash_np
    rng = np.random.default_rng(3)
    n = 2000
    cols = [rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32),
            rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32),
            rng.integers(0, 65536, n).astype(np.uint16), rng.integers(0, 65536, n).astype(np.uint16),
            rng.integers(0, 256, n).astype(np.uint8)]
    o = Oracle()
    exp = flowhash_np(*cols)
    got = np.array([o.flow_hash(*(int(c[i]) for c in cols)) for i in range(n)], np.uint32)
    np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize("ci", range(2))
def test_classify_v4_lb_vs_reference(golden, ci):
    g = golden("classify_v4_lb.npz")
    gate, src, sw = (int(x) for x in g["configs"][ci])
    o = Oracle(ct_proto_gate=gate, ingress_src_identity=src, ingress_secctx_world=sw)
    for k, v in zip(g["ipc_keys"], g["ipc_vals"]):
        assert o.ipcache_update(k, v) == 0
    for k, e, ep in zip(g["pol_keys"], g["pol_entries"], g["pol_ep"]):
        assert o.policy_update(int(ep), k, e) == 0
    for k, v in zip(g["lb_keys"], g["lb_vals"]):
        assert o.lb_update(k, v) == 0
    t = _tuples(g)
    v, idt, st, probes = o.classify_v4_lb(t)
    np.testing.assert_array_equal(v, g[f"c{ci}_verdict"])
    np.testing.assert_array_equal(idt, g[f"c{ci}_identity"])
    np.testing.assert_array_equal(st, g[f"c{ci}_stage"])
    assert probes == int(g[f"c{ci}_nprobes"].sum())
    for k, ep, fe in zip(g["pol_keys"], g["pol_ep"], g[f"c{ci}_final_entries"]):
        rc, raw = o.policy_lookup(int(ep), k)
        got = np.frombuffer(raw, L.POLICY_ENTRY)[0]
        assert (int(got["packets"]), int(got["bytes"])) == (int(fe["packets"]), int(fe["bytes"]))
    # metrics: drop reasons (incl. 158 egress) and forwards, from the
    # reference's update_metrics call sites
    np.testing.assert_array_equal(o.metrics(), g[f"c{ci}_metrics"])
    assert (st == 6).sum() > 0


def _cascade_oracle(g, ci, **extra):
    gate, src, sw = (int(x) for x in g["configs"][ci])
    o = Oracle(ct_proto_gate=gate, ingress_src_identity=src, ingress_secctx_world=sw, **extra)
    for k, v in zip(g["ipc_keys"], g["ipc_vals"]):
        assert o.ipcache_update(k, v) == 0
    for k, e, ep in zip(g["pol_keys"], g["pol_entries"], g["pol_ep"]):
        assert o.policy_update(int(ep), k, e) == 0
    for k, v in zip(g["lb_keys"], g["lb_vals"]):
        assert o.lb_update(k, v) == 0
    for w, name in ((0, "dyn4"), (1, "fix4")):
        for k in g[name]:
            assert o.cidr_update(w, k) == 0
    for k in g["endpoints"]:
        assert o.endpoint_update(k) == 0
    return o


@pytest.mark.parametrize("ci", range(2))
def test_classify_v4_cascade_vs_reference(golden, ci):
    """BASELINE config 5 whole: tests/golden/cascade_v4.npz composes the
    reference's XDP program (libref_xdp: bpf_xdp.c check_v4 on the ingress
    packets' frames) with its ingress decision (libref_policy) and, for
    egress packets, its service step (libref_lbl) and egress decision.  The
    restatement or_classify_v4_cascade reproduces every verdict (an XDP drop:
    CGPU_VERDICT_XDP_DROP, stage 8), identity, stage, lookup count, counter
    and metric."""
    g = golden("cascade_v4.npz")
    o = _cascade_oracle(g, ci)
    t = _tuples(g)
    v, idt, st, probes = o.classify_v4_cascade(t)
    np.testing.assert_array_equal(v, g[f"c{ci}_verdict"])
    np.testing.assert_array_equal(idt, g[f"c{ci}_identity"])
    np.testing.assert_array_equal(st, g[f"c{ci}_stage"])
    assert probes == int(g[f"c{ci}_nprobes"].sum())
    for k, ep, fe in zip(g["pol_keys"], g["pol_ep"], g[f"c{ci}_final_entries"]):
        rc, raw = o.policy_lookup(int(ep), k)
        got = np.frombuffer(raw, L.POLICY_ENTRY)[0]
        assert (int(got["packets"]), int(got["bytes"])) == (int(fe["packets"]), int(fe["bytes"]))
    np.testing.assert_array_equal(o.metrics(), g[f"c{ci}_metrics"])
    xd = v == L.VERDICT_XDP_DROP
    ing = (t["flags"] & 1) == 0
    # both XDP outcomes, both deny maps and the endpoint check all decide some packets
    assert xd.sum() > 500 and (ing & ~xd).sum() > 500 and not xd[~ing].any()
    assert set(np.unique(g["xdp_probes"][ing & xd]).tolist()) >= {1, 2, 3}
    # the fast LPM of the optimized CPU baseline gives the same answers
    o.set_fast(True)
    v2, _, _, _ = o.classify_v4_cascade(t, nthreads=3)
    np.testing.assert_array_equal(v2, g[f"c{ci}_verdict"])


@pytest.mark.parametrize("ci", range(2))
def test_classify_v6_lb_vs_reference(golden, ci):
    """the IPv6 egress path with lb6_local in front (bpf_lxc.c:108-203):
    tests/golden/classify_v6_lb.npz composes libref_lbl6 (lib/lb.h's IPv6
    service step with and without CONNTRACK) and libref_policy's v6 decision"""
    g = golden("classify_v6_lb.npz")
    gate, src = (int(x) for x in g["configs"][ci])
    o = Oracle(ct_proto_gate=gate, ingress_src_identity=src, router_ip=g["router_ip"].tobytes())
    for k, v in zip(g["ipc_keys"], g["ipc_vals"]):
        assert o.ipcache_update(k, v) == 0
    for k, e, ep in zip(g["pol_keys"], g["pol_entries"], g["pol_ep"]):
        assert o.policy_update(int(ep), k, e) == 0
    for k, v in zip(g["lb_keys"], g["lb_vals"]):
        assert o.lb6_update(k, v) == 0
    t = _tuples(g)
    v, idt, st, probes = o.classify_v6_lb(t, nthreads=3)
    np.testing.assert_array_equal(v, g[f"c{ci}_verdict"])
    np.testing.assert_array_equal(idt, g[f"c{ci}_identity"])
    np.testing.assert_array_equal(st, g[f"c{ci}_stage"])
    assert probes == int(g[f"c{ci}_nprobes"].sum())
    for k, ep, fe in zip(g["pol_keys"], g["pol_ep"], g[f"c{ci}_final_entries"]):
        rc, raw = o.policy_lookup(int(ep), k)
        got = np.frombuffer(raw, L.POLICY_ENTRY)[0]
        assert (int(got["packets"]), int(got["bytes"])) == (int(fe["packets"]), int(fe["bytes"]))
    np.testing.assert_array_equal(o.metrics(), g[f"c{ci}_metrics"])
    assert (st == 6).sum() > 0 and (g[f"c{ci}_tdaddr"] != g["t_daddr"]).any()


def test_flow_hash6_three_ways():
    """cgpu_flow_hash6 (the library, host side), or_flow_hash6 (restatement)
    and shard.flowhash6_np (sharder / synthetic traffic) agree"""
    from cilium_amd.engine import Engine
    from cilium_amd.shard import flowhash6_np
    rng = np.random.default_rng(6)
    n = 300
    s16 = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    d16 = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    sp, dp = rng.integers(0, 65536, (2, n)).astype(np.uint16)
    pr = rng.integers(0, 256, n).astype(np.uint8)
    exp = flowhash6_np(s16, d16, sp, dp, pr)
    e, o = Engine(device=-1), Oracle()
    for i in range(n):
        args = (s16[i].tobytes(), d16[i].tobytes(), int(sp[i]), int(dp[i]), int(pr[i]))
        assert e.flow_hash6(*args) == o.flow_hash6(*args) == int(exp[i])
    e.close()
