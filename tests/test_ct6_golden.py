"""Pin the CPU restatement of IPv6 stateful conntrack (oracle/cgpu_oracle.c
or_classify_v6_ct, SURVEY §8f row 3, cilium_ct6_global) to the reference.

tests/golden/ct6.npz was produced by the reference's own bpf/lib/conntrack.h
(ct_lookup6 :288-412, ct_create6 :588-639, ct_delete6 :564-570), policy.h and
eps.h compiled as host C under the endpoint config and driven packet by packet
in the order of ipv6_l3_from_lxc / ipv6_policy (bpf_lxc.c:108-203, :731-800;
oracle/ref/harness_ct.c ref_ct_classify_v6): ICMPv6 echo (128 / 129), errors
(1-4) related to a connection, other ICMPv6 types, TCP closing by the
union-tcp_flags quirk, the ingress reverse-NAT index taken from the
destination address, the ROUTER_IP /64 cluster fallback.  4 batches with CT
entries installed beforehand and policy keys deleted between batches 1 and 2;
a second run on a 64-entry map with a reserved ingress source identity.
Bit-exact: verdict, ct_lookup6 result, identity, stage, the whole CT map after
every batch and the policy entry counters.
"""
import numpy as np

from cilium_amd import layouts as L
from oracle import Oracle


def ct6_oracle(g, ct_max=1 << 20, src_identity=0):
    o = Oracle(router_ip=g["router_ip"].tobytes(), ingress_src_identity=src_identity)
    o.ct6_set_max(ct_max)
    for k, v in zip(g["ipc_keys"], g["ipc_vals"]):
        assert o.ipcache_update(k, v) == 0
    for k, e, ep in zip(g["pol_keys"], g["pol_entries"], g["pol_ep"]):
        assert o.policy_update(int(ep), k, e) == 0
    for ep, sl in enumerate(g["seclabels"]):
        assert o.lxc_update(ep, L.lxc_info(b"\0" * 6, 0, b"\0" * 16, 0, int(sl))) == 0
    return o


def stream(g, prefix="t_"):
    return {k[len(prefix):]: g[k] for k in g.files if k.startswith(prefix)}


def test_ct6_layout():
    assert L.CT6_TUPLE.itemsize == 38 and L.CT_ENTRY.itemsize == 56


def test_ct6_stream_vs_reference(golden):
    g = golden("ct6.npz")
    o = ct6_oracle(g)
    for k, v in zip(g["pre_keys"], g["pre_vals"]):
        assert o.ct6_update(k, v) == 0
    t = stream(g)
    cuts, nows = g["cuts"], g["nows"]
    off = 0
    for bi in range(4):
        if bi == 2:
            for d in g["pol_del"]:
                assert o.policy_delete(int(g["pol_ep"][d]), g["pol_keys"][d]) == 0
        sl = slice(int(cuts[bi]), int(cuts[bi + 1]))
        tb = {k: v[sl] for k, v in t.items()}
        v, cr, idt, st, _ = o.classify_v6_ct(tb, int(nows[bi]))
        np.testing.assert_array_equal(v, g["b_verdict"][sl], err_msg=f"batch {bi}")
        np.testing.assert_array_equal(cr, g["b_ct_ret"][sl], err_msg=f"batch {bi}")
        np.testing.assert_array_equal(idt, g["b_identity"][sl], err_msg=f"batch {bi}")
        np.testing.assert_array_equal(st, g["b_stage"][sl], err_msg=f"batch {bi}")
        n = int(g["dump_n"][bi])
        keys, vals = o.ct6_dump()
        np.testing.assert_array_equal(keys, g["dump_keys"][off:off + n], err_msg=f"batch {bi}")
        np.testing.assert_array_equal(vals, g["dump_vals"][off:off + n], err_msg=f"batch {bi}")
        off += n
    deleted = set(g["pol_del"].tolist())
    for i, (k, ep, fe) in enumerate(zip(g["pol_keys"], g["pol_ep"], g["final_entries"])):
        rc, raw = o.policy_lookup(int(ep), k)
        if i in deleted:
            assert rc != 0
            continue
        got = np.frombuffer(raw, L.POLICY_ENTRY)[0]
        assert (got["packets"], got["bytes"]) == (fe["packets"], fe["bytes"])
    cr, v = g["b_ct_ret"], g["b_verdict"]
    for s in (L.CT_NEW, L.CT_ESTABLISHED, L.CT_REPLY, L.CT_RELATED, L.CT_NONE):
        assert (cr == s).sum() > 0, s
    assert (v == L.DROP_POLICY).sum() > 0 and (v == 0).sum() > 0 and (v > 0).sum() > 0
    assert ((cr == L.CT_REPLY) & (g["b_stage"] == 0) & (v == 0)).sum() > 0
    assert ((cr == L.CT_ESTABLISHED) & (v == L.DROP_POLICY)).sum() > 0
    # ingress entries carry the reverse-NAT index of the destination address
    assert (g["dump_vals"]["rev_nat_index"] > 2).sum() > 0


def test_ct6_small_map_vs_reference(golden):
    g = golden("ct6.npz")
    o = ct6_oracle(g, ct_max=64, src_identity=2)
    t = stream(g, "t2_")
    v, cr, idt, st, _ = o.classify_v6_ct(t, 500)
    np.testing.assert_array_equal(v, g["s_verdict"])
    np.testing.assert_array_equal(cr, g["s_ct_ret"])
    np.testing.assert_array_equal(idt, g["s_identity"])
    np.testing.assert_array_equal(st, g["s_stage"])
    keys, vals = o.ct6_dump()
    np.testing.assert_array_equal(keys, g["s_dump_keys"])
    np.testing.assert_array_equal(vals, g["s_dump_vals"])
    assert (g["s_verdict"] == L.DROP_CT_CREATE_FAILED).sum() > 0
    assert o.ct6_count() == 64


def test_ct6_gc_and_map_ops():
    o = Oracle()
    o.ct6_set_max(4)
    keys = np.zeros(5, L.CT6_TUPLE)
    keys["daddr"][:, 15] = np.arange(5)
    vals = np.zeros(5, L.CT_ENTRY)
    vals["lifetime"] = [10, 20, 30, 40, 50]
    for i in range(4):
        assert o.ct6_update(keys[i], vals[i]) == 0
    assert o.ct6_update(keys[4], vals[4]) == -7
    assert o.ct6_update(keys[0], vals[4]) == 0
    assert o.ct6_lookup(keys[0])[0] == 0
    assert o.ct6_gc(31) == 2
    k, v = o.ct6_dump()
    assert sorted(v["lifetime"].tolist()) == [40, 50]
    assert o.ct6_delete(keys[3]) == 0 and o.ct6_delete(keys[3]) == -2
