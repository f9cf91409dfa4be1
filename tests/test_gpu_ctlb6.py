"""GPU parity of the IPv6 stateful service step (cgpu_classify_v6_ctlb: lb6_local
with CONNTRACK in front of the IPv6 egress conntrack path; VERDICT r2 next 7,
SURVEY §8f rows 1 + 3) through the C ABI, against the reference's golden
vectors (tests/golden/ctlb6.npz: 4 batches, CT_SERVICE entries installed
beforehand, service backends deleted and re-added and policy keys deleted
between batches) and against the CPU restatement (pinned to that fixture) on
larger streams: verdict, ct_lookup6 result, identity, stage, the frame's
translated daddr / dport, the whole cilium_ct6_global map, the policy
counters and the metrics, bit for bit."""
import numpy as np
import pytest

from cilium_amd import build, layouts as L, synth

pytestmark = pytest.mark.gpu

DROP_NO_SERVICE = -158


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU test needs a device"
    build.build()
    return torch


def _engine(**kw):
    from cilium_amd.engine import Engine
    return Engine(device=0, **kw)


def _run(torch, e, t, now):
    out = e.classify_v6_ctlb(synth.to_device(t), now)
    torch.cuda.synchronize()
    return {"verdict": out["verdict"].cpu().numpy(), "ct_ret": out["ct_ret"].cpu().numpy(),
            "identity": out["identity"].cpu().numpy().view(np.uint32),
            "stage": out["stage"].cpu().numpy(), "xdaddr": out["daddr"].cpu().numpy(),
            "xdport": out["dport"].cpu().numpy().view(np.uint16)}


def _check(out, exp, t, msg):
    for f in ("verdict", "ct_ret", "identity", "stage", "xdaddr"):
        np.testing.assert_array_equal(out[f], exp[f], err_msg=f"{msg} {f}")
    m = ((t["flags"] & 1) == 0) | np.isin(t["proto"], [6, 17])
    np.testing.assert_array_equal(out["xdport"][m], exp["xdport"][m], err_msg=f"{msg} xdport")


def _golden_engine(g, ct_max=1 << 20):
    e = _engine(ct_max=ct_max, ct6_max=ct_max, ipv6_router_ip=g["router_ip"].tobytes())
    for k, v in zip(g["ipc_keys"], g["ipc_vals"]):
        assert e.ipcache_update(k, v) == 0
    for k, en, ep in zip(g["pol_keys"], g["pol_entries"], g["pol_ep"]):
        assert e.policy_update(int(ep), k, en) == 0
    for k, v in zip(g["lb_keys"], g["lb_vals"]):
        assert e.lb6_update(k, v) == 0
    synth.load_lxc(e, g["seclabels"])
    e.commit()
    return e


def test_ctlb6_golden_stream(torch_cuda, golden):
    g = golden("ctlb6.npz")
    e = _golden_engine(g)
    for k, v in zip(g["pre_keys"], g["pre_vals"]):
        assert e.ct6_update(k, v) == 0
    t = {k[2:]: g[k] for k in g.files if k.startswith("t_")}
    cuts, nows = g["cuts"], g["nows"]
    off = 0
    for bi in range(4):
        if bi == 2:
            for d in g["pol_del"]:
                assert e.policy_delete(int(g["pol_ep"][d]), g["pol_keys"][d]) == 0
            for d in g["svc_del"]:
                assert e.lb6_delete(g["lb_keys"][d]) == 0
            e.commit()
        if bi == 3:
            for d, v in zip(g["svc_readd"], g["readd_vals"]):
                assert e.lb6_update(g["lb_keys"][d], v) == 0
            e.commit()
        sl = slice(int(cuts[bi]), int(cuts[bi + 1]))
        tb = {k: x[sl] for k, x in t.items()}
        out = _run(torch_cuda, e, tb, int(nows[bi]))
        _check(out, {f: g["b_" + f][sl] for f in ("verdict", "ct_ret", "identity", "stage", "xdaddr",
                                                  "xdport")}, tb, f"batch {bi}")
        n = int(g["dump_n"][bi])
        keys, vals = e.ct6_dump()
        np.testing.assert_array_equal(keys, g["dump_keys"][off:off + n], err_msg=f"batch {bi}")
        np.testing.assert_array_equal(vals, g["dump_vals"][off:off + n], err_msg=f"batch {bi}")
        assert e.ct6_count() == n
        off += n
    deleted = set(g["pol_del"].tolist())
    for i, (k, ep, fe) in enumerate(zip(g["pol_keys"], g["pol_ep"], g["final_entries"])):
        if i in deleted:
            continue
        rc, got = e.policy_lookup(int(ep), k)
        assert rc == 0
        assert (int(got["packets"]), int(got["bytes"])) == (int(fe["packets"]), int(fe["bytes"]))
    assert e.ct4_count() == 0
    e.close()


def test_ctlb6_golden_small_map(torch_cuda, golden):
    """CT_MAP_SIZE 48: order-free checks as test_ctlb_golden_small_map."""
    g = golden("ctlb6.npz")
    e = _golden_engine(g, ct_max=48)
    t = {k[3:]: g[k] for k in g.files if k.startswith("t2_")}
    out = _run(torch_cuda, e, t, 500)
    v, cr = out["verdict"], out["ct_ret"]
    assert e.ct6_count() == 48
    fail = v == L.DROP_CT_CREATE_FAILED
    assert (cr[fail] == L.CT_NEW).all()
    assert (g["s_svc_hit"][v == DROP_NO_SERVICE] == 1).all()
    gated = (g["s_ct_ret"] == L.CT_NONE) & (g["s_stage"] == 4)
    np.testing.assert_array_equal(v[gated], g["s_verdict"][gated])
    e.close()


@pytest.fixture(scope="module")
def cfg_ctlb6():
    T = synth.make_tables6(n_prefixes=20_000, n_identities=500, n_endpoints=3, keys_per_ep=4000)
    svcs = synth.make_services6(T, 3000)
    t, loc, seclabels, svcs = synth.make_ctlb6_workload(T, svcs, 40_000, mean_pkts=10.0, span=0.05)
    return T, svcs, t, seclabels


def test_ctlb6_stream_vs_restatement(torch_cuda, cfg_ctlb6):
    """~400k IPv6 packets of 40k connections (40 % to 3000 services, loopback
    backends) in 3 batches, 10 % of the backends deleted before batch 1 and
    half of them back with new targets before batch 2: everything bit-exact,
    map, counters and metrics included."""
    from oracle import Oracle
    torch = torch_cuda
    T, svcs, t, seclabels = cfg_ctlb6
    o = Oracle(**T.oracle_config())
    for k, v in zip(T.ipc_keys, T.ipc_vals):
        assert o.ipcache_update(k, v) == 0
    for k, en, ep in zip(T.pol_keys, T.pol_entries, T.pol_ep):
        assert o.policy_update(int(ep), k, en) == 0
    synth.load_services6(o, svcs)
    synth.load_lxc(o, seclabels)
    o.ct6_set_max(1 << 18)
    e = _engine(**T.engine_config(), ct_max=1 << 18)
    synth.load_engine(e, T)
    synth.load_services6(e, svcs)
    synth.load_lxc(e, seclabels)
    e.commit()
    rng = np.random.Generator(np.random.PCG64(14))
    ns = len(svcs.vip)
    gone = rng.choice(np.arange(ns, len(svcs.keys)), (len(svcs.keys) - ns) // 10, replace=False)
    back = gone[: len(gone) // 2]
    nv = svcs.vals[back].copy()
    nv["target"] = svcs.vals["target"][rng.integers(ns, len(svcs.keys), len(back))]
    n = len(t["saddr"])
    cuts = np.linspace(0, n, 4).astype(np.int64)
    nows = [1000, 1004, 1100]
    for bi in range(3):
        if bi == 1:
            for d in gone:
                assert e.lb6_delete(svcs.keys[d]) == 0 and o.lb6_delete(svcs.keys[d]) == 0
        if bi == 2:
            for d, v in zip(back, nv):
                assert e.lb6_update(svcs.keys[d], v) == 0 and o.lb6_update(svcs.keys[d], v) == 0
        e.commit()
        tb = {k: x[cuts[bi]:cuts[bi + 1]] for k, x in t.items()}
        out = _run(torch, e, tb, nows[bi])
        exp = o.classify_v6_ctlb(tb, nows[bi])
        _check(out, exp, tb, f"batch {bi}")
        assert e.ct6_count() == o.ct6_count()
    assert (exp["verdict"] == DROP_NO_SERVICE).sum() > 0
    ek, ev = e.ct6_dump()
    ok, ov = o.ct6_dump()
    np.testing.assert_array_equal(ek, ok)
    np.testing.assert_array_equal(ev, ov)
    assert (ek["flags"] == 4).sum() > 1000  # CT_SERVICE entries
    np.testing.assert_array_equal(e.metrics(), o.metrics())
    for k, ep in zip(T.pol_keys[:4000], T.pol_ep[:4000]):
        rc, got = e.policy_lookup(int(ep), k)
        _, raw = o.policy_lookup(int(ep), k)
        exp = np.frombuffer(raw, L.POLICY_ENTRY)[0]
        assert (int(got["packets"]), int(got["bytes"])) == (int(exp["packets"]), int(exp["bytes"]))
    e.close()


def test_ctlb6_empty_and_plain(torch_cuda, cfg_ctlb6):
    """An empty batch; a batch without service traffic equals
    cgpu_classify_v6_ct on a second context."""
    T, svcs, t, seclabels = cfg_ctlb6
    e = _engine(**T.engine_config(), ct_max=1 << 18)
    synth.load_engine(e, T)
    synth.load_services6(e, svcs)
    synth.load_lxc(e, seclabels)
    e.commit()
    out = e.classify_v6_ctlb(synth.to_device({k: x[:0] for k, x in t.items()}), 1)
    torch_cuda.cuda.synchronize()
    assert out["verdict"].numel() == 0
    plain = {k: x[:50_000] for k, x in t.items()}
    isv = (plain["daddr"][:, :4] == [0xFD, 0, 0, 0x96]).all(axis=1) | \
        (plain["saddr"][:, :4] == [0xFD, 0, 0, 0x96]).all(axis=1)
    plain = {k: x[~isv] for k, x in plain.items()}
    a = _run(torch_cuda, e, plain, 10)
    f = _engine(**T.engine_config(), ct_max=1 << 18)
    synth.load_engine(f, T)
    synth.load_lxc(f, seclabels)
    f.commit()
    b = f.classify_v6_ct(synth.to_device(plain), 10)
    torch_cuda.cuda.synchronize()
    np.testing.assert_array_equal(a["verdict"], b["verdict"].cpu().numpy())
    np.testing.assert_array_equal(a["ct_ret"], b["ct_ret"].cpu().numpy())
    np.testing.assert_array_equal(a["xdaddr"], plain["daddr"])
    ek, ev = e.ct6_dump()
    fk, fv = f.ct6_dump()
    np.testing.assert_array_equal(ek, fk)
    np.testing.assert_array_equal(ev, fv)
    e.close()
    f.close()
