"""GPU parity of the service load balancer through the C
ABI: cgpu_lb4_select against the reference's bpf_lb.c / lb4_local golden
vectors (hash injected), cgpu_classify_v4_lb (BASELINE config 5 egress path)
against the composed reference path, and both against the CPU restatement at
larger sizes with the default flow hash.  Bit-exact."""
import numpy as np
import pytest

from cilium_amd import build, layouts as L, synth

pytestmark = pytest.mark.gpu

VARIANTS = {"both": L.LB_L3 | L.LB_L4, "l3": L.LB_L3, "l4": L.LB_L4}


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU test needs a device"
    build.build()
    return torch


# cgpu_config defaults of _engine (tests switch the classify schedule through
# cgpu_config.schedule: the old variant numbers 0 / 3 / 8)
_DEFAULTS = {}
SCHED_OF = {0: 2, 3: 1, 8: 0}  # CGPU_SCHED_GLOBAL_CTR, CGPU_SCHED_PER_LANE, default x4


def _engine(**kw):
    from cilium_amd.engine import Engine
    return Engine(device=0, **{**_DEFAULTS, **kw})


def _dev(torch, t):
    view = {np.dtype(np.uint32): np.int32, np.dtype(np.uint16): np.int16,
            np.dtype(np.uint8): np.uint8}
    return {k: torch.from_numpy(np.ascontiguousarray(v).view(view[np.asarray(v).dtype])).cuda()
            for k, v in t.items()}


def _np(x, dt):
    return x.cpu().numpy().view(dt)


def _lb_run(torch, e, t, mode):
    d = _dev(torch, {k: t[k] for k in ("saddr", "daddr", "sport", "dport", "proto", "hash")
                     if k in t})
    out = e.lb4_select(d, mode)
    torch.cuda.synchronize()
    return {"ret": _np(out["ret"], np.int32), "saddr": _np(out["saddr"], np.uint32),
            "daddr": _np(out["daddr"], np.uint32), "dport": _np(out["dport"], np.uint16),
            "rev_nat": _np(out["rev_nat"], np.uint16), "slave": _np(out["slave"], np.uint16)}


@pytest.mark.parametrize("variant", sorted(VARIANTS))
def test_lb_netdev_golden(torch_cuda, golden, variant):
    g = golden("lb4.npz")
    e = _engine(lb_flags=VARIANTS[variant])
    assert e.lb4_update_batch(g["keys"], g["vals"]) == 0
    e.commit()
    t = {k[2:]: g[k] for k in g.files if k.startswith("t_")}
    out = _lb_run(torch_cuda, e, t, L.LB_NETDEV)
    np.testing.assert_array_equal(out["ret"], g[f"nd_{variant}_ret"])
    np.testing.assert_array_equal(out["daddr"], g[f"nd_{variant}_daddr"])
    np.testing.assert_array_equal(out["dport"], g[f"nd_{variant}_dport"])
    e.close()


@pytest.mark.parametrize("ct", [1, 0])
def test_lb_lxc_golden(torch_cuda, golden, ct):
    g = golden("lb4.npz")
    e = _engine(ct_proto_gate=ct)
    assert e.lb4_update_batch(g["keys"], g["vals"]) == 0
    e.commit()
    t = {k[2:]: g[k] for k in g.files if k.startswith("t_")}
    out = _lb_run(torch_cuda, e, t, L.LB_LXC)
    px = "lx_" if ct else "lxnoct_"
    ref = np.where(g[px + "ret"] < 0, g[px + "ret"],
                   np.where(g[px + "svc_hit"] == 1, 1 + g[px + "loopback"].astype(np.int32), 0))
    np.testing.assert_array_equal(out["ret"], ref)
    np.testing.assert_array_equal(out["saddr"], g[px + "saddr"])
    np.testing.assert_array_equal(out["daddr"], g[px + "daddr"])
    np.testing.assert_array_equal(out["dport"], g[px + "dport"])
    ok = g[px + "ret"] >= 0
    np.testing.assert_array_equal(out["rev_nat"][ok], g[px + "rev_nat"][ok])
    np.testing.assert_array_equal(out["slave"][ok], g[px + "slave"][ok])
    e.close()


@pytest.mark.parametrize("ci", range(2))
def test_classify_v4_lb_golden(torch_cuda, golden, ci):
    torch = torch_cuda
    g = golden("classify_v4_lb.npz")
    gate, src, sw = (int(x) for x in g["configs"][ci])
    e = _engine(ct_proto_gate=gate, ingress_src_identity=src, ingress_secctx_world=sw)
    for k, v in zip(g["ipc_keys"], g["ipc_vals"]):
        assert e.ipcache_update(k, v) == 0
    for k, en, ep in zip(g["pol_keys"], g["pol_entries"], g["pol_ep"]):
        assert e.policy_update(int(ep), k, en) == 0
    assert e.lb4_update_batch(g["lb_keys"], g["lb_vals"]) == 0
    e.commit()
    t = {k[2:]: g[k] for k in g.files if k.startswith("t_") and k != "t_opts"}
    out = e.classify_v4_lb(synth.to_device(t))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out["verdict"].cpu().numpy(), g[f"c{ci}_verdict"])
    np.testing.assert_array_equal(out["identity"].cpu().numpy().view(np.uint32),
                                  g[f"c{ci}_identity"])
    np.testing.assert_array_equal(out["stage"].cpu().numpy(), g[f"c{ci}_stage"])
    for k, ep, fe in zip(g["pol_keys"], g["pol_ep"], g[f"c{ci}_final_entries"]):
        rc, got = e.policy_lookup(int(ep), k)
        assert (int(got["packets"]), int(got["bytes"])) == (int(fe["packets"]), int(fe["bytes"]))
    np.testing.assert_array_equal(e.metrics(), g[f"c{ci}_metrics"])  # the reference's
    e.close()


@pytest.mark.parametrize("variant", [0, 3, 8])
@pytest.mark.parametrize("ci", range(2))
def test_classify_v4_cascade_golden(torch_cuda, golden, ci, variant, monkeypatch):
    """BASELINE config 5 whole (cgpu_classify_v4_cascade) against the
    reference's XDP program + ingress decision and service step + egress
    decision (tests/golden/cascade_v4.npz), on every classify schedule: the
    x4 kernel's XDP stage and the per-lane kernels' must agree."""
    torch = torch_cuda
    monkeypatch.setitem(_DEFAULTS, "schedule", SCHED_OF[variant])
    g = golden("cascade_v4.npz")
    gate, src, sw = (int(x) for x in g["configs"][ci])
    e = _engine(ct_proto_gate=gate, ingress_src_identity=src, ingress_secctx_world=sw)
    for k, v in zip(g["ipc_keys"], g["ipc_vals"]):
        assert e.ipcache_update(k, v) == 0
    for k, en, ep in zip(g["pol_keys"], g["pol_entries"], g["pol_ep"]):
        assert e.policy_update(int(ep), k, en) == 0
    assert e.lb4_update_batch(g["lb_keys"], g["lb_vals"]) == 0
    for w, name in ((0, "dyn4"), (1, "fix4")):
        for k in g[name]:
            assert e.cidr_update(w, k) == 0
    for k in g["endpoints"]:
        assert e.endpoint_update(k) == 0
    e.commit()
    t = {k[2:]: g[k] for k in g.files if k.startswith("t_") and k != "t_opts"}
    out = e.classify_v4_cascade(synth.to_device(t))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out["verdict"].cpu().numpy(), g[f"c{ci}_verdict"])
    np.testing.assert_array_equal(out["identity"].cpu().numpy().view(np.uint32),
                                  g[f"c{ci}_identity"])
    np.testing.assert_array_equal(out["stage"].cpu().numpy(), g[f"c{ci}_stage"])
    for k, ep, fe in zip(g["pol_keys"], g["pol_ep"], g[f"c{ci}_final_entries"]):
        rc, got = e.policy_lookup(int(ep), k)
        assert (int(got["packets"]), int(got["bytes"])) == (int(fe["packets"]), int(fe["bytes"]))
    np.testing.assert_array_equal(e.metrics(), g[f"c{ci}_metrics"])
    e.close()


@pytest.mark.parametrize("variant", [0, 3, 8])
def test_classify_v4_cascade_scale_vs_oracle(torch_cuda, variant, monkeypatch):
    """Config-1 tables + 50k services + the config-5 deny set (16k dyn4,
    200k fix4) and endpoints, 1M tuples plus a ragged tail, every schedule,
    against the restatement (or_classify_v4_cascade)."""
    from oracle import Oracle
    torch = torch_cuda
    monkeypatch.setitem(_DEFAULTS, "schedule", SCHED_OF[variant])
    T = synth.make_tables(**synth.CONFIGS["cpu"])
    T.n_endpoints = 1
    S = synth.make_services(T, 50_000)
    P = synth.make_prefilter4(T)
    t = synth.add_prefilter_traffic(synth.add_service_traffic(synth.make_tuples(T, (1 << 20) + 3), S), P)
    o = Oracle(**T.oracle_config())
    synth.load_oracle(o, T)
    synth.load_services(o, S)
    synth.load_prefilter4(o, P)
    v0, i0, s0, _ = o.classify_v4_cascade(t, nthreads=8)
    e = _engine(**T.engine_config(), lb_max_entries=len(S.keys))
    synth.load_engine(e, T)
    synth.load_services(e, S)
    synth.load_prefilter4(e, P)
    e.commit()
    out = e.classify_v4_cascade(synth.to_device(t))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out["verdict"].cpu().numpy(), v0)
    np.testing.assert_array_equal(out["identity"].cpu().numpy().view(np.uint32), i0)
    np.testing.assert_array_equal(out["stage"].cpu().numpy(), s0)
    np.testing.assert_array_equal(e.metrics(), o.metrics())
    for k, ep in zip(T.pol_keys[:4000], T.pol_ep[:4000]):
        rc, got = e.policy_lookup(int(ep), k)
        _, raw = o.policy_lookup(int(ep), k)
        exp = np.frombuffer(raw, L.POLICY_ENTRY)[0]
        assert (int(got["packets"]), int(got["bytes"])) == (int(exp["packets"]), int(exp["bytes"]))
    assert (v0 == L.VERDICT_XDP_DROP).sum() > 10_000
    e.close()


@pytest.mark.parametrize("fix_on", [1, 0])
def test_classify_v4_cascade_filter_maps_off(torch_cuda, fix_on):
    """The cascade with the dyn4 LPM map disabled (cgpu_config.prefilter_dyn4
    = 0, the agent's PreFilter without the dyn map) and, second, the fix4
    map too: the XDP stage then checks only what remains (bpf_xdp.c:97-121
    under CIDR4_LPM_PREFILTER / CIDR4_FILTER), against the restatement
    configured the same way; schedule x4, 256k tuples."""
    from oracle import Oracle
    torch = torch_cuda
    T = synth.make_tables(**synth.CONFIGS["cpu"])
    T.n_endpoints = 1
    S = synth.make_services(T, 20_000)
    P = synth.make_prefilter4(T)
    t = synth.add_prefilter_traffic(synth.add_service_traffic(synth.make_tuples(T, (1 << 18) + 7), S), P,
                                    deny_frac=0.2)
    o = Oracle(**T.oracle_config(), dyn4=0, fix4=fix_on)
    synth.load_oracle(o, T)
    synth.load_services(o, S)
    synth.load_prefilter4(o, P)
    v0, i0, s0, _ = o.classify_v4_cascade(t, nthreads=8)
    e = _engine(**T.engine_config(), lb_max_entries=len(S.keys), prefilter_dyn4=0, prefilter_fix4=fix_on)
    synth.load_engine(e, T)
    synth.load_services(e, S)
    synth.load_prefilter4(e, P)
    e.commit()
    out = e.classify_v4_cascade(synth.to_device(t))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out["verdict"].cpu().numpy(), v0)
    np.testing.assert_array_equal(out["identity"].cpu().numpy().view(np.uint32), i0)
    np.testing.assert_array_equal(out["stage"].cpu().numpy(), s0)
    np.testing.assert_array_equal(e.metrics(), o.metrics())
    # the stray destinations still drop at check_v4_endpoint
    assert (v0 == L.VERDICT_XDP_DROP).sum() > 500
    e.close()


@pytest.fixture(scope="module")
def cfg_lb():
    T = synth.make_tables(**synth.CONFIGS["cpu"])
    S = synth.make_services(T, 50_000)
    t = synth.add_service_traffic(synth.make_tuples(T, 1 << 20), S)
    return T, S, t


def _oracle(T, S, **cfg):
    from oracle import Oracle
    o = Oracle(**T.oracle_config(), **cfg)
    synth.load_oracle(o, T)
    synth.load_services(o, S)
    return o


@pytest.mark.parametrize("with_hash", [True, False])
def test_classify_v4_lb_scale_vs_oracle(torch_cuda, cfg_lb, with_hash):
    """50k services (~170k map entries) + config-1 tables, 1M tuples, with
    the hash column and with the in-kernel default flow hash (sport)."""
    torch = torch_cuda
    T, S, t = cfg_lb
    if not with_hash:
        t = {k: v for k, v in t.items() if k != "hash"}
    o = _oracle(T, S)
    v0, i0, s0, _ = o.classify_v4_lb(t, nthreads=8)
    e = _engine(**T.engine_config(), lb_max_entries=len(S.keys))
    synth.load_engine(e, T)
    synth.load_services(e, S)
    e.commit()
    out = e.classify_v4_lb(synth.to_device(t))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out["verdict"].cpu().numpy(), v0)
    np.testing.assert_array_equal(out["identity"].cpu().numpy().view(np.uint32), i0)
    np.testing.assert_array_equal(out["stage"].cpu().numpy(), s0)
    np.testing.assert_array_equal(e.metrics(), o.metrics())
    for k, ep in zip(T.pol_keys[:4000], T.pol_ep[:4000]):
        rc, got = e.policy_lookup(int(ep), k)
        _, raw = o.policy_lookup(int(ep), k)
        exp = np.frombuffer(raw, L.POLICY_ENTRY)[0]
        assert (int(got["packets"]), int(got["bytes"])) == (int(exp["packets"]), int(exp["bytes"]))
    assert (s0 == 6).sum() == 0  # well-formed services never drop
    e.close()


@pytest.mark.parametrize("mode", [L.LB_NETDEV, L.LB_LXC])
@pytest.mark.parametrize("n", [1, 63, 100_003])
def test_lb_select_scale_vs_oracle(torch_cuda, cfg_lb, mode, n):
    T, S, t_full = cfg_lb
    t = {k: v[:n] for k, v in t_full.items()}
    o = _oracle(T, S)
    ref, _ = o.lb4(t, mode, nthreads=8)
    e = _engine(**T.engine_config(), lb_max_entries=len(S.keys))
    synth.load_services(e, S)
    e.commit()
    out = _lb_run(torch_cuda, e, t, mode)
    for k in ("ret", "saddr", "daddr", "dport", "rev_nat", "slave"):
        np.testing.assert_array_equal(out[k], ref[k], err_msg=k)
    e.close()


def test_lb_update_delete_sequences(torch_cuda, cfg_lb):
    """Map entries removed and services rewritten through the lbmap
    UpdateService sequence between commits; GPU vs the restatement loaded
    with the engine's dumped map after each commit."""
    from oracle import Oracle

    from cilium_amd.engine import LBMap
    T, S, t_full = cfg_lb
    t = {k: v[:200_000] for k, v in t_full.items()}
    e = _engine(**T.engine_config(), lb_max_entries=len(S.keys) + 1000)
    synth.load_services(e, S)
    rng = np.random.default_rng(5)
    m = LBMap(e)
    for rnd in range(3):
        for i in rng.choice(len(S.keys), 500, replace=False):
            e.lb4_delete(S.keys[i])
        for j in rng.choice(len(S.vip), 50, replace=False):
            vip = int(L.be_to_host4(int(S.vip[j])))
            port = L.ntohs(int(S.port[j]))
            bes = [(int(rng.integers(1, 2**32)), int(rng.integers(0, 65536)), 1)
                   for _ in range(int(rng.integers(1, 5)))]
            m.UpdateService(vip, port, bes, rev_nat=7)
        e.commit()
        dump = m.DumpServiceMapsToUserspace()
        o = Oracle(**T.oracle_config())
        assert o.lb_update_batch(np.array([k for k, _ in dump], L.LB4_KEY),
                                 np.array([v for _, v in dump], L.LB4_SERVICE)) == 0
        ref, _ = o.lb4(t, L.LB_LXC, nthreads=8)
        out = _lb_run(torch_cuda, e, t, L.LB_LXC)
        for k in ("ret", "daddr", "dport", "slave"):
            np.testing.assert_array_equal(out[k], ref[k], err_msg=f"round {rnd} {k}")
        assert (ref["ret"] == L.DROP_NO_SERVICE).sum() > 0
    e.close()


@pytest.mark.parametrize("variant", [3, 8])
@pytest.mark.parametrize("ci", range(2))
def test_classify_v6_lb_golden(torch_cuda, golden, ci, variant, monkeypatch):
    """cgpu_classify_v6_lb against the reference's IPv6 service step
    (lib/lb.h lb6_local, CT and no-CT builds) composed with its v6 decision
    (tests/golden/classify_v6_lb.npz), hash injected; on the one-tuple-per-lane
    kernel (3) and the x4 schedule (8, the default)."""
    torch = torch_cuda
    monkeypatch.setitem(_DEFAULTS, "schedule", SCHED_OF[variant])
    g = golden("classify_v6_lb.npz")
    gate, src = (int(x) for x in g["configs"][ci])
    e = _engine(ct_proto_gate=gate, ingress_src_identity=src, ipv6_router_ip=g["router_ip"].tobytes())
    for k, v in zip(g["ipc_keys"], g["ipc_vals"]):
        assert e.ipcache_update(k, v) == 0
    for k, en, ep in zip(g["pol_keys"], g["pol_entries"], g["pol_ep"]):
        assert e.policy_update(int(ep), k, en) == 0
    assert e.lb6_update_batch(g["lb_keys"], g["lb_vals"]) == 0
    assert e.lb6_count() == len({bytes(k) for k in g["lb_keys"]})
    e.commit()
    t = {k[2:]: g[k] for k in g.files if k.startswith("t_")}
    out = e.classify_v6_lb(synth.to_device(t))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out["verdict"].cpu().numpy(), g[f"c{ci}_verdict"])
    np.testing.assert_array_equal(out["identity"].cpu().numpy().view(np.uint32), g[f"c{ci}_identity"])
    np.testing.assert_array_equal(out["stage"].cpu().numpy(), g[f"c{ci}_stage"])
    for k, ep, fe in zip(g["pol_keys"], g["pol_ep"], g[f"c{ci}_final_entries"]):
        rc, got = e.policy_lookup(int(ep), k)
        assert (int(got["packets"]), int(got["bytes"])) == (int(fe["packets"]), int(fe["bytes"]))
    np.testing.assert_array_equal(e.metrics(), g[f"c{ci}_metrics"])
    e.close()


@pytest.fixture(scope="module")
def cfg_lb6():
    T = synth.make_tables6(n_prefixes=20_000, n_identities=500, n_endpoints=3, keys_per_ep=6000)
    S = synth.make_services6(T, 20_000)
    t = synth.add_service_traffic6(synth.make_tuples6(T, 1 << 19), S)
    return T, S, t


@pytest.mark.parametrize("with_hash", [True, False])
def test_classify_v6_lb_scale_vs_oracle(torch_cuda, cfg_lb6, with_hash):
    """20k IPv6 services (~70k map entries) + 20k v6 ipcache prefixes, 512k
    tuples: GPU == restatement, with the hash column and with the in-kernel
    cgpu_flow_hash6 (sport)."""
    from oracle import Oracle
    torch = torch_cuda
    T, S, t = cfg_lb6
    if not with_hash:
        t = {k: v for k, v in t.items() if k != "hash"}
    o = Oracle(**T.oracle_config())
    synth.load_oracle(o, T)
    synth.load_services6(o, S)
    v0, i0, s0, _ = o.classify_v6_lb(t, nthreads=8)
    e = _engine(**T.engine_config(), lb_max_entries=len(S.keys))
    synth.load_engine(e, T)
    synth.load_services6(e, S)
    e.commit()
    out = e.classify_v6_lb(synth.to_device(t))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out["verdict"].cpu().numpy(), v0)
    np.testing.assert_array_equal(out["identity"].cpu().numpy().view(np.uint32), i0)
    np.testing.assert_array_equal(out["stage"].cpu().numpy(), s0)
    np.testing.assert_array_equal(e.metrics(), o.metrics())
    eg = (t["flags"] & 1) == 1
    svc = eg & (t["daddr"][:, :4] == np.array([0xFD, 0, 0, 0x96], np.uint8)).all(1)
    assert svc.sum() > 10_000 and (s0[svc] != 6).all()  # well-formed services never drop
    e.close()


def test_lb6_map_ops(torch_cuda):
    """cilium_lb6_services map semantics through the ABI: NOEXIST / EXIST,
    delete, lookup, GetNextKey over every key, a re-commit after deletes"""
    from cilium_amd.engine import BPF_EXIST, BPF_NOEXIST
    e = _engine()
    k = np.zeros((), L.LB6_KEY)
    k["address"][:] = np.arange(16, dtype=np.uint8)
    k["dport"] = L.htons(80)
    v = np.zeros((), L.LB6_SERVICE)
    v["count"] = 1
    assert e.lb6_update(k, v, BPF_EXIST) == -2           # -ENOENT
    assert e.lb6_update(k, v, BPF_NOEXIST) == 0
    assert e.lb6_update(k, v, BPF_NOEXIST) == -17        # -EEXIST
    ks = []
    for sl in (1, 2, 300):
        kk = k.copy()
        kk["slave"] = sl
        vv = v.copy()
        vv["target"][:] = 7
        assert e.lb6_update(kk, vv) == 0
        ks.append(kk)
    assert e.lb6_count() == 4
    assert [int(x["slave"]) for x in e.lb6_keys()] == [0, 1, 2, 300]
    rc, got = e.lb6_lookup(ks[2])
    assert rc == 0 and bytes(got["target"]) == bytes([7] * 16)
    assert e.lb6_delete(ks[1]) == 0 and e.lb6_delete(ks[1]) == -2
    e.commit()
    assert e.lb6_count() == 3
    e.close()
