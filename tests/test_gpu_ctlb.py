"""GPU parity of the stateful service step (cgpu_classify_v4_ctlb: lb4_local
with CONNTRACK in front of the egress conntrack path; VERDICT r2 next 7,
SURVEY §8f rows 1 + 3) through the C ABI, against the reference's golden
vectors (tests/golden/ctlb4.npz: 4 batches with CT_SERVICE entries installed
beforehand, service backends deleted and re-added and policy keys deleted
between batches) and against the CPU restatement (pinned to that fixture) on
larger streams: every packet's verdict, ct_lookup4 result, identity, stage
and translated daddr / dport, the whole CT map after every batch (service,
address and ICMP entries), the policy counters and the metrics, bit for
bit."""
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
    out = e.classify_v4_ctlb(synth.to_device(t), now)
    torch.cuda.synchronize()
    return {"verdict": out["verdict"].cpu().numpy(), "ct_ret": out["ct_ret"].cpu().numpy(),
            "identity": out["identity"].cpu().numpy().view(np.uint32),
            "stage": out["stage"].cpu().numpy(),
            "xdaddr": out["daddr"].cpu().numpy().view(np.uint32),
            "xdport": out["dport"].cpu().numpy().view(np.uint16)}


def _golden_engine(g, ct_max=1 << 20):
    e = _engine(ct_max=ct_max)
    for k, v in zip(g["ipc_keys"], g["ipc_vals"]):
        assert e.ipcache_update(k, v) == 0
    for k, en, ep in zip(g["pol_keys"], g["pol_entries"], g["pol_ep"]):
        assert e.policy_update(int(ep), k, en) == 0
    for k, v in zip(g["lb_keys"], g["lb_vals"]):
        assert e.lb4_update(k, v) == 0
    synth.load_lxc(e, g["seclabels"])
    e.commit()
    return e


def _check(out, exp, t, msg):
    for f in ("verdict", "ct_ret", "identity", "stage", "xdaddr"):
        np.testing.assert_array_equal(out[f], exp[f], err_msg=f"{msg} {f}")
    m = ((t["flags"] & 1) == 0) | np.isin(t["proto"], [6, 17])
    np.testing.assert_array_equal(out["xdport"][m], exp["xdport"][m], err_msg=f"{msg} xdport")


def test_ctlb_golden_stream(torch_cuda, golden):
    g = golden("ctlb4.npz")
    e = _golden_engine(g)
    for k, v in zip(g["pre_keys"], g["pre_vals"]):
        assert e.ct4_update(k, v) == 0
    t = {k[2:]: g[k] for k in g.files if k.startswith("t_")}
    cuts, nows = g["cuts"], g["nows"]
    off = 0
    for bi in range(4):
        if bi == 2:
            for d in g["pol_del"]:
                assert e.policy_delete(int(g["pol_ep"][d]), g["pol_keys"][d]) == 0
            for d in g["svc_del"]:
                assert e.lb4_delete(g["lb_keys"][d]) == 0
            e.commit()
        if bi == 3:
            for d, v in zip(g["svc_readd"], g["readd_vals"]):
                assert e.lb4_update(g["lb_keys"][d], v) == 0
            e.commit()
        sl = slice(int(cuts[bi]), int(cuts[bi + 1]))
        tb = {k: x[sl] for k, x in t.items()}
        out = _run(torch_cuda, e, tb, int(nows[bi]))
        _check(out, {f: g["b_" + f][sl] for f in ("verdict", "ct_ret", "identity", "stage", "xdaddr",
                                                  "xdport")}, tb, f"batch {bi}")
        n = int(g["dump_n"][bi])
        keys, vals = e.ct4_dump()
        np.testing.assert_array_equal(keys, g["dump_keys"][off:off + n], err_msg=f"batch {bi}")
        np.testing.assert_array_equal(vals, g["dump_vals"][off:off + n], err_msg=f"batch {bi}")
        assert e.ct4_count() == n
        off += n
    deleted = set(g["pol_del"].tolist())
    for i, (k, ep, fe) in enumerate(zip(g["pol_keys"], g["pol_ep"], g["final_entries"])):
        if i in deleted:
            continue
        rc, got = e.policy_lookup(int(ep), k)
        assert rc == 0
        assert (int(got["packets"]), int(got["bytes"])) == (int(fe["packets"]), int(fe["bytes"]))
    e.close()


def test_ctlb_golden_small_map(torch_cuda, golden):
    """At CT_MAP_SIZE 48 the map fills during the batch: which creates fail
    depends on the order lanes reach the capacity check (cgpu.h), so the
    checks are order-free: exactly 48 entries, every DROP_CT_CREATE_FAILED
    is a CT_NEW, every DROP_NO_SERVICE a packet aimed at a service, and
    packets capacity cannot influence (protocol gate, non-service policy
    drops of CT_NEW packets) match the reference."""
    g = golden("ctlb4.npz")
    e = _golden_engine(g, ct_max=48)
    t = {k[3:]: g[k] for k in g.files if k.startswith("t2_")}
    out = _run(torch_cuda, e, t, 500)
    v, cr = out["verdict"], out["ct_ret"]
    assert e.ct4_count() == 48
    fail = v == L.DROP_CT_CREATE_FAILED
    assert fail.sum() > 0 and (cr[fail] == L.CT_NEW).all()
    assert (g["s_svc_hit"][v == DROP_NO_SERVICE] == 1).all()
    gated = (g["s_ct_ret"] == L.CT_NONE) & (g["s_stage"] == 4)
    np.testing.assert_array_equal(v[gated], g["s_verdict"][gated])
    e.close()


def _pair(torch, T, svcs, t, seclabels, batches, nows, ct_max=1 << 20, churn=None, schedule=0):
    """Engine and restatement side by side over consecutive batches;
    churn(bi) -> [(op, key, val)] service map changes before batch bi."""
    from oracle import Oracle
    o = Oracle(**T.oracle_config())
    synth.load_oracle(o, T)
    synth.load_services(o, svcs)
    synth.load_lxc(o, seclabels)
    o.ct_set_max(ct_max)
    e = _engine(**T.engine_config(), ct_max=ct_max, schedule=schedule)
    synth.load_engine(e, T)
    synth.load_services(e, svcs)
    synth.load_lxc(e, seclabels)
    e.commit()
    n = len(t["saddr"])
    cuts = np.linspace(0, n, batches + 1).astype(np.int64)
    for bi in range(batches):
        for op, k, v in (churn(bi) if churn else ()):
            if op == "del":
                assert e.lb4_delete(k) == 0 and o.lb_delete(k) == 0
            else:
                assert e.lb4_update(k, v) == 0 and o.lb_update(k, v) == 0
        e.commit()
        tb = {k: x[cuts[bi]:cuts[bi + 1]] for k, x in t.items()}
        out = _run(torch, e, tb, int(nows[bi]))
        exp = o.classify_v4_ctlb(tb, int(nows[bi]))
        _check(out, exp, tb, f"batch {bi}")
        assert e.ct4_count() == o.ct4_count()
    return e, o


def _assert_same_map(e, o):
    ek, ev = e.ct4_dump()
    ok, ov = o.ct4_dump()
    np.testing.assert_array_equal(ek, ok)
    np.testing.assert_array_equal(ev, ov)


@pytest.fixture(scope="module")
def cfg_ctlb():
    T = synth.make_tables(**synth.CONFIGS["cpu"])
    T.n_endpoints = 4
    svcs = synth.make_services(T, 4000)
    t, locals_be, seclabels, svcs = synth.make_ctlb_workload(T, svcs, 60_000, mean_pkts=10.0,
                                                             span=0.05)
    return T, svcs, t, seclabels


@pytest.mark.parametrize("sched", [0, 8 << 8])
def test_ctlb_stream_vs_restatement(torch_cuda, cfg_ctlb, sched):
    """~600k packets of 60k connections (40 % to 4000 services, loopback
    backends) in 3 batches, 10 % of the backends deleted before batch 1 and
    half of them back with new targets before batch 2: everything
    bit-exact, counters and metrics included.  Also with the group keys cut
    to 8 bits (CGPU_SCHED_CT_SORT_BITS(8)): every walker group mixes
    connections of both orientations (kernels.hip CT_DFLT)."""
    T, svcs, t, seclabels = cfg_ctlb
    rng = np.random.Generator(np.random.PCG64(12))
    ns = len(svcs.vip)
    gone = rng.choice(np.arange(ns, len(svcs.keys)), (len(svcs.keys) - ns) // 10, replace=False)
    back = gone[: len(gone) // 2]
    nv = svcs.vals[back].copy()
    nv["target"] = svcs.vals["target"][rng.integers(ns, len(svcs.keys), len(back))]

    def churn(bi):
        if bi == 1:
            return [("del", svcs.keys[d], None) for d in gone]
        if bi == 2:
            return [("put", svcs.keys[d], v) for d, v in zip(back, nv)]
        return []
    e, o = _pair(torch_cuda, T, svcs, t, seclabels, 3, [1000, 1004, 1100], churn=churn, schedule=sched)
    _assert_same_map(e, o)
    np.testing.assert_array_equal(e.metrics(), o.metrics())
    for k, ep in zip(T.pol_keys[:6000], T.pol_ep[:6000]):
        rc, got = e.policy_lookup(int(ep), k)
        _, raw = o.policy_lookup(int(ep), k)
        exp = np.frombuffer(raw, L.POLICY_ENTRY)[0]
        assert (int(got["packets"]), int(got["bytes"])) == (int(exp["packets"]), int(exp["bytes"]))
    keys, _ = e.ct4_dump()
    assert (keys["flags"] == 4).sum() > 1000  # CT_SERVICE entries
    e.close()


def test_ctlb_phase2_and_serial(torch_cuda, cfg_ctlb):
    """Packets whose own address pair receives owed address entries (a
    source equal to its destination, IPV4_LOOPBACK or 0.0.0.0 endpoints):
    phase 2 in pair order; and a batch where such a packet itself owes an
    entry to another pair (a service reached from IPV4_LOOPBACK), which runs
    as one serial group.  Both bit-exact."""
    T, svcs, t, seclabels = cfg_ctlb
    lo = 0x1ffff50a  # IPV4_LOOPBACK (node_config.h:45, raw network-order word)
    base = {k: x[:40_000].copy() for k, x in t.items()}
    eg = (base["flags"] & 1) == 1
    rng = np.random.Generator(np.random.PCG64(3))
    # self-addressed and loopback-address packets on backend pairs
    pick = rng.choice(len(base["saddr"]), 400, replace=False)
    tg = svcs.vals["target"][len(svcs.vip):]
    base["saddr"][pick[:200]] = tg[pick[:200] % len(tg)]
    base["daddr"][pick[:200]] = base["saddr"][pick[:200]]
    base["daddr"][pick[200:300]] = lo
    base["saddr"][pick[300:]] = 0
    e, o = _pair(torch_cuda, T, svcs, base, seclabels, 2, [1500, 1501])
    _assert_same_map(e, o)
    # a service reached from IPV4_LOOPBACK: serial batch
    ser = {k: x[40_000:60_000].copy() for k, x in t.items()}
    idx = np.flatnonzero((ser["flags"] & 1) == 1)[:50]
    ser["saddr"][idx] = lo
    ser["daddr"][idx] = svcs.vip[idx % len(svcs.vip)]
    out = _run(torch_cuda, e, ser, 1502)
    exp = o.classify_v4_ctlb(ser, 1502)
    _check(out, exp, ser, "serial")
    _assert_same_map(e, o)
    np.testing.assert_array_equal(e.metrics(), o.metrics())
    e.close()


def test_ctlb_dropped_service_packets_after_phase2_batch(torch_cuda, cfg_ctlb):
    """DROP_NO_SERVICE packets (services whose every backend was deleted,
    lb.h:745-751) at the very indices where the previous batch on the same
    context carried phase-2 packets (self-addressed, loopback and 0.0.0.0
    pairs): the per-packet phase-2 class scratch is reused across batches,
    so a dropped packet must not inherit the stale class.  Bit-exact."""
    T, svcs, t, seclabels = cfg_ctlb
    lo = 0x1ffff50a  # IPV4_LOOPBACK (node_config.h:45, raw network-order word)
    rng = np.random.Generator(np.random.PCG64(41))
    a = {k: x[:30_000].copy() for k, x in t.items()}
    pick = rng.choice(np.flatnonzero((a["flags"] & 1) == 1), 600, replace=False)
    tg = svcs.vals["target"][len(svcs.vip):]
    a["saddr"][pick[:300]] = tg[pick[:300] % len(tg)]
    a["daddr"][pick[:300]] = a["saddr"][pick[:300]]
    a["daddr"][pick[300:450]] = lo
    a["saddr"][pick[450:]] = 0
    b = {k: x[30_000:60_000].copy() for k, x in t.items()}
    dead = np.arange(20)  # services whose backends all go before batch b
    b["flags"][pick] |= 1
    b["proto"][pick] = 6
    b["daddr"][pick] = svcs.vip[dead[np.arange(len(pick)) % len(dead)]]
    b["dport"][pick] = np.where(svcs.port[dead[np.arange(len(pick)) % len(dead)]] != 0,
                                svcs.port[dead[np.arange(len(pick)) % len(dead)]], b["dport"][pick])
    gone = np.flatnonzero(np.isin(svcs.keys["address"], svcs.vip[dead]) & (svcs.keys["slave"] > 0))
    from oracle import Oracle
    o = Oracle(**T.oracle_config())
    synth.load_oracle(o, T)
    synth.load_services(o, svcs)
    synth.load_lxc(o, seclabels)
    o.ct_set_max(1 << 20)
    e = _engine(**T.engine_config(), ct_max=1 << 20)
    synth.load_engine(e, T)
    synth.load_services(e, svcs)
    synth.load_lxc(e, seclabels)
    e.commit()
    _check(_run(torch_cuda, e, a, 2000), o.classify_v4_ctlb(a, 2000), a, "phase-2 batch")
    for d in gone:
        assert e.lb4_delete(svcs.keys[d]) == 0 and o.lb_delete(svcs.keys[d]) == 0
    e.commit()
    out = _run(torch_cuda, e, b, 2001)
    exp = o.classify_v4_ctlb(b, 2001)
    _check(out, exp, b, "drop batch")
    assert (out["verdict"][pick] == DROP_NO_SERVICE).sum() > 300
    _assert_same_map(e, o)
    np.testing.assert_array_equal(e.metrics(), o.metrics())
    e.close()


def test_ctlb_empty_and_plain(torch_cuda, cfg_ctlb):
    """An empty batch; a batch without any service traffic equals
    cgpu_classify_v4_ct on a second context."""
    T, svcs, t, seclabels = cfg_ctlb
    e = _engine(**T.engine_config(), ct_max=1 << 20)
    synth.load_engine(e, T)
    synth.load_services(e, svcs)
    synth.load_lxc(e, seclabels)
    e.commit()
    out = e.classify_v4_ctlb({k: synth.to_device({k: x[:0]})[k] for k, x in t.items()}, 1)
    torch_cuda.cuda.synchronize()
    assert out["verdict"].numel() == 0
    plain = {k: x[:50_000] for k, x in t.items()}
    vipset = np.isin(plain["daddr"], svcs.vip) | np.isin(plain["saddr"], svcs.vip)
    plain = {k: x[~vipset] for k, x in plain.items()}
    a = _run(torch_cuda, e, plain, 10)
    f = _engine(**T.engine_config(), ct_max=1 << 20)
    synth.load_engine(f, T)
    synth.load_lxc(f, seclabels)
    f.commit()
    b = f.classify_v4_ct(synth.to_device(plain), 10)
    torch_cuda.cuda.synchronize()
    np.testing.assert_array_equal(a["verdict"], b["verdict"].cpu().numpy())
    np.testing.assert_array_equal(a["ct_ret"], b["ct_ret"].cpu().numpy())
    ek, ev = e.ct4_dump()
    fk, fv = f.ct4_dump()
    np.testing.assert_array_equal(ek, fk)
    np.testing.assert_array_equal(ev, fv)
    e.close()
    f.close()
