"""GPU parity of IPv6 stateful conntrack (cilium_ct6_global)
through the C ABI: cgpu_classify_v6_ct + the cgpu_ct6_* map calls against the
reference's ct_lookup6 / ct_create6 golden vectors (tests/golden/ct6.npz) and
against the CPU restatement (pinned to that fixture) on larger streams.
Verdicts, ct_lookup6 results, identities, stages, the whole CT map, policy
counters and metrics are compared bit for bit."""
import numpy as np
import pytest

from cilium_amd import build, layouts as L, synth

pytestmark = pytest.mark.gpu


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
    out = e.classify_v6_ct(synth.to_device(t), now)
    torch.cuda.synchronize()
    return (out["verdict"].cpu().numpy(), out["ct_ret"].cpu().numpy(),
            out["identity"].cpu().numpy().view(np.uint32), out["stage"].cpu().numpy())


def _golden_engine(g, ct_max=1 << 20, src_identity=0):
    e = _engine(ct_max=ct_max, ct6_max=ct_max, ipv6_router_ip=g["router_ip"].tobytes(),
                ingress_src_identity=src_identity)
    for k, v in zip(g["ipc_keys"], g["ipc_vals"]):
        assert e.ipcache_update(k, v) == 0
    for k, en, ep in zip(g["pol_keys"], g["pol_entries"], g["pol_ep"]):
        assert e.policy_update(int(ep), k, en) == 0
    synth.load_lxc(e, g["seclabels"])
    e.commit()
    return e


def test_ct6_golden_stream(torch_cuda, golden):
    g = golden("ct6.npz")
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
            e.commit()
        sl = slice(int(cuts[bi]), int(cuts[bi + 1]))
        v, cr, idt, st = _run(torch_cuda, e, {k: x[sl] for k, x in t.items()}, int(nows[bi]))
        np.testing.assert_array_equal(v, g["b_verdict"][sl], err_msg=f"batch {bi}")
        np.testing.assert_array_equal(cr, g["b_ct_ret"][sl], err_msg=f"batch {bi}")
        np.testing.assert_array_equal(idt, g["b_identity"][sl], err_msg=f"batch {bi}")
        np.testing.assert_array_equal(st, g["b_stage"][sl], err_msg=f"batch {bi}")
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
    assert e.ct4_count() == 0  # the IPv4 map is another map
    e.close()


def test_ct6_golden_small_map(torch_cuda, golden):
    """CT_MAP_SIZE 64 with a reserved ingress source identity: order-free
    checks (which creates fail depends on lane order, cgpu.h)."""
    g = golden("ct6.npz")
    e = _golden_engine(g, ct_max=64, src_identity=2)
    t = {k[3:]: g[k] for k in g.files if k.startswith("t2_")}
    v, cr, idt, st = _run(torch_cuda, e, t, 500)
    assert e.ct6_count() == 64
    fail = v == L.DROP_CT_CREATE_FAILED
    assert fail.sum() > 0 and (cr[fail] == L.CT_NEW).all()
    gated = g["s_ct_ret"] == L.CT_NONE
    np.testing.assert_array_equal(v[gated], g["s_verdict"][gated])
    new = ~gated & (cr == L.CT_NEW)
    np.testing.assert_array_equal(idt[new], g["s_identity"][new])
    e.close()


@pytest.fixture(scope="module")
def cfg_ct6():
    T = synth.make_tables6(n_prefixes=20_000, n_identities=500, n_endpoints=3, keys_per_ep=4000)
    t, loc, seclabels = synth.make_ct6_workload(T, 40_000, mean_pkts=10.0, span=0.05)
    return T, t, loc, seclabels


@pytest.mark.parametrize("sched", [0, 8 << 8])
def test_ct6_stream_vs_restatement(torch_cuda, cfg_ct6, sched):
    """~400k IPv6 packets of 40k connections in 3 batches, 1500 policy keys
    deleted before the middle batch, then ctmap GC and one more batch:
    everything bit-exact, map, counters and metrics included.  Also with the
    group keys cut to 8 bits (CGPU_SCHED_CT_SORT_BITS(8)): every walker group
    mixes connections of both orientations (kernels.hip CT_DFLT)."""
    from oracle import Oracle
    torch = torch_cuda
    T, t, loc, seclabels = cfg_ct6
    o = Oracle(**T.oracle_config())
    for k, v in zip(T.ipc_keys, T.ipc_vals):
        assert o.ipcache_update(k, v) == 0
    for k, en, ep in zip(T.pol_keys, T.pol_entries, T.pol_ep):
        assert o.policy_update(int(ep), k, en) == 0
    synth.load_lxc(o, seclabels)
    o.ct6_set_max(1 << 18)
    e = _engine(**T.engine_config(), ct_max=1 << 18, schedule=sched)
    synth.load_engine(e, T)
    synth.load_lxc(e, seclabels)
    e.commit()
    rng = np.random.Generator(np.random.PCG64(13))
    dels = rng.choice(len(T.pol_keys), 1500, replace=False)
    n = len(t["saddr"])
    cuts = np.linspace(0, n, 4).astype(np.int64)
    nows = [1000, 1004, 1100]
    for bi in range(3):
        if bi == 1:
            for d in dels:
                assert e.policy_delete(int(T.pol_ep[d]), T.pol_keys[d]) == 0
                assert o.policy_delete(int(T.pol_ep[d]), T.pol_keys[d]) == 0
            e.commit()
        tb = {k: x[cuts[bi]:cuts[bi + 1]] for k, x in t.items()}
        v, cr, idt, st = _run(torch, e, tb, nows[bi])
        v0, cr0, i0, s0, _ = o.classify_v6_ct(tb, nows[bi])
        np.testing.assert_array_equal(v, v0, err_msg=f"batch {bi}")
        np.testing.assert_array_equal(cr, cr0, err_msg=f"batch {bi}")
        np.testing.assert_array_equal(idt, i0, err_msg=f"batch {bi}")
        np.testing.assert_array_equal(st, s0, err_msg=f"batch {bi}")
        assert e.ct6_count() == o.ct6_count()
    for s_ in (L.CT_NEW, L.CT_ESTABLISHED, L.CT_REPLY, L.CT_RELATED, L.CT_NONE):
        assert (cr0 == s_).sum() > 0, s_
    ek, ev = e.ct6_dump()
    ok, ov = o.ct6_dump()
    np.testing.assert_array_equal(ek, ok)
    np.testing.assert_array_equal(ev, ov)
    np.testing.assert_array_equal(e.metrics(), o.metrics())
    assert e.ct6_gc(1100 + 61) == o.ct6_gc(1100 + 61)
    tb = {k: x[:50_000] for k, x in t.items()}
    v, cr, idt, st = _run(torch, e, tb, 1200)
    v0, cr0, i0, s0, _ = o.classify_v6_ct(tb, 1200)
    np.testing.assert_array_equal(v, v0)
    np.testing.assert_array_equal(cr, cr0)
    ek, ev = e.ct6_dump()
    ok, ov = o.ct6_dump()
    np.testing.assert_array_equal(ek, ok)
    np.testing.assert_array_equal(ev, ov)
    e.close()


def test_ct6_unaligned_columns_rejected(torch_cuda, cfg_ct6):
    T, t, loc, seclabels = cfg_ct6
    e = _engine(**T.engine_config())
    e.commit()
    d = synth.to_device({k: x[:64] for k, x in t.items()})
    raw = torch_cuda.zeros(64 * 16 + 8, dtype=torch_cuda.uint8, device="cuda")
    d["saddr"] = raw[8:].view(64, 16)
    with pytest.raises(Exception):
        e.classify_v6_ct(d, 1)
    e.close()
