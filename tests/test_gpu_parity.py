"""GPU parity: the HIP path (through the C ABI) against the reference's
golden vectors and, at larger sizes, against the CPU restatement (oracle).
Every comparison is bit-exact (integer path)."""
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


# cgpu_config defaults of _engine (tests switch the classify schedule through
# cgpu_config.schedule: the old variant numbers 0 / 3 / 8)
_DEFAULTS = {}
SCHED_OF = {0: 2, 3: 1, 8: 0}  # CGPU_SCHED_GLOBAL_CTR, CGPU_SCHED_PER_LANE, default x4


def _engine(**kw):
    from cilium_amd.engine import Engine
    return Engine(device=0, **{**_DEFAULTS, **kw})


def _np(t, dt=None):
    a = t.cpu().numpy()
    return a.view(dt) if dt is not None else a


def _classify(torch, e, t, stage=True):
    d = synth.to_device(t)
    out = e.classify_v4(d, stage=stage)
    torch.cuda.synchronize()
    return (_np(out["verdict"]), _np(out["identity"], np.uint32),
            _np(out["stage"]) if stage else None)


@pytest.mark.parametrize("ci", range(5))
def test_classify_v4_golden(torch_cuda, golden, ci):
    g = golden("classify_v4.npz")
    gate, src, sw = (int(x) for x in g["configs"][ci])
    e = _engine(ct_proto_gate=gate, ingress_src_identity=src, ingress_secctx_world=sw)
    for k, v in zip(g["ipc_keys"], g["ipc_vals"]):
        assert e.ipcache_update(k, v) == 0
    for k, en, ep in zip(g["pol_keys"], g["pol_entries"], g["pol_ep"]):
        assert e.policy_update(int(ep), k, en) == 0
    e.commit()
    t = {k[2:]: g[k] for k in g.files if k.startswith("t_")}
    v, idt, st = _classify(torch_cuda, e, t)
    np.testing.assert_array_equal(v, g[f"c{ci}_verdict"])
    np.testing.assert_array_equal(idt, g[f"c{ci}_identity"])
    np.testing.assert_array_equal(st, g[f"c{ci}_stage"])
    for k, ep, fe in zip(g["pol_keys"], g["pol_ep"], g[f"c{ci}_final_entries"]):
        rc, got = e.policy_lookup(int(ep), k)
        assert rc == 0
        assert (int(got["packets"]), int(got["bytes"])) == (int(fe["packets"]), int(fe["bytes"]))
    # cilium_metrics as the reference's update_metrics call sites left it
    np.testing.assert_array_equal(e.metrics(), g[f"c{ci}_metrics"])
    e.close()


def test_prefilter_golden(torch_cuda, golden):
    from test_oracle_golden import parse_frames
    torch = torch_cuda
    g = golden("xdp_prefilter.npz")
    e = _engine()
    for w, name in enumerate(("dyn4", "fix4", "dyn6", "fix6")):
        for k in g[name]:
            assert e.cidr_update(w, k) == 0
    for k in g["endpoints"]:
        assert e.endpoint_update(k) == 0
    e.commit()
    fam, flags, s4, d4, s6, d6 = parse_frames(g)
    v4, v6 = fam == 4, fam == 6
    dev = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).view(dt)).cuda()  # noqa: E731
    o4 = e.prefilter_v4(dev(s4[v4], np.int32), dev(d4[v4], np.int32), dev(flags[v4], np.uint8))
    o6 = e.prefilter_v6(dev(s6[v6], np.uint8), dev(d6[v6], np.uint8), dev(flags[v6], np.uint8))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_np(o4), g["verdict"][v4])
    np.testing.assert_array_equal(_np(o6), g["verdict"][v6])
    e.close()


@pytest.fixture(scope="module")
def cfg1():
    T = synth.make_tables(**synth.CONFIGS["cpu"])
    t = synth.make_tuples(T, 1 << 20)
    return T, t


def _oracle_run(T, t, **cfg):
    from oracle import Oracle
    o = Oracle(**T.oracle_config(), **cfg)
    synth.load_oracle(o, T)
    v, idt, st, probes = o.classify_v4(t, nthreads=8)
    return o, v, idt, st, probes


def test_classify_config1_vs_oracle(torch_cuda, cfg1):
    """SURVEY §8d config 1 (10k prefixes, 16k MapState, 1M tuples)."""
    T, t = cfg1
    o, v0, i0, s0, _ = _oracle_run(T, t)
    e = _engine(**T.engine_config())
    synth.load_engine(e, T)
    e.commit()
    v, idt, st = _classify(torch_cuda, e, t)
    np.testing.assert_array_equal(v, v0)
    np.testing.assert_array_equal(idt, i0)
    np.testing.assert_array_equal(st, s0)
    # every per-entry counter
    for k, ep in zip(T.pol_keys, T.pol_ep):
        rc, got = e.policy_lookup(int(ep), k)
        rc0, raw = o.policy_lookup(int(ep), k)
        exp = np.frombuffer(raw, L.POLICY_ENTRY)[0]
        assert rc == 0 and rc0 == 0
        assert (int(got["packets"]), int(got["bytes"])) == (int(exp["packets"]), int(exp["bytes"]))
    np.testing.assert_array_equal(e.metrics(), o.metrics())
    e.close()


@pytest.mark.parametrize("n", [0, 1, 63, 257, 100_003])
def test_ragged_sizes(torch_cuda, cfg1, n):
    T, t_full = cfg1
    t = {k: v[:n] for k, v in t_full.items()}
    e = _engine(**T.engine_config())
    synth.load_engine(e, T)
    e.commit()
    if n == 0:
        d = synth.to_device(t)
        out = e.classify_v4(d)
        torch_cuda.cuda.synchronize()
        assert out["verdict"].numel() == 0
        return
    o, v0, i0, s0, _ = _oracle_run(T, t)
    v, idt, st = _classify(torch_cuda, e, t)
    np.testing.assert_array_equal(v, v0)
    np.testing.assert_array_equal(idt, i0)
    np.testing.assert_array_equal(st, s0)
    e.close()


def test_counter_bind_fold_and_reset(torch_cuda, cfg1):
    torch = torch_cuda
    T, t = cfg1
    t = {k: v[:200_000] for k, v in t.items()}
    o, v0, _, _, _ = _oracle_run(T, t)
    e = _engine(**T.engine_config())
    synth.load_engine(e, T)
    e.commit()
    buf = torch.zeros(e.counter_delta_bytes() // 8, dtype=torch.int64, device="cuda")
    e.counter_bind(buf)
    d = synth.to_device(t)
    for _ in range(3):
        e.classify_v4(d, stage=False)
    torch.cuda.synchronize()
    # the bound buffer holds exactly 3x the oracle's metrics
    met = buf[-256 * 4 * 2:].cpu().numpy().view(np.uint64).reshape(256, 4, 2)
    np.testing.assert_array_equal(met, 3 * o.metrics())
    e.counter_fold()
    torch.cuda.synchronize()
    assert int(buf.abs().sum()) == 0
    np.testing.assert_array_equal(e.metrics(), 3 * o.metrics())
    k, ep = T.pol_keys[0], int(T.pol_ep[0])
    rc, got = e.policy_lookup(ep, k)
    _, raw = o.policy_lookup(ep, k)
    exp = np.frombuffer(raw, L.POLICY_ENTRY)[0]
    assert int(got["packets"]) == 3 * int(exp["packets"])
    e.counters_reset()
    assert int(e.metrics().sum()) == 0
    e.counter_bind(None)
    e.close()


def test_update_commit_sequences(torch_cuda, cfg1):
    """Random upsert/delete rounds (ipcache + policy), commit after each, the
    GPU agrees with the restatement fed the same operations; re-adding a key
    restarts its counters from the supplied entry (kernel htab replace)."""
    from oracle import Oracle
    torch = torch_cuda
    T, t_full = cfg1
    t = {k: v[:50_000] for k, v in t_full.items()}
    rng = np.random.default_rng(7)
    e = _engine(**T.engine_config())
    o = Oracle(**T.oracle_config())
    synth.load_engine(e, T)
    synth.load_oracle(o, T)
    d = synth.to_device(t)
    for rnd in range(4):
        # delete 5% of ipcache entries and policy keys, re-add some with new labels
        for i in rng.choice(len(T.ipc_keys), len(T.ipc_keys) // 20, replace=False):
            k = T.ipc_keys[i]
            r1, r2 = e.ipcache_delete(k), o.ipcache_delete(k)
            assert (r1 == 0) == (r2 == 0)
            if rng.random() < 0.5:
                v = L.remote_info(int(rng.integers(256, 1256)))
                assert e.ipcache_update(k, v) == 0 and o.ipcache_update(k, v) == 0
        for i in rng.choice(len(T.pol_keys), len(T.pol_keys) // 20, replace=False):
            k, ep = T.pol_keys[i], int(T.pol_ep[i])
            r1, r2 = e.policy_delete(ep, k), o.policy_delete(ep, k)
            assert (r1 == 0) == (r2 == 0)
            if rng.random() < 0.5:
                en = L.policy_entry(int(rng.integers(0, 3)) * 1000, 5, 500)
                assert e.policy_update(ep, k, en) == 0 and o.policy_update(ep, k, en) == 0
        e.commit()
        out = e.classify_v4(d)
        v0, i0, s0, _ = o.classify_v4(t, nthreads=8)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(_np(out["verdict"]), v0, err_msg=f"round {rnd}")
        np.testing.assert_array_equal(_np(out["identity"], np.uint32), i0)
        np.testing.assert_array_equal(_np(out["stage"]), s0)
    for k, ep in zip(T.pol_keys, T.pol_ep):
        rc, got = e.policy_lookup(int(ep), k)
        rc0, raw = o.policy_lookup(int(ep), k)
        assert (rc == 0) == (rc0 == 0)
        if rc == 0:
            exp = np.frombuffer(raw, L.POLICY_ENTRY)[0]
            assert (int(got["packets"]), int(got["bytes"]), int(got["proxy_port"])) == \
                (int(exp["packets"]), int(exp["bytes"]), int(exp["proxy_port"]))
    np.testing.assert_array_equal(e.metrics(), o.metrics())
    e.close()


def _v6(rng, n, roots):
    a = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    r = roots[rng.integers(0, len(roots), n)]
    a[:, :3] = r
    return a


def test_prefilter_scale_vs_oracle(torch_cuda):
    """Larger prefilter sets (v4 dyn/fix, v6 dyn over few /24 roots + /128
    fix, endpoints) against the restatement, incl. disabled-dyn configs."""
    from oracle import Oracle
    torch = torch_cuda
    rng = np.random.default_rng(11)
    n = 300_000
    roots = rng.integers(0, 256, (64, 3), dtype=np.uint8)
    dyn6 = []
    for i in range(20_000):
        k = np.zeros((), L.LPM_V6_KEY)
        k["prefixlen"] = int(rng.choice([20, 24, 32, 48, 56, 64, 96, 127]))
        k["addr"][:] = _v6(rng, 1, roots)[0]
        if i < 4:  # a few short prefixes (root-level "short" entries) on 2 roots
            k["prefixlen"] = [8, 16, 12, 16][i]
            k["addr"][:3] = roots[i % 2]
        dyn6.append(k)
    fix6 = []
    for _ in range(5_000):
        k = np.zeros((), L.LPM_V6_KEY)
        k["prefixlen"] = 128
        k["addr"][:] = _v6(rng, 1, roots)[0]
        fix6.append(k)
    dyn4, fix4 = [], []
    for _ in range(20_000):
        k = np.zeros((), L.LPM_V4_KEY)
        k["prefixlen"] = int(rng.choice([8, 16, 20, 24, 28, 30, 32]))
        k["addr"][:] = rng.integers(0, 256, 4, dtype=np.uint8)
        dyn4.append(k)
    for _ in range(5_000):
        k = np.zeros((), L.LPM_V4_KEY)
        k["prefixlen"] = 32
        k["addr"][:] = rng.integers(0, 256, 4, dtype=np.uint8)
        fix4.append(k)
    ep4 = rng.integers(0, 2**32, 4000, dtype=np.uint64).astype(np.uint32)
    ep6 = _v6(rng, 4000, roots)
    s6 = np.where(rng.random((n, 1)) < 0.5,
                  np.array([k["addr"] for k in dyn6])[rng.integers(0, len(dyn6), n)],
                  rng.integers(0, 256, (n, 16), dtype=np.uint8))  # mostly uncovered
    s6[: n // 10] = np.array([k["addr"] for k in fix6])[rng.integers(0, len(fix6), n // 10)]
    d6 = np.where(rng.random((n, 1)) < 0.3, ep6[rng.integers(0, 4000, n)], _v6(rng, n, roots))
    s4 = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    d4 = np.where(rng.random(n) < 0.3, ep4[rng.integers(0, 4000, n)],
                  rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32))
    flags = rng.choice(np.array([0] * 30 + [1, 2], np.uint8), n)
    dev = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).view(dt)).cuda()  # noqa: E731
    for dyn_on in (1, 0):
        e = _engine(prefilter_dyn4=dyn_on, prefilter_dyn6=dyn_on)
        o = Oracle(dyn4=dyn_on, dyn6=dyn_on)
        for w, ks in ((0, dyn4), (1, fix4), (2, dyn6), (3, fix6)):
            for k in ks:
                assert e.cidr_update(w, k) == 0 and o.cidr_update(w, k) == 0
        for a in ep4:
            ek = np.zeros((), L.ENDPOINT_KEY)
            ek["ip"][:4] = np.frombuffer(int(a).to_bytes(4, "little"), np.uint8)
            ek["family"] = 1
            assert e.endpoint_update(ek) == 0 and o.endpoint_update(ek) == 0
        for a in ep6:
            ek = np.zeros((), L.ENDPOINT_KEY)
            ek["ip"][:] = a
            ek["family"] = 2
            assert e.endpoint_update(ek) == 0 and o.endpoint_update(ek) == 0
        e.commit()
        g4 = e.prefilter_v4(dev(s4, np.int32), dev(d4, np.int32), dev(flags, np.uint8))
        g6 = e.prefilter_v6(dev(s6, np.uint8), dev(d6, np.uint8), dev(flags, np.uint8))
        torch.cuda.synchronize()
        r4, _ = o.prefilter_v4(s4, d4, flags, nthreads=8)
        r6, _ = o.prefilter_v6(s6, d6, flags, nthreads=8)
        np.testing.assert_array_equal(_np(g4), r4)
        np.testing.assert_array_equal(_np(g6), r6)
        assert (r6 == L.XDP_DROP).mean() > 0.2 and (r6 == L.XDP_PASS).mean() > 0.05
        e.close()


def _classify6(torch, e, t, stage=True):
    d = synth.to_device(t)
    out = e.classify_v6(d, stage=stage)
    torch.cuda.synchronize()
    return (_np(out["verdict"]), _np(out["identity"], np.uint32),
            _np(out["stage"]) if stage else None)


@pytest.mark.parametrize("ci", range(4))
def test_classify_v6_golden(torch_cuda, golden, ci):
    g = golden("classify_v6.npz")
    gate, src = (int(x) for x in g["configs"][ci])
    e = _engine(ct_proto_gate=gate, ingress_src_identity=src,
                ipv6_router_ip=g["router_ip"].tobytes())
    for k, v in zip(g["ipc_keys"], g["ipc_vals"]):
        assert e.ipcache_update(k, v) == 0
    for k, en, ep in zip(g["pol_keys"], g["pol_entries"], g["pol_ep"]):
        assert e.policy_update(int(ep), k, en) == 0
    e.commit()
    t = {k[2:]: g[k] for k in g.files if k.startswith("t_")}
    v, idt, st = _classify6(torch_cuda, e, t)
    np.testing.assert_array_equal(v, g[f"c{ci}_verdict"])
    np.testing.assert_array_equal(idt, g[f"c{ci}_identity"])
    np.testing.assert_array_equal(st, g[f"c{ci}_stage"])
    for k, ep, fe in zip(g["pol_keys"], g["pol_ep"], g[f"c{ci}_final_entries"]):
        rc, got = e.policy_lookup(int(ep), k)
        assert (int(got["packets"]), int(got["bytes"])) == (int(fe["packets"]), int(fe["bytes"]))
    np.testing.assert_array_equal(e.metrics(), g[f"c{ci}_metrics"])
    e.close()


@pytest.mark.parametrize("variant", [3, 8])
def test_classify_v6_scale_vs_oracle(torch_cuda, variant, monkeypatch):
    """20k IPv6 ipcache prefixes (lengths 0..128, tombstones, static-part
    entries) + policy, 400k tuples: GPU == restatement, bit-exact, on the
    one-tuple-per-lane kernel (3) and the x4 schedule (8, the default)."""
    monkeypatch.setitem(_DEFAULTS, "schedule", SCHED_OF[variant])
    from oracle import Oracle
    rng = np.random.default_rng(21)
    T = synth.make_tables(n_prefixes=100, n_identities=500, n_endpoints=3, keys_per_ep=6000)
    roots = rng.integers(0, 256, (32, 4), dtype=np.uint8)
    keys = np.zeros(20_000, L.IPCACHE_KEY)
    keys["family"] = 2
    lens = rng.choice([0, 8, 16, 20, 32, 40, 48, 56, 64, 72, 96, 112, 120, 127, 128], len(keys))
    keys["prefixlen"] = 32 + lens
    addr = rng.integers(0, 256, (len(keys), 16), dtype=np.uint8)
    addr[:, :4] = roots[rng.integers(0, len(roots), len(keys))]
    keys["ip"] = addr
    keys[:3]["prefixlen"] = [0, 24, 30]          # static-part entries
    keys[:3]["family"] = [0, 0, 2]
    vals = np.zeros(len(keys), L.REMOTE_ENDPOINT_INFO)
    vals["sec_label"] = rng.integers(256, 756, len(keys))
    vals["sec_label"][rng.random(len(keys)) < 0.03] = 0
    vals["sec_label"][rng.random(len(keys)) < 0.01] = 0xF0000000  # >= 2^30: indirect
    router = bytes(addr[5][:8]) + bytes(8)
    n = 400_000
    base = addr[rng.integers(0, len(keys), n)].copy()
    cut = rng.integers(0, 17, n)
    noise = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    mask = np.arange(16)[None, :] >= cut[:, None]
    sa = np.where(mask, noise, base).astype(np.uint8)
    base = addr[rng.integers(0, len(keys), n)].copy()
    da = np.where(np.arange(16)[None, :] >= rng.integers(0, 17, n)[:, None], noise[::-1], base)
    da[: n // 20, :8] = np.frombuffer(router[:8], np.uint8)
    t = {"saddr": sa, "daddr": da.astype(np.uint8),
         "dport": synth.zipf_ports(rng, n).byteswap(),
         "proto": rng.choice(np.array([6, 6, 17, 58, 1], np.uint8), n),
         "flags": rng.integers(0, 4, n).astype(np.uint8),
         "len": rng.integers(64, 9000, n).astype(np.uint32),
         "ep": rng.integers(0, 3, n).astype(np.uint16)}
    cfg_e = dict(T.engine_config(), ipv6_router_ip=router)
    e = _engine(**cfg_e)
    o = Oracle(router_ip=router)
    for k, v in zip(keys, vals):
        assert e.ipcache_update(k, v) == 0 and o.ipcache_update(k, v) == 0
    for k, en, ep in zip(T.pol_keys, T.pol_entries, T.pol_ep):
        assert e.policy_update(int(ep), k, en) == 0 and o.policy_update(int(ep), k, en) == 0
    e.commit()
    v0, i0, s0, _ = o.classify_v6(t, nthreads=8)
    v, idt, st = _classify6(torch_cuda, e, t)
    np.testing.assert_array_equal(v, v0)
    np.testing.assert_array_equal(idt, i0)
    np.testing.assert_array_equal(st, s0)
    np.testing.assert_array_equal(e.metrics(), o.metrics())
    assert len(np.unique(i0)) > 100
    e.close()


@pytest.mark.parametrize("variant", [0, 3, 8])
def test_kernel_variants_exact(torch_cuda, cfg1, variant, monkeypatch):
    """Every classify schedule / counter strategy gives the reference's
    verdicts, identities, stages, per-entry counters and metrics."""
    T, t = cfg1
    monkeypatch.setitem(_DEFAULTS, "schedule", SCHED_OF[variant])
    o, v0, i0, s0, _ = _oracle_run(T, t)
    e = _engine(**T.engine_config())
    synth.load_engine(e, T)
    e.commit()
    v, idt, st = _classify(torch_cuda, e, t)
    np.testing.assert_array_equal(v, v0)
    np.testing.assert_array_equal(idt, i0)
    np.testing.assert_array_equal(st, s0)
    for k, ep in zip(T.pol_keys[::7], T.pol_ep[::7]):
        rc, got = e.policy_lookup(int(ep), k)
        _, raw = o.policy_lookup(int(ep), k)
        exp = np.frombuffer(raw, L.POLICY_ENTRY)[0]
        assert (int(got["packets"]), int(got["bytes"])) == (int(exp["packets"]), int(exp["bytes"]))
    np.testing.assert_array_equal(e.metrics(), o.metrics())
    e.close()


def test_slot_reuse_within_one_commit(torch_cuda):
    """A counter slot freed and reused before one commit: the newest entry's
    supplied counters win (kernel htab: the update replaces the value)."""
    e = _engine(policy_max_total=64, hot_counter_slots=0)
    a, b = L.policy_key(300, 80, 6, 0), L.policy_key(301, 443, 6, 0)
    assert e.policy_update(0, a, L.policy_entry(0, 0, 0)) == 0
    assert e.policy_delete(0, a) == 0
    assert e.policy_update(0, b, L.policy_entry(0, 5, 500)) == 0   # reuses a's slot
    assert e.policy_update(0, a, L.policy_entry(0, 7, 700)) == 0
    assert e.policy_update(0, a, L.policy_entry(0, 9, 900)) == 0   # same key twice
    e.commit()
    assert [int(x) for x in e.policy_lookup(0, b)[1][["packets", "bytes"]].item()] == [5, 500]
    assert [int(x) for x in e.policy_lookup(0, a)[1][["packets", "bytes"]].item()] == [9, 900]
    e.close()


@pytest.mark.parametrize("n", [1, 5, 4099, (1 << 20) - 3])
@pytest.mark.parametrize("variant", [3, 8])
def test_ragged_batches_long_packets(torch_cuda, cfg1, n, variant, monkeypatch):
    """Batch sizes that are not a multiple of the per-lane group, and packet
    lengths past every packed-counter bound (2^16 cold, 2^18 hot): verdicts,
    identities, stages, per-entry counters and metrics stay exact."""
    T, t_full = cfg1
    monkeypatch.setitem(_DEFAULTS, "schedule", SCHED_OF[variant])
    t = {k: np.ascontiguousarray(v[:n]) for k, v in t_full.items()}
    rng = np.random.default_rng(n)
    t["len"] = rng.choice(np.array([64, 1500, 65535, 65536, 70000, 262143, 262144, 9_000_000],
                                   np.uint32), n)
    o, v0, i0, s0, _ = _oracle_run(T, t)
    e = _engine(**T.engine_config())
    synth.load_engine(e, T)
    e.commit()
    v, idt, st = _classify(torch_cuda, e, t)
    np.testing.assert_array_equal(v, v0)
    np.testing.assert_array_equal(idt, i0)
    np.testing.assert_array_equal(st, s0)
    for k, ep in zip(T.pol_keys[::5], T.pol_ep[::5]):
        _, got = e.policy_lookup(int(ep), k)
        _, raw = o.policy_lookup(int(ep), k)
        exp = np.frombuffer(raw, L.POLICY_ENTRY)[0]
        assert (int(got["packets"]), int(got["bytes"])) == (int(exp["packets"]), int(exp["bytes"]))
    np.testing.assert_array_equal(e.metrics(), o.metrics())
    e.close()


def test_unaligned_columns_take_scalar_schedule(torch_cuda, cfg1, monkeypatch):
    """Column views that start off a 16-byte boundary cannot use the vector
    schedule; the launcher picks the per-element one and results stay exact."""
    T, t_full = cfg1
    monkeypatch.setitem(_DEFAULTS, "schedule", 0)
    n = 100_001
    t = {k: np.ascontiguousarray(v[1:n + 1]) for k, v in t_full.items()}
    o, v0, i0, s0, _ = _oracle_run(T, t)
    e = _engine(**T.engine_config())
    synth.load_engine(e, T)
    e.commit()
    d = synth.to_device({k: np.concatenate([x[:1], x]) for k, x in t.items()})
    d = {k: x[1:] for k, x in d.items()}  # views one element past an aligned base
    out = e.classify_v4(d, stage=True)
    torch_cuda.cuda.synchronize()
    np.testing.assert_array_equal(_np(out["verdict"]), v0)
    np.testing.assert_array_equal(_np(out["identity"], np.uint32), i0)
    np.testing.assert_array_equal(_np(out["stage"]), s0)
    np.testing.assert_array_equal(e.metrics(), o.metrics())
    e.close()


def _lpm_shapes_tables(rng):
    """ipcache contents that force every compressed-LPM shape (tables.h
    lpm16c): uniform /16 leaves, 16/32/64-byte run nodes, /16 arrays whose
    /24 entries are leaves, byte-level run nodes or 256-leaf arrays, run
    starts at the last address of a /16, tombstones and labels >= 2^30."""
    cidrs = [("0.0.0.0/0", L.WORLD_ID), ("10.7.0.0/16", L.CLUSTER_ID)]
    lab = lambda: int(rng.choice([rng.integers(256, 70000), rng.integers(1 << 30, 1 << 32)]))
    cidrs += [(f"20.1.{16 * i}.0/20", lab()) for i in range(2)]            # kind 0/1 nodes
    cidrs += [(f"20.2.{3 * i}.0/24", lab()) for i in range(5)]             # kind 2 node
    cidrs += [(f"20.3.{7 * i}.0/24", lab()) for i in range(11)]            # /16 array of leaves
    cidrs += [("20.4.255.255/32", lab()), ("20.4.0.0/32", lab()), ("20.5.128.0/17", 0)]
    cidrs += [(f"20.6.{i}.{j}/32", lab()) for i in range(0, 256, 3) for j in rng.choice(256, 40, replace=False)]
    cidrs += [(f"20.6.{i}.{16 * j}/28", lab()) for i in range(1, 256, 3) for j in range(0, 16, 5)]
    cidrs += [(f"20.7.{i}.{4 * j}/30", lab()) for i in range(8) for j in range(0, 64, 2)]
    cidrs += [("20.8.0.0/16", 0), ("20.8.1.0/24", lab()), ("20.9.0.0/15", lab())]
    seen, keys, vals = set(), [], []
    for c, v in cidrs:
        if c in seen:
            continue
        seen.add(c)
        keys.append(L.ipcache_key(c))
        vals.append(L.remote_info(v, 0))
    return np.array(keys), np.array(vals)


@pytest.mark.parametrize("variant", [3, 8])
def test_lpm_shapes_exact(torch_cuda, variant, monkeypatch):
    """Every ipcache LPM table shape resolves the same identity as the
    restatement (egress lookups of daddr; ingress of saddr)."""
    from oracle import Oracle
    monkeypatch.setitem(_DEFAULTS, "schedule", SCHED_OF[variant])
    rng = np.random.default_rng(7)
    keys, vals = _lpm_shapes_tables(rng)
    n = 1 << 18
    hi = rng.choice(np.array([0x1401, 0x1402, 0x1403, 0x1404, 0x1405, 0x1406, 0x1407, 0x1408,
                              0x1409, 0x140A, 0x0A07, 0x0B00], np.uint32), n)
    lo = rng.integers(0, 1 << 16, n, dtype=np.uint32)
    edge = rng.random(n) < 0.2
    lo = np.where(edge, rng.choice(np.array([0, 1, 255, 256, 0x7FFF, 0x8000, 0xFFFE, 0xFFFF],
                                            np.uint32), n), lo)
    addr = ((hi << 16) | lo).astype(np.uint32).byteswap()
    t = {"saddr": addr, "daddr": addr[::-1].copy(),
         "dport": np.full(n, L.htons(80), np.uint16), "proto": np.full(n, 6, np.uint8),
         "flags": (rng.random(n) < 0.5).astype(np.uint8), "len": np.full(n, 100, np.uint32),
         "ep": np.zeros(n, np.uint16)}
    e = _engine(policy_max_total=1 << 12, max_endpoints=4)
    o = Oracle()
    for k, v in zip(keys, vals):
        assert e.ipcache_update(k, v) == 0 and o.ipcache_update(k, v) == 0
    pk, pe = L.policy_key(0, 80, 6, 1), L.policy_entry(0)
    assert e.policy_update(0, pk, pe) == 0 and o.policy_update(0, pk, pe) == 0
    e.commit()
    v0, i0, s0, _ = o.classify_v4(t, nthreads=8)
    v, idt, st = _classify(torch_cuda, e, t)
    np.testing.assert_array_equal(idt, i0)
    np.testing.assert_array_equal(v, v0)
    np.testing.assert_array_equal(st, s0)
    assert len(np.unique(i0)) > 1000
    e.close()


@pytest.mark.parametrize("lds_mode", [0, 1, 2])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_prefilter6_cover_shapes(torch_cuda, seed, lds_mode, monkeypatch):
    """The v6 any-match cover (tables.h cover6) over every prefix-length class
    and stride boundary: /0../16 (root fill), /17../24 (expanded into b24
    entries), /25../32 (expanded into b32 entries, also over /32s with deeper
    prefixes), /33../64 (/32 node), /65../128 (/64 node or inline), nested
    and overlapping prefixes, all-ones boundaries; addresses drawn at and
    around the edges of every prefix.  Under each LDS staging mode of
    k_prefilter_v6_q (0: root in HBM, 1: u16 root in LDS, 2: root bitmaps +
    u16 b24 blocks in LDS).  Bit-exact against the restatement's kernel-like
    LPM trie."""
    monkeypatch.setitem(_DEFAULTS, "schedule", (lds_mode + 1) << 4)  # CGPU_SCHED_PF6_LDS
    _cover6_case(torch_cuda, seed, np.random.default_rng(100 + seed).integers(0, 256, (6, 2), dtype=np.uint8))


@pytest.mark.parametrize("n_roots,root_bytes", [(3, 4), (40, 4), (150, 4), (600, 4), (3, 7), (24, 6)])
def test_prefilter6_dense_nodes(torch_cuda, n_roots, root_bytes):
    """Thousands of prefixes under a few /32s (root_bytes 4) or packed into a
    few /56s and /48s (7, 6): /32 nodes of every sub-range split, 0..6 and
    COVER6_LONG (tables.h cover6 node32), with boundaries at 0 and
    0xFFFFFFFF (the flip bit, the open last interval)."""
    rng = np.random.default_rng(7 + n_roots + root_bytes)
    _cover6_case(torch_cuda, 1, rng.integers(0, 256, (n_roots, root_bytes), dtype=np.uint8), rng=rng,
                 lens=[0, 0, 0, 0, 0, 33, 40, 48, 56, 63, 64, 64, 65, 80, 96, 112, 127, 128])


@pytest.mark.parametrize("seed", [1, 2])
def test_prefilter6_split_nodes(torch_cuda, seed):
    """/32s packed with /60../64 prefixes (and /128s in the same /64s), from
    8 to 1500 per /32 and clustered into 2^20 / 2^24 windows, so the /32
    nodes take every sub-range split (tables.h cover6 node32: s = 0..6) and
    the long-node fallback (COVER6_LONG); boundaries at 0 and 0xFFFFFFFF of
    bits 32..63 (the flip bit, the open last interval).  Packets sit on, just
    below and just above every interval edge."""
    from oracle import Oracle
    torch = torch_cuda
    rng = np.random.default_rng(300 + seed)
    specs = [(8, 32), (20, 32), (40, 32), (60, 32), (150, 32), (250, 32), (400, 32), (1500, 32),
             (200, 20), (100, 24)]
    keys, edges = [], []
    for si, (cnt, wb) in enumerate(specs):
        top = int(rng.integers(0, 2**32))
        base = int(rng.integers(0, 2**32 - (1 << wb) + 1)) if wb < 32 else 0
        xs = base + rng.integers(0, 1 << wb, cnt).astype(np.int64)
        if si == 0:
            xs[:2] = [0, 0xFFFFFFFF]
        for x in xs:
            ln = int(rng.choice([60, 62, 63, 64, 64, 64]))
            lo32 = int(x) & ~((1 << (64 - ln)) - 1)
            keys.append((ln, (top << 32) | lo32, int(rng.integers(0, 2**63))))
            for e in (lo32 - 1, lo32, lo32 + (1 << (64 - ln)) - 1, lo32 + (1 << (64 - ln))):
                if 0 <= e < 2**32:
                    edges.append((top << 32) | e)
        for x in rng.choice(xs, cnt // 10):
            keys.append((128, (top << 32) | int(x), int(rng.integers(0, 2**63))))
    k6 = np.zeros(len(keys), L.LPM_V6_KEY)
    for i, (ln, hi, lo) in enumerate(keys):
        a = np.frombuffer(hi.to_bytes(8, "big") + lo.to_bytes(8, "big"), np.uint8)
        k6[i]["prefixlen"] = ln
        k6[i]["addr"][:] = a & synth.MASK6[ln]
    n = 200_000
    hi = np.array(edges, np.uint64)[rng.integers(0, len(edges), n)]
    s6 = np.zeros((n, 16), np.uint8)
    s6[:, :8] = hi.astype(">u8").view(np.uint8).reshape(n, 8)
    s6[:, 8:] = rng.integers(0, 256, (n, 8), dtype=np.uint8)
    deep = rng.random(n) < 0.1  # exactly on a /128 key
    s6[deep] = k6["addr"][rng.integers(0, len(k6), int(deep.sum()))]
    eps = rng.integers(0, 256, (16, 16), dtype=np.uint8)
    d6 = eps[rng.integers(0, len(eps), n)]
    flags = np.zeros(n, np.uint8)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    e = _engine(prefilter_dyn6=1)
    o = Oracle(dyn6=1)
    for a in eps:
        ek = np.zeros((), L.ENDPOINT_KEY)
        ek["ip"][:] = a
        ek["family"] = L.ENDPOINT_KEY_IPV6
        assert e.endpoint_update(ek) == 0 and o.endpoint_update(ek) == 0
    for k in np.unique(k6):
        assert e.cidr_update(2, k) == 0 and o.cidr_update(2, k) == 0
    e.commit()
    g = e.prefilter_v6(dev(s6), dev(d6), dev(flags))
    torch.cuda.synchronize()
    r, _ = o.prefilter_v6(s6, d6, flags, nthreads=8)
    np.testing.assert_array_equal(_np(g), r)
    assert 0.2 < (r == L.XDP_DROP).mean() < 0.95
    e.close()


def _cover6_case(torch, seed, roots, rng=None, lens=None):
    from oracle import Oracle
    rng = rng if rng is not None else np.random.default_rng(100 + seed)
    lens = lens or [0, 1, 8, 15, 16, 17, 20, 27, 28, 29, 30, 31, 32, 33, 40, 48, 63, 64, 65, 80, 96,
                    112, 127, 128]
    keys = []
    for i in range(3000):
        k = np.zeros((), L.LPM_V6_KEY)
        # the first keys: short prefixes over the roots (not in the dense /32 cases)
        ln = (int(rng.choice(lens[5:])) if i > 3 or roots.shape[1] > 2 else
              [0, 8, 16, 1][i] if seed == 3 else 17)
        a = rng.integers(0, 256, 16, dtype=np.uint8)
        a[:roots.shape[1]] = roots[rng.integers(0, len(roots))]
        r = rng.random()
        if r < 0.2:
            a[2:] = 0xFF
        elif r < 0.3:
            a[4:] = 0
        k["prefixlen"] = ln
        k["addr"][:] = a
        keys.append(k)
    keys = np.array(keys, L.LPM_V6_KEY)
    n = 200_000
    base = keys["addr"][rng.integers(0, len(keys), n)].copy()
    bits = np.unpackbits(base, axis=1)
    cut = rng.integers(0, 129, n)
    noise = np.unpackbits(rng.integers(0, 256, (n, 16), dtype=np.uint8), axis=1)
    mode = rng.integers(0, 3, n)  # 0: random below the cut, 1: all zeros, 2: all ones
    below = np.arange(128)[None, :] >= cut[:, None]
    fill = np.where(mode[:, None] == 0, noise, np.where(mode[:, None] == 1, 0, 1)).astype(np.uint8)
    bits = np.where(below, fill, bits)
    s6 = np.packbits(bits, axis=1)
    s6[: n // 20] = rng.integers(0, 256, (n // 20, 16), dtype=np.uint8)
    eps = rng.integers(0, 256, (16, 16), dtype=np.uint8)
    d6 = eps[rng.integers(0, len(eps), n)]  # uncovered sources then PASS
    flags = np.zeros(n, np.uint8)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    for dyn_on in (1, 0):
        e = _engine(prefilter_dyn6=dyn_on)
        o = Oracle(dyn6=dyn_on)
        for a in eps:
            ek = np.zeros((), L.ENDPOINT_KEY)
            ek["ip"][:] = a
            ek["family"] = L.ENDPOINT_KEY_IPV6
            assert e.endpoint_update(ek) == 0 and o.endpoint_update(ek) == 0
        for k in keys:
            assert e.cidr_update(2, k) == 0 and o.cidr_update(2, k) == 0
            if int(k["prefixlen"]) == 128:
                assert e.cidr_update(3, k) == 0 and o.cidr_update(3, k) == 0
        e.commit()
        g = e.prefilter_v6(dev(s6), dev(d6), dev(flags))
        torch.cuda.synchronize()
        r, _ = o.prefilter_v6(s6, d6, flags, nthreads=8)
        np.testing.assert_array_equal(_np(g), r)
        if dyn_on and seed != 3:
            assert 0.1 < (r == L.XDP_DROP).mean() < 0.99
        elif dyn_on:
            assert (r == L.XDP_DROP).all()  # the /0 deny prefix covers everything
        e.close()
