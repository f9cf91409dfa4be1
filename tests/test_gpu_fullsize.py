"""GPU parity at the BASELINE.json table sizes
over multi-million-tuple slices, and the N > 1 counter path (two engine
contexts over the two flow-hash shards, summed as RCCL SUM does, folded)
against one context and the restatement.  Bit-exact throughout.

The full 64M-tuple batches run in bench.py (parity_vs_oracle); these tests
use the same tables with a 4M slice of the same seeded stream so that the
whole module stays within a few minutes on one MI355X."""
import numpy as np
import pytest

from cilium_amd import build, layouts as L, shard, synth

pytestmark = pytest.mark.gpu

N_SLICE = 4 << 20


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU test needs a device"
    build.build()
    return torch


def _engine(**kw):
    from cilium_amd.engine import Engine
    return Engine(device=0, **kw)


def _np(t, dt=None):
    a = t.cpu().numpy()
    return a.view(dt) if dt is not None else a


def _entry_counters(e, T):
    """(packets, bytes) of every policy entry, in T.pol_keys order."""
    got = e.policy_counters(T.pol_ep, T.pol_keys)
    return got[:, 0], got[:, 1]


def _oracle_counters(o, T):
    pk = np.empty(len(T.pol_keys), np.uint64)
    by = np.empty(len(T.pol_keys), np.uint64)
    for i, (k, ep) in enumerate(zip(T.pol_keys, T.pol_ep)):
        rc, raw = o.policy_lookup(int(ep), k)
        assert rc == 0
        ent = np.frombuffer(raw, L.POLICY_ENTRY)[0]
        pk[i], by[i] = ent["packets"], ent["bytes"]
    return pk, by


@pytest.fixture(scope="module")
def cfg2():
    from oracle import Oracle
    T = synth.make_tables(**synth.CONFIGS["gpu"])
    t = synth.make_tuples(T, N_SLICE)
    o = Oracle(**T.oracle_config())
    synth.load_oracle(o, T)
    v, idt, st, _ = o.classify_v4(t, nthreads=16)
    return T, t, o, (v, idt, st)


def test_config2_fullsize(torch_cuda, cfg2):
    """Config 2: 100k IPv4 ipcache prefixes + 64k policy entries (4 ep x
    16k): verdict, identity, stage, every per-entry counter and the
    {reason, dir} metrics (bpf/lib/policy.h:46-110, eps.h:70-80)."""
    torch = torch_cuda
    T, t, o, (v0, i0, s0) = cfg2
    assert len(T.ipc_keys) >= 100_000 and len(T.pol_keys) == 64_000
    e = _engine(**T.engine_config())
    synth.load_engine(e, T)
    e.commit()
    out = e.classify_v4(synth.to_device(t))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_np(out["verdict"]), v0)
    np.testing.assert_array_equal(_np(out["identity"], np.uint32), i0)
    np.testing.assert_array_equal(_np(out["stage"]), s0)
    gp, gb = _entry_counters(e, T)
    op, ob = _oracle_counters(o, T)
    np.testing.assert_array_equal(gp, op)
    np.testing.assert_array_equal(gb, ob)
    np.testing.assert_array_equal(e.metrics(), o.metrics())
    # every stage and verdict class occurs at this size
    assert set(np.unique(s0)) >= {0, 1, 2, 3}
    e.close()


def test_config2_two_context_shard_merge(torch_cuda, cfg2):
    """SURVEY §8e on one device: two engine contexts over the two flow-hash
    shards, delta buffers bound, summed with the u64 addition of
    cgpu_counters_allreduce (RCCL refuses two ranks on one GPU: "invalid
    usage", tools/rccl_two_rank_probe.py, DESIGN §5 -- the ABI collective
    itself runs in bench.py at N > 1 with its own check), then counter_fold
    on both: both contexts report the counters of one context over the whole
    batch, which equal the restatement's; verdicts of each shard equal the
    oracle's."""
    torch = torch_cuda
    T, t, o, (v0, i0, s0) = cfg2
    world = 2
    owner = shard.shard_of(t, world)
    engines, bufs = [], []
    for r in range(world):
        e = _engine(**T.engine_config())
        synth.load_engine(e, T)
        e.commit()
        b = torch.zeros(e.counter_delta_bytes() // 8, dtype=torch.int64, device="cuda")
        e.counter_bind(b)
        engines.append(e)
        bufs.append(b)
    assert engines[0].checksum() == engines[1].checksum()
    for r, e in enumerate(engines):
        idx = np.nonzero(owner == r)[0]
        out = e.classify_v4(synth.to_device(shard.take(t, idx)))
        torch.cuda.synchronize()
        np.testing.assert_array_equal(_np(out["verdict"]), v0[idx])
        np.testing.assert_array_equal(_np(out["identity"], np.uint32), i0[idx])
        np.testing.assert_array_equal(_np(out["stage"]), s0[idx])
    total = bufs[0] + bufs[1]  # the all-reduce (integer SUM, order-free)
    for e, b in zip(engines, bufs):
        b.copy_(total)
        e.counter_fold()
    torch.cuda.synchronize()
    op, ob = _oracle_counters(o, T)
    for e in engines:
        gp, gb = _entry_counters(e, T)
        np.testing.assert_array_equal(gp, op)
        np.testing.assert_array_equal(gb, ob)
        np.testing.assert_array_equal(e.metrics(), o.metrics())
    for e in engines:
        e.counter_bind(None)
        e.close()


def test_config5_fullsize(torch_cuda):
    """Config 5: 1M IPv4 services (lb4_local, bpf/lib/lb.h:604-651 in the
    bpf_lxc.c:444-469 order) in front of the config-2 tables; the skb->hash
    stand-in is computed in the kernel from sport (cgpu_flow_hash)."""
    from oracle import Oracle
    torch = torch_cuda
    cfg = synth.CONFIGS["cascade"]
    T = synth.make_tables(**cfg)
    S = synth.make_services(T, cfg["n_services"])
    t = synth.add_service_traffic(synth.make_tuples(T, N_SLICE), S)
    del t["hash"]
    o = Oracle(**T.oracle_config())
    synth.load_oracle(o, T)
    synth.load_services(o, S)
    v0, i0, s0, _ = o.classify_v4_lb(t, nthreads=16)
    e = _engine(**T.engine_config(), lb_max_entries=len(S.keys))
    synth.load_engine(e, T)
    synth.load_services(e, S)
    e.commit()
    out = e.classify_v4_lb(synth.to_device(t))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_np(out["verdict"]), v0)
    np.testing.assert_array_equal(_np(out["identity"], np.uint32), i0)
    np.testing.assert_array_equal(_np(out["stage"]), s0)
    gp, gb = _entry_counters(e, T)
    op, ob = _oracle_counters(o, T)
    np.testing.assert_array_equal(gp, op)
    np.testing.assert_array_equal(gb, ob)
    np.testing.assert_array_equal(e.metrics(), o.metrics())
    assert len(S.vip) == 1_000_000
    e.close()


def test_config5_cascade_fullsize(torch_cuda):
    """Config 5 as BASELINE names it, "prefilter -> ipcache identity ->
    policy verdict -> LB": every ingress tuple first meets the netdev's XDP
    prefilter (bpf_xdp.c:97-121 check_v4 over a 16k-prefix dyn4 LPM + 200k
    fix4 /32s, then check_v4_endpoint on daddr), every egress tuple the
    service step over 1M services; then ipcache -> policy
    (cgpu_classify_v4_cascade).  Verdict, identity, stage, every entry's
    counters and the metrics equal the restatement's composition
    (or_classify_v4_cascade)."""
    from oracle import Oracle
    torch = torch_cuda
    cfg = synth.CONFIGS["cascade"]
    T = synth.make_tables(**cfg)
    S = synth.make_services(T, cfg["n_services"])
    P = synth.make_prefilter4(T)
    t = synth.add_prefilter_traffic(synth.add_service_traffic(synth.make_tuples(T, N_SLICE), S), P)
    del t["hash"]
    o = Oracle(**T.oracle_config())
    synth.load_oracle(o, T)
    synth.load_services(o, S)
    synth.load_prefilter4(o, P)
    v0, i0, s0, _ = o.classify_v4_cascade(t, nthreads=16)
    ing = (t["flags"] & 1) == 0
    xd = v0 == L.VERDICT_XDP_DROP
    assert xd.sum() > 0.03 * ing.sum() and not xd[~ing].any()
    e = _engine(**T.engine_config(), lb_max_entries=len(S.keys))
    synth.load_engine(e, T)
    synth.load_services(e, S)
    synth.load_prefilter4(e, P)
    e.commit()
    out = e.classify_v4_cascade(synth.to_device(t))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_np(out["verdict"]), v0)
    np.testing.assert_array_equal(_np(out["identity"], np.uint32), i0)
    np.testing.assert_array_equal(_np(out["stage"]), s0)
    gp, gb = _entry_counters(e, T)
    op, ob = _oracle_counters(o, T)
    np.testing.assert_array_equal(gp, op)
    np.testing.assert_array_equal(gb, ob)
    np.testing.assert_array_equal(e.metrics(), o.metrics())
    e.close()


def test_config3_fullsize(torch_cuda):
    """Config 3: the XDP IPv6 prefilter over the 1M-prefix deny set (dyn6 +
    /128 fix6 under 256 /24 roots, bpf/bpf_xdp.c:132-156) and 4k endpoints,
    over a 4M-packet slice of the bench stream."""
    from oracle import Oracle
    torch = torch_cuda
    P = synth.make_prefilter6(**synth.PF6_CONFIG)
    p = synth.make_packets6(P, N_SLICE)
    assert len(P.dyn6) + len(P.fix6) == 1_000_000
    o = Oracle(**P.oracle_config())
    synth.load_prefilter6(o, P)
    r0, _ = o.prefilter_v6(p["saddr"], p["daddr"], p["flags"], nthreads=16)
    e = _engine(**P.engine_config())
    synth.load_prefilter6(e, P)
    e.commit()
    d = synth.packets6_to_device(p)
    g = e.prefilter_v6(d["saddr"], d["daddr"], d["flags"])
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_np(g), r0)
    assert 0.5 < (r0 == L.XDP_DROP).mean() < 0.97  # 50% inside a deny prefix + non-endpoint daddrs
    e.close()


def test_v6_config2_size(torch_cuda):
    """IPv6 classify at config-2 size (bench.py --config v6): 100k IPv6
    ipcache prefixes + the 64k-entry MapState over a 4M slice; verdict,
    identity, stage, per-entry counters and metrics (bpf/lib/eps.h:56-66,
    bpf_lxc.c:170-187, policy.h:46-110)."""
    from oracle import Oracle
    torch = torch_cuda
    T = synth.make_tables6(**synth.CONFIGS["v6"])
    t = synth.make_tuples6(T, N_SLICE)
    o = Oracle(**T.oracle_config())
    synth.load_oracle(o, T)
    v0, i0, s0, _ = o.classify_v6(t, nthreads=16)
    e = _engine(**T.engine_config())
    synth.load_engine(e, T)
    e.commit()
    out = e.classify_v6(synth.to_device(t))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_np(out["verdict"]), v0)
    np.testing.assert_array_equal(_np(out["identity"], np.uint32), i0)
    np.testing.assert_array_equal(_np(out["stage"]), s0)
    gp, gb = _entry_counters(e, T)
    op, ob = _oracle_counters(o, T)
    np.testing.assert_array_equal(gp, op)
    np.testing.assert_array_equal(gb, ob)
    np.testing.assert_array_equal(e.metrics(), o.metrics())
    assert len(T.ipc_keys) >= 100_000 and set(np.unique(s0)) >= {0, 1, 2, 3}
    e.close()
