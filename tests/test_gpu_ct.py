"""GPU parity of stateful conntrack through the C ABI:
cgpu_classify_v4_ct + the cilium_ct4_global map calls against the reference's
conntrack.h / policy.h golden vectors (tests/golden/ct4.npz, a 4-batch
stream with pre-installed entries and policy deletes between batches) and
against the CPU restatement (pinned to that fixture) on larger streams.
Every packet's verdict, ct_lookup4 result, identity and policy stage, the
whole CT map after every batch, the policy counters and the metrics are
compared bit for bit."""
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
    out = e.classify_v4_ct(synth.to_device(t), now)
    torch.cuda.synchronize()
    return (out["verdict"].cpu().numpy(), out["ct_ret"].cpu().numpy(),
            out["identity"].cpu().numpy().view(np.uint32), out["stage"].cpu().numpy())


def _golden_engine(g, ct_max=1 << 20):
    e = _engine(ct_max=ct_max)
    for k, v in zip(g["ipc_keys"], g["ipc_vals"]):
        assert e.ipcache_update(k, v) == 0
    for k, en, ep in zip(g["pol_keys"], g["pol_entries"], g["pol_ep"]):
        assert e.policy_update(int(ep), k, en) == 0
    synth.load_lxc(e, g["seclabels"])
    e.commit()
    return e


def test_ct_golden_stream(torch_cuda, golden):
    g = golden("ct4.npz")
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
            e.commit()
        sl = slice(int(cuts[bi]), int(cuts[bi + 1]))
        v, cr, idt, st = _run(torch_cuda, e, {k: x[sl] for k, x in t.items()}, int(nows[bi]))
        np.testing.assert_array_equal(v, g["b_verdict"][sl], err_msg=f"batch {bi}")
        np.testing.assert_array_equal(cr, g["b_ct_ret"][sl], err_msg=f"batch {bi}")
        np.testing.assert_array_equal(idt, g["b_identity"][sl], err_msg=f"batch {bi}")
        np.testing.assert_array_equal(st, g["b_stage"][sl], err_msg=f"batch {bi}")
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


def test_ct_golden_small_map(torch_cuda, golden):
    """At CT_MAP_SIZE 64 the map fills during the batch.  Which creates fail
    then depends on the order lanes reach the capacity check (cgpu.h), so
    the checks are the order-free ones: the map holds exactly 64 entries,
    every DROP_CT_CREATE_FAILED is an allowed CT_NEW, and packets the map's
    capacity cannot influence (policy drops, protocol gate) match."""
    g = golden("ct4.npz")
    e = _golden_engine(g, ct_max=64)
    t = {k[3:]: g[k] for k in g.files if k.startswith("t2_")}
    v, cr, idt, st = _run(torch_cuda, e, t, 500)
    assert e.ct4_count() == 64
    fail = v == L.DROP_CT_CREATE_FAILED
    assert fail.sum() > 0 and (cr[fail] == L.CT_NEW).all()
    gated = g["s_ct_ret"] == L.CT_NONE
    np.testing.assert_array_equal(v[gated], g["s_verdict"][gated])
    np.testing.assert_array_equal(idt[~gated & (cr == L.CT_NEW)],
                                  g["s_identity"][~gated & (cr == L.CT_NEW)])
    e.close()


def _pair(torch, T, t, locals_be, seclabels, batches, nows, ct_max=1 << 18, pre=None,
          deletes=None, schedule=0):
    """Engine and restatement side by side over consecutive batches."""
    from oracle import Oracle
    o = Oracle(**T.oracle_config())
    synth.load_oracle(o, T)
    synth.load_lxc(o, seclabels)
    o.ct_set_max(ct_max)
    e = _engine(**T.engine_config(), ct_max=ct_max, schedule=schedule)
    synth.load_engine(e, T)
    synth.load_lxc(e, seclabels)
    e.commit()
    for k, v in (pre or ()):
        assert e.ct4_update(k, v) == 0 and o.ct4_update(k, v) == 0
    n = len(t["saddr"])
    cuts = np.linspace(0, n, batches + 1).astype(np.int64)
    for bi in range(batches):
        if deletes is not None and bi == batches // 2:
            for k, ep in deletes:
                assert e.policy_delete(int(ep), k) == 0 and o.policy_delete(int(ep), k) == 0
            e.commit()
        tb = {k: x[cuts[bi]:cuts[bi + 1]] for k, x in t.items()}
        v, cr, idt, st = _run(torch, e, tb, int(nows[bi]))
        v0, cr0, i0, s0, _ = o.classify_v4_ct(tb, int(nows[bi]))
        np.testing.assert_array_equal(v, v0, err_msg=f"batch {bi}")
        np.testing.assert_array_equal(cr, cr0, err_msg=f"batch {bi}")
        np.testing.assert_array_equal(idt, i0, err_msg=f"batch {bi}")
        np.testing.assert_array_equal(st, s0, err_msg=f"batch {bi}")
        assert e.ct4_count() == o.ct4_count()
    return e, o


def _assert_same_map(e, o):
    ek, ev = e.ct4_dump()
    ok, ov = o.ct4_dump()
    np.testing.assert_array_equal(ek, ok)
    np.testing.assert_array_equal(ev, ov)


@pytest.fixture(scope="module")
def cfg_ct():
    T = synth.make_tables(**synth.CONFIGS["cpu"])
    T.n_endpoints = 1
    t, locals_be, seclabels = synth.make_ct_workload(T, 60_000, mean_pkts=10.0, span=0.05)
    return T, t, locals_be, seclabels


def test_ct_stream_vs_restatement(torch_cuda, cfg_ct):
    """~600k packets of 60k connections in 3 batches (connections span batch
    boundaries), 2000 policy keys deleted before the middle batch, then
    GC: everything bit-exact, counters and metrics included."""
    T, t, locals_be, seclabels = cfg_ct
    rng = np.random.Generator(np.random.PCG64(11))
    dels = rng.choice(len(T.pol_keys), 2000, replace=False)
    e, o = _pair(torch_cuda, T, t, locals_be, seclabels, 3, [1000, 1004, 1100],
                 deletes=[(T.pol_keys[d], T.pol_ep[d]) for d in dels])
    _assert_same_map(e, o)
    np.testing.assert_array_equal(e.metrics(), o.metrics())
    gone = set(dels.tolist())
    for i, (k, ep) in enumerate(zip(T.pol_keys[:6000], T.pol_ep[:6000])):
        if i in gone:
            continue
        rc, got = e.policy_lookup(int(ep), k)
        _, raw = o.policy_lookup(int(ep), k)
        exp = np.frombuffer(raw, L.POLICY_ENTRY)[0]
        assert (int(got["packets"]), int(got["bytes"])) == (int(exp["packets"]), int(exp["bytes"]))
    # ctmap GC on the map the device wrote, then another batch on the result
    assert e.ct4_gc(1100 + 61) == o.ct4_gc(1100 + 61)
    _assert_same_map(e, o)
    tb = {k: x[:50_000] for k, x in t.items()}
    v, cr, idt, st = _run(torch_cuda, e, tb, 1200)
    v0, cr0, i0, s0, _ = o.classify_v4_ct(tb, 1200)
    np.testing.assert_array_equal(v, v0)
    np.testing.assert_array_equal(cr, cr0)
    _assert_same_map(e, o)
    e.close()


def test_ct_elephant_and_edges(torch_cuda, cfg_ct):
    """One connection with 200k packets in a batch (one long lane), a batch
    of untracked protocols only, pre-installed closing entries, an empty
    batch."""
    T, t, locals_be, seclabels = cfg_ct
    n = 200_000
    rng = np.random.Generator(np.random.PCG64(5))
    eg = rng.random(n) < 0.5
    a, b = int(locals_be[0]), int(t["daddr"][t["flags"] & 1 == 1][0])
    ele = {
        "saddr": np.where(eg, a, b).astype(np.uint32), "daddr": np.where(eg, b, a).astype(np.uint32),
        "sport": np.where(eg, 0x3930, 0x5000).astype(np.uint16),
        "dport": np.where(eg, 0x5000, 0x3930).astype(np.uint16),
        "proto": np.full(n, 6, np.uint8),
        "l4b": ((5 << 4) | (rng.random(n) < 0.01) | (rng.choice([2, 16, 24, 17], n) << 8)).astype(np.uint16),
        "flags": eg.astype(np.uint8), "len": rng.integers(64, 1500, n).astype(np.uint32),
        "ep": np.zeros(n, np.uint16),
    }
    pre = []
    for i in range(64):  # closing / half-closed entries on pairs the stream uses
        k = np.zeros((), L.CT4_TUPLE)
        k["daddr"], k["saddr"] = t["saddr"][i], t["daddr"][i]
        k["dport"], k["sport"], k["nexthdr"] = t["dport"][i], t["sport"][i], t["proto"][i]
        k["flags"] = L.TUPLE_F_OUT if t["flags"][i] & 1 else L.TUPLE_F_IN
        v = np.zeros((), L.CT_ENTRY)
        v["bits"] = [1, 2, 3, 19][i % 4]
        v["lifetime"] = 10
        pre.append((k, v))
    gated = {k: x[:1000].copy() for k, x in t.items()}
    gated["proto"][:] = 47
    mix = {k: np.concatenate([ele[k], gated[k], t[k][:100_000]]) for k in ele}
    e, o = _pair(torch_cuda, T, mix, locals_be, seclabels, 2, [2000, 2001], pre=pre)
    _assert_same_map(e, o)
    out = e.classify_v4_ct({k: synth.to_device({k: x[:0]})[k] for k, x in mix.items()}, 2002)
    torch_cuda.cuda.synchronize()
    assert out["verdict"].numel() == 0
    e.close()


def test_ct_crowded_map_no_duplicates(torch_cuda, cfg_ct):
    """A crowded, contended map: 2,000 connections with ~40
    packets each into a CT_MAP_SIZE of 4,096 (8,192 slots; ~2,900 live
    entries and their tombstones at the end, so long linear-probe clusters),
    below capacity so that no create can fail, over 4 batches so entries are found, closed into tombstones and
    reclaimed across batches, with lanes of every XCD claiming neighbouring
    slots.  A chain ended early by a stale EMPTY read would store a key twice:
    every dumped key is unique, and map, verdicts and counts equal the
    restatement's."""
    T, _, _, _ = cfg_ct
    t, locals_be, seclabels = synth.make_ct_workload(T, 2_000, seed=77, mean_pkts=40.0, span=0.5)
    e, o = _pair(torch_cuda, T, t, locals_be, seclabels, 4, [3000, 3010, 3020, 3030], ct_max=4096)
    keys, _ = e.ct4_dump()
    assert len(keys) > 2_000
    assert len(np.unique(keys.view(np.uint8).reshape(len(keys), -1), axis=0)) == len(keys)
    _assert_same_map(e, o)
    np.testing.assert_array_equal(e.metrics(), o.metrics())
    e.close()


def test_ct_many_connections_per_pair(torch_cuda, cfg_ct):
    """Phase 1 groups by connection, phase 2 by address pair: 3,000
    overlapping connections over FOUR address pairs (one endpoint, four
    remotes), so every pair's creates owe hundreds of ICMP entries to phase 2
    and its ICMP errors must see exactly the entries created before them in
    batch order; ICMP echo connections of a pair share their ids.  Two
    batches, map, verdicts, ct results and counters bit-exact against the
    restatement."""
    T, _, _, _ = cfg_ct
    t, locals_be, seclabels = synth.make_ct_workload(T, 3_000, seed=91, n_remote=4, mean_pkts=12.0,
                                                     span=0.6)
    err = (t["proto"] == 1) & np.isin(t["l4b"], [3, 11, 12])
    lo, hi = np.minimum(t["saddr"], t["daddr"]), np.maximum(t["saddr"], t["daddr"])
    pairs = np.unique(lo.astype(np.uint64) << np.uint64(32) | hi.astype(np.uint64))
    assert err.sum() > 100 and len(pairs) <= 4
    e, o = _pair(torch_cuda, T, t, locals_be, seclabels, 2, [3000, 3002])
    _assert_same_map(e, o)
    np.testing.assert_array_equal(e.metrics(), o.metrics())
    e.close()


def test_ct_orientation_defaults_edges(torch_cuda, cfg_ct):
    """The walker leaves a result unstored when it equals its orientation's
    default (kernels.hip CT_DFLT / ct_orient) and the finish rebuilds it
    from the tuple alone.  Exact for any mix of connections in a group, so
    here the group keys are cut to 8 bits (CGPU_SCHED_CT_SORT_BITS: 256
    groups, every one mixing connections of both orientations) over tuples
    that stress the orientation: initiators with the LOWER source port
    (groups of orientation 1), equal ports (ties broken by address), equal
    ports AND addresses (a tuple equal to its reverse), ICMP echo both ways
    and ICMP timestamps (a zero type word), and connections whose first
    packet in a batch is a reply (their entries from the batch before).
    Three batches, the 24-bit default beside it; verdicts, ct results, map
    and metrics bit-exact against the restatement."""
    T, _, _, _ = cfg_ct
    t, locals_be, seclabels = synth.make_ct_workload(T, 6_000, seed=123, mean_pkts=12.0, span=0.7)
    tcpudp = np.isin(t["proto"], [6, 17])
    sw = lambda x: x.astype(np.uint16).byteswap()  # noqa: E731
    lo, hi = np.minimum(sw(t["sport"]), sw(t["dport"])), np.maximum(sw(t["sport"]), sw(t["dport"]))
    # direction-free connection and address-pair hashes (both directions of
    # a connection take the same changes)
    pk = (np.minimum(t["saddr"], t["daddr"]).astype(np.uint64) * np.uint64(2654435761)
          ^ np.maximum(t["saddr"], t["daddr"]).astype(np.uint64)) % np.uint64(97)
    ck = (pk * np.uint64(40503) + lo.astype(np.uint64) * np.uint64(65537) + hi.astype(np.uint64)) % np.uint64(3)
    # a third of the TCP / UDP connections: the local port below the remote
    # one in host order, so those the endpoint initiates start in
    # orientation 1 (their groups store every result)
    eg = (t["flags"] & 1) == 1  # egress: sport is the local port
    flip = tcpudp & (ck == 0)
    t["sport"] = np.where(flip, sw(np.where(eg, lo, hi)), t["sport"]).astype(np.uint16)
    t["dport"] = np.where(flip, sw(np.where(eg, hi, lo)), t["dport"]).astype(np.uint16)
    # equal ports on some connections, equal addresses on a few of those
    tie = tcpudp & (pk < 9)
    t["sport"] = np.where(tie, t["dport"], t["sport"]).astype(np.uint16)
    same = tie & (pk < 2)
    t["daddr"] = np.where(same, t["saddr"], t["daddr"]).astype(np.uint32)
    ic = t["proto"] == 1
    assert flip.sum() > 1000 and tie.sum() > 100 and same.sum() > 10 and ic.sum() > 100
    for sched in (8 << 8, 0):  # CGPU_SCHED_CT_SORT_BITS(8), then the default 24 bits
        e, o = _pair(torch_cuda, T, t, locals_be, seclabels, 3, [4000, 4003, 4009], schedule=sched)
        _assert_same_map(e, o)
        np.testing.assert_array_equal(e.metrics(), o.metrics())
        e.close()


def test_ct_jumbo_counters_one_slot(torch_cuda, cfg_ct):
    """~2.2M packets of 65,535 bytes hit ONE policy slot in
    one batch, 2^37.07 bytes, past the 37-bit byte field of the packed
    per-slot accumulator that the finish sums over a whole PKC_CHUNK.  Every
    packet of >= 2^11 bytes must take the exact two-word path: the slot's
    packet and byte counters, every other slot's, and the metrics equal the
    restatement's."""
    from oracle import Oracle
    T, t, locals_be, seclabels = cfg_ct
    o = Oracle(**T.oracle_config())
    synth.load_oracle(o, T)
    synth.load_lxc(o, seclabels)
    o.ct_set_max(1 << 18)
    probe = {k: x[:20_000] for k, x in t.items()}
    v0, cr0, _, _, _ = o.classify_v4_ct(probe, 10)
    cand = np.flatnonzero((v0 == 0) & (probe["flags"] & 1 == 1) & (probe["proto"] == 6))
    assert len(cand), "no allowed egress TCP packet to replicate"
    j = int(cand[0])
    n, n_conn = 2_200_000, 20_000
    rng = np.random.Generator(np.random.PCG64(23))
    conn = rng.integers(0, n_conn, n)
    jumbo = {
        "saddr": np.full(n, probe["saddr"][j], np.uint32), "daddr": np.full(n, probe["daddr"][j], np.uint32),
        "sport": (1024 + conn).astype(np.uint16), "dport": np.full(n, probe["dport"][j], np.uint16),
        "proto": np.full(n, 6, np.uint8), "l4b": np.full(n, (5 << 4) | (16 << 8), np.uint16),
        "flags": np.full(n, probe["flags"][j], np.uint8), "len": np.full(n, 65535, np.uint32),
        "ep": np.full(n, probe["ep"][j], np.uint16),
    }
    o2 = Oracle(**T.oracle_config())
    synth.load_oracle(o2, T)
    synth.load_lxc(o2, seclabels)
    o2.ct_set_max(1 << 18)
    e = _engine(**T.engine_config(), ct_max=1 << 18)
    synth.load_engine(e, T)
    synth.load_lxc(e, seclabels)
    e.commit()
    v, cr, idt, st = _run(torch_cuda, e, jumbo, 20)
    ve, cre, ie, se, _ = o2.classify_v4_ct(jumbo, 20)
    np.testing.assert_array_equal(v, ve)
    np.testing.assert_array_equal(cr, cre)
    assert (v == 0).sum() > (1 << 21), "the jumbo packets must be allowed to count"
    np.testing.assert_array_equal(e.metrics(), o2.metrics())
    big = 0
    for k, ep in zip(T.pol_keys, T.pol_ep):
        rc, got = e.policy_lookup(int(ep), k)
        _, raw = o2.policy_lookup(int(ep), k)
        exp = np.frombuffer(raw, L.POLICY_ENTRY)[0]
        assert (int(got["packets"]), int(got["bytes"])) == (int(exp["packets"]), int(exp["bytes"]))
        big = max(big, int(exp["bytes"]))
    assert big >= 1 << 37, "one slot must pass the packed byte field"
    e.close()


@pytest.mark.parametrize("v6", [False, True])
def test_ct_device_gc_and_compaction(torch_cuda, cfg_ct, v6):
    """ctmap.GC (RemoveExpired) and the tombstone compaction run on the device
    map (k_ct_gc, k_ct_rehash) with the map never leaving the device between
    batches: 6 rounds of {batch, GC} over a CT_MAP_SIZE-4096 map (8192
    slots) whose UDP / ICMP / SYN-only entries (60 s lifetime) expire
    between rounds (every third GC reaps the established TCP entries too),
    so a later batch finds more than a quarter of the slots tombstones and
    compacts the table first.  Verdicts, ct results, the GC's deleted counts,
    the live counts and the whole map equal the restatement's carried the
    same way; the live connections' TCP entries survive the compactions."""
    from oracle import Oracle
    T, _, _, _ = cfg_ct
    if v6:
        T = synth.make_tables6(n_prefixes=5000, n_identities=200, n_endpoints=1, keys_per_ep=4000)
        t, _, seclabels = synth.make_ct6_workload(T, 1_800, seed=33, mean_pkts=6.0, span=0.9)
    else:
        t, _, seclabels = synth.make_ct_workload(T, 1_800, seed=33, mean_pkts=6.0, span=0.9)
    ct_max = 1 << 12
    o = Oracle(**T.oracle_config())
    synth.load_oracle(o, T)
    synth.load_lxc(o, seclabels)
    o.ct_set_max(ct_max)
    o.ct6_set_max(ct_max)
    e = _engine(**T.engine_config(), ct_max=ct_max)
    synth.load_engine(e, T)
    synth.load_lxc(e, seclabels)
    e.commit()
    run_o = o.classify_v6_ct if v6 else o.classify_v4_ct
    run_e = e.classify_v6_ct if v6 else e.classify_v4_ct
    gc_o = o.ct6_gc if v6 else o.ct4_gc
    gc_e = e.ct6_gc if v6 else e.ct4_gc
    n = len(t["proto"])
    rng = np.random.Generator(np.random.PCG64(8))
    deleted = 0
    for rnd in range(6):
        # each round a different window of the stream, 120 s later
        lo = int(rng.integers(0, n // 2))
        tb = {k: x[lo:lo + n // 2] for k, x in t.items()}
        now = 1000 + 120 * rnd
        out = run_e(synth.to_device(tb), now)
        torch_cuda.cuda.synchronize()
        v0, cr0, i0, _, _ = run_o(tb, now)
        np.testing.assert_array_equal(out["verdict"].cpu().numpy(), v0, err_msg=f"round {rnd}")
        np.testing.assert_array_equal(out["ct_ret"].cpu().numpy(), cr0, err_msg=f"round {rnd}")
        np.testing.assert_array_equal(out["identity"].cpu().numpy().view(np.uint32), i0)
        assert not (out["verdict"].cpu().numpy() == L.DROP_CT_CREATE_FAILED).any()
        # every third GC also reaps the established TCP entries (21600 s), so
        # more than a quarter of the slots are tombstones at the next batch
        gt = now + (30_000 if rnd % 3 == 1 else 100)
        d_e, d_o = gc_e(gt), gc_o(gt)
        assert d_e == d_o, f"round {rnd}: GC deleted {d_e} vs {d_o}"
        deleted += d_o
        assert (e.ct6_count() if v6 else e.ct4_count()) == (o.ct6_count() if v6 else o.ct4_count())
    st = e.ct_stats(v6)
    assert deleted > 2 * ct_max and st["compactions"] >= 1, (deleted, st)
    ek, ev = (e.ct6_dump() if v6 else e.ct4_dump())
    ok, ov = (o.ct6_dump() if v6 else o.ct4_dump())
    np.testing.assert_array_equal(ek, ok)
    np.testing.assert_array_equal(ev, ov)
    e.close()


@pytest.mark.parametrize("v6", [False, True])
def test_ct_lru_evicts_instead_of_failing(torch_cuda, cfg_ct, v6):
    """LRU mode (cgpu_config.ct_lru; the reference's CT_MAP4 / CT_MAP6 are
    BPF_MAP_TYPE_LRU_HASH, bpf/bpf_lxc.c:53-75): a CT_MAP_SIZE-4096 map is
    filled by one stream, then a stream of other connections needs ~3,000
    more entries.  Properties (the victim choice is the engine's own):
    no DROP_CT_CREATE_FAILED, the live count never exceeds the map size,
    every packet of the second batch gets exactly what the restatement gives
    it starting from the map the batch found (no key the batch touches is
    evicted), and the map afterwards is the restatement's minus evicted
    entries of the first stream that the second batch never touched."""
    from oracle import Oracle
    T, _, _, _ = cfg_ct
    if v6:
        T = synth.make_tables6(n_prefixes=5000, n_identities=200, n_endpoints=1, keys_per_ep=4000)
        mk, run, dump, upd = synth.make_ct6_workload, "classify_v6_ct", "ct6_dump", "ct6_update"
    else:
        mk, run, dump, upd = synth.make_ct_workload, "classify_v4_ct", "ct4_dump", "ct4_update"
    ta, _, seclabels = mk(T, 1_400, seed=41, mean_pkts=5.0, span=0.9)
    tb, _, _ = mk(T, 1_400, seed=42, mean_pkts=5.0, span=0.9)
    ct_max = 1 << 12
    e = _engine(**T.engine_config(), ct_max=ct_max, ct_lru=1)
    synth.load_engine(e, T)
    synth.load_lxc(e, seclabels)
    e.commit()
    count = e.ct6_count if v6 else e.ct4_count
    for bi, (tt, now) in enumerate(((ta, 1000), (tb, 1010))):
        pre_k, pre_v = getattr(e, dump)()
        o = Oracle(**T.oracle_config())
        synth.load_oracle(o, T)
        synth.load_lxc(o, seclabels)
        o.ct_set_max(1 << 20)
        o.ct6_set_max(1 << 20)
        for k, v in zip(pre_k, pre_v):
            assert getattr(o, upd)(k, v) == 0
        out = getattr(e, run)(synth.to_device(tt), now)
        torch_cuda.cuda.synchronize()
        v0, cr0, i0, _, _ = getattr(o, run)(tt, now)
        v = out["verdict"].cpu().numpy()
        assert not (v == L.DROP_CT_CREATE_FAILED).any(), f"batch {bi}"
        np.testing.assert_array_equal(v, v0, err_msg=f"batch {bi}")
        np.testing.assert_array_equal(out["ct_ret"].cpu().numpy(), cr0, err_msg=f"batch {bi}")
        np.testing.assert_array_equal(out["identity"].cpu().numpy().view(np.uint32), i0)
        assert count() <= ct_max
        gk, gv = getattr(e, dump)()
        ok_, ov = getattr(o, dump)()
        gb = {a.tobytes(): b.tobytes() for a, b in zip(gk, gv)}
        ob = {a.tobytes(): b.tobytes() for a, b in zip(ok_, ov)}
        pre = {a.tobytes(): b.tobytes() for a, b in zip(pre_k, pre_v)}
        for kk, vv in gb.items():
            assert ob.get(kk) == vv
        gone = set(ob) - set(gb)
        # only untouched entries of the map the batch found were evicted
        assert all(kk in pre and ob[kk] == pre[kk] for kk in gone)
        if bi == 1:
            # (capacity reserved by other workgroups counts as taken while a
            # batch runs, so evictions start a little before the map is full)
            assert len(gone) > 300
    e.close()


def test_ct_lru_many_batches_gc_compaction(torch_cuda, cfg_ct):
    """LRU mode over eight batches of fresh connections into a CT_MAP_SIZE-
    4096 map, a device GC between some of them: evictions and GC deletes
    leave tombstones until a batch compacts the map on the device
    (cgpu_ct_stats); every batch still gets exactly the restatement's
    results from the map it found, never DROP_CT_CREATE_FAILED, and only
    untouched entries disappear."""
    from oracle import Oracle
    T, _, _, _ = cfg_ct
    ct_max = 1 << 12
    streams = [synth.make_ct_workload(T, 1_200, seed=60 + b, mean_pkts=5.0, span=0.9) for b in range(8)]
    seclabels = streams[0][2]
    e = _engine(**T.engine_config(), ct_max=ct_max, ct_lru=1)
    synth.load_engine(e, T)
    for _, _, sl in streams:
        synth.load_lxc(e, sl)
    e.commit()
    for bi, (tt, _, sl) in enumerate(streams):
        now = 1000 + 20 * bi
        if bi == 3:
            e.ct4_gc(now)  # RemoveExpired: the expired entries of early batches
        if bi == 5:
            e.ct4_gc(now + 100_000)  # everything: tombstones past a quarter of the slots
        pre_k, pre_v = e.ct4_dump()
        o = Oracle(**T.oracle_config())
        synth.load_oracle(o, T)
        for _, _, sl2 in streams:
            synth.load_lxc(o, sl2)
        o.ct_set_max(1 << 20)
        for k, v in zip(pre_k, pre_v):
            assert o.ct4_update(k, v) == 0
        out = e.classify_v4_ct(synth.to_device(tt), now)
        torch_cuda.cuda.synchronize()
        v0, cr0, i0, _, _ = o.classify_v4_ct(tt, now)
        v = out["verdict"].cpu().numpy()
        assert not (v == L.DROP_CT_CREATE_FAILED).any(), f"batch {bi}"
        np.testing.assert_array_equal(v, v0, err_msg=f"batch {bi}")
        np.testing.assert_array_equal(out["ct_ret"].cpu().numpy(), cr0, err_msg=f"batch {bi}")
        np.testing.assert_array_equal(out["identity"].cpu().numpy().view(np.uint32), i0)
        assert e.ct4_count() <= ct_max
        gk, gv = e.ct4_dump()
        ok_, ov = o.ct4_dump()
        gb = {a.tobytes(): b.tobytes() for a, b in zip(gk, gv)}
        ob = {a.tobytes(): b.tobytes() for a, b in zip(ok_, ov)}
        pre = {a.tobytes(): b.tobytes() for a, b in zip(pre_k, pre_v)}
        for kk, vv in gb.items():
            assert ob.get(kk) == vv
        assert all(kk in pre and ob[kk] == pre[kk] for kk in set(ob) - set(gb))
    assert e.ct_stats(False)["compactions"] >= 1
    e.close()
