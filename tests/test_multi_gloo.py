"""N>1 path on CPU: world_size 2 over gloo.

Each rank takes its flow-hash shard of one tuple stream, classifies it (the
CPU restatement stands in for the GPU here: the test is about the
shard/merge protocol, not the kernel), packs its per-entry counters into a
delta buffer, and the delta is SUM-all-reduced with the same helper bench.py
uses.  The merged counters and the concatenated verdicts must equal one
process classifying the whole stream."""
import os
import socket

import numpy as np
import pytest

from cilium_amd import layouts as L, shard, synth


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _counters(o, T):
    out = np.zeros(2 * len(T.pol_keys) + 256 * 4 * 2, np.uint64)
    for i, (k, ep) in enumerate(zip(T.pol_keys, T.pol_ep)):
        rc, raw = o.policy_lookup(int(ep), k)
        e = np.frombuffer(raw, L.POLICY_ENTRY)[0]
        out[2 * i], out[2 * i + 1] = e["packets"], e["bytes"]
    out[2 * len(T.pol_keys):] = o.metrics().ravel()
    return out


def _worker(rank, world, port, q):
    import sys
    import torch
    import torch.distributed as dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "oracle"))
    from oracle import Oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    T = synth.make_tables(n_prefixes=3000, n_identities=300, n_endpoints=2, keys_per_ep=2000)
    t = synth.make_tuples(T, 200_000)
    t["sport"] = np.random.default_rng(5).integers(1024, 65536, len(t["saddr"])).astype(np.uint16)
    owner = shard.shard_of(t, world)
    mine = np.nonzero(owner == rank)[0]
    o = Oracle(**T.oracle_config())
    synth.load_oracle(o, T)
    part = shard.take({k: v for k, v in t.items() if k != "sport"}, mine)
    v, idt, st, _ = o.classify_v4(part, nthreads=2)
    delta = torch.from_numpy(_counters(o, T).view(np.int64).copy())
    shard.allreduce_counters(delta)
    # gather verdicts to rank 0 (test only; the product keeps them sharded)
    objs = [None] * world
    dist.all_gather_object(objs, (mine, v, idt))
    if rank == 0:
        q.put((delta.numpy().view(np.uint64).copy(), objs))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_partition_is_exact():
    T = synth.make_tables(n_prefixes=500, n_identities=50, keys_per_ep=300)
    t = synth.make_tuples(T, 50_000)
    for world in (1, 2, 3, 8):
        own = shard.shard_of(t, world)
        assert own.min() >= 0 and own.max() < world
        counts = np.bincount(own, minlength=world)
        assert counts.sum() == 50_000
        if world > 1:  # roughly balanced
            assert counts.min() > 0.8 * 50_000 / world
    # deterministic and flow-consistent
    assert np.array_equal(shard.shard_of(t, 8), shard.shard_of(t, 8))


def test_gloo_world2_counters_match_single_process():
    import sys
    import torch.multiprocessing as mp
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "oracle"))
    from oracle import Oracle
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    merged, objs = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    T = synth.make_tables(n_prefixes=3000, n_identities=300, n_endpoints=2, keys_per_ep=2000)
    t = synth.make_tuples(T, 200_000)
    o = Oracle(**T.oracle_config())
    synth.load_oracle(o, T)
    v, idt, _, _ = o.classify_v4(t, nthreads=2)
    np.testing.assert_array_equal(merged, _counters(o, T))
    v2 = np.empty_like(v)
    i2 = np.empty_like(idt)
    for mine, vv, ii in objs:
        v2[mine], i2[mine] = vv, ii
    np.testing.assert_array_equal(v2, v)
    np.testing.assert_array_equal(i2, idt)


def _ct_worker(rank, world, port, q):
    import sys
    import torch
    import torch.distributed as dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "oracle"))
    from oracle import Oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    T = synth.make_tables(n_prefixes=3000, n_identities=300, n_endpoints=2, keys_per_ep=2000)
    t, _, sl = synth.make_ct_workload(T, 20_000, mean_pkts=6.0, span=0.05)
    mine = np.nonzero(shard.ct_shard_of(t, world) == rank)[0]
    o = Oracle(**T.oracle_config())
    synth.load_oracle(o, T)
    synth.load_lxc(o, sl)
    part = shard.take(t, mine)
    v, cr, idt, st, _ = o.classify_v4_ct(part, 1000)
    delta = torch.from_numpy(_counters(o, T).view(np.int64).copy())
    shard.allreduce_counters(delta)
    keys, vals = o.ct4_dump()
    objs = [None] * world
    dist.all_gather_object(objs, (mine, v, cr, keys, vals))
    if rank == 0:
        q.put((delta.numpy().view(np.uint64).copy(), objs))
    dist.destroy_process_group()


def test_ct_pair_shards_world2():
    """Stateful path sharded by address pair (shard.ct_shard_of): each rank
    runs conntrack over its own packets with its own map.  The verdicts,
    ct_lookup4 results, merged counters and the union of the two maps equal
    one process running the whole stream in order."""
    import multiprocessing as mp
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "oracle"))
    from oracle import Oracle
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ct_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    delta, objs = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    T = synth.make_tables(n_prefixes=3000, n_identities=300, n_endpoints=2, keys_per_ep=2000)
    t, _, sl = synth.make_ct_workload(T, 20_000, mean_pkts=6.0, span=0.05)
    o = Oracle(**T.oracle_config())
    synth.load_oracle(o, T)
    synth.load_lxc(o, sl)
    v, cr, idt, st, _ = o.classify_v4_ct(t, 1000)
    gv, gcr = np.empty_like(v), np.empty_like(cr)
    keys, vals = [], []
    for mine, pv, pcr, k, vv in objs:
        gv[mine], gcr[mine] = pv, pcr
        keys.append(k)
        vals.append(vv)
    np.testing.assert_array_equal(gv, v)
    np.testing.assert_array_equal(gcr, cr)
    np.testing.assert_array_equal(delta, _counters(o, T))
    uk, uv = L.ct_sorted(np.concatenate(keys), np.concatenate(vals))
    ok, ov = o.ct4_dump()
    np.testing.assert_array_equal(uk, ok)
    np.testing.assert_array_equal(uv, ov)
    assert (cr == L.CT_REPLY).sum() > 0 and len(objs[0][0]) > 0 and len(objs[1][0]) > 0


def test_ct_workload_rank_streams_are_pair_shards():
    T = synth.make_tables(n_prefixes=3000, n_identities=300, n_endpoints=2, keys_per_ep=2000)
    for r in range(3):
        t, _, _ = synth.make_ct_workload(T, 2000, gpu_id=r, world=3)
        assert (shard.ct_shard_of(t, 3) == r).all()


def test_config4_rank_streams_partition_by_shard_of():
    """bench.py config 4 at world 8: every rank draws its own seeded tuples
    and redraws source ports (shard.assign_shard_sports) until each tuple
    hashes to that rank.  The union of the 8 rank streams is then exactly
    partitioned by shard_of: every tuple is owned by the rank that holds it,
    no rank's stream is empty, and the redraw leaves the tuples' other
    fields as generated."""
    T = synth.make_tables(n_prefixes=500, n_identities=50, keys_per_ep=300)
    world, n = 8, 20_000
    streams = []
    for r in range(world):
        t = synth.make_tuples(T, n, gpu_id=r)
        before = {k: v.copy() for k, v in t.items() if k != "sport"}
        t["sport"] = shard.assign_shard_sports(t, world, r, seed=synth.SEED + 0x5B0 + r)
        assert (shard.shard_of(t, world) == r).all()
        for k, v in before.items():
            np.testing.assert_array_equal(t[k], v)
        streams.append(t)
    union = {k: np.concatenate([s[k] for s in streams]) for k in streams[0]}
    owner = shard.shard_of(union, world)
    np.testing.assert_array_equal(owner, np.repeat(np.arange(world), n))
    assert np.bincount(owner, minlength=world).tolist() == [n] * world
    # the ranks' streams differ (per-rank seeds), so the stream is world x n tuples
    assert not np.array_equal(streams[0]["saddr"], streams[1]["saddr"])
