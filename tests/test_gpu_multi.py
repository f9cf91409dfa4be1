"""SURVEY §8e with the engine in separate processes (config 4's protocol at
world 2 on the one-GPU box).

Two ranks, one process each, both on cuda:0: every rank builds the same
replicated tables, classifies its flowhash % 2 shard of one tuple stream
through libcgpu.so, and the ranks' counter delta buffers are SUM-reduced over
a torch.distributed process group (gloo: RCCL refuses two ranks on one GPU,
tools/rccl_two_rank_probe.py) before each rank's cgpu_counter_fold.  The
ranks check what bench.py checks at N > 1 (table checksums and counter slot
layouts equal, before and after cgpu_counters_rebalance).  Every rank's
folded per-entry counters and metrics must equal the restatement over the
whole stream, and the union of the shards' verdicts must equal its
verdicts."""
import os
import socket

import numpy as np
import pytest

from cilium_amd import layouts as L, shard, synth

pytestmark = pytest.mark.gpu

N = 1 << 20


def _tables():
    return synth.make_tables(n_prefixes=20_000, n_identities=500, n_endpoints=4, keys_per_ep=4000)


def _stream(T):
    t = synth.make_tuples(T, N)
    t["sport"] = np.random.default_rng(11).integers(1024, 65536, N).astype(np.uint16)
    return t


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry_counters(get, T):
    out = np.zeros((len(T.pol_keys), 2), np.uint64)
    for i, (k, ep) in enumerate(zip(T.pol_keys, T.pol_ep)):
        rc, e = get(int(ep), k)
        assert rc == 0
        out[i] = int(e["packets"]), int(e["bytes"])
    return out


def _rank(rank, world, port, q):
    import torch
    import torch.distributed as dist
    from cilium_amd.engine import Engine
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        T = _tables()
        t = _stream(T)
        mine = np.nonzero(shard.shard_of(t, world) == rank)[0]
        e = Engine(device=0, **T.engine_config())
        synth.load_engine(e, T)
        e.commit()
        delta = torch.zeros(e.counter_delta_bytes() // 8, dtype=torch.int64, device="cuda")
        e.counter_bind(delta)

        def agree(x):
            v = torch.tensor([x & 0x7FFFFFFFFFFFFFFF], dtype=torch.int64)
            lo, hi = v.clone(), v.clone()
            dist.all_reduce(lo, op=dist.ReduceOp.MIN)
            dist.all_reduce(hi, op=dist.ReduceOp.MAX)
            return int(lo) == int(hi)

        def reduce_fold():
            torch.cuda.synchronize()
            host = delta.cpu()
            dist.all_reduce(host, op=dist.ReduceOp.SUM)  # u64 SUM as int64 bits
            delta.copy_(host.cuda())
            e.counter_fold()
            torch.cuda.synchronize()

        ok = [agree(e.checksum()), agree(e.counter_layout_checksum())]
        d = synth.to_device(shard.take({k: v for k, v in t.items() if k != "sport"}, mine))
        out = e.classify_v4(d)
        reduce_fold()
        # the control plane's rebalance on the identical folded totals: every
        # rank must move the same slots before the next slot-wise sum
        e.counters_rebalance()
        ok.append(agree(e.counter_layout_checksum()))
        out2 = e.classify_v4(d)
        reduce_fold()
        torch.cuda.synchronize()
        v = out["verdict"].cpu().numpy()
        same = bool(np.array_equal(v, out2["verdict"].cpu().numpy()))
        cnt = _entry_counters(e.policy_lookup, T)
        res = (rank, mine, v, out["identity"].cpu().numpy().view(np.uint32), ok, same, cnt, e.metrics())
        objs = [None] * world
        dist.all_gather_object(objs, res)
        if rank == 0:
            q.put(objs)
        e.counter_bind(None)
        e.close()
    finally:
        dist.destroy_process_group()


def test_two_process_shards_gloo_reduce_equal_one_stream():
    import multiprocessing as mp
    from oracle import Oracle
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        objs = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    T = _tables()
    t = _stream(T)
    o = Oracle(**T.oracle_config())
    synth.load_oracle(o, T)
    tt = {k: v for k, v in t.items() if k != "sport"}
    v0, i0, _, _ = o.classify_v4(tt, nthreads=8)
    o.classify_v4(tt, nthreads=8)  # the ranks classified their shards twice
    want = _entry_counters(lambda ep, k: (lambda r: (r[0], np.frombuffer(r[1], L.POLICY_ENTRY)[0]))(
        o.policy_lookup(ep, k)), T)
    gv, gi = np.empty_like(v0), np.empty_like(i0)
    for rank, mine, v, idt, ok, same, cnt, met in objs:
        assert all(ok), (rank, ok)  # checksums / slot layouts agree across ranks
        assert same
        gv[mine], gi[mine] = v, idt
        np.testing.assert_array_equal(cnt, want)
        np.testing.assert_array_equal(met, o.metrics())
    np.testing.assert_array_equal(gv, v0)
    np.testing.assert_array_equal(gi, i0)
