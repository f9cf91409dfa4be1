"""Snapshot publication (cgpu_commit) on the GPU: incremental commits of
small ipcache / policy deltas equal a full recompile and the restatement,
a single-key policy commit is sub-millisecond, classification launches are
never blocked by a commit running on another thread, and the multi-GPU
counter reduction of the C ABI (cgpu_counters_allreduce over RCCL) is the
identity on a one-rank communicator.

Reference semantics: map writes land per key (pkg/endpoint/endpoint.go:
2572-2652 syncPolicyMap; pkg/datapath/ipcache/listener.go:78-127) while the
datapath keeps running (bpf/lib/policy.h:46-110, bpf/lib/eps.h:56-80)."""
import errno
import threading
import time

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


def _np(t, dt=None):
    a = t.cpu().numpy()
    return a.view(dt) if dt is not None else a


def _check(torch, e, o, t, d, what):
    out = e.classify_v4(d)
    v0, i0, s0, _ = o.classify_v4(t, nthreads=16)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_np(out["verdict"]), v0, err_msg=what)
    np.testing.assert_array_equal(_np(out["identity"], np.uint32), i0, err_msg=what)
    np.testing.assert_array_equal(_np(out["stage"]), s0, err_msg=what)


def _cidr_key(rng, ln):
    a = int(rng.integers(0, 2**32))
    a &= (0xFFFFFFFF << (32 - ln)) & 0xFFFFFFFF if ln else 0
    return L.ipcache_key(f"{a >> 24}.{(a >> 16) & 255}.{(a >> 8) & 255}.{a & 255}/{ln}")


def _mutate(rng, T, e, o, n_ipc, n_pol, lens=(8, 12, 16, 20, 24, 28, 30, 32)):
    """n_ipc ipcache writes (new prefixes of every length, relabels incl.
    tombstones and labels >= 2^30, deletes) and n_pol policy writes, applied
    to the engine and the restatement alike."""
    for _ in range(n_ipc):
        r = rng.random()
        if r < 0.4:
            k = _cidr_key(rng, int(rng.choice(lens)))
        else:
            k = T.ipc_keys[rng.integers(0, len(T.ipc_keys))]
        if r > 0.8:
            assert (e.ipcache_delete(k) == 0) == (o.ipcache_delete(k) == 0)
            continue
        lab = int(rng.choice([0, 2, 3, rng.integers(256, 1256), rng.integers(1 << 30, 1 << 32)]))
        v = L.remote_info(lab, 0)
        assert e.ipcache_update(k, v) == 0 and o.ipcache_update(k, v) == 0
    for _ in range(n_pol):
        i = rng.integers(0, len(T.pol_keys))
        k, ep = T.pol_keys[i], int(T.pol_ep[i])
        r = rng.random()
        if r < 0.3:
            assert (e.policy_delete(ep, k) == 0) == (o.policy_delete(ep, k) == 0)
            continue
        if r < 0.6:  # a key that may not exist yet
            k = L.policy_key(int(rng.integers(256, 1256)), int(rng.choice(synth.PORTS64)),
                             int(rng.choice([6, 17])), int(rng.integers(0, 2)))
        en = L.policy_entry(int(rng.integers(0, 3)) * 1000, 0, 0)
        assert e.policy_update(ep, k, en) == 0 and o.policy_update(ep, k, en) == 0


def _full_copy(e, T):
    """A fresh context loaded with e's current mirror (full compile)."""
    f = _engine(**T.engine_config())
    keys = e.ipcache_keys()
    for k in keys:
        rc, v = e.ipcache_lookup(k)
        assert rc == 0 and f.ipcache_update(k, v) == 0
    for ep in range(T.n_endpoints):
        ks, ents = e.policy_dump(ep)
        for k, en in zip(ks, ents):
            assert f.policy_update(ep, k, L.policy_entry(L.ntohs(int(en["proxy_port"])))) == 0
    f.commit()
    return f


def test_incremental_commits_match_full_and_oracle(torch_cuda):
    """Rounds of small deltas (patched in place), then a large one (full
    recompile): after every commit the verdicts, identities and stages equal
    the restatement's and a context compiled from scratch over the same
    mirror."""
    from oracle import Oracle
    torch = torch_cuda
    T = synth.make_tables(**synth.CONFIGS["cpu"])
    t = synth.make_tuples(T, 1 << 19)
    d = synth.to_device(t)
    e = _engine(**T.engine_config())
    o = Oracle(**T.oracle_config())
    synth.load_engine(e, T)
    synth.load_oracle(o, T)
    e.commit()
    rng = np.random.default_rng(5)
    for rnd, (ni, npol) in enumerate([(1, 0), (0, 1), (5, 5), (40, 40), (300, 300), (5000, 100),
                                      (3, 6000), (1, 1)]):
        _mutate(rng, T, e, o, ni, npol)
        e.commit()
        _check(torch, e, o, t, d, f"round {rnd}")
        f = _full_copy(e, T)
        assert f.checksum() == e.checksum()
        out = f.classify_v4(d)
        torch.cuda.synchronize()
        ref = e.classify_v4(d)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(_np(out["verdict"]), _np(ref["verdict"]))
        np.testing.assert_array_equal(_np(out["identity"]), _np(ref["identity"]))
        f.close()
    # counters: the reference's per-entry semantics survive the commits
    e.counters_reset()
    o.counters_reset()
    _check(torch, e, o, t, d, "counters")
    rc, got = e.policy_lookup_batch(T.pol_ep, T.pol_keys)
    for i in np.nonzero(rc == 0)[0][::13]:
        r0, raw = o.policy_lookup(int(T.pol_ep[i]), T.pol_keys[i])
        exp = np.frombuffer(raw, L.POLICY_ENTRY)[0]
        assert r0 == 0
        assert (int(got[i]["packets"]), int(got[i]["bytes"])) == (int(exp["packets"]), int(exp["bytes"]))
    np.testing.assert_array_equal(e.metrics(), o.metrics())
    e.close()


def test_static_part_and_short_prefix_changes(torch_cuda):
    """Changes that reach every address: /0, static-part entries (prefixlen
    < 32) and a /1 -- the incremental path recompiles what they cover."""
    from oracle import Oracle
    torch = torch_cuda
    T = synth.make_tables(n_prefixes=3000, n_identities=300, n_endpoints=2, keys_per_ep=3000)
    t = synth.make_tuples(T, 1 << 17)
    d = synth.to_device(t)
    e = _engine(**T.engine_config())
    o = Oracle(**T.oracle_config())
    synth.load_engine(e, T)
    synth.load_oracle(o, T)
    e.commit()
    k0 = L.ipcache_key("0.0.0.0/0")
    stat = np.zeros((), L.IPCACHE_KEY)
    stat["prefixlen"] = 24
    for what, key, lab in [("relabel /0", k0, 777), ("static /24", stat, 555), ("/1", L.ipcache_key("128.0.0.0/1"), 900),
                           ("delete /0", k0, None), ("delete static", stat, None)]:
        if lab is None:
            assert e.ipcache_delete(key) == 0 and o.ipcache_delete(key) == 0
        else:
            v = L.remote_info(lab, 0)
            assert e.ipcache_update(key, v) == 0 and o.ipcache_update(key, v) == 0
        e.commit()
        _check(torch, e, o, t, d, what)
    e.close()


def test_single_key_policy_commit_is_submillisecond(torch_cuda):
    """Config-2 tables: a one-key policy write + commit patches the policy
    table in place and uploads only its group: < 1 ms median."""
    from oracle import Oracle
    torch = torch_cuda
    T = synth.make_tables(**synth.CONFIGS["gpu"])
    e = _engine(**T.engine_config())
    synth.load_engine(e, T)
    t0 = time.perf_counter()
    e.commit()
    full = time.perf_counter() - t0
    times = []
    rng = np.random.default_rng(3)
    for i in range(60):
        k = L.policy_key(int(rng.integers(256, 1256)), 80, 6, i & 1)
        assert e.policy_update(i % 4, k, L.policy_entry(0, 0, 0)) == 0
        t0 = time.perf_counter()
        e.commit()
        times.append(time.perf_counter() - t0)
    med = float(np.median(times[10:]))
    print(f"full commit {full * 1e3:.1f} ms, single-key policy commit median {med * 1e6:.0f} us, "
          f"max {max(times[10:]) * 1e6:.0f} us")
    assert med < 1e-3, times
    # and the result is the reference's
    o = Oracle(**T.oracle_config())
    synth.load_oracle(o, T)
    rng = np.random.default_rng(3)
    for i in range(60):
        k = L.policy_key(int(rng.integers(256, 1256)), 80, 6, i & 1)
        assert o.policy_update(i % 4, k, L.policy_entry(0, 0, 0)) == 0
    t = synth.make_tuples(T, 1 << 20)
    _check(torch, e, o, t, synth.to_device(t), "after single-key commits")
    e.close()


def test_commit_does_not_block_classification(torch_cuda):
    """Config 5 (1M services + config-2 tables): one thread classifies in a
    loop while another rewrites the service map and commits (the LB group
    recompile takes most of a second).  No launch waits for the commit; the
    batch after the commit is bit-exact against the restatement."""
    from oracle import Oracle
    torch = torch_cuda
    cfg = synth.CONFIGS["cascade"]
    T = synth.make_tables(**cfg)
    S = synth.make_services(T, cfg["n_services"])
    t = synth.add_service_traffic(synth.make_tuples(T, 1 << 22), S)
    del t["hash"]
    e = _engine(**T.engine_config(), lb_max_entries=len(S.keys))
    synth.load_engine(e, T)
    synth.load_services(e, S)
    e.commit()
    d = synth.to_device(t)
    out = {"verdict": torch.empty(len(t["saddr"]), dtype=torch.int32, device="cuda"),
           "identity": torch.empty(len(t["saddr"]), dtype=torch.int32, device="cuda"),
           "stage": None}
    stream = torch.cuda.Stream()
    e.classify_v4_lb(d, out=out, stream=stream)
    stream.synchronize()
    # the commit thread: drop every 10th service, then commit
    drop = np.zeros(len(S.keys), bool)
    drop[np.isin(S.keys["address"], S.vip[::10])] = True
    stop = threading.Event()
    span = {}

    def committer():
        for k in S.keys[drop]:
            assert e.lb4_delete(k) == 0
        span["t0"] = time.perf_counter()
        e.commit()
        span["t1"] = time.perf_counter()
        stop.set()

    lat = []
    th = threading.Thread(target=committer)
    th.start()
    with torch.cuda.stream(stream):
        while not stop.is_set():
            t0 = time.perf_counter()
            e.classify_v4_lb(d, out=out, stream=stream)
            lat.append((t0, time.perf_counter() - t0))
            stream.synchronize()
    th.join()
    commit_s = span["t1"] - span["t0"]
    during = [x for t0, x in lat if span["t0"] <= t0 <= span["t1"]]
    print(f"commit {commit_s * 1e3:.0f} ms; {len(during)} launches during it, "
          f"max enqueue {max(during) * 1e3:.2f} ms" if during else "no launch overlapped")
    assert commit_s > 0.05
    assert len(during) >= 2
    assert max(during) < commit_s / 4
    # the next batch sees the new services, bit-exact
    o = Oracle(**T.oracle_config())
    synth.load_oracle(o, T)
    synth.load_services(o, synth.Services(S.keys[~drop], S.vals[~drop], S.vip, S.port))
    e.classify_v4_lb(d, out=out, stream=stream)
    stream.synchronize()
    v0, i0, _, _ = o.classify_v4_lb(t, nthreads=16)
    np.testing.assert_array_equal(_np(out["verdict"]), v0)
    np.testing.assert_array_equal(_np(out["identity"], np.uint32), i0)
    e.close()


def test_counter_slot_quarantine_across_commits(torch_cuda):
    """A deleted key's counter slot is not handed to a new key while a
    snapshot that still maps it may run: with every slot in use, deleting
    and re-adding keys across commits keeps every key's counters exact."""
    from oracle import Oracle
    torch = torch_cuda
    e = _engine(policy_max_total=64, hot_counter_slots=0, max_endpoints=2)
    o = Oracle()
    keys = [L.policy_key(300 + i, 80, 6, 1) for i in range(40)]
    for k in keys:
        assert e.policy_update(0, k, L.policy_entry(0)) == 0 and o.policy_update(0, k, L.policy_entry(0)) == 0
    n = 4096
    e.commit()
    rng = np.random.default_rng(1)
    for rnd in range(30):
        i = int(rng.integers(0, len(keys)))
        assert e.policy_delete(0, keys[i]) == 0 and o.policy_delete(0, keys[i]) == 0
        keys[i] = L.policy_key(5000 + rnd, 80, 6, 1)
        assert e.policy_update(0, keys[i], L.policy_entry(0)) == 0
        assert o.policy_update(0, keys[i], L.policy_entry(0)) == 0
        e.commit()
        t = {"saddr": np.zeros(n, np.uint32), "daddr": np.zeros(n, np.uint32),
             "dport": np.full(n, L.htons(80), np.uint16), "proto": np.full(n, 6, np.uint8),
             "flags": np.ones(n, np.uint8), "len": rng.integers(64, 1500, n).astype(np.uint32),
             "ep": np.zeros(n, np.uint16)}
        ids = np.array([int(k["sec_label"]) for k in keys], np.uint32)
        lab = ids[rng.integers(0, len(ids), n)]
        for j, x in enumerate(lab[:64]):
            assert e.ipcache_update(L.ipcache_key(f"10.9.{j}.1/32"), L.remote_info(int(x))) in (0,)
            assert o.ipcache_update(L.ipcache_key(f"10.9.{j}.1/32"), L.remote_info(int(x))) == 0
        t["daddr"] = np.array([L.ip4_be((10 << 24) | (9 << 16) | (j % 64 << 8) | 1) for j in range(n)], np.uint32)
        e.commit()
        _check(torch, e, o, t, synth.to_device(t), f"round {rnd}")
    for k in keys:
        rc, got = e.policy_lookup(0, k)
        r0, raw = o.policy_lookup(0, k)
        exp = np.frombuffer(raw, L.POLICY_ENTRY)[0]
        assert rc == 0 and r0 == 0
        assert (int(got["packets"]), int(got["bytes"])) == (int(exp["packets"]), int(exp["bytes"]))
    e.close()


def test_counters_allreduce_one_rank(torch_cuda):
    """cgpu_comm_init + cgpu_counters_allreduce on a one-rank communicator:
    the SUM is the identity, so the folded counters equal the restatement's
    (the N-rank algebra is covered on CPU, tests/test_multi_gloo.py)."""
    from oracle import Oracle
    from cilium_amd.engine import Engine
    torch = torch_cuda
    T = synth.make_tables(**synth.CONFIGS["cpu"])
    t = synth.make_tuples(T, 1 << 20)
    e = _engine(**T.engine_config())
    synth.load_engine(e, T)
    e.commit()
    e.comm_init(Engine.comm_id(), 1, 0)
    buf = torch.zeros(e.counter_delta_bytes() // 8, dtype=torch.int64, device="cuda")
    e.counter_bind(buf)
    e.classify_v4(synth.to_device(t), stage=False)
    before = buf.clone()
    e.counters_allreduce()
    torch.cuda.synchronize()
    assert torch.equal(before, buf)
    e.counter_fold()
    o = Oracle(**T.oracle_config())
    synth.load_oracle(o, T)
    o.classify_v4(t, nthreads=16)
    np.testing.assert_array_equal(e.metrics(), o.metrics())
    got = e.policy_counters(T.pol_ep, T.pol_keys)
    for i in range(0, len(T.pol_keys), 97):
        _, raw = o.policy_lookup(int(T.pol_ep[i]), T.pol_keys[i])
        exp = np.frombuffer(raw, L.POLICY_ENTRY)[0]
        assert (int(got[i, 0]), int(got[i, 1])) == (int(exp["packets"]), int(exp["bytes"]))
    e.counter_bind(None)
    e.close()


def test_counter_slot_layout_deterministic(torch_cuda):
    """Counter slots are assigned from the sequence of map operations and
    commits alone: two contexts applying the same delete/insert
    churn over a small slot space -- one with classify launches in flight
    between commits, one idle -- report the same counter layout checksum
    after every commit, so the slot-by-slot RCCL SUM adds like to like."""
    torch = torch_cuda
    busy = _engine(policy_max_total=64, hot_counter_slots=8, max_endpoints=2)
    idle = _engine(policy_max_total=64, hot_counter_slots=8, max_endpoints=2)
    keys = [L.policy_key(300 + i, 80 if i % 3 else 0, 6 if i % 3 else 0, 1) for i in range(44)]
    for e in (busy, idle):
        for k in keys:
            assert e.policy_update(0, k, L.policy_entry(0)) == 0
        e.commit()
    n = 1 << 20
    rng = np.random.default_rng(7)
    t = {"saddr": np.zeros(n, np.uint32), "daddr": rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32),
         "dport": np.full(n, L.htons(80), np.uint16), "proto": np.full(n, 6, np.uint8),
         "flags": np.ones(n, np.uint8), "len": np.full(n, 100, np.uint32), "ep": np.zeros(n, np.uint16)}
    d = synth.to_device(t)
    for rnd in range(40):
        i = int(rng.integers(0, len(keys)))
        new = L.policy_key(7000 + rnd, 0 if rnd % 2 else 443, 0 if rnd % 2 else 6, 1)
        for e in (busy, idle):
            assert e.policy_delete(0, keys[i]) == 0
            rc = e.policy_update(0, new, L.policy_entry(0))
            assert rc == 0, rc
        keys[i] = new
        for _ in range(3):
            busy.classify_v4(d, stage=False)  # launches still running at the commit
        busy.commit()
        idle.commit()
        assert busy.counter_layout_checksum() == idle.counter_layout_checksum(), f"round {rnd}"
        assert busy.checksum() == idle.checksum()
    torch.cuda.synchronize()
    busy.close()
    idle.close()


def test_table_verify_detects_corruption(torch_cuda):
    """SURVEY §5 failure detection: every commit checks the device's sum of
    each uploaded group against the host image; cgpu_table_verify re-checks
    the published snapshot, and a flipped byte in any group is an EIO that
    names it; a fresh commit from the host mirror repairs it."""
    from cilium_amd._abi import CgpuError
    T = synth.make_tables(n_prefixes=3000, n_identities=200, n_endpoints=2, keys_per_ep=2000)
    e = _engine(**T.engine_config())
    synth.load_engine(e, T)
    e.endpoint_update(L.endpoint_key("10.1.0.1"))
    e.commit()
    e.verify()
    for group, off in ((0, 4096 + 3), (1, 77)):
        assert e.L.cgpu__test_corrupt(e.h, group, off, 0x10) == 0
        with pytest.raises(CgpuError) as ex:
            e.verify()
        assert ex.value.errno == errno.EIO
        # the host mirror is authoritative: rewrite the group and commit
        if group == 0:
            k, v = T.ipc_keys[0], T.ipc_vals[0]
            assert e.ipcache_delete(k) == 0
            e.commit()
            assert e.ipcache_update(k, v) == 0
        else:
            k, en, ep = T.pol_keys[0], T.pol_entries[0], T.pol_ep[0]
            assert e.policy_delete(int(ep), k) == 0
            e.commit()
            assert e.policy_update(int(ep), k, en) == 0
        e.commit()
        e.verify()
    e.close()


def test_mirror_save_restore_resumes(torch_cuda, tmp_path):
    """SURVEY §5 checkpoint / resume on the device: after classify and
    conntrack batches, a checkpoint restored into a fresh context (then
    committed) holds the same per-entry counters and conntrack map, and the
    next batches on both contexts produce identical verdicts, counters and
    maps."""
    torch = torch_cuda
    T = synth.make_tables(**synth.CONFIGS["cpu"])
    T.n_endpoints = 1
    t = synth.make_tuples(T, 1 << 18)
    tc, locals_be, seclabels = synth.make_ct_workload(T, 5000, mean_pkts=8.0)
    e = _engine(**T.engine_config(), ct_max=1 << 16)
    synth.load_engine(e, T)
    synth.load_lxc(e, seclabels)
    e.commit()
    e.classify_v4(synth.to_device(t), stage=False)
    half = len(tc["saddr"]) // 2
    first = {k: v[:half] for k, v in tc.items()}
    rest = {k: v[half:] for k, v in tc.items()}
    e.classify_v4_ct(synth.to_device(first), 100)
    torch.cuda.synchronize()
    path = str(tmp_path / "ckpt.bin")
    e.mirror_save(path)
    f = _engine(**T.engine_config(), ct_max=1 << 16)
    f.mirror_restore(path)
    f.commit()
    np.testing.assert_array_equal(f.policy_counters(T.pol_ep, T.pol_keys),
                                  e.policy_counters(T.pol_ep, T.pol_keys))
    for a, b in zip(e.ct4_dump(), f.ct4_dump()):
        np.testing.assert_array_equal(a, b)
    outs = []
    for x in (e, f):
        o = x.classify_v4_ct(synth.to_device(rest), 104)
        torch.cuda.synchronize()
        outs.append({k: v.cpu().numpy() for k, v in o.items() if v is not None})
    for k in outs[0]:
        np.testing.assert_array_equal(outs[0][k], outs[1][k], err_msg=k)
    np.testing.assert_array_equal(f.policy_counters(T.pol_ep, T.pol_keys),
                                  e.policy_counters(T.pol_ep, T.pol_keys))
    for a, b in zip(e.ct4_dump(), f.ct4_dump()):
        np.testing.assert_array_equal(a, b)
    e.close()
    f.close()


def test_counters_rebalance_popularity(torch_cuda):
    """cgpu_counters_rebalance: after traffic, the most-hit keys take the hot
    (LDS) counter slots and carry their counters; every per-entry counter and
    the metrics stay equal to the restatement's across the move, further
    batches and later map changes; a second rebalance on the same totals
    moves nothing; replicas with the same totals choose the same layout."""
    from oracle import Oracle
    torch = torch_cuda
    T = synth.make_tables(**synth.CONFIGS["cpu"])
    t1 = synth.make_tuples(T, 1 << 20)
    t2 = synth.make_tuples(T, 1 << 20, gpu_id=5)
    o = Oracle(**T.oracle_config())
    synth.load_oracle(o, T)
    es = []
    for _ in range(2):
        e = _engine(**T.engine_config(), hot_counter_slots=2048)
        synth.load_engine(e, T)
        e.commit()
        es.append(e)
    e, r = es
    for x in es:
        x.classify_v4(synth.to_device(t1), stage=False)
    o.classify_v4(t1, nthreads=16)
    lay0 = e.counter_layout_checksum()
    moved = e.counters_rebalance()
    assert moved > 0 and r.counters_rebalance() == moved
    assert e.counter_layout_checksum() != lay0
    assert e.counter_layout_checksum() == r.counter_layout_checksum()
    assert e.counters_rebalance() == 0  # stable on the same totals

    def same():
        torch.cuda.synchronize()
        got = e.policy_counters(T.pol_ep, T.pol_keys)
        for i in range(len(T.pol_keys)):
            _, raw = o.policy_lookup(int(T.pol_ep[i]), T.pol_keys[i])
            exp = np.frombuffer(raw, L.POLICY_ENTRY)[0]
            assert (int(got[i, 0]), int(got[i, 1])) == (int(exp["packets"]), int(exp["bytes"])), i
        np.testing.assert_array_equal(e.metrics(), o.metrics())
    same()
    out = e.classify_v4(synth.to_device(t2))
    v0, i0, s0, _ = o.classify_v4(t2, nthreads=16)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out["verdict"].cpu().numpy(), v0)
    same()
    # map changes after the move: deletes, re-adds, new keys
    for i in range(0, 400, 7):
        k, ep = T.pol_keys[i], int(T.pol_ep[i])
        assert e.policy_delete(ep, k) == 0 and o.policy_delete(ep, k) == 0
    for i in range(0, 400, 14):
        k, en, ep = T.pol_keys[i], T.pol_entries[i], int(T.pol_ep[i])
        assert e.policy_update(ep, k, en) == 0 and o.policy_update(ep, k, en) == 0
    e.commit()
    out = e.classify_v4(synth.to_device(t1))
    v0, i0, s0, _ = o.classify_v4(t1, nthreads=16)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out["verdict"].cpu().numpy(), v0)
    np.testing.assert_array_equal(e.metrics(), o.metrics())
    for x in es:
        x.close()
