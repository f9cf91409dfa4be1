"""The threaded restatement of the stateful paths (Oracle.sharded, the CPU
baseline of bench.py --config ct / ct6 / ctlb / ctlb6): packets split into
independent conntrack groups run on separate threads in views with their own
conntrack maps.  For address-pair shards (shard.ct_shard_of: every key a
packet touches carries its pair) the result must equal the sequential
restatement exactly: verdicts, ct results, identities, stages, the reference
map-operation count, the merged conntrack map and the metrics."""
import numpy as np
import pytest

from cilium_amd import shard, synth
from oracle import Oracle


def _oracle(T, sl, S=None, v6=False):
    o = Oracle(**T.oracle_config())
    synth.load_oracle(o, T)
    synth.load_lxc(o, sl)
    if S is not None:
        (synth.load_services6 if v6 else synth.load_services)(o, S)
    return o


@pytest.mark.parametrize("v6", [False, True])
def test_pair_sharded_ct_equals_sequential(v6):
    if v6:
        T = synth.make_tables6(n_prefixes=3000, n_identities=300, n_endpoints=2, keys_per_ep=2000)
        t, _, sl = synth.make_ct6_workload(T, 20_000, mean_pkts=6.0, span=0.05)
    else:
        T = synth.make_tables(n_prefixes=3000, n_identities=300, n_endpoints=2, keys_per_ep=2000)
        t, _, sl = synth.make_ct_workload(T, 20_000, mean_pkts=6.0, span=0.05)
    meth = "classify_v6_ct" if v6 else "classify_v4_ct"
    seq = _oracle(T, sl)
    ref = getattr(seq, meth)(t, 1000)
    par = _oracle(T, sl)
    got, wall = par.sharded(meth, t, 1000, shard.ct_shard_of(t, 7), nthreads=4)
    assert wall > 0
    for a, b in zip(got, ref):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(par.metrics(), seq.metrics())
    dump = "ct6_dump" if v6 else "ct4_dump"
    for a, b in zip(getattr(par, dump)(), getattr(seq, dump)()):
        np.testing.assert_array_equal(a, b)


def test_conn_sharded_ctlb_close_to_sequential():
    """The service path threaded by connection (shard.conn_shard_of, the RSS
    analogue, bench.py's CPU baseline for ctlb): not an exact partition
    (ICMP-related entries are shared by the connections of an address pair,
    replies from a VIP and from its backend meet in the backend's pair), so
    bench.py reports how many results equal the sequential run's.  On the
    bench's kind of stream nearly all do; the map holds the same keys."""
    T = synth.make_tables(n_prefixes=3000, n_identities=300, n_endpoints=2, keys_per_ep=2000)
    S = synth.make_services(T, 3000)
    t, _, sl, S = synth.make_ctlb_workload(T, S, 20_000, mean_pkts=8.0, loop_frac=1e-4)
    seq = _oracle(T, sl, S)
    ref = seq.classify_v4_ctlb(t, 1000)
    par = _oracle(T, sl, S)
    got, _ = par.sharded("classify_v4_ctlb", t, 1000, shard.conn_shard_of(t, 5), nthreads=4)
    for k in ("verdict", "ct_ret", "identity", "xdaddr", "xdport"):
        assert np.mean(got[k] == ref[k]) > 0.99, k
    # a single shard is the sequential run itself
    one = _oracle(T, sl, S)
    got1, _ = one.sharded("classify_v4_ctlb", t, 1000, np.zeros(len(t["saddr"]), np.int64), nthreads=4)
    for k in ("verdict", "ct_ret", "identity", "stage", "xdaddr", "xdport"):
        np.testing.assert_array_equal(got1[k], ref[k], err_msg=k)


@pytest.mark.parametrize("v6", [False, True])
def test_component_sharded_ctlb_equals_sequential(v6):
    """The service path threaded over shard.svc_component_shard_of (bench.py's
    ctlb / ctlb6 cpu_baseline): the connected components
    of the address pairs a packet can touch through any backend of its
    service are independent conntrack groups, so the threaded run equals the
    sequential one exactly -- every output, the metrics and the whole map --
    with loopback backends (1 % of the connections) in the stream."""
    from cilium_amd import layouts as L
    if v6:
        T = synth.make_tables6(n_prefixes=3000, n_identities=300, n_endpoints=2, keys_per_ep=2000)
        S = synth.make_services6(T, 3000)
        t, _, sl, S = synth.make_ctlb6_workload(T, S, 20_000, mean_pkts=8.0, loop_frac=1e-2)
    else:
        T = synth.make_tables(n_prefixes=3000, n_identities=300, n_endpoints=2, keys_per_ep=2000)
        S = synth.make_services(T, 3000)
        t, _, sl, S = synth.make_ctlb_workload(T, S, 20_000, mean_pkts=8.0, loop_frac=1e-2)
    meth = "classify_v6_ctlb" if v6 else "classify_v4_ctlb"
    seq = _oracle(T, sl, S, v6)
    ref = getattr(seq, meth)(t, 1000)
    par = _oracle(T, sl, S, v6)
    comp = shard.svc_component_shard_of(t, S.keys, S.vals, 16, 0 if v6 else L.IPV4_LOOPBACK)
    assert len(np.unique(comp)) == 16
    got, _ = par.sharded(meth, t, 1000, comp, nthreads=4)
    for k in ("verdict", "ct_ret", "identity", "stage", "xdaddr", "xdport"):
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
    np.testing.assert_array_equal(par.metrics(), seq.metrics())
    dump = "ct6_dump" if v6 else "ct4_dump"
    for a, b in zip(getattr(par, dump)(), getattr(seq, dump)()):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("v6", [False, True])
def test_sharded_steps_equals_sequential_with_gc(v6):
    """Oracle.sharded_steps (bench.py --ct-persist): pair-shard views whose
    maps persist over batches at advancing times with ctmap.GC between them
    give the sequential restatement's results, GC counts and map."""
    if v6:
        T = synth.make_tables6(n_prefixes=3000, n_identities=300, n_endpoints=2, keys_per_ep=2000)
        t, _, sl = synth.make_ct6_workload(T, 10_000, mean_pkts=6.0, span=0.05)
    else:
        T = synth.make_tables(n_prefixes=3000, n_identities=300, n_endpoints=2, keys_per_ep=2000)
        t, _, sl = synth.make_ct_workload(T, 10_000, mean_pkts=6.0, span=0.05)
    meth = "classify_v6_ct" if v6 else "classify_v4_ct"
    ops = [("cls", 1000), ("cls", 1030), ("gc", 1065), ("cls", 1070), ("cls", 1100), ("gc", 1200),
           ("cls", 1201)]
    seq = _oracle(T, sl)
    dels = []
    for op, tm in ops:
        if op == "gc":
            dels.append((seq.ct6_gc if v6 else seq.ct4_gc)(tm))
        else:
            ref = getattr(seq, meth)(t, tm)
    par = _oracle(T, sl)
    got, walls, gdels = par.sharded_steps(meth, t, shard.ct_shard_of(t, 7), 4, ops)
    assert len(walls) == len(ops) and gdels == dels and dels[0] > 0
    for a, b in zip(got, ref):
        np.testing.assert_array_equal(a, b)
    dump = "ct6_dump" if v6 else "ct4_dump"
    for a, b in zip(getattr(par, dump)(), getattr(seq, dump)()):
        np.testing.assert_array_equal(a, b)
