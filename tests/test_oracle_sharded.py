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
