"""Host-resident forms of the service, cascade, IPv6 and prefilter paths
(cgpu_classify_v4_lb_host, _v4_cascade_host, _v6_host, _v6_lb_host,
cgpu_prefilter_v4_host / _v6_host): the same tuples from host
memory -- pageable numpy arrays, page-locked tensors, v6 address rows at an
odd byte offset -- over several staging chunks with a ragged last one give
exactly the results, per-entry counters and metrics of the device call, and
the restatement's (oracle/cgpu_oracle.c)."""
import os
import sys

import numpy as np
import pytest

from cilium_amd import layouts as L
from cilium_amd import synth

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "oracle"))

VIEW = {np.uint32: np.int32, np.uint16: np.int16, np.uint8: np.uint8, np.int32: np.int32}


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU test needs a device"
    from cilium_amd import build
    build.build()
    return torch


def _hostcols(torch, t, pinned):
    cols = {k: np.ascontiguousarray(v) for k, v in t.items()}
    if not pinned:
        return cols
    return {k: torch.from_numpy(v.view(VIEW.get(v.dtype.type, v.dtype))).pin_memory() for k, v in cols.items()}


def _odd_rows(a):
    """a (n, 16) uint8 copy whose rows start one byte past a 16-byte boundary"""
    buf = np.empty(a.size + 17, np.uint8)
    off = (-buf.ctypes.data) % 16 + 1
    v = buf[off:off + a.size].reshape(a.shape)
    v[:] = a
    assert v.ctypes.data % 16 == 1
    return v


def _counters(e, T, n=4000):
    out = []
    for k, ep in zip(T.pol_keys[:n], T.pol_ep[:n]):
        rc, got = e.policy_lookup(int(ep), k)
        assert rc == 0
        out.append((int(got["packets"]), int(got["bytes"])))
    return out


def _same(got, dev, ref=None):
    np.testing.assert_array_equal(got["verdict"], dev["verdict"].cpu().numpy())
    np.testing.assert_array_equal(got["identity"], dev["identity"].cpu().numpy().view(np.uint32))
    np.testing.assert_array_equal(got["stage"], dev["stage"].cpu().numpy())
    if ref is not None:
        v, i, s = ref
        np.testing.assert_array_equal(got["verdict"], v)
        np.testing.assert_array_equal(got["identity"], i)
        np.testing.assert_array_equal(got["stage"], s)


@pytest.fixture(scope="module")
def cfg_cascade():
    """Config-1 tables, 50k services, the config-5 deny set; 7M + 333 tuples
    (two staging chunks with the hash column, 22 B per tuple)."""
    from oracle import Oracle
    T = synth.make_tables(**synth.CONFIGS["cpu"])
    T.n_endpoints = 1
    S = synth.make_services(T, 50_000)
    P = synth.make_prefilter4(T)
    t = synth.add_prefilter_traffic(synth.add_service_traffic(synth.make_tuples(T, 7 * (1 << 20) + 333), S), P)
    o = Oracle(**T.oracle_config())
    synth.load_oracle(o, T)
    synth.load_services(o, S)
    synth.load_prefilter4(o, P)
    return T, S, P, t, o


def _engine4(T, S, P):
    from cilium_amd.engine import Engine
    e = Engine(device=0, **T.engine_config(), lb_max_entries=len(S.keys))
    synth.load_engine(e, T)
    synth.load_services(e, S)
    synth.load_prefilter4(e, P)
    e.commit()
    return e


@pytest.mark.parametrize("xdp", [True, False])
@pytest.mark.parametrize("with_hash,pinned", [(True, True), (False, False), (True, False)])
def test_lb_cascade_host(torch_cuda, cfg_cascade, xdp, with_hash, pinned):
    torch = torch_cuda
    T, S, P, t, o = cfg_cascade
    if not with_hash:
        t = {k: v for k, v in t.items() if k != "hash"}
    ed, eh = _engine4(T, S, P), _engine4(T, S, P)
    dev = ed.classify_v4_lb(synth.to_device(t), xdp=xdp)
    torch.cuda.synchronize()
    got = eh.classify_v4_lb_host(_hostcols(torch, t, pinned), xdp=xdp)
    o.counters_reset()
    ref = (o.classify_v4_cascade if xdp else o.classify_v4_lb)(t, nthreads=16)[:3]
    _same(got, dev, ref)
    np.testing.assert_array_equal(eh.metrics(), ed.metrics())
    np.testing.assert_array_equal(eh.metrics(), o.metrics())
    assert _counters(eh, T) == _counters(ed, T)
    if xdp:
        assert (got["verdict"] == L.VERDICT_XDP_DROP).sum() > 50_000
    ed.close()
    eh.close()


def test_prefilter_v4_host(torch_cuda, cfg_cascade):
    torch = torch_cuda
    T, S, P, t, o = cfg_cascade
    e = _engine4(T, S, P)
    sa, da, fl = (np.ascontiguousarray(t[k]) for k in ("saddr", "daddr", "flags"))
    dv = e.prefilter_v4(*(torch.from_numpy(x.view(VIEW[x.dtype.type])).cuda() for x in (sa, da, fl)))
    torch.cuda.synchronize()
    got = e.prefilter_host(sa, da, fl)
    ref, _ = o.prefilter_v4(sa, da, fl, nthreads=16)
    np.testing.assert_array_equal(got, dv.cpu().numpy())
    np.testing.assert_array_equal(got, ref)
    assert (ref == L.XDP_DROP).any() and (ref != L.XDP_DROP).any()
    e.close()


@pytest.fixture(scope="module")
def cfg_v6():
    """20k IPv6 prefixes, 20k v6 services; 4M + 5 tuples (two staging
    chunks at 42-46 B per tuple)."""
    from oracle import Oracle
    T = synth.make_tables6(n_prefixes=20_000, n_identities=500, n_endpoints=3, keys_per_ep=6000)
    S = synth.make_services6(T, 20_000)
    t = synth.add_service_traffic6(synth.make_tuples6(T, 4 * (1 << 20) + 5), S)
    o = Oracle(**T.oracle_config())
    synth.load_oracle(o, T)
    synth.load_services6(o, S)
    return T, S, t, o


@pytest.mark.parametrize("lb", [False, True])
@pytest.mark.parametrize("layout", ["pinned", "pageable", "odd"])
def test_v6_host(torch_cuda, cfg_v6, lb, layout):
    from cilium_amd.engine import Engine
    torch = torch_cuda
    T, S, t, o = cfg_v6
    if lb and layout == "odd":
        t = {k: v for k, v in t.items() if k != "hash"}

    def engine():
        e = Engine(device=0, **T.engine_config(), lb_max_entries=len(S.keys))
        synth.load_engine(e, T)
        synth.load_services6(e, S)
        e.commit()
        return e
    ed, eh = engine(), engine()
    dt = synth.to_device(t)
    dev = ed.classify_v6_lb(dt) if lb else ed.classify_v6(dt)
    torch.cuda.synchronize()
    cols = _hostcols(torch, t, layout == "pinned")
    if layout == "odd":
        cols["saddr"], cols["daddr"] = _odd_rows(t["saddr"]), _odd_rows(t["daddr"])
    got = eh.classify_v6_host(cols, lb=lb)
    o.counters_reset()
    ref = (o.classify_v6_lb if lb else o.classify_v6)(t, nthreads=16)[:3]
    _same(got, dev, ref)
    np.testing.assert_array_equal(eh.metrics(), ed.metrics())
    np.testing.assert_array_equal(eh.metrics(), o.metrics())
    assert _counters(eh, T) == _counters(ed, T)
    ed.close()
    eh.close()


def test_prefilter_v6_host(torch_cuda):
    """200k-prefix v6 deny set, 6M + 11 packets (two chunks at 33 B each),
    address rows at an odd offset."""
    from oracle import Oracle

    from cilium_amd.engine import Engine
    torch = torch_cuda
    P = synth.make_prefilter6(n_prefixes=200_000, n_roots=64, n_endpoints=512)
    p = synth.make_packets6(P, 6 * (1 << 20) + 11)
    o = Oracle(**P.oracle_config())
    synth.load_prefilter6(o, P)
    ref, _ = o.prefilter_v6(p["saddr"], p["daddr"], p["flags"], nthreads=16)
    e = Engine(device=0, **P.engine_config())
    synth.load_prefilter6(e, P)
    e.commit()
    d = synth.packets6_to_device(p)
    dv = e.prefilter_v6(d["saddr"], d["daddr"], d["flags"])
    torch.cuda.synchronize()
    got = e.prefilter_host(_odd_rows(p["saddr"]), _odd_rows(p["daddr"]), p["flags"], v6=True)
    np.testing.assert_array_equal(got, dv.cpu().numpy())
    np.testing.assert_array_equal(got, ref)
    pl = _hostcols(torch, p, True)
    got2 = e.prefilter_host(pl["saddr"], pl["daddr"], pl["flags"], v6=True)
    np.testing.assert_array_equal(got2, ref)
    e.close()


def test_host_paths_errors(torch_cuda):
    """null columns and a service call with neither hash nor sport fail
    with -EINVAL before anything is queued; n = 0 is a no-op."""
    import ctypes as C
    import errno

    from cilium_amd._abi import TuplesV4
    from cilium_amd.engine import Engine
    e = Engine(device=0)
    e.commit()
    z = np.zeros(4, np.uint32)
    tv = TuplesV4(*([z.ctypes.data] * 7))
    out = C.c_void_p(z.ctypes.data)
    for fn in ("cgpu_classify_v4_lb_host", "cgpu_classify_v4_cascade_host"):
        assert getattr(e.L, fn)(e.h, C.byref(tv), None, None, 4, out, out, None, None) == -errno.EINVAL
        assert getattr(e.L, fn)(e.h, C.byref(tv), None, None, 0, out, out, None, None) == 0
    assert e.L.cgpu_prefilter_v4_host(e.h, None, out, out, 4, out, None) == -errno.EINVAL
    assert e.L.cgpu_prefilter_v6_host(e.h, out, out, out, 0, out, None) == 0
    e.close()


@pytest.mark.parametrize("n", [1, 63, 4097])
def test_host_paths_small_batches(torch_cuda, cfg_cascade, cfg_v6, n):
    """Batches smaller than a vector quad, a wave and a staging alignment
    unit, through each host form (stage output omitted on one of them):
    equal to the device calls over the same tuples."""
    torch = torch_cuda
    T, S, P, t, _ = cfg_cascade
    t = {k: v[:n] for k, v in t.items()}
    ed, eh = _engine4(T, S, P), _engine4(T, S, P)
    dev = ed.classify_v4_lb(synth.to_device(t), xdp=True)
    torch.cuda.synchronize()
    got = eh.classify_v4_lb_host(_hostcols(torch, t, False), xdp=True)
    _same(got, dev)
    np.testing.assert_array_equal(eh.metrics(), ed.metrics())
    sa, da, fl = (np.ascontiguousarray(t[k]) for k in ("saddr", "daddr", "flags"))
    pv = eh.prefilter_host(sa, da, fl)
    dv = ed.prefilter_v4(*(torch.from_numpy(x.view(VIEW[x.dtype.type])).cuda() for x in (sa, da, fl)))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(pv, dv.cpu().numpy())
    ed.close()
    eh.close()
    from cilium_amd.engine import Engine
    T6, S6, t6, _ = cfg_v6
    t6 = {k: v[:n] for k, v in t6.items()}

    def engine():
        e = Engine(device=0, **T6.engine_config(), lb_max_entries=len(S6.keys))
        synth.load_engine(e, T6)
        synth.load_services6(e, S6)
        e.commit()
        return e
    ed, eh = engine(), engine()
    dev = ed.classify_v6(synth.to_device(t6), stage=False)
    torch.cuda.synchronize()
    got = eh.classify_v6_host(_hostcols(torch, t6, True), stage=False)
    np.testing.assert_array_equal(got["verdict"], dev["verdict"].cpu().numpy())
    np.testing.assert_array_equal(got["identity"], dev["identity"].cpu().numpy().view(np.uint32))
    assert got["stage"] is None
    np.testing.assert_array_equal(eh.metrics(), ed.metrics())
    ed.close()
    eh.close()
