"""GPU parity of the raw-frame path (cgpu_frames_parse / cgpu_classify_frames,
SURVEY §8f row 2) through the C ABI: against the reference's golden vectors
(tests/golden/frames.npz, built from the reference's own bpf/lib headers) and,
at larger sizes, against the CPU restatement pinned by those vectors.
Bit-exact throughout."""
import numpy as np
import pytest

from cilium_amd import build, layouts as L, synth
from test_frames_golden import VARIANTS, frame_oracle, frames_of

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU test needs a device"
    build.build()
    return torch


def _engine(gate, verify, n_ep=5, **kw):
    from cilium_amd.engine import Engine
    e = Engine(device=0, ct_proto_gate=gate, **kw)
    info = L.lxc_info(synth.LXC_MAC, synth.LXC_IPV4_RAW, synth.LXC_IP6, verify)
    for ep in range(n_ep):
        assert e.lxc_update(ep, info) == 0
    return e


def _parse(torch, e, f):
    out = e.frames_parse(synth.frames_to_device(f))
    torch.cuda.synchronize()
    r = {k: v.cpu().numpy() for k, v in out.items()}
    r["dport"] = r["dport"].view(np.uint16)
    return r


def _check_parse(got, exp, frag_key="flags"):
    np.testing.assert_array_equal(got["status"], exp["status"])
    ok = exp["status"] == 0
    for k in ("family", "saddr", "daddr", "dport", "proto"):
        np.testing.assert_array_equal(got[k][ok], exp[k][ok], err_msg=k)
    np.testing.assert_array_equal(got["flags"][ok], exp[frag_key][ok])


@pytest.mark.parametrize("variant", sorted(VARIANTS))
def test_frames_parse_golden(torch_cuda, golden, variant):
    g = golden("frames.npz")
    e = _engine(*VARIANTS[variant])
    e.commit()
    got = _parse(torch_cuda, e, frames_of(g))
    exp = {k: g[f"{variant}_{k}"] for k in ("status", "family", "saddr", "daddr", "dport",
                                             "proto")}
    exp["flags"] = (g["flags"] & 1) | (g[f"{variant}_frag"] << 1)
    _check_parse(got, exp)
    e.close()


@pytest.mark.parametrize("variant", sorted(VARIANTS))
@pytest.mark.parametrize("stride", [64, 128, 256])
def test_frames_parse_vs_restatement(torch_cuda, variant, stride):
    """200k frames of every class; narrower slots exercise DROP_SNAPLEN."""
    rng = np.random.Generator(np.random.PCG64(0xF0 + stride))
    f = synth.make_frames(rng, 200_000, width=256)
    f["data"] = np.ascontiguousarray(f["data"][:, :stride])
    e = _engine(*VARIANTS[variant])
    e.commit()
    got = _parse(torch_cuda, e, f)
    o = frame_oracle(*VARIANTS[variant])
    _check_parse(got, o.frames_parse(f))
    if stride == 64:
        assert (got["status"] == L.DROP_SNAPLEN).sum() > 0
    e.close()


def _classify_frames(torch, e, f):
    out = e.classify_frames(synth.frames_to_device(f))
    torch.cuda.synchronize()
    return (out["verdict"].cpu().numpy(), out["identity"].cpu().numpy().view(np.uint32),
            out["stage"].cpu().numpy())


SCHED_FRAMES_SPLIT = 8  # CGPU_SCHED_FRAMES_SPLIT: header pass + classify pass instead of the fused kernel


@pytest.mark.parametrize("gate,verify", [(1, 7), (0, 7), (1, 0)])
@pytest.mark.parametrize("stride,sched", [(128, 0), (64, 0), (64, SCHED_FRAMES_SPLIT)])
def test_classify_frames_vs_restatement(torch_cuda, gate, verify, stride, sched):
    """Mixed v4 / v6 frames through the whole decision: verdicts, identities,
    stages, per-entry counters and metrics equal the restatement's: the
    parse pass + classify pass (128-byte slots, or the split schedule), and
    with 64-byte slots the default fused kernel (the classify kernel parses
    the slots itself, staged through LDS)."""
    T = synth.make_tables(n_prefixes=5000, n_identities=300, n_endpoints=5, keys_per_ep=3000)
    rng = np.random.Generator(np.random.PCG64(0xC1A55 + gate + verify))
    pool = T.pfx_addr.astype(np.uint32).byteswap()
    f = synth.make_frames(rng, 300_000, width=128, addr4=pool)
    f["data"] = np.ascontiguousarray(f["data"][:, :stride])
    e = _engine(gate, verify, **T.engine_config(), schedule=sched)
    synth.load_engine(e, T)
    e.commit()
    o = frame_oracle(gate, verify, **T.oracle_config())
    synth.load_oracle(o, T)
    v, idt, st = _classify_frames(torch_cuda, e, f)
    ov, oi, ost, _ = o.classify_frames(f, nthreads=8)
    np.testing.assert_array_equal(v, ov)
    np.testing.assert_array_equal(idt, oi)
    np.testing.assert_array_equal(st, ost)
    assert len(np.unique(st)) >= 5
    np.testing.assert_array_equal(e.metrics(), o.metrics())
    for k, en, ep in zip(T.pol_keys[::7], T.pol_entries[::7], T.pol_ep[::7]):
        rc, got = e.policy_lookup(int(ep), k)
        orc, raw = o.policy_lookup(int(ep), k)
        want = np.frombuffer(raw, L.POLICY_ENTRY)[0]
        assert rc == 0 and orc == 0
        assert (int(got["packets"]), int(got["bytes"])) == (int(want["packets"]),
                                                           int(want["bytes"]))
    e.close()


@pytest.mark.parametrize("stride,sched", [(128, 0), (64, 0), (64, SCHED_FRAMES_SPLIT)])
@pytest.mark.parametrize("kind", ["runt", "v6", "not_classified"])
@pytest.mark.parametrize("tail", [1, 2, 3, 63, 65])
def test_classify_frames_ragged_tail(torch_cuda, tail, kind, stride, sched):
    """Batches of 4k + tail frames whose last partial quad starts with a frame
    the x4 schedule does not carry through its cascade: a runt the parse
    drops (DROP_INVALID, counted in the metrics), an IPv6 frame (its v4
    columns are placeholders until the v6 pass scatters its result back) or
    an egress ARP frame (FRAME_NOT_CLASSIFIED: stage 7, no metrics).  The
    tail lanes repeat that frame's columns and must count nothing: verdicts,
    identities, stages and metrics equal the restatement's."""
    T = synth.make_tables(n_prefixes=2000, n_identities=100, n_endpoints=5, keys_per_ep=500)
    rng = np.random.Generator(np.random.PCG64(0x7A11 + tail))
    pool = T.pfx_addr.astype(np.uint32).byteswap()
    n = 4 * 5000 + tail
    f = synth.make_frames(rng, n, width=128, addr4=pool)
    f["data"] = np.ascontiguousarray(f["data"][:, :stride])
    o = frame_oracle(1, 7, **T.oracle_config())
    synth.load_oracle(o, T)
    at = n - tail
    if kind == "runt":
        f["len"][at] = 10
    else:
        p = o.frames_parse(f)
        want = (p["status"] == 0) & (p["family"] == 6) if kind == "v6" else \
            p["status"] == L.FRAME_NOT_CLASSIFIED
        j = int(np.flatnonzero(want[:at])[0])
        for k in ("data", "len", "flags", "ep"):
            f[k][at] = f[k][j]
    e = _engine(1, 7, **T.engine_config(), schedule=sched)
    synth.load_engine(e, T)
    e.commit()
    v, idt, st = _classify_frames(torch_cuda, e, f)
    ov, oi, ost, _ = o.classify_frames(f, nthreads=4)
    if kind == "runt":
        assert ov[at] == L.DROP_INVALID
    elif kind == "not_classified":
        assert ost[at] == 7
    np.testing.assert_array_equal(v, ov)
    np.testing.assert_array_equal(idt, oi)
    np.testing.assert_array_equal(st, ost)
    np.testing.assert_array_equal(e.metrics(), o.metrics())
    e.close()


def test_classify_frames_equals_classify_v4(torch_cuda):
    """Config-2 style tuples serialized as frames (64-byte slots) classify
    exactly as the tuples themselves do through cgpu_classify_v4."""
    T = synth.make_tables(n_prefixes=20_000, n_identities=500, n_endpoints=4, keys_per_ep=4000)
    t = synth.make_tuples(T, 1 << 20)
    f = synth.frames_from_tuples(t, stride=64)
    from cilium_amd.engine import Engine
    e1 = Engine(device=0, **T.engine_config())
    synth.load_engine(e1, T)
    e1.commit()
    e2 = Engine(device=0, **T.engine_config())
    synth.load_engine(e2, T)
    e2.commit()
    d = synth.to_device(t)
    out = e1.classify_v4(d)
    v, idt, st = _classify_frames(torch_cuda, e2, f)
    torch_cuda.cuda.synchronize()
    np.testing.assert_array_equal(v, out["verdict"].cpu().numpy())
    np.testing.assert_array_equal(idt, out["identity"].cpu().numpy().view(np.uint32))
    np.testing.assert_array_equal(st, out["stage"].cpu().numpy())
    np.testing.assert_array_equal(e1.metrics(), e2.metrics())
    e1.close()
    e2.close()


def test_frames_bad_layout_rejected(torch_cuda):
    import errno
    import ctypes as C
    from cilium_amd._abi import Frames, lib
    torch = torch_cuda
    e = _engine(1, 7)
    e.commit()
    buf = torch.zeros(4 * 256 + 16, dtype=torch.uint8, device="cuda")
    col = torch.zeros(4, dtype=torch.int32, device="cuda")
    v = torch.zeros(4, dtype=torch.int32, device="cuda")
    for stride, off in ((48, 0), (72, 0), (64, 4)):
        fr = Frames(buf.data_ptr() + off, col.data_ptr(), col.data_ptr(), col.data_ptr(), stride, 0)
        rc = lib().cgpu_classify_frames(e.h, C.byref(fr), 4, v.data_ptr(), v.data_ptr(), None,
                                        None)
        assert rc == -errno.EINVAL, (stride, off, rc)
    e.close()
