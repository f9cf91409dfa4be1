"""Pin the CPU restatement of the raw-frame path (oracle/cgpu_oracle.c
or_frames_parse / or_classify_frames) to the reference.

tests/golden/frames.npz was produced by the reference's own bpf/lib/{ipv4,
ipv6,lxc,lb,conntrack}.h compiled as host C (oracle/ref/harness_frame.c):
the steps of handle_ipv4_from_lxc / ipv6_l3_from_lxc (egress) and
ipv4_policy / ipv6_policy (ingress) before the ipcache lookup, with an empty
conntrack map, under three builds of the endpoint program:
  ct    : lxc_config.h as written (CONNTRACK, SMAC/DMAC/SIP checks)
  noct  : without CONNTRACK (conntrack.h stubs)
  nover : with DISABLE_{SMAC,DMAC,SIP}_VERIFICATION
Every check is bit-exact.
"""
import numpy as np
import pytest

from cilium_amd import layouts as L, synth
from oracle import Oracle

# variant -> (ct_proto_gate, verify bits)
VARIANTS = {"ct": (1, 7), "noct": (0, 7), "nover": (1, 0)}


def frame_oracle(gate, verify, n_ep=5, **kw):
    o = Oracle(ct_proto_gate=gate, **kw)
    info = L.lxc_info(synth.LXC_MAC, synth.LXC_IPV4_RAW, synth.LXC_IP6, verify)
    for ep in range(n_ep):
        assert o.lxc_update(ep, info) == 0
    return o


def frames_of(g):
    return {k: g[k] for k in ("data", "len", "flags", "ep")}


@pytest.mark.parametrize("variant", sorted(VARIANTS))
def test_harness_config_matches_synth(golden, variant):
    """The endpoint identity the harness was compiled with is the one the
    tests install (LXC_MAC, NODE_MAC, LXC_IPV4, LXC_IP, verify bits)."""
    g = golden("frames.npz")
    cfg = g[f"{variant}_config"].tobytes()
    assert cfg[0:6] == synth.LXC_MAC
    assert cfg[6:12] == L.NODE_MAC
    assert int.from_bytes(cfg[12:16], "little") == synth.LXC_IPV4_RAW
    assert cfg[16:32] == synth.LXC_IP6
    assert cfg[32] == VARIANTS[variant][1]


@pytest.mark.parametrize("variant", sorted(VARIANTS))
def test_frames_parse_vs_reference(golden, variant):
    g = golden("frames.npz")
    o = frame_oracle(*VARIANTS[variant])
    out = o.frames_parse(frames_of(g))
    np.testing.assert_array_equal(out["status"], g[f"{variant}_status"])
    ok = g[f"{variant}_status"] == 0
    assert ok.sum() > 1000
    np.testing.assert_array_equal(out["family"][ok], g[f"{variant}_family"][ok])
    np.testing.assert_array_equal(out["saddr"][ok], g[f"{variant}_saddr"][ok])
    np.testing.assert_array_equal(out["daddr"][ok], g[f"{variant}_daddr"][ok])
    np.testing.assert_array_equal(out["dport"][ok], g[f"{variant}_dport"][ok])
    np.testing.assert_array_equal(out["proto"][ok], g[f"{variant}_proto"][ok])
    np.testing.assert_array_equal(out["flags"][ok] >> 1, g[f"{variant}_frag"][ok])
    np.testing.assert_array_equal(out["flags"] & 1, g["flags"] & 1)


def test_frames_fixture_covers_every_outcome(golden):
    """Every drop the frame path can produce occurs in the fixture."""
    g = golden("frames.npz")
    seen = set(np.unique(g["ct_status"]).tolist()) | set(np.unique(g["nover_status"]).tolist())
    want = {0, L.FRAME_NOT_CLASSIFIED, L.DROP_INVALID_SMAC, L.DROP_INVALID_DMAC,
            L.DROP_INVALID_SIP, L.DROP_INVALID, L.DROP_CT_INVALID_HDR, L.DROP_CT_UNKNOWN_PROTO,
            L.DROP_UNKNOWN_L3, L.DROP_INVALID_EXTHDR, L.DROP_FRAG_NOSUPPORT, L.EFAULT_LOAD}
    assert want <= seen, want - seen
    ok = g["ct_status"] == 0
    fam = g["ct_family"][ok]
    assert (fam == 4).sum() > 500 and (fam == 6).sum() > 200
    # ICMP echo request -> dport 8 / 128 raw, TCP/UDP ports, fragments on ingress
    assert {8, 128} <= set(g["ct_dport"][ok].tolist())
    assert g["ct_frag"][ok].sum() > 50
    assert not g["noct_dport"][g["noct_status"] == 0].any()


def test_frames_snaplen(golden):
    """A narrower slot than the frame: results equal the full-width parse
    wherever the headers fit, DROP_SNAPLEN exactly where a read the
    reference makes lies past the slot (but inside len)."""
    g = golden("frames.npz")
    o = frame_oracle(1, 7)
    full = o.frames_parse(frames_of(g))
    n_snap = 0
    for stride in (64, 128):
        f = frames_of(g)
        f["data"] = np.ascontiguousarray(g["data"][:, :stride])
        out = o.frames_parse(f)
        snap = out["status"] == L.DROP_SNAPLEN
        assert (g["len"][snap] > stride).all()
        n_snap += int(snap.sum())
        same = ~snap
        np.testing.assert_array_equal(out["status"][same], full["status"][same])
        ok = same & (full["status"] == 0)
        for k in ("dport", "proto", "family", "flags"):
            np.testing.assert_array_equal(out[k][ok], full[k][ok])
    assert n_snap > 0


def test_classify_frames_composes_tuple_decision(golden):
    """or_classify_frames == parse + or_classify_v4 / v6 on the tuples that
    reach policy; frame-level outcomes map to verdict/stage/metrics."""
    g = golden("frames.npz")
    T = synth.make_tables(n_prefixes=3000, n_identities=200, n_endpoints=5, keys_per_ep=2000)
    o = frame_oracle(1, 7, **{})
    synth.load_oracle(o, T)
    f = frames_of(g)
    v, idt, st, _ = o.classify_frames(f)
    m = o.metrics()
    p = frame_oracle(1, 7)
    synth.load_oracle(p, T)
    t = p.frames_parse(f)
    for fam in (4, 6):
        sel = (t["status"] == 0) & (t["family"] == fam)
        tt = {"dport": t["dport"][sel], "proto": t["proto"][sel], "flags": t["flags"][sel],
              "len": f["len"][sel], "ep": f["ep"][sel]}
        if fam == 4:
            tt["saddr"] = t["saddr"][sel, :4].copy().view(np.uint32).ravel()
            tt["daddr"] = t["daddr"][sel, :4].copy().view(np.uint32).ravel()
            vv, ii, ss, _ = p.classify_v4(tt)
        else:
            tt["saddr"], tt["daddr"] = t["saddr"][sel], t["daddr"][sel]
            vv, ii, ss, _ = p.classify_v6(tt)
        np.testing.assert_array_equal(v[sel], vv)
        np.testing.assert_array_equal(idt[sel], ii)
        np.testing.assert_array_equal(st[sel], ss)
    pre = t["status"] != 0
    nc = t["status"] == L.FRAME_NOT_CLASSIFIED
    np.testing.assert_array_equal(v[pre & ~nc], t["status"][pre & ~nc])
    assert (v[nc] == 0).all() and (st[nc] == 7).all() and (idt[pre] == 0).all()
    gated = t["status"] == L.DROP_CT_UNKNOWN_PROTO
    assert (st[gated] == 4).all() and (st[pre & ~nc & ~gated] == 5).all()
    # metrics: tuple-decision part from p, frame drops added here
    exp = p.metrics()
    dirs = np.where(f["flags"] & 1, L.METRIC_EGRESS, L.METRIC_INGRESS)
    drop = pre & ~nc
    reason = (-t["status"][drop]) & 0xff
    np.add.at(exp, (reason, dirs[drop], 0), 1)
    np.add.at(exp, (reason, dirs[drop], 1), f["len"][drop].astype(np.uint64))
    np.testing.assert_array_equal(m, exp)


def test_frames_from_tuples_equal_tuples():
    """synth.frames_from_tuples (the bench's frame batch) reaches policy with
    exactly the tuple it was built from: restatement verdicts, identities,
    stages and metrics equal or_classify_v4 on the tuples."""
    T = synth.make_tables(n_prefixes=3000, n_identities=200, n_endpoints=4, keys_per_ep=2000)
    t = synth.make_tuples(T, 50_000)
    f = synth.frames_from_tuples(t, stride=64)
    a = Oracle(**T.oracle_config())
    synth.load_oracle(a, T)
    b = Oracle(**T.oracle_config())
    synth.load_oracle(b, T)
    va, ia, sa, pa = a.classify_v4(t)
    vb, ib, sb, pb = b.classify_frames(f)
    np.testing.assert_array_equal(va, vb)
    np.testing.assert_array_equal(ia, ib)
    np.testing.assert_array_equal(sa, sb)
    assert pa == pb
    np.testing.assert_array_equal(a.metrics(), b.metrics())
