"""The composition of the endpoint program, compiled from the reference
instead of restated.

tests/golden/ct4.npz, ctlb4.npz, ct6.npz and ctlb6.npz were produced by
oracle/ref/harness_ct.c and harness_ctlb.c, which call the reference's lib/
functions in the order bpf_lxc.c does, that order written out by hand.
oracle/ref/harness_lxc.c compiles bpf/bpf_lxc.c itself and runs its entry
points tail_handle_ipv4 / tail_handle_ipv6 (egress: handle_ipv4_from_lxc,
bpf_lxc.c:408-669; handle_ipv6 -> ipv6_l3_from_lxc, :82-403) and
tail_ipv4_policy / tail_ipv6_policy (ingress: ipv4_policy, :862-964;
ipv6_policy, :718-860).  Replaying each fixture's batches through
it must reproduce the fixture: every packet's verdict, ct_lookup4 result,
identity, policy stage, the frame after the service step, the conntrack map
after every batch and the policy entries' counters.  Two known differences,
both from the reference's build, not its logic:
  * SECLABEL is node_config.h's compile-time 2 in the compiled program (the
    agent generates it per endpoint), so an egress create's src_sec_id reads
    2 where the fixture holds the endpoint's label;
  * a proxy-redirected frame has its daddr / dport rewritten to the proxy
    (lib/lxc.h:97-140), so the post-service frame is compared for the others.
The ingress source identity comes from the reference's host-device program
compiled whole as well (oracle/ref/harness_netdev.c: bpf_netdev.c under its
node_config.h / netdev_config.h, the cilium_host build; handle_ipv4 /
handle_ipv6 run to the tail call into the endpoint's policy program, whose
skb->cb[CB_SRC_LABEL] is the identity ipv4_policy / ipv6_policy receive).
Only the stateless fixture's ingress_secctx_world form (the cilium_net
build, where derive_ipv4_sec_ctx gives WORLD_ID, bpf_netdev.c:45-62) is a
constant here: netdev_config.h compiles the FROM_HOST form.

Development container only: skipped where the reference harness was not
built (it compiles /root/reference, which never reaches the GPU box)."""
import ctypes as C
import os

import numpy as np
import pytest

from cilium_amd import layouts as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "_ref", "libref_lxc.so")
NETDEV = os.path.join(ROOT, "oracle", "_ref", "libref_netdev.so")
XDP = os.path.join(ROOT, "oracle", "_ref", "libref_xdp.so")
pytestmark = pytest.mark.skipif(not os.path.exists(LIB), reason="reference harness not built (oracle/_ref)")

SECLABEL_BUILD = 2  # bpf/node_config.h


def _lib():
    lib = C.CDLL(LIB)
    vp, ip, u32p = C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_uint32)
    lib.ref_lxc_reset.argtypes = [C.c_size_t]
    lib.ref_lxc_reset.restype = None
    lib.ref_lxc_set_now.argtypes = [C.c_uint32]
    lib.ref_lxc_set_now.restype = None
    lib.ref_lxc_ct_clear.restype = None
    for f in ("ref_lxc_policy_update", "ref_lxc_policy_read"):
        getattr(lib, f).argtypes = [C.c_int, vp, vp]
    lib.ref_lxc_policy_delete.argtypes = [C.c_int, vp]
    for f in ("ref_lxc_ipcache_update", "ref_lxc_svc_update", "ref_lxc_ct_update"):
        getattr(lib, f).argtypes = [vp, vp]
    lib.ref_lxc_svc_delete.argtypes = [vp]
    lib.ref_lxc_ct_count.restype = C.c_size_t
    lib.ref_lxc_ct_entry.argtypes = [C.c_size_t, vp, vp]
    lib.ref_lxc_src_identity.argtypes = [C.c_uint32, C.c_uint32]
    lib.ref_lxc_src_identity.restype = C.c_uint32
    lib.ref_lxc_metrics.argtypes = [vp]
    lib.ref_lxc_metrics.restype = None
    lib.ref_lxc_v4.argtypes = [C.c_uint32, C.c_uint32, C.c_uint16, C.c_uint16, C.c_uint8, C.c_uint16,
                               C.c_uint8, C.c_uint32, C.c_int, C.c_uint32, C.c_uint32, ip, u32p, ip, ip,
                               u32p, C.POINTER(C.c_uint16)]
    lib.ref_lxc_v6.argtypes = [C.c_char_p, C.c_char_p, C.c_uint16, C.c_uint16, C.c_uint8, C.c_uint16,
                               C.c_uint8, C.c_uint32, C.c_int, C.c_uint32, C.c_uint32, ip, u32p, ip, ip,
                               C.c_char_p, C.POINTER(C.c_uint16)]
    lib.ref_lxc_src_identity6.argtypes = [C.c_char_p, C.c_uint32]
    lib.ref_lxc_src_identity6.restype = C.c_uint32
    for f in ("ref_lxc_svc6_update", "ref_lxc_ct6_update"):
        getattr(lib, f).argtypes = [vp, vp]
    lib.ref_lxc_svc6_delete.argtypes = [vp]
    lib.ref_lxc_ct6_count.restype = C.c_size_t
    lib.ref_lxc_ct6_entry.argtypes = [C.c_size_t, vp, vp]
    return lib


def _nd():
    nd = C.CDLL(NETDEV)
    u32p = C.POINTER(C.c_uint32)
    nd.ref_netdev_reset.restype = None
    nd.ref_netdev_ipcache_update.argtypes = [C.c_void_p, C.c_void_p]
    nd.ref_netdev_v4.argtypes = [C.c_uint32, C.c_uint32, C.c_uint8, C.c_uint32, u32p]
    nd.ref_netdev_v6.argtypes = [C.c_char_p, C.c_char_p, C.c_uint8, C.c_uint32, u32p]
    return nd


class _Netdev:
    """The source identity bpf_netdev.c hands the endpoint's policy program."""

    def __init__(self, ipc_keys, ipc_vals):
        self.nd = _nd()
        self.nd.ref_netdev_reset()
        for k, v in zip(ipc_keys, ipc_vals):
            assert self.nd.ref_netdev_ipcache_update(_b(k), _b(v)) >= 0
        self.lab = C.c_uint32()

    def src4(self, saddr, daddr, proto, src):
        assert self.nd.ref_netdev_v4(int(saddr), int(daddr), int(proto), int(src), C.byref(self.lab)) == 0
        return self.lab.value

    def src6(self, saddr, daddr, proto, src):
        assert self.nd.ref_netdev_v6(bytes(saddr), bytes(daddr), int(proto), int(src), C.byref(self.lab)) == 0
        return self.lab.value


def _b(x):
    return np.ascontiguousarray(x).tobytes()


def _dump(lib, v6):
    n = (lib.ref_lxc_ct6_count if v6 else lib.ref_lxc_ct_count)()
    kt = L.CT6_TUPLE if v6 else L.CT4_TUPLE
    keys = np.zeros(n, kt)
    vals = np.zeros(n, L.CT_ENTRY)
    kb, vb = C.create_string_buffer(kt.itemsize), C.create_string_buffer(56)
    for i in range(n):
        assert (lib.ref_lxc_ct6_entry if v6 else lib.ref_lxc_ct_entry)(i, kb, vb) == 0
        keys[i] = np.frombuffer(kb.raw, kt)[0]
        vals[i] = np.frombuffer(vb.raw, L.CT_ENTRY)[0]
    return L.ct_sorted(keys, vals)


def _run(lib, t, now, hashes=None, nd=None):
    n = len(t["saddr"])
    v6 = np.asarray(t["saddr"]).ndim == 2
    out = {k: np.zeros(n, dt) for k, dt in (("verdict", np.int32), ("ct_ret", np.uint8),
                                             ("identity", np.uint32), ("stage", np.uint8),
                                             ("xdport", np.uint16))}
    out["xdaddr"] = np.zeros((n, 16), np.uint8) if v6 else np.zeros(n, np.uint32)
    v, cr, st = C.c_int(), C.c_int(), C.c_int()
    idv, xd = C.c_uint32(), C.c_uint32()
    xd6 = C.create_string_buffer(16)
    xp = C.c_uint16()
    lib.ref_lxc_set_now(now)
    for i in range(n):
        eg = int(t["flags"][i]) & 1
        h = int(hashes[i]) if hashes is not None else 0
        cols = (int(t["sport"][i]), int(t["dport"][i]), int(t["proto"][i]), int(t["l4b"][i]),
                int(t["flags"][i]), int(t["len"][i]), int(t["ep"][i]), h)
        if v6:
            sa, da = t["saddr"][i].tobytes(), t["daddr"][i].tobytes()
            src = 0 if eg else nd.src6(sa, da, int(t["proto"][i]), 0)
            lib.ref_lxc_v6(sa, da, *cols, src, C.byref(v), C.byref(idv), C.byref(cr), C.byref(st), xd6,
                           C.byref(xp))
            out["xdaddr"][i] = np.frombuffer(xd6.raw, np.uint8)
        else:
            src = 0 if eg else nd.src4(t["saddr"][i], t["daddr"][i], t["proto"][i], 0)
            lib.ref_lxc_v4(int(t["saddr"][i]), int(t["daddr"][i]), *cols, src, C.byref(v), C.byref(idv),
                           C.byref(cr), C.byref(st), C.byref(xd), C.byref(xp))
            out["xdaddr"][i] = xd.value
        out["verdict"][i], out["ct_ret"][i], out["identity"][i] = v.value, cr.value, idv.value
        out["stage"][i], out["xdport"][i] = st.value, xp.value
    return out


def _cmp_dump(got, want, seclabels):
    (gk, gv), (wk, wv) = got, want
    np.testing.assert_array_equal(gk, wk)
    rest = [f for f in L.CT_ENTRY.names if f != "src_sec_id"]
    for f in rest:
        np.testing.assert_array_equal(gv[f], wv[f], err_msg=f)
    same = gv["src_sec_id"] == wv["src_sec_id"]
    built = (gv["src_sec_id"] == SECLABEL_BUILD) & np.isin(wv["src_sec_id"], seclabels)
    assert (same | built).all()


@pytest.mark.parametrize("fixture", ["ct4.npz", "ctlb4.npz", "ct6.npz", "ctlb6.npz"])
def test_compiled_endpoint_program_reproduces_fixture(golden, fixture):
    g = golden(fixture)
    lib = _lib()
    svc = "lb_keys" in g.files
    v6 = "6" in fixture
    svc_update = lib.ref_lxc_svc6_update if v6 else lib.ref_lxc_svc_update
    svc_delete = lib.ref_lxc_svc6_delete if v6 else lib.ref_lxc_svc_delete
    lib.ref_lxc_reset(1 << 20)
    for k, v in zip(g["ipc_keys"], g["ipc_vals"]):
        lib.ref_lxc_ipcache_update(_b(k), _b(v))
    nd = _Netdev(g["ipc_keys"], g["ipc_vals"])
    for k, e, ep in zip(g["pol_keys"], g["pol_entries"], g["pol_ep"]):
        assert lib.ref_lxc_policy_update(int(ep), _b(k), _b(e)) == 0
    if svc:
        for k, v in zip(g["lb_keys"], g["lb_vals"]):
            svc_update(_b(k), _b(v))
    for k, v in zip(g["pre_keys"], g["pre_vals"]):
        assert (lib.ref_lxc_ct6_update if v6 else lib.ref_lxc_ct_update)(_b(k), _b(v)) == 0
    t = {k[2:]: g[k] for k in g.files if k.startswith("t_")}
    cuts, nows = g["cuts"], g["nows"]
    off = 0
    for bi in range(4):
        if bi == 2:
            for d in g["pol_del"]:
                assert lib.ref_lxc_policy_delete(int(g["pol_ep"][d]), _b(g["pol_keys"][d])) == 0
            if svc:
                for d in g["svc_del"]:
                    assert svc_delete(_b(g["lb_keys"][d])) == 0
        if bi == 3 and svc:
            for d, v in zip(g["svc_readd"], g["readd_vals"]):
                svc_update(_b(g["lb_keys"][d]), _b(v))
        sl = slice(int(cuts[bi]), int(cuts[bi + 1]))
        tb = {k: x[sl] for k, x in t.items()}
        o = _run(lib, tb, int(nows[bi]), tb.get("hash"), nd)
        msg = f"{fixture} batch {bi}"
        np.testing.assert_array_equal(o["verdict"], g["b_verdict"][sl], err_msg=msg)
        np.testing.assert_array_equal(o["ct_ret"], g["b_ct_ret"][sl], err_msg=msg)
        np.testing.assert_array_equal(o["identity"], g["b_identity"][sl], err_msg=msg)
        probed = g["b_stage"][sl] <= 3
        np.testing.assert_array_equal(o["stage"][probed], g["b_stage"][sl][probed], err_msg=msg)
        if svc:
            eg = (tb["flags"] & 1).astype(bool) & (o["verdict"] <= 0)
            np.testing.assert_array_equal(o["xdaddr"][eg], g["b_xdaddr"][sl][eg], err_msg=msg)
            np.testing.assert_array_equal(o["xdport"][eg], g["b_xdport"][sl][eg], err_msg=msg)
        n = int(g["dump_n"][bi])
        _cmp_dump(_dump(lib, v6), (g["dump_keys"][off:off + n], g["dump_vals"][off:off + n]),
                  g["seclabels"])
        off += n
    deleted = set(g["pol_del"].tolist())
    buf = C.create_string_buffer(24)
    for i, (k, ep, fe) in enumerate(zip(g["pol_keys"], g["pol_ep"], g["final_entries"])):
        if i in deleted:
            continue
        assert lib.ref_lxc_policy_read(int(ep), _b(k), buf) == 0
        got = np.frombuffer(buf.raw, L.POLICY_ENTRY)[0]
        assert (int(got["packets"]), int(got["bytes"])) == (int(fe["packets"]), int(fe["bytes"]))


@pytest.mark.parametrize("cfg", [0, 2, 3, 4])
def test_compiled_endpoint_program_reproduces_stateless_fixture(golden, cfg):
    """tests/golden/classify_v4.npz (harness_policy.c: the stateless
    decision, every packet CT_NEW) under its CONNTRACK configurations: the
    compiled program with an empty conntrack map before every packet gives
    the fixture's verdict, identity and stage for every TCP / UDP tuple
    (ICMP tuples carry a policy port the frame's type does not; the other
    protocols are the gate's, compared too)."""
    g = golden("classify_v4.npz")
    gate, src_cfg, secctx_world = (int(x) for x in g["configs"][cfg])
    assert gate == 1
    lib = _lib()
    lib.ref_lxc_reset(1 << 20)
    for k, v in zip(g["ipc_keys"], g["ipc_vals"]):
        lib.ref_lxc_ipcache_update(_b(k), _b(v))
    nd = _Netdev(g["ipc_keys"], g["ipc_vals"])
    for k, e, ep in zip(g["pol_keys"], g["pol_entries"], g["pol_ep"]):
        assert lib.ref_lxc_policy_update(int(ep), _b(k), _b(e)) == 0
    t = {k[2:]: g[k] for k in g.files if k.startswith("t_")}
    n = len(t["saddr"])
    v, cr, st = C.c_int(), C.c_int(), C.c_int()
    idv, xd = C.c_uint32(), C.c_uint32()
    xp = C.c_uint16()
    got = np.zeros((n, 3), np.int64)
    for i in range(n):
        lib.ref_lxc_ct_clear()
        eg = int(t["flags"][i]) & 1
        src = 0
        if not eg:
            # WORLD_ID: the cilium_net form (derive_ipv4_sec_ctx)
            src = 2 if secctx_world else nd.src4(t["saddr"][i], t["daddr"][i], t["proto"][i], src_cfg)
        lib.ref_lxc_v4(int(t["saddr"][i]), int(t["daddr"][i]), 0, int(t["dport"][i]), int(t["proto"][i]),
                       0, int(t["flags"][i]), int(t["len"][i]), int(t["ep"][i]), 0, src, C.byref(v),
                       C.byref(idv), C.byref(cr), C.byref(st), C.byref(xd), C.byref(xp))
        got[i] = v.value, idv.value, st.value
    keep = t["proto"] != 1
    gated = ~np.isin(t["proto"], [1, 6, 17])
    assert keep.sum() > 4000 and gated.sum() > 0
    np.testing.assert_array_equal(got[keep, 0], g[f"c{cfg}_verdict"][keep])
    np.testing.assert_array_equal(got[keep & ~gated, 1], g[f"c{cfg}_identity"][keep & ~gated])
    np.testing.assert_array_equal(got[keep & ~gated, 2], g[f"c{cfg}_stage"][keep & ~gated])


# IPv6 extension-header numbers (ipv6_hdrlen walks them, lib/ipv6.h:61-98):
# a tuple's nexthdr is the final protocol after them, so a tuple naming one
# has no frame of that form (the v6 fixtures' gated tuples include 0)
V6_EXT = (0, 43, 44, 50, 51, 59, 60)


def _stateless_replay(g, gate_src, v6, lib, nd, src_cfg):
    """Every tuple of a stateless fixture through the compiled endpoint
    program with an empty conntrack map (the fixture's every-packet-CT_NEW
    scope); ingress tuples carry the identity the compiled bpf_netdev.c hands
    over.  Returns (verdict, identity, stage) per tuple."""
    t = {k[2:]: g[k] for k in g.files if k.startswith("t_")}
    n = len(t["proto"])
    v, cr, st = C.c_int(), C.c_int(), C.c_int()
    idv, xd = C.c_uint32(), C.c_uint32()
    xd6 = C.create_string_buffer(16)
    xp = C.c_uint16()
    got = np.zeros((n, 3), np.int64)
    sport = t.get("sport", np.zeros(n, np.uint16))
    hashes = t.get("hash", np.zeros(n, np.uint32))
    for i in range(n):
        if v6 and int(t["proto"][i]) in V6_EXT:
            continue
        lib.ref_lxc_ct_clear()
        eg = int(t["flags"][i]) & 1
        cols = (int(sport[i]), int(t["dport"][i]), int(t["proto"][i]), 0, int(t["flags"][i]),
                int(t["len"][i]), int(t["ep"][i]), int(hashes[i]))
        if v6:
            sa, da = t["saddr"][i].tobytes(), t["daddr"][i].tobytes()
            src = 0 if eg else nd.src6(sa, da, t["proto"][i], src_cfg)
            lib.ref_lxc_v6(sa, da, *cols, src, C.byref(v), C.byref(idv), C.byref(cr), C.byref(st), xd6,
                           C.byref(xp))
        else:
            src = 0 if eg else nd.src4(t["saddr"][i], t["daddr"][i], t["proto"][i], src_cfg)
            lib.ref_lxc_v4(int(t["saddr"][i]), int(t["daddr"][i]), *cols, src, C.byref(v), C.byref(idv),
                           C.byref(cr), C.byref(st), C.byref(xd), C.byref(xp))
        got[i] = v.value, idv.value, st.value
    return t, got


@pytest.mark.parametrize("fixture,cfg", [("classify_v4_lb.npz", 0), ("classify_v6.npz", 0),
                                         ("classify_v6.npz", 2), ("classify_v6.npz", 3),
                                         ("classify_v6_lb.npz", 0)])
def test_compiled_endpoint_program_reproduces_restated_orders(golden, fixture, cfg):
    """The fixtures whose endpoint-program order the harnesses restate step by
    step -- config 5's egress service step before ipcache and policy
    (classify_v4_lb.npz: lb4_local, then ipcache on tuple.daddr and policy on
    the rewritten dport, bpf_lxc.c:444-505), the IPv6 decision (classify_v6.npz:
    ipv6_l3_from_lxc / ipv6_policy with the ROUTER_IP /64 fallback,
    bpf_lxc.c:158-203, :731-800) and the IPv6 service step
    (classify_v6_lb.npz, bpf_lxc.c:108-139) -- replayed through the compiled
    bpf_lxc.c: verdict of every TCP / UDP / gated tuple, and identity and
    stage of every tuple that reached a policy probe (ICMP tuples carry a
    policy port the frame's type does not; the CONNTRACK builds only)."""
    g = golden(fixture)
    v6 = "v6" in fixture
    row = [int(x) for x in g["configs"][cfg]]
    gate, src_cfg = row[0], row[1]
    assert gate == 1
    lib = _lib()
    lib.ref_lxc_reset(1 << 20)
    for k, v in zip(g["ipc_keys"], g["ipc_vals"]):
        lib.ref_lxc_ipcache_update(_b(k), _b(v))
    for k, e, ep in zip(g["pol_keys"], g["pol_entries"], g["pol_ep"]):
        assert lib.ref_lxc_policy_update(int(ep), _b(k), _b(e)) == 0
    if "lb_keys" in g.files:
        upd = lib.ref_lxc_svc6_update if v6 else lib.ref_lxc_svc_update
        for k, v in zip(g["lb_keys"], g["lb_vals"]):
            upd(_b(k), _b(v))
    nd = _Netdev(g["ipc_keys"], g["ipc_vals"])
    t, got = _stateless_replay(g, row, v6, lib, nd, src_cfg)
    icmp = np.isin(t["proto"], [1, 58])
    gated = ~np.isin(t["proto"], [1, 6, 17, 58])
    keep = ~icmp & ~(np.isin(t["proto"], V6_EXT) & v6)
    assert keep.sum() > 3000 and gated.sum() > 0
    np.testing.assert_array_equal(got[keep, 0], g[f"c{cfg}_verdict"][keep])
    probed = keep & (g[f"c{cfg}_stage"] <= 3) & ~gated
    assert probed.sum() > 2000
    np.testing.assert_array_equal(got[probed, 1], g[f"c{cfg}_identity"][probed])
    np.testing.assert_array_equal(got[probed, 2], g[f"c{cfg}_stage"][probed])
    if "lb_keys" in g.files:
        # the service step's drops are the compiled program's too
        drop = keep & (g[f"c{cfg}_verdict"] == -158)
        assert drop.sum() > 0 and (got[drop, 0] == -158).all()


def test_compiled_endpoint_program_reproduces_frame_parse(golden):
    """tests/golden/frames.npz (harness_frame.c: the header steps before
    policy, bpf_lxc.c's dispatch and handlers restated in order) against the
    compiled program on the raw frames, in the build the compiled harness
    has (CONNTRACK, the SMAC / DMAC / SIP checks disabled: the fixture's
    "nover" variant): every frame's status -- reached policy, not
    classified, or the drop before policy -- and, for frames that reached
    policy, the protocol and the port the policy step sees and the
    addresses (the first conntrack key's, in either order)."""
    g = golden("frames.npz")
    lib = _lib()
    lib.ref_lxc_frame.argtypes = [C.c_char_p, C.c_uint32, C.c_uint32, C.c_uint8, C.c_int,
                                  C.POINTER(C.c_int), C.POINTER(C.c_int), C.c_char_p, C.c_char_p,
                                  C.POINTER(C.c_uint16), C.POINTER(C.c_uint8)]
    lib.ref_lxc_reset(1 << 20)
    data, ln, fl, ep = g["data"], g["len"], g["flags"], g["ep"]
    n, width = data.shape
    st, fam = C.c_int(), C.c_int()
    kd, ks = C.create_string_buffer(16), C.create_string_buffer(16)
    dp, pr = C.c_uint16(), C.c_uint8()
    status = np.zeros(n, np.int64)
    family = np.zeros(n, np.int64)
    port = np.zeros(n, np.uint16)
    proto = np.zeros(n, np.uint8)
    addrs = [None] * n
    for i in range(n):
        stored = min(int(ln[i]), width)
        assert lib.ref_lxc_frame(data[i].tobytes(), stored, int(ln[i]), int(fl[i]), int(ep[i]),
                                 C.byref(st), C.byref(fam), kd, ks, C.byref(dp), C.byref(pr)) == 0
        status[i], family[i], port[i], proto[i] = st.value, fam.value, dp.value, pr.value
        addrs[i] = {kd.raw, ks.raw}
    want = g["nover_status"].astype(np.int64)
    np.testing.assert_array_equal(status, want)
    ok = want == 0
    assert ok.sum() > 1000 and len(np.unique(want)) >= 6
    np.testing.assert_array_equal(family[ok], g["nover_family"][ok])
    nofrag = ok & (g["nover_frag"] == 0)
    np.testing.assert_array_equal(proto[nofrag], g["nover_proto"][nofrag])
    np.testing.assert_array_equal(port[nofrag], g["nover_dport"][nofrag])
    for i in np.flatnonzero(ok):
        assert addrs[i] == {g["nover_saddr"][i].tobytes(), g["nover_daddr"][i].tobytes()}, i


def _xdp_frame(saddr, daddr):
    """Ethernet + a 20-byte IPv4 header carrying the tuple's addresses
    (network-order u32 as stored): what check_v4 reads."""
    h = bytearray(20)
    h[0], h[9] = 0x45, 6
    h[12:16] = int(saddr).to_bytes(4, "little")
    h[16:20] = int(daddr).to_bytes(4, "little")
    return bytes(6) + bytes([2, 0, 0, 0, 0, 1]) + (0x0800).to_bytes(2, "big") + bytes(h)


@pytest.mark.parametrize("cfg", [0, 1])
def test_compiled_programs_reproduce_cascade(golden, cfg):
    """tests/golden/cascade_v4.npz (BASELINE config 5 whole) replayed through
    the reference's programs compiled whole, in the order a packet meets
    them: an ingress packet through bpf_xdp.c (libref_xdp, xdp_start on its
    frame) and, if XDP_PASS, bpf_netdev.c's identity into bpf_lxc.c's
    ipv4_policy; an egress packet through bpf_lxc.c's handle_ipv4_from_lxc
    (service step, ipcache, policy).  Verdict of every TCP / UDP / gated
    packet and every XDP drop, identity and stage of every packet that
    reached a policy probe."""
    g = golden("cascade_v4.npz")
    row = [int(x) for x in g["configs"][cfg]]
    gate, src_cfg = row[0], row[1]
    if not gate:
        pytest.skip("the compiled endpoint program is the CONNTRACK build")
    lib = _lib()
    lib.ref_lxc_reset(1 << 20)
    for k, v in zip(g["ipc_keys"], g["ipc_vals"]):
        lib.ref_lxc_ipcache_update(_b(k), _b(v))
    for k, e, ep in zip(g["pol_keys"], g["pol_entries"], g["pol_ep"]):
        assert lib.ref_lxc_policy_update(int(ep), _b(k), _b(e)) == 0
    for k, v in zip(g["lb_keys"], g["lb_vals"]):
        lib.ref_lxc_svc_update(_b(k), _b(v))
    x = C.CDLL(XDP)
    x.ref_xdp_reset.restype = None
    x.ref_xdp_cidr_update.argtypes = [C.c_int, C.c_void_p]
    x.ref_xdp_endpoint_update.argtypes = [C.c_void_p]
    x.ref_xdp_run.argtypes = [C.c_char_p, C.c_uint32, C.POINTER(C.c_uint64)]
    x.ref_xdp_reset()
    for w, name in ((0, "dyn4"), (1, "fix4")):
        for k in g[name]:
            assert x.ref_xdp_cidr_update(w, _b(k)) >= 0
    for k in g["endpoints"]:
        assert x.ref_xdp_endpoint_update(_b(k)) >= 0
    nd = _Netdev(g["ipc_keys"], g["ipc_vals"])
    t, got = _stateless_replay(g, row, False, lib, nd, src_cfg)
    ing = (t["flags"] & 1) == 0
    pc = C.c_uint64()
    xv = np.zeros(len(ing), np.int64)
    for i in np.flatnonzero(ing):
        fr = _xdp_frame(t["saddr"][i], t["daddr"][i])
        xv[i] = x.ref_xdp_run(fr, len(fr), C.byref(pc))
    drop = ing & (xv == L.XDP_DROP)
    got[drop] = L.VERDICT_XDP_DROP, 0, L.STAGE_XDP_DROP
    want = g[f"c{cfg}_verdict"]
    np.testing.assert_array_equal(drop, want == L.VERDICT_XDP_DROP)
    icmp = t["proto"] == 1
    gated = ~np.isin(t["proto"], [1, 6, 17])
    keep = ~icmp | drop
    assert drop.sum() > 500 and (ing & ~drop & keep).sum() > 500
    np.testing.assert_array_equal(got[keep, 0], want[keep])
    probed = keep & (g[f"c{cfg}_stage"] <= 3) & ~gated
    np.testing.assert_array_equal(got[probed, 1], g[f"c{cfg}_identity"][probed])
    np.testing.assert_array_equal(got[probed, 2], g[f"c{cfg}_stage"][probed])
