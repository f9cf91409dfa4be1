"""C-ABI checks that need no GPU: the library loads, exports every symbol
include/cgpu.h declares, and the host mirror follows bpf(2) map semantics
(pkg/bpf/bpf.go conventions: 0 or -errno).  No compute call is made here;
batch entry points on a host-only context must fail loudly (-ENODEV)."""
import ctypes as C
import errno
import os
import re

import numpy as np
import pytest

from cilium_amd import build, layouts as L
from cilium_amd._abi import Frames, PROTOS, TuplesV4, TuplesV4Ct, lib
from cilium_amd.engine import (CIDR_V4_DYN, CIDR_V4_FIX, CIDR_V6_DYN, CIDR_V6_FIX, BPF_EXIST,
                               BPF_NOEXIST, CIDRMap, Engine, IPCacheMap, PolicyMap)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def built():
    build.build()


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "cgpu.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(cgpu_[a-z0-9_]+)\s*\(", src)))


def test_exports_every_declared_symbol():
    syms = declared_symbols()
    assert len(syms) >= 30
    L_ = C.CDLL(build.LIB)
    missing = [s for s in syms if not hasattr(L_, s)]
    assert not missing, missing
    # the ctypes table covers the whole header too
    # (cgpu__* are test hooks, exported but deliberately not in the header)
    protos = {p for p in PROTOS if not p.startswith("cgpu__")}
    assert set(syms) == protos, set(syms) ^ protos


def test_library_is_gfx950():
    data = open(build.LIB, "rb").read()
    assert b"gfx950" in data


def test_host_only_context_has_no_cpu_path():
    e = Engine(device=-1)
    L_ = lib()
    tv = TuplesV4()
    v = np.zeros(4, np.int32)
    rc = L_.cgpu_classify_v4(e.h, C.byref(tv), 4, v.ctypes.data, v.ctypes.data, None, None)
    assert rc == -errno.ENODEV
    assert b"no CPU classification path" in L_.cgpu_last_error()
    assert L_.cgpu_prefilter_v4(e.h, None, None, None, 1, None, None) == -errno.ENODEV
    assert L_.cgpu_commit(e.h, None) == -errno.ENODEV
    fr = Frames(0, 0, 0, 0, 64, 0)
    assert L_.cgpu_classify_frames(e.h, C.byref(fr), 1, None, None, None, None) == -errno.ENODEV
    assert L_.cgpu_frames_parse(e.h, C.byref(fr), 1, None, None) == -errno.ENODEV
    assert L_.cgpu_l3_compile(e.h, None, None, None, 3, None) == -errno.EINVAL
    tc = TuplesV4Ct()
    assert L_.cgpu_classify_v4_ct(e.h, C.byref(tc), 1, 0, None, None, None, None,
                                  None) == -errno.ENODEV


def test_lxc_info_semantics():
    """Per-endpoint lxc_config.h identity (cgpu_lxc_*): update replaces,
    lookup round-trips the 32-byte record, delete of a missing id is
    -ENOENT, unknown verify bits / ids beyond the u16 ep column are -EINVAL,
    and the record counts in the replica checksum."""
    from cilium_amd import synth
    e = Engine(device=-1)
    info = L.lxc_info(synth.LXC_MAC, synth.LXC_IPV4_RAW, synth.LXC_IP6, 7)
    assert e.lxc_lookup(3) is None
    assert e.lxc_update(3, info) == 0
    got = e.lxc_lookup(3)
    assert got.tobytes() == info.tobytes()
    info2 = info.copy()
    info2["verify"] = 1
    assert e.lxc_update(3, info2) == 0
    assert e.lxc_lookup(3)["verify"] == 1
    assert e.lxc_delete(3) == 0
    assert e.lxc_delete(3) == -errno.ENOENT
    bad = info.copy()
    bad["verify"] = 8
    rc = lib().cgpu_lxc_update(e.h, 1, bad.tobytes())
    assert rc == -errno.EINVAL
    assert lib().cgpu_lxc_update(e.h, 65536, info.tobytes()) == -errno.EINVAL
    assert bytes(e.cfg.node_mac) == L.NODE_MAC


def test_policy_map_semantics():
    e = Engine(device=-1, policy_max_per_ep=4, max_endpoints=8)
    k = L.policy_key(300, 80, 6, 0)
    assert e.policy_update(0, k, L.policy_entry(4000)) == 0
    assert e.policy_update(0, k, L.policy_entry(0), BPF_NOEXIST) == -errno.EEXIST
    assert e.policy_update(0, L.policy_key(1, 1, 6, 0), L.policy_entry(), BPF_EXIST) == -errno.ENOENT
    rc, ent = e.policy_lookup(0, k)
    assert rc == 0 and ent["proxy_port"] == L.htons(4000)
    # pad bits are part of the key (kernel htab memcmp)
    assert e.policy_lookup(0, L.policy_key(300, 80, 6, 0, pad_bits=1))[0] == -errno.ENOENT
    for i in range(3):
        assert e.policy_update(0, L.policy_key(400 + i, 0, 0, 1), L.policy_entry()) == 0
    assert e.policy_update(0, L.policy_key(999, 0, 0, 1), L.policy_entry()) == -errno.E2BIG
    assert len(e.policy_keys(0)) == 4
    assert e.policy_delete(0, L.policy_key(999, 0, 0, 1)) == -errno.ENOENT
    assert e.policy_update(9, k, L.policy_entry()) == -errno.EINVAL
    assert e.policy_flush(0) == 0 and e.policy_keys(0) == []
    # Go mirror
    pm = PolicyMap(e, 1)
    pm.Allow(256, 443, 6, 1, proxy_port=15001)
    assert pm.Exists(256, 443, 6, 1) and not pm.Exists(256, 443, 17, 1)
    d = pm.DumpToSlice()
    assert len(d) == 1 and d[0][1]["proxy_port"] == L.htons(15001)
    pm.Delete(256, 443, 6, 1)
    assert pm.DumpToSlice() == []


def test_ipcache_lpm_semantics():
    e = Engine(device=-1, ipcache_max=3)
    assert e.ipcache_update(L.ipcache_key("10.0.0.0/8"), L.remote_info(100)) == 0
    # same prefix with different host bits is the same LPM element
    assert e.ipcache_update(L.ipcache_key("10.9.9.9/8"), L.remote_info(101)) == 0
    assert len(e.ipcache_keys()) == 1
    assert e.ipcache_update(L.ipcache_key("10.1.0.0/16"), L.remote_info(0)) == 0  # tombstone
    assert e.ipcache_update(L.ipcache_key("192.168.0.0/16"), L.remote_info(7)) == 0
    assert e.ipcache_update(L.ipcache_key("172.16.0.0/12"), L.remote_info(7)) == -errno.ENOSPC
    rc, v = e.ipcache_lookup(L.ipcache_key("10.1.2.3/32"))
    assert rc == 0 and v["sec_label"] == 0  # tombstone shadows 10/8
    rc, v = e.ipcache_lookup(L.ipcache_key("10.2.2.3/32"))
    assert rc == 0 and v["sec_label"] == 101
    assert e.ipcache_lookup(L.ipcache_key("11.0.0.1/32"))[0] == -errno.ENOENT
    bad = L.ipcache_key("10.0.0.0/8")
    bad["prefixlen"] = 161
    assert e.ipcache_update(bad, L.remote_info(1)) == -errno.EINVAL
    assert e.ipcache_delete(L.ipcache_key("10.0.0.0/9")) == -errno.ENOENT
    m = IPCacheMap(e)
    m.OnIPIdentityCacheChange("delete", "10.1.0.0/16", 0)
    assert e.ipcache_lookup(L.ipcache_key("10.1.2.3/32"))[1]["sec_label"] == 101
    m.OnIPIdentityCacheChange("delete", "10.1.0.0/16", 0)  # ENOENT tolerated
    tomb = IPCacheMap(e, supports_delete=False)
    tomb.Delete("192.168.0.0/16")
    assert e.ipcache_lookup(L.ipcache_key("192.168.1.1/32"))[1]["sec_label"] == 0


def test_cidr_and_endpoint_maps():
    e = Engine(device=-1)
    dyn = CIDRMap(e, CIDR_V4_DYN)
    fix = CIDRMap(e, CIDR_V4_FIX)
    dyn.InsertCIDR("192.0.2.0/24")
    fix.InsertCIDR("198.51.100.7/32")
    with pytest.raises(ValueError):
        fix.InsertCIDR("198.51.100.0/24")  # checkPrefixlen: fix maps are /32 only
    assert dyn.CIDRExists("192.0.2.77/32")  # LPM lookup
    assert fix.CIDRExists("198.51.100.7/32") and not fix.CIDRExists("198.51.100.8/32")
    assert dyn.CIDRDump() == ["192.0.2.0/24"] and fix.CIDRDump() == ["198.51.100.7/32"]
    dyn6 = CIDRMap(e, CIDR_V6_DYN)
    dyn6.InsertCIDR("2001:db8::/32")
    assert dyn6.CIDRExists("2001:db8::1/128")
    CIDRMap(e, CIDR_V6_FIX).InsertCIDR("2001:db8::5/128")
    assert CIDRMap(e, CIDR_V6_FIX).CIDRDump() == ["2001:db8::5/128"]
    dyn.DeleteCIDR("192.0.2.0/24")
    assert dyn.CIDRDump() == []
    k = L.lpm_key("10.0.0.0/8")
    k["prefixlen"] = 33
    assert e.cidr_update(CIDR_V4_DYN, k) == -errno.EINVAL
    ek = L.endpoint_key("10.0.0.5")
    assert e.endpoint_update(ek) == 0 and e.endpoint_lookup(ek) == 0
    assert e.endpoint_update(ek, BPF_NOEXIST) == -errno.EEXIST
    assert e.endpoint_delete(ek) == 0 and e.endpoint_lookup(ek) == -errno.ENOENT


def test_lb4_map_semantics():
    """cilium_lb4_services through the C ABI: bpf(2) flags, capacity (E2BIG
    like the kernel htab), exact lookup, GetNextKey order, and the lbmap
    UpdateService / DeleteService write sequence (lbmap.go:350-428)."""
    from cilium_amd.engine import LBMap
    e = Engine(device=-1, lb_max_entries=8)
    k = L.lb4_key("10.96.0.10", 80, 0)
    assert e.lb4_update(k, L.lb4_service(0, 0, 2)) == 0
    assert e.lb4_update(k, L.lb4_service(), BPF_NOEXIST) == -errno.EEXIST
    assert e.lb4_update(L.lb4_key("10.96.0.11", 80, 0), L.lb4_service(), BPF_EXIST) == -errno.ENOENT
    rc, v = e.lb4_lookup(k)
    assert rc == 0 and int(v["count"]) == 2
    # the slave number is part of the key
    assert e.lb4_lookup(L.lb4_key("10.96.0.10", 80, 1))[0] == -errno.ENOENT
    m = LBMap(e)
    m.UpdateService("10.96.0.10", 80, [("10.1.0.1", 8080, 1), ("10.1.0.2", 8080, 0)], rev_nat=3)
    assert e.lb4_count() == 3
    bes = m.LookupService("10.96.0.10", 80)
    assert [L.be_to_host4(int(b["target"])) for b in bes] == [0x0A010001, 0x0A010002]
    assert int(e.lb4_lookup(k)[1]["weight"]) == L.htons(1)  # nNonZeroWeights, network order
    m.UpdateService("10.96.0.10", 80, [("10.1.0.3", 0, 0)])  # shrink: slave 2 removed
    assert e.lb4_count() == 2
    m.UpdateService("10.96.0.20", 0, [("10.1.0.4", 0, 0)] * 5)
    assert e.lb4_count() == 8
    assert e.lb4_update(L.lb4_key("10.96.0.30", 0, 0), L.lb4_service()) == -errno.E2BIG
    keys = e.lb4_keys()
    assert len(keys) == 8 and len({bytes(k) for k in keys}) == 8
    m.DeleteService("10.96.0.20", 0)
    assert e.lb4_count() == 2
    kk = np.array([L.lb4_key("10.96.1.1", 53, s) for s in range(3)], L.LB4_KEY)
    vv = np.array([L.lb4_service("10.2.0.1", 53, 2)] * 3, L.LB4_SERVICE)
    assert e.lb4_update_batch(kk, vv) == 0 and e.lb4_count() == 5
    assert e.lb4_update_batch(kk, vv, BPF_NOEXIST) == -errno.EEXIST
    assert e.lb4_delete(L.lb4_key("10.96.1.1", 53, 7)) == -errno.ENOENT
    # the default flow hash equals the sharder's
    from cilium_amd.shard import flowhash_np
    a = [np.array([x], dt) for x, dt in ((0x0100000A, np.uint32), (0x0200000A, np.uint32),
                                          (1234, np.uint16), (80, np.uint16), (6, np.uint8))]
    assert e.flow_hash(*(int(x[0]) for x in a)) == int(flowhash_np(*a)[0])
    # batch entry points have no CPU path
    from cilium_amd._abi import Lb4Out, Lb4Tuples
    assert lib().cgpu_lb4_select(e.h, 0, C.byref(Lb4Tuples()), 1, C.byref(Lb4Out()), None) == \
        -errno.ENODEV
    assert lib().cgpu_classify_v4_lb(e.h, C.byref(TuplesV4()), None, None, 1, None, None, None,
                                     None) == -errno.ENODEV


def test_bad_flags_and_abi_version():
    e = Engine(device=-1)
    assert e.policy_update(0, L.policy_key(1, 1, 6, 0), L.policy_entry(), 3) == -errno.EINVAL
    from cilium_amd._abi import CgpuConfig
    cfg = CgpuConfig()
    lib().cgpu_config_default(C.byref(cfg))
    cfg.abi_version = 99
    h = C.c_void_p()
    assert lib().cgpu_ctx_create(C.byref(cfg), -1, C.byref(h)) == -errno.EINVAL


def _ct_key(i, proto=6, flags=0):
    k = np.zeros((), L.CT4_TUPLE)
    k["daddr"], k["saddr"], k["dport"], k["sport"] = 0x0A000001 + i, 0x0B000001, 80, 1000 + i
    k["nexthdr"], k["flags"] = proto, flags
    return k


def test_ct_map_semantics():
    """cilium_ct4_global through the bpf(2)-style calls (pkg/maps/ctmap):
    BPF_ANY/NOEXIST/EXIST, -E2BIG past CT_MAP_SIZE, delete, get_next_key
    walking the whole map, GC by lifetime (ctmap.go doFiltering), Flush."""
    e = Engine(device=-1, ct_max=8)
    v = np.zeros((), L.CT_ENTRY)
    for i in range(8):
        v["lifetime"] = 100 + i
        v["rx_packets"] = i
        assert e.ct4_update(_ct_key(i), v) == 0
    assert e.ct4_count() == 8
    assert e.ct4_update(_ct_key(8), v) == -errno.E2BIG
    assert e.ct4_update(_ct_key(3), v, BPF_NOEXIST) == -errno.EEXIST
    assert e.ct4_update(_ct_key(9), v, BPF_EXIST) == -errno.ENOENT
    rc, got = e.ct4_lookup(_ct_key(2))
    assert rc == 0 and got["rx_packets"] == 2 and got["lifetime"] == 102
    # the key is the whole 14-byte tuple: flags and nexthdr distinguish entries
    assert e.ct4_lookup(_ct_key(2, flags=1))[0] == -errno.ENOENT
    assert e.ct4_lookup(_ct_key(2, proto=17))[0] == -errno.ENOENT
    assert e.ct4_delete(_ct_key(2)) == 0 and e.ct4_delete(_ct_key(2)) == -errno.ENOENT
    assert e.ct4_update(_ct_key(8), v) == 0  # room again
    keys, vals = e.ct4_dump()
    assert len(keys) == 8 and sorted(keys["daddr"].tolist()) == sorted(
        [0x0A000001 + i for i in (0, 1, 3, 4, 5, 6, 7, 8)])
    assert e.ct_stats(False)["live"] == 8
    assert e.ct4_gc(104) == 3  # lifetimes 100, 101, 103
    assert e.ct4_count() == 5
    # cgpu_ct_stats: the live count; the host GC rebuilt the table (no
    # tombstones left), and compaction counts only device compactions
    st = e.ct_stats(False)
    assert st["live"] == 5 and st["tombstones"] == 0 and st["compactions"] == 0
    assert e.ct_stats(True) == {"live": 0, "tombstones": 0, "compactions": 0}
    assert sorted(e.ct4_dump()[1]["lifetime"].tolist()) == [104, 105, 106, 107, 107]
    e.ct4_flush()
    assert e.ct4_count() == 0 and len(e.ct4_dump()[0]) == 0
    with pytest.raises(Exception):
        Engine(device=-1, ct_max=0)


def test_ct_map_matches_restatement_under_churn():
    """Random update/delete/GC churn: the engine's map (open addressing with
    tombstones and compaction) holds exactly what the restatement holds."""
    from oracle import Oracle
    rng = np.random.Generator(np.random.PCG64(7))
    e = Engine(device=-1, ct_max=64)
    o = Oracle()
    o.ct_set_max(64)
    for step in range(3000):
        i = int(rng.integers(0, 96))
        k = _ct_key(i, proto=int(rng.choice([1, 6, 17])), flags=int(rng.integers(0, 4)))
        op = rng.random()
        if op < 0.6:
            v = np.zeros((), L.CT_ENTRY)
            v["lifetime"] = int(rng.integers(0, 1000))
            v["tx_bytes"] = step
            assert e.ct4_update(k, v) == o.ct4_update(k, v)
        elif op < 0.98:
            assert e.ct4_delete(k) == o.ct4_delete(k)
        else:
            t = int(rng.integers(0, 1000))
            assert e.ct4_gc(t) == o.ct4_gc(t)
        assert e.ct4_count() == o.ct4_count()
    ek, ev = e.ct4_dump()
    ok, ov = o.ct4_dump()
    np.testing.assert_array_equal(ek, ok)
    np.testing.assert_array_equal(ev, ov)


def test_no_diagnostic_variants_ship():
    """Only schedules that compute the reference's results ship in the
    product library: no ablation switches are read from the environment."""
    data = open(build.LIB, "rb").read()
    for knob in (b"CGPU_PF6_Q", b"CGPU_CT_CHUNK", b"CGPU_POL_BPB", b"CGPU_POL_LOAD_PCT", b"CGPU_LB_VIP_BITS"):
        assert knob not in data, knob


def test_batch_ops_and_dump_host_only():
    """cgpu_*_update_batch apply in order and stop at the first failure;
    cgpu_policy_dump / cgpu_policy_lookup_batch mirror DumpToSlice /
    per-key lookups (host-only context: counters are the supplied ones)."""
    e = Engine(device=-1, max_endpoints=4, policy_max_per_ep=8)
    keys = np.array([L.policy_key(300 + i, 80, 6, i & 1) for i in range(10)])
    ents = np.array([L.policy_entry(i, 10 * i, 100 * i) for i in range(10)])
    eps = np.zeros(10, np.uint32)
    rc = e.policy_update_batch(eps, keys, ents)
    assert rc == -errno.E2BIG  # the 9th write hits policy_max_per_ep
    assert e.L.cgpu_policy_count(e.h, 0) == 8
    k, v = e.policy_dump(0)
    assert len(k) == 8
    order = np.argsort(k.view(np.uint64))
    assert (k.view(np.uint64)[order] == k.view(np.uint64)).all()  # GetNextKey order
    got = {int(x["sec_label"]): (int(y["packets"]), int(y["bytes"]), L.ntohs(int(y["proxy_port"])))
           for x, y in zip(k, v)}
    assert got == {300 + i: (10 * i, 100 * i, i) for i in range(8)}
    rc, out = e.policy_lookup_batch(np.array([0, 0, 9], np.uint32), keys[[1, 9, 0]])
    assert list(rc) == [0, -errno.ENOENT, -errno.EINVAL]
    assert int(out[0]["packets"]) == 10
    ik = np.array([L.ipcache_key(f"10.0.{i}.0/24") for i in range(5)])
    iv = np.array([L.remote_info(500 + i) for i in range(5)])
    assert e.ipcache_update_batch(ik, iv) == 0
    assert e.ipcache_update_batch(ik[:2], iv[:2], BPF_NOEXIST) == -errno.EEXIST
    assert len(e.ipcache_keys()) == 5
    ck = np.array([L.lpm_key(f"2001:db8:{i}::/48") for i in range(4)])
    assert e.cidr_update_batch(CIDR_V6_DYN, ck) == 0
    assert len(e.cidr_keys(CIDR_V6_DYN)) == 4
    e.close()


def test_prefilter_revision_routing_and_undo():
    """pkg/policy/prefilter.go: selectMap routes /32 and /128 to the exact
    maps and shorter prefixes to the LPM maps; a stale revision is refused;
    a failed Insert leaves nothing behind and a failed Delete re-inserts
    what it removed; Delete checks existence first (LPM lookup)."""
    from cilium_amd.engine import PreFilter
    e = Engine(device=-1, cidr_fix_max=3)
    pf = PreFilter(e)
    assert pf.Revision() == 1
    pf.Insert(1, ["10.0.0.0/8", "192.168.1.1/32", "2001:db8::/32", "2001:db8::1/128"])
    assert pf.Revision() == 2
    assert CIDRMap(e, CIDR_V4_DYN).CIDRDump() == ["10.0.0.0/8"]
    assert CIDRMap(e, CIDR_V4_FIX).CIDRDump() == ["192.168.1.1/32"]
    assert CIDRMap(e, CIDR_V6_DYN).CIDRDump() == ["2001:db8::/32"]
    assert CIDRMap(e, CIDR_V6_FIX).CIDRDump() == ["2001:db8::1/128"]
    with pytest.raises(OSError) as ex:
        pf.Insert(1, ["10.1.0.0/16"])  # revision 1 is stale
    assert ex.value.errno == errno.ESTALE and "Latest revision is 2 not 1" in str(ex.value)
    pf.Insert(0, ["10.1.0.0/16"])  # revision 0: no check
    assert pf.Revision() == 3
    # fix4 holds at most 3 keys: the 3rd /32 fails, the two before it are undone
    with pytest.raises(OSError) as ex:
        pf.Insert(3, ["172.16.0.1/32", "172.16.0.2/32", "172.16.0.3/32", "172.16.9.0/24"])
    assert ex.value.errno == errno.E2BIG
    assert CIDRMap(e, CIDR_V4_FIX).CIDRDump() == ["192.168.1.1/32"]
    assert CIDRMap(e, CIDR_V4_DYN).CIDRDump() == ["10.0.0.0/8", "10.1.0.0/16"]
    assert pf.Revision() == 3
    # Delete: existence first; a /24 under 10.0.0.0/8 "exists" (LPM lookup)
    # but its exact delete fails, so the /16 removed before it comes back
    with pytest.raises(OSError) as ex:
        pf.Delete(3, ["10.1.0.0/16", "10.2.3.0/24"])
    assert ex.value.errno == errno.ENOENT
    assert CIDRMap(e, CIDR_V4_DYN).CIDRDump() == ["10.0.0.0/8", "10.1.0.0/16"]
    with pytest.raises(OSError) as ex:
        pf.Delete(3, ["10.1.0.0/16", "11.0.0.0/8"])  # 11/8 missing: nothing deleted
    assert ex.value.errno == errno.ENOENT
    pf.Delete(3, ["10.1.0.0/16", "2001:db8::1/128"])
    assert pf.Revision() == 4
    dump, rev = pf.Dump()
    assert dump == ["10.0.0.0/8", "192.168.1.1/32", "2001:db8::/32"] and rev == 4
    e.close()
    # the reference's default config disables the LPM maps (prefilter.go:284-289)
    e2 = Engine(device=-1, prefilter_dyn4=0, prefilter_dyn6=0)
    with pytest.raises(OSError) as ex:
        PreFilter(e2).Insert(0, ["10.0.0.0/8"])
    assert ex.value.errno == errno.EOPNOTSUPP
    PreFilter(e2).Insert(0, ["10.0.0.1/32"])
    e2.close()


def _ct6_key(i, flags=0, proto=6):
    k = np.zeros((), L.CT6_TUPLE)
    k["daddr"][:] = np.frombuffer(bytes([0xf0, 0x0d] + [0] * 13 + [i]), np.uint8)
    k["saddr"][:] = np.frombuffer(bytes([0xbe, 0xef] + [0] * 13 + [1]), np.uint8)
    k["dport"], k["sport"], k["nexthdr"], k["flags"] = 0x5000, 0x3930, proto, flags
    return k


def test_ct6_map_semantics():
    """cilium_ct6_global through the bpf(2)-style calls: capacity ct6_max,
    BPF_ANY/NOEXIST/EXIST, the whole 38-byte tuple as the key, get_next_key,
    GC by lifetime, Flush; independent of cilium_ct4_global."""
    e = Engine(device=-1, ct_max=100, ct6_max=8)
    v = np.zeros((), L.CT_ENTRY)
    for i in range(8):
        v["lifetime"] = 100 + i
        v["tx_packets"] = i
        assert e.ct6_update(_ct6_key(i), v) == 0
    assert e.ct6_count() == 8 and e.ct4_count() == 0
    assert e.ct6_update(_ct6_key(8), v) == -errno.E2BIG
    assert e.ct6_update(_ct6_key(3), v, BPF_NOEXIST) == -errno.EEXIST
    assert e.ct6_update(_ct6_key(9), v, BPF_EXIST) == -errno.ENOENT
    rc, got = e.ct6_lookup(_ct6_key(2))
    assert rc == 0 and got["tx_packets"] == 2 and got["lifetime"] == 102
    assert e.ct6_lookup(_ct6_key(2, flags=1))[0] == -errno.ENOENT
    assert e.ct6_lookup(_ct6_key(2, proto=58))[0] == -errno.ENOENT
    assert e.ct6_delete(_ct6_key(2)) == 0 and e.ct6_delete(_ct6_key(2)) == -errno.ENOENT
    assert e.ct6_update(_ct6_key(8), v) == 0
    keys, vals = e.ct6_dump()
    assert len(keys) == 8 and sorted(keys["daddr"][:, 15].tolist()) == [0, 1, 3, 4, 5, 6, 7, 8]
    assert (keys["saddr"][:, 0] == 0xbe).all() and (keys["nexthdr"] == 6).all()
    assert e.ct6_gc(104) == 3
    assert e.ct6_count() == 5
    e.ct6_flush()
    assert e.ct6_count() == 0
    e.close()


def test_host_batch_entry_errors():
    """cgpu_classify_v4_host (host-resident batches): a null
    column or output is -EINVAL, a host-only context -ENODEV (no CPU path),
    an empty batch is a no-op."""
    e = Engine(device=-1)
    L_ = lib()
    n = 8
    cols = [np.zeros(n, dt) for dt in (np.uint32, np.uint32, np.uint16, np.uint8, np.uint8,
                                        np.uint32, np.uint16)]
    v = np.zeros(n, np.int32)
    i = np.zeros(n, np.uint32)
    tv = TuplesV4(*[c.ctypes.data for c in cols])
    assert L_.cgpu_classify_v4_host(e.h, C.byref(tv), n, v.ctypes.data, i.ctypes.data, None,
                                    None) == -errno.ENODEV
    assert L_.cgpu_classify_v4_host(e.h, C.byref(tv), n, None, i.ctypes.data, None,
                                    None) == -errno.EINVAL
    bad = TuplesV4(*([c.ctypes.data for c in cols[:3]] + [0] + [c.ctypes.data for c in cols[4:]]))
    assert L_.cgpu_classify_v4_host(e.h, C.byref(bad), n, v.ctypes.data, i.ctypes.data, None,
                                    None) == -errno.EINVAL
    assert L_.cgpu_classify_v4_host(e.h, None, n, v.ctypes.data, i.ctypes.data, None,
                                    None) == -errno.EINVAL
    assert L_.cgpu_classify_v4_host(None, C.byref(tv), n, v.ctypes.data, i.ctypes.data, None,
                                    None) == -errno.EINVAL
    # the service / cascade / v6 / prefilter host forms
    sp = np.zeros(n, np.uint16)
    a16 = np.zeros((n, 16), np.uint8)
    from cilium_amd._abi import TuplesV6
    tv6 = TuplesV6(*([a16.ctypes.data] * 2 + [c.ctypes.data for c in cols[2:]]))
    for fn in ("cgpu_classify_v4_lb_host", "cgpu_classify_v4_cascade_host"):
        f = getattr(L_, fn)
        assert f(e.h, C.byref(tv), sp.ctypes.data, None, n, v.ctypes.data, i.ctypes.data, None,
                 None) == -errno.ENODEV
        assert f(e.h, C.byref(tv), None, None, n, v.ctypes.data, i.ctypes.data, None,
                 None) == -errno.EINVAL
    assert L_.cgpu_classify_v6_lb_host(e.h, C.byref(tv6), None, None, n, v.ctypes.data,
                                       i.ctypes.data, None, None) == -errno.EINVAL
    assert L_.cgpu_classify_v6_lb_host(e.h, C.byref(tv6), sp.ctypes.data, None, n, v.ctypes.data,
                                       i.ctypes.data, None, None) == -errno.ENODEV
    assert L_.cgpu_classify_v6_host(e.h, C.byref(tv6), n, v.ctypes.data, i.ctypes.data, None,
                                    None) == -errno.ENODEV
    assert L_.cgpu_classify_v6_host(e.h, C.byref(tv6), n, None, i.ctypes.data, None,
                                    None) == -errno.EINVAL
    pv = np.zeros(n, np.uint8)
    assert L_.cgpu_prefilter_v4_host(e.h, cols[0].ctypes.data, cols[1].ctypes.data, cols[4].ctypes.data,
                                     n, pv.ctypes.data, None) == -errno.ENODEV
    assert L_.cgpu_prefilter_v6_host(e.h, a16.ctypes.data, a16.ctypes.data, None, n, pv.ctypes.data,
                                     None) == -errno.EINVAL
    assert L_.cgpu_prefilter_v6_host(e.h, a16.ctypes.data, a16.ctypes.data, None, 0, pv.ctypes.data,
                                     None) == -errno.ENODEV
    e.close()


def test_frames_host_and_staging_entry_errors():
    """cgpu_classify_frames_host: bad frame columns / stride / output are
    -EINVAL, a host-only context -ENODEV; cgpu_host_stage_release and
    cgpu_host_stage_bytes on a context that never staged anything; and
    cgpu_table_bytes reports zeros before the first commit."""
    from cilium_amd._abi import Frames
    e = Engine(device=-1)
    L_ = lib()
    n = 4
    data = np.zeros((n, 64), np.uint8)
    ln = np.full(n, 60, np.uint32)
    fl = np.zeros(n, np.uint8)
    ep = np.zeros(n, np.uint16)
    v = np.zeros(n, np.int32)
    i = np.zeros(n, np.uint32)
    fr = Frames(data.ctypes.data, ln.ctypes.data, fl.ctypes.data, ep.ctypes.data, 64, 0)
    assert L_.cgpu_classify_frames_host(e.h, C.byref(fr), n, v.ctypes.data, i.ctypes.data, None,
                                        None) == -errno.ENODEV
    assert L_.cgpu_classify_frames_host(e.h, C.byref(fr), n, None, i.ctypes.data, None,
                                        None) == -errno.EINVAL
    bad = Frames(data.ctypes.data, ln.ctypes.data, fl.ctypes.data, ep.ctypes.data, 40, 0)
    assert L_.cgpu_classify_frames_host(e.h, C.byref(bad), n, v.ctypes.data, i.ctypes.data, None,
                                        None) == -errno.EINVAL
    assert L_.cgpu_classify_frames_host(None, C.byref(fr), n, v.ctypes.data, i.ctypes.data, None,
                                        None) == -errno.EINVAL
    assert L_.cgpu_host_stage_release(e.h) == 0
    assert L_.cgpu_host_stage_bytes(e.h) == 0
    assert L_.cgpu_host_stage_release(None) == -errno.EINVAL
    assert set(e.table_bytes().values()) == {0}
    e.close()
