"""TEST INFRASTRUCTURE — ctypes wrapper of the CPU restatement (liboracle.so).

Only tests/, bench.py's ``cpu_baseline`` leg and ``__graft_entry__.smoke()``
may import this module, and only as the checker / the timed CPU baseline.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")


class OrConfig(C.Structure):
    _fields_ = [
        ("host_id", C.c_uint32), ("world_id", C.c_uint32), ("cluster_id", C.c_uint32),
        ("health_id", C.c_uint32), ("ipv4_cluster_mask", C.c_uint32),
        ("ipv4_cluster_range", C.c_uint32), ("ct_proto_gate", C.c_int),
        ("ingress_src_identity", C.c_uint32), ("ingress_secctx_world", C.c_int),
        ("dyn4", C.c_int), ("fix4", C.c_int), ("dyn6", C.c_int), ("fix6", C.c_int),
        ("router_ip", C.c_uint8 * 16),
        ("lb_l3", C.c_int), ("lb_l4", C.c_int), ("ipv4_loopback", C.c_uint32),
        ("node_mac", C.c_uint8 * 6),
    ]


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        vp, sz = C.c_void_p, C.c_size_t
        L.or_create.restype = vp
        L.or_destroy.argtypes = [vp]
        L.or_set_config.argtypes = [vp, C.POINTER(OrConfig)]
        L.or_default_config.argtypes = [C.POINTER(OrConfig)]
        for f in ("or_ipcache_update", "or_ipcache_lookup"):
            getattr(L, f).argtypes = [vp, vp, vp]
        L.or_ipcache_delete.argtypes = [vp, vp]
        L.or_ipcache_count.argtypes = [vp]
        L.or_ipcache_count.restype = sz
        L.or_policy_update.argtypes = [vp, C.c_uint32, vp, vp]
        L.or_policy_lookup.argtypes = [vp, C.c_uint32, vp, vp]
        L.or_policy_delete.argtypes = [vp, C.c_uint32, vp]
        L.or_cidr_update.argtypes = [vp, C.c_int, vp]
        L.or_cidr_delete.argtypes = [vp, C.c_int, vp]
        L.or_endpoint_update.argtypes = [vp, vp]
        L.or_endpoint_delete.argtypes = [vp, vp]
        L.or_classify_v4.argtypes = [vp, sz] + [vp] * 10 + [C.c_int, C.POINTER(C.c_uint64)]
        L.or_classify_v6.argtypes = [vp, sz] + [vp] * 10 + [C.c_int, C.POINTER(C.c_uint64)]
        L.or_prefilter_v4.argtypes = [vp, sz, vp, vp, vp, vp, C.c_int, C.POINTER(C.c_uint64)]
        L.or_prefilter_v6.argtypes = [vp, sz, vp, vp, vp, vp, C.c_int, C.POINTER(C.c_uint64)]
        L.or_lb_update.argtypes = [vp, vp, vp]
        L.or_lb_delete.argtypes = [vp, vp]
        L.or_lb_update_many.argtypes = [vp, vp, vp, sz]
        L.or_flow_hash.argtypes = [C.c_uint32, C.c_uint32, C.c_uint16, C.c_uint16, C.c_uint8]
        L.or_flow_hash.restype = C.c_uint32
        L.or_lb4.argtypes = [vp, C.c_int, sz] + [vp] * 13 + [C.c_int, C.POINTER(C.c_uint64)]
        L.or_classify_v4_lb.argtypes = [vp, sz] + [vp] * 12 + [C.c_int, C.POINTER(C.c_uint64)]
        L.or_classify_v6_lb.argtypes = [vp, sz] + [vp] * 12 + [C.c_int, C.POINTER(C.c_uint64)]
        L.or_classify_v4_cascade.argtypes = [vp, sz] + [vp] * 12 + [C.c_int, C.POINTER(C.c_uint64)]
        L.or_lb6_update.argtypes = [vp, vp, vp]
        L.or_lb6_delete.argtypes = [vp, vp]
        L.or_flow_hash6.argtypes = [vp, vp, C.c_uint16, C.c_uint16, C.c_uint8]
        L.or_flow_hash6.restype = C.c_uint32
        L.or_lxc_update.argtypes = [vp, C.c_uint32, vp]
        L.or_frames_parse.argtypes = [vp, sz, vp, C.c_uint32] + [vp] * 10
        L.or_classify_frames.argtypes = [vp, sz, vp, C.c_uint32] + [vp] * 6 + [
            C.c_int, C.POINTER(C.c_uint64)]
        L.or_ct_set_max.argtypes = [vp, sz]
        L.or_ct_set_max.restype = None
        L.or_ct4_update.argtypes = [vp, vp, vp]
        L.or_ct4_delete.argtypes = [vp, vp]
        L.or_ct4_lookup.argtypes = [vp, vp, vp]
        L.or_ct4_count.argtypes = [vp]
        L.or_ct4_count.restype = sz
        L.or_ct4_dump.argtypes = [vp, vp, vp, sz]
        L.or_ct4_dump.restype = sz
        L.or_ct4_gc.argtypes = [vp, C.c_uint32]
        L.or_ct4_gc.restype = sz
        L.or_classify_v4_ct.argtypes = [vp, sz] + [vp] * 9 + [C.c_uint32] + [vp] * 4 + [
            C.POINTER(C.c_uint64)]
        L.or_ct6_set_max.argtypes = [vp, sz]
        L.or_ct6_set_max.restype = None
        L.or_ct6_update.argtypes = [vp, vp, vp]
        L.or_ct6_delete.argtypes = [vp, vp]
        L.or_ct6_lookup.argtypes = [vp, vp, vp]
        L.or_ct6_count.argtypes = [vp]
        L.or_ct6_count.restype = sz
        L.or_ct6_dump.argtypes = [vp, vp, vp, sz]
        L.or_ct6_dump.restype = sz
        L.or_ct6_gc.argtypes = [vp, C.c_uint32]
        L.or_ct6_gc.restype = sz
        L.or_classify_v4_ctlb.argtypes = [vp, sz] + [vp] * 10 + [C.c_uint32] + [vp] * 6 + [
            C.POINTER(C.c_uint64)]
        L.or_classify_v6_ctlb.argtypes = [vp, sz] + [vp] * 10 + [C.c_uint32] + [vp] * 6 + [
            C.POINTER(C.c_uint64)]
        L.or_classify_v6_ct.argtypes = [vp, sz] + [vp] * 9 + [C.c_uint32] + [vp] * 4 + [
            C.POINTER(C.c_uint64)]
        u32 = C.c_uint32
        L.or_l3_compile.argtypes = [vp, vp, vp, vp, vp, u32, vp, vp, vp, u32, vp, vp, u32, u32, vp]
        L.or_view_create.argtypes = [vp]
        L.or_view_create.restype = vp
        L.or_view_merge.argtypes = [vp, vp]
        L.or_view_merge.restype = None
        L.or_view_destroy.argtypes = [vp]
        L.or_view_destroy.restype = None
        L.or_metrics_read.argtypes = [vp, vp]
        L.or_probe_split.argtypes = [vp, vp]
        L.or_probe_split.restype = None
        L.or_set_fast.argtypes = [vp, C.c_int]
        L.or_ipcache_lookup4.argtypes = [vp, C.c_uint32, vp]
        L.or_ipcache_lookup6.argtypes = [vp, C.c_char_p, vp]
        L.or_counters_reset.argtypes = [vp]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _b(x):
    """numpy scalar/record -> bytes buffer kept alive by caller."""
    return np.ascontiguousarray(x).tobytes()


class Oracle:
    def __init__(self, **cfg):
        self.L = lib()
        self.h = self.L.or_create()
        self.cfg = OrConfig()
        self.L.or_default_config(C.byref(self.cfg))
        self.configure(**cfg)

    def configure(self, **kw):
        for k, v in kw.items():
            if k in ("router_ip", "node_mac"):
                getattr(self.cfg, k)[:] = bytes(v)
                continue
            setattr(self.cfg, k, v)
        self.L.or_set_config(self.h, C.byref(self.cfg))

    def close(self):
        if self.h:
            self.L.or_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --- tables ---
    def ipcache_update(self, key, val):
        return self.L.or_ipcache_update(self.h, _b(key), _b(val))

    def ipcache_delete(self, key):
        return self.L.or_ipcache_delete(self.h, _b(key))

    def ipcache_lookup(self, key):
        out = C.create_string_buffer(8)
        r = self.L.or_ipcache_lookup(self.h, _b(key), out)
        return r, out.raw

    def policy_update(self, ep, key, entry):
        return self.L.or_policy_update(self.h, ep, _b(key), _b(entry))

    def policy_delete(self, ep, key):
        return self.L.or_policy_delete(self.h, ep, _b(key))

    def policy_lookup(self, ep, key):
        out = C.create_string_buffer(24)
        r = self.L.or_policy_lookup(self.h, ep, _b(key), out)
        return r, out.raw

    def cidr_update(self, which, key):
        return self.L.or_cidr_update(self.h, which, _b(key))

    def cidr_delete(self, which, key):
        return self.L.or_cidr_delete(self.h, which, _b(key))

    def endpoint_update(self, key):
        return self.L.or_endpoint_update(self.h, _b(key))

    def endpoint_delete(self, key):
        return self.L.or_endpoint_delete(self.h, _b(key))

    # --- batch ---
    def classify_v4(self, t, nthreads=1):
        n = len(t["saddr"])
        verdict = np.empty(n, np.int32)
        identity = np.empty(n, np.uint32)
        stage = np.empty(n, np.uint8)
        probes = C.c_uint64(0)
        arrs = [np.ascontiguousarray(t[k], dt) for k, dt in (
            ("saddr", np.uint32), ("daddr", np.uint32), ("dport", np.uint16),
            ("proto", np.uint8), ("flags", np.uint8), ("len", np.uint32), ("ep", np.uint16))]
        self.L.or_classify_v4(self.h, n, *[_p(a) for a in arrs], _p(verdict), _p(identity),
                              _p(stage), nthreads, C.byref(probes))
        return verdict, identity, stage, probes.value

    def classify_v6(self, t, nthreads=1):
        n = len(t["flags"])
        verdict = np.empty(n, np.int32)
        identity = np.empty(n, np.uint32)
        stage = np.empty(n, np.uint8)
        probes = C.c_uint64(0)
        arrs = [np.ascontiguousarray(t[k], dt) for k, dt in (
            ("saddr", np.uint8), ("daddr", np.uint8), ("dport", np.uint16),
            ("proto", np.uint8), ("flags", np.uint8), ("len", np.uint32), ("ep", np.uint16))]
        self.L.or_classify_v6(self.h, n, *[_p(a) for a in arrs], _p(verdict), _p(identity),
                              _p(stage), nthreads, C.byref(probes))
        return verdict, identity, stage, probes.value

    def prefilter_v4(self, saddr, daddr, flags, nthreads=1):
        n = len(flags)
        out = np.empty(n, np.uint8)
        probes = C.c_uint64(0)
        s, d, f = (np.ascontiguousarray(saddr, np.uint32), np.ascontiguousarray(daddr, np.uint32),
                   np.ascontiguousarray(flags, np.uint8))
        self.L.or_prefilter_v4(self.h, n, _p(s), _p(d), _p(f), _p(out), nthreads, C.byref(probes))
        return out, probes.value

    def prefilter_v6(self, saddr16, daddr16, flags, nthreads=1):
        n = len(flags)
        out = np.empty(n, np.uint8)
        probes = C.c_uint64(0)
        s, d, f = (np.ascontiguousarray(saddr16, np.uint8), np.ascontiguousarray(daddr16, np.uint8),
                   np.ascontiguousarray(flags, np.uint8))
        self.L.or_prefilter_v6(self.h, n, _p(s), _p(d), _p(f), _p(out), nthreads, C.byref(probes))
        return out, probes.value

    # --- service load balancer ---
    def lb_update(self, key, val):
        return self.L.or_lb_update(self.h, _b(key), _b(val))

    def lb_update_batch(self, keys, vals):
        k, v = np.ascontiguousarray(keys), np.ascontiguousarray(vals)
        assert k.itemsize == 8 and v.itemsize == 12 and len(k) == len(v)
        return self.L.or_lb_update_many(self.h, _p(k), _p(v), len(k))

    def lb_delete(self, key):
        return self.L.or_lb_delete(self.h, _b(key))

    def flow_hash(self, saddr, daddr, sport, dport, proto):
        return self.L.or_flow_hash(saddr, daddr, sport, dport, proto)

    def lb4(self, t, mode, nthreads=1):
        """t: saddr/daddr (u32 network order), sport/dport (u16 network order),
        proto, optional hash.  mode 0 = bpf_lb.c handle_ipv4, 1 = lb4_local."""
        n = len(t["daddr"])
        cols = [np.ascontiguousarray(t[k], dt) for k, dt in (
            ("saddr", np.uint32), ("daddr", np.uint32), ("sport", np.uint16),
            ("dport", np.uint16), ("proto", np.uint8))]
        h = None if t.get("hash") is None else np.ascontiguousarray(t["hash"], np.uint32)
        out = {"ret": np.empty(n, np.int32), "saddr": np.empty(n, np.uint32),
               "daddr": np.empty(n, np.uint32), "tdaddr": np.empty(n, np.uint32),
               "dport": np.empty(n, np.uint16), "rev_nat": np.empty(n, np.uint16),
               "slave": np.empty(n, np.uint16)}
        probes = C.c_uint64(0)
        rc = self.L.or_lb4(self.h, mode, n, *[_p(a) for a in cols], _p(h),
                           *[_p(out[k]) for k in ("ret", "saddr", "daddr", "tdaddr", "dport",
                                                  "rev_nat", "slave")],
                           nthreads, C.byref(probes))
        assert rc == 0, rc
        return out, probes.value

    def classify_v4_lb(self, t, nthreads=1):
        """classify_v4 with the egress service step first (config 5)."""
        n = len(t["saddr"])
        verdict = np.empty(n, np.int32)
        identity = np.empty(n, np.uint32)
        stage = np.empty(n, np.uint8)
        probes = C.c_uint64(0)
        arrs = [np.ascontiguousarray(t[k], dt) for k, dt in (
            ("saddr", np.uint32), ("daddr", np.uint32), ("sport", np.uint16),
            ("dport", np.uint16), ("proto", np.uint8), ("flags", np.uint8), ("len", np.uint32),
            ("ep", np.uint16))]
        h = None if t.get("hash") is None else np.ascontiguousarray(t["hash"], np.uint32)
        rc = self.L.or_classify_v4_lb(self.h, n, *[_p(a) for a in arrs], _p(h), _p(verdict),
                                      _p(identity), _p(stage), nthreads, C.byref(probes))
        assert rc == 0, rc
        return verdict, identity, stage, probes.value

    def classify_v4_cascade(self, t, nthreads=1):
        """BASELINE config 5 whole: the XDP prefilter (bpf_xdp.c check_v4)
        before every ingress tuple, the service step before every egress one,
        then ipcache -> policy (or_classify_v4_cascade).  An XDP drop: verdict
        XDP_DROP_VERDICT, identity 0, stage 8, nothing counted."""
        n = len(t["saddr"])
        verdict = np.empty(n, np.int32)
        identity = np.empty(n, np.uint32)
        stage = np.empty(n, np.uint8)
        probes = C.c_uint64(0)
        arrs = [np.ascontiguousarray(t[k], dt) for k, dt in (
            ("saddr", np.uint32), ("daddr", np.uint32), ("sport", np.uint16),
            ("dport", np.uint16), ("proto", np.uint8), ("flags", np.uint8), ("len", np.uint32),
            ("ep", np.uint16))]
        h = None if t.get("hash") is None else np.ascontiguousarray(t["hash"], np.uint32)
        rc = self.L.or_classify_v4_cascade(self.h, n, *[_p(a) for a in arrs], _p(h), _p(verdict),
                                           _p(identity), _p(stage), nthreads, C.byref(probes))
        assert rc == 0, rc
        return verdict, identity, stage, probes.value

    # --- IPv6 service map ---
    def lb6_update(self, key, val):
        return self.L.or_lb6_update(self.h, _b(key), _b(val))

    def lb6_update_batch(self, keys, vals):
        for k, v in zip(keys, vals):
            rc = self.lb6_update(k, v)
            if rc:
                return rc
        return 0

    def lb6_delete(self, key):
        return self.L.or_lb6_delete(self.h, _b(key))

    def flow_hash6(self, saddr16, daddr16, sport, dport, proto):
        return self.L.or_flow_hash6(bytes(saddr16), bytes(daddr16), sport, dport, proto)

    def classify_v6_lb(self, t, nthreads=1):
        """classify_v6 with the egress service step of ipv6_l3_from_lxc first."""
        n = len(t["flags"])
        verdict = np.empty(n, np.int32)
        identity = np.empty(n, np.uint32)
        stage = np.empty(n, np.uint8)
        probes = C.c_uint64(0)
        arrs = [np.ascontiguousarray(t[k], dt) for k, dt in (
            ("saddr", np.uint8), ("daddr", np.uint8), ("sport", np.uint16),
            ("dport", np.uint16), ("proto", np.uint8), ("flags", np.uint8), ("len", np.uint32),
            ("ep", np.uint16))]
        h = None if t.get("hash") is None else np.ascontiguousarray(t["hash"], np.uint32)
        rc = self.L.or_classify_v6_lb(self.h, n, *[_p(a) for a in arrs], _p(h), _p(verdict),
                                      _p(identity), _p(stage), nthreads, C.byref(probes))
        assert rc == 0, rc
        return verdict, identity, stage, probes.value

    # --- raw frames ---
    def lxc_update(self, ep, info):
        return self.L.or_lxc_update(self.h, ep, _b(info))

    @staticmethod
    def _frame_cols(f):
        data = np.ascontiguousarray(f["data"], np.uint8)
        assert data.ndim == 2
        return (data, np.ascontiguousarray(f["len"], np.uint32),
                np.ascontiguousarray(f["flags"], np.uint8), np.ascontiguousarray(f["ep"], np.uint16))

    def frames_parse(self, f):
        data, ln, fl, ep = self._frame_cols(f)
        n = len(ln)
        out = {"status": np.empty(n, np.int32), "family": np.empty(n, np.uint8),
               "saddr": np.empty((n, 16), np.uint8), "daddr": np.empty((n, 16), np.uint8),
               "dport": np.empty(n, np.uint16), "proto": np.empty(n, np.uint8),
               "flags": np.empty(n, np.uint8)}
        self.L.or_frames_parse(self.h, n, _p(data), data.shape[1], _p(ln), _p(fl), _p(ep),
                               *[_p(out[k]) for k in ("status", "family", "saddr", "daddr",
                                                      "dport", "proto", "flags")])
        return out

    def classify_frames(self, f, nthreads=1):
        data, ln, fl, ep = self._frame_cols(f)
        n = len(ln)
        verdict = np.empty(n, np.int32)
        identity = np.empty(n, np.uint32)
        stage = np.empty(n, np.uint8)
        probes = C.c_uint64(0)
        self.L.or_classify_frames(self.h, n, _p(data), data.shape[1], _p(ln), _p(fl), _p(ep),
                                  _p(verdict), _p(identity), _p(stage), nthreads,
                                  C.byref(probes))
        return verdict, identity, stage, probes.value

    # --- conntrack ---
    def ct_set_max(self, n):
        self.L.or_ct_set_max(self.h, n)

    def ct4_update(self, key, val):
        return self.L.or_ct4_update(self.h, _b(key), _b(val))

    def ct4_delete(self, key):
        return self.L.or_ct4_delete(self.h, _b(key))

    def ct4_lookup(self, key):
        out = C.create_string_buffer(56)
        r = self.L.or_ct4_lookup(self.h, _b(key), out)
        return r, out.raw

    def ct4_count(self):
        return self.L.or_ct4_count(self.h)

    def ct4_dump(self):
        from cilium_amd import layouts as Ly
        n = self.ct4_count()
        keys = np.zeros(n, Ly.CT4_TUPLE)
        vals = np.zeros(n, Ly.CT_ENTRY)
        k = self.L.or_ct4_dump(self.h, _p(keys), _p(vals), n)
        assert k == n
        return Ly.ct_sorted(keys, vals)

    def ct4_gc(self, time):
        return self.L.or_ct4_gc(self.h, time)

    def classify_v4_ct(self, t, now):
        n = len(t["saddr"])
        verdict = np.empty(n, np.int32)
        ct_ret = np.empty(n, np.uint8)
        identity = np.empty(n, np.uint32)
        stage = np.empty(n, np.uint8)
        probes = C.c_uint64(0)
        arrs = [np.ascontiguousarray(t[k], dt) for k, dt in (
            ("saddr", np.uint32), ("daddr", np.uint32), ("sport", np.uint16),
            ("dport", np.uint16), ("proto", np.uint8), ("l4b", np.uint16), ("flags", np.uint8),
            ("len", np.uint32), ("ep", np.uint16))]
        rc = self.L.or_classify_v4_ct(self.h, n, *[_p(a) for a in arrs], now, _p(verdict),
                                      _p(ct_ret), _p(identity), _p(stage), C.byref(probes))
        assert rc == 0, rc
        return verdict, ct_ret, identity, stage, probes.value

    def classify_v4_ctlb(self, t, now):
        """or_classify_v4_ctlb: the stateful service step + conntrack; t as
        classify_v4_ct plus an optional "hash" column (skb->hash)."""
        n = len(t["saddr"])
        out = {"verdict": np.empty(n, np.int32), "ct_ret": np.empty(n, np.uint8),
               "identity": np.empty(n, np.uint32), "stage": np.empty(n, np.uint8),
               "xdaddr": np.empty(n, np.uint32), "xdport": np.empty(n, np.uint16)}
        probes = C.c_uint64(0)
        arrs = [np.ascontiguousarray(t[k], dt) for k, dt in (
            ("saddr", np.uint32), ("daddr", np.uint32), ("sport", np.uint16),
            ("dport", np.uint16), ("proto", np.uint8), ("l4b", np.uint16), ("flags", np.uint8),
            ("len", np.uint32), ("ep", np.uint16))]
        h = np.ascontiguousarray(t["hash"], np.uint32) if t.get("hash") is not None else None
        rc = self.L.or_classify_v4_ctlb(self.h, n, *[_p(a) for a in arrs],
                                        None if h is None else _p(h), now,
                                        *[_p(out[k]) for k in ("verdict", "ct_ret", "identity",
                                                               "stage", "xdaddr", "xdport")],
                                        C.byref(probes))
        assert rc == 0, rc
        out["probes"] = probes.value
        return out

    # --- IPv6 conntrack (cilium_ct6_global) ---
    def ct6_set_max(self, n):
        self.L.or_ct6_set_max(self.h, n)

    def ct6_update(self, key, val):
        return self.L.or_ct6_update(self.h, _b(key), _b(val))

    def ct6_delete(self, key):
        return self.L.or_ct6_delete(self.h, _b(key))

    def ct6_lookup(self, key):
        out = C.create_string_buffer(56)
        r = self.L.or_ct6_lookup(self.h, _b(key), out)
        return r, out.raw

    def ct6_count(self):
        return self.L.or_ct6_count(self.h)

    def ct6_dump(self):
        from cilium_amd import layouts as Ly
        n = self.ct6_count()
        keys = np.zeros(n, Ly.CT6_TUPLE)
        vals = np.zeros(n, Ly.CT_ENTRY)
        k = self.L.or_ct6_dump(self.h, _p(keys), _p(vals), n)
        assert k == n
        return Ly.ct_sorted(keys, vals)

    def ct6_gc(self, time):
        return self.L.or_ct6_gc(self.h, time)

    def classify_v6_ct(self, t, now):
        n = len(t["saddr"])
        verdict = np.empty(n, np.int32)
        ct_ret = np.empty(n, np.uint8)
        identity = np.empty(n, np.uint32)
        stage = np.empty(n, np.uint8)
        probes = C.c_uint64(0)
        arrs = [np.ascontiguousarray(t[k], dt) for k, dt in (
            ("saddr", np.uint8), ("daddr", np.uint8), ("sport", np.uint16),
            ("dport", np.uint16), ("proto", np.uint8), ("l4b", np.uint16), ("flags", np.uint8),
            ("len", np.uint32), ("ep", np.uint16))]
        rc = self.L.or_classify_v6_ct(self.h, n, *[_p(a) for a in arrs], now, _p(verdict),
                                      _p(ct_ret), _p(identity), _p(stage), C.byref(probes))
        assert rc == 0, rc
        return verdict, ct_ret, identity, stage, probes.value

    def classify_v6_ctlb(self, t, now):
        """or_classify_v6_ctlb: classify_v6_ct with the stateful service
        step; t may carry a "hash" column.  xdaddr is (n, 16) uint8."""
        n = len(t["saddr"])
        out = {"verdict": np.empty(n, np.int32), "ct_ret": np.empty(n, np.uint8),
               "identity": np.empty(n, np.uint32), "stage": np.empty(n, np.uint8),
               "xdaddr": np.empty((n, 16), np.uint8), "xdport": np.empty(n, np.uint16)}
        probes = C.c_uint64(0)
        arrs = [np.ascontiguousarray(t[k], dt) for k, dt in (
            ("saddr", np.uint8), ("daddr", np.uint8), ("sport", np.uint16),
            ("dport", np.uint16), ("proto", np.uint8), ("l4b", np.uint16), ("flags", np.uint8),
            ("len", np.uint32), ("ep", np.uint16))]
        h = np.ascontiguousarray(t["hash"], np.uint32) if t.get("hash") is not None else None
        rc = self.L.or_classify_v6_ctlb(self.h, n, *[_p(a) for a in arrs],
                                        None if h is None else _p(h), now,
                                        *[_p(out[k]) for k in ("verdict", "ct_ret", "identity",
                                                               "stage", "xdaddr", "xdport")],
                                        C.byref(probes))
        assert rc == 0, rc
        out["probes"] = probes.value
        return out

    # --- threaded stateful runs over independent shards ---
    def sharded(self, method, t, now, shard, nthreads):
        """Run the stateful `method` ("classify_v4_ct", "classify_v6_ct",
        "classify_v4_ctlb", "classify_v6_ctlb") over the packets of `t`
        split by `shard` (one id per packet), each shard on its own thread
        in a view with its own conntrack maps starting EMPTY (this context's
        maps must be empty), packets of a shard in batch order.  For shards
        that share no conntrack key (shard.ct_shard_of: every key a packet
        touches carries its address pair) this is exactly the sequential
        result.  Returns (results in batch order as `method` returns them,
        the wall seconds of the parallel section alone).  Afterwards this
        context holds the union of the shard maps and the summed metrics."""
        import threading
        import time as _time
        assert self.ct4_count() == 0 and self.ct6_count() == 0, "sharded run needs empty CT maps"
        shard = np.asarray(shard)
        ids = np.unique(shard)
        order = np.argsort(shard, kind="stable")
        bounds = np.searchsorted(shard[order], ids, side="left").tolist() + [len(order)]
        parts = [order[bounds[k]:bounds[k + 1]] for k in range(len(ids))]
        subs = [{k: (None if v is None else np.ascontiguousarray(v[p])) for k, v in t.items()}
                for p in parts]
        views = [Oracle.__new__(Oracle) for _ in parts]
        for v in views:
            v.L, v.cfg = self.L, self.cfg
            v.h = self.L.or_view_create(self.h)
        res = [None] * len(parts)
        nxt = [0]
        lock = threading.Lock()

        def run():
            while True:
                with lock:
                    k = nxt[0]
                    nxt[0] += 1
                if k >= len(parts):
                    return
                res[k] = getattr(views[k], method)(subs[k], now)

        th = [threading.Thread(target=run) for _ in range(max(1, min(nthreads, len(parts))))]
        c0 = _time.perf_counter()
        for x in th:
            x.start()
        for x in th:
            x.join()
        wall = _time.perf_counter() - c0
        for v in views:
            self.L.or_view_merge(self.h, v.h)
            self.L.or_view_destroy(v.h)
            v.h = None
        n = len(t["saddr"])
        if isinstance(res[0], dict):
            out = {}
            for key, val in res[0].items():
                if key == "probes":
                    out[key] = sum(r[key] for r in res)
                    continue
                a = np.empty((n,) + val.shape[1:], val.dtype)
                for p, r in zip(parts, res):
                    a[p] = r[key]
                out[key] = a
            return out, wall
        outs = []
        for j, val in enumerate(res[0]):
            if not isinstance(val, np.ndarray):
                outs.append(sum(r[j] for r in res))
                continue
            a = np.empty((n,) + val.shape[1:], val.dtype)
            for p, r in zip(parts, res):
                a[p] = r[j]
            outs.append(a)
        return tuple(outs), wall

    def sharded_steps(self, method, t, shard, nthreads, ops):
        """The steady-state form of `sharded`: one view per shard whose
        conntrack maps PERSIST across `ops`, a list of ("cls", now) -- the
        whole batch `t` again at time now -- and ("gc", time) -- ctmap.GC
        RemoveExpired on every view (a shard's entries carry its address
        pairs, so GC per shard = GC of the union).  Returns (the results of
        the last "cls" as `method` returns them, in batch order; the wall
        seconds of every op; the entries every "gc" deleted)."""
        import threading
        import time as _time
        assert self.ct4_count() == 0 and self.ct6_count() == 0, "sharded run needs empty CT maps"
        v6 = "v6" in method
        shard = np.asarray(shard)
        ids = np.unique(shard)
        order = np.argsort(shard, kind="stable")
        bounds = np.searchsorted(shard[order], ids, side="left").tolist() + [len(order)]
        parts = [order[bounds[k]:bounds[k + 1]] for k in range(len(ids))]
        subs = [{k: (None if v is None else np.ascontiguousarray(v[p])) for k, v in t.items()}
                for p in parts]
        views = [Oracle.__new__(Oracle) for _ in parts]
        for v in views:
            v.L, v.cfg = self.L, self.cfg
            v.h = self.L.or_view_create(self.h)
        walls, dels, res = [], [], [None] * len(parts)
        for op, tm in ops:
            nxt = [0]
            lock = threading.Lock()
            got = [0] * len(parts)

            def run():
                while True:
                    with lock:
                        k = nxt[0]
                        nxt[0] += 1
                    if k >= len(parts):
                        return
                    if op == "cls":
                        res[k] = getattr(views[k], method)(subs[k], tm)
                    else:
                        got[k] = (views[k].ct6_gc if v6 else views[k].ct4_gc)(tm)

            th = [threading.Thread(target=run) for _ in range(max(1, min(nthreads, len(parts))))]
            c0 = _time.perf_counter()
            for x in th:
                x.start()
            for x in th:
                x.join()
            walls.append(_time.perf_counter() - c0)
            if op == "gc":
                dels.append(int(sum(got)))
        for v in views:
            self.L.or_view_merge(self.h, v.h)
            self.L.or_view_destroy(v.h)
            v.h = None
        n = len(t["saddr"])
        outs = []
        for j, val in enumerate(res[0]):
            if not isinstance(val, np.ndarray):
                outs.append(sum(r[j] for r in res))
                continue
            a = np.empty((n,) + val.shape[1:], val.dtype)
            for p, r in zip(parts, res):
                a[p] = r[j]
            outs.append(a)
        return tuple(outs), walls, dels

    # --- L3 MapState compilation ---
    @staticmethod
    def l3_compile(prog, ep_sets, id_sets, flags=3):
        """prog: cilium_amd.policy.L3Program; *_sets: [[Label]].
        -> allow (n_ep, n_id) uint8: bit 0 ingress, bit 1 egress."""
        eo, el = prog.label_sets(ep_sets)
        io, il = prog.label_sets(id_sets)
        allow = np.zeros((len(ep_sets), len(id_sets)), np.uint8)

        def p(a):
            return None if a is None or len(a) == 0 else a.ctypes.data_as(C.c_void_p)
        lib().or_l3_compile(p(prog.selectors), p(prog.reqs), p(prog.values), p(prog.rule_subject),
                            p(prog.rule_clauses), len(prog.rule_subject), p(prog.clauses), p(eo),
                            p(el), len(ep_sets), p(io), p(il), len(id_sets), flags, p(allow))
        return allow

    def ipcache_lookup_addr(self, addr):
        """The batch paths' ipcache lookup of one address (network-order u32
        for IPv4, 16 bytes for IPv6): (rc, 8 value bytes)."""
        buf = C.create_string_buffer(8)
        if isinstance(addr, (bytes, bytearray, np.ndarray)) and len(bytes(addr)) == 16:
            rc = self.L.or_ipcache_lookup6(self.h, bytes(addr), buf)
        else:
            rc = self.L.or_ipcache_lookup4(self.h, int(addr), buf)
        return rc, buf.raw

    def set_fast(self, on=True):
        """or_set_fast: the optimized CPU ipcache (DIR-24-8 for IPv4, a
        multibit trie for IPv6, oracle/fast_lpm.h) built from the current
        ipcache, or back to the kernel-like trie.  Same answers; an ipcache
        change drops it."""
        rc = self.L.or_set_fast(self.h, 1 if on else 0)
        assert rc == 0, rc

    PROBE_MAPS = ("ipcache", "policy", "lb", "prefilter", "endpoint")

    def probe_split(self):
        """Reference map lookups since the last call, by map (or_probe_split,
        read and reset; after `sharded` the views' lookups are included):
        the roofline prices each at the gather ceiling of its tier.  A
        stateful call's conntrack operations are its probe count minus the
        sum of these."""
        out = np.zeros(len(self.PROBE_MAPS), np.uint64)
        self.L.or_probe_split(self.h, _p(out))
        return {k: int(v) for k, v in zip(self.PROBE_MAPS, out)}

    def metrics(self):
        out = np.zeros((256, 4, 2), np.uint64)
        self.L.or_metrics_read(self.h, _p(out))
        return out

    def counters_reset(self):
        self.L.or_counters_reset(self.h)
