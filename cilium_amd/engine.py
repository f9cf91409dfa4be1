"""Python face of the engine: a thin wrapper over the C ABI (include/cgpu.h).

The map objects mirror the method sets of the reference's Go map wrappers so
that tests read like the reference's own callers:

* :class:`PolicyMap`  — pkg/maps/policymap/policymap.go (Allow/AllowKey/Exists/
  Delete/DeleteKey/DumpToSlice/Flush)
* :class:`IPCacheMap` — pkg/maps/ipcache/ipcache.go (Update/Delete with the
  tombstone-on-ENOSYS variant, NewKey) and the IPIdentityMappingListener hook
  (pkg/ipcache/listener.go:36-48, pkg/datapath/ipcache/listener.go:78-127)
* :class:`CIDRMap`    — pkg/maps/cidrmap/cidrmap.go (InsertCIDR/DeleteCIDR/
  CIDRExists/CIDRDump, checkPrefixlen)
* :class:`LBMap`      — pkg/maps/lbmap/lbmap.go (UpdateService/DeleteService/
  LookupService/DumpServiceMapsToUserspace over cilium_lb4_services)

Batch entry points take torch CUDA tensors (device memory) and launch on the
caller's current HIP stream.  Nothing here computes a verdict on the CPU.
"""
from __future__ import annotations

import ctypes as C
import errno
import ipaddress

import numpy as np

from . import layouts as L
from ._abi import (CgpuConfig, CgpuError, CtlbOut, FrameTuples, Frames, Lb4Out, Lb4Tuples, TuplesV4,
                   TuplesV4Ct, TuplesV6Ct, TuplesV6, check, lib)

CIDR_V4_DYN, CIDR_V4_FIX, CIDR_V6_DYN, CIDR_V6_FIX = 0, 1, 2, 3
BPF_ANY, BPF_NOEXIST, BPF_EXIST = 0, 1, 2


def _buf(x) -> bytes:
    return np.ascontiguousarray(x).tobytes()


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def _stream(stream):
    if stream is None:
        import torch
        stream = torch.cuda.current_stream()
    return C.c_void_p(stream.cuda_stream)


class Engine:
    """One cgpu context bound to one GPU (device=-1: host-only, table ops)."""

    def __init__(self, device: int = 0, **cfg):
        self.L = lib()
        self.cfg = CgpuConfig()
        self.L.cgpu_config_default(C.byref(self.cfg))
        for k, v in cfg.items():
            if not hasattr(self.cfg, k):
                raise TypeError(f"unknown config field {k}")
            if k in ("ipv6_router_ip", "node_mac"):
                getattr(self.cfg, k)[:] = bytes(v)
                continue
            setattr(self.cfg, k, v)
        h = C.c_void_p()
        check(self.L.cgpu_ctx_create(C.byref(self.cfg), device, C.byref(h)), "cgpu_ctx_create")
        self.h = h
        self.device = device
        self._bound = None

    def close(self):
        if getattr(self, "h", None):
            self.L.cgpu_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------- raw map ops
    def ipcache_update(self, key, val, flags=BPF_ANY) -> int:
        return self.L.cgpu_ipcache_update(self.h, _buf(key), _buf(val), flags)

    def ipcache_delete(self, key) -> int:
        return self.L.cgpu_ipcache_delete(self.h, _buf(key))

    def ipcache_lookup(self, key):
        out = C.create_string_buffer(8)
        rc = self.L.cgpu_ipcache_lookup(self.h, _buf(key), out)
        return rc, (np.frombuffer(out.raw, L.REMOTE_ENDPOINT_INFO)[0] if rc == 0 else None)

    def ipcache_update_batch(self, keys, vals, flags=BPF_ANY) -> int:
        k = np.ascontiguousarray(keys, L.IPCACHE_KEY)
        v = np.ascontiguousarray(vals, L.REMOTE_ENDPOINT_INFO)
        assert len(k) == len(v)
        return self.L.cgpu_ipcache_update_batch(self.h, k.ctypes.data, v.ctypes.data, len(k), flags)

    def ipcache_keys(self):
        keys, prev = [], None
        out = C.create_string_buffer(24)
        while self.L.cgpu_ipcache_get_next_key(self.h, prev, out) == 0:
            prev = out.raw
            keys.append(np.frombuffer(prev, L.IPCACHE_KEY)[0])
        return keys

    def policy_update(self, ep, key, entry, flags=BPF_ANY) -> int:
        return self.L.cgpu_policy_update(self.h, ep, _buf(key), _buf(entry), flags)

    def policy_delete(self, ep, key) -> int:
        return self.L.cgpu_policy_delete(self.h, ep, _buf(key))

    def policy_lookup(self, ep, key):
        out = C.create_string_buffer(24)
        rc = self.L.cgpu_policy_lookup(self.h, ep, _buf(key), out)
        return rc, (np.frombuffer(out.raw, L.POLICY_ENTRY)[0] if rc == 0 else None)

    def policy_keys(self, ep):
        keys, prev = [], None
        out = C.create_string_buffer(8)
        while self.L.cgpu_policy_get_next_key(self.h, ep, prev, out) == 0:
            prev = out.raw
            keys.append(np.frombuffer(prev, L.POLICY_KEY)[0])
        return keys

    def policy_flush(self, ep) -> int:
        return self.L.cgpu_policy_flush(self.h, ep)

    def policy_update_batch(self, eps, keys, entries, flags=BPF_ANY) -> int:
        e = np.ascontiguousarray(eps, np.uint32)
        k = np.ascontiguousarray(keys, L.POLICY_KEY)
        v = np.ascontiguousarray(entries, L.POLICY_ENTRY)
        assert len(e) == len(k) == len(v)
        return self.L.cgpu_policy_update_batch(self.h, e.ctypes.data, k.ctypes.data, v.ctypes.data,
                                               len(k), flags)

    def policy_lookup_batch(self, eps, keys):
        """(rc[n], entries[n]) of cgpu_policy_lookup_batch (one device read)."""
        e = np.ascontiguousarray(eps, np.uint32)
        k = np.ascontiguousarray(keys, L.POLICY_KEY)
        out = np.zeros(len(k), L.POLICY_ENTRY)
        rc = np.zeros(len(k), np.int32)
        check(self.L.cgpu_policy_lookup_batch(self.h, e.ctypes.data, k.ctypes.data, len(k),
                                              out.ctypes.data, rc.ctypes.data),
              "cgpu_policy_lookup_batch")
        return rc, out

    def policy_counters(self, eps, keys) -> np.ndarray:
        """(n, 2) uint64 {packets, bytes} of present keys (raises if any is absent)."""
        rc, out = self.policy_lookup_batch(eps, keys)
        assert (rc == 0).all(), "policy key absent"
        return np.stack([out["packets"], out["bytes"]], 1).astype(np.uint64)

    def policy_dump(self, ep):
        """DumpToSlice of one endpoint's map: (keys, entries)."""
        n = C.c_size_t()
        rc = self.L.cgpu_policy_dump(self.h, ep, None, None, 0, C.byref(n))
        keys = np.zeros(n.value, L.POLICY_KEY)
        ents = np.zeros(n.value, L.POLICY_ENTRY)
        if n.value:
            check(self.L.cgpu_policy_dump(self.h, ep, keys.ctypes.data, ents.ctypes.data, n.value,
                                          C.byref(n)), "cgpu_policy_dump")
        elif rc < 0:
            check(rc, "cgpu_policy_dump")
        return keys, ents

    @staticmethod
    def _cidr_buf(key) -> bytes:
        raw = _buf(key)
        return raw + bytes(20 - len(raw))

    def cidr_update(self, which, key, flags=BPF_ANY) -> int:
        return self.L.cgpu_cidr_update(self.h, which, self._cidr_buf(key), flags)

    def cidr_update_batch(self, which, keys, flags=BPF_ANY) -> int:
        """keys: LPM_V4_KEY / LPM_V6_KEY records (padded to 20-byte keys)."""
        k = np.ascontiguousarray(keys)
        buf = np.zeros((len(k), 20), np.uint8)
        buf[:, :k.dtype.itemsize] = k.view(np.uint8).reshape(len(k), k.dtype.itemsize)
        return self.L.cgpu_cidr_update_batch(self.h, which, buf.ctypes.data, len(k), flags)

    def cidr_delete(self, which, key) -> int:
        return self.L.cgpu_cidr_delete(self.h, which, self._cidr_buf(key))

    def cidr_lookup(self, which, key) -> int:
        return self.L.cgpu_cidr_lookup(self.h, which, self._cidr_buf(key))

    def cidr_keys(self, which):
        keys, prev = [], None
        out = C.create_string_buffer(20)
        dt = L.LPM_V4_KEY if which in (CIDR_V4_DYN, CIDR_V4_FIX) else L.LPM_V6_KEY
        while self.L.cgpu_cidr_get_next_key(self.h, which, prev, out) == 0:
            prev = out.raw
            keys.append(np.frombuffer(prev[:dt.itemsize], dt)[0])
        return keys

    def endpoint_update(self, key, flags=BPF_ANY) -> int:
        return self.L.cgpu_endpoint_update(self.h, _buf(key), flags)

    def endpoint_delete(self, key) -> int:
        return self.L.cgpu_endpoint_delete(self.h, _buf(key))

    def endpoint_lookup(self, key) -> int:
        return self.L.cgpu_endpoint_lookup(self.h, _buf(key))

    def lb4_update(self, key, val, flags=BPF_ANY) -> int:
        return self.L.cgpu_lb4_update(self.h, _buf(key), _buf(val), flags)

    def lb4_update_batch(self, keys, vals, flags=BPF_ANY) -> int:
        k = np.ascontiguousarray(keys, L.LB4_KEY)
        v = np.ascontiguousarray(vals, L.LB4_SERVICE)
        assert len(k) == len(v)
        return self.L.cgpu_lb4_update_batch(self.h, k.ctypes.data, v.ctypes.data, len(k), flags)

    def lb4_delete(self, key) -> int:
        return self.L.cgpu_lb4_delete(self.h, _buf(key))

    def lb4_lookup(self, key):
        out = C.create_string_buffer(12)
        rc = self.L.cgpu_lb4_lookup(self.h, _buf(key), out)
        return rc, (np.frombuffer(out.raw, L.LB4_SERVICE)[0] if rc == 0 else None)

    def lb4_keys(self):
        keys, prev = [], None
        out = C.create_string_buffer(8)
        while self.L.cgpu_lb4_get_next_key(self.h, prev, out) == 0:
            prev = out.raw
            keys.append(np.frombuffer(prev, L.LB4_KEY)[0])
        return keys

    def lb4_count(self) -> int:
        return self.L.cgpu_lb4_count(self.h)

    # --- cilium_lb6_services ---
    def lb6_update(self, key, val, flags=BPF_ANY) -> int:
        return self.L.cgpu_lb6_update(self.h, _buf(key), _buf(val), flags)

    def lb6_update_batch(self, keys, vals, flags=BPF_ANY) -> int:
        k = np.ascontiguousarray(keys, L.LB6_KEY)
        v = np.ascontiguousarray(vals, L.LB6_SERVICE)
        assert len(k) == len(v)
        return self.L.cgpu_lb6_update_batch(self.h, k.ctypes.data, v.ctypes.data, len(k), flags)

    def lb6_delete(self, key) -> int:
        return self.L.cgpu_lb6_delete(self.h, _buf(key))

    def lb6_lookup(self, key):
        out = C.create_string_buffer(24)
        rc = self.L.cgpu_lb6_lookup(self.h, _buf(key), out)
        return rc, (np.frombuffer(out.raw, L.LB6_SERVICE)[0] if rc == 0 else None)

    def lb6_keys(self):
        keys, prev = [], None
        out = C.create_string_buffer(20)
        while self.L.cgpu_lb6_get_next_key(self.h, prev, out) == 0:
            prev = out.raw
            keys.append(np.frombuffer(prev, L.LB6_KEY)[0])
        return keys

    def lb6_count(self) -> int:
        return self.L.cgpu_lb6_count(self.h)

    def flow_hash6(self, saddr16, daddr16, sport, dport, proto) -> int:
        return self.L.cgpu_flow_hash6(bytes(saddr16), bytes(daddr16), sport, dport, proto)

    # --- conntrack map cilium_ct4_global ---
    def ct4_update(self, key, val, flags=BPF_ANY) -> int:
        return self.L.cgpu_ct4_update(self.h, _buf(key), _buf(val), flags)

    def ct4_delete(self, key) -> int:
        return self.L.cgpu_ct4_delete(self.h, _buf(key))

    def ct4_lookup(self, key):
        out = C.create_string_buffer(56)
        rc = self.L.cgpu_ct4_lookup(self.h, _buf(key), out)
        return rc, (np.frombuffer(out.raw, L.CT_ENTRY)[0] if rc == 0 else None)

    def ct4_count(self) -> int:
        return self.L.cgpu_ct4_count(self.h)

    def ct4_gc(self, time: int) -> int:
        d = C.c_uint64()
        check(self.L.cgpu_ct4_gc(self.h, time, C.byref(d)), "cgpu_ct4_gc")
        return d.value

    def ct_stats(self, v6: bool = False) -> dict:
        """cgpu_ct_stats: live entries, tombstones and compactions of the map."""
        out = np.zeros(3, np.uint64)
        check(self.L.cgpu_ct_stats(self.h, int(v6), out.ctypes.data_as(C.c_void_p)), "cgpu_ct_stats")
        return {"live": int(out[0]), "tombstones": int(out[1]), "compactions": int(out[2])}

    def ct4_flush(self) -> None:
        check(self.L.cgpu_ct4_flush(self.h), "cgpu_ct4_flush")

    def ct4_dump(self):
        """(keys, vals) of the whole map via get_next_key + lookup, sorted
        canonically (layouts.ct_sorted)."""
        keys, vals, prev = [], [], None
        out = C.create_string_buffer(14)
        cap = self.ct4_count()
        while self.L.cgpu_ct4_get_next_key(self.h, prev, out) == 0:
            # a key stored twice would restart the walk forever
            if len(keys) > cap:
                raise AssertionError("cilium_ct4_global holds a key twice")
            prev = out.raw
            rc, v = self.ct4_lookup(np.frombuffer(prev, L.CT4_TUPLE)[0])
            assert rc == 0
            keys.append(np.frombuffer(prev, L.CT4_TUPLE)[0])
            vals.append(v)
        return L.ct_sorted(np.array(keys, L.CT4_TUPLE), np.array(vals, L.CT_ENTRY))

    # --- cilium_ct6_global (IPv6 conntrack) ---
    def ct6_update(self, key, val, flags=BPF_ANY) -> int:
        return self.L.cgpu_ct6_update(self.h, _buf(key), _buf(val), flags)

    def ct6_delete(self, key) -> int:
        return self.L.cgpu_ct6_delete(self.h, _buf(key))

    def ct6_lookup(self, key):
        out = C.create_string_buffer(56)
        rc = self.L.cgpu_ct6_lookup(self.h, _buf(key), out)
        return rc, (np.frombuffer(out.raw, L.CT_ENTRY)[0] if rc == 0 else None)

    def ct6_count(self) -> int:
        return self.L.cgpu_ct6_count(self.h)

    def ct6_gc(self, time: int) -> int:
        d = C.c_uint64()
        check(self.L.cgpu_ct6_gc(self.h, time, C.byref(d)), "cgpu_ct6_gc")
        return d.value

    def ct6_flush(self) -> None:
        check(self.L.cgpu_ct6_flush(self.h), "cgpu_ct6_flush")

    def ct6_dump(self):
        keys, vals, prev = [], [], None
        out = C.create_string_buffer(38)
        cap = self.ct6_count()
        while self.L.cgpu_ct6_get_next_key(self.h, prev, out) == 0:
            # a key stored twice would restart the walk forever
            if len(keys) > cap:
                raise AssertionError("cilium_ct6_global holds a key twice")
            prev = out.raw
            rc, v = self.ct6_lookup(np.frombuffer(prev, L.CT6_TUPLE)[0])
            assert rc == 0
            keys.append(np.frombuffer(prev, L.CT6_TUPLE)[0])
            vals.append(v)
        return L.ct_sorted(np.array(keys, L.CT6_TUPLE), np.array(vals, L.CT_ENTRY))

    # --- L3 MapState compilation ---
    def l3_compile(self, prog, ep_sets, id_sets, flags: int = 3) -> np.ndarray:
        """cgpu_l3_compile: prog = cilium_amd.policy.L3Program, *_sets =
        [[Label]] (endpoint / identity label arrays) or their interned form
        prog.label_sets(...) (offsets, LABEL records).  -> (n_ep, n_id) uint8,
        bit 0 ingress Allowed, bit 1 egress Allowed."""
        from . import policy as P
        eo, el = ep_sets if isinstance(ep_sets, tuple) else prog.label_sets(ep_sets)
        io, il = id_sets if isinstance(id_sets, tuple) else prog.label_sets(id_sets)
        allow = np.zeros((len(eo) - 1, len(io) - 1), np.uint8)
        cp, ce, ci = P.c_program(prog), P.c_label_sets(eo, el), P.c_label_sets(io, il)
        check(self.L.cgpu_l3_compile(self.h, C.byref(cp), C.byref(ce), C.byref(ci), flags,
                                     allow.ctypes.data), "cgpu_l3_compile")
        return allow

    def mapstate_sync(self, msp) -> dict:
        """cgpu_mapstate_sync: msp = cilium_amd.policy.compile_mapstate(...).
        Computes every endpoint's desired MapState on the device and syncs
        it into the host mirror's policy maps (visible after commit()).
        -> the sync counts {desired, added, updated, deleted, unchanged,
        failed}; raises on the first failing key like syncPolicyMap's error."""
        from . import policy as P
        m = msp
        cp, ce, ci = P.c_program(m.prog), P.c_label_sets(*m.ep_sets), P.c_label_sets(*m.id_sets)
        spec, stats = P.c_mapstate_spec(m), P.CMapStateStats()
        rc = self.L.cgpu_mapstate_sync(self.h, C.byref(cp), C.byref(ce), C.byref(ci),
                                       C.byref(spec), C.byref(stats))
        out = {n: getattr(stats, n) for n, _ in P.CMapStateStats._fields_}
        check(rc, "cgpu_mapstate_sync")
        return out

    def flow_hash(self, saddr, daddr, sport, dport, proto) -> int:
        return self.L.cgpu_flow_hash(saddr, daddr, sport, dport, proto)

    def commit(self) -> int:
        ep = C.c_uint64()
        check(self.L.cgpu_commit(self.h, C.byref(ep)), "cgpu_commit")
        return ep.value

    def checksum(self) -> int:
        s = C.c_uint64()
        check(self.L.cgpu_table_checksum(self.h, C.byref(s)), "cgpu_table_checksum")
        return s.value

    def mirror_save(self, path: str) -> None:
        """cgpu_mirror_save: checkpoint the host mirror (+ counters, CT maps)."""
        check(self.L.cgpu_mirror_save(self.h, str(path).encode()), "cgpu_mirror_save")

    def mirror_restore(self, path: str) -> None:
        """cgpu_mirror_restore into this (empty) context; commit afterwards."""
        check(self.L.cgpu_mirror_restore(self.h, str(path).encode()), "cgpu_mirror_restore")

    def verify(self) -> None:
        """cgpu_table_verify: the device tables still equal the host images
        (raises CgpuError EIO naming the group otherwise)."""
        check(self.L.cgpu_table_verify(self.h), "cgpu_table_verify")

    TABLES = ("ipcache", "policy", "prefilter", "endpoint", "lb4", "lxc", "lb6", "ct4", "ct6")

    def table_bytes(self) -> dict:
        """cgpu_table_bytes: device bytes of each table group of the published
        snapshot and of the conntrack maps."""
        out = np.zeros(len(self.TABLES), np.uint64)
        check(self.L.cgpu_table_bytes(self.h, out.ctypes.data_as(C.c_void_p)), "cgpu_table_bytes")
        return {k: int(v) for k, v in zip(self.TABLES, out)}

    def counter_layout_checksum(self) -> int:
        s = C.c_uint64()
        check(self.L.cgpu_counter_layout_checksum(self.h, C.byref(s)), "cgpu_counter_layout_checksum")
        return s.value

    # -------------------------------------------------------------- batches
    def classify_v4(self, t: dict, out: dict | None = None, stage: bool = True, stream=None):
        """t: dict of CUDA tensors saddr/daddr (int32 view of network-order
        u32), dport (int16), proto/flags (uint8), len (int32), ep (int16)."""
        import torch
        n = t["saddr"].numel()
        dev = t["saddr"].device
        if out is None:
            out = {"verdict": torch.empty(n, dtype=torch.int32, device=dev),
                   "identity": torch.empty(n, dtype=torch.int32, device=dev),
                   "stage": torch.empty(n, dtype=torch.uint8, device=dev) if stage else None}
        tv = TuplesV4(*[t[k].data_ptr() for k in
                        ("saddr", "daddr", "dport", "proto", "flags", "len", "ep")])
        check(self.L.cgpu_classify_v4(self.h, C.byref(tv), n, _ptr(out["verdict"]),
                                      _ptr(out["identity"]), _ptr(out.get("stage")),
                                      _stream(stream)), "cgpu_classify_v4")
        return out

    @staticmethod
    def _hptr(x):
        if x is None:
            return None
        return C.c_void_p(x.data_ptr() if hasattr(x, "data_ptr") else x.ctypes.data)

    def _host_call(self, fn, tv_cls, t, n, out, stage, stream, lb):
        """The host-resident classify entry points: t holds HOST arrays
        (numpy, or CPU tensors -- page-locked ones overlap the copies with
        the classify) with the dtypes of the device call; outputs are host
        numpy arrays, complete when `stream` is (the call synchronizes it
        before returning unless out is given)."""
        p = self._hptr
        given = out is not None
        if out is None:
            out = {"verdict": np.empty(n, np.int32), "identity": np.empty(n, np.uint32),
                   "stage": np.empty(n, np.uint8) if stage else None}
        tv = tv_cls(*[p(t[k]).value for k in ("saddr", "daddr", "dport", "proto", "flags", "len", "ep")])
        lbargs = (p(t.get("sport")), p(t.get("hash"))) if lb else ()
        check(getattr(self.L, fn)(self.h, C.byref(tv), *lbargs, n, p(out["verdict"]),
                                  p(out["identity"]), p(out.get("stage")), _stream(stream)), fn)
        if not given:
            import torch
            (stream or torch.cuda.current_stream()).synchronize()
        return out

    def classify_v4_host(self, t: dict, out: dict | None = None, stage: bool = True, stream=None):
        """cgpu_classify_v4_host: classify_v4 over host arrays (_host_call)."""
        return self._host_call("cgpu_classify_v4_host", TuplesV4, t, len(t["saddr"]), out, stage,
                               stream, False)

    def classify_v4_lb_host(self, t: dict, out: dict | None = None, stage: bool = True, stream=None,
                            xdp: bool = False):
        """cgpu_classify_v4_lb_host / cgpu_classify_v4_cascade_host (xdp):
        classify_v4_lb over host arrays; t holds "hash" or "sport" too."""
        fn = "cgpu_classify_v4_cascade_host" if xdp else "cgpu_classify_v4_lb_host"
        return self._host_call(fn, TuplesV4, t, len(t["saddr"]), out, stage, stream, True)

    def classify_v6_host(self, t: dict, out: dict | None = None, stage: bool = True, stream=None,
                         lb: bool = False):
        """cgpu_classify_v6_host / cgpu_classify_v6_lb_host (lb): classify_v6
        over host arrays (saddr / daddr (n, 16) uint8, any alignment)."""
        fn = "cgpu_classify_v6_lb_host" if lb else "cgpu_classify_v6_host"
        return self._host_call(fn, TuplesV6, t, len(t["flags"]), out, stage, stream, lb)

    def prefilter_host(self, saddr, daddr, flags, v6: bool = False, out=None, stream=None):
        """cgpu_prefilter_v4_host / _v6_host over host arrays; returns the
        verdict bytes (synchronizes `stream` unless out is given)."""
        p = self._hptr
        given = out is not None
        if out is None:
            out = np.empty(len(flags), np.uint8)
        fn = "cgpu_prefilter_v6_host" if v6 else "cgpu_prefilter_v4_host"
        check(getattr(self.L, fn)(self.h, p(saddr), p(daddr), p(flags), len(flags), p(out),
                                  _stream(stream)), fn)
        if not given:
            import torch
            (stream or torch.cuda.current_stream()).synchronize()
        return out

    def classify_v4_ct(self, t: dict, now: int, out: dict | None = None, stage: bool = True,
                       stream=None):
        """Stateful classification (cgpu_classify_v4_ct): t holds CUDA tensors
        saddr/daddr (int32), sport/dport (int16, network order), proto/flags
        (uint8), l4b (int16: TCP header bytes 12-13 / ICMP type), len (int32),
        ep (int16); now = bpf_ktime_get_sec() of the batch."""
        import torch
        n = t["saddr"].numel()
        dev = t["saddr"].device
        if out is None:
            out = {"verdict": torch.empty(n, dtype=torch.int32, device=dev),
                   "ct_ret": torch.empty(n, dtype=torch.uint8, device=dev),
                   "identity": torch.empty(n, dtype=torch.int32, device=dev),
                   "stage": torch.empty(n, dtype=torch.uint8, device=dev) if stage else None}
        tv = TuplesV4Ct(*[t[k].data_ptr() for k in
                          ("saddr", "daddr", "sport", "dport", "proto", "l4b", "flags", "len", "ep")])
        check(self.L.cgpu_classify_v4_ct(self.h, C.byref(tv), n, now, _ptr(out["verdict"]),
                                         _ptr(out["ct_ret"]), _ptr(out["identity"]),
                                         _ptr(out.get("stage")), _stream(stream)),
              "cgpu_classify_v4_ct")
        return out

    def classify_v4_ctlb(self, t: dict, now: int, out: dict | None = None, stage: bool = True,
                         xlate: bool = True, stream=None):
        """cgpu_classify_v4_ctlb: classify_v4_ct with the stateful service
        step (lb4_local with CONNTRACK) in front; t may carry a "hash" column
        (skb->hash, int32).  out adds "daddr" / "dport": the frame after the
        service step (xlate=False: not written)."""
        import torch
        n = t["saddr"].numel()
        dev = t["saddr"].device
        if out is None:
            out = {"verdict": torch.empty(n, dtype=torch.int32, device=dev),
                   "ct_ret": torch.empty(n, dtype=torch.uint8, device=dev),
                   "identity": torch.empty(n, dtype=torch.int32, device=dev),
                   "stage": torch.empty(n, dtype=torch.uint8, device=dev) if stage else None,
                   "daddr": torch.empty(n, dtype=torch.int32, device=dev) if xlate else None,
                   "dport": torch.empty(n, dtype=torch.int16, device=dev) if xlate else None}
        tv = TuplesV4Ct(*[t[k].data_ptr() for k in
                          ("saddr", "daddr", "sport", "dport", "proto", "l4b", "flags", "len", "ep")])
        ov = CtlbOut(*[_ptr(out.get(k)) for k in ("verdict", "ct_ret", "identity", "stage", "daddr",
                                                   "dport")])
        check(self.L.cgpu_classify_v4_ctlb(self.h, C.byref(tv), _ptr(t.get("hash")), n, now,
                                           C.byref(ov), _stream(stream)), "cgpu_classify_v4_ctlb")
        return out

    def classify_v6_ct(self, t: dict, now: int, out: dict | None = None, stage: bool = True,
                       stream=None):
        """cgpu_classify_v6_ct: as classify_v4_ct with saddr / daddr (n, 16)
        uint8 tensors (16-byte aligned rows)."""
        import torch
        n = t["saddr"].shape[0]
        dev = t["saddr"].device
        if out is None:
            out = {"verdict": torch.empty(n, dtype=torch.int32, device=dev),
                   "ct_ret": torch.empty(n, dtype=torch.uint8, device=dev),
                   "identity": torch.empty(n, dtype=torch.int32, device=dev),
                   "stage": torch.empty(n, dtype=torch.uint8, device=dev) if stage else None}
        tv = TuplesV6Ct(*[t[k].data_ptr() for k in
                          ("saddr", "daddr", "sport", "dport", "proto", "l4b", "flags", "len", "ep")])
        check(self.L.cgpu_classify_v6_ct(self.h, C.byref(tv), n, now, _ptr(out["verdict"]),
                                         _ptr(out["ct_ret"]), _ptr(out["identity"]),
                                         _ptr(out.get("stage")), _stream(stream)),
              "cgpu_classify_v6_ct")
        return out

    def classify_v6_ctlb(self, t: dict, now: int, out: dict | None = None, stage: bool = True,
                         xlate: bool = True, stream=None):
        """cgpu_classify_v6_ctlb: classify_v6_ct with the stateful service
        step (lb6_local with CONNTRACK) in front; out "daddr" is (n, 16)
        uint8."""
        import torch
        n = t["saddr"].shape[0]
        dev = t["saddr"].device
        if out is None:
            out = {"verdict": torch.empty(n, dtype=torch.int32, device=dev),
                   "ct_ret": torch.empty(n, dtype=torch.uint8, device=dev),
                   "identity": torch.empty(n, dtype=torch.int32, device=dev),
                   "stage": torch.empty(n, dtype=torch.uint8, device=dev) if stage else None,
                   "daddr": torch.empty((n, 16), dtype=torch.uint8, device=dev) if xlate else None,
                   "dport": torch.empty(n, dtype=torch.int16, device=dev) if xlate else None}
        tv = TuplesV6Ct(*[t[k].data_ptr() for k in
                          ("saddr", "daddr", "sport", "dport", "proto", "l4b", "flags", "len", "ep")])
        ov = CtlbOut(*[_ptr(out.get(k)) for k in ("verdict", "ct_ret", "identity", "stage", "daddr",
                                                   "dport")])
        check(self.L.cgpu_classify_v6_ctlb(self.h, C.byref(tv), _ptr(t.get("hash")), n, now,
                                           C.byref(ov), _stream(stream)), "cgpu_classify_v6_ctlb")
        return out

    def classify_v4_lb(self, t: dict, out: dict | None = None, stage: bool = True, stream=None,
                       xdp: bool = False):
        """classify_v4 with the egress service step first (BASELINE config 5).
        t additionally holds "hash" (int32 view of skb->hash) or "sport".
        xdp=True: cgpu_classify_v4_cascade, the netdev's XDP prefilter before
        every ingress tuple too (the full config-5 cascade)."""
        import torch
        n = t["saddr"].numel()
        dev = t["saddr"].device
        if out is None:
            out = {"verdict": torch.empty(n, dtype=torch.int32, device=dev),
                   "identity": torch.empty(n, dtype=torch.int32, device=dev),
                   "stage": torch.empty(n, dtype=torch.uint8, device=dev) if stage else None}
        tv = TuplesV4(*[t[k].data_ptr() for k in
                        ("saddr", "daddr", "dport", "proto", "flags", "len", "ep")])
        fn = "cgpu_classify_v4_cascade" if xdp else "cgpu_classify_v4_lb"
        check(getattr(self.L, fn)(self.h, C.byref(tv), _ptr(t.get("sport")), _ptr(t.get("hash")), n,
                                  _ptr(out["verdict"]), _ptr(out["identity"]), _ptr(out.get("stage")),
                                  _stream(stream)), fn)
        return out

    def classify_v4_cascade(self, t: dict, out: dict | None = None, stage: bool = True, stream=None):
        """BASELINE config 5 whole (cgpu_classify_v4_cascade): XDP prefilter
        -> ipcache -> policy for ingress tuples, service step -> ipcache ->
        policy for egress ones."""
        return self.classify_v4_lb(t, out=out, stage=stage, stream=stream, xdp=True)

    def lb4_select(self, t: dict, mode: int, out: dict | None = None, stream=None):
        """Service translation alone: t holds saddr/daddr (int32 views),
        dport/sport (int16 views), proto (uint8), optional hash (int32)."""
        import torch
        n = t["daddr"].numel()
        dev = t["daddr"].device
        if out is None:
            out = {"ret": torch.empty(n, dtype=torch.int32, device=dev),
                   "saddr": torch.empty(n, dtype=torch.int32, device=dev),
                   "daddr": torch.empty(n, dtype=torch.int32, device=dev),
                   "dport": torch.empty(n, dtype=torch.int16, device=dev),
                   "rev_nat": torch.empty(n, dtype=torch.int16, device=dev),
                   "slave": torch.empty(n, dtype=torch.int16, device=dev)}
        tv = Lb4Tuples(*[_ptr(t.get(k)) for k in ("saddr", "daddr", "sport", "dport", "proto",
                                                  "hash")])
        ov = Lb4Out(*[_ptr(out.get(k)) for k in ("ret", "saddr", "daddr", "dport", "rev_nat",
                                                 "slave")])
        check(self.L.cgpu_lb4_select(self.h, mode, C.byref(tv), n, C.byref(ov), _stream(stream)),
              "cgpu_lb4_select")
        return out

    def classify_v6(self, t: dict, out: dict | None = None, stage: bool = True, stream=None):
        """t: saddr/daddr uint8 CUDA tensors of shape (n, 16) (16-byte
        aligned), the other columns as classify_v4."""
        import torch
        n = t["flags"].numel()
        dev = t["flags"].device
        if out is None:
            out = {"verdict": torch.empty(n, dtype=torch.int32, device=dev),
                   "identity": torch.empty(n, dtype=torch.int32, device=dev),
                   "stage": torch.empty(n, dtype=torch.uint8, device=dev) if stage else None}
        tv = TuplesV6(*[t[k].data_ptr() for k in
                        ("saddr", "daddr", "dport", "proto", "flags", "len", "ep")])
        check(self.L.cgpu_classify_v6(self.h, C.byref(tv), n, _ptr(out["verdict"]),
                                      _ptr(out["identity"]), _ptr(out.get("stage")),
                                      _stream(stream)), "cgpu_classify_v6")
        return out

    def classify_v6_lb(self, t: dict, out: dict | None = None, stage: bool = True, stream=None):
        """classify_v6 with the egress service step of ipv6_l3_from_lxc first;
        t additionally holds "hash" (int32 view of skb->hash) or "sport"."""
        import torch
        n = t["flags"].numel()
        dev = t["flags"].device
        if out is None:
            out = {"verdict": torch.empty(n, dtype=torch.int32, device=dev),
                   "identity": torch.empty(n, dtype=torch.int32, device=dev),
                   "stage": torch.empty(n, dtype=torch.uint8, device=dev) if stage else None}
        tv = TuplesV6(*[t[k].data_ptr() for k in
                        ("saddr", "daddr", "dport", "proto", "flags", "len", "ep")])
        check(self.L.cgpu_classify_v6_lb(self.h, C.byref(tv), _ptr(t.get("sport")),
                                         _ptr(t.get("hash")), n, _ptr(out["verdict"]),
                                         _ptr(out["identity"]), _ptr(out.get("stage")),
                                         _stream(stream)), "cgpu_classify_v6_lb")
        return out

    def prefilter_v4(self, saddr, daddr, flags, out=None, stream=None):
        import torch
        n = flags.numel()
        if out is None:
            out = torch.empty(n, dtype=torch.uint8, device=flags.device)
        check(self.L.cgpu_prefilter_v4(self.h, _ptr(saddr), _ptr(daddr), _ptr(flags), n,
                                       _ptr(out), _stream(stream)), "cgpu_prefilter_v4")
        return out

    def prefilter_v6(self, saddr16, daddr16, flags, out=None, stream=None):
        import torch
        n = flags.numel()
        if out is None:
            out = torch.empty(n, dtype=torch.uint8, device=flags.device)
        check(self.L.cgpu_prefilter_v6(self.h, _ptr(saddr16), _ptr(daddr16), _ptr(flags), n,
                                       _ptr(out), _stream(stream)), "cgpu_prefilter_v6")
        return out

    # ---------------------------------------------------------- raw frames
    def lxc_update(self, ep: int, info) -> int:
        """info: a layouts.LXC_INFO record (lxc_config.h of endpoint ep)."""
        return check(self.L.cgpu_lxc_update(self.h, ep, _buf(info)), "cgpu_lxc_update")

    def lxc_delete(self, ep: int) -> int:
        return self.L.cgpu_lxc_delete(self.h, ep)

    def lxc_lookup(self, ep: int):
        out = np.zeros((), L.LXC_INFO)
        rc = self.L.cgpu_lxc_lookup(self.h, ep, out.ctypes.data_as(C.c_void_p))
        return None if rc == -errno.ENOENT else (check(rc, "cgpu_lxc_lookup"), out)[1]

    @staticmethod
    def _frames(f: dict) -> Frames:
        data = f["data"]
        assert data.dim() == 2 and data.is_contiguous()
        return Frames(data.data_ptr(), f["len"].data_ptr(), f["flags"].data_ptr(),
                      f["ep"].data_ptr(), data.shape[1], 0)

    def frames_parse(self, f: dict, out: dict | None = None, stream=None):
        """f: CUDA tensors data (n, stride) uint8, len int32, flags uint8,
        ep int16.  Returns the policy tuple columns (cgpu_frames_parse)."""
        import torch
        n = f["len"].numel()
        dev = f["len"].device
        if out is None:
            out = {"status": torch.empty(n, dtype=torch.int32, device=dev),
                   "family": torch.empty(n, dtype=torch.uint8, device=dev),
                   "saddr": torch.empty((n, 16), dtype=torch.uint8, device=dev),
                   "daddr": torch.empty((n, 16), dtype=torch.uint8, device=dev),
                   "dport": torch.empty(n, dtype=torch.int16, device=dev),
                   "proto": torch.empty(n, dtype=torch.uint8, device=dev),
                   "flags": torch.empty(n, dtype=torch.uint8, device=dev)}
        fr = self._frames(f)
        ot = FrameTuples(*[_ptr(out.get(k)) for k in ("status", "family", "saddr", "daddr",
                                                      "dport", "proto", "flags")])
        check(self.L.cgpu_frames_parse(self.h, C.byref(fr), n, C.byref(ot), _stream(stream)),
              "cgpu_frames_parse")
        return out

    def classify_frames(self, f: dict, out: dict | None = None, stage: bool = True, stream=None):
        """Raw frames to verdicts in one pass (cgpu_classify_frames)."""
        import torch
        n = f["len"].numel()
        dev = f["len"].device
        if out is None:
            out = {"verdict": torch.empty(n, dtype=torch.int32, device=dev),
                   "identity": torch.empty(n, dtype=torch.int32, device=dev),
                   "stage": torch.empty(n, dtype=torch.uint8, device=dev) if stage else None}
        fr = self._frames(f)
        check(self.L.cgpu_classify_frames(self.h, C.byref(fr), n, _ptr(out["verdict"]),
                                          _ptr(out["identity"]), _ptr(out.get("stage")),
                                          _stream(stream)), "cgpu_classify_frames")
        return out

    def classify_frames_host(self, f: dict, out: dict | None = None, stage: bool = True, stream=None):
        """cgpu_classify_frames_host: f holds HOST arrays (numpy, or CPU
        tensors -- page-locked ones are read by the CUs) data (n, stride)
        uint8, len, flags, ep; outputs are host arrays, complete when
        `stream` is (synchronized here unless out is given)."""
        import numpy as np
        n = len(f["len"])

        def ptr(x):
            if x is None:
                return None
            return x.data_ptr() if hasattr(x, "data_ptr") else x.ctypes.data
        data = f["data"]
        assert data.ndim == 2 if hasattr(data, "ndim") else data.dim() == 2
        given = out is not None
        if out is None:
            out = {"verdict": np.empty(n, np.int32), "identity": np.empty(n, np.uint32),
                   "stage": np.empty(n, np.uint8) if stage else None}
        fr = Frames(ptr(data), ptr(f["len"]), ptr(f["flags"]), ptr(f["ep"]), data.shape[1], 0)
        check(self.L.cgpu_classify_frames_host(self.h, C.byref(fr), n, C.c_void_p(ptr(out["verdict"])),
                                               C.c_void_p(ptr(out["identity"])),
                                               C.c_void_p(ptr(out.get("stage"))), _stream(stream)),
              "cgpu_classify_frames_host")
        if not given:
            import torch
            (stream or torch.cuda.current_stream()).synchronize()
        return out

    def host_stage_release(self) -> None:
        """cgpu_host_stage_release: free the host-batch device staging."""
        check(self.L.cgpu_host_stage_release(self.h), "cgpu_host_stage_release")

    def host_stage_bytes(self) -> int:
        """cgpu_host_stage_bytes: device bytes the host-batch staging holds."""
        return int(self.L.cgpu_host_stage_bytes(self.h))

    # ------------------------------------------------------------- counters
    def counter_delta_bytes(self) -> int:
        return self.L.cgpu_counter_delta_bytes(self.h)

    def counter_bind(self, tensor) -> None:
        """Accumulate launches into `tensor` (CUDA int64, >= delta bytes)."""
        if tensor is None:
            check(self.L.cgpu_counter_bind(self.h, None, 0), "cgpu_counter_bind")
        else:
            check(self.L.cgpu_counter_bind(self.h, _ptr(tensor),
                                           tensor.numel() * tensor.element_size()),
                  "cgpu_counter_bind")
        self._bound = tensor

    def counter_fold(self, stream=None) -> None:
        check(self.L.cgpu_counter_fold(self.h, _stream(stream)), "cgpu_counter_fold")

    def metrics(self) -> np.ndarray:
        out = np.zeros((256, 4, 2), np.uint64)
        check(self.L.cgpu_metrics_read(self.h, out.ctypes.data_as(C.c_void_p)),
              "cgpu_metrics_read")
        return out

    def counters_rebalance(self) -> int:
        """cgpu_counters_rebalance: hot (LDS) counter slots to the most-hit
        keys; returns how many keys moved."""
        m = C.c_uint64()
        check(self.L.cgpu_counters_rebalance(self.h, C.byref(m)), "cgpu_counters_rebalance")
        return m.value

    def stream_release(self, stream) -> None:
        """cgpu_stream_release: free the stream's packed counter buffer."""
        check(self.L.cgpu_stream_release(self.h, _stream(stream)), "cgpu_stream_release")

    def counters_reset(self) -> None:
        check(self.L.cgpu_counters_reset(self.h), "cgpu_counters_reset")

    # ------------------------------------------- multi-GPU
    @staticmethod
    def comm_id() -> bytes:
        """A fresh communicator id (rank 0 creates it and shares it)."""
        buf = C.create_string_buffer(128)
        check(lib().cgpu_comm_id_create(buf), "cgpu_comm_id_create")
        return buf.raw

    def comm_init(self, comm_id: bytes, nranks: int, rank: int) -> None:
        assert len(comm_id) == 128
        check(self.L.cgpu_comm_init(self.h, comm_id, nranks, rank), "cgpu_comm_init")

    def counters_allreduce(self, stream=None) -> None:
        """RCCL SUM of the delta buffer over the communicator's ranks."""
        check(self.L.cgpu_counters_allreduce(self.h, _stream(stream)), "cgpu_counters_allreduce")


# ---------------------------------------------------------------------------
# Go-API mirrors
# ---------------------------------------------------------------------------
class PolicyMap:
    """pkg/maps/policymap.PolicyMap over one endpoint's map (ports host order)."""

    def __init__(self, engine: Engine, ep: int):
        self.e, self.ep = engine, ep

    def Allow(self, identity, dport, proto, direction, proxy_port=0):  # noqa: N802
        rc = self.e.policy_update(self.ep, L.policy_key(identity, dport, proto, direction),
                                  L.policy_entry(proxy_port))
        check(rc, "PolicyMap.Allow")

    def AllowKey(self, key, proxy_port=0):  # noqa: N802 (key: host-order fields)
        self.Allow(int(key["sec_label"]), int(key["dport"]), int(key["protocol"]),
                   int(key["egress"]) & 1, proxy_port)

    def Exists(self, identity, dport, proto, direction) -> bool:  # noqa: N802
        rc, _ = self.e.policy_lookup(self.ep, L.policy_key(identity, dport, proto, direction))
        return rc == 0

    def Delete(self, identity, dport, proto, direction):  # noqa: N802
        check(self.e.policy_delete(self.ep, L.policy_key(identity, dport, proto, direction)),
              "PolicyMap.Delete")

    def DeleteKey(self, key):  # noqa: N802
        self.Delete(int(key["sec_label"]), int(key["dport"]), int(key["protocol"]),
                    int(key["egress"]) & 1)

    def DumpToSlice(self):  # noqa: N802
        out = []
        for k in self.e.policy_keys(self.ep):
            rc, ent = self.e.policy_lookup(self.ep, k)
            if rc == 0:
                out.append((k, ent))
        return out

    def Flush(self):  # noqa: N802
        check(self.e.policy_flush(self.ep), "PolicyMap.Flush")


class IPCacheMap:
    """pkg/maps/ipcache.Map + the ipcache listener hook."""

    def __init__(self, engine: Engine, supports_delete: bool = True):
        self.e = engine
        self.supports_delete = supports_delete

    def Update(self, cidr: str, identity: int, tunnel: int = 0):  # noqa: N802
        check(self.e.ipcache_update(L.ipcache_key(cidr), L.remote_info(identity, tunnel)),
              "ipcache.Update")

    def Delete(self, cidr: str):  # noqa: N802
        # pkg/maps/ipcache/ipcache.go:182-200: without delete support the
        # entry is overwritten with zeroes (a tombstone that still matches)
        if not self.supports_delete:
            return self.Update(cidr, 0, 0)
        check(self.e.ipcache_delete(L.ipcache_key(cidr)), "ipcache.Delete")

    # IPIdentityMappingListener.OnIPIdentityCacheChange (listener.go:78-127)
    def OnIPIdentityCacheChange(self, modType: str, cidr: str, identity: int,  # noqa: N802
                                hostIP: int = 0):
        if modType == "upsert":
            self.Update(cidr, identity, hostIP)
        elif modType == "delete":
            try:
                self.Delete(cidr)
            except CgpuError as ex:
                if ex.errno != errno.ENOENT:
                    raise


class CIDRMap:
    """pkg/maps/cidrmap.CIDRMap (prefilter maps)."""

    def __init__(self, engine: Engine, which: int):
        self.e, self.which = engine, which
        self.v6 = which in (CIDR_V6_DYN, CIDR_V6_FIX)
        self.prefixlen = 0 if which in (CIDR_V4_DYN, CIDR_V6_DYN) else (128 if self.v6 else 32)
        self.dynamic = which in (CIDR_V4_DYN, CIDR_V6_DYN)

    def _check(self, plen, op):
        # checkPrefixlen (cidrmap.go:75-83)
        if self.prefixlen != 0 and ((self.dynamic and self.prefixlen < plen) or
                                    (not self.dynamic and self.prefixlen != plen)):
            raise ValueError(f"Unable to {op} element with dynamic prefix length "
                             f"cm.Prefixlen={self.prefixlen} key.Prefixlen={plen}")

    def InsertCIDR(self, cidr: str):  # noqa: N802
        k = L.lpm_key(cidr)
        self._check(int(k["prefixlen"]), "update")
        check(self.e.cidr_update(self.which, k), "InsertCIDR")

    def DeleteCIDR(self, cidr: str):  # noqa: N802
        k = L.lpm_key(cidr)
        self._check(int(k["prefixlen"]), "delete")
        check(self.e.cidr_delete(self.which, k), "DeleteCIDR")

    def CIDRExists(self, cidr: str) -> bool:  # noqa: N802
        return self.e.cidr_lookup(self.which, L.lpm_key(cidr)) == 0

    def CIDRDump(self):  # noqa: N802
        out = []
        for k in self.e.cidr_keys(self.which):
            raw = bytes(k["addr"])
            addr = ipaddress.ip_address(raw)
            out.append(f"{addr}/{int(k['prefixlen'])}")
        return out


class PreFilter:
    """pkg/policy/prefilter.go PreFilter (Insert / Delete / Dump with the
    revision check, selectMap routing and undo), over cgpu_prefilter_*.
    CIDRs are strings; IPv4 ones go to the v4 maps (net.IPNet mask of 32
    bits), IPv6 ones to the v6 maps."""

    PREFIX = np.dtype([("bits", "<u4"), ("prefixlen", "<u4"), ("addr", "u1", (16,))])

    def __init__(self, engine: Engine):
        self.e = engine

    @classmethod
    def _prefixes(cls, cidrs):
        out = np.zeros(len(cidrs), cls.PREFIX)
        for i, c in enumerate(cidrs):
            net = ipaddress.ip_network(c, strict=False)
            raw = net.network_address.packed
            out[i]["bits"] = net.max_prefixlen
            out[i]["prefixlen"] = net.prefixlen
            out[i]["addr"][:len(raw)] = np.frombuffer(raw, np.uint8)
        return out

    def Insert(self, revision: int, cidrs):  # noqa: N802
        p = self._prefixes(cidrs)
        check(self.e.L.cgpu_prefilter_insert(self.e.h, revision, p.ctypes.data, len(p)),
              "PreFilter.Insert")

    def Delete(self, revision: int, cidrs):  # noqa: N802
        p = self._prefixes(cidrs)
        check(self.e.L.cgpu_prefilter_delete(self.e.h, revision, p.ctypes.data, len(p)),
              "PreFilter.Delete")

    def Revision(self) -> int:  # noqa: N802
        r = C.c_int64()
        check(self.e.L.cgpu_prefilter_revision(self.e.h, C.byref(r)), "PreFilter.Revision")
        return r.value

    def Dump(self):  # noqa: N802
        """(CIDR strings of the maps in prefilter.go order v4 dyn, v4 fix,
        v6 dyn, v6 fix; revision)"""
        out = []
        for which in (CIDR_V4_DYN, CIDR_V4_FIX, CIDR_V6_DYN, CIDR_V6_FIX):
            out += CIDRMap(self.e, which).CIDRDump()
        return out, self.Revision()


class LBMap:
    """pkg/maps/lbmap over cilium_lb4_services (IPv4): the frontend/backend
    writes of UpdateService (lbmap.go:350-428: backends at slaves 1..n, then
    the master slot 0 {count, weight}, then stale slaves removed) and
    DeleteService."""

    def __init__(self, engine: Engine):
        self.e = engine

    def UpdateService(self, vip: str, port: int, backends, rev_nat: int = 0):  # noqa: N802
        """backends: [(target, port, weight), ...] (ports host order)."""
        rc, old = self.e.lb4_lookup(L.lb4_key(vip, port, 0))
        existing = int(old["count"]) if rc == 0 else 0
        for i, (tgt, bport, w) in enumerate(backends):
            check(self.e.lb4_update(L.lb4_key(vip, port, i + 1),
                                    L.lb4_service(tgt, bport, 0, rev_nat, w)), "UpdateService")
        nonzero = sum(1 for b in backends if b[2])
        check(self.e.lb4_update(L.lb4_key(vip, port, 0),
                                L.lb4_service(0, 0, len(backends), 0, nonzero)), "UpdateService")
        for s in range(len(backends) + 1, existing + 1):
            self.e.lb4_delete(L.lb4_key(vip, port, s))

    def DeleteService(self, vip: str, port: int):  # noqa: N802
        rc, old = self.e.lb4_lookup(L.lb4_key(vip, port, 0))
        if rc != 0:
            raise CgpuError(errno.ENOENT, f"service {vip}:{port} not found")
        for s in range(int(old["count"]), -1, -1):
            self.e.lb4_delete(L.lb4_key(vip, port, s))

    def LookupService(self, vip: str, port: int):  # noqa: N802
        rc, master = self.e.lb4_lookup(L.lb4_key(vip, port, 0))
        if rc != 0:
            return None
        out = []
        for s in range(1, int(master["count"]) + 1):
            rc, be = self.e.lb4_lookup(L.lb4_key(vip, port, s))
            if rc == 0:
                out.append(be)
        return out

    def DumpServiceMapsToUserspace(self):  # noqa: N802
        return [(k, self.e.lb4_lookup(k)[1]) for k in self.e.lb4_keys()]
