"""ctypes prototypes of include/cgpu.h (the product's C ABI).

Loading fails loudly: there is no Python or CPU fallback for any entry point.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libcgpu.so")

CGPU_ABI_VERSION = 2


class CgpuConfig(C.Structure):
    _fields_ = [
        ("abi_version", C.c_uint32),
        ("ipcache_max", C.c_uint32), ("policy_max_per_ep", C.c_uint32),
        ("policy_max_total", C.c_uint32), ("max_endpoints", C.c_uint32),
        ("cidr_dyn_max", C.c_uint32), ("cidr_fix_max", C.c_uint32),
        ("endpoints_max", C.c_uint32),
        ("host_id", C.c_uint32), ("world_id", C.c_uint32), ("cluster_id", C.c_uint32),
        ("health_id", C.c_uint32),
        ("ipv4_cluster_mask", C.c_uint32), ("ipv4_cluster_range", C.c_uint32),
        ("ipv6_router_ip", C.c_uint8 * 16),
        ("ct_proto_gate", C.c_uint8), ("ingress_secctx_world", C.c_uint8),
        ("prefilter_fix4", C.c_uint8), ("prefilter_dyn4", C.c_uint8),
        ("prefilter_fix6", C.c_uint8), ("prefilter_dyn6", C.c_uint8),
        ("reserved0", C.c_uint8 * 2),
        ("ingress_src_identity", C.c_uint32),
        ("hot_counter_slots", C.c_uint32),
        ("lb_max_entries", C.c_uint32), ("ipv4_loopback", C.c_uint32),
        ("lb_flags", C.c_uint32),
        ("node_mac", C.c_uint8 * 6), ("reserved1", C.c_uint8 * 2),
        ("ct_max", C.c_uint32), ("schedule", C.c_uint32), ("ct6_max", C.c_uint32),
        ("ct_lru", C.c_uint32), ("reserved", C.c_uint32 * 1),
    ]


class TuplesV4(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in
                ("saddr", "daddr", "dport", "proto", "flags", "len", "ep")]


class TuplesV6(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in
                ("saddr", "daddr", "dport", "proto", "flags", "len", "ep")]


class TuplesV4Ct(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in
                ("saddr", "daddr", "sport", "dport", "proto", "l4", "flags", "len", "ep")]


class TuplesV6Ct(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in
                ("saddr", "daddr", "sport", "dport", "proto", "l4", "flags", "len", "ep")]


class Lb4Tuples(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("saddr", "daddr", "sport", "dport", "proto", "hash")]


class Lb4Out(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("ret", "saddr", "daddr", "dport", "rev_nat", "slave")]


class CtlbOut(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("verdict", "ct_ret", "identity", "stage", "daddr", "dport")]


class Frames(C.Structure):
    _fields_ = [("data", C.c_void_p), ("len", C.c_void_p), ("flags", C.c_void_p),
                ("ep", C.c_void_p), ("stride", C.c_uint32), ("reserved", C.c_uint32)]


class FrameTuples(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in
                ("status", "family", "saddr", "daddr", "dport", "proto", "flags")]


vp, sz, u32, u64, i32 = C.c_void_p, C.c_size_t, C.c_uint32, C.c_uint64, C.c_int

# name -> (restype, argtypes)
PROTOS = {
    "cgpu_config_default": (None, [C.POINTER(CgpuConfig)]),
    "cgpu_ctx_create": (i32, [C.POINTER(CgpuConfig), i32, C.POINTER(vp)]),
    "cgpu_ctx_destroy": (None, [vp]),
    "cgpu_last_error": (C.c_char_p, []),
    "cgpu_version": (C.c_char_p, []),
    "cgpu_ipcache_update": (i32, [vp, vp, vp, u64]),
    "cgpu_ipcache_delete": (i32, [vp, vp]),
    "cgpu_ipcache_lookup": (i32, [vp, vp, vp]),
    "cgpu_ipcache_get_next_key": (i32, [vp, vp, vp]),
    "cgpu_ipcache_count": (sz, [vp]),
    "cgpu_ipcache_update_batch": (i32, [vp, vp, vp, sz, u64]),
    "cgpu_policy_update": (i32, [vp, u32, vp, vp, u64]),
    "cgpu_policy_delete": (i32, [vp, u32, vp]),
    "cgpu_policy_lookup": (i32, [vp, u32, vp, vp]),
    "cgpu_policy_get_next_key": (i32, [vp, u32, vp, vp]),
    "cgpu_policy_flush": (i32, [vp, u32]),
    "cgpu_policy_count": (sz, [vp, u32]),
    "cgpu_policy_update_batch": (i32, [vp, vp, vp, vp, sz, u64]),
    "cgpu_policy_lookup_batch": (i32, [vp, vp, vp, sz, vp, vp]),
    "cgpu_policy_dump": (i32, [vp, u32, vp, vp, sz, C.POINTER(sz)]),
    "cgpu_cidr_update": (i32, [vp, i32, vp, u64]),
    "cgpu_cidr_delete": (i32, [vp, i32, vp]),
    "cgpu_cidr_lookup": (i32, [vp, i32, vp]),
    "cgpu_cidr_get_next_key": (i32, [vp, i32, vp, vp]),
    "cgpu_cidr_update_batch": (i32, [vp, i32, vp, sz, u64]),
    "cgpu_prefilter_insert": (i32, [vp, C.c_int64, vp, sz]),
    "cgpu_prefilter_delete": (i32, [vp, C.c_int64, vp, sz]),
    "cgpu_prefilter_revision": (i32, [vp, C.POINTER(C.c_int64)]),
    "cgpu_endpoint_update": (i32, [vp, vp, u64]),
    "cgpu_endpoint_delete": (i32, [vp, vp]),
    "cgpu_endpoint_lookup": (i32, [vp, vp]),
    "cgpu_lb4_update": (i32, [vp, vp, vp, u64]),
    "cgpu_lb4_update_batch": (i32, [vp, vp, vp, sz, u64]),
    "cgpu_lb4_delete": (i32, [vp, vp]),
    "cgpu_lb4_lookup": (i32, [vp, vp, vp]),
    "cgpu_lb4_get_next_key": (i32, [vp, vp, vp]),
    "cgpu_lb4_count": (sz, [vp]),
    "cgpu_lb6_update": (i32, [vp, vp, vp, u64]),
    "cgpu_lb6_update_batch": (i32, [vp, vp, vp, sz, u64]),
    "cgpu_lb6_delete": (i32, [vp, vp]),
    "cgpu_lb6_lookup": (i32, [vp, vp, vp]),
    "cgpu_lb6_get_next_key": (i32, [vp, vp, vp]),
    "cgpu_lb6_count": (sz, [vp]),
    "cgpu_flow_hash6": (u32, [vp, vp, C.c_uint16, C.c_uint16, C.c_uint8]),
    "cgpu_flow_hash": (u32, [u32, u32, C.c_uint16, C.c_uint16, C.c_uint8]),
    "cgpu_commit": (i32, [vp, C.POINTER(u64)]),
    "cgpu_table_checksum": (i32, [vp, C.POINTER(u64)]),
    "cgpu_table_verify": (i32, [vp]),
    "cgpu_mirror_save": (i32, [vp, C.c_char_p]),
    "cgpu_mirror_restore": (i32, [vp, C.c_char_p]),
    "cgpu__test_corrupt": (i32, [vp, i32, sz, C.c_uint8]),
    "cgpu_counter_layout_checksum": (i32, [vp, C.POINTER(u64)]),
    "cgpu_classify_v4": (i32, [vp, C.POINTER(TuplesV4), sz, vp, vp, vp, vp]),
    "cgpu_classify_v4_host": (i32, [vp, C.POINTER(TuplesV4), sz, vp, vp, vp, vp]),
    "cgpu_classify_v6": (i32, [vp, C.POINTER(TuplesV6), sz, vp, vp, vp, vp]),
    "cgpu_classify_v6_lb": (i32, [vp, C.POINTER(TuplesV6), vp, vp, sz, vp, vp, vp, vp]),
    "cgpu_classify_v4_lb": (i32, [vp, C.POINTER(TuplesV4), vp, vp, sz, vp, vp, vp, vp]),
    "cgpu_classify_v4_cascade": (i32, [vp, C.POINTER(TuplesV4), vp, vp, sz, vp, vp, vp, vp]),
    "cgpu_classify_v4_lb_host": (i32, [vp, C.POINTER(TuplesV4), vp, vp, sz, vp, vp, vp, vp]),
    "cgpu_classify_v4_cascade_host": (i32, [vp, C.POINTER(TuplesV4), vp, vp, sz, vp, vp, vp, vp]),
    "cgpu_classify_v6_host": (i32, [vp, C.POINTER(TuplesV6), sz, vp, vp, vp, vp]),
    "cgpu_classify_v6_lb_host": (i32, [vp, C.POINTER(TuplesV6), vp, vp, sz, vp, vp, vp, vp]),
    "cgpu_lb4_select": (i32, [vp, i32, C.POINTER(Lb4Tuples), sz, C.POINTER(Lb4Out), vp]),
    "cgpu_prefilter_v4": (i32, [vp, vp, vp, vp, sz, vp, vp]),
    "cgpu_prefilter_v6": (i32, [vp, vp, vp, vp, sz, vp, vp]),
    "cgpu_prefilter_v4_host": (i32, [vp, vp, vp, vp, sz, vp, vp]),
    "cgpu_prefilter_v6_host": (i32, [vp, vp, vp, vp, sz, vp, vp]),
    "cgpu_lxc_update": (i32, [vp, u32, vp]),
    "cgpu_lxc_delete": (i32, [vp, u32]),
    "cgpu_lxc_lookup": (i32, [vp, u32, vp]),
    "cgpu_frames_parse": (i32, [vp, C.POINTER(Frames), sz, C.POINTER(FrameTuples), vp]),
    "cgpu_classify_frames": (i32, [vp, C.POINTER(Frames), sz, vp, vp, vp, vp]),
    "cgpu_classify_frames_host": (i32, [vp, C.POINTER(Frames), sz, vp, vp, vp, vp]),
    "cgpu_ct4_update": (i32, [vp, vp, vp, u64]),
    "cgpu_ct4_delete": (i32, [vp, vp]),
    "cgpu_ct4_lookup": (i32, [vp, vp, vp]),
    "cgpu_ct4_get_next_key": (i32, [vp, vp, vp]),
    "cgpu_ct4_count": (sz, [vp]),
    "cgpu_ct4_gc": (i32, [vp, u32, C.POINTER(u64)]),
    "cgpu_ct_stats": (i32, [vp, C.c_int, vp]),
    "cgpu_ct4_flush": (i32, [vp]),
    "cgpu_classify_v4_ct": (i32, [vp, C.POINTER(TuplesV4Ct), sz, u32, vp, vp, vp, vp, vp]),
    "cgpu_classify_v4_ctlb": (i32, [vp, C.POINTER(TuplesV4Ct), vp, sz, u32, C.POINTER(CtlbOut), vp]),
    "cgpu_ct6_update": (i32, [vp, vp, vp, u64]),
    "cgpu_ct6_delete": (i32, [vp, vp]),
    "cgpu_ct6_lookup": (i32, [vp, vp, vp]),
    "cgpu_ct6_get_next_key": (i32, [vp, vp, vp]),
    "cgpu_ct6_count": (sz, [vp]),
    "cgpu_ct6_gc": (i32, [vp, u32, C.POINTER(u64)]),
    "cgpu_ct6_flush": (i32, [vp]),
    "cgpu_classify_v6_ctlb": (i32, [vp, C.POINTER(TuplesV6Ct), vp, sz, u32, C.POINTER(CtlbOut), vp]),
    "cgpu_classify_v6_ct": (i32, [vp, C.POINTER(TuplesV6Ct), sz, u32, vp, vp, vp, vp, vp]),
    "cgpu_l3_compile": (i32, [vp, vp, vp, vp, u32, vp]),
    "cgpu_mapstate_sync": (i32, [vp, vp, vp, vp, vp, vp]),
    "cgpu_counter_delta_bytes": (sz, [vp]),
    "cgpu_counter_bind": (i32, [vp, vp, sz]),
    "cgpu_counter_fold": (i32, [vp, vp]),
    "cgpu_metrics_read": (i32, [vp, vp]),
    "cgpu_counters_reset": (i32, [vp]),
    "cgpu_stream_release": (i32, [vp, vp]),
    "cgpu_host_stage_release": (i32, [vp]),
    "cgpu_table_bytes": (i32, [vp, vp]),
    "cgpu_host_stage_bytes": (sz, [vp]),
    "cgpu_counters_rebalance": (i32, [vp, C.POINTER(u64)]),
    "cgpu_comm_id_create": (i32, [vp]),
    "cgpu_comm_init": (i32, [vp, vp, i32, i32]),
    "cgpu_counters_allreduce": (i32, [vp, vp]),
}

_lib = None


class CgpuLibraryMissing(RuntimeError):
    pass


def lib():
    """Load libcgpu.so (built by cilium_amd.build / __graft_entry__.build)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise CgpuLibraryMissing(
                f"{LIB_PATH} is missing: build it with `python -m cilium_amd.build` "
                "(there is no CPU fallback for the classification path)")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in PROTOS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


class CgpuError(OSError):
    pass


def check(rc: int, what: str) -> int:
    if rc < 0:
        msg = lib().cgpu_last_error().decode(errors="replace")
        raise CgpuError(-rc, f"{what}: {os.strerror(-rc)} ({msg})")
    return rc
