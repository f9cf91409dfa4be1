"""Where the host-resident line (bench.py --host-tuples) loses time against
the link: the copy pattern of cgpu_classify_v4_host timed piece by piece
(torch copies on side streams, no classify) beside the real call.

  python tools/hs_probe.py [--n 67108864] [--chunk 4194304]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

EL = {"saddr": 4, "daddr": 4, "dport": 2, "proto": 1, "flags": 1, "len": 4, "ep": 2}


def timed(fn, reps=3):
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 26)
    ap.add_argument("--chunk", type=int, default=1 << 22)
    args = ap.parse_args()
    n, ch = args.n, args.chunk
    dev = torch.device("cuda:0")
    hcol = {k: torch.empty(n * e, dtype=torch.uint8).pin_memory() for k, e in EL.items()}
    hout = [torch.empty(n * 4, dtype=torch.uint8).pin_memory() for _ in range(2)]
    dst = [{k: torch.empty(ch * e, dtype=torch.uint8, device=dev) for k, e in EL.items()} for _ in range(2)]
    dout = [[torch.empty(ch * 4, dtype=torch.uint8, device=dev) for _ in range(2)] for _ in range(2)]
    h2d, d2h = torch.cuda.Stream(), torch.cuda.Stream()
    res = {"n": n, "chunk": ch, "h2d_bytes": 18 * n, "d2h_bytes": 8 * n,
           "env": {k: os.environ.get(k) for k in ("HSA_ENABLE_SDMA", "HIP_FORCE_DEV_KERNARG") if os.environ.get(k)}}

    def up():
        with torch.cuda.stream(h2d):
            for k0 in range(0, n, ch):
                b = (k0 // ch) & 1
                for k, e in EL.items():
                    dst[b][k].copy_(hcol[k][k0 * e:(k0 + ch) * e], non_blocking=True)

    def down():
        with torch.cuda.stream(d2h):
            for k0 in range(0, n, ch):
                b = (k0 // ch) & 1
                for j in range(2):
                    hout[j][k0 * 4:(k0 + ch) * 4].copy_(dout[b][j], non_blocking=True)

    def both():
        up()
        down()

    big = torch.empty(18 * ch, dtype=torch.uint8, device=dev)
    hbig = torch.empty(18 * n, dtype=torch.uint8).pin_memory()

    def up_packed():
        with torch.cuda.stream(h2d):
            for k0 in range(0, n, ch):
                big.copy_(hbig[k0 * 18:(k0 + ch) * 18], non_blocking=True)

    def up_whole():
        with torch.cuda.stream(h2d):
            big2 = torch.empty(18 * n, dtype=torch.uint8, device=dev)
            big2.copy_(hbig, non_blocking=True)

    for name, fn in (("h2d_columns", up), ("d2h_columns", down), ("h2d_and_d2h", both),
                     ("h2d_packed_chunks", up_packed), ("h2d_one_copy", up_whole)):
        fn()  # warm
        res[name + "_ms"] = round(timed(fn), 3)

    cs = torch.cuda.Stream()
    dv = [torch.empty(ch, dtype=torch.int32, device=dev) for _ in range(2)]
    ev_in = [torch.cuda.Event() for _ in range(2)]
    ev_cls = [torch.cuda.Event() for _ in range(2)]
    ev_out = [torch.cuda.Event() for _ in range(2)]

    def mimic(d2h_on_cs=False):
        """the cgpu_classify_v4_host schedule with a stand-in kernel for the
        classify (reads saddr, writes both outputs)"""
        nch = n // ch

        def upload(k):
            b = k & 1
            if k >= 2:
                h2d.wait_event(ev_cls[b])
            with torch.cuda.stream(h2d):
                for kk, e in EL.items():
                    dst[b][kk].copy_(hcol[kk][k * ch * e:(k + 1) * ch * e], non_blocking=True)
                ev_in[b].record(h2d)
        upload(0)
        for k in range(nch):
            if k + 1 < nch:
                upload(k + 1)
            b = k & 1
            cs.wait_event(ev_in[b])
            if k >= 2:
                cs.wait_event(ev_out[b])
            with torch.cuda.stream(cs):
                torch.add(dst[b]["saddr"].view(torch.int32), 1, out=dv[b])
                dout[b][0].view(torch.int32).copy_(dv[b])
                dout[b][1].view(torch.int32).copy_(dv[b])
                ev_cls[b].record(cs)
            q = cs if d2h_on_cs else d2h
            if not d2h_on_cs:
                d2h.wait_event(ev_cls[b])
            with torch.cuda.stream(q):
                for j in range(2):
                    hout[j][k * ch * 4:(k + 1) * ch * 4].copy_(dout[b][j], non_blocking=True)
                ev_out[b].record(q)
        torch.cuda.current_stream().wait_event(ev_out[0])
        torch.cuda.current_stream().wait_event(ev_out[1])

    for name, fn in (("mimic", mimic), ("mimic_d2h_on_cs", lambda: mimic(True))):
        fn()
        res[name + "_ms"] = round(timed(fn), 3)
    res["h2d_columns_gbs"] = round(18 * n / res["h2d_columns_ms"] / 1e6, 2)
    res["d2h_columns_gbs"] = round(8 * n / res["d2h_columns_ms"] / 1e6, 2)
    res["h2d_one_copy_gbs"] = round(18 * n / res["h2d_one_copy_ms"] / 1e6, 2)

    # host-side cost of queueing the uploads: torch copies and hipMemcpyAsync
    # straight from the runtime on the same page-locked columns
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]

    class Attr(ctypes.Structure):
        _fields_ = [("type", ctypes.c_int), ("device", ctypes.c_int), ("devicePointer", ctypes.c_void_p),
                    ("hostPointer", ctypes.c_void_p), ("isManaged", ctypes.c_int), ("flags", ctypes.c_uint)]
    at = Attr()
    rc = hip.hipPointerGetAttributes(ctypes.byref(at), ctypes.c_void_p(hcol["saddr"].data_ptr()))
    res["pinned_attr"] = {"rc": rc, "type": at.type, "flags": at.flags, "dev_ptr_eq_host": at.devicePointer == hcol["saddr"].data_ptr()}

    def enqueue(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        return round((t1 - t0) * 1e3, 3), round((time.perf_counter() - t0) * 1e3, 3)
    res["enqueue_torch_ms"] = enqueue(up)
    sh = h2d.cuda_stream

    def up_hip():
        for k0 in range(0, n, ch):
            b = (k0 // ch) & 1
            for k, e in EL.items():
                hip.hipMemcpyAsync(ctypes.c_void_p(dst[b][k].data_ptr()), ctypes.c_void_p(hcol[k].data_ptr() + k0 * e),
                                   ch * e, 1, ctypes.c_void_p(sh))
    res["enqueue_hip_ms"] = enqueue(up_hip)
    from bench import numa_nodes, gpu_numa_node
    res["numa"] = {"gpu": gpu_numa_node(torch, dev), "inputs": numa_nodes(hcol["saddr"]),
                   "out0": numa_nodes(hout[0]), "out1": numa_nodes(hout[1])}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
