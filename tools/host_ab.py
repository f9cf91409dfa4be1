"""Timing-only A/B of the host-resident path (cgpu_classify_v4_host /
cgpu_classify_frames_host) across diagnostic builds of the library
(tools/diag_ab.py variants, same semantics, other staging parameters).

    python tools/host_ab.py [tuples|frames|v6|pf6] variant ...    (GPU box)

Each variant: config-2 tables, the 64M-tuple batch (or its 64-byte frames)
in page-locked host memory, outputs into page-locked memory, 2 warmup calls
and 8 timed ones on one stream."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import diag_ab  # noqa: E402
from cilium_amd import synth  # noqa: E402


def main():
    kind = sys.argv[1]
    names = sys.argv[2:]
    if kind in ("v6", "pf6"):
        return main6(kind, names)
    T = synth.make_tables(**synth.CONFIGS["gpu"])
    n = synth.CONFIGS["gpu"]["n_tuples"]
    tup = synth.make_tuples(T, n)
    view = {np.uint32: np.int32, np.uint16: np.int16, np.uint8: np.uint8}
    if kind == "frames":
        fr = synth.frames_from_tuples(tup, stride=64)
        d = {"data": torch.from_numpy(np.ascontiguousarray(fr["data"])).pin_memory(),
             "len": torch.from_numpy(np.ascontiguousarray(fr["len"], np.uint32).view(np.int32)).pin_memory(),
             "flags": torch.from_numpy(np.ascontiguousarray(fr["flags"], np.uint8)).pin_memory(),
             "ep": torch.from_numpy(np.ascontiguousarray(fr["ep"], np.uint16).view(np.int16)).pin_memory()}
    else:
        d = {k: torch.from_numpy(np.ascontiguousarray(tup[k], dt).view(view[dt])).pin_memory()
             for k, dt in synth.TUPLE_DTYPES.items() if k in tup}
    out = {"verdict": torch.empty(n, dtype=torch.int32).pin_memory(),
           "identity": torch.empty(n, dtype=torch.int32).pin_memory(), "stage": None}
    for name in names:
        diag_ab.load(name)
        from cilium_amd.engine import Engine
        e = Engine(device=0, **T.engine_config())
        synth.load_engine(e, T)
        e.commit()
        st = torch.cuda.current_stream()
        run = (lambda: e.classify_frames_host(d, out=out, stream=st)) if kind == "frames" else \
              (lambda: e.classify_v4_host(d, out=out, stream=st))
        for _ in range(2):
            run()
        torch.cuda.synchronize()
        ts = []
        for _ in range(8):
            t0 = time.perf_counter()
            run()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        ms = 1e3 * float(np.median(ts))
        print(json.dumps({"variant": name, "kind": kind, "median_ms": round(ms, 3),
                          "gpps": round(n / ms / 1e6, 3)}), flush=True)
        e.host_stage_release()
        e.close()


def _time(name, kind, n, run):
    for _ in range(2):
        run()
    torch.cuda.synchronize()
    ts = []
    for _ in range(8):
        t0 = time.perf_counter()
        run()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ms = 1e3 * float(np.median(ts))
    print(json.dumps({"variant": name, "kind": kind, "median_ms": round(ms, 3),
                      "gpps": round(n / ms / 1e6, 3)}), flush=True)


def main6(kind, names):
    """v6: cgpu_classify_v6_host over bench.py --config v6's batch; pf6:
    cgpu_prefilter_v6_host over --config pf6's packets"""
    n = synth.CONFIGS["gpu"]["n_tuples"]
    if kind == "v6":
        T = synth.make_tables6(**synth.CONFIGS["v6"])
        tup = synth.make_tuples6(T, n)
        cfg = T.engine_config()
    else:
        P = synth.make_prefilter6(**synth.PF6_CONFIG)
        tup = synth.make_packets6(P, n)
        cfg = P.engine_config()
    view = {np.uint32: np.int32, np.uint16: np.int16, np.uint8: np.uint8}
    d = {k: torch.from_numpy(np.ascontiguousarray(v).view(view[v.dtype.type])).pin_memory()
         for k, v in tup.items()}
    out = {"verdict": torch.empty(n, dtype=torch.int32).pin_memory(),
           "identity": torch.empty(n, dtype=torch.int32).pin_memory(), "stage": None}
    vb = torch.empty(n, dtype=torch.uint8).pin_memory()
    for name in names:
        diag_ab.load(name)
        from cilium_amd.engine import Engine
        e = Engine(device=0, **cfg)
        if kind == "v6":
            synth.load_engine(e, T)
        else:
            synth.load_prefilter6(e, P)
        e.commit()
        st = torch.cuda.current_stream()
        run = (lambda: e.classify_v6_host(d, out=out, stream=st)) if kind == "v6" else \
              (lambda: e.prefilter_host(d["saddr"], d["daddr"], d["flags"], v6=True, out=vb, stream=st))
        _time(name, kind, n, run)
        e.host_stage_release()
        e.close()


if __name__ == "__main__":
    main()
