"""Conntrack walker scan (diagnostic, not part of the product): the stateful
path over 64M packets at several packets-per-connection, one batch each from
an empty map, so a rocprofv3 kernel trace separates where the walk's time
goes: the per-connection slow path (probes, creates) against the per-packet
steps.  Run under rocprofv3 --kernel-trace; prints one line per workload
with the wall time of the call.

    python tools/ct_scan.py [pkts_per_conn ...]   (default 1 8 32 256)

CT_SCAN_DIAG=1: load tools/_diag/libcgpu_walk_clock.so (python tools/diag_ab.py
build walk_clock) and print the walk's per-wave timeline: when waves finish,
how many steps their busiest lane took.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from cilium_amd import synth  # noqa: E402
from cilium_amd.engine import Engine  # noqa: E402

DIAG = os.environ.get("CT_SCAN_DIAG") == "1"
if DIAG:
    import ctypes as C
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import diag_ab  # noqa: E402
    diag_ab.load("walk_clock")
    from cilium_amd import _abi  # noqa: E402


def walk_timeline():
    buf = (C.c_ulonglong * (4 * 8192))()
    assert _abi._lib.cgpu_diag_walk_clock(buf, 4 * 8192) == 0
    a = np.frombuffer(buf, np.uint64).reshape(-1, 4).astype(np.float64)
    a = a[a[:, 1] > 0]
    t0 = a[:, 0].min()
    dur = (a[:, 1] - t0) / 100.0  # us since the first wave started
    st = (a[:, 0] - t0) / 100.0
    q = np.percentile(dur, [10, 50, 90, 99, 100])
    mx = a[:, 2]
    top = np.argsort(dur)[-3:]
    print(f"  waves {len(a)}: start max {st.max():.0f} us; end p10/50/90/99/max "
          f"{' / '.join(f'{x:.0f}' for x in q)} us; busiest-lane steps p50 {np.median(mx):.0f} max "
          f"{mx.max():.0f}; lane steps total {a[:, 3].sum():.0f}; us per step of the 3 last waves "
          f"{' '.join(f'{(a[i, 1] - a[i, 0]) / 100.0 / max(a[i, 2], 1):.2f}' for i in top)}", flush=True)

n = int(os.environ.get("CT_SCAN_PACKETS", 1 << 26))
ppc = [float(x) for x in sys.argv[1:]] or [1.0, 8.0, 32.0, 256.0]
T = synth.make_tables(**synth.CONFIGS["gpu"])
for m in ppc:
    t, _, seclabels = synth.make_ct_workload(T, int(n / m) + 1, mean_pkts=m)
    k = min(n, len(t["saddr"]))
    t = {a: np.ascontiguousarray(v[:k]) for a, v in t.items()}
    ct_max = 1 << max(20, int(np.ceil(np.log2(2.5 * k / m))))
    e = Engine(device=0, **T.engine_config(), ct_max=ct_max)
    synth.load_engine(e, T)
    synth.load_lxc(e, seclabels)
    e.commit()
    d = synth.to_device(t)
    out = e.classify_v4_ct(d, 1000)  # warm (allocations, code objects)
    torch.cuda.synchronize()
    e.ct4_flush()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = e.classify_v4_ct(d, 1000, out=out)
    torch.cuda.synchronize()
    ms = 1e3 * (time.perf_counter() - t0)
    print(f"pkts_per_conn {m:g}: {k} packets, {ms:.2f} ms, {k / ms / 1e3:.1f} Mpps, "
          f"{e.ct4_count()} entries", flush=True)
    if DIAG:
        walk_timeline()
    e.close()
    del d, out
    torch.cuda.empty_cache()
