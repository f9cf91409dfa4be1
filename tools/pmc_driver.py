"""Minimal driver for rocprofv3 PMC passes: one bench workload (CGPU_PMC_CONFIG =
gpu (config 2, default) / cascade (config 5) / pf6 (config 3) / v6 (IPv6
classify at config-2 size) / ct (conntrack)), one 64M-tuple
batch resident in HBM, 3 launches (classify variant from CGPU_CLASSIFY_VARIANT)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from cilium_amd import synth  # noqa: E402
from cilium_amd.engine import Engine  # noqa: E402

name = os.environ.get("CGPU_PMC_CONFIG", "gpu")
cfg = synth.CONFIGS["gpu" if name in ("pf6", "ct") else name]
n = int(os.environ.get("CGPU_PMC_TUPLES", cfg["n_tuples"]))
if name == "v6":
    T = synth.make_tables6(**cfg)
    t = synth.make_tuples6(T, n)
    e = Engine(device=0, **T.engine_config())
    synth.load_engine(e, T)
    e.commit()
    d = synth.to_device(t)
    out = {"verdict": torch.empty(n, dtype=torch.int32, device="cuda"),
           "identity": torch.empty(n, dtype=torch.int32, device="cuda"), "stage": None}
    for _ in range(3):
        e.classify_v6(d, out=out)
    torch.cuda.synchronize()
    print("ok", name, n)
    sys.exit(0)
if name == "ct":
    # bench.py --config ct: 64M packets of 2M connections from an empty map
    import numpy as np
    T = synth.make_tables(**cfg)
    t, _, seclabels = synth.make_ct_workload(T, n // 32, mean_pkts=32)
    n = min(n, len(t["saddr"]))
    t = {k: np.ascontiguousarray(v[:n]) for k, v in t.items()}
    ct_max = 1 << max(20, int(np.ceil(np.log2(2.5 * n / 32))))
    e = Engine(device=0, **T.engine_config(), ct_max=ct_max)
    synth.load_engine(e, T)
    synth.load_lxc(e, seclabels)
    e.commit()
    d = synth.to_device(t)
    out = {"verdict": torch.empty(n, dtype=torch.int32, device="cuda"),
           "identity": torch.empty(n, dtype=torch.int32, device="cuda"), "stage": None,
           "ct_ret": torch.empty(n, dtype=torch.uint8, device="cuda")}
    for _ in range(3):
        e.ct4_flush()
        e.classify_v4_ct(d, 1000, out=out)
    torch.cuda.synchronize()
    print("ok", name, n)
    sys.exit(0)
if name == "pf6":
    # config 3: the v6 prefilter sets of bench.py --config pf6
    P = synth.make_prefilter6(**synth.PF6_CONFIG)
    t = synth.make_packets6(P, n)
    e = Engine(device=0, **P.engine_config())
    synth.load_prefilter6(e, P)
    e.commit()
    d = synth.packets6_to_device(t, "cuda")
    v = torch.empty(n, dtype=torch.uint8, device="cuda")
    for _ in range(3):
        e.prefilter_v6(d["saddr"], d["daddr"], d["flags"], out=v)
else:
    T = synth.make_tables(**cfg)
    t = synth.make_tuples(T, n)
    ecfg = T.engine_config()
    S = None
    if name == "cascade":
        # config 5: bench.py --config cascade's services and traffic
        S = synth.make_services(T, cfg["n_services"])
        t = synth.add_service_traffic(t, S)
        del t["hash"]
        ecfg["lb_max_entries"] = len(S.keys)
    e = Engine(device=0, **ecfg)
    synth.load_engine(e, T)
    if S is not None:
        synth.load_services(e, S)
    e.commit()
    d = synth.to_device(t)
    out = {"verdict": torch.empty(n, dtype=torch.int32, device="cuda"),
           "identity": torch.empty(n, dtype=torch.int32, device="cuda"), "stage": None}
    # as bench.py: warm traffic, then the popularity rebalance of the
    # counter slots (cgpu_counters_rebalance), then the measured launches
    (e.classify_v4_lb if S is not None else e.classify_v4)(d, out=out)
    torch.cuda.synchronize()
    e.counter_fold()
    torch.cuda.synchronize()
    e.counters_rebalance()
    for _ in range(3):
        (e.classify_v4_lb if S is not None else e.classify_v4)(d, out=out)
torch.cuda.synchronize()
print("ok", name, n)
