"""Timing-only A/B of diagnostic builds of the classify kernel (never the
product library: these builds drop work and give wrong counters).

    python tools/diag_ab.py build            # in the dev container: tools/_diag/*.so
    python tools/diag_ab.py run [variants]   # on the GPU box
    (CGPU_AB_CONFIG = gpu (config 2, default) / pf6 (config 3) / v6 / ct / ct6 / ctlb / ctlb6)

Each variant is cilium_amd/csrc compiled with extra -D flags into
tools/_diag/libcgpu_<name>.so; `run` loads each in turn into the Engine
(cilium_amd._abi's loader is pointed at it), commits the workload's tables and
times 10 launches of its 64M-tuple batch with HIP events.""" 
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
DIAG = os.path.join(ROOT, "tools", "_diag")
VARIANTS = {"product": (), "no_cold_atomics": ("CGPU_DIAG_NO_COLD",),
            "nc_p1_l2": ("CGPU_DIAG_NO_COLD", "CGPU_DIAG_P1_SMALL"),
            "nc_p2_l2": ("CGPU_DIAG_NO_COLD", "CGPU_DIAG_P2_SMALL"),
            "nc_lpm_l2": ("CGPU_DIAG_NO_COLD", "CGPU_DIAG_LPM_SMALL"),
            "nc_all_l2": ("CGPU_DIAG_NO_COLD", "CGPU_DIAG_P1_SMALL", "CGPU_DIAG_P2_SMALL",
                          "CGPU_DIAG_LPM_SMALL"),
            "one_wg_per_cu": ("CGPU_DIAG_LDS_PAD=65536",),
            "store_sc1": ("CGPU_DIAG_STORE_SC1",),
            "pf6_no_node": ("CGPU_DIAG_PF6_NO_NODE",), "pf6_no_ep": ("CGPU_DIAG_PF6_NO_EP",),
            "pf6_no_cover": ("CGPU_DIAG_PF6_NO_COVER",),
            "pf6_prefetch": ("CGPU_DIAG_PF6_PREFETCH",),
            "pf6_q4": ("CGPU_DIAG_PF6_Q=4",),
            "pf6_q2": ("CGPU_DIAG_PF6_Q=2",),
            "pf6_q2_prefetch": ("CGPU_DIAG_PF6_Q=2", "CGPU_DIAG_PF6_PREFETCH"),
            "ct_coherent_probe": ("CGPU_DIAG_CT_COHERENT_PROBE",),
            "walk_clock": ("CGPU_DIAG_WALK_CLOCK",),
            "v6_q3": ("CGPU_DIAG_V6_Q=3",), "v6_q4": ("CGPU_DIAG_V6_Q=4",),
            "v6_no_trie": ("CGPU_DIAG_V6_NO_TRIE",), "v6_l64": ("CGPU_V6T_NB=7",),
            "v6_l64_q3": ("CGPU_V6T_NB=7", "CGPU_DIAG_V6_Q=3"),
            "v6_pre_q1": ("CGPU_DIAG_IPC6_PRE_Q=1",), "v6_pre_q4": ("CGPU_DIAG_IPC6_PRE_Q=4",),
            "ct_prefetch": ("CGPU_CT_PREFETCH",),
            "ctc3": ("CTC=3",), "ctc2": ("CTC=2",),
            "v6_no_h64": ("CGPU_DIAG_V6_NO_H64",), "v6_pre_w2": ("CGPU_IPC6_MINW=2",), "v6_pre_q1_w2": ("CGPU_IPC6_MINW=2", "CGPU_DIAG_IPC6_PRE_Q=1"),
            "v6_pre_q4_w2": ("CGPU_IPC6_MINW=2", "CGPU_DIAG_IPC6_PRE_Q=4"), "ct_q2": ("CGPU_CT_Q=2",), "ct_q1": ("CGPU_CT_Q=1",),
            "policy_probes": ("CGPU_POLICY_Q_PROBES=1",), "walk_svc_minb1": ("CGPU_WALK_MINB_SVC=1",),
            "svc_decq": ("CGPU_CT_SVC_DECQ=1",), "svc_decq6": ("CGPU_CT_SVC_DECQ6=1",),
            "walk_w4": ("CGPU_WALK_W=4",), "walk_w3": ("CGPU_WALK_W=3",),
            "cc_probe2": ("CC_PROBE=2",), "cc_probe4": ("CC_PROBE=4",),
            "owed_by_pair": ("CGPU_OWED_BY_KEY=0",), "ct_len_sort": ("CGPU_CT_LH=0",),
            "v6_full_line": ("CGPU_V6T_FULL_LINE=1",),
            "hs_g256": ("CGPU_HS_COPY_G=256",), "hs_g512": ("CGPU_HS_COPY_G=512",),
            "hs_g64": ("CGPU_HS_COPY_G=64",), "hs_chunk23": ("CGPU_HS_CHUNK_LOG2=23",),
            "hs_chunk21": ("CGPU_HS_CHUNK_LOG2=21",), "hs_chunk24": ("CGPU_HS_CHUNK_LOG2=24",),
            "ct_noret": ("CGPU_DIAG_NO_RET",), "ret_default": ("CGPU_DIAG_RET_DEFAULT",),
            "ct_ret_small": ("CGPU_DIAG_RET_SMALL",), "ct_ret_nt": ("CGPU_DIAG_RET_NT",),
            "walk_grid1024": ("CT_WALK_GRID=1024",), "walk_grid2048": ("CT_WALK_GRID=2048",), "walk_grid4096": ("CT_WALK_GRID=4096",),
            "walk_grid8192": ("CT_WALK_GRID=8192",), "retb32": ("CT_RETB=32",),
            "g4096_retb32": ("CT_WALK_GRID=4096", "CT_RETB=32"), "g8192_retb32": ("CT_WALK_GRID=8192", "CT_RETB=32"),
            "walk_grid16384": ("CT_WALK_GRID=16384",), "walk_grid32768": ("CT_WALK_GRID=32768",),
            "ff_nostage": ("CGPU_FF_STAGE=0",), "ff_pool0": ("CGPU_FF_POOL=0",), "ff_pool8": ("CGPU_FF_POOL=8",),
            "ff_pool2": ("CGPU_FF_POOL=2",), "fin_q2": ("CGPU_CT_FQ=2",), "fin_q3": ("CGPU_CT_FQ=3",), "fin_q4": ("CGPU_CT_FQ=4",),
            "prep_q3": ("CGPU_CT_Q=3",), "prep_q2": ("CGPU_CT_Q=2",),
            "fin_nt512": ("CGPU_CT_FNT=512",), "fin_q3_nt512": ("CGPU_CT_FQ=3", "CGPU_CT_FNT=512"),
            "fin_q2_nt512": ("CGPU_CT_FQ=2", "CGPU_CT_FNT=512"), "walk_svc_minb3": ("CGPU_WALK_MINB_SVC=3",),
            "ct_create_noloop": ("CGPU_CT_CREATE_LOOP=0",),
            "svc_q1": ("CGPU_CT_SVC_Q=1",), "svc_q2": ("CGPU_CT_SVC_Q=2",), "svc_q4": ("CGPU_CT_SVC_Q=4",),
            "svc_pre6_off": ("CGPU_CT_SVC_PRE6=0",), "ff_h1": ("CGPU_FF_H=1",), "ff_h4": ("CGPU_FF_H=4",),
            # policy table slots per key (hopscotch, round 6): 2 = 2 MiB at config 2
            # (the product), 4 = 4 MiB, 8 = 8 MiB (round 5's footprint)
            "pol_spk4": ("CGPU_POL_SLOTS_PER_KEY=4",), "pol_spk8": ("CGPU_POL_SLOTS_PER_KEY=8",),
            "pol_spk2": ("CGPU_POL_SLOTS_PER_KEY=2",),
            # the v6 pre-pass: addresses behind the direction flag (round 5's form)
            "v6_pre_nospec": ("CGPU_IPC6_SPEC=0",),
            "v6_pre_q3": ("CGPU_DIAG_IPC6_PRE_Q=3",), "v6_pre_q4b": ("CGPU_DIAG_IPC6_PRE_Q=4",),
            # LB frontend slots per frontend (hopscotch, round 6): 2 = 32 MiB at config 5
            "lb_fe4": ("CGPU_LB_SLOTS_PER_FE=4",), "lb_fe8": ("CGPU_LB_SLOTS_PER_FE=8",),
            "lb_fe16": ("CGPU_LB_SLOTS_PER_FE=16",),
            # the cascade kernel's tuples per lane (product 2, r6_l; sep_q2 was
            # the same define on the stages-apart source)
            "xdp_q4": ("CGPU_XDP_Q=4",), "no_defer_cold": ("CGPU_X4_DEFER_COLD=0",), "no_ct_dflt": ("CGPU_CT_DFLT=0",),
            # (group-default conntrack results, the walker storing only the
            # results that differ from its group's orientation default and the
            # finish resolving the rest from a 2-MiB bitmap: ct 10.95 -> 10.73
            # ms, r6_p; the source change is r6_p/ct_dflt_experiment.patch)
            # (the v6 pre-pass's entry stores deferred the same way measured
            # 2.659 -> 2.650 ms, r6_o: not kept)
            # (round 6 also measured the deferral on the two-tuples-per-lane
            # cascade kernel, 2.931 -> 2.921 ms, and on the fused frames
            # kernel, 2.46 -> 2.72 ms with spills: r6_n; neither kept)
            # host staging uploads by the CUs for every batch (product: DMA
            # below 64-B columns; r6_m measured DMA both ways as hs_up_dma)
            "hs_up_cu": ("CGPU_HS_UP_DMA_BELOW=0",),
            # conntrack walker: records in flight ahead (product 2; the
            # generic ring measured 11.44-11.51 ms against 11.09, r6_k; the
            # macro left the tree with the result)
            }


def build(names):
    from cilium_amd import build as b
    os.makedirs(DIAG, exist_ok=True)
    for n in names:
        if n != "product":
            b.build(force=True, defines=VARIANTS[n], out=os.path.join(DIAG, f"libcgpu_{n}.so"))


def load(name):
    from cilium_amd import _abi
    path = _abi.LIB_PATH if name == "product" else os.path.join(DIAG, f"libcgpu_{name}.so")
    L = C.CDLL(path)
    for fn, (res, args) in _abi.PROTOS.items():
        f = getattr(L, fn, None)  # a diag build may predate newer entry points
        if f is not None:
            f.restype, f.argtypes = res, args
    _abi._lib = L


def _workload(conf):
    """(engine factory, launch fn, n) for CGPU_AB_CONFIG = gpu / pf6 / v6."""
    import torch
    from cilium_amd import synth
    from cilium_amd.engine import Engine
    if conf == "pf6":
        P = synth.make_prefilter6(**synth.PF6_CONFIG)
        n = synth.CONFIGS["gpu"]["n_tuples"]
        d = synth.packets6_to_device(synth.make_packets6(P, n), "cuda")
        v = torch.empty(n, dtype=torch.uint8, device="cuda")

        def make():
            e = Engine(device=0, **P.engine_config())
            synth.load_prefilter6(e, P)
            return e
        return make, lambda e: e.prefilter_v6(d["saddr"], d["daddr"], d["flags"], out=v), n
    if conf in ("ct", "ct6"):
        # bench.py --config ct / ct6: 64M packets of 2M connections, every
        # launch from an empty map (flush + classify, as a bench step)
        import numpy as np
        v6 = conf == "ct6"
        T = (synth.make_tables6 if v6 else synth.make_tables)(**synth.CONFIGS["v6" if v6 else "gpu"])
        n = synth.CONFIGS["v6" if v6 else "gpu"]["n_tuples"]
        tup, _, seclabels = (synth.make_ct6_workload if v6 else synth.make_ct_workload)(T, n // 32, mean_pkts=32)
        n = min(n, len(tup["saddr"]))
        tup = {k: np.ascontiguousarray(v[:n]) for k, v in tup.items()}
        ct_max = 1 << max(20, int(np.ceil(np.log2(2.5 * n / 32))))
        d = synth.to_device(tup)
        out = {"verdict": torch.empty(n, dtype=torch.int32, device="cuda"),
               "identity": torch.empty(n, dtype=torch.int32, device="cuda"), "stage": None,
               "ct_ret": torch.empty(n, dtype=torch.uint8, device="cuda")}

        def make():
            cfg = T.engine_config()
            if os.environ.get("CGPU_AB_HOT"):
                cfg["hot_counter_slots"] = int(os.environ["CGPU_AB_HOT"])
            e = Engine(device=0, **cfg, ct_max=ct_max)
            synth.load_engine(e, T)
            synth.load_lxc(e, seclabels)
            return e

        def step(e):
            if v6:
                e.ct6_flush()
                e.classify_v6_ct(d, 1000, out=out)
            else:
                e.ct4_flush()
                e.classify_v4_ct(d, 1000, out=out)
        return make, step, n
    if conf == "ctlb6":
        # bench.py --config ctlb6
        import numpy as np
        T = synth.make_tables6(**synth.CONFIGS["v6"])
        S = synth.make_services6(T, 100_000)
        n = synth.CONFIGS["v6"]["n_tuples"]
        tup, _, seclabels, S = synth.make_ctlb6_workload(T, S, n // 32, mean_pkts=32, loop_frac=1e-4)
        n = min(n, len(tup["saddr"]))
        tup = {k: np.ascontiguousarray(v[:n]) for k, v in tup.items()}
        ct_max = 1 << max(20, int(np.ceil(np.log2(4.5 * n / 32))))
        d = synth.to_device(tup)
        out = {"verdict": torch.empty(n, dtype=torch.int32, device="cuda"),
               "identity": torch.empty(n, dtype=torch.int32, device="cuda"), "stage": None,
               "ct_ret": torch.empty(n, dtype=torch.uint8, device="cuda"),
               "daddr": torch.empty((n, 16), dtype=torch.uint8, device="cuda"),
               "dport": torch.empty(n, dtype=torch.int16, device="cuda")}

        def make():
            e = Engine(device=0, **T.engine_config(), lb_max_entries=len(S.keys), ct_max=ct_max)
            synth.load_engine(e, T)
            synth.load_lxc(e, seclabels)
            synth.load_services6(e, S)
            return e

        def step(e):
            e.ct6_flush()
            e.classify_v6_ctlb(d, 1000, out=out)
        return make, step, n
    if conf == "ctlb":
        # bench.py --config ctlb: 64M packets behind the service step, every
        # launch from an empty map
        import numpy as np
        T = synth.make_tables(**synth.CONFIGS["gpu"])
        S = synth.make_services(T, synth.CONFIGS["cascade"]["n_services"])
        n = synth.CONFIGS["gpu"]["n_tuples"]
        tup, _, seclabels, S = synth.make_ctlb_workload(T, S, n // 32, mean_pkts=32, loop_frac=1e-4)
        n = min(n, len(tup["saddr"]))
        tup = {k: np.ascontiguousarray(v[:n]) for k, v in tup.items()}
        ct_max = 1 << max(20, int(np.ceil(np.log2(4.5 * n / 32))))
        d = synth.to_device(tup)
        out = {"verdict": torch.empty(n, dtype=torch.int32, device="cuda"),
               "identity": torch.empty(n, dtype=torch.int32, device="cuda"), "stage": None,
               "ct_ret": torch.empty(n, dtype=torch.uint8, device="cuda"),
               "daddr": torch.empty(n, dtype=torch.int32, device="cuda"),
               "dport": torch.empty(n, dtype=torch.int16, device="cuda")}

        def make():
            e = Engine(device=0, **T.engine_config(), lb_max_entries=len(S.keys), ct_max=ct_max)
            synth.load_engine(e, T)
            synth.load_lxc(e, seclabels)
            synth.load_services(e, S)
            return e

        def step(e):
            e.ct4_flush()
            e.classify_v4_ctlb(d, 1000, out=out)
        return make, step, n
    if conf == "cascade":
        # bench.py --config cascade: config 5 whole (XDP prefilter | 1M services)
        cfg = synth.CONFIGS["cascade"]
        T = synth.make_tables(**cfg)
        S = synth.make_services(T, cfg["n_services"])
        P = synth.make_prefilter4(T)
        n = cfg["n_tuples"]
        t = synth.add_prefilter_traffic(synth.add_service_traffic(synth.make_tuples(T, n), S), P)
        del t["hash"]
        d = synth.to_device(t, "cuda")
        out = {"verdict": torch.empty(n, dtype=torch.int32, device="cuda"),
               "identity": torch.empty(n, dtype=torch.int32, device="cuda"), "stage": None}

        def make():
            e = Engine(device=0, **T.engine_config(), lb_max_entries=len(S.keys))
            synth.load_engine(e, T)
            synth.load_services(e, S)
            synth.load_prefilter4(e, P)
            return e
        return make, lambda e: e.classify_v4_cascade(d, out=out), n
    if conf == "frames":
        # bench.py --config frames: config-2 tuples as 64-byte frame slots;
        # CGPU_AB_SCHED = cgpu_config.schedule (8: the split header + classify passes; 0: the fused default)
        T = synth.make_tables(**synth.CONFIGS["gpu"])
        n = synth.CONFIGS["gpu"]["n_tuples"]
        d = synth.frames_to_device(synth.frames_from_tuples(synth.make_tuples(T, n), stride=64), "cuda")
        out = {"verdict": torch.empty(n, dtype=torch.int32, device="cuda"),
               "identity": torch.empty(n, dtype=torch.int32, device="cuda"), "stage": None}
        sched = int(os.environ.get("CGPU_AB_SCHED", "0"))

        def make():
            cfg = T.engine_config()
            if os.environ.get("CGPU_AB_HOT"):
                cfg["hot_counter_slots"] = int(os.environ["CGPU_AB_HOT"])
            e = Engine(device=0, **cfg, schedule=sched)
            synth.load_engine(e, T)
            return e
        return make, lambda e: e.classify_frames(d, out=out), n
    v6 = conf == "v6"
    T = (synth.make_tables6 if v6 else synth.make_tables)(**synth.CONFIGS[conf])
    n = synth.CONFIGS[conf]["n_tuples"]
    d = synth.to_device((synth.make_tuples6 if v6 else synth.make_tuples)(T, n))
    out = {"verdict": torch.empty(n, dtype=torch.int32, device="cuda"),
           "identity": torch.empty(n, dtype=torch.int32, device="cuda"), "stage": None}

    def make():
        cfg = T.engine_config()
        if os.environ.get("CGPU_AB_HOT"):  # LDS hot counter slots (bench.py --hot-slots)
            cfg["hot_counter_slots"] = int(os.environ["CGPU_AB_HOT"])
        e = Engine(device=0, **cfg)
        synth.load_engine(e, T)
        return e
    return make, lambda e: (e.classify_v6 if v6 else e.classify_v4)(d, out=out), n


def run(names):
    import torch
    make, launch, n = _workload(os.environ.get("CGPU_AB_CONFIG", "gpu"))
    for name in names:
        load(name)
        e = make()
        e.commit()
        for _ in range(3):
            launch(e)
        if os.environ.get("CGPU_AB_REBALANCE"):  # as bench.py after its warmup
            torch.cuda.synchronize()
            e.counters_rebalance()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
        for a, b in ev:
            a.record()
            launch(e)
            b.record()
        torch.cuda.synchronize()
        ms = sorted(a.elapsed_time(b) for a, b in ev)
        print(json.dumps({"variant": name, "median_ms": round(ms[5], 4), "min_ms": round(ms[0], 4),
                          "gpps": round(n / ms[5] / 1e6, 2)}), flush=True)
        e.close()


if __name__ == "__main__":
    names = sys.argv[2:] or list(VARIANTS)
    (build if sys.argv[1] == "build" else run)(names)
