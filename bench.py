"""Headline benchmark: Mpps of verdict-exact L3/L4 classification (ipcache
LPM identity + per-endpoint policy-map cascade) per BASELINE.json, and the
fraction of the HBM roofline.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

A step = one classify pass over one 64M-tuple batch already resident in HBM
(config 2: 100k IPv4 ipcache prefixes + 64k policy entries), plus the RCCL
all-reduce of the per-entry/per-reason counter deltas (N > 1) and their fold
into the totals.  Tables are replicated (same seed on every rank); tuple
streams are seeded per rank, so per-GPU work is fixed (weak scaling).
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mpps classified (LPM ipcache + policy map) at 1/2/4/8 GPUs; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
B_IN, B_OUT = 18, 8    # v4 classify tuple bytes in / out


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="gpu", choices=["gpu", "cpu"])
    ap.add_argument("--tuples", type=int, default=0, help="tuples per GPU per step")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="PMC-derived HBM bytes per launch (profiles/*), if present")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    import numpy as np
    import torch
    import torch.distributed as dist

    from cilium_amd import shard, synth
    from cilium_amd.engine import Engine

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    cfg = synth.CONFIGS[args.config]
    n = args.tuples or cfg["n_tuples"]
    t0 = time.time()
    T = synth.make_tables(**cfg)
    tup = synth.make_tuples(T, n, gpu_id=rank)
    log(f"[rank {rank}] synthetic tables ({len(T.ipc_keys)} ipcache, {len(T.pol_keys)} policy) "
        f"+ {n} tuples in {time.time() - t0:.1f}s")

    e = Engine(device=local, **T.engine_config())
    synth.load_engine(e, T)
    t0 = time.time()
    e.commit()
    log(f"[rank {rank}] commit {time.time() - t0:.2f}s, checksum {e.checksum():#x}")
    d = synth.to_device(tup, dev)
    out = {"verdict": torch.empty(n, dtype=torch.int32, device=dev),
           "identity": torch.empty(n, dtype=torch.int32, device=dev), "stage": None}
    delta = torch.zeros(e.counter_delta_bytes() // 8, dtype=torch.int64, device=dev)
    e.counter_bind(delta)
    stream = torch.cuda.current_stream()

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        e.classify_v4(d, out=out, stream=stream)
        if ev is not None:
            ev[1].record(stream)
        if world > 1:
            shard.allreduce_counters(delta)  # RCCL over xGMI: integer SUM, order-independent
        e.counter_fold(stream)

    for _ in range(args.warmup):
        step()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for k in range(args.steps):
        step(evs[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    kern_ms = sum(a.elapsed_time(b) for a, b in evs) / args.steps
    if world > 1:
        tt = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(tt[0]), float(tt[1])
    ms_per_step = 1e3 * elapsed / args.steps
    value = world * n * args.steps / elapsed / 1e6

    # counters replicated across ranks must agree
    if world > 1:
        cs = torch.tensor([e.checksum() & 0x7FFFFFFFFFFFFFFF], dtype=torch.int64, device=dev)
        lo, hi = cs.clone(), cs.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        assert int(lo) == int(hi), "replicated tables differ across ranks"

    result = None
    if rank == 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        from oracle import Oracle  # CPU restatement: checker + CPU baseline only

        o = Oracle(**T.oracle_config())
        synth.load_oracle(o, T)
        threads = args.cpu_threads or min(int(os.environ.get("OMP_NUM_THREADS", "0")) or
                                          os.cpu_count(), os.cpu_count())
        cpu = None
        c0 = time.perf_counter()
        v0, i0, _, probes = o.classify_v4(tup, nthreads=threads)
        c_el = time.perf_counter() - c0
        if not args.no_cpu_baseline:
            cpu = {"value": round(n / c_el / 1e6, 3), "unit": "Mpps", "cores": threads,
                   "kind": "port",
                   "sample": f"rank-0 batch, all {n} tuples, config-2 tables; oracle/cgpu_oracle.c "
                             f"(kernel-like LPM trie + open hash), {threads} threads, "
                             f"{c_el:.2f}s wall"}
        parity = bool(np.array_equal(out["verdict"].cpu().numpy(), v0) and
                      np.array_equal(out["identity"].cpu().numpy().view(np.uint32), i0))
        probes_per = probes / n
        b_alg = B_IN + B_OUT + 64.0 * probes_per
        achieved = b_alg * n / (kern_ms * 1e-3) / 1e9
        traffic = None
        if os.path.exists(args.traffic_json):
            try:
                traffic = json.load(open(args.traffic_json)).get("hbm_bytes_per_launch")
            except (OSError, ValueError):
                traffic = None
        result = {
            "metric": METRIC, "value": round(value, 2), "unit": "Mpps", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (seeded PCG64 tables + tuples, SURVEY §8d)",
            "config": {"workload": "config2: 100k IPv4 ipcache LPM + 64k policy entries "
                                   "(4 ep x 16k), 64M-tuple batches per GPU, bit-exact verdicts"
                       if args.config == "gpu" else "config1 (CPU-scale)",
                       "tuples_per_gpu": n, "ipcache_prefixes": int(len(T.ipc_keys)),
                       "policy_entries": int(len(T.pol_keys)), "parallelism": f"shard{world}",
                       "kernel_ms": round(kern_ms, 4), "probes_per_tuple": round(probes_per, 4),
                       "b_alg_per_tuple": round(b_alg, 2), "parity_vs_oracle": parity},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic},
            "cpu_baseline": cpu,
        }
        if not parity:
            log("WARNING: GPU verdicts differ from the restatement")
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    e.close()
    if rank == 0:
        print(json.dumps(result), flush=True)


if __name__ == "__main__":
    main()
