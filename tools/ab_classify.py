"""Interleaved same-process A/B of classify kernel variants (HIP events).

    python tools/ab_classify.py [--variants 0,1] [--rounds 5] [--iters 5] [--tuples N]

Each round runs every variant `iters` times back to back; reports the median
and min kernel time per variant over rounds and checks that every variant's
outputs are bit-identical.
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,3,9")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--tuples", type=int, default=64 << 20)
    ap.add_argument("--config", default="gpu")
    args = ap.parse_args()
    import numpy as np
    import torch

    from cilium_amd import synth
    from cilium_amd.engine import Engine

    cfg = dict(synth.CONFIGS[args.config])
    T = synth.make_tables(**cfg)
    t = synth.make_tuples(T, args.tuples)
    e = Engine(device=0, **T.engine_config())
    synth.load_engine(e, T)
    e.commit()
    d = synth.to_device(t)
    n = args.tuples
    variants = [int(v) for v in args.variants.split(",")]
    outs = {}
    times = {v: [] for v in variants}
    for r in range(args.rounds):
        for v in variants:
            os.environ["CGPU_CLASSIFY_VARIANT"] = str(v)
            out = {"verdict": torch.empty(n, dtype=torch.int32, device="cuda"),
                   "identity": torch.empty(n, dtype=torch.int32, device="cuda"), "stage": None}
            e.classify_v4(d, out=out)  # warm
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(args.iters):
                e.classify_v4(d, out=out)
            b.record()
            torch.cuda.synchronize()
            times[v].append(a.elapsed_time(b) / args.iters)
            if r == 0:
                outs[v] = (out["verdict"].cpu().numpy(), out["identity"].cpu().numpy())
    ref = outs[variants[0]]
    res = {}
    for v in variants:
        same = all(np.array_equal(x, y) for x, y in zip(outs[v], ref))
        med = statistics.median(times[v])
        res[v] = {"median_ms": round(med, 4), "min_ms": round(min(times[v]), 4),
                  "gpps": round(n / med / 1e6, 3), "identical": same}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
