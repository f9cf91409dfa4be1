"""Same-process A/B of engine configurations on the config-2 workload.

    python tools/ab_engine.py --confs '{"hot_counter_slots": 8192}' '{"hot_counter_slots": 4096}'

Each configuration gets its own engine (same tables); rounds interleave the
configurations; reports median kernel time and checks bit-identical outputs.
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
    ap.add_argument("--confs", nargs="+", default=["{}"])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--tuples", type=int, default=64 << 20)
    args = ap.parse_args()
    import numpy as np
    import torch

    from cilium_amd import synth
    from cilium_amd.engine import Engine

    T = synth.make_tables(**synth.CONFIGS["gpu"])
    t = synth.make_tuples(T, args.tuples)
    d = synth.to_device(t)
    n = args.tuples
    confs = [json.loads(c) for c in args.confs]
    engines = []
    for c in confs:
        env = c.pop("env", {})
        for k, v in env.items():
            os.environ[k] = str(v)
        e = Engine(device=0, **{**T.engine_config(), **c})
        synth.load_engine(e, T)
        e.commit()
        engines.append((e, env))
    times = [[] for _ in confs]
    outs = []
    for r in range(args.rounds):
        for ci, (e, env) in enumerate(engines):
            for k, v in env.items():
                os.environ[k] = str(v)
            out = {"verdict": torch.empty(n, dtype=torch.int32, device="cuda"),
                   "identity": torch.empty(n, dtype=torch.int32, device="cuda"), "stage": None}
            e.classify_v4(d, out=out)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(args.iters):
                e.classify_v4(d, out=out)
            b.record()
            torch.cuda.synchronize()
            times[ci].append(a.elapsed_time(b) / args.iters)
            for k in env:
                os.environ.pop(k, None)
            if r == 0:
                outs.append((out["verdict"].cpu().numpy(), out["identity"].cpu().numpy()))
    res = []
    for ci, c in enumerate(args.confs):
        med = statistics.median(times[ci])
        same = all(np.array_equal(x, y) for x, y in zip(outs[ci], outs[0]))
        res.append({"conf": c, "median_ms": round(med, 4), "gpps": round(n / med / 1e6, 3),
                    "identical": same})
    print(json.dumps(res))


if __name__ == "__main__":
    main()
