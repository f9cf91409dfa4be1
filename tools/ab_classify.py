"""Interleaved same-process A/B of classify configurations (HIP events).

    python tools/ab_classify.py [--configs 3:1,3:4,0:1] [--rounds 5] [--iters 5]

A configuration is VARIANT:BPB[:LOADPCT] — the kernel counter strategy
(CGPU_CLASSIFY_VARIANT) and the policy-table layout chosen at commit
(CGPU_POL_BPB slots per bucket, CGPU_POL_LOAD_PCT load factor).  Each round
runs every configuration `iters` times back to back; reports median / min
kernel time and checks that every configuration's outputs are bit-identical.
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
    ap.add_argument("--configs", default="3:1,3:4,0:1,9:1")
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
    d = synth.to_device(t)
    n = args.tuples
    confs = list(args.configs.split(","))
    engines = {}
    for c in confs:
        parts = c.split(":")
        key = tuple(parts[1:])
        if key in engines:
            continue
        os.environ["CGPU_POL_BPB"] = parts[1] if len(parts) > 1 else "1"
        if len(parts) > 2:
            os.environ["CGPU_POL_LOAD_PCT"] = parts[2]
        else:
            os.environ.pop("CGPU_POL_LOAD_PCT", None)
        e = Engine(device=0, **T.engine_config())
        synth.load_engine(e, T)
        e.commit()
        engines[key] = e
    outs, times = {}, {c: [] for c in confs}
    for r in range(args.rounds):
        for c in confs:
            parts = c.split(":")
            os.environ["CGPU_CLASSIFY_VARIANT"] = parts[0]
            e = engines[tuple(parts[1:])]
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
            times[c].append(a.elapsed_time(b) / args.iters)
            if r == 0:
                outs[c] = (out["verdict"].cpu().numpy(), out["identity"].cpu().numpy())
    ref = outs[confs[0]]
    res = {}
    for c in confs:
        same = all(np.array_equal(x, y) for x, y in zip(outs[c], ref))
        med = statistics.median(times[c])
        res[c] = {"median_ms": round(med, 4), "min_ms": round(min(times[c]), 4),
                  "gpps": round(n / med / 1e6, 3), "identical": same}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
