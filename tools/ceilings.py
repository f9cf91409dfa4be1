"""Fold the output of tools/microbench/ceilings.hip into profiles/ceilings.json,
the measured transaction ceilings bench.py prices its roofline with.

    ./tools/microbench/ceilings > gpurun_out/<tag>/ceilings.jsonl     (GPU box)
    python3 tools/ceilings.py gpurun_out/<tag>/ceilings.jsonl profiles/ceilings.json

gather[S]  best random-gather rate (G loads/s, over the widths 4 / 8 / 16 B,
           1-16 loads in flight per lane, 16 or 32 waves per CU) from a table
           of S bytes: the ceiling of the cache tier a table of that size
           lives in.
atomic     best rate of no-return packed u64 atomicAdd at random slots.
stream     coalesced 16-B-per-lane read / write rates (GB/s).
mix        measured mixes of two tiers against bench.py's composition of a
           path's gathers (time >= max(all loads / R(small), big-table loads
           / R(big))): composed_over_measured >= 1 means the composed rate
           is a ceiling the mix does not beat.
"""
import json
import sys


def fold(rows):
    dev = next((r for r in rows if r["kind"] == "device"), {})
    gather = {}
    for r in rows:
        if r["kind"] == "gather":
            s = int(r["table_bytes"])
            gather[s] = max(gather.get(s, 0.0), float(r["g_per_s"]))
    atom = [r for r in rows if r["kind"] == "atomic"]
    stream = next((r for r in rows if r["kind"] == "stream"), None)
    sizes = sorted(gather)

    def rate(s):
        best = gather[sizes[0]]
        for x in sizes:
            if x <= s:
                best = gather[x]
        return best
    mixes = []
    for r in rows:
        if r["kind"] != "mix":
            continue
        f = float(r["small_frac"])
        # bench.py's composition: every load at least at the small tier's
        # cost, the big table's loads at least at the big tier's
        pred = 1.0 / max(1.0 / rate(int(r["small_bytes"])), (1 - f) / rate(int(r["big_bytes"])))
        mixes.append({"small_bytes": int(r["small_bytes"]), "big_bytes": int(r["big_bytes"]),
                      "small_frac": f, "measured_g_per_s": float(r["g_per_s"]),
                      "composed_g_per_s": round(pred, 2),
                      "composed_over_measured": round(pred / float(r["g_per_s"]), 4)})
    return {
        "device": dev,
        "gather": [[s, round(gather[s], 2)] for s in sizes],
        "atomic_g_per_s": round(max(float(r["g_per_s"]) for r in atom), 3) if atom else None,
        "atomic_sum_ok": all(r.get("sum_ok") is True for r in atom) if atom else None,
        "atomic": [{"slots": r["slots"], "g_per_s": r["g_per_s"], "sum_ok": r.get("sum_ok")} for r in atom],
        "stream": {"read_gbs": stream["read_gbs"], "write_gbs": stream["write_gbs"]} if stream else None,
        "mix": mixes,
        "source": "tools/microbench/ceilings.hip on one MI355X (gather: best over widths 4/8/16 B, "
                  "K 4/8/16 loads in flight per lane, 16/32 waves per CU; uniformly random "
                  "W-aligned offsets)",
    }


def main():
    src, dst = sys.argv[1], sys.argv[2]
    rows = [json.loads(x) for x in open(src) if x.strip()]
    out = fold(rows)
    json.dump(out, open(dst, "w"), indent=1)
    for s, g in out["gather"]:
        print(f"{s / 2**20:10.3f} MiB  {g:8.1f} G/s")
    print("atomic", out["atomic_g_per_s"], "sum_ok", out["atomic_sum_ok"], "stream", out["stream"])
    for m in out["mix"]:
        print(m)


if __name__ == "__main__":
    main()
