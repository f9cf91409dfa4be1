"""Summarize bench JSON lines (one file each) as a table row per file:
    python tools/bench_table.py profiles/r6_final/bench_*.json"""
import json
import sys

for f in sys.argv[1:]:
    try:
        r = json.load(open(f))
    except (OSError, ValueError) as e:
        print(f, "unreadable:", e)
        continue
    c, ro = r.get("config", {}), r.get("roofline") or {}
    cb, co = r.get("cpu_baseline") or {}, r.get("cpu_baseline_optimized") or {}
    print(f"{f.split('/')[-1]:28s} value {r['value']:>10} ms/step {r['ms_per_step']:>8} "
          f"kern {c.get('kernel_ms')} parity {c.get('parity_vs_oracle')} "
          f"roof {ro.get('bound')} {ro.get('frac')} ref_fp {ro.get('frac_at_reference_footprint')} "
          f"traffic {round(ro['traffic'] / 1e9, 2) if ro.get('traffic') else None} "
          f"b_alg {(ro.get('b_alg') or {}).get('frac')} cpu {cb.get('value')}/{co.get('value')} x{cb.get('cores')}")
