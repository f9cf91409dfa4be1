"""Idle time between kernels inside one step of a conntrack pipeline, from a
rocprofv3 kernel trace: the cost of the host reads that size later passes.

  python tools/trace_gaps.py <run_kernel_trace.csv> <first kernel of a step> [min_gap_us]

A step runs from one launch of the named kernel to the next; the script
reports, for the last complete steps, the span, the summed kernel time, the
summed idle time and the gaps above min_gap_us with the kernel before them.
"""
import csv
import sys


def main():
    path, first = sys.argv[1], sys.argv[2]
    min_gap = float(sys.argv[3]) if len(sys.argv) > 3 else 5.0
    rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                   for r in csv.DictReader(open(path))), key=lambda x: x[0])
    starts = [i for i, r in enumerate(rows) if first in r[2]]
    if len(starts) < 2:
        sys.exit(f"fewer than two launches of {first!r}")
    for a, b in list(zip(starts, starts[1:]))[-3:]:
        step = rows[a:b]
        span = (step[-1][1] - step[0][0]) / 1e3
        busy = sum(e - s for s, e, _ in step) / 1e3
        gaps = []
        for (s0, e0, n0), (s1, _, n1) in zip(step, step[1:]):
            g = (s1 - e0) / 1e3
            if g > min_gap:
                gaps.append((round(g, 1), n0.split("(")[0][-60:], n1.split("(")[0][-60:]))
        print(f"step: {len(step)} kernels, span {span:.1f} us, busy {busy:.1f} us, idle {span - busy:.1f} us")
        for g in gaps:
            print("   gap %7.1f us after %s -> %s" % g)


if __name__ == "__main__":
    main()
