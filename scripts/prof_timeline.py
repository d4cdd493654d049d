"""Per-step kernel timeline from a rocprofv3 kernel-trace database: for one
steady-state step (delimited by a marker kernel), list each kernel's duration
and the idle gap before it; summarise busy vs. idle time per step.
    python scripts/prof_timeline.py <db> [--marker conv_fwd_c8] [--step -5]"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    marker = sys.argv[sys.argv.index("--marker") + 1] if "--marker" in sys.argv else "conv_fwd_c8"
    which = int(sys.argv[sys.argv.index("--step") + 1]) if "--step" in sys.argv else -5
    c = sqlite3.connect(db)
    rows = sorted(c.execute("select name, start, end from kernels"), key=lambda r: r[1])
    starts = [i for i, r in enumerate(rows) if marker in r[0]]
    # a step starts at the first marker kernel of a group
    steps = [s for k, s in enumerate(starts) if k == 0 or s - starts[k - 1] > 2]
    a, b = steps[which], steps[which + 1]
    t0 = rows[a][1]
    prev_end = t0
    busy = 0
    print(f"{'start':>8} {'dur':>7} {'gap':>6}  kernel")
    for name, s, e in rows[a:b]:
        gap = max(0, s - prev_end)
        busy += e - max(s, prev_end) if e > prev_end else 0
        print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.2f} {gap / 1e3:6.2f}  {name.split('(')[0][:90]}")
        prev_end = max(prev_end, e)
    span = rows[b][1] - t0
    print(f"step span {span / 1e3:.1f} us, busy {busy / 1e3:.1f} us, idle {(span - busy) / 1e3:.1f} us, "
          f"{b - a} kernels")
    spans = [(rows[steps[k + 1]][1] - rows[steps[k]][1]) / 1e3 for k in range(len(steps) - 1)]
    spans.sort()
    print(f"median step span over {len(spans)} steps: {spans[len(spans) // 2]:.1f} us")


if __name__ == "__main__":
    main()
