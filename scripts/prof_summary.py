"""Summarise a rocprofv3 kernel-trace database (.db) or kernel_stats csv:
per-kernel calls / total / mean time, sorted by total.  Usage:
    python scripts/prof_summary.py <dir-or-db> [--steps N] [--top K] [--last-ms T] [--marker NAME]
--last-ms keeps only the kernels that started in the last T ms of the trace
(e.g. the timed steps after a warm-up that ran MIOpen's solver search)."""
import glob
import os
import sqlite3
import sys


def main():
    path = sys.argv[1]
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else None
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 40
    last = float(sys.argv[sys.argv.index("--last-ms") + 1]) if "--last-ms" in sys.argv else None
    dbs = [path] if path.endswith(".db") else glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
    rows = {}
    for db in dbs:
        c = sqlite3.connect(db)
        q = "select name, duration from kernels"
        if last is not None:
            end = c.execute("select max(end) from kernels").fetchone()[0]
            q += f" where start >= {int(end - last * 1e6)}"
        for name, dur in c.execute(q):
            r = rows.setdefault(name, [0, 0])
            r[0] += 1
            r[1] += dur
    tot = sum(v[1] for v in rows.values())
    print(f"{'total_us':>10} {'calls':>6} {'mean_us':>9} {'pct':>6}  kernel")
    for name, (n, d) in sorted(rows.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{d/1e3:10.1f} {n:6d} {d/n/1e3:9.2f} {100*d/tot:5.1f}%  {name[:150]}")
    marker = sys.argv[sys.argv.index("--marker") + 1] if "--marker" in sys.argv else None
    if marker:  # steps = calls of a once-per-step kernel (e.g. sgd_kernel)
        steps = sum(n for name, (n, _) in rows.items() if marker in name) or steps
    print(f"TOTAL kernel time {tot/1e3:.1f} us" + (f" = {tot/1e3/steps:.1f} us/step over {steps} steps" if steps else ""))


if __name__ == "__main__":
    main()
