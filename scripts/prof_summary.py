"""Summarise a rocprofv3 kernel-trace database (.db) or kernel_stats csv:
per-kernel calls / total / mean time, sorted by total.  Usage:
    python scripts/prof_summary.py <dir-or-db> [--steps N] [--top K]"""
import glob
import os
import sqlite3
import sys


def main():
    path = sys.argv[1]
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else None
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 40
    dbs = [path] if path.endswith(".db") else glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
    rows = {}
    for db in dbs:
        c = sqlite3.connect(db)
        for name, dur in c.execute("select name, duration from kernels"):
            r = rows.setdefault(name, [0, 0])
            r[0] += 1
            r[1] += dur
    tot = sum(v[1] for v in rows.values())
    print(f"{'total_us':>10} {'calls':>6} {'mean_us':>9} {'pct':>6}  kernel")
    for name, (n, d) in sorted(rows.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{d/1e3:10.1f} {n:6d} {d/n/1e3:9.2f} {100*d/tot:5.1f}%  {name[:150]}")
    print(f"TOTAL kernel time {tot/1e3:.1f} us" + (f" = {tot/1e3/steps:.1f} us/step" if steps else ""))


if __name__ == "__main__":
    main()
