"""Per-kernel PMC counter totals from rocprofv3 databases:
    python scripts/pmc_summary.py <dir> [name-filter]"""
import glob
import sqlite3
import sys

d = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
res = {}
for db in glob.glob(d + "/**/*.db", recursive=True):
    c = sqlite3.connect(db)
    for k, n, v, cnt in c.execute("select kernel_name, counter_name, sum(value), count(distinct dispatch_id) "
                                  "from counters_collection group by kernel_name, counter_name"):
        if flt in k:
            res.setdefault(k, {})[n] = (v, cnt)
for k, cs in res.items():
    print(k[:100])
    for n, (v, cnt) in sorted(cs.items()):
        print(f"   {n:28s} {v / cnt:16.0f} per dispatch")
