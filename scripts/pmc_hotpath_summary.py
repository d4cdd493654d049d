"""Join rocprofv3 PMC passes with their kernel traces: per dl:: kernel, mean
duration, HBM bytes (FETCH_SIZE + WRITE_SIZE, KB in the counter), achieved
GB/s, and MFMA busy / LDS bank-conflict ratios.
    python scripts/pmc_hotpath_summary.py <pass-dir> [<pass-dir> ...]"""
import glob
import sqlite3
import sys
from collections import defaultdict

cnt = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for d in sys.argv[1:]:
    for db in glob.glob(d + "/**/*.db", recursive=True):
        c = sqlite3.connect(db)
        try:
            for k, n, v in c.execute("select kernel_name, counter_name, sum(value) from counters_collection "
                                     "group by dispatch_id, counter_name"):
                cnt[k][n].append(v)
        except sqlite3.OperationalError:
            pass
        try:
            for k, t in c.execute("select name, duration from kernels"):
                dur[k].append(t)
        except sqlite3.OperationalError:
            pass


def short(k):
    k = k.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    return k[-70:]


# MFMA busy: SQ_VALU_MFMA_BUSY_CYCLES (summed over every SIMD: 16 cycles per
# 16x16x32 bf16 MFMA = its peak rate) over (GRBM_GUI_ACTIVE per XCD x 256 CUs x 4
# SIMDs); GRBM_GUI_ACTIVE is reported summed over the 8 XCD instances.
# LDS: bank-conflict cycles per LDS instruction.
NCU, NXCD, NSIMD = 256, 8, 4
print(f"{'kernel':70s} {'us':>8s} {'fetchMB':>9s} {'writeMB':>9s} {'GB/s':>7s} {'MFMAbusy%':>9s} {'LDScf/ins':>9s}")
for k in sorted(cnt):
    if "dl::" not in k:
        continue
    cs = cnt[k]
    mean = lambda n: sum(cs[n]) / len(cs[n]) if cs.get(n) else float("nan")  # noqa: E731
    t = sum(dur[k]) / len(dur[k]) / 1e3 if dur.get(k) else float("nan")
    f, w = mean("FETCH_SIZE") / 1e3, mean("WRITE_SIZE") / 1e3
    gbs = (f + w) / t * 1e3 if t == t else float("nan")
    mf = 100 * mean("SQ_VALU_MFMA_BUSY_CYCLES") / max(mean("GRBM_GUI_ACTIVE") / NXCD * NCU * NSIMD, 1)
    lds = mean("SQ_LDS_BANK_CONFLICT") / max(mean("SQ_INSTS_LDS"), 1)
    print(f"{short(k):70s} {t:8.1f} {f:9.1f} {w:9.1f} {gbs:7.0f} {mf:9.1f} {lds:9.2f}")
    print(f"{'':70s} raw: GRBM_GUI_ACTIVE {mean('GRBM_GUI_ACTIVE'):.0f} MFMA_BUSY {mean('SQ_VALU_MFMA_BUSY_CYCLES'):.0f} "
          f"SQ_BUSY {mean('SQ_BUSY_CYCLES'):.0f} INSTS_MFMA {mean('SQ_INSTS_MFMA'):.0f} WAVES {mean('SQ_WAVES'):.0f}")
