"""Steady-state kernel breakdown from a rocprofv3 --kernel-trace database:
kernels between the last K+1 occurrences of a step-boundary kernel (default:
the fused SGD kernel that ends every training step), grouped by family.

    python scripts/prof_steady.py gpurun_out/prof_r50/run_results.db [--steps 10] [--marker sgd_kernel]
"""
import collections
import sqlite3
import sys

FAMILIES = [("igemm_fwd", "MIOpen igemm fwd (asm)"), ("igemm_bwd", "MIOpen igemm bwd-data (asm)"),
            ("igemm_wrw", "MIOpen igemm wgrad (asm)"), ("kernel_grouped_conv_fwd", "CK conv fwd"),
            ("bwd_weight", "CK conv wgrad"), ("bwd_data", "CK conv bwd-data"), ("bn_nhwc", "HIP BN (bn_nhwc)"),
            ("BatchNorm", "MIOpen BatchNorm"), ("elementwise", "torch elementwise"), ("SubTensor", "MIOpen SubTensor"),
            ("rocclr", "rocclr copy/fill"), ("pool", "maxpool"), ("reduce", "torch reduce"),
            ("Cijk", "hipBLASLt/rocBLAS gemm")]


def main():
    db = sys.argv[1]
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 10
    marker = sys.argv[sys.argv.index("--marker") + 1] if "--marker" in sys.argv else "sgd_kernel"
    rows = list(sqlite3.connect(db).execute("select name, start, end from kernels order by start"))
    ends = [i for i, r in enumerate(rows) if marker in r[0]]
    steps = min(steps, len(ends) - 1)
    win = rows[ends[-1 - steps] + 1: ends[-1] + 1]
    span = (win[-1][2] - win[0][1]) / 1e6 / steps
    agg = collections.defaultdict(lambda: [0.0, 0])
    for n, s, e in win:
        k = next((lab for key, lab in FAMILIES if key in n), n)
        agg[k][0] += (e - s) / 1e6 / steps
        agg[k][1] += 1
    busy = sum(v[0] for v in agg.values())
    print(f"{steps} steady-state steps: span {span:.2f} ms/step, kernel busy {busy:.2f} ms/step, "
          f"{len(win) // steps} kernels/step")
    for k, (ms, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:25]:
        print(f"{ms:9.3f} ms/step {n // steps:6d}/step {100 * ms / busy:5.1f}%  {k[:110]}")


if __name__ == "__main__":
    main()
