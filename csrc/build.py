"""Build the native library ``torch_distlearn_amd/_C*.so`` for gfx950 (MI355X).

Every ``csrc/**/*.hip`` kernel file and the C++ runtime/bindings are compiled
with ``hipcc --offload-arch=gfx950`` into objects (in parallel, incrementally)
and linked into one in-tree Python extension that also links RCCL.  Nothing is
JIT-compiled at import time and nothing is installed into site-packages: the
built ``.so`` lives next to the Python package so it travels with the repo to
the GPU box.

Usage:  python csrc/build.py [--force] [-j N] [--verbose]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
PKG = os.path.join(ROOT, "torch_distlearn_amd")
BUILD = os.path.join(ROOT, "build", "native")
ARCH = os.environ.get("DISTLEARN_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")


TESTING = os.path.join(CSRC, "testing")  # test/diagnostic kernels -> separate _C_testing extension


def ext_path(name: str = "_C") -> str:
    return os.path.join(PKG, name + sysconfig.get_config_var("EXT_SUFFIX"))


def _sources(testing: bool = False):
    srcs = []
    for d, _, files in os.walk(CSRC):
        if (os.path.commonpath([d, TESTING]) == TESTING) != testing:
            continue
        for f in sorted(files):
            if f.endswith((".hip", ".cpp")):
                srcs.append(os.path.join(d, f))
    return sorted(srcs)


def _headers():
    hs = []
    for d, _, files in os.walk(CSRC):
        for f in files:
            if f.endswith((".h", ".hpp", ".inc")):
                hs.append(os.path.join(d, f))
    return hs


def _includes():
    import pybind11

    return [
        "-I" + os.path.join(CSRC, "include"),
        "-I" + CSRC,
        "-I" + pybind11.get_include(),
        "-I" + sysconfig.get_paths()["include"],
    ]


COMMON = ["-O3", "-fPIC", "-std=c++17", "-Wno-unused-result", "-Wno-unused-command-line-argument"]


def _obj_for(src: str) -> str:
    rel = os.path.relpath(src, CSRC).replace(os.sep, "__")
    return os.path.join(BUILD, rel + ".o")


def _deps_mtime(obj: str, newest_header: float) -> float:
    """Newest mtime among the headers ``obj`` was compiled from (its -MMD
    dependency file); every header when there is no dependency file."""
    dep = obj + ".d"
    if not os.path.exists(dep):
        return newest_header
    try:
        text = open(dep).read().replace("\\\n", " ")
        files = text.split(":", 1)[1].split()
        return max([os.path.getmtime(f) for f in files if f.endswith((".h", ".hpp", ".inc"))] + [0.0])
    except (OSError, IndexError):
        return newest_header


def _compile(src: str, force: bool, verbose: bool, newest_header: float):
    obj = _obj_for(src)
    if (not force and os.path.exists(obj)
            and os.path.getmtime(obj) >= max(os.path.getmtime(src), _deps_mtime(obj, newest_header))):
        return obj, 0.0, False
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-c", src, "-o", obj, "-MMD", "-MF", obj + ".d"] + COMMON + _includes()
    cmd += os.environ.get("DISTLEARN_CFLAGS", "").split()  # A/B experiments (e.g. -DDL_FWD_SWAP=0)
    if "bindings" in src or "testing" in src:
        cmd += ["-fvisibility=hidden"]
    t0 = time.time()
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    # the object is as old as the sources it was compiled from: a source edited
    # while hipcc ran (minutes for conv_igemm.hip) is newer and rebuilds next time
    os.utime(obj, (t0 - 1.0, t0 - 1.0))
    return obj, time.time() - t0, True


def _flags_changed() -> bool:
    """Objects are reused by mtime only, so a change of DISTLEARN_CFLAGS (e.g. a
    diagnostic -DDL_WGRAD_STAMPS build and back) forces a full rebuild: an object
    compiled under other flags must never be linked silently."""
    os.makedirs(BUILD, exist_ok=True)
    stamp = os.path.join(BUILD, "cflags.txt")
    cur = os.environ.get("DISTLEARN_CFLAGS", "").strip()
    old = open(stamp).read() if os.path.exists(stamp) else None
    if old != cur:
        with open(stamp, "w") as f:
            f.write(cur)
        return old is not None or bool(cur)
    return False


def build(force: bool = False, jobs: int | None = None, verbose: bool = False) -> str:
    """Build the product extension ``_C`` and the test-support ``_C_testing``."""
    force = _flags_changed() or force
    out = _build_ext("_C", _sources(False), force, jobs, verbose, ["-lrccl"])
    _build_ext("_C_testing", _sources(True), force, jobs, verbose, [])
    return out


def _build_ext(name, srcs, force, jobs, verbose, libs) -> str:
    os.makedirs(BUILD, exist_ok=True)
    hdr = max([os.path.getmtime(h) for h in _headers()] + [0.0])
    jobs = jobs or min(8, os.cpu_count() or 4)
    objs = []
    rebuilt = False
    with cf.ThreadPoolExecutor(jobs) as ex:
        futs = {ex.submit(_compile, s, force, verbose, hdr): s for s in srcs}
        for f in cf.as_completed(futs):
            obj, dt, did = f.result()
            objs.append(obj)
            rebuilt |= did
            if did:
                print(f"[distlearn build] {os.path.relpath(futs[f], ROOT)}  {dt:.1f}s", flush=True)
    out = ext_path(name)
    if rebuilt or force or not os.path.exists(out) or any(os.path.getmtime(o) > os.path.getmtime(out) for o in objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out] + sorted(objs) + [
            "-L" + os.path.join(ROCM, "lib")] + libs
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        print(f"[distlearn build] linked {os.path.relpath(out, ROOT)}", flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("--verbose", action="store_true")
    a = ap.parse_args()
    build(a.force, a.j, a.verbose)


if __name__ == "__main__":
    sys.exit(main())
