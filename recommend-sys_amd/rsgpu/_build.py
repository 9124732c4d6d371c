"""Builds librsgpu.so (gfx950 only) in-tree with hipcc.

Objects go to recommend-sys_amd/build/, the shared library to recommend-sys_amd/rsgpu/librsgpu.so
(git-ignored, but shipped to the GPU box by gpurun).  Incremental: a source is recompiled when it or
any header is newer than its object.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)                 # recommend-sys_amd/
REPO = os.path.dirname(ROOT)
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build")
INCLUDE = os.path.join(REPO, "include")
LIB = os.path.join(PKG_DIR, "librsgpu.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

# -ffp-contract=off: parity kernels must not fuse a*b+c (the Go reference never does);
# fast kernels opt back in locally with `#pragma clang fp contract(fast)`.
# -fno-slp-vectorize: hipcc's SLP pass packs independent f32 FMAs into v_pk_* plus v_mov
# shuffles, which costs issue slots on the latency chain of the SGD kernels.
CFLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-slp-vectorize",
          f"--offload-arch={ARCH}",
          "-Wall", "-Wno-unused-result", f"-I{INCLUDE}", f"-I{CSRC}"]


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def _headers():
    return glob.glob(os.path.join(CSRC, "*.hpp")) + glob.glob(os.path.join(INCLUDE, "*.h"))


def _deps(path, seen=None):
    """The source and every local header it includes (transitively)."""
    seen = set() if seen is None else seen
    if path in seen or not os.path.exists(path):
        return seen
    seen.add(path)
    for line in open(path, errors="ignore"):
        line = line.strip()
        if line.startswith("#include \""):
            name = line.split('"')[1]
            for d in (os.path.dirname(path), CSRC, INCLUDE):
                cand = os.path.join(d, name)
                if os.path.exists(cand):
                    _deps(cand, seen)
                    break
    return seen


def _compile(src: str, obj: str) -> None:
    cmd = [HIPCC] + CFLAGS + ["-c", src, "-o", obj]
    if src.endswith(".cpp"):
        cmd = [HIPCC, "-x", "hip"] + CFLAGS + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")


def build(verbose: bool = False, jobs: int = 8) -> str:
    srcs = _sources()
    hdr_time = max((os.path.getmtime(h) for h in _headers()), default=0.0)
    # a library newer than every source is current even where the objects are absent (the GPU
    # box's snapshot ships librsgpu.so but not build/): never recompile there
    if os.path.exists(LIB) and os.path.getmtime(LIB) + 1.0 >= max(
            [hdr_time] + [os.path.getmtime(s) for s in srcs]):
        return LIB
    os.makedirs(BUILD, exist_ok=True)
    todo = []
    objs = []
    for s in srcs:
        o = os.path.join(BUILD, os.path.basename(s) + ".o")
        objs.append(o)
        if not os.path.exists(o) or os.path.getmtime(o) < max(os.path.getmtime(d) for d in _deps(s)):
            todo.append((s, o))
    if todo:
        with cf.ThreadPoolExecutor(max_workers=min(jobs, len(todo))) as ex:
            for f in [ex.submit(_compile, s, o) for s, o in todo]:
                f.result()
            if verbose:
                print(f"compiled {len(todo)} sources")
    newest = max(os.path.getmtime(o) for o in objs)
    if todo or not os.path.exists(LIB) or os.path.getmtime(LIB) < newest:
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB] + objs + [
            "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
    return LIB


HOST = os.path.join(ROOT, "host")
HOST_LIB = os.path.join(HOST, "librscore.so")
HOST_TEST = os.path.join(HOST, "tests", "core_test")
CXX = os.environ.get("CXX", "g++")


def build_host(verbose: bool = False) -> str:
    """C++ mirror of the Go core API (host/core.cpp) -> host/librscore.so linked against
    librsgpu.so, and its test binary host/tests/core_test.  rpath $ORIGIN-relative, so both run
    from the snapshot on the GPU box."""
    lib = build(verbose)
    flags = ["-O2", "-std=c++17", "-fPIC", "-pthread", "-Wall", "-Wextra", f"-I{INCLUDE}", f"-I{HOST}"]
    steps = [
        ([os.path.join(HOST, "core.cpp")], HOST_LIB,
         ["-shared", f"-L{PKG_DIR}", "-lrsgpu", "-Wl,-rpath,$ORIGIN/../rsgpu"]),
        ([os.path.join(HOST, "tests", "core_test.cpp")], HOST_TEST,
         [f"-L{HOST}", "-lrscore", f"-L{PKG_DIR}", "-lrsgpu",
          "-Wl,-rpath,$ORIGIN/..", "-Wl,-rpath,$ORIGIN/../../rsgpu"]),
    ]
    deps = [os.path.join(HOST, "core.hpp"), os.path.join(HOST, "gosort.hpp"), os.path.join(INCLUDE, "rsgpu.h"), lib]
    for srcs, out, extra in steps:
        newest = max(os.path.getmtime(p) for p in srcs + deps)
        if os.path.exists(out) and os.path.getmtime(out) >= newest:
            continue
        r = subprocess.run([CXX] + flags + srcs + ["-o", out] + extra, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"{CXX} failed for {srcs[0]}:\n{r.stderr}")
        if verbose:
            print(f"built {out}")
        deps.append(out)
    return HOST_LIB


if __name__ == "__main__":
    print(build(verbose=True))
    print(build_host(verbose=True))
