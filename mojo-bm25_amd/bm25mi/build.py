"""Build the in-tree shared libraries (no JIT cache: the .so files travel with
the repo snapshot to the GPU box).

  libbm25mi.so     hipcc --offload-arch=gfx950: kernels + C-ABI (the product)
  libbm25synth.so  g++: synthetic index / query generator (bench + tests data)
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(PKG_DIR), "csrc")
REPO = os.path.dirname(os.path.dirname(PKG_DIR))
# The product library.  (scripts/variant_lib_time.py points this at a variant
# build inside its own child processes before bm25mi._capi is imported.)
LIB = os.path.join(PKG_DIR, "libbm25mi.so")
SYNTH_LIB = os.path.join(PKG_DIR, "libbm25synth.so")

HIP_SOURCES = ["bm25mi_kernels.hip", "bm25mi_large.hip", "bm25mi_build.hip", "bm25mi_sort.hip",
               "bm25mi_dense.hip", "bm25mi_capi.cpp"]
ARCH = os.environ.get("BM25_OFFLOAD_ARCH", "gfx950")


def _stale(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def build(force: bool = False, verbose: bool = False) -> None:
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    hdrs = [os.path.join(CSRC, "bm25mi_internal.h"), os.path.join(REPO, "include", "bm25mi.h")]
    lib = os.path.join(PKG_DIR, "libbm25mi.so")
    objdir = os.path.join(PKG_DIR, "_obj")
    os.makedirs(objdir, exist_ok=True)
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wno-unused-result",
             "-Wno-unused-value"]
    srcs = [os.path.join(CSRC, src) for src in HIP_SOURCES]
    # the library travels without its objects (.gpurunignore): up to date when
    # newer than every source and header
    lib_fresh = not force and not _stale(lib, srcs + hdrs)
    objs, jobs = [], []
    for src in ([] if lib_fresh else HIP_SOURCES):
        o = os.path.join(objdir, os.path.splitext(src)[0] + ".o")
        objs.append(o)
        if force or _stale(o, [os.path.join(CSRC, src)] + hdrs):
            jobs.append([hipcc] + flags + ["-c", "-o", o + ".tmp", os.path.join(CSRC, src)])
    if jobs:  # one hipcc per translation unit, in parallel
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(len(jobs)) as ex:
            list(ex.map(lambda c: _run(c, verbose), jobs))
        for c in jobs:
            os.replace(c[-2], c[-2][:-4])
    if not lib_fresh and (force or jobs or _stale(lib, objs)):
        tmp = lib + ".tmp"
        _run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs, verbose)
        os.replace(tmp, lib)
    sdeps = [os.path.join(CSRC, "synth.cpp")]
    if force or _stale(SYNTH_LIB, sdeps):
        tmp = SYNTH_LIB + ".tmp"
        _run(["g++", "-O2", "-ffp-contract=off", "-std=c++17", "-fPIC", "-shared", "-pthread",
              "-o", tmp, sdeps[0]], verbose)
        os.replace(tmp, SYNTH_LIB)


def build_asan_check(verbose: bool = False) -> str:
    """tests/asan/host_check built against every source with AddressSanitizer
    on the host side (-Xarch_host -fsanitize=address; device code as usual),
    into mojo-bm25_amd/bm25mi/_asan/ (rebuilt when a source is newer).  Test
    infrastructure for tests/test_host.py (SURVEY.md:235), not the product."""
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    out = os.path.join(PKG_DIR, "_asan")
    os.makedirs(out, exist_ok=True)
    exe = os.path.join(out, "host_check")
    main = os.path.join(REPO, "tests", "asan", "host_check.cpp")
    srcs = [os.path.join(CSRC, s) for s in HIP_SOURCES] + [main]
    hdrs = [os.path.join(CSRC, "bm25mi_internal.h"), os.path.join(REPO, "include", "bm25mi.h")]
    if not _stale(exe, srcs + hdrs):
        return exe
    flags = [f"--offload-arch={ARCH}", "-O1", "-g", "-std=c++17", "-fPIC", "-w",
             "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer"]
    jobs, objs = [], []
    for src in srcs:
        o = os.path.join(out, os.path.splitext(os.path.basename(src))[0] + ".o")
        objs.append(o)
        jobs.append([hipcc] + flags + ["-c", "-o", o, src])
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(len(jobs)) as ex:
        list(ex.map(lambda c: _run(c, verbose), jobs))
    _run([hipcc, f"--offload-arch={ARCH}", "-fsanitize=address", "-fno-gpu-sanitize", "-o",
          exe + ".tmp"] + objs, verbose)
    os.replace(exe + ".tmp", exe)
    return exe


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
