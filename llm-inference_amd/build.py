#!/usr/bin/env python3
"""Build libllmi.so (HIP kernels + C ABI + decode engine) for gfx950, in-tree.

    python llm-inference_amd/build.py [--force] [-j N]

Plain hipcc, no CMake: each csrc/*.hip is compiled to build/*.o with
--offload-arch=gfx950, then linked with RCCL into lib/libllmi.so. Objects are
rebuilt only when a source or any csrc/include header is newer.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
_TAG = os.environ.get("LLMI_BUILD_TAG", "")  # tuning variants: build_<tag>/, lib/libllmi_<tag>.so
BUILD = os.path.join(HERE, "build" + (f"_{_TAG}" if _TAG else ""))
LIBDIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIBDIR, f"libllmi_{_TAG}.so" if _TAG else "libllmi.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("LLMI_ARCH", "gfx950")

CFLAGS = [*os.environ.get("LLMI_EXTRA_CFLAGS", "").split(), "-std=c++17", "-O3", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
          "-I" + os.path.join(REPO, "include"), "-I" + CSRC, "-D__HIP_PLATFORM_AMD__"]
LDFLAGS = ["-shared", f"--offload-arch={ARCH}", "-L/opt/rocm/lib", "-lrccl", "-lamdhip64",
           "-Wl,-rpath,/opt/rocm/lib"]


def _headers():
    return glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(REPO, "include", "*.h"))


def _includes(path, seen=None):
    """path plus every csrc/include header it pulls in through #include "..." (transitively)."""
    import re
    seen = set() if seen is None else seen
    if path in seen or not os.path.exists(path):
        return seen
    seen.add(path)
    with open(path, errors="replace") as f:
        for m in re.finditer(r'^\s*#\s*include\s+"([^"]+)"', f.read(), re.M):
            for d in (os.path.dirname(path), CSRC, os.path.join(REPO, "include")):
                q = os.path.normpath(os.path.join(d, m.group(1)))
                if os.path.exists(q):
                    _includes(q, seen)
                    break
    return seen


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src, obj):
    cmd = [HIPCC, *CFLAGS, "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, jobs: int = 4, verbose: bool = True) -> str:
    os.makedirs(BUILD, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    hdrs = _headers()
    todo = []
    objs = []
    for s in srcs:
        o = os.path.join(BUILD, os.path.basename(s)[:-4] + ".o")
        objs.append(o)
        if force or _stale(o, sorted(_includes(s))):
            todo.append((s, o))
    if todo:
        with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            futs = {ex.submit(_compile, s, o): s for s, o in todo}
            for f in cf.as_completed(futs):
                f.result()
                if verbose:
                    print(f"[llmi build] compiled {os.path.basename(futs[f])}", flush=True)
    if force or todo or _stale(LIB, objs):
        cmd = [HIPCC, *objs, *LDFLAGS, "-o", LIB]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if verbose:
            print(f"[llmi build] linked {LIB}", flush=True)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=4)
    args = ap.parse_args()
    try:
        build(args.force, args.j)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
