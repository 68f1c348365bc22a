"""Build the hhuff HIP library in-tree: h2o_amd/libhhuff.so for gfx950 (hipcc, no JIT cache).

    python -m h2o_amd.build          # rebuild if any source is newer than the .so
    python -m h2o_amd.build --force
"""
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libhhuff.so")
ARCH = os.environ.get("HHUFF_ARCH", "gfx950")

HIPCC_FLAGS = ["-O3", "--offload-arch=" + ARCH, "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall",
               "-Wno-unused-function"]


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def deps():
    return sources() + sorted(glob.glob(os.path.join(CSRC, "*.h"))) + [os.path.join(ROOT, "include", "hhuff.h")]


def stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(p) > t for p in deps())


def _compile(hipcc, src, obj, extra, verbose):
    cmd = [hipcc] + HIPCC_FLAGS + ["-c", "-I" + os.path.join(ROOT, "include"), "-I" + CSRC] + extra + [src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def build(force=False, verbose=True, extra=()):
    """One object per translation unit, compiled in parallel (the units share no device symbols), then linked."""
    if not force and not stale():
        return LIB
    from concurrent.futures import ThreadPoolExecutor

    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    objdir = os.path.join(ROOT, "build", "obj")
    os.makedirs(objdir, exist_ok=True)
    srcs = sources()
    objs = [os.path.join(objdir, os.path.basename(s) + ".o") for s in srcs]
    with ThreadPoolExecutor(max_workers=min(len(srcs), os.cpu_count() or 1, 8)) as ex:
        for f in [ex.submit(_compile, hipcc, s, o, list(extra), verbose) for s, o in zip(srcs, objs)]:
            f.result()
    cmd = [hipcc, "--offload-arch=" + ARCH, "-shared", "-fPIC"] + objs + ["-o", LIB + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
