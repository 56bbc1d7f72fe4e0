"""Build the gfx950 library in-tree: shippingenv_amd/_lib/libshipenv_hip.so.

    python -m shippingenv_amd.build

hipcc only (no torch extension machinery): the library is a plain C-ABI shared
object. -ffp-contract=off keeps the reference's unfused f64 arithmetic.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "shipenv.hip")
MAPSRC = os.path.join(HERE, "csrc", "mapload.cpp")  # host-only: the JPEG map loader
DEPS = [SRC, MAPSRC, os.path.join(HERE, "csrc", "philox.h"), os.path.join(HERE, "csrc", "qpolicy.h"), os.path.join(HERE, "csrc", "replay.h"), os.path.join(HERE, "csrc", "server.h"),
        os.path.join(HERE, "csrc", "qtrain.h"),
        os.path.join(ROOT, "include", "shipenv.h")]
OUT = os.path.join(HERE, "_lib", "libshipenv_hip.so")
ARCH = os.environ.get("SHIPENV_OFFLOAD_ARCH", "gfx950")

FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-fno-fast-math",
         "-Wall", "-Wextra", f"--offload-arch={ARCH}"]


def hipcc():
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm is required to build libshipenv_hip.so)")


STAMP = OUT + ".cmd"  # the flags that built OUT: options, defines and arch (no paths: the
                      # tree travels to the GPU box under another root)


def _flags():
    extra = os.environ.get("SHIPENV_HIPCC_DEFINES", "").split()  # e.g. -DSHIPENV_TRACE=1 (the instrumentation builds)
    return FLAGS + extra


def _command(out):
    return [hipcc()] + _flags() + ["-o", out, SRC, MAPSRC]


def up_to_date():
    """OUT is newer than every source and was built by the same command line (an A/B build
    with other defines or another SHIPENV_OFFLOAD_ARCH never reuses a stale library)."""
    if not os.path.exists(OUT) or not os.path.exists(STAMP):
        return False
    with open(STAMP) as f:
        if f.read() != " ".join(_flags()):
            return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(d) <= t for d in DEPS)


def build(force=False, verbose=True):
    if not force and up_to_date():
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    tmp = OUT + ".tmp"
    cmd = _command(tmp)
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, OUT)
    with open(STAMP, "w") as f:
        f.write(" ".join(_flags()))
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
