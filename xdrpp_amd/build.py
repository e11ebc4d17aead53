"""Build libxdrgpu.so in-tree with hipcc for gfx950.

    python -m xdrpp_amd.build          (or __graft_entry__.build())
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
SOURCES = [os.path.join(CSRC, "plan.cpp"), os.path.join(CSRC, "xdrgpu.hip"),
           os.path.join(CSRC, "rpc.hip")]
DEPS = SOURCES + [os.path.join(CSRC, h) for h in ("plan.h", "kernels.h", "dev_common.h", "var_kernels.h")] \
    + [os.path.join(ROOT, "include", "xdrgpu.h")]
OUT = os.path.join(PKG, "libxdrgpu.so")
ARCH = os.environ.get("XDRG_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.isabs(c) and os.path.exists(c) or not os.path.isabs(c)):
            return c
    return "hipcc"


def up_to_date() -> bool:
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(d) <= t for d in DEPS)


def build(force: bool = False, verbose: bool = True) -> str:
    if not force and up_to_date():
        return OUT
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
           "-I", os.path.join(ROOT, "include"), "-o", OUT] + SOURCES
    if verbose:
        print("[xdrpp_amd.build]", " ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
