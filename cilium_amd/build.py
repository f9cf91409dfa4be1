"""Build libcgpu.so (C ABI + gfx950 kernels) in-tree with hipcc.

    python -m cilium_amd.build            # or __graft_entry__.build()

The shared library is written next to this file so that it travels to the
GPU box with the repository snapshot; it is git-ignored.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libcgpu.so")
SOURCES = ["host.cpp", "kernels.hip"]
HEADERS = ["tables.h", "launch.h"]
ARCH = os.environ.get("CGPU_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for p in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc"):
        if p and os.path.exists(p):
            return p
    return "hipcc"


def stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps.append(os.path.join(ROOT, "include", "cgpu.h"))
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False, defines=(), out: str = LIB) -> str:
    """defines: extra -D flags for timing-only tool builds (tools/diag_ab.py),
    written to another path; the product library never gets them."""
    if out == LIB and defines:
        raise ValueError("diagnostic defines only for a separate output path")
    if out == LIB and not force and not stale():
        return LIB
    objs = []
    for src in SOURCES:
        obj = os.path.join(CSRC, src.rsplit(".", 1)[0] + (".o" if out == LIB else ".diag.o"))
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
               "-fvisibility=hidden", "-Wall", "-Wno-unused-function",
               *[f"-D{d}" for d in defines],
               "-I", os.path.join(ROOT, "include"), "-c", os.path.join(CSRC, src), "-o", obj]
        if src.endswith(".cpp"):
            cmd[1:1] = ["-x", "hip"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        objs.append(obj)
    tmp = out + ".tmp"
    # RCCL (cgpu_counters_allreduce) from the ROCm install the library runs on
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", tmp,
           "-L/opt/rocm/lib", "-Wl,-rpath,/opt/rocm/lib", "-lrccl"]
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)
    for o in objs:
        os.remove(o)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
