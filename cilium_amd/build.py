"""Build libcgpu.so (C ABI + gfx950 kernels) in-tree with hipcc.

    python -m cilium_amd.build            # or __graft_entry__.build()

The shared library is written next to this file so that it travels to the
GPU box with the repository snapshot; it is git-ignored.
"""
from __future__ import annotations

import json
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


BUILD_JSON = os.path.join(HERE, "libcgpu.build.json")


def _sha256(path: str) -> str:
    import hashlib
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def src_sha256() -> str:
    """Hash of the library's sources (csrc + include/cgpu.h): what a build
    of them contains, independent of where and when it was compiled."""
    import hashlib
    h = hashlib.sha256()
    for p in sorted([os.path.join(CSRC, f) for f in SOURCES + HEADERS] +
                    [os.path.join(ROOT, "include", "cgpu.h")]):
        h.update(os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def lib_identity(path: str = LIB) -> dict:
    """The identity of the library file at `path` (the one a process loads):
    its own sha256 and, from libcgpu.build.json when that describes this very
    file, the sources it was built from and the git HEAD at build time
    (written only by build(); without it, or for another file, the sources
    and HEAD are reported unknown, never guessed).
    Profile summaries (tools/pmc_summary.py) are stamped with it and
    bench.py prints a PMC traffic figure only for the identity it loaded."""
    ident = {"lib_sha256": _sha256(path) if os.path.exists(path) else None,
             "src_sha256": None, "git_head": None}
    try:
        b = json.load(open(BUILD_JSON))
        if b.get("lib_sha256") == ident["lib_sha256"]:
            ident.update(src_sha256=b.get("src_sha256"), git_head=b.get("git_head"),
                         git_dirty=b.get("git_dirty"))
    except (OSError, ValueError):
        pass
    return ident


def _write_build_json() -> None:
    head, dirty = None, None
    try:
        head = subprocess.run(["git", "-C", ROOT, "rev-parse", "HEAD"], capture_output=True,
                              text=True, check=True).stdout.strip()
        dirty = bool(subprocess.run(["git", "-C", ROOT, "status", "--porcelain", "--",
                                     "cilium_amd/csrc", "include"], capture_output=True, text=True,
                                    check=True).stdout.strip())
    except (OSError, subprocess.CalledProcessError):
        pass
    rec = {"lib_sha256": _sha256(LIB), "src_sha256": src_sha256(), "git_head": head,
           "git_dirty": dirty, "arch": ARCH}
    with open(BUILD_JSON + ".tmp", "w") as f:
        json.dump(rec, f, indent=1)
    os.replace(BUILD_JSON + ".tmp", BUILD_JSON)


def build(force: bool = False, verbose: bool = False, defines=(), out: str = LIB) -> str:
    """defines: extra -D flags for timing-only tool builds (tools/diag_ab.py),
    written to another path; the product library never gets them."""
    if out == LIB and defines:
        raise ValueError("diagnostic defines only for a separate output path")
    if out == LIB and not force and not stale():
        return LIB
    objs = []
    for src in SOURCES:
        # (diagnostic objects named after their library: parallel tool builds)
        obj = os.path.join(CSRC, src.rsplit(".", 1)[0] +
                           (".o" if out == LIB else f".diag.{os.path.basename(out)}.o"))
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
    if out == LIB:
        _write_build_json()
    return out


SAN_DIR = os.path.join(HERE, "_san")
SAN_FLAGS = {
    # each -fsanitize= directly after -Xarch_host: host code only (the
    # device code is the product's, unchanged)
    "asan": ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
             "-fno-omit-frame-pointer"],
    "tsan": ["-Xarch_host", "-fsanitize=thread"],
}


def build_sanitized(kind: str, force: bool = False) -> tuple[str, str]:
    """SURVEY §5 sanitizers: the library with its host code instrumented
    (AddressSanitizer + UndefinedBehaviorSanitizer, or ThreadSanitizer) and
    the host-only ABI driver tests/sanitize/abi_host_driver.cpp linked
    against it, in cilium_amd/_san/ (development container; never shipped).
    Returns (library, driver)."""
    os.makedirs(SAN_DIR, exist_ok=True)
    lib = os.path.join(SAN_DIR, f"libcgpu_{kind}.so")
    drv = os.path.join(SAN_DIR, f"abi_host_driver_{kind}")
    src = os.path.join(ROOT, "tests", "sanitize", "abi_host_driver.cpp")
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [src, os.path.join(ROOT, "include", "cgpu.h")]
    if not force and os.path.exists(drv) and os.path.exists(lib) and             all(os.path.getmtime(d) < os.path.getmtime(drv) for d in deps):
        return lib, drv
    flags = SAN_FLAGS[kind]
    objs = []
    for src_ in SOURCES:
        host = src_.endswith(".cpp")
        # the device code is not instrumented: one kernels object serves both kinds
        obj = os.path.join(SAN_DIR, src_.rsplit(".", 1)[0] + (f".{kind}.o" if host else ".plain.o"))
        if not host and os.path.exists(obj) and all(
                os.path.getmtime(d) < os.path.getmtime(obj) for d in deps):
            objs.append(obj)
            continue
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-O1" if host else "-O3", "-g", "-std=c++17", "-fPIC",
               "-fvisibility=hidden", "-Wno-unused-function", "-I", os.path.join(ROOT, "include"),
               "-c", os.path.join(CSRC, src_), "-o", obj]
        if host:
            cmd[1:1] = ["-x", "hip"] + flags
        subprocess.run(cmd, check=True)
        objs.append(obj)
    link_san = ["-fsanitize=address,undefined"] if kind == "asan" else ["-fsanitize=thread"]
    subprocess.run([hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", lib,
                    "-L/opt/rocm/lib", "-Wl,-rpath,/opt/rocm/lib", "-lrccl"], check=True)
    clang = "/opt/rocm/lib/llvm/bin/clang++"
    subprocess.run([clang, "-O1", "-g", "-std=c++17", *link_san, "-fno-omit-frame-pointer",
                    "-I", os.path.join(ROOT, "include"), "-I", "/opt/rocm/include",
                    "-D__HIP_PLATFORM_AMD__", src, "-o", drv, lib,
                    f"-Wl,-rpath,{SAN_DIR}", "-Wl,-rpath,/opt/rocm/lib", "-pthread"], check=True)
    for o in objs:
        if not o.endswith(".plain.o"):
            os.remove(o)
    return lib, drv


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
