"""Sanitizers: the C ABI's host code under AddressSanitizer +
UndefinedBehaviorSanitizer and under ThreadSanitizer.

cilium_amd.build.build_sanitized() builds libcgpu with -fsanitize on the host
code only (each flag after -Xarch_host; GPU sanitizers do not exist on this
pool) and links tests/sanitize/abi_host_driver.cpp against it.  The driver
drives every table, PreFilter, conntrack (v4 and v6) and checkpoint call on
host-only contexts, including the error paths (bad prefix lengths, full maps,
stale revisions with undo, corrupted checkpoints); in "tsan" mode four
writer threads, a walker / GC / PreFilter thread and a checkpoint thread share
one context (the mirror lock's contract).  Any sanitizer report fails the run
(halt_on_error).  __graft_entry__.build() builds the binaries; this test
builds them itself when they are missing or stale (~1.5 min each)."""
import os
import subprocess

import pytest

from cilium_amd import build


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_abi_host_code_under_sanitizer(kind, tmp_path):
    _, drv = build.build_sanitized(kind)
    env = dict(os.environ)
    env.update(ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               TSAN_OPTIONS="halt_on_error=1:report_thread_leaks=0")
    r = subprocess.run([drv, kind, str(tmp_path)], env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-6000:]
    assert f"sanitizer driver ({kind}) ok" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
    assert "WARNING: ThreadSanitizer" not in r.stderr
