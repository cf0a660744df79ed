"""The host C/C++ under AddressSanitizer + UBSan (the reference
runs `go test --race`; the build's native host code gets the sanitizers).

Builds oracle/build/liboracle_asan.so and etcd_amd/libhbnode_asan.so
(`make asan`, -fsanitize=address,undefined, -fno-sanitize-recover=undefined)
and runs the CPU suites that drive them — MemoryStorage KATs (libhbnode),
the oracle KATs, the wire decoder, Tick and the workload generators — in a
child python with the sanitizer runtimes preloaded.  Any ASan report or UB
aborts the child, so the test fails with the report in its message.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SUITES = ["tests/test_storage.py", "tests/test_oracle_kat.py", "tests/test_wire.py", "tests/test_tick.py",
          "tests/test_workloads.py", "tests/test_route.py"]


def _runtime(name):
    out = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    return out if os.path.isabs(out) and os.path.exists(out) else None


def test_host_libraries_under_asan_ubsan():
    asan, ubsan = _runtime("libasan.so"), _runtime("libubsan.so")
    if not asan or not ubsan:
        pytest.skip("gcc sanitizer runtimes not installed")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True)
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "etcd_amd", "csrc"), "asan"], check=True)
    env = dict(os.environ,
               ORC_LIB=os.path.join(ROOT, "oracle", "build", "liboracle_asan.so"),
               HBN_LIB=os.path.join(ROOT, "etcd_amd", "libhbnode_asan.so"),
               LD_PRELOAD=f"{asan}:{ubsan}",
               ASAN_OPTIONS="detect_leaks=0",  # the interpreter's own allocations are not ours
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    # -s: a sanitizer report goes to fd 2 and must survive the child's abort
    r = subprocess.run([sys.executable, "-m", "pytest", *SUITES, "-q", "-s", "-x", "-m", "not gpu",
                        "-p", "no:cacheprovider"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    out = r.stdout + r.stderr
    bad = [ln for ln in out.splitlines() if "runtime error:" in ln or "AddressSanitizer" in ln]
    assert r.returncode == 0 and not bad, out[-6000:]


def test_host_threading_under_tsan():
    """libhbnode's host threading under ThreadSanitizer: the Pool (hbpool.h:
    run / prewake / post / STOP, partners spinning or not, small and large
    cycles, 1-16 workers, two nodes' pools at once) and the router's threaded
    passes (hbroute.cpp), driven by tests/tsan/pool_tsan.cpp with no GPU.
    Any race report fails the test."""
    exe = os.path.join(ROOT, "oracle", "build", "pool_tsan")
    os.makedirs(os.path.dirname(exe), exist_ok=True)
    cc = subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-fsanitize=thread", "-pthread", "-o", exe,
                         os.path.join(ROOT, "tests", "tsan", "pool_tsan.cpp"),
                         os.path.join(ROOT, "etcd_amd", "csrc", "hbroute.cpp")], capture_output=True, text=True)
    if cc.returncode != 0 and "tsan" in (cc.stderr or "").lower():
        pytest.skip("gcc ThreadSanitizer runtime not installed")
    assert cc.returncode == 0, cc.stderr[-3000:]
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, TSAN_OPTIONS="halt_on_error=0:exitcode=66"))
    out = r.stdout + r.stderr
    assert "WARNING: ThreadSanitizer" not in out, out[-6000:]
    assert r.returncode == 0 and "pool_tsan ok" in out, out[-3000:]
