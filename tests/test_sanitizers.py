"""Sanitizer builds of the host code (CPU only, no GPU code is instrumented).

Always run (fast builds, tests/sanitize/Makefile):
  - san_host under AddressSanitizer + UndefinedBehaviorSanitizer: cv_api.cpp's host logic — key dedupe,
    the packing thread pool and its copies, the staging layout (range and compact forms), the host
    pipeline's sub-chunk plan, shard ranges, per-transaction AND, C-ABI argument guards;
  - san_host under ThreadSanitizer: the worker pool's generation handshake, par_copy, shard threads;
  - the oracle's CPU tests against an ASan + UBSan build of oracle/cv_oracle.c (python with the ASan
    runtime preloaded).
The device-logic tests against the ASan + UBSan build of tests/host_harness.cpp take ~5 min (80 s
build + 3 min of instrumented -O0 field arithmetic): `make -C tests/sanitize check` runs them with all
of the above (log in profiles/r03_sanitizers.log); here they run only when CV_SANITIZE_FULL=1.
"""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(REPO, "tests", "sanitize")
OUT = os.path.join(SAN, "_build")
CLANG = "/opt/rocm/llvm/bin/clang"


def _make(*targets):
    r = subprocess.run(["make", "-s", "-C", SAN, "-j4"] + [f"_build/{t}" for t in targets],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout + r.stderr


def _run(cmd, env_extra, timeout=600):
    env = dict(os.environ)
    env.update(env_extra)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=REPO)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    for bad in ("ERROR: AddressSanitizer", "runtime error:", "WARNING: ThreadSanitizer", "ERROR: LeakSanitizer"):
        assert bad not in out, out[-4000:]
    return out


def _asan_rt():
    return subprocess.run([CLANG, "-print-file-name=libclang_rt.asan-x86_64.so"], capture_output=True,
                          text=True, check=True).stdout.strip()


def test_host_logic_asan_ubsan():
    _make("san_host")
    out = _run([os.path.join(OUT, "san_host")],
               {"ASAN_OPTIONS": "halt_on_error=1:detect_leaks=1", "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"})
    assert "all checks passed" in out


def test_host_threads_tsan():
    _make("san_host_tsan")
    out = _run([os.path.join(OUT, "san_host_tsan"), "--threads"], {"TSAN_OPTIONS": "halt_on_error=1"})
    assert "all checks passed" in out


def _pytest_under_asan(tests, extra_env):
    env = {"LD_PRELOAD": _asan_rt(), "ASAN_OPTIONS": "detect_leaks=0:halt_on_error=1",
           "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"}
    env.update(extra_env)
    return _run(["python", "-m", "pytest", "-q", "-p", "no:cacheprovider", "-m", "not gpu"] + tests, env, timeout=900)


def test_oracle_under_asan_ubsan():
    _make("libcvoracle.so")
    out = _pytest_under_asan(["tests/test_oracle.py"], {"CV_ORACLE_LIB": os.path.join(OUT, "libcvoracle.so")})
    assert " passed" in out and " failed" not in out


@pytest.mark.skipif(os.environ.get("CV_SANITIZE_FULL") != "1",
                    reason="~5 min: set CV_SANITIZE_FULL=1 or run `make -C tests/sanitize check`")
def test_device_logic_under_asan_ubsan():
    _make("libcvhost.so", "libcvoracle.so")
    out = _pytest_under_asan(["tests/test_device_logic.py"], {"CV_HOST_LIB": os.path.join(OUT, "libcvhost.so"),
                                                              "CV_ORACLE_LIB": os.path.join(OUT, "libcvoracle.so")})
    assert " passed" in out and " failed" not in out
