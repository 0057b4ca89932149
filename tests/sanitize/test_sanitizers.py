"""Host-code sanitizer runs (SURVEY.md 5 "race detection / sanitizers";
CPU only -- GPU-side ASan is not available on the MI355X pool).

The CPU oracle (gcc ASan + UBSan) runs the golden-vector oracle tests, and
the product library's host code (clang ASan + UBSan via -Xarch_host: ABI
argument validation, error plumbing, handle bookkeeping) runs the no-GPU ABI
tests, each in a child process with its sanitizer runtime preloaded.  Any
sanitizer report fails the test.  Builds: tests/sanitize/build.sh (into
build/asan/, rebuilt when a source is newer)."""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.join(ROOT, "build", "asan")
BUILD = os.path.join(ROOT, "tests", "sanitize", "build.sh")


def _stale(target, sources):
    return not os.path.exists(target) or \
        max(os.path.getmtime(s) for s in sources) > os.path.getmtime(target)


def _build(what, target, sources):
    if _stale(target, sources):
        subprocess.run(["bash", BUILD, what], check=True, cwd=ROOT, capture_output=True)


def _run(preload, extra_env, tests):
    env = dict(os.environ, LD_PRELOAD=preload,
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:detect_odr_violation=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", **extra_env)
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider",
                        "-m", "not gpu", *tests], env=env, cwd=ROOT, capture_output=True,
                       text=True, timeout=600)
    out = r.stdout + r.stderr
    assert "AddressSanitizer" not in out and "runtime error:" not in out, out[-4000:]
    assert r.returncode == 0, out[-4000:]
    return out


def test_oracle_under_asan_ubsan():
    asan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True,
                          text=True).stdout.strip()
    if not os.path.isabs(asan) or not os.path.exists(asan):
        pytest.skip("gcc's libasan not available")
    target = os.path.join(OUT, "liboracle.so")
    _build("oracle", target, glob.glob(os.path.join(ROOT, "oracle", "*.c")) + [BUILD])
    out = _run(asan, {"ORACLE_LIB": target}, ["tests/test_oracle.py"])
    assert "passed" in out


def test_product_host_code_under_asan_ubsan():
    rt = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    if not rt or not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("clang ASan runtime / hipcc not available")
    target = os.path.join(OUT, "libdronerl.so")
    srcs = glob.glob(os.path.join(ROOT, "drone_rl_amd", "csrc", "*")) + \
        [os.path.join(ROOT, "include", "dronerl.h"), BUILD]
    _build("product", target, srcs)
    out = _run(rt[-1], {"DRONERL_LIB": target}, ["tests/test_abi.py"])
    assert "passed" in out
