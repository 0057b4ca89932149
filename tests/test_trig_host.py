"""Host check of the env kernel's f64 sincos (drone_rl_amd/csrc/trig.h):
the same source compiled with g++ (-ffp-contract=off, real fma()) must be
within 1 ulp of numpy's sin/cos (glibc, <= 1 ulp of the true value) over
the fast range, including the quadrant boundaries and tiny arguments."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def trig(tmp_path_factory):
    so = str(tmp_path_factory.mktemp("trig") / "libtrig.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
                    os.path.join(HERE, "c", "trig_host.cpp"), "-o", so], check=True)
    lib = ctypes.CDLL(so)

    def f(x):
        x = np.ascontiguousarray(x, np.float64)
        s, c = np.empty_like(x), np.empty_like(x)
        p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        lib.trig_sincos(ctypes.c_int64(len(x)), p(x), p(s), p(c))
        return s, c
    f.lib = lib
    return f


def _ulps(a, b):
    return np.abs(a - b) / np.spacing(np.abs(b))


def test_sincos_within_one_ulp(trig):
    rng = np.random.default_rng(0)
    xs = [rng.uniform(-4, 4, 400000), rng.uniform(-400, 400, 200000),
          rng.uniform(-5e5, 5e5, 200000), rng.normal(0, 1e-3, 50000),
          (np.arange(-2000, 2000) * (np.pi / 2))[:, None] + np.array([-1e-9, 0, 1e-9]),
          np.array([0.0, -0.0, 1e-300, -1e-300, np.pi / 4, -np.pi / 4, 3 * np.pi / 4])]
    x = np.concatenate([np.ravel(v) for v in xs])
    s, c = trig(x)
    rs, rc = np.sin(x), np.cos(x)
    # near zeros of sin/cos the result is tiny: compare absolutely there
    us = np.where(np.abs(rs) > 1e-8, _ulps(s, rs), np.abs(s - rs) / 2.3e-16)
    uc = np.where(np.abs(rc) > 1e-8, _ulps(c, rc), np.abs(c - rc) / 2.3e-16)
    assert us.max() <= 1.0, (us.max(), x[us.argmax()])
    assert uc.max() <= 1.0, (uc.max(), x[uc.argmax()])
    # most results are the correctly rounded value
    assert (us == 0).mean() > 0.8 and (uc == 0).mean() > 0.8


def test_sincosf_within_two_ulp(trig):
    """The f32-state-mode sincos (sincosf_medium) against float64 sin / cos
    rounded to f32, over the fast range."""
    lib = trig.lib
    rng = np.random.default_rng(1)
    xs = [rng.uniform(-4, 4, 400000), rng.uniform(-400, 400, 200000),
          rng.uniform(-5e5, 5e5, 200000), rng.normal(0, 1e-3, 50000),
          (np.arange(-2000, 2000) * (np.pi / 2))[:, None] + np.array([-1e-6, 0, 1e-6]),
          np.array([0.0, -0.0, 1e-30, -1e-30, np.pi / 4, -np.pi / 4])]
    x = np.concatenate([np.ravel(v) for v in xs]).astype(np.float32)
    s, c = np.empty_like(x), np.empty_like(x)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    lib.trig_sincosf(ctypes.c_int64(len(x)), p(x), p(s), p(c))
    xd = x.astype(np.float64)
    rs, rc = np.sin(xd).astype(np.float32), np.cos(xd).astype(np.float32)

    def ulps(a, b):
        return np.abs(a.astype(np.float64) - b) / np.spacing(np.abs(b)).astype(np.float64)
    # near zeros of sin/cos: compare absolutely (f32 epsilon)
    us = np.where(np.abs(rs) > 1e-6, ulps(s, rs), np.abs(s - rs) / 1.2e-7)
    uc = np.where(np.abs(rc) > 1e-6, ulps(c, rc), np.abs(c - rc) / 1.2e-7)
    assert us.max() <= 2.0, (us.max(), x[us.argmax()])
    assert uc.max() <= 2.0, (uc.max(), x[uc.argmax()])
    assert (us == 0).mean() > 0.7 and (uc == 0).mean() > 0.7
