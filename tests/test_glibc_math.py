"""csrc/glibc_math.h (the device restatement of glibc 2.35 __log_fma/__exp_fma/__pow_fma)
compiled for the host must agree bit for bit with the host libm (the libm the
reference's math/numpy calls resolve to) on the argument distributions of the path."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "glibc_math_host.cpp")
LIB = os.path.join(ROOT, "tests", "native", "build", "libgm_host.so")


@pytest.fixture(scope="module")
def gm():
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    subprocess.check_call(["g++", "-O2", "-std=c++20", "-fPIC", "-shared", "-ffp-contract=off", "-fno-builtin",
                           "-I" + os.path.join(ROOT, "marl-optimal-execution_amd", "csrc"), SRC, "-o", LIB, "-lm"])
    L = ctypes.CDLL(LIB)
    L.gm_check.restype = ctypes.c_int64
    L.gm_check.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                           ctypes.POINTER(ctypes.c_int64)]
    return L


def _check(L, mode, x, y=None):
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.ascontiguousarray(x if y is None else y, dtype=np.float64)
    first = ctypes.c_int64()
    bad = L.gm_check(mode, x.ctypes.data, y.ctypes.data, len(x), ctypes.byref(first))
    assert bad == 0, "first mismatch at x=%r y=%r" % (x[first.value], y[first.value])


N = 400_000


def test_log(gm):
    rs = np.random.RandomState(0)
    u = rs.rand(N)
    _check(gm, 0, 1.0 - u)                       # legacy exponential: -log(1 - u)
    _check(gm, 0, u)                             # legacy gauss: log(r2), r2 in (0, 1)
    _check(gm, 0, 1 + (rs.rand(N) - 0.5) * 0.2)  # the near-1 polynomial branch
    _check(gm, 0, np.exp(rs.uniform(-700, 700, N)))
    _check(gm, 0, rs.rand(N) * 1e-310)           # subnormal inputs


def test_exp(gm):
    rs = np.random.RandomState(1)
    _check(gm, 1, -1.67e-12 * np.floor(rs.uniform(0, 2.4e13, N)))   # SMRO exp(-gamma d)
    _check(gm, 1, rs.uniform(-750, 750, N))
    _check(gm, 1, rs.uniform(-1e-15, 1e-15, N))


def test_pow(gm):
    rs = np.random.RandomState(2)
    d = np.floor(rs.uniform(0, 2.5e13, N))
    _check(gm, 2, np.full(N, 1 - 1.67e-15), d)         # (1 - kappa) ** delta
    _check(gm, 2, np.full(N, 1 - 1.67e-15), 2 * d)
    _check(gm, 2, rs.uniform(0.05, 1, N), np.full(N, 3.0))   # LatencyModel x ** 3
    _check(gm, 2, rs.rand(N) * 0.25, np.full(N, 1 / 3.0))   # get_wake_time cube root
    _check(gm, 2, rs.uniform(0, 10, N), rs.uniform(-50, 50, N))
    _check(gm, 2, -rs.uniform(0, 10, N), np.floor(rs.uniform(-50, 50, N)))
    _check(gm, 2, rs.uniform(0, 3, N), rs.uniform(-3000, 3000, N))
