"""The GPU response writer's number formatting (reporter_amd/csrc/pyrepr.h,
compiled for the host here): py_repr must be Python's float repr (json.dumps
writes floats with it, py/reporter_service.py's response bodies) for every
double it does not hand back (-1: the host writer's), and py_round3 must be
report()'s round(x, 3) as report.cpp implements it.  Epoch times with
fractions, km lengths, powers of two and ten and their neighbours, random
doubles over the supported exponent range."""
import ctypes as C
import math
import random
import struct

import numpy as np
import pytest

from reporter_amd import _lib


def _L():
    L = _lib.lib()
    L.otm_debug_py_repr.argtypes = [C.c_double, C.c_char_p]
    L.otm_debug_py_repr.restype = C.c_int
    L.otm_debug_py_round3.argtypes = [C.c_double, C.POINTER(C.c_double)]
    L.otm_debug_py_round3.restype = C.c_int
    return L


def _repr(L, d):
    buf = C.create_string_buffer(64)
    n = L.otm_debug_py_repr(d, buf)
    return None if n < 0 else buf.raw[:n].decode()


def _values(rng, n):
    vals = [0.0, -0.0, 1.0, -1.0, 0.5, 0.1, 0.2, 0.3, 1e15, 9007199254740991.0, 4503599627370496.0,
            2.0 ** -10, 1462826734.0, 1462826734.5, 0.001, 0.999, 1.234, 12.345]
    for e in range(-10, 53):
        p = 2.0 ** e
        vals += [p, math.nextafter(p, 0.0), math.nextafter(p, math.inf)]
    for k in range(-3, 16):
        p = 10.0 ** k
        vals += [p, math.nextafter(p, 0.0), math.nextafter(p, math.inf)]
    for _ in range(n):
        vals.append(1462826734.0 + rng.random() * 1e5)               # epoch times with fractions
        vals.append(rng.randint(0, 10 ** 6) / 1000.0)                 # km lengths (3 decimals)
        vals.append(rng.randint(1, 10 ** 7) * 0.001)                  # metres x 0.001
        vals.append(math.ldexp(rng.random() + 0.5, rng.randint(-9, 52)))  # any exponent in range
        vals.append(struct.unpack("<d", struct.pack("<Q", rng.getrandbits(52) | (rng.randint(1013, 1074) << 52)))[0])
    return vals


def test_py_repr_matches_python():
    L = _L()
    rng = random.Random(77)
    n_host = 0
    vals = _values(rng, 40000)
    for v in vals:
        got = _repr(L, v)
        if got is None:
            n_host += 1
            assert not (2.0 ** -10 <= abs(v) < 2.0 ** 52), v  # only out-of-range values go to the host
            continue
        assert got == repr(v), (v, got)
    assert n_host < len(vals) // 100


def test_py_repr_hands_back_out_of_range():
    L = _L()
    for v in (2.0 ** 52, 2.0 ** 53, 1e300, 1e-300, 2.0 ** -11, float("inf"), float("nan"), 5e-324):
        assert _repr(L, v) is None, v


def test_py_round3_matches_report_rounding():
    L = _L()
    rng = random.Random(78)
    xs = [0.0, 0.0005, 0.0015, 0.0025, 1.0005, 2.675, 1.2345, 0.001]
    xs += [rng.randint(0, 10 ** 7) * 0.001 for _ in range(20000)]
    xs += [rng.random() * 1000.0 for _ in range(20000)]
    out = C.c_double()
    for x in xs:
        assert L.otm_debug_py_round3(x, C.byref(out)) == 1
        want = float("%.3f" % x)
        assert out.value == want, (x, out.value, want)
        assert round(x, 3) == want
