"""String.valueOf of float / double partition keys: Java 8 Float.toString / Double.toString, three
restatements (the engine's csrc/java_fmt.h through the host K_gen build, the oracle's
java_fp_string, tests/java_fmt.py) checked against each other on random and structured bit
patterns, and against outputs of the JDK the reference targets that its documentation and bug
tracker record (no JVM here to run): the E-notation thresholds 10^-3 / 10^7, subnormal minima,
NaN / Infinity / -0.0, and JDK-4511638's non-shortest 2.0E23 -> 1.9999999999999998E23."""
import ctypes
import random

import numpy as np
import pytest

import java_fmt as J
from harness import App, oracle_lib
from kgen_host import lib as kgen_lib

KNOWN_F = [(0.1, "0.1"), (1.0e10, "1.0E10"), (1.0, "1.0"), (100.0, "100.0"), (1.0e7, "1.0E7"),
           (1234567.0, "1234567.0"), (0.001, "0.001"), (1.0e-4, "1.0E-4"), (-2.5, "-2.5"),
           (3.4028235e38, "3.4028235E38"), (1.4e-45, "1.4E-45"), (1.17549435e-38, "1.17549435E-38"),
           (0.0, "0.0"), (-0.0, "-0.0"), (16777216.0, "1.6777216E7"), (0.33333334, "0.33333334"),
           (float("inf"), "Infinity"), (float("-inf"), "-Infinity")]
KNOWN_D = [(0.1, "0.1"), (1.0 / 3, "0.3333333333333333"), (100.0, "100.0"), (1.0e7, "1.0E7"),
           (4.9e-324, "4.9E-324"), (1.7976931348623157e308, "1.7976931348623157E308"), (0.001, "0.001"),
           (1.0e-4, "1.0E-4"), (2.2250738585072014e-308, "2.2250738585072014E-308"),
           (123456789.0, "1.23456789E8"), (0.30000000000000004, "0.30000000000000004"),
           (2.0e23, "1.9999999999999998E23"), (-0.0, "-0.0"), (float(np.float32(0.1)), "0.10000000149011612")]


def _c(fn, bits, is_double):
    buf = ctypes.create_string_buffer(64)
    fn.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
    n = fn(bits, int(is_double), buf, 64)
    assert n > 0
    return buf.value.decode()


def _all(bits, is_double):
    p = J.double_to_string(bits) if is_double else J.float_to_string(bits)
    return p, _c(oracle_lib().oracle_java_fmt, bits, is_double), _c(kgen_lib().kgh_java_fmt, bits, is_double)


def test_known_jdk_outputs():
    for v, want in KNOWN_F:
        assert set(_all(J.f32(v), False)) == {want}, v
    for v, want in KNOWN_D:
        assert set(_all(J.f64(v), True)) == {want}, v
    assert set(_all(0x7FC00000, False)) == {"NaN"} and set(_all(0x7FF8000000000000, True)) == {"NaN"}


@pytest.mark.parametrize("is_double", [False, True])
def test_three_restatements_agree(is_double):
    rng = random.Random(11 + is_double)
    vals = [rng.getrandbits(64 if is_double else 32) for _ in range(6000)]
    for e in range(-60, 60):
        for m in (1, 2, 3, 5, 9.5, 1.1, 0.3, 7.25):
            x = m * 10.0 ** e
            vals.append(J.f64(x) if is_double else J.f32(float(np.float32(x))) if abs(x) < 3e38 else 0)
    for v in vals:
        a, b, c = _all(v, is_double)
        assert a == b == c, hex(v)
        if a not in ("NaN", "Infinity", "-Infinity"):  # the text parses back to the same value
            back = float(a)
            assert (J.f64(back) if is_double else J.f32(float(np.float32(back)))) == v, (hex(v), a)


@pytest.mark.parametrize("key_type", ["float", "double"])
@pytest.mark.parametrize("seed", range(4))
def test_float_key_fanout_host_build(seed, key_type):
    """A stream the partition does not key, the partition keyed by float / double values: the host
    build of K_gen (java_fmt.h) orders the keys like the oracle (java_fp_string)."""
    from fuzz_apps import fanout_app, fanout_events
    from kgen_host import KGenHostEngine
    src = fanout_app(seed, key_type)
    o, g = App(src), App(src, engine_factory=lambda blob: KGenHostEngine(blob, R=4096, N=4096, LC=4096))
    for stream, row, t in fanout_events(seed, keys=24 + 5 * seed, key_type=key_type):
        o.send(stream, [row], [t])
        g.send(stream, [row], [t])
    assert len(o.matches) > 20
    assert g.matches == o.matches
