"""gr_math.h (shared by kernel and oracle) vs float64 references, on the CPU build."""
import numpy as np
import pytest

import oracle


def ulp_err(got, ref):
    ref32 = ref.astype(np.float32)
    spacing = np.spacing(np.abs(ref32)).astype(np.float64)
    return np.abs(got.astype(np.float64) - ref) / spacing


RNG = np.random.default_rng(0)
CASES = [
    (0, np.exp, RNG.uniform(-20, 20, 20000), 4),
    (1, np.tanh, np.concatenate([RNG.uniform(-10, 10, 20000), RNG.normal(0, 0.1, 5000)]), 4),
    (2, np.log, np.concatenate([RNG.uniform(1e-7, 1, 20000), np.float32(5.96e-8) * np.arange(1, 100)]), 4),
]


@pytest.mark.parametrize("fn,ref,x,max_ulp", CASES)
def test_unary(fn, ref, x, max_ulp):
    x = x.astype(np.float32)
    got = oracle.test_math(fn, x)
    err = ulp_err(got, ref(x.astype(np.float64)))
    assert err.max() <= max_ulp, (err.max(), x[err.argmax()])


def test_sincos_abs_error():
    x = np.concatenate([RNG.uniform(-7, 7, 20000), RNG.uniform(0, 6.2832, 5000)]).astype(np.float32)
    s = oracle.test_math(3, x)
    c = oracle.test_math(4, x)
    xd = x.astype(np.float64)
    assert np.abs(s - np.sin(xd)).max() < 2.5e-7
    assert np.abs(c - np.cos(xd)).max() < 2.5e-7


def test_atan2():
    y = RNG.uniform(-5, 5, 20000).astype(np.float32)
    x = RNG.uniform(-5, 5, 20000).astype(np.float32)
    got = oracle.test_math(5, y, x)
    assert np.abs(got - np.arctan2(y.astype(np.float64), x.astype(np.float64))).max() < 5e-7
    assert oracle.test_math(5, np.zeros(1, np.float32), np.zeros(1, np.float32))[0] == 0.0


def test_sqrt_div_correctly_rounded():
    x = RNG.uniform(0, 100, 10000).astype(np.float32)
    y = RNG.uniform(0.1, 100, 10000).astype(np.float32)
    assert np.array_equal(oracle.test_math(6, x), np.sqrt(x))
    assert np.array_equal(oracle.test_math(7, x, y), x / y)
