"""The CPU oracle itself: math, RNG and a few hand-checked semantics of the
reference algorithm (test infrastructure checks)."""
import math

import numpy as np
import pytest


def _ulp_diff(a, b):
    a = np.float32(a).view(np.int32).astype(np.int64)
    b = np.float32(b).view(np.int32).astype(np.int64)
    return abs(int(a) - int(b))


def test_sincos_correctly_rounded(oracle_mod):
    L = oracle_mod.lib()
    xs = np.random.RandomState(0).uniform(0, 6.2831855, 4000).astype(np.float32)
    xs = np.concatenate([xs, np.float32([0.0, 1e-8, 6.2831855, 3.1415927, 1.5707964, 4.712389])])
    worst = 0
    for x in xs:
        worst = max(worst, _ulp_diff(L.ptor_sinf(float(x)), math.sin(float(x))),
                    _ulp_diff(L.ptor_cosf(float(x)), math.cos(float(x))))
    assert worst <= 1


def test_pow_correctly_rounded(oracle_mod):
    L = oracle_mod.lib()
    y = float(np.float32(1.0) / np.float32(31.0))
    xs = np.random.RandomState(1).uniform(0, 1, 4000).astype(np.float32)
    xs = np.concatenate([xs, np.float32([2 ** -24, 1e-30, 0.5, 1.0])])
    worst = max(_ulp_diff(L.ptor_powf(float(x), y), math.pow(float(x), y)) for x in xs)
    assert worst <= 1
    assert L.ptor_powf(0.0, y) == 0.0
    assert L.ptor_powf(1.0, y) == 1.0


def test_util_hash_known_values(oracle_mod):
    # utilHash (utility.h:43-53) evaluated independently in Python
    def h(a):
        m = 0xFFFFFFFF
        a = ((a + 0x7ed55d16) + (a << 12)) & m
        a = ((a ^ 0xc761c23c) ^ (a >> 19)) & m
        a = ((a + 0x165667b1) + (a << 5)) & m
        a = ((a + 0xd3a2646c) ^ (a << 9)) & m
        a = ((a + 0xfd7046c5) + (a << 3)) & m
        a = ((a ^ 0xb55a4f09) ^ (a >> 16)) & m
        return a
    L = oracle_mod.lib()
    for a in [0, 1, 2, 12345, 0x80000000, 0xFFFFFFFF, 0x80000000 | (5 << 22) | 17]:
        assert L.ptor_hash(a) == h(a)


def test_minstd_uniform_first_draw(oracle_mod):
    # makeSeededRandomEngine + thrust minstd_rand + uniform_real_distribution<float>(0,1)
    def first(iter_, index, depth):
        def h(a):
            m = 0xFFFFFFFF
            a = ((a + 0x7ed55d16) + (a << 12)) & m
            a = ((a ^ 0xc761c23c) ^ (a >> 19)) & m
            a = ((a + 0x165667b1) + (a << 5)) & m
            a = ((a + 0xd3a2646c) ^ (a << 9)) & m
            a = ((a + 0xfd7046c5) + (a << 3)) & m
            a = ((a ^ 0xb55a4f09) ^ (a >> 16)) & m
            return a
        s = h(0x80000000 | (depth << 22) | iter_) ^ h(index)
        x = s % 2147483647 or 1
        x = (x * 48271) % 2147483647
        return np.float32(np.float32(x - 1) / np.float32(2147483648.0))
    L = oracle_mod.lib()
    for args in [(0, 0, 5), (1, 77, 4), (499, 799999, 1), (3, 123456, 16)]:
        assert np.float32(L.ptor_u01_first(*args)) == first(*args)


def test_bmp_writer_matches_reference_layout(oracle_mod):
    img = np.zeros((2 * 3, 3), np.float32)
    img[0] = [1.0, 0.5, 0.0]      # (x=0,y=0) -> bytes 255,127,0 in x,y,z order
    b = oracle_mod.to_bmp_bytes(img, 2, 3, 1)
    assert len(b) == 54 + 18
    assert b[:2] == b"BM" and int.from_bytes(b[2:6], "little") == 72
    assert int.from_bytes(b[18:22], "little") == 2 and int.from_bytes(b[22:26], "little") == 3
    assert list(b[54:57]) == [255, 127, 0]
