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


def test_seeding_at_the_iteration_ids_the_bench_publishes(oracle_mod):
    """utility.h:58-62 at the ids of the full-spp runs: iterations up to 4095
    (configs[4]: 4096 spp) at depth 16, 1023 (1M target, configs[2]) at depth 8
    and 5, 255 (configs[1]), for the first, middle and last pixel slots.  The
    seed word (1 << 31) | depth << 22 | iter keeps depth and iter apart up to
    iter 2^22 - 1; past it they overlap by OR, as in the reference."""
    m = 0xFFFFFFFF

    def h(a):
        a = ((a + 0x7ed55d16) + (a << 12)) & m
        a = ((a ^ 0xc761c23c) ^ (a >> 19)) & m
        a = ((a + 0x165667b1) + (a << 5)) & m
        a = ((a + 0xd3a2646c) ^ (a << 9)) & m
        a = ((a + 0xfd7046c5) + (a << 3)) & m
        a = ((a ^ 0xb55a4f09) ^ (a >> 16)) & m
        return a

    def first(iter_, index, depth):
        word = (0x80000000 | (depth << 22) | iter_) & m   # int arithmetic on 32 bits, as in the reference
        x = (h(word) ^ h(index)) % 2147483647 or 1          # thrust minstd seed: s mod m, 0 -> 1
        x = (x * 48271) % 2147483647
        return np.float32(np.float32(x - 1) / np.float32(2147483648.0))

    L = oracle_mod.lib()
    npix = 1280 * 1024
    cases = [(4095, i, d) for i in (0, npix // 2, npix - 1) for d in (16, 9, 1)]
    cases += [(1023, i, d) for i in (0, 777_777, npix - 1) for d in (8, 5, 1)]
    cases += [(1023, 2800 * 2240 - 1, 5), (255, 1_000_000, 8), (254, 3, 7), ((1 << 22) - 1, 42, 16),
              (1 << 22, 42, 16), (4095, 0x7FFFFFFF, 16)]
    for args in cases:
        assert np.float32(L.ptor_u01_first(*args)) == first(*args), args
    # depth 16 and iter 4095 occupy disjoint bits; the overlap only starts at iter 2^22
    assert (16 << 22) & 4095 == 0 and (16 << 22) & (1 << 22) == 0


def test_bmp_writer_matches_reference_layout(oracle_mod):
    img = np.zeros((2 * 3, 3), np.float32)
    img[0] = [1.0, 0.5, 0.0]      # (x=0,y=0) -> bytes 255,127,0 in x,y,z order
    b = oracle_mod.to_bmp_bytes(img, 2, 3, 1)
    assert len(b) == 54 + 18
    assert b[:2] == b"BM" and int.from_bytes(b[2:6], "little") == 72
    assert int.from_bytes(b[18:22], "little") == 2 and int.from_bytes(b[22:26], "little") == 3
    assert list(b[54:57]) == [255, 127, 0]
