"""The 64-bit column bound of the lane-distributed Montgomery product
(csrc/mont29.hpp, Mont29::NORM_IN_CYCLE): enumerate the products every column
receives during its L-row stay in a lane -- one m*n per row, and in squaring
rows the cyclic-tournament a*b slots (sq_raw / sq_dbl) -- and check the bound
the kernel relies on: a column gains < (L + 1) 2^59.01 over one stay, so shapes
with L <= 30 need no carry folds inside a product cycle.  Pure enumeration of
the kernel's slot rule, no GPU."""
import math

import pytest

MAX_AB = math.log2((2 ** 29 + 127) ** 2)   # almost-Montgomery digits <= 2^29 + 127
MAX_MN = 58.0                              # quotient digit < 2^29, modulus digits < 2^29


def sq_raw(L, d):
    return d == 0 or (L % 2 == 0 and d == L // 2)


def sq_dbl(L, d):
    return d > 0 and (d <= L // 2 if L % 2 == 1 else d < L // 2)


def stay_weights(L, G, square):
    """max over (column, lane) of the a*b and m*n product counts (a*b doubled
    counts 2) a column collects while it is in one lane, over a whole product
    (KD = G L rows)"""
    KD = G * L
    ab, mn = {}, {}
    for r in range(KD):
        R = r % L
        for g in range(G):
            for j in range(L):
                c = r + g * L + j          # the logical column of slot j in lane g at row r
                key = (c, g)
                mn[key] = mn.get(key, 0) + 1
                if square:
                    d = (j - R) % L
                    w = 2 if sq_dbl(L, d) else 1 if sq_raw(L, d) else 0
                else:
                    w = 1
                ab[key] = ab.get(key, 0) + w
    return max(ab.values()), max(mn.values()), max(ab[k] + mn[k] for k in ab)


@pytest.mark.parametrize("L,G", [(9, 4), (18, 4), (27, 4), (27, 8), (30, 2), (31, 2), (36, 4)])
def test_stay_bound(L, G):
    for square in (False, True):
        ab, mn, tot = stay_weights(L, G, square)
        assert mn == L                      # one m*n product per row of the stay
        assert ab <= L + 2                  # the tournament never exceeds L + 2 a*b units
        bound = math.log2(ab * 2 ** MAX_AB + mn * 2 ** MAX_MN + 2 ** 29 + 2 ** 35)
        if L <= 30:
            assert bound < 64, (L, square, bound)   # NORM_IN_CYCLE = L > 30: no folds needed


def test_tournament_counts_every_pair_twice():
    """the squaring slots issue each unordered pair twice and each diagonal once
    (the identity the rows rely on: sum over rows of the slots = a^2)"""
    for L in (9, 18, 27, 36):
        cnt = {}
        for R in range(L):
            for j in range(L):
                d = (j - R) % L
                w = 2 if sq_dbl(L, d) else 1 if sq_raw(L, d) else 0
                key = (min(R, j), max(R, j))
                cnt[key] = cnt.get(key, 0) + w
        assert all(v == (1 if a == b else 2) for (a, b), v in cnt.items()), L
