"""CPU checks of bench.py's issue model for the metric-2 launch: the sliding-window
schedule that slide_products() counts (modexp.hip modexp_slide_kernel) really
computes base^e, and the window width matches capi.cpp choose_slide_window."""
import os
import random
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fs-dkr_amd")]

import bench  # noqa: E402


def _schedule_exponent(e, w):
    """Replays the kernel's window scan on exponents instead of group elements:
    returns (the exponent the schedule builds, squarings, window products)."""
    bits = bin(e)[2:][::-1]
    bit = lambda i: bits[i] == "1"
    i = len(bits) - 1
    j = max(i - w + 1, 0)
    while not bit(j):
        j += 1
    acc = int(bits[j:i + 1][::-1], 2)          # first window: a table load
    i = j - 1
    sq = mul = 0
    while i >= 0:
        if not bit(i):
            acc, sq, i = acc * 2, sq + 1, i - 1
            continue
        j = max(i - w + 1, 0)
        while not bit(j):
            j += 1
        d = int(bits[j:i + 1][::-1], 2)
        assert d % 2 == 1 and d < (1 << w)       # an odd power from the table
        acc = (acc << (i - j + 1)) + d
        sq, mul, i = sq + i - j + 1, mul + 1, j - 1
    return acc, sq, mul


def test_slide_window_width():
    assert bench.slide_window(2048) == 7    # capi.cpp choose_slide_window: 64 + 2048/8 < 32 + 2048/7
    assert bench.slide_window(256) == 5


def test_slide_schedule_rebuilds_exponent():
    rnd = random.Random(7)
    exps = [rnd.getrandbits(2048) | (1 << 2047) | 1 for _ in range(8)] + [1, 3, (1 << 2048) - 1, 1 << 2047]
    for e in exps:
        for w in (1, 4, 6, 7):
            acc, sq, mul = _schedule_exponent(e, w)
            assert acc == e
            msq, mmul = bench.slide_products(e, w)
            # slide_products adds the table build (x R^2, x^2, 2^(w-1) - 1 products) and the exit product
            assert msq == sq + 1 and mmul == mul + 1 + (1 << (w - 1)) - 1 + 1


def test_slide_issue_below_fixed_windows():
    rnd = random.Random(1234)
    Ns = [rnd.getrandbits(2048) | 1 | (1 << 2047) for _ in range(16)]
    ratio = bench.slide_issued(144, 4, Ns) / bench.kernel_issued(144, 4, 2048)
    assert 0.94 < ratio < 0.97
