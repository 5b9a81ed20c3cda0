"""GPU modular inverse (inverse.hip, Pornin binary GCD over G cooperating
lanes) against Python's pow(y, -1, m): units, non-units, edge values."""
import random

import pytest

pytestmark = pytest.mark.gpu


def _case(rnd, bits, kind):
    if kind == "rsa2":            # N^2 of a 2048-bit-class N (4096-bit modulus)
        n = rnd.getrandbits(bits // 2) | 1 | (1 << (bits // 2 - 1))
        return n * n
    return rnd.getrandbits(bits) | 1 | (1 << (bits - 1))


@pytest.mark.parametrize("limbs", [64, 96, 128, 192])
def test_inverse_matches_python(gpu_ctx, limbs):
    rnd = random.Random(limbs)
    bits = 32 * limbs
    ys, ms = [], []
    for k in range(300):
        m = _case(rnd, bits, "rsa2" if k % 3 == 0 else "odd")
        if k % 50 == 0:
            m = _case(rnd, bits - rnd.randrange(1, 200), "odd")       # shorter moduli in a wide slot
        r = k % 10
        if r == 0:
            y = 0
        elif r == 1:
            y = 1
        elif r == 2:
            y = m - 1
        elif r == 3:                                                 # non-unit: shares a factor
            f = rnd.getrandbits(64) | 1
            m = m - m % f + f if (m - m % f + f) % 2 else m - m % f + 2 * f
            m |= 1
            y = (f * rnd.getrandbits(bits // 2)) % m
        elif r == 4:
            y = rnd.getrandbits(rnd.randrange(1, 64))               # tiny y
        else:
            y = rnd.randrange(m)
        ys.append(y)
        ms.append(m)
    got = gpu_ctx.mod_inverse(ys, ms, limbs)
    for k, (y, m, g) in enumerate(zip(ys, ms, got)):
        try:
            want = pow(y, -1, m)
        except ValueError:
            want = None
        if m == 1:
            continue
        assert g == want, (k, hex(y)[:40], hex(m)[:40])
