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


@pytest.mark.parametrize("limbs", [64, 128])
@pytest.mark.parametrize("kind", ["units", "one_non_unit", "zero", "singletons"])
def test_simultaneous_inverse_groups(gpu_ctx, limbs, kind):
    """Instances sharing a modulus are inverted together (Montgomery's trick,
    inverse_batch_kernel: prefix products, ONE binary-GCD inverse, a backward
    pass): exact inverses and unit flags equal pow(y, -1, m), including a group
    whose product is not a unit (every element of it then inverted on its own),
    y = 0 and groups of one.  FSDKR_CFG_INV_EACH (one inverse each) gives the
    same results."""
    from fsdkr._native import FSDKR_CFG_INV_EACH
    rnd = random.Random(1000 * limbs + len(kind))
    bits = 32 * limbs
    mods = [_case(rnd, bits, "rsa2" if limbs == 128 else "odd") for _ in range(5)]
    # modulus 2 with a small factor 3: its group gets a non-unit in "one_non_unit"
    mods[2] = 3 * (rnd.getrandbits(bits - 3) | 1 | (1 << (bits - 4)))
    ys, ms = [], []
    for k in range(5 * 37 if kind != "singletons" else 5):
        m = mods[k % 5]
        ys.append(rnd.randrange(1, m))
        ms.append(m)
    if kind == "one_non_unit":
        ys[7] = 3 * rnd.randrange(1, mods[2] // 3)   # k = 7: modulus 2's group
    if kind == "zero":
        ys[3] = 0
    got = gpu_ctx.mod_inverse(ys, ms, limbs)
    old = gpu_ctx.set_flags(gpu_ctx.flags | FSDKR_CFG_INV_EACH)
    try:
        ref = gpu_ctx.mod_inverse(ys, ms, limbs)
    finally:
        gpu_ctx.set_flags(old)
    for k, (y, m, g) in enumerate(zip(ys, ms, got)):
        try:
            want = pow(y, -1, m)
        except ValueError:
            want = None
        assert g == want, (kind, k)
    assert got == ref
