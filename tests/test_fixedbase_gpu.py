"""Fixed-base (BGMW) exponentiation engine vs Python pow: bit-exact on shared
bases with exponents of every size class collect() uses (0, 1, 256, 769, 2048,
2816 bits), unreduced bases, several moduli per launch, and every lanes-per-
instance variant."""
import random

import pytest

pytestmark = pytest.mark.gpu


def _case(limbs, seed, n_bases=5, per_base=40):
    rnd = random.Random(seed)
    mods = [rnd.getrandbits(32 * limbs) | 1 | (1 << (32 * limbs - 1)) for _ in range(3)]
    mods.append(rnd.getrandbits(16 * limbs) | 1 | (1 << (16 * limbs - 1)))     # half-width modulus in a wide slot
    bmod = [k % len(mods) for k in range(n_bases)]
    bases = [rnd.getrandbits(32 * limbs) for _ in range(n_bases)]                  # unreduced for the small modulus
    bases[0] = 0
    bases[1] = 1
    sizes = [0, 1, 2, 63, 256, 769, 2048, 2816]
    bidx, exps = [], []
    for b in range(n_bases):
        for k in range(per_base):
            bits = sizes[k % len(sizes)]
            e = rnd.getrandbits(bits) if bits > 2 else bits
            if k % 11 == 5:
                e = (1 << bits) - 1 if bits else 0          # all-ones windows
            bidx.append(b)
            exps.append(e)
    return bases, bmod, mods, bidx, exps


@pytest.mark.parametrize("limbs", [64, 96])
@pytest.mark.parametrize("group", [0, 2, 4, 8])
def test_fixed_base_matches_pow(gpu_ctx, limbs, group):
    if limbs == 96 and group not in (0, 4):
        pytest.skip("3072-bit moduli run with 4 lanes per instance")
    bases, bmod, mods, bidx, exps = _case(limbs, 1000 + limbs + group)
    gpu_ctx.set_modexp_group(group)
    try:
        out = gpu_ctx.fixed_base_modexp(bases, bmod, mods, bidx, exps, limbs)
    finally:
        gpu_ctx.set_modexp_group(0)
    want = [pow(bases[b], e, mods[bmod[b]]) for b, e in zip(bidx, exps)]
    bad = [k for k in range(len(want)) if out[k] != want[k]]
    assert not bad, f"{len(bad)} mismatches, first {bad[:5]}"


def test_fixed_base_large_batch(gpu_ctx):
    """Ring-Pedersen shape: 16 bases x 256 exponents of 2048 bits."""
    rnd = random.Random(7)
    mods = [rnd.getrandbits(2048) | 1 | (1 << 2047) for _ in range(16)]
    bases = [rnd.getrandbits(2047) for _ in range(16)]
    bidx = [k // 256 for k in range(16 * 256)]
    exps = [rnd.getrandbits(2048) for _ in bidx]
    out = gpu_ctx.fixed_base_modexp(bases, list(range(16)), mods, bidx, exps, 64)
    for k in range(0, len(exps), 97):
        assert out[k] == pow(bases[bidx[k]], exps[k], mods[bidx[k]])


@pytest.mark.parametrize("top_bits", [3, 40, 256, 8200])
def test_fixed_base_window_widths(gpu_ctx, top_bits):
    """Every window width of fb_window (w = 1 .. 8 by the largest exponent): the
    schedule's 2^w digit bins span one to four 64-lane scan passes of fb_sched."""
    rnd = random.Random(top_bits)
    mods = [rnd.getrandbits(2048) | 1 | (1 << 2047) for _ in range(2)]
    bases = [rnd.getrandbits(2048) % mods[k % 2] for k in range(3)]
    bidx, exps = [], []
    for k in range(96):
        b = k % 3
        bits = [0, 1, top_bits // 2, top_bits][k % 4]
        e = rnd.getrandbits(bits) if bits > 1 else bits
        if k % 7 == 3:
            e = (1 << top_bits) - 1                         # every digit at its maximum
        bidx.append(b)
        exps.append(e)
    out = gpu_ctx.fixed_base_modexp(bases, [0, 1, 0], mods, bidx, exps, 64)
    want = [pow(bases[b], e, mods[[0, 1, 0][b]]) for b, e in zip(bidx, exps)]
    bad = [k for k in range(len(want)) if out[k] != want[k]]
    assert not bad, f"{len(bad)} mismatches, first {bad[:5]}"


@pytest.fixture
def comb_mode(gpu_ctx):
    """The fixed-base engine for the duration of a test: 0 BGMW only
    (FSDKR_CFG_FB_BGMW), 2 a comb wherever one fits (FSDKR_CFG_FB_COMB), 1 chosen."""
    from fsdkr._native import FSDKR_CFG_FB_BGMW, FSDKR_CFG_FB_COMB
    old = gpu_ctx.flags

    def set_mode(m):
        base = old & ~(FSDKR_CFG_FB_BGMW | FSDKR_CFG_FB_COMB)
        gpu_ctx.set_flags(base | {0: FSDKR_CFG_FB_BGMW, 1: 0, 2: FSDKR_CFG_FB_COMB}[m])
    yield set_mode
    gpu_ctx.set_flags(old)


@pytest.mark.parametrize("limbs", [64, 96])
@pytest.mark.parametrize("mode", [0, 2])
def test_comb_matches_pow(gpu_ctx, comb_mode, limbs, mode):
    """Lim-Lee comb (comb.hip, forced by FSDKR_CFG_FB_COMB) and BGMW (FSDKR_CFG_FB_BGMW) on the
    mixed case: zero / one / unreduced bases, half-width modulus, exponents of
    0 .. 2816 bits including all-ones rows and columns of the bit array."""
    comb_mode(mode)
    bases, bmod, mods, bidx, exps = _case(limbs, 3000 + limbs + mode, per_base=48)
    out = gpu_ctx.fixed_base_modexp(bases, bmod, mods, bidx, exps, limbs)
    want = [pow(bases[b], e, mods[bmod[b]]) for b, e in zip(bidx, exps)]
    bad = [k for k in range(len(want)) if out[k] != want[k]]
    assert not bad, f"{len(bad)} mismatches, first {bad[:5]}"


@pytest.mark.parametrize("limbs", [64, 96])
def test_comb_ring_pedersen_shape(gpu_ctx, comb_mode, limbs):
    """M = 256 exponents of the modulus' size per base (ring-Pedersen T^Z): the
    default mode takes the comb here; every result checked."""
    comb_mode(1)
    rnd = random.Random(limbs)
    bits = 32 * limbs
    mods = [rnd.getrandbits(bits) | 1 | (1 << (bits - 1)) for _ in range(3)]
    bases = [rnd.getrandbits(bits) % mods[k] for k in range(3)]
    bidx = [k // 256 for k in range(3 * 256)]
    exps = [rnd.getrandbits(bits) for _ in bidx]
    exps[5], exps[300], exps[600] = 0, (1 << bits) - 1, 1
    out = gpu_ctx.fixed_base_modexp(bases, [0, 1, 2], mods, bidx, exps, limbs)
    want = [pow(bases[b], e, mods[b]) for b, e in zip(bidx, exps)]
    bad = [k for k in range(len(want)) if out[k] != want[k]]
    assert not bad, f"{len(bad)} mismatches, first {bad[:5]}"
