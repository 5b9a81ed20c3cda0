"""The one-wave cooperative modexp (csrc/coop.hip: separated Montgomery over
28-bit digits, one instance per wave, sliding windows over its own exponent),
selected by the context's modexp group FSDKR_COOP_GROUP = 256, bit-exact
against Python's pow: 2048- and 4096-bit odd moduli (GA's N^2 and random),
exponents of 0 / 1 / 2 / a few bits / 256 / 2048 bits, bases 0, 1, N - 1 and
above N, moduli with high zero limbs."""
import random

import pytest

pytestmark = pytest.mark.gpu

COOP = 256


def _run(ctx, bases, exps, mods, idx, limbs):
    ctx.set_modexp_group(COOP)
    try:
        return ctx.modexp_batch(bases, exps, mods, idx, limbs)
    finally:
        ctx.set_modexp_group(0)


@pytest.mark.parametrize("limbs", [64, 128])
def test_coop_random(gpu_ctx, limbs):
    rng = random.Random(0xC00 + limbs)
    bits = 32 * limbs
    mods = [rng.getrandbits(bits) | 1 | (1 << (bits - 1)) for _ in range(5)]
    mods.append(rng.getrandbits(bits - 70) | 1)                 # high limbs zero
    if limbs == 128:
        n = rng.getrandbits(2048) | 1 | (1 << 2047)
        mods.append(n * n)                                        # GA's modulus N^2
    count = 96
    idx = [rng.randrange(len(mods)) for _ in range(count)]
    bases = [rng.getrandbits(bits) for _ in range(count)]
    ebits = [0, 1, 2, 3, 17, 256, 2048, bits]
    exps = [rng.getrandbits(ebits[i % len(ebits)]) if ebits[i % len(ebits)] else 0 for i in range(count)]
    exps[5] = 1
    exps[6] = 2
    bases[7] = 0
    bases[8] = 1
    bases[9] = mods[idx[9]] - 1
    got = _run(gpu_ctx, bases, exps, mods, idx, limbs)
    want = [pow(b, e, mods[k]) for b, e, k in zip(bases, exps, idx)]
    bad = [i for i in range(count) if got[i] != want[i]]
    assert not bad, (bad[:5], limbs)


def test_coop_ga_shape(gpu_ctx):
    """GA's chains: s^N mod N^2 for 2 x 64 bases per receiver (a shard's slice)."""
    rng = random.Random(7)
    ns = [rng.getrandbits(2048) | 1 | (1 << 2047) for _ in range(4)]
    mods = [n * n for n in ns]
    idx = [i // 32 for i in range(128)]
    bases = [rng.getrandbits(2048) for _ in range(128)]
    exps = [ns[k] for k in idx]
    got = _run(gpu_ctx, bases, exps, mods, idx, 128)
    assert got == [pow(b, e, mods[k]) for b, e, k in zip(bases, exps, idx)]
