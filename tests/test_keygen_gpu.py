"""GPU key generation against the oracle: Miller-Rabin verdicts
of fsdkr_miller_rabin bit for bit against oracle.keygen.strong_probable_prime
(strong pseudoprimes, Carmichael numbers, primes, semiprimes, long 2-adic
tails), and the batched prime walk / keypairs / correct-key proofs against the
oracle for the same draws."""
import random

import pytest

from oracle import keygen as ok
from oracle import paillier, zk_paillier
from oracle.rng import Rng

pytestmark = pytest.mark.gpu


def _cases(rnd, bits):
    """(candidate, base) pairs of one width class."""
    out = []
    p1 = Rng(("mrp", bits)).prime(bits // 2)
    p2 = Rng(("mrq", bits)).prime(bits // 2)
    pr = Rng(("mrr", bits)).prime(bits)
    for c in (pr, p1 * p2, p1 * p1):
        for b in (2, 3, 1, c - 1, c - 2, rnd.randrange(2, c - 1), rnd.randrange(2, c - 1)):
            out.append((c, b))
    for _ in range(40):                                   # random odd numbers, random bases
        c = rnd.getrandbits(bits) | 1 | (1 << (bits - 1))
        out.append((c, rnd.randrange(2, c - 1)))
    for s in (1, 2, 17, 64, 200):                         # long 2-adic tails: c = 1 + d 2^s
        for _ in range(3):
            d = rnd.getrandbits(bits - s - 1) | 1 | (1 << (bits - s - 2))
            c = 1 + (d << s)
            out.append((c, rnd.randrange(2, c - 1)))
    # a prime with a long 2-adic tail: walk k 2^200 + 1 until prime
    k = (1 << (bits - 202)) | 1
    while not ok.is_probable_prime((k << 200) + 1):
        k += 2
    c = (k << 200) + 1
    out += [(c, b) for b in (2, 3, 5, rnd.randrange(2, c - 1))]
    return out


@pytest.mark.parametrize("limbs", [32, 64, 96])
def test_miller_rabin_matches_oracle(gpu_ctx, limbs):
    rnd = random.Random(limbs)
    cases = _cases(rnd, 32 * limbs)
    # the small strong pseudoprimes and Carmichael numbers ride in every width
    for n, liars, w in [(2047, (2,), 3), (1373653, (2, 3), 5), (3215031751, (2, 3, 5, 7), 11),
                        (2152302898747, (2, 3, 5, 7, 11), 13)]:
        cases += [(n, b) for b in liars + (w,)]
    cases += [(n, b) for n in (561, 41041, 825265) for b in (2, 3, 5)] + [(5, 2), (7, 3), (9, 2)]
    got = gpu_ctx.miller_rabin([c for c, _ in cases], [b for _, b in cases], limbs)
    want = [1 if ok.strong_probable_prime(c, b) else 0 for c, b in cases]
    bad = [k for k in range(len(cases)) if got[k] != want[k]]
    assert not bad, f"{len(bad)} mismatches, first {cases[bad[0]]}: gpu {got[bad[0]]}"
    assert sum(want) > 20 and len(want) - sum(want) > 20


def test_miller_rabin_rejects_bad_input(gpu_ctx):
    from fsdkr._native import FsdkrError
    with pytest.raises(FsdkrError):
        gpu_ctx.miller_rabin([10], [3], 32)          # even
    with pytest.raises(FsdkrError):
        gpu_ctx.miller_rabin([3], [2], 32)           # below 5
    with pytest.raises(FsdkrError):
        gpu_ctx.miller_rabin([7], [2], 48)           # no such width


@pytest.mark.parametrize("bits,count,span", [(512, 6, 0), (1024, 3, 0), (256, 8, 24)])
def test_sample_primes_match_oracle(gpu_ctx, bits, count, span):
    """fsdkr_sample_primes (the C-ABI prime walk) against the oracle's walk for the same draws."""
    from fsdkr import keygen
    got = keygen.sample_primes(gpu_ctx, Rng(("sp", bits)), bits, count, span=span or None)
    want = ok.sample_primes(Rng(("sp", bits)), bits, count, span=span)
    assert got == want


@pytest.mark.parametrize("span,window", [(0, 0), (24, 4), (8, 3)])
def test_walk_schedule_matches_oracle(gpu_ctx, span, window):
    """Short walks (span 8/24) and small windows fail often, exercising the redraw
    passes and the passer queue of the C walk; the primes equal the oracle's."""
    from fsdkr import keygen
    got = keygen.sample_primes(gpu_ctx, Rng(("sched", span)), 192, 10, window=window or None, span=span or None)
    want = ok.sample_primes(Rng(("sched", span)), 192, 10, span=span)
    assert got == want


def test_sample_primes_draw_errors(gpu_ctx):
    """An RNG that raises aborts the walk with that exception; bad widths are refused."""
    from fsdkr import keygen
    from fsdkr._native import FsdkrError

    class Broken:
        def bits(self, k):
            raise OSError("entropy source gone")
    with pytest.raises(OSError):
        keygen.sample_primes(gpu_ctx, Broken(), 512, 2)
    with pytest.raises(FsdkrError):
        gpu_ctx.sample_primes(Rng("x").bits, 4096, 1)   # 128-limb candidates: no MR shape


def test_single_keypair_matches_oracle_paillier(gpu_ctx):
    """The distribute() path: p then q, exactly paillier.keypair_with_modulus_size (Rng.prime)."""
    from fsdkr import keygen
    ek, dk = keygen.keypair_with_modulus_size(gpu_ctx, Rng("kp"), 2048)
    ek_o, dk_o = paillier.keypair_with_modulus_size(2048, Rng("kp"))
    assert (ek.n, dk.p, dk.q) == (ek_o.n, dk_o.p, dk_o.q)
    assert ek.n.bit_length() == 2048


def test_refresh_keys_batch(gpu_ctx):
    """Batched keypairs + NiCorrectKeyProof::proof against the oracle."""
    from fsdkr import keygen
    keys = keygen.refresh_keys(gpu_ctx, Rng("rk"), 1024, 5)
    want = ok.keypairs_with_modulus_size(Rng("rk"), 1024, 5)
    assert [(ek.n, dk.p, dk.q) for ek, dk, _ in keys] == want
    for ek, dk, ck in keys:
        ref = zk_paillier.NiCorrectKeyProof.proof(dk.p, dk.q)
        assert tuple(ck.sigma_vec) == tuple(ref.sigma_vec)
        assert zk_paillier.NiCorrectKeyProof(tuple(ck.sigma_vec)).verify(ek.n)


class _TopThenRandom:
    """Draws all-ones for the first `top` starts (start = 2^bits - 1), then seeded draws."""

    def __init__(self, top, seed):
        self.top, self.rng = top, Rng(seed)

    def bits(self, k):
        if self.top:
            self.top -= 1
            return (1 << k) - 1
        return self.rng.bits(k)


def test_walk_stays_below_two_to_bits(gpu_ctx):
    """A start within the walk's span of 2^bits (the sieve offsets
    used to run past it, so a (bits+1)-bit prime could come out): the walk
    ends at 2^bits, redraws, and every prime has exactly `bits` bits; the
    oracle's walk takes the same draws to the same primes."""
    from fsdkr import keygen
    bits = 192
    got = keygen.sample_primes(gpu_ctx, _TopThenRandom(3, "top"), bits, 3)
    want = ok.sample_primes(_TopThenRandom(3, "top"), bits, 3)
    assert got == want
    assert all(p.bit_length() == bits for p in got)
