"""Key generation on the CPU: the oracle's restated prime walk
is pinned to Rng.prime (the walk every oracle key and golden fixture was made
with), Miller-Rabin to known strong pseudoprimes, and the product's host
pieces (sieve, witness bases, batched walk schedule) to the oracle."""
import pytest

from oracle import keygen as ok
from oracle import bigint
from oracle.rng import Rng


@pytest.mark.parametrize("bits", [128, 256, 512])
def test_oracle_walk_is_rng_prime(bits):
    for s in range(3):
        assert ok.sample_primes(Rng(("kg", bits, s)), bits, 1)[0] == Rng(("kg", bits, s)).prime(bits)


def test_oracle_batch_is_sequential_walks():
    rng = Rng("batch")
    got = ok.sample_primes(rng, 256, 6)
    rng2 = Rng("batch")
    starts = [rng2.bits(256) | (3 << 254) | 1 for _ in range(6)]
    assert got == [ok.walk(s, 4 * 256) for s in starts]
    assert all(bigint.is_probable_prime(p) for p in got)


# strong pseudoprimes (the smallest to the listed bases) and Carmichael numbers
SPSP = [(2047, (2,), 3), (1373653, (2, 3), 5), (25326001, (2, 3, 5), 7), (3215031751, (2, 3, 5, 7), 11),
        (2152302898747, (2, 3, 5, 7, 11), 13)]


@pytest.mark.parametrize("n,liars,witness", SPSP)
def test_strong_pseudoprimes(n, liars, witness):
    assert all(ok.strong_probable_prime(n, b) for b in liars)
    assert not ok.strong_probable_prime(n, witness)
    assert not ok.is_probable_prime(n)


def test_carmichael_and_primes():
    for n in (561, 41041, 825265, 321197185):
        assert not ok.strong_probable_prime(n, 2) or not ok.is_probable_prime(n)
    for p in ((1 << 521) - 1, (1 << 607) - 1, 2 ** 127 - 1):
        assert ok.is_probable_prime(p)
        assert all(ok.strong_probable_prime(p, b) for b in (2, 3, p - 1, 1))
    assert not ok.is_probable_prime(((1 << 521) - 1) * ((1 << 127) - 1))


def test_oracle_walk_stops_at_two_to_bits():
    """The walk from 2^bits - 1 (composite for these bits) has no candidate left
    below 2^bits: None, not the (bits+1)-bit prime 2^bits + 1 (bits = 64: Fermat
    F6 is composite; bits = 16: 65537 is prime)."""
    assert ok.walk((1 << 16) - 1, 64, 16) is None
    assert ok.walk((1 << 16) - 1, 64) == 65537
    assert ok.walk((1 << 192) - 1, 4 * 192, 192) is None
