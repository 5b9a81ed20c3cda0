"""Key generation restated on the CPU — TEST INFRASTRUCTURE ONLY (the checker of
fsdkr.keygen and of the fsdkr_miller_rabin C ABI; never the product path).

Reference call sites: Paillier::keypair_with_modulus_size
at refresh_message.rs:118 (distribute), ring_pedersen_proof.rs:50
(RingPedersenStatement::generate) and add_party_message.rs:51
(generate_h1_h2_n_tilde); NiCorrectKeyProof::proof at refresh_message.rs:119.
The prime generator itself lives in kzen-paillier 0.4.3 (Cargo.toml:13-16, a
dependency that is not vendored): a random candidate with its top bits and
its low bit set, trial division by small primes, then probabilistic tests.
It draws from the OS RNG, so its primes cannot be reproduced; the restated
walk below is the one the oracle's key generation already uses
(oracle/rng.py Rng.prime: random start, first probable prime within 4*bits odd
steps), with the probabilistic test made explicit:

  * trial division by the odd primes below 2000;
  * a strong-probable-prime (Miller–Rabin) round to base 2;
  * MR_ROUNDS further rounds to bases derived from the candidate
    (witness_bases: SHA-256 counter stream, reduced into [2, c-2]), so the
    test is deterministic and does not consume draws of the caller's RNG.

For random k-bit candidates (k >= 512) base 2 plus 8 independent rounds accept
a composite with probability < 2^-100 (Damgard-Landrock-Pomerance bound), so
the first accepted candidate of a walk equals the first prime of the walk of
Rng.prime (GMP mpz_probab_prime_p).  Parity with kzen-paillier's own primes
is unpinned (OS randomness)."""
import hashlib

from . import bigint

MR_ROUNDS = 8
SIEVE_LIMIT = 2000


def _odd_primes_below(n):
    flags = bytearray([1]) * n
    flags[0:2] = b"\x00\x00"
    for i in range(2, int(n ** 0.5) + 1):
        if flags[i]:
            flags[i * i::i] = bytearray(len(flags[i * i::i]))
    return [i for i in range(3, n) if flags[i]]


SMALL_PRIMES = _odd_primes_below(SIEVE_LIMIT)


def strong_probable_prime(c: int, b: int) -> bool:
    """One Miller–Rabin round: c - 1 = d 2^s; b^d == 1 or b^(d 2^j) == c - 1, j < s."""
    d, s = c - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    x = bigint.mod_pow(b, d, c)
    if x == 1 or x == c - 1:
        return True
    for _ in range(s - 1):
        x = x * x % c
        if x == c - 1:
            return True
        if x == 1:
            return False
    return False


def witness_bases(c: int, rounds: int = MR_ROUNDS):
    """Bases of the extra rounds: 2 + (SHA-256("fsdkr-mr" | c | j | ctr) stream mod (c - 3))."""
    nb = (c.bit_length() + 7) // 8
    cb = c.to_bytes(nb, "big")
    out = []
    for j in range(rounds):
        stream = b""
        ctr = 0
        while len(stream) < nb + 8:
            stream += hashlib.sha256(b"fsdkr-mr" + cb + j.to_bytes(4, "little") + ctr.to_bytes(4, "little")).digest()
            ctr += 1
        out.append(2 + int.from_bytes(stream[:nb + 8], "big") % (c - 3))
    return out


def is_probable_prime(c: int, rounds: int = MR_ROUNDS) -> bool:
    if c < 5 or c % 2 == 0:
        return c in (2, 3)
    for p in SMALL_PRIMES:
        if c % p == 0:
            return c == p
    if not strong_probable_prime(c, 2):
        return False
    return all(strong_probable_prime(c, b) for b in witness_bases(c, rounds))


def walk(start: int, span: int, bits: int = 0):
    """First probable prime among start, start+2, ... (span candidates, and
    below 2^bits when bits is given: a `bits`-bit prime), else None."""
    c = start
    for _ in range(span):
        if bits and c >> bits:
            return None
        if is_probable_prime(c):
            return c
        c += 2
    return None


def _draw_start(rng, bits):
    return rng.bits(bits) | (3 << (bits - 2)) | 1


def sample_primes(rng, bits: int, count: int, span: int = 0):
    """`count` primes by independent walks of `span` (default 4*bits) odd
    candidates.  Pass 1 draws every walk's start in walk order; a walk that
    ends without a prime draws a new start in a later pass (walks in index
    order).  count = 1 is exactly Rng.prime."""
    span = span or 4 * bits
    starts = [_draw_start(rng, bits) for _ in range(count)]
    out = [None] * count
    todo = list(range(count))
    while todo:
        for w in todo:
            out[w] = walk(starts[w], span, bits)
        todo = [w for w in todo if out[w] is None]
        for w in todo:
            starts[w] = _draw_start(rng, bits)
    return out


def keypairs_with_modulus_size(rng, bits: int, count: int):
    """`count` Paillier keypairs (n, p, q): primes 2k, 2k+1 of one batch; a pair
    with p == q redraws q (pairs in order, after the batch)."""
    primes = sample_primes(rng, bits // 2, 2 * count)
    out = []
    for k in range(count):
        p, q = primes[2 * k], primes[2 * k + 1]
        while p == q:
            q = sample_primes(rng, bits // 2, 1)[0]
        out.append((p * q, p, q))
    return out
