"""kzen-paillier 0.4.3 (/root/reference/Cargo.toml:13-16) — TEST INFRASTRUCTURE ONLY.

Only the operations the refresh path calls: keypair_with_modulus_size
(refresh_message.rs:118), encrypt_with_chosen_randomness (:75-81), encrypt
(:232), mul (:223-227), add (:233), decrypt (:439) [dep, published algorithm]."""
from dataclasses import dataclass

from . import bigint


@dataclass(frozen=True)
class EncryptionKey:
    n: int
    nn: int

    @staticmethod
    def from_n(n: int) -> "EncryptionKey":
        return EncryptionKey(n, n * n)


@dataclass(frozen=True)
class DecryptionKey:
    p: int
    q: int


def keypair_with_modulus_size(bits: int, rng):
    while True:
        p = rng.prime(bits // 2)
        q = rng.prime(bits // 2)
        if p != q:
            return EncryptionKey.from_n(p * q), DecryptionKey(p, q)


def encrypt_with_chosen_randomness(ek: EncryptionKey, m: int, r: int) -> int:
    """c = (m*n + 1 mod n^2) * r^n mod n^2."""
    rn = bigint.mod_pow(r, ek.n, ek.nn)
    gm = (m * ek.n + 1) % ek.nn
    return gm * rn % ek.nn


def encrypt(ek: EncryptionKey, m: int, rng) -> int:
    """Paillier::encrypt with fresh randomness r <- U[0, n) (Randomness::sample)."""
    return encrypt_with_chosen_randomness(ek, m, rng.sample_below(ek.n))


def mul(ek: EncryptionKey, c: int, m: int) -> int:
    """Homomorphic scalar multiplication: c^m mod n^2."""
    return bigint.mod_pow(c, m, ek.nn)


def add(ek: EncryptionKey, c1: int, c2: int) -> int:
    return c1 * c2 % ek.nn


def _l_trunc(u: int, n: int) -> int:
    """L(u) = (u - 1) / n with BigInt division (truncating toward zero): L(0) = 0."""
    v = u - 1
    return v // n if v >= 0 else -((-v) // n)


def decrypt(dk: DecryptionKey, c: int) -> int:
    """kzen-paillier's CRT decryption [dep, published algorithm]: per prime,
    m_p = L_p(c^(p-1) mod p^2) h_p mod p with h_p = L_p(g^(p-1) mod p^2)^-1,
    g = n + 1, then m = m_q + q ((m_p - m_q) q^-1 mod p).  For a unit c this is
    the unique m of c = (1+n)^m r^n (= L(c^lambda) mu mod n); for p | c the p
    half is L_p(0) h_p = 0 (truncating division), which fixes the reference's
    decryption of a non-unit ciphertext sum (JoinMessage::collect has no PDL
    check that would have rejected such a ciphertext first)."""
    p, q = dk.p, dk.q
    n = p * q
    out = []
    for a in (p, q):
        aa = a * a
        h = pow(_l_trunc(bigint.mod_pow((n + 1) % aa, a - 1, aa), a), -1, a)
        d = bigint.mod_pow(c % aa, a - 1, aa)
        out.append(_l_trunc(d, a) * h % a)
    mp, mq = out
    return mq + q * ((mp - mq) * pow(q, -1, p) % p)
