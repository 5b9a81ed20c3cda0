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


def decrypt(dk: DecryptionKey, c: int) -> int:
    """m = L(c^lambda mod n^2) * mu mod n (kzen-paillier computes the same value
    through CRT; both are the unique m of c = (1+n)^m r^n)."""
    n = dk.p * dk.q
    nn = n * n
    lam = (dk.p - 1) * (dk.q - 1)
    u = bigint.mod_pow(c, lam, nn)
    L = (u - 1) // n
    mu = pow(lam, -1, n)
    return L * mu % n
