"""zk-paillier 0.4.4 (/root/reference/Cargo.toml:32) — TEST INFRASTRUCTURE ONLY.

The crate is not vendored; these are restatements of its published algorithms
as called by the reference [dep, unverified]:
  NiCorrectKeyProof::proof / verify  (refresh_message.rs:119,376-378,401-404)
  CompositeDLogProof::prove / verify (add_party_message.rs:84-85, refresh_message.rs:415-422)
  DLogStatement {N, g, ni}           (range_proofs.rs:25, refresh_message.rs:40)
PARITY UNPINNED: SALT_STRING bytes, the alpha-primorial constant and the
CompositeDLogProof transcript order are restated from the crate as published,
not checked against it (no crate source here)."""
from dataclasses import dataclass
from typing import List

from . import bigint
from .hashing import compute_digest

SALT_STRING = bytes([75, 90, 101, 110])   # b"KZen"
M2 = 11
DIGEST_SIZE = 256
ALPHA = 6370                               # primorial bound of correct_key_ni.rs [dep, unverified]


def _primorial(bound: int) -> int:
    sieve = bytearray([1]) * bound
    sieve[0:2] = b"\x00\x00"
    for i in range(2, int(bound ** 0.5) + 1):
        if sieve[i]:
            sieve[i * i::i] = bytearray(len(sieve[i * i::i]))
    p = 1
    for i, v in enumerate(sieve):
        if v:
            p *= i
    return p


ALPHA_PRIMORIAL = _primorial(ALPHA)
SMALL_PRIMES = [i for i in range(2, ALPHA) if ALPHA_PRIMORIAL % i == 0 and all(i % d for d in range(2, int(i ** 0.5) + 1))]


@dataclass(frozen=True)
class DLogStatement:
    N: int
    g: int
    ni: int


def mask_generation(out_length: int, seed: int) -> int:
    msklen = out_length // DIGEST_SIZE + 1
    acc = 0
    for j in range(msklen):
        acc += compute_digest(seed, j) << (j * DIGEST_SIZE)
    return acc


def correct_key_rho(n: int, salt: bytes = SALT_STRING) -> List[int]:
    key_length = n.bit_length()
    salt_bn = bigint.from_bytes(salt)
    return [mask_generation(key_length, compute_digest(n, salt_bn, i)) % n for i in range(M2)]


@dataclass(frozen=True)
class NiCorrectKeyProof:
    sigma_vec: tuple

    @staticmethod
    def proof(p: int, q: int, salt: bytes = SALT_STRING) -> "NiCorrectKeyProof":
        n = p * q
        phi = (p - 1) * (q - 1)
        ninv = pow(n, -1, phi)
        return NiCorrectKeyProof(tuple(bigint.mod_pow(r, ninv, n) for r in correct_key_rho(n, salt)))

    def verify(self, n: int, salt: bytes = SALT_STRING) -> bool:
        if len(self.sigma_vec) < M2:
            raise bigint.PanicError("NiCorrectKeyProof: sigma_vec too short")
        rho = correct_key_rho(n, salt)
        gcd_ok = bigint.gcd(ALPHA_PRIMORIAL, n) == 1
        derived = [bigint.mod_pow(self.sigma_vec[i], n, n) for i in range(M2)]
        return rho == derived and gcd_ok


K = 128
K_PRIME = 128
SAMPLE_S = 256


@dataclass(frozen=True)
class CompositeDLogProof:
    x: int
    y: int

    @staticmethod
    def challenge(x: int, st: DLogStatement) -> int:
        return compute_digest(x, st.g, st.N, st.ni)

    @staticmethod
    def prove(st: DLogStatement, secret: int, rng) -> "CompositeDLogProof":
        R = (1 << (K + K_PRIME + SAMPLE_S)) * st.N
        r = rng.sample_below(R)
        x = bigint.mod_pow(st.g, r, st.N)
        e = CompositeDLogProof.challenge(x, st)
        return CompositeDLogProof(x, r + e * secret)

    def verify(self, st: DLogStatement) -> bool:
        if st.N <= (1 << K):
            return False
        if bigint.gcd(st.g, st.N) != 1 or bigint.gcd(st.ni, st.N) != 1:
            return False
        e = CompositeDLogProof.challenge(self.x, st)
        ni_e = bigint.mod_pow(st.ni, e, st.N)
        g_y = bigint.mod_pow(st.g, self.y, st.N)
        return self.x == bigint.mod_mul(g_y, ni_e, st.N)
