"""Restatement of AliceProof from /root/reference/src/range_proofs.rs — TEST
INFRASTRUCTURE ONLY.  (BobProof/BobProofExt :205-590 are never called by the
refresh path and are out of scope)"""
from dataclasses import dataclass

from . import bigint
from . import secp256k1 as ec
from .hashing import chain_bigint
from .paillier import EncryptionKey
from .zk_paillier import DLogStatement


@dataclass(frozen=True)
class AliceProof:                  # :100-108
    z: int
    e: int
    s: int
    s1: int
    s2: int


def _challenge(ek: EncryptionKey, cipher, z, u, w):
    return chain_bigint(ek.n, ek.n + 1, cipher, z, u, w)


def generate(a: int, cipher: int, ek: EncryptionKey, st: DLogStatement, r: int, rng) -> AliceProof:
    """:168-202 with AliceZkpRound1::from (:40-74) and AliceZkpRound2::from (:83-96)."""
    q = ec.Q
    h1, h2, Nt = st.g, st.ni, st.N
    alpha = rng.sample_below(q ** 3)
    beta = rng.from_modulo(ek.n)
    gamma = rng.sample_below(q ** 3 * Nt)
    ro = rng.sample_below(q * Nt)
    z = bigint.mod_pow(h1, a, Nt) * bigint.mod_pow(h2, ro, Nt) % Nt
    u = (alpha * ek.n + 1) * bigint.mod_pow(beta, ek.n, ek.nn) % ek.nn
    w = bigint.mod_pow(h1, alpha, Nt) * bigint.mod_pow(h2, gamma, Nt) % Nt
    e = _challenge(ek, cipher, z, u, w)
    s = bigint.mod_pow(r, e, ek.n) * beta % ek.n
    s1 = e * a + alpha
    s2 = e * ro + gamma
    return AliceProof(z, e, s, s1, s2)


def verify(pf: AliceProof, cipher: int, ek: EncryptionKey, st: DLogStatement) -> bool:
    """:112-164 (the hash runs after the modexps; no early exit other than the
    s1 bound and the two non-invertible cases)."""
    N, NN = ek.n, ek.nn
    Nt, h1, h2 = st.N, st.g, st.ni
    if pf.s1 > ec.Q ** 3:
        return False
    z_e_inv = bigint.mod_inv(bigint.mod_pow(pf.z, pf.e, Nt), Nt)
    if z_e_inv is None:
        return False
    w = bigint.mod_pow(h1, pf.s1, Nt) * bigint.mod_pow(h2, pf.s2, Nt) * z_e_inv % Nt
    gs1 = (pf.s1 * N + 1) % NN
    c_e_inv = bigint.mod_inv(bigint.mod_pow(cipher, pf.e, NN), NN)
    if c_e_inv is None:
        return False
    u = gs1 * bigint.mod_pow(pf.s, N, NN) * c_e_inv % NN
    return _challenge(ek, cipher, pf.z, u, w) == pf.e
