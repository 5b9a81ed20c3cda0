"""Restatement of /root/reference/src/ring_pedersen_proof.rs — TEST INFRASTRUCTURE ONLY."""
from dataclasses import dataclass
from typing import Tuple

from . import bigint
from . import paillier
from .hashing import chain_bigint


@dataclass(frozen=True)
class RingPedersenStatement:      # :30-38
    S: int
    T: int
    N: int
    phi: int
    ek: paillier.EncryptionKey


@dataclass(frozen=True)
class RingPedersenWitness:        # :40-45
    p: int
    q: int
    lam: int


@dataclass(frozen=True)
class RingPedersenProof:          # :79-84
    A: Tuple[int, ...]
    Z: Tuple[int, ...]


def generate(key_bits: int, rng):
    """:48-74."""
    ek, dk = paillier.keypair_with_modulus_size(key_bits, rng)
    phi = (dk.p - 1) * (dk.q - 1)
    r = rng.sample_below(ek.n)
    lam = rng.sample_below(phi)
    t = bigint.mod_pow(r, 2, ek.n)
    s = bigint.mod_pow(t, lam, ek.n)
    return RingPedersenStatement(s, t, ek.n, phi, ek), RingPedersenWitness(dk.p, dk.q, lam)


def challenge_bits(A, M: int):
    """e = H(A_0..A_{M-1}); bit i = Lsb0 bit i of e.to_bytes() (:130-142).
    Indexing past the byte vector panics (e with leading zero bytes)."""
    e = chain_bigint(*A[:M])
    eb = bigint.to_bytes(e)
    if 8 * len(eb) < M:
        raise bigint.PanicError("RingPedersenProof: challenge shorter than M bits (BitVec index)")
    return [(eb[i >> 3] >> (i & 7)) & 1 for i in range(M)]


def prove(wit: RingPedersenWitness, st: RingPedersenStatement, M: int, rng) -> RingPedersenProof:
    """:88-124."""
    a = [rng.sample_below(st.phi) for _ in range(M)]
    A = [bigint.mod_pow(st.T, ai, st.N) for ai in a]
    bits = challenge_bits(A, M)
    Z = [bigint.mod_add(a[i], bits[i] * wit.lam, st.phi) for i in range(M)]
    return RingPedersenProof(tuple(A), tuple(Z))


def verify(pf: RingPedersenProof, st: RingPedersenStatement, M: int) -> bool:
    """:126-157 (returns False for FsDkrError::RingPedersenProofError).  The hash
    loop indexes A[0..M) first; inside the check loop, bit i of the challenge
    (BitVec index) and Z[i] are read at iteration i, so a failing check before
    either index is reached returns the error, not the panic."""
    if len(pf.A) < M:
        raise bigint.PanicError("RingPedersenProof: A shorter than M")
    eb = bigint.to_bytes(chain_bigint(*pf.A[:M]))
    # the M exponentiations T^Z_i are independent: computed concurrently, consumed in order
    todo = min(M, len(pf.Z), 8 * len(eb))
    lhs_all = list(bigint.pool().map(lambda z: bigint.outcome(bigint.mod_pow, st.T, z, st.N), pf.Z[:todo]))
    for i in range(M):
        if i >= 8 * len(eb):
            raise bigint.PanicError("RingPedersenProof: challenge shorter than M bits (BitVec index)")
        bit = (eb[i >> 3] >> (i & 7)) & 1
        if i >= len(pf.Z):
            raise bigint.PanicError("RingPedersenProof: Z shorter than M")
        lhs = bigint.settle(lhs_all[i])
        rhs = bigint.mod_mul(pf.A[i], bigint.mod_pow(st.S, bit, st.N), st.N)
        if lhs != rhs:
            return False
    return True
