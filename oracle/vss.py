"""Feldman VSS and Lagrange re-mapping from curv-kzen 0.10
(cryptographic_primitives/secret_sharing/feldman_vss.rs) [dep, published
algorithm] as called at refresh_message.rs:62,180-182,213-217 —
TEST INFRASTRUCTURE ONLY."""
from dataclasses import dataclass, field
from typing import List

from . import secp256k1 as ec


@dataclass
class VerifiableSS:
    threshold: int
    share_count: int
    commitments: List = field(default_factory=list)   # points G*a_k, k = 0..t

    @staticmethod
    def share(t: int, n: int, secret: int, rng):
        """Random degree-t polynomial with a_0 = secret (top coefficient nonzero:
        Polynomial::sample_exact_with_fixed_const_term); shares f(1..n)."""
        if not t < n:
            from .bigint import PanicError
            raise PanicError("VerifiableSS::share: t < n")
        coeffs = [secret % ec.Q] + [rng.sample_below(ec.Q) for _ in range(t)]
        while t > 0 and coeffs[-1] == 0:
            coeffs[-1] = rng.sample_below(ec.Q)
        shares = []
        for i in range(1, n + 1):
            acc = 0
            for a in reversed(coeffs):
                acc = (acc * i + a) % ec.Q
            shares.append(acc)
        commitments = [ec.mul(ec.G, a) for a in coeffs]
        return VerifiableSS(t, n, commitments), shares

    def get_point_commitment(self, index: int):
        """Horner over the commitments: sum_k A_k * index^k."""
        comm = list(reversed(self.commitments))
        acc = comm[0]
        for c in comm[1:]:
            acc = ec.add(c, ec.mul(acc, index))
        return acc

    def validate_share_public(self, point, index: int) -> bool:
        return point == self.get_point_commitment(index)


def map_share_to_new_params(index: int, s: List[int]) -> int:
    """Lagrange coefficient at 0 for party `index` (0-based) over the set s
    (0-based indices; evaluation points are index+1)."""
    xi = index + 1
    num, den = 1, 1
    for j in s:
        if j == index:
            continue
        xj = j + 1
        num = num * xj % ec.Q
        den = den * (xj - xi) % ec.Q
    return num * pow(den, -1, ec.Q) % ec.Q
