"""Restatement of /root/reference/src/zk_pdl_with_slack.rs — TEST INFRASTRUCTURE ONLY."""
from dataclasses import dataclass

from . import bigint
from . import secp256k1 as ec
from .hashing import chain_bigint
from .paillier import EncryptionKey


class PDLwSlackError(Exception):
    """FsDkrError::PDLwSlackProof{is_u1_eq, is_u2_eq, is_u3_eq} (error.rs:26-31)."""

    def __init__(self, is_u1_eq, is_u2_eq, is_u3_eq):
        super().__init__(f"PDLwSlackProof u1={is_u1_eq} u2={is_u2_eq} u3={is_u3_eq}")
        self.flags = (is_u1_eq, is_u2_eq, is_u3_eq)


@dataclass(frozen=True)
class PDLwSlackStatement:          # :24-32
    ciphertext: int
    ek: EncryptionKey
    Q: tuple
    G: tuple
    h1: int
    h2: int
    N_tilde: int


@dataclass(frozen=True)
class PDLwSlackProof:              # :41-50
    z: int
    u1: tuple
    u2: int
    u3: int
    s1: int
    s2: int
    s3: int


def commitment_unknown_order(h1, h2, N_tilde, x, r):
    """:170-188 — h1^x * h2^r mod N~, negative r through h2^-1 (unwrap: panics
    if h2 is not invertible)."""
    h1_x = bigint.mod_pow(h1, x, N_tilde)
    if r < 0:
        h2_inv = bigint.mod_inv(h2, N_tilde)
        if h2_inv is None:
            raise bigint.PanicError("commitment_unknown_order: mod_inv(h2).unwrap()")
        h2_r = bigint.mod_pow(h2_inv, -r, N_tilde)
    else:
        h2_r = bigint.mod_pow(h2, r, N_tilde)
    return bigint.mod_mul(h1_x, h2_r, N_tilde)


def challenge(st: PDLwSlackStatement, z, u1, u2, u3) -> int:
    """:87-95 / :114-122."""
    return chain_bigint(ec.to_bigint_compressed(st.G), ec.to_bigint_compressed(st.Q), st.ciphertext, z,
                        ec.to_bigint_compressed(u1), u2, u3)


def prove(x: int, r: int, st: PDLwSlackStatement, rng) -> PDLwSlackProof:
    """:53-111 (x is the Scalar witness, r the Paillier randomness)."""
    q3 = ec.Q ** 3
    alpha = rng.sample_below(q3)
    beta = rng.sample_range(1, st.ek.n - 1)
    rho = rng.sample_below(ec.Q * st.N_tilde)
    gamma = rng.sample_below(q3 * st.N_tilde)
    z = commitment_unknown_order(st.h1, st.h2, st.N_tilde, x, rho)
    u1 = ec.mul(st.G, alpha)
    u2 = commitment_unknown_order(st.ek.n + 1, beta, st.ek.nn, alpha, st.ek.n)
    u3 = commitment_unknown_order(st.h1, st.h2, st.N_tilde, alpha, gamma)
    e = challenge(st, z, u1, u2, u3)
    s1 = e * x + alpha
    s2 = commitment_unknown_order(r, beta, st.ek.n, e, 1)
    s3 = e * rho + gamma
    return PDLwSlackProof(z, u1, u2, u3, s1, s2, s3)


def verify(pf: PDLwSlackProof, st: PDLwSlackStatement) -> None:
    """:113-167.  Raises PDLwSlackError on failure, PanicError where the
    reference panics (non-invertible ciphertext / z at :180)."""
    e = challenge(st, pf.z, pf.u1, pf.u2, pf.u3)
    g_s1 = ec.mul(st.G, pf.s1)
    e_fe_neg = ec.scalar(ec.Q - e)
    y_minus_e = ec.mul(st.Q, e_fe_neg)
    u1_test = ec.add(g_s1, y_minus_e)
    u2_test_tmp = commitment_unknown_order(st.ek.n + 1, pf.s2, st.ek.nn, pf.s1, st.ek.n)
    u2_test = commitment_unknown_order(u2_test_tmp, st.ciphertext, st.ek.nn, 1, -e)
    u3_test_tmp = commitment_unknown_order(st.h1, st.h2, st.N_tilde, pf.s1, pf.s3)
    u3_test = commitment_unknown_order(u3_test_tmp, pf.z, st.N_tilde, 1, -e)
    f1, f2, f3 = pf.u1 == u1_test, pf.u2 == u2_test, pf.u3 == u3_test
    if not (f1 and f2 and f3):
        raise PDLwSlackError(f1, f2, f3)
