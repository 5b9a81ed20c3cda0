"""Fiat–Shamir hashing — TEST INFRASTRUCTURE ONLY.

curv-kzen 0.10 `DigestExt::chain_bigint(n)` = `update(n.to_bytes())` and
`result_bigint()` = `BigInt::from_bytes(finalize())` [dep, unverified]; used at
zk_pdl_with_slack.rs:87-95,114-122, range_proofs.rs:150-157,183-190,
ring_pedersen_proof.rs:95-105,130-135 with H = Sha256 (test.rs:19).
zk-paillier 0.4.4 `compute_digest` is the same construction [dep, unverified]."""
import hashlib

from .bigint import from_bytes, to_bytes


def chain_bigint(*values: int) -> int:
    h = hashlib.sha256()
    for v in values:
        h.update(to_bytes(v))
    return from_bytes(h.digest())


compute_digest = chain_bigint
