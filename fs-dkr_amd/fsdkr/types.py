"""Product-side message types with the reference's field names
(refresh_message.rs:31-48, add_party_message.rs:36-45, zk_pdl_with_slack.rs:24-50,
range_proofs.rs:101-108, ring_pedersen_proof.rs:30-38,79-84; zk-paillier
DLogStatement / NiCorrectKeyProof / CompositeDLogProof; kzen-paillier keys;
multi-party-ecdsa LocalKey).  The batching layer reads these by attribute, so
any structurally identical objects work as well.  Points are affine (x, y)
tuples or None for the point at infinity."""
from dataclasses import dataclass, field
from typing import List, Optional, Tuple


@dataclass(frozen=True)
class EncryptionKey:
    n: int
    nn: int


@dataclass(frozen=True)
class DecryptionKey:
    p: int
    q: int


@dataclass(frozen=True)
class DLogStatement:
    N: int
    g: int
    ni: int


@dataclass(frozen=True)
class PDLwSlackProof:
    z: int
    u1: Optional[Tuple[int, int]]
    u2: int
    u3: int
    s1: int
    s2: int
    s3: int


@dataclass(frozen=True)
class AliceProof:
    z: int
    e: int
    s: int
    s1: int
    s2: int


@dataclass(frozen=True)
class RingPedersenStatement:
    S: int
    T: int
    N: int
    phi: int
    ek: EncryptionKey


@dataclass(frozen=True)
class RingPedersenProof:
    A: Tuple[int, ...]
    Z: Tuple[int, ...]


@dataclass(frozen=True)
class NiCorrectKeyProof:
    sigma_vec: Tuple[int, ...]


@dataclass(frozen=True)
class CompositeDLogProof:
    x: int
    y: int


@dataclass
class VerifiableSS:
    threshold: int
    share_count: int
    commitments: List = field(default_factory=list)


@dataclass
class RefreshMessage:
    old_party_index: int
    party_index: int
    pdl_proof_vec: List[PDLwSlackProof]
    range_proofs: List[AliceProof]
    coefficients_committed_vec: VerifiableSS
    points_committed_vec: List
    points_encrypted_vec: List[int]
    dk_correctness_proof: NiCorrectKeyProof
    dlog_statement: DLogStatement
    ek: EncryptionKey
    remove_party_indices: List[int]
    public_key: object
    ring_pedersen_statement: RingPedersenStatement
    ring_pedersen_proof: RingPedersenProof


@dataclass
class JoinMessage:
    ek: EncryptionKey
    dk_correctness_proof: NiCorrectKeyProof
    party_index: Optional[int]
    dlog_statement: DLogStatement
    composite_dlog_proof_base_h1: CompositeDLogProof
    composite_dlog_proof_base_h2: CompositeDLogProof
    ring_pedersen_statement: RingPedersenStatement
    ring_pedersen_proof: RingPedersenProof


@dataclass
class LocalKey:
    paillier_dk: DecryptionKey
    pk_vec: List
    x_i: int
    y: object
    paillier_key_vec: List[EncryptionKey]
    y_sum_s: object
    h1_h2_n_tilde_vec: List[DLogStatement]
    vss_scheme: VerifiableSS
    i: int
    t: int
    n: int


@dataclass
class Keys:
    """The Paillier pair of multi-party-ecdsa gg_2020 party_i::Keys that
    JoinMessage::collect consumes (add_party_message.rs:139, :189-193)."""
    ek: EncryptionKey
    dk: DecryptionKey
