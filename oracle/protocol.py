"""Restatement of /root/reference/src/refresh_message.rs,
/root/reference/src/add_party_message.rs and /root/reference/src/error.rs —
TEST INFRASTRUCTURE ONLY.

Randomness is injected through `rng` (oracle.rng.Rng); the reference draws
from the OS RNG.  `key_bits` generalises PAILLIER_KEY_SIZE (lib.rs:26) so
config 5 (3072-bit keys) and fast small-key unit tests can use
the same code; with key_bits=2048 it is the reference's constant.
GG20 keygen (multi-party-ecdsa) is out of scope: `simulate_keygen` builds the
LocalKey fields a keygen produces with a trusted dealer (test helper)."""
import copy
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from . import bigint
from . import paillier
from . import range_proofs
from . import ring_pedersen
from . import secp256k1 as ec
from . import zk_pdl_with_slack as pdl
from .vss import VerifiableSS, map_share_to_new_params
from .zk_paillier import CompositeDLogProof, DLogStatement, NiCorrectKeyProof

PAILLIER_KEY_SIZE = 2048   # lib.rs:26
M_SECURITY = 256           # lib.rs:27


# ------------------------------------------------------------------ errors ----
class FsDkrError(Exception):
    """error.rs:6-60.  `variant` is the Rust variant name, `fields` its payload."""

    def __init__(self, variant: str, **fields):
        super().__init__(f"{variant}{fields}")
        self.variant = variant
        self.fields = fields

    def as_tuple(self):
        return (self.variant, tuple(sorted(self.fields.items())))


# ---------------------------------------------------------------- messages ----
@dataclass
class LocalKey:
    """multi-party-ecdsa gg_2020 LocalKey fields (add_party_message.rs:280-291)."""
    paillier_dk: paillier.DecryptionKey
    pk_vec: List
    x_i: int                      # keys_linear.x_i
    y: object                     # keys_linear.y
    paillier_key_vec: List[paillier.EncryptionKey]
    y_sum_s: object
    h1_h2_n_tilde_vec: List[DLogStatement]
    vss_scheme: VerifiableSS
    i: int
    t: int
    n: int

    def clone(self):
        return copy.deepcopy(self)


@dataclass
class RefreshMessage:
    """refresh_message.rs:31-48."""
    old_party_index: int
    party_index: int
    pdl_proof_vec: List[pdl.PDLwSlackProof]
    range_proofs: List[range_proofs.AliceProof]
    coefficients_committed_vec: VerifiableSS
    points_committed_vec: List
    points_encrypted_vec: List[int]
    dk_correctness_proof: NiCorrectKeyProof
    dlog_statement: DLogStatement
    ek: paillier.EncryptionKey
    remove_party_indices: List[int]
    public_key: object
    ring_pedersen_statement: ring_pedersen.RingPedersenStatement
    ring_pedersen_proof: ring_pedersen.RingPedersenProof


@dataclass
class JoinMessage:
    """add_party_message.rs:36-45."""
    ek: paillier.EncryptionKey
    dk_correctness_proof: NiCorrectKeyProof
    party_index: Optional[int]
    dlog_statement: DLogStatement
    composite_dlog_proof_base_h1: CompositeDLogProof
    composite_dlog_proof_base_h2: CompositeDLogProof
    ring_pedersen_statement: ring_pedersen.RingPedersenStatement
    ring_pedersen_proof: ring_pedersen.RingPedersenProof

    def get_party_index(self) -> int:       # :127-130
        if self.party_index is None:
            raise FsDkrError("NewPartyUnassignedIndexError")
        return self.party_index

    def set_party_index(self, i: int):      # :95-97
        self.party_index = i


@dataclass
class Keys:
    """The Paillier part of multi-party-ecdsa gg_2020 party_i::Keys used by the join path."""
    ek: paillier.EncryptionKey
    dk: paillier.DecryptionKey


# ------------------------------------------------------------ setup helpers ---
def generate_h1_h2_n_tilde(key_bits: int, rng):
    """add_party_message.rs:50-66."""
    ek_t, dk_t = paillier.keypair_with_modulus_size(key_bits, rng)
    phi = (dk_t.p - 1) * (dk_t.q - 1)
    h1 = rng.sample_below(ek_t.n)
    while True:
        xhi = rng.sample_below(phi)
        xhi_inv = bigint.mod_inv(xhi, phi)
        if xhi_inv is not None:
            break
    h2 = bigint.mod_pow(h1, xhi, ek_t.n)
    xhi = phi - xhi
    xhi_inv = phi - xhi_inv
    return ek_t.n, h1, h2, xhi, xhi_inv


def generate_dlog_statement_proofs(key_bits: int, rng):
    """add_party_message.rs:69-92."""
    n_tilde, h1, h2, xhi, xhi_inv = generate_h1_h2_n_tilde(key_bits, rng)
    st1 = DLogStatement(n_tilde, h1, h2)
    st2 = DLogStatement(n_tilde, h2, h1)
    return st1, CompositeDLogProof.prove(st1, xhi, rng), CompositeDLogProof.prove(st2, xhi_inv, rng)


def simulate_keygen(t: int, n: int, rng, key_bits: int = PAILLIER_KEY_SIZE) -> List[LocalKey]:
    """Trusted-dealer stand-in for GG20 keygen (test.rs:226-236): the LocalKey
    fields collect() reads, with a consistent Shamir sharing of one secret."""
    secret = rng.sample_below(ec.Q)
    vss, shares = VerifiableSS.share(t, n, secret, rng)
    keys = [paillier.keypair_with_modulus_size(key_bits, rng) for _ in range(n)]
    stmts = [generate_dlog_statement_proofs(key_bits, rng)[0] for _ in range(n)]
    pk_vec = [ec.mul(ec.G, s) for s in shares]
    y = ec.mul(ec.G, secret)
    out = []
    for i in range(n):
        out.append(LocalKey(paillier_dk=keys[i][1], pk_vec=list(pk_vec), x_i=shares[i], y=pk_vec[i],
                            paillier_key_vec=[k[0] for k in keys], y_sum_s=y, h1_h2_n_tilde_vec=list(stmts),
                            vss_scheme=copy.deepcopy(vss), i=i + 1, t=t, n=n))
    return out


# ------------------------------------------------------------- distribute -----
def _rp_generate_and_prove(key_bits: int, M: int, rng):
    """RingPedersenStatement::generate + prove (refresh_message.rs:121-124).  A
    challenge with a leading zero byte makes the reference prover panic
    (BitVec index, ring_pedersen_proof.rs:106-110); the seeded generator
    redraws instead."""
    while True:
        st, wit = ring_pedersen.generate(key_bits, rng)
        try:
            return st, ring_pedersen.prove(wit, st, M, rng)
        except bigint.PanicError:
            continue


def distribute(old_party_index: int, local_key: LocalKey, new_n: int, rng, key_bits: int = PAILLIER_KEY_SIZE,
               M: int = M_SECURITY, randomness: Optional[List[int]] = None):
    """refresh_message.rs:51-145.  Returns (RefreshMessage, new DecryptionKey).
    `randomness` optionally fixes the Paillier r_i of :74 (job-1 parity)."""
    if not local_key.t <= new_n // 2:
        raise bigint.PanicError("distribute: assert!(t <= new_n / 2)")
    secret = local_key.x_i
    if new_n <= local_key.t:
        raise FsDkrError("NewPartyUnassignedIndexError")
    vss, shares = VerifiableSS.share(local_key.t, new_n, secret, rng)
    local_key.vss_scheme = copy.deepcopy(vss)
    points_committed = [ec.mul(ec.G, s) for s in shares]
    enc, rand = [], []
    for i in range(len(shares)):
        ek_i = local_key.paillier_key_vec[i]
        r = randomness[i] if randomness is not None else rng.sample_below(ek_i.n)
        enc.append(paillier.encrypt_with_chosen_randomness(ek_i, shares[i], r))
        rand.append(r)
    pdl_vec, rp_vec = [], []
    for i in range(len(shares)):
        st = pdl.PDLwSlackStatement(enc[i], local_key.paillier_key_vec[i], points_committed[i], ec.G,
                                    local_key.h1_h2_n_tilde_vec[i].g, local_key.h1_h2_n_tilde_vec[i].ni,
                                    local_key.h1_h2_n_tilde_vec[i].N)
        pdl_vec.append(pdl.prove(shares[i], rand[i], st, rng))
    for i in range(len(shares)):
        rp_vec.append(range_proofs.generate(shares[i], enc[i], local_key.paillier_key_vec[i],
                                            local_key.h1_h2_n_tilde_vec[i], rand[i], rng))
    ek, dk = paillier.keypair_with_modulus_size(key_bits, rng)
    ck = NiCorrectKeyProof.proof(dk.p, dk.q)
    rp_st, rp_pf = _rp_generate_and_prove(key_bits, M, rng)
    msg = RefreshMessage(old_party_index=old_party_index, party_index=local_key.i, pdl_proof_vec=pdl_vec,
                         range_proofs=rp_vec, coefficients_committed_vec=vss, points_committed_vec=points_committed,
                         points_encrypted_vec=enc, dk_correctness_proof=ck,
                         dlog_statement=local_key.h1_h2_n_tilde_vec[local_key.i - 1], ek=ek,
                         remove_party_indices=[], public_key=local_key.y_sum_s,
                         ring_pedersen_statement=rp_st, ring_pedersen_proof=rp_pf)
    return msg, dk


# ---------------------------------------------------------------- collect -----
def validate_collect(msgs: List[RefreshMessage], t: int, n: int):
    """refresh_message.rs:147-191."""
    if len(msgs) <= t:
        raise FsDkrError("PartiesThresholdViolation", threshold=t, refreshed_keys=len(msgs))
    ref_len = len(msgs[0].pdl_proof_vec)
    for k, m in enumerate(msgs):
        a, b, c = len(m.pdl_proof_vec), len(m.points_committed_vec), len(m.points_encrypted_vec)
        if not (a == ref_len and b == ref_len and c == ref_len):
            raise FsDkrError("SizeMismatchError", refresh_message_index=k, pdl_proof_len=a,
                             points_commited_len=b, points_encrypted_len=c)
    for m in msgs:
        for i in range(n):
            if i >= len(m.points_committed_vec):
                raise bigint.PanicError("validate_collect: points_committed_vec[i] out of bounds")
            if not m.coefficients_committed_vec.validate_share_public(m.points_committed_vec[i], i + 1):
                raise FsDkrError("PublicShareValidationError")


def get_ciphertext_sum(msgs: List[RefreshMessage], party_index: int, t: int, ek: paillier.EncryptionKey, rng):
    """refresh_message.rs:193-237.  Returns (ciphertext_sum, li_vec)."""
    cts = [m.points_encrypted_vec[party_index - 1] for m in msgs]
    indices = [msgs[i].old_party_index - 1 for i in range(t + 1)]
    li = [map_share_to_new_params(indices[i], indices) for i in range(t + 1)]
    mapped = [paillier.mul(ek, cts[i], li[i]) for i in range(t + 1)]
    acc = paillier.encrypt(ek, 0, rng)
    for c in mapped:
        acc = paillier.add(ek, acc, c)
    return acc, li


def collect(msgs: List[RefreshMessage], local_key: LocalKey, new_dk: paillier.DecryptionKey,
            joins: List[JoinMessage], rng, key_bits: int = PAILLIER_KEY_SIZE, M: int = M_SECURITY):
    """refresh_message.rs:321-467.  Mutates local_key exactly as the reference
    (including the progressive paillier_key_vec update before a later failure
    and the pk_vec insert quirk).  Raises FsDkrError / PanicError."""
    new_n = len(msgs) + len(joins)
    validate_collect(msgs, local_key.t, new_n)
    # the n^2 pair checks are independent: statements are built in the reference's
    # order (stopping where building one fails), verified concurrently, and their
    # outcomes consumed in that same order below
    jobs, build_err = [], None
    try:
        for m in msgs:
            for i in range(new_n):
                st = pdl.PDLwSlackStatement(m.points_encrypted_vec[i], local_key.paillier_key_vec[i],
                                            m.points_committed_vec[i], ec.G, local_key.h1_h2_n_tilde_vec[i].g,
                                            local_key.h1_h2_n_tilde_vec[i].ni, local_key.h1_h2_n_tilde_vec[i].N)
                jobs.append((m, i, st))
    except Exception as e:
        build_err = e

    def _pair(job):
        m, i, st = job
        r_pdl = bigint.outcome(lambda: pdl.verify(m.pdl_proof_vec[i], st))
        r_rng = None
        if r_pdl[0] and i < len(m.range_proofs):
            r_rng = bigint.outcome(range_proofs.verify, m.range_proofs[i], st.ciphertext, st.ek,
                                   local_key.h1_h2_n_tilde_vec[i])
        return r_pdl, r_rng

    for (m, i, st), (r_pdl, r_rng) in zip(jobs, bigint.pool().map(_pair, jobs)):
        try:
            bigint.settle(r_pdl)
        except pdl.PDLwSlackError as e:
            raise FsDkrError("PDLwSlackProof", is_u1_eq=e.flags[0], is_u2_eq=e.flags[1], is_u3_eq=e.flags[2])
        if i >= len(m.range_proofs):
            raise bigint.PanicError("collect: range_proofs[i] out of bounds")
        if not bigint.settle(r_rng):
            raise FsDkrError("RangeProof", party_index=i)
    if build_err is not None:
        raise build_err
    for m in msgs:
        if not ring_pedersen.verify(m.ring_pedersen_proof, m.ring_pedersen_statement, M):
            raise FsDkrError("RingPedersenProofError")
    for j in joins:
        if not ring_pedersen.verify(j.ring_pedersen_proof, j.ring_pedersen_statement, M):
            raise FsDkrError("RingPedersenProofError")
    old_ek = local_key.paillier_key_vec[local_key.i - 1]
    ct_sum, li = get_ciphertext_sum(msgs, local_key.i, local_key.vss_scheme.threshold, old_ek, rng)
    for m in msgs:
        if not m.dk_correctness_proof.verify(m.ek.n):
            raise FsDkrError("PaillierVerificationError", party_index=m.party_index)
        nl = m.ek.n.bit_length()
        if nl > key_bits or nl < key_bits - 1:
            raise FsDkrError("ModuliTooSmall", party_index=m.party_index, moduli_size=nl)
        local_key.paillier_key_vec[m.party_index - 1] = m.ek
    for j in joins:
        pi = j.get_party_index()
        if not j.dk_correctness_proof.verify(j.ek.n):
            raise FsDkrError("PaillierVerificationError", party_index=pi)
        st_h2 = DLogStatement(j.dlog_statement.N, j.dlog_statement.ni, j.dlog_statement.g)
        if not j.composite_dlog_proof_base_h1.verify(j.dlog_statement) or \
                not j.composite_dlog_proof_base_h2.verify(st_h2):
            raise FsDkrError("DLogProofValidation", party_index=pi)
        nl = j.ek.n.bit_length()
        if nl > key_bits or nl < key_bits - 1:
            raise FsDkrError("ModuliTooSmall", party_index=j.get_party_index(), moduli_size=nl)
        local_key.paillier_key_vec[pi - 1] = j.ek
    new_share = paillier.decrypt(local_key.paillier_dk, ct_sum)
    x = ec.scalar(new_share)
    local_key.paillier_dk = new_dk
    local_key.x_i = x
    local_key.y = ec.mul(ec.G, x)
    for i in range(len(msgs) + len(joins)):
        v = ec.mul(msgs[0].points_committed_vec[i], li[0])
        local_key.pk_vec.insert(i, v)
        for j in range(1, local_key.t + 1):
            local_key.pk_vec[i] = ec.add(local_key.pk_vec[i], ec.mul(msgs[j].points_committed_vec[i], li[j]))


# ---------------------------------------------------------------- replace -----
def replace(joins: List[JoinMessage], key: LocalKey, old_to_new: Dict[int, int], new_n: int, rng,
            key_bits: int = PAILLIER_KEY_SIZE, M: int = M_SECURITY):
    """refresh_message.rs:239-319.  The reference iterates a HashMap (random
    order); the oracle iterates new indices in ascending order."""
    current_len = len(key.paillier_key_vec)
    remap = {}
    for old in old_to_new:
        remap[old_to_new[old]] = (key.paillier_key_vec[old - 1], key.h1_h2_n_tilde_vec[old - 1])
    for new in sorted(remap):
        if new <= current_len:
            key.paillier_key_vec[new - 1], key.h1_h2_n_tilde_vec[new - 1] = remap[new]
        else:
            key.paillier_key_vec.insert(new - 1, remap[new][0])
            key.h1_h2_n_tilde_vec.insert(new - 1, remap[new][1])
    for j in joins:
        pi = j.get_party_index()
        if pi <= current_len:
            key.paillier_key_vec[pi - 1] = j.ek
            key.h1_h2_n_tilde_vec[pi - 1] = j.dlog_statement
        else:
            key.paillier_key_vec.insert(pi - 1, j.ek)
            key.h1_h2_n_tilde_vec.insert(pi - 1, j.dlog_statement)
    old_party_index = key.i
    key.i = old_to_new[key.i]
    key.n = new_n
    return distribute(old_party_index, key, new_n, rng, key_bits, M)


# ------------------------------------------------------------------- join -----
def join_distribute(rng, key_bits: int = PAILLIER_KEY_SIZE, M: int = M_SECURITY):
    """add_party_message.rs:101-124 (Keys::create(0): only its Paillier pair is used)."""
    ek, dk = paillier.keypair_with_modulus_size(key_bits, rng)
    st, p1, p2 = generate_dlog_statement_proofs(key_bits, rng)
    rp_st, rp_pf = _rp_generate_and_prove(key_bits, M, rng)
    msg = JoinMessage(ek=ek, dk_correctness_proof=NiCorrectKeyProof.proof(dk.p, dk.q), party_index=None,
                      dlog_statement=st, composite_dlog_proof_base_h1=p1, composite_dlog_proof_base_h2=p2,
                      ring_pedersen_statement=rp_st, ring_pedersen_proof=rp_pf)
    return msg, Keys(ek, dk)


def join_collect(self_msg: JoinMessage, msgs: List[RefreshMessage], keys: Keys, joins: List[JoinMessage], t: int,
                 n: int, rng, key_bits: int = PAILLIER_KEY_SIZE, M: int = M_SECURITY) -> LocalKey:
    """add_party_message.rs:136-294."""
    validate_collect(msgs, t, n)
    for m in msgs:
        if not ring_pedersen.verify(m.ring_pedersen_proof, m.ring_pedersen_statement, M):
            raise FsDkrError("RingPedersenProofValidation", party_index=m.party_index)
    for j in joins:
        if not ring_pedersen.verify(j.ring_pedersen_proof, j.ring_pedersen_statement, M):
            if j.party_index is not None:
                raise FsDkrError("RingPedersenProofValidation", party_index=j.party_index)
            raise FsDkrError("RingPedersenProofError")
    party_index = self_msg.get_party_index()
    for j in joins:
        j.get_party_index()
    ct_sum, li = get_ciphertext_sum(msgs, party_index, t, keys.ek, rng)
    new_share = paillier.decrypt(keys.dk, ct_sum)
    x = ec.scalar(new_share)
    pk_vec = [ec.mul(msgs[0].points_committed_vec[i], li[0]) for i in range(n)]
    for i in range(n):
        for j in range(1, t + 1):
            pk_vec[i] = ec.add(pk_vec[i], ec.mul(msgs[j].points_committed_vec[i], li[j]))
    available = {m.party_index: m.ek for m in msgs}
    available[party_index] = keys.ek
    for j in joins:
        available[j.party_index] = j.ek
    avail_st = {m.party_index: m.dlog_statement for m in msgs}
    avail_st[party_index] = self_msg.dlog_statement
    for j in joins:
        avail_st[j.party_index] = j.dlog_statement
    pk_list = [available.get(p, paillier.EncryptionKey(0, 0)) for p in range(1, n + 1)]
    st_list = [avail_st[p] if p in avail_st else generate_dlog_statement_proofs(key_bits, rng)[0]
               for p in range(1, n + 1)]
    for m in msgs:
        if m.public_key != msgs[0].public_key:
            raise FsDkrError("BroadcastedPublicKeyError")
    vss, _ = VerifiableSS.share(t, n, x, rng)
    return LocalKey(paillier_dk=keys.dk, pk_vec=pk_vec, x_i=x, y=ec.mul(ec.G, x), paillier_key_vec=pk_list,
                    y_sum_s=msgs[0].public_key, h1_h2_n_tilde_vec=st_list, vss_scheme=vss, i=party_index, t=t, n=n)


def reconstruct(indices: List[int], shares: List[int]) -> int:
    """VerifiableSS::reconstruct (test.rs:62-64): Lagrange interpolation at 0."""
    return sum(map_share_to_new_params(indices[k], indices) * shares[k] for k in range(len(indices))) % ec.Q
