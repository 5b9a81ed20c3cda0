"""Negative operands on the GPU path: one
sender's negative BigInt gets the reference's outcome for that instance --
the oracle's panic, error or plain residue -- and every other instance of the
batch is verified as usual.  Each case runs refresh.collect (or collect_many)
and the oracle (restatement of refresh_message.rs:321-467) on the same
messages: the outcome (Ok / FsDkrError variant + payload / panic), the
paillier_key_vec side effects and, on success, the updated LocalKey must be
identical (helpers of tests/test_edge_outcomes_gpu.py)."""
import copy
import dataclasses
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from test_edge_outcomes_gpu import KB, _check, _dkr, _joins_setup  # noqa: E402
from test_negative_operands import (_alice, _pdl, dkr_negative_a, dkr_negative_c, dkr_negative_s3,  # noqa: E402
                                    dkr_negative_z)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dkr5():
    return _dkr(2, 5, "neg-gpu-t2n5")


def test_negative_s1_from_one_sender(gpu_ctx, dkr5):
    """The verdict's case: one sender's PDL s1 < 0 among valid proofs -> that
    pair's panic (u2_test_tmp = h^s1, zk_pdl_with_slack.rs:139); an earlier
    failing pair is reported first; the same s1 in another message alone."""
    keys, msgs, dks, _ = dkr5
    m2 = _pdl(msgs, 3, 1, s1=lambda p: -p.s1)
    _check(gpu_ctx, m2, keys[0], dks[0], expect="panic")
    m3 = _pdl(m2, 1, 4, u2=lambda p: p.u2 + 1)      # pair (1, 4) precedes (3, 1)
    _check(gpu_ctx, m3, keys[0], dks[0], expect="PDLwSlackProof")
    m4 = _pdl(msgs, 0, 0, s1=lambda p: -1)
    _check(gpu_ctx, m4, keys[0], dks[0], expect="panic")


def test_negative_pdl_u2_u3(gpu_ctx, dkr5):
    keys, msgs, dks, _ = dkr5
    ro = _check(gpu_ctx, _pdl(msgs, 2, 2, u2=lambda p: -p.u2), keys[0], dks[0], expect="PDLwSlackProof")
    assert ro[1] == {"is_u1_eq": True, "is_u2_eq": False, "is_u3_eq": True}
    ro = _check(gpu_ctx, _pdl(msgs, 4, 0, u3=lambda p: -p.u3, u2=lambda p: -p.u2), keys[0], dks[0],
                expect="PDLwSlackProof")
    assert ro[1] == {"is_u1_eq": True, "is_u2_eq": False, "is_u3_eq": False}


@pytest.fixture(scope="module")
def neg_s3():
    return dkr_negative_s3(2, 5, "neg-s3-gpu-t2n5", {2, 5})


def test_negative_pdl_s3(gpu_ctx, neg_s3):
    """s3 < 0 raises h2^-1 to |s3| (commitment_unknown_order,
    zk_pdl_with_slack.rs:177-184): valid proofs from two senders -> Ok with the
    oracle's LocalKey; a wrong u3 on such a pair -> a new challenge, all false; a sign-flipped
    positive s3 -> u3 false; h2 not a unit -> the mod_inv unwrap panic."""
    keys, msgs, dks = neg_s3
    assert sum(p.s3 < 0 for m in msgs for p in m.pdl_proof_vec) == 10
    for r in (0, 3):
        assert _check(gpu_ctx, msgs, keys[r], dks[r]) is None
    ro = _check(gpu_ctx, _pdl(msgs, 1, 3, u3=lambda p: p.u3 + 1), keys[0], dks[0], expect="PDLwSlackProof")
    assert ro[1] == {"is_u1_eq": False, "is_u2_eq": False, "is_u3_eq": False}   # u3 is hashed into e
    ro = _check(gpu_ctx, _pdl(msgs, 0, 2, s3=lambda p: -p.s3), keys[0], dks[0], expect="PDLwSlackProof")
    assert ro[1] == {"is_u1_eq": True, "is_u2_eq": True, "is_u3_eq": False}
    ro = _check(gpu_ctx, _pdl(msgs, 4, 1, s3=lambda p: -p.s3), keys[0], dks[0], expect="PDLwSlackProof")
    assert ro[1] == {"is_u1_eq": True, "is_u2_eq": True, "is_u3_eq": False}
    key = keys[0].clone()
    st = key.h1_h2_n_tilde_vec[3]
    key.h1_h2_n_tilde_vec[3] = dataclasses.replace(st, ni=0)
    # the first message's s3 is positive: its u3 fails before any unwrap is reached
    _check(gpu_ctx, msgs, key, dks[0], expect="PDLwSlackProof")
    _check(gpu_ctx, _pdl(msgs, 0, 3, s3=lambda p: -p.s3), key, dks[0], expect="panic")


def test_negative_z(gpu_ctx):
    """z < 0 is hashed as |z| and reduced in z^e mod N~ (zk_pdl_with_slack.rs:114-122,
    151-157; range_proofs.rs:129,150-157): valid PDL proofs carrying z - N~ -> Ok
    with the oracle's LocalKey; a sign-flipped PDL / Alice z -> the oracle's outcome
    (the same challenge, z^e off by (-1)^e: Ok for an even e); z = -N~ (residue 0,
    no z^-1) -> the oracle's outcome."""
    keys, msgs, dks = dkr_negative_z(2, 5, "neg-z-gpu-t2n5", {3})
    assert all(p.z < 0 for p in msgs[2].pdl_proof_vec)
    for r in (0, 2):
        assert _check(gpu_ctx, msgs, keys[r], dks[r]) is None
    # -z: the same hash, z^e times (-1)^e -- fails only for an odd challenge
    outs = [_check(gpu_ctx, _pdl(msgs, k, i, z=lambda p: -p.z), keys[0], dks[0]) for k in (0, 1) for i in range(5)]
    outs += [_check(gpu_ctx, _alice(msgs, k, i, z=lambda a: -a.z), keys[0], dks[0]) for k, i in ((1, 3), (3, 0), (4, 4))]
    assert {o[0] for o in outs if o} == {"PDLwSlackProof", "RangeProof"}, outs
    nt = keys[0].h1_h2_n_tilde_vec[1].N
    _check(gpu_ctx, _pdl(msgs, 3, 1, z=lambda p: -nt), keys[0], dks[0])
    _check(gpu_ctx, _alice(msgs, 4, 1, z=lambda a: -nt), keys[0], dks[0])


def test_negative_ciphertext(gpu_ctx):
    """c < 0: both proofs hash |c| (zk_pdl_with_slack.rs:117, range_proofs.rs:153),
    c^e, c^-1 and the share decryption reduce it (:136-142, range_proofs.rs:142,
    refresh_message.rs:221-234).  Valid proofs over c - N^2 (one sender, the
    local party's own ciphertext among them) -> Ok with the oracle's LocalKey;
    a sign-flipped c and c = -N^2 -> the oracle's outcome."""
    keys, msgs, dks = dkr_negative_c(2, 5, "neg-c-gpu-t2n5", {2})
    assert all(c < 0 for c in msgs[1].points_encrypted_vec)
    for r in (0, 1, 4):   # receiver 1 decrypts its own negative ciphertext
        assert _check(gpu_ctx, msgs, keys[r], dks[r]) is None
    outs = []
    for k, i in ((0, 2), (3, 4), (4, 0), (2, 3)):
        m2 = copy.deepcopy(msgs)
        m2[k].points_encrypted_vec[i] = -m2[k].points_encrypted_vec[i]
        outs.append(_check(gpu_ctx, m2, keys[0], dks[0]))
    assert any(outs), outs
    m3 = copy.deepcopy(msgs)
    m3[3].points_encrypted_vec[2] = -keys[0].paillier_key_vec[2].n ** 2
    _check(gpu_ctx, m3, keys[0], dks[0])


def test_negative_ring_pedersen_a(gpu_ctx):
    """A_k < 0: the challenge hashes |A_k|, mod_mul reduces it (ring_pedersen_proof.rs:
    130-153).  Valid proofs over A_k - N (one sender) -> Ok with the oracle's
    LocalKey; a sign-flipped A_k (the same challenge, the check against -A_k)
    -> the oracle's RingPedersenProofError; both beside a negative Z (panic)."""
    keys, msgs, dks = dkr_negative_a(2, 5, "neg-a-gpu-t2n5", {5})
    assert sum(a < 0 for a in msgs[4].ring_pedersen_proof.A) == 86
    for r in (0, 3):
        assert _check(gpu_ctx, msgs, keys[r], dks[r]) is None
    m2 = copy.deepcopy(msgs)
    pf = m2[1].ring_pedersen_proof
    m2[1].ring_pedersen_proof = dataclasses.replace(pf, A=tuple(-a if k == 17 else a for k, a in enumerate(pf.A)))
    _check(gpu_ctx, m2, keys[0], dks[0], expect="RingPedersenProofError")
    m3 = copy.deepcopy(msgs)
    pf = m3[4].ring_pedersen_proof
    m3[4].ring_pedersen_proof = dataclasses.replace(pf, Z=tuple(-z if k == 200 else z for k, z in enumerate(pf.Z)))
    _check(gpu_ctx, m3, keys[0], dks[0], expect="panic")


def test_negative_alice_operands(gpu_ctx, dkr5):
    keys, msgs, dks, _ = dkr5
    _check(gpu_ctx, _alice(msgs, 1, 2, e=lambda a: -a.e), keys[0], dks[0], expect="panic")
    _check(gpu_ctx, _alice(msgs, 2, 0, s1=lambda a: -a.s1), keys[0], dks[0], expect="panic")
    _check(gpu_ctx, _alice(msgs, 0, 3, s2=lambda a: -a.s2), keys[0], dks[0], expect="panic")
    # z^e not invertible (z = 0): false before the negative s1's panic
    ro = _check(gpu_ctx, _alice(msgs, 1, 1, s1=lambda a: -a.s1, z=lambda a: 0), keys[0], dks[0], expect="RangeProof")
    assert ro[1] == {"party_index": 1}
    # the PDL check of the same pair fails first
    m2 = _pdl(_alice(msgs, 2, 4, e=lambda a: -a.e), 2, 4, u2=lambda p: p.u2 + 1)
    _check(gpu_ctx, m2, keys[0], dks[0], expect="PDLwSlackProof")


def test_negative_bases_are_residues(gpu_ctx, dkr5):
    """s2 - k N^2 and s - k N^2: the same proof to GMP's mod_pow -> Ok, and the
    LocalKey is updated exactly as the oracle's."""
    keys, msgs, dks, _ = dkr5
    nn = [k.n ** 2 for k in keys[0].paillier_key_vec]
    m2 = _pdl(msgs, 1, 2, s2=lambda p: p.s2 - nn[2])
    m2 = _alice(m2, 3, 4, s=lambda a: a.s - 2 * nn[4])
    assert _check(gpu_ctx, m2, keys[0], dks[0]) is None
    m3 = _alice(m2, 0, 0, s=lambda a: -a.s)           # a different residue: the proof fails
    _check(gpu_ctx, m3, keys[0], dks[0], expect="RangeProof")


def test_negative_ring_pedersen_z(gpu_ctx, dkr5):
    keys, msgs, dks, _ = dkr5
    m2 = copy.deepcopy(msgs)
    pf = m2[2].ring_pedersen_proof
    m2[2].ring_pedersen_proof = dataclasses.replace(pf, Z=tuple(-z if k == 40 else z for k, z in enumerate(pf.Z)))
    _check(gpu_ctx, m2, keys[0], dks[0], expect="panic")
    m3 = copy.deepcopy(m2)                             # check 3 fails before index 40 is reached
    pf = m3[2].ring_pedersen_proof
    m3[2].ring_pedersen_proof = dataclasses.replace(pf, Z=tuple(z + (k == 3) for k, z in enumerate(pf.Z)))
    _check(gpu_ctx, m3, keys[0], dks[0], expect="RingPedersenProofError")


@pytest.mark.parametrize("case", ["x1", "x2", "x1_y1", "x2_y2", "x1_y2"])
def test_negative_dlog_commitment(gpu_ctx, case):
    keys, msgs, dks, jm, _ = _joins_setup("neg-dlog-x")
    j2 = copy.deepcopy(jm)
    for part in case.split("_"):
        attr = "composite_dlog_proof_base_h1" if part[1] == "1" else "composite_dlog_proof_base_h2"
        p = getattr(j2, attr)
        setattr(j2, attr, dataclasses.replace(p, **{part[0]: -getattr(p, part[0])}))
    assert _check(gpu_ctx, msgs, keys[1], dks[1], [j2]) is not None


@pytest.mark.parametrize("which", ["y1", "y2"])
def test_negative_dlog_response(gpu_ctx, which):
    keys, msgs, dks, jm, _ = _joins_setup("neg-dlog")
    attr = "composite_dlog_proof_base_h1" if which == "y1" else "composite_dlog_proof_base_h2"
    j2 = copy.deepcopy(jm)
    p = getattr(j2, attr)
    setattr(j2, attr, dataclasses.replace(p, y=-p.y))
    _check(gpu_ctx, msgs, keys[1], dks[1], [j2], expect="panic")
    if which == "y2":   # proof 1 fails: proof 2 (and its panic) never runs
        p1 = j2.composite_dlog_proof_base_h1
        j2.composite_dlog_proof_base_h1 = dataclasses.replace(p1, x=p1.x + 1)
        _check(gpu_ctx, msgs, keys[1], dks[1], [j2], expect="DLogProofValidation")


def test_collect_many_negative_session_alone(gpu_ctx, dkr5):
    """collect_many: the session holding a negative s1 panics, the regular
    sessions around it succeed, each as the oracle says."""
    keys, msgs, dks, _ = dkr5
    m2 = _pdl(msgs, 4, 2, s1=lambda p: -p.s1)
    sessions = [(msgs, 0), (m2, 1), (msgs, 2)]
    _collect_many_like_oracle(gpu_ctx, keys, dks, sessions)


def test_collect_many_negative_z_session(gpu_ctx):
    """collect_many: a session of valid negative-z proofs (its own batch, neg_bits)
    beside regular sessions of the same keys."""
    keys, msgs, dks = dkr_negative_z(2, 5, "neg-z-many", {1})
    m_ok = _pdl(msgs, 0, 0, z=lambda p: p.z)
    _collect_many_like_oracle(gpu_ctx, keys, dks, [(msgs, 0), (m_ok, 3), (msgs, 4)])


def test_collect_many_negative_c_session(gpu_ctx):
    keys, msgs, dks = dkr_negative_c(2, 5, "neg-c-many", {4})
    m2 = copy.deepcopy(msgs)
    m2[0].points_encrypted_vec[3] = -m2[0].points_encrypted_vec[3]
    _collect_many_like_oracle(gpu_ctx, keys, dks, [(msgs, 0), (m2, 1), (msgs, 3)])


def test_collect_many_negative_s3_session(gpu_ctx, neg_s3):
    """collect_many: a session of valid negative-s3 proofs (packed on its own,
    pdl_s3_neg) succeeds beside regular sessions; one with a broken u3 fails."""
    keys, msgs, dks = neg_s3
    m2 = _pdl(msgs, 1, 0, u3=lambda p: p.u3 + 1)
    _collect_many_like_oracle(gpu_ctx, keys, dks, [(msgs, 0), (m2, 1), (msgs, 4)])


def _collect_many_like_oracle(gpu_ctx, keys, dks, sessions):
    from fsdkr import refresh
    from test_edge_outcomes_gpu import _same_key
    from oracle import protocol
    from oracle.rng import Rng
    gk = [keys[p].clone() for _, p in sessions]
    out = refresh.collect_many([(copy.deepcopy(m), k, dks[p], []) for (m, p), k in zip(sessions, gk)],
                               ctx=gpu_ctx, key_bits=KB)
    for (m, p), k, o in zip(sessions, gk, out):
        ko = keys[p].clone()
        try:
            protocol.collect(copy.deepcopy(m), ko, dks[p], [], Rng("a8"), KB)
            want = None
        except protocol.FsDkrError as e:
            want = (e.variant, e.fields)
        except Exception:
            want = "panic"
        if want is None:
            assert o is None, o
            _same_key(ko, k)
        elif want == "panic":
            assert isinstance(o, refresh.FsDkrPanic), o
        else:
            assert isinstance(o, refresh.FsDkrError) and (o.variant, o.fields) == want, (o, want)
