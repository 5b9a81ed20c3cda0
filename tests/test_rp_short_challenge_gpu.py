"""RingPedersenProof::verify with a challenge shorter than M bits
(ring_pedersen_proof.rs:135-142; VERDICT r3 "what's missing" 2).

The challenge is e = SHA-256(A_0 .. A_255) read as BitVec::from_vec(e.to_bytes()):
curv's to_bytes is the minimal big-endian magnitude, so a digest whose top byte
is zero leaves 31 bytes = 248 bits and bitwise_e[248] panics -- unless a check
at an index below 248 already returned RingPedersenProofError.  No honest
prover emits such a proof (its own loop indexes the same bits, :106-116), so
the proofs here are built by hand: a fresh witness lambda over the message's
own (N, T, phi), S = T^lambda, A_i = T^a_i with a_0 re-drawn until the digest's
top byte is zero (about 256 draws), and Z_i = a_i + e_i lambda mod phi for the
248 readable bits (Z_248.. are never read).

Three outcomes, GPU (ped_hash_kernel's panic index 1 + 8 * digest bytes,
csrc/vhash.hip) against the oracle (oracle/ring_pedersen.py):
  1. RefreshMessage::collect, the proof otherwise valid: panic;
  2. the same proof with Z_5 off by one: RingPedersenProofError wins;
  3. JoinMessage::collect (add_party_message.rs:146-168) on the same proof: panic.
"""
import copy

import pytest

from oracle import bigint, protocol
from oracle.hashing import chain_bigint
from oracle.ring_pedersen import RingPedersenProof, RingPedersenStatement
from oracle.rng import Rng

pytestmark = pytest.mark.gpu

KB = 1024
M = 256


def short_challenge_proof(st, rng, max_draws=20000):
    """(statement, proof, bits) with SHA-256(A) < 2^248: a valid proof for the
    readable bits.  Deterministic for a given rng."""
    lam = rng.sample_below(st.phi)
    S = pow(st.T, lam, st.N)
    a = [rng.sample_below(st.phi) for _ in range(M)]
    A = [pow(st.T, x, st.N) for x in a]
    for _ in range(max_draws):
        eb = bigint.to_bytes(chain_bigint(*A))
        if len(eb) < 32:
            break
        a[0] = rng.sample_below(st.phi)
        A[0] = pow(st.T, a[0], st.N)
    else:
        raise AssertionError("no short challenge found")
    readable = 8 * len(eb)
    bits = [(eb[i >> 3] >> (i & 7)) & 1 for i in range(readable)]
    Z = [(a[i] + bits[i] * lam) % st.phi if i < readable else a[i] for i in range(M)]
    st2 = RingPedersenStatement(S, st.T, st.N, st.phi, st.ek)
    return st2, RingPedersenProof(tuple(A), tuple(Z)), bits


def _outcome_oracle(fn):
    try:
        fn()
    except protocol.FsDkrError as e:
        return (e.variant, e.fields)
    except Exception as e:   # PanicError / IndexError: the reference panics
        return ("panic", type(e).__name__)
    return None


def _outcome_gpu(fn):
    from fsdkr import refresh
    try:
        fn()
    except refresh.FsDkrError as e:
        return (e.variant, e.fields)
    except refresh.FsDkrPanic:
        return ("panic", "")
    return None


@pytest.fixture(scope="module")
def refresh_set():
    rng = Rng("rp-short-t2n5")
    keys = protocol.simulate_keygen(2, 5, rng, KB)
    msgs, dks = [], []
    for key in keys:
        m, dk = protocol.distribute(key.i, key, 5, rng, KB)
        msgs.append(m)
        dks.append(dk)
    st, pf, bits = short_challenge_proof(msgs[2].ring_pedersen_statement, Rng("rp-short-draw"))
    return keys, msgs, dks, st, pf, bits


def test_short_challenge_fixture_is_short(refresh_set):
    _, _, _, st, pf, bits = refresh_set
    assert len(bits) == 248
    # every readable check holds: only the BitVec index stops the reference
    for i in range(248):
        assert pow(st.T, pf.Z[i], st.N) == pf.A[i] * pow(st.S, bits[i], st.N) % st.N


def test_refresh_collect_panics_at_bit_248(gpu_ctx, refresh_set):
    from fsdkr import refresh
    keys, msgs, dks, st, pf, _ = refresh_set
    m2 = copy.deepcopy(msgs)
    m2[2].ring_pedersen_statement, m2[2].ring_pedersen_proof = st, pf
    ko, kg = keys[0].clone(), keys[0].clone()
    ro = _outcome_oracle(lambda: protocol.collect(copy.deepcopy(m2), ko, dks[0], [], Rng("a8"), KB))
    rg = _outcome_gpu(lambda: refresh.collect(copy.deepcopy(m2), kg, dks[0], [], ctx=gpu_ctx, key_bits=KB))
    assert ro is not None and ro[0] == "panic", ro
    assert rg is not None and rg[0] == "panic", rg
    assert [k.n for k in ko.paillier_key_vec] == [k.n for k in kg.paillier_key_vec]


def test_refresh_collect_earlier_failure_wins(gpu_ctx, refresh_set):
    from fsdkr import refresh
    keys, msgs, dks, st, pf, _ = refresh_set
    m2 = copy.deepcopy(msgs)
    m2[2].ring_pedersen_statement = st
    m2[2].ring_pedersen_proof = RingPedersenProof(pf.A, tuple(z + (k == 5) for k, z in enumerate(pf.Z)))
    ko, kg = keys[1].clone(), keys[1].clone()
    ro = _outcome_oracle(lambda: protocol.collect(copy.deepcopy(m2), ko, dks[1], [], Rng("a8"), KB))
    rg = _outcome_gpu(lambda: refresh.collect(copy.deepcopy(m2), kg, dks[1], [], ctx=gpu_ctx, key_bits=KB))
    assert ro == rg == ("RingPedersenProofError", {}), (ro, rg)
    assert [k.n for k in ko.paillier_key_vec] == [k.n for k in kg.paillier_key_vec]


def test_join_collect_panics_on_short_challenge(gpu_ctx):
    """JoinMessage::collect verifies every refresh message's ring-Pedersen proof
    first (add_party_message.rs:146-154): the short challenge panics there."""
    from fsdkr import join
    rng = Rng("rp-short-join")
    t, n = 1, 4
    all_keys = protocol.simulate_keygen(t, n, rng, KB)
    keys = [k.clone() for k in all_keys[:3]]
    jm, kk = protocol.join_distribute(rng, KB)
    jm.set_party_index(4)
    msgs = [protocol.replace([jm], key, {1: 1, 2: 2, 3: 3}, 4, rng, KB)[0] for key in keys]
    # unmodified: both sides recover the same key
    lo = protocol.join_collect(jm, copy.deepcopy(msgs), kk, [], t, n, Rng("jc"), KB)
    lg = join.collect(jm, copy.deepcopy(msgs), kk, [], t, n, ctx=gpu_ctx, key_bits=KB, rng=Rng("jc"))
    assert (lo.x_i, lo.y, lo.pk_vec) == (lg.x_i, lg.y, lg.pk_vec)
    st, pf, _ = short_challenge_proof(msgs[1].ring_pedersen_statement, Rng("rp-short-join-draw"))
    m2 = copy.deepcopy(msgs)
    m2[1].ring_pedersen_statement, m2[1].ring_pedersen_proof = st, pf
    ro = _outcome_oracle(lambda: protocol.join_collect(jm, copy.deepcopy(m2), kk, [], t, n, Rng("jc"), KB))
    rg = _outcome_gpu(lambda: join.collect(jm, copy.deepcopy(m2), kk, [], t, n, ctx=gpu_ctx, key_bits=KB,
                                           rng=Rng("jc")))
    assert ro is not None and ro[0] == "panic", ro
    assert rg is not None and rg[0] == "panic", rg
    # an earlier failing check in the same proof: the join path's error variant
    m3 = copy.deepcopy(m2)
    m3[1].ring_pedersen_proof = RingPedersenProof(pf.A, tuple(z + (k == 7) for k, z in enumerate(pf.Z)))
    ro = _outcome_oracle(lambda: protocol.join_collect(jm, copy.deepcopy(m3), kk, [], t, n, Rng("jc"), KB))
    rg = _outcome_gpu(lambda: join.collect(jm, copy.deepcopy(m3), kk, [], t, n, ctx=gpu_ctx, key_bits=KB,
                                           rng=Rng("jc")))
    assert ro == rg and ro[0] == "RingPedersenProofValidation", (ro, rg)
