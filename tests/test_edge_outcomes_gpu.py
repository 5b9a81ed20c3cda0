"""Reference outcomes for adversarial shapes the kernels used to reject with
UnsupportedInput (VERDICT r1 "what's missing" 3): each case runs the GPU
collect() and the oracle (restatement of refresh_message.rs:321-467) on the
same messages; the outcome (Ok / FsDkrError variant + payload / panic), the
paillier_key_vec side effects and, on success, the updated LocalKey must be
identical.

Cases: commitment vectors of another length (curv Horner over the message's
own vector, refresh_message.rs:180-182; empty -> unwrap panic), short
range_proofs / A / Z / sigma_vec (index panics at the reference's position),
a LocalKey holding fewer keys than receivers (:334), an ek.n wider than the
batch (its correct-key proof at 4096 bits, then ModuliTooSmall, :376-391),
ek.n in {0, 1}, and EVEN ring-Pedersen / composite-DLog moduli (valid and
tampered proofs: Montgomery half modulo the odd part, 2-adic half in pow2.hip)."""
import copy

import pytest

from oracle import bigint, paillier, protocol
from oracle import secp256k1 as ec
from oracle.hashing import chain_bigint
from oracle.ring_pedersen import RingPedersenProof, RingPedersenStatement
from oracle.rng import Rng
from oracle.zk_paillier import CompositeDLogProof, DLogStatement, NiCorrectKeyProof

pytestmark = pytest.mark.gpu

KB = 1024
M = 256


def _dkr(t, n, seed, key_bits=KB):
    rng = Rng(seed)
    keys = protocol.simulate_keygen(t, n, rng, key_bits)
    msgs, dks = [], []
    for key in keys:
        m, dk = protocol.distribute(key.i, key, n, rng, key_bits)
        msgs.append(m)
        dks.append(dk)
    return keys, msgs, dks, rng


def _both(msgs, key, dk, joins, key_bits=KB, ctx=None):
    from fsdkr import refresh
    ko, kg = key.clone(), key.clone()
    ro = rg = None
    try:
        protocol.collect(copy.deepcopy(msgs), ko, dk, copy.deepcopy(joins), Rng("a8"), key_bits)
    except protocol.FsDkrError as e:
        ro = (e.variant, e.fields)
    except Exception as e:  # PanicError / IndexError / ZeroDivisionError: the reference panics
        ro = ("panic", type(e).__name__)
    try:
        refresh.collect(copy.deepcopy(msgs), kg, dk, copy.deepcopy(joins), ctx=ctx, key_bits=key_bits)
    except refresh.FsDkrError as e:
        rg = (e.variant, e.fields)
    except refresh.FsDkrPanic:
        rg = ("panic", "")
    return ro, rg, ko, kg


def _same(ro, rg):
    if ro is not None and ro[0] == "panic":
        return rg is not None and rg[0] == "panic"
    return ro == rg


def _same_key(a, b):
    assert (a.x_i, a.y, a.pk_vec) == (b.x_i, b.y, b.pk_vec)
    assert [k.n for k in a.paillier_key_vec] == [k.n for k in b.paillier_key_vec]


@pytest.fixture(scope="module")
def dkr5():
    return _dkr(2, 5, "edge-t2n5")


def _check(gpu_ctx, msgs, key, dk, joins=(), key_bits=KB, expect=None):
    ro, rg, ko, kg = _both(msgs, key, dk, list(joins), key_bits, gpu_ctx)
    assert _same(ro, rg), (ro, rg)
    if expect is not None:
        assert (ro[0] if ro else None) == expect, ro
    assert [k.n for k in ko.paillier_key_vec] == [k.n for k in kg.paillier_key_vec]
    if ro is None:
        _same_key(ko, kg)
    return ro


# --------------------------------------------------------------- commitments --
def test_commitments_extra_infinity_top(gpu_ctx, dkr5):
    """A degree-(t+1) vector whose top commitment is the point at infinity: same
    polynomial, every share validates -> Ok."""
    keys, msgs, dks, _ = dkr5
    m2 = copy.deepcopy(msgs)
    m2[2].coefficients_committed_vec.commitments.append(None)
    _check(gpu_ctx, m2, keys[0], dks[0], expect=None)


def test_commitments_truncated(gpu_ctx, dkr5):
    keys, msgs, dks, _ = dkr5
    m2 = copy.deepcopy(msgs)
    m2[3].coefficients_committed_vec.commitments.pop()
    _check(gpu_ctx, m2, keys[0], dks[0], expect="PublicShareValidationError")


def test_commitments_empty_panics(gpu_ctx, dkr5):
    keys, msgs, dks, _ = dkr5
    m2 = copy.deepcopy(msgs)
    m2[1].coefficients_committed_vec.commitments.clear()
    _check(gpu_ctx, m2, keys[0], dks[0], expect="panic")


def test_short_committed_points_checks_message0_first(gpu_ctx, dkr5):
    """points_committed_vec shorter than new_n: message 0's first shares are
    validated before the index panic (refresh_message.rs:177-188)."""
    keys, msgs, dks, _ = dkr5
    m2 = copy.deepcopy(msgs)
    for m in m2:
        m.pdl_proof_vec.pop()
        m.points_committed_vec.pop()
        m.points_encrypted_vec.pop()
    _check(gpu_ctx, m2, keys[0], dks[0], expect="panic")
    m3 = copy.deepcopy(m2)
    m3[0].points_committed_vec[1] = ec.mul(ec.G, 777)
    _check(gpu_ctx, m3, keys[0], dks[0], expect="PublicShareValidationError")


# --------------------------------------------------------------- short vectors --
def test_short_range_proofs_panic(gpu_ctx, dkr5):
    keys, msgs, dks, _ = dkr5
    m2 = copy.deepcopy(msgs)
    del m2[1].range_proofs[3:]
    _check(gpu_ctx, m2, keys[0], dks[0], expect="panic")
    # an earlier failing pair wins over the later index panic
    p = m2[0].pdl_proof_vec[2]
    m2[0].pdl_proof_vec[2] = type(p)(**{**p.__dict__, "u2": p.u2 + 1})
    _check(gpu_ctx, m2, keys[0], dks[0], expect="PDLwSlackProof")


def test_localkey_with_fewer_keys_panics(gpu_ctx, dkr5):
    keys, msgs, dks, _ = dkr5
    k = keys[0].clone()
    k.paillier_key_vec = k.paillier_key_vec[:3]
    _check(gpu_ctx, msgs, k, dks[0], expect="panic")


def test_short_ring_pedersen_vectors(gpu_ctx, dkr5):
    keys, msgs, dks, _ = dkr5
    m2 = copy.deepcopy(msgs)
    pf = m2[2].ring_pedersen_proof
    m2[2].ring_pedersen_proof = RingPedersenProof(pf.A[:M - 1], pf.Z)          # hash loop panics
    _check(gpu_ctx, m2, keys[0], dks[0], expect="panic")
    m3 = copy.deepcopy(msgs)
    pf = m3[2].ring_pedersen_proof
    m3[2].ring_pedersen_proof = RingPedersenProof(pf.A, pf.Z[:100])           # Z[100] panics
    _check(gpu_ctx, m3, keys[0], dks[0], expect="panic")
    m4 = copy.deepcopy(m3)
    pf = m4[2].ring_pedersen_proof
    m4[2].ring_pedersen_proof = RingPedersenProof(pf.A, (pf.Z[0] + 1,) + tuple(pf.Z[1:]))   # check 0 fails first
    _check(gpu_ctx, m4, keys[0], dks[0], expect="RingPedersenProofError")


def test_short_sigma_vec_panics(gpu_ctx, dkr5):
    keys, msgs, dks, _ = dkr5
    m2 = copy.deepcopy(msgs)
    m2[1].dk_correctness_proof = NiCorrectKeyProof(m2[1].dk_correctness_proof.sigma_vec[:10])
    _check(gpu_ctx, m2, keys[0], dks[0], expect="panic")


# --------------------------------------------------------------- Paillier keys --
def test_ek_zero_and_one(gpu_ctx, dkr5):
    keys, msgs, dks, _ = dkr5
    m2 = copy.deepcopy(msgs)
    m2[3].ek = paillier.EncryptionKey(1, 1)          # every value is 0 mod 1: proof Ok, then ModuliTooSmall
    _check(gpu_ctx, m2, keys[0], dks[0], expect="ModuliTooSmall")
    m3 = copy.deepcopy(msgs)
    m3[3].ek = paillier.EncryptionKey(0, 0)          # rho = mask % 0
    _check(gpu_ctx, m3, keys[0], dks[0], expect="panic")


def test_oversize_ek_moduli_too_small(gpu_ctx):
    """A 2048-bit session whose message carries a valid 4096-bit key: the
    correct-key proof is verified at 128 limbs, then ModuliTooSmall{4096}."""
    keys, msgs, dks, rng = _dkr(1, 3, "edge-oversize", key_bits=2048)
    ek, dk = paillier.keypair_with_modulus_size(4096, rng)
    m2 = copy.deepcopy(msgs)
    m2[2].ek = ek
    m2[2].dk_correctness_proof = NiCorrectKeyProof.proof(dk.p, dk.q)
    ro = _check(gpu_ctx, m2, keys[0], dks[0], key_bits=2048, expect="ModuliTooSmall")
    assert ro[1] == {"party_index": 3, "moduli_size": ek.n.bit_length()}
    # the same key with a broken proof: PaillierVerificationError before the size check
    m3 = copy.deepcopy(m2)
    sv = m3[2].dk_correctness_proof.sigma_vec
    m3[2].dk_correctness_proof = NiCorrectKeyProof((sv[0] + 1,) + tuple(sv[1:]))
    _check(gpu_ctx, m3, keys[0], dks[0], key_bits=2048, expect="PaillierVerificationError")


# --------------------------------------------------------------- even moduli --
def _even_rp(st, rp_pf, twos, rng):
    """A VALID ring-Pedersen proof for N' = 2^twos * N: T' odd with T' = T (mod N),
    S' = T'^lam, A_i = T'^a_i mod N', Z_i = a_i + e_i lam mod phi(N) (T'^phi = 1
    mod 2^twos for twos <= 4, since 4 | phi)."""
    N2 = st.N << twos
    T2 = st.T if st.T & 1 else st.T + st.N
    lam = rng.sample_below(st.phi)
    S2 = pow(T2, lam, N2)
    while True:
        a = [rng.sample_below(st.phi) for _ in range(M)]
        A = [pow(T2, x, N2) for x in a]
        eb = bigint.to_bytes(chain_bigint(*A))
        if 8 * len(eb) >= M:
            break
    bits = [(eb[i >> 3] >> (i & 7)) & 1 for i in range(M)]
    Z = [(a[i] + bits[i] * lam) % st.phi for i in range(M)]
    return RingPedersenStatement(S2, T2, N2, st.phi, st.ek), RingPedersenProof(tuple(A), tuple(Z))


def test_even_ring_pedersen_modulus(gpu_ctx, dkr5):
    keys, msgs, dks, rng = dkr5
    for twos in (1, 4):
        m2 = copy.deepcopy(msgs)
        st, pf = _even_rp(m2[1].ring_pedersen_statement, m2[1].ring_pedersen_proof, twos, rng)
        m2[1].ring_pedersen_statement, m2[1].ring_pedersen_proof = st, pf
        ro = _check(gpu_ctx, m2, keys[0], dks[0])
        assert ro is None, ro                       # valid proof modulo an even N
        m3 = copy.deepcopy(m2)                      # one Z off: the 2-adic or odd half fails
        m3[1].ring_pedersen_proof = RingPedersenProof(pf.A, tuple(z + (k == 9) for k, z in enumerate(pf.Z)))
        _check(gpu_ctx, m3, keys[0], dks[0], expect="RingPedersenProofError")
        m4 = copy.deepcopy(m2)                      # A_i + N: same residue mod N, differs mod 2^twos
        m4[1].ring_pedersen_proof = RingPedersenProof(
            tuple(x + (st.N >> twos) if k == 3 else x for k, x in enumerate(pf.A)), pf.Z)
        _check(gpu_ctx, m4, keys[0], dks[0])
    # N = 0: the first mod_pow divides by zero
    m5 = copy.deepcopy(msgs)
    s = m5[4].ring_pedersen_statement
    m5[4].ring_pedersen_statement = RingPedersenStatement(s.S, s.T, 0, s.phi, s.ek)
    _check(gpu_ctx, m5, keys[0], dks[0], expect="panic")


def _joins_setup(seed):
    rng = Rng(seed)
    t, n = 1, 4
    all_keys = protocol.simulate_keygen(t, n, rng, KB)
    keys = [k.clone() for k in all_keys[:3]]
    jm, kk = protocol.join_distribute(rng, KB)
    jm.set_party_index(4)
    msgs, dks = [], []
    for key in keys:
        m, dk = protocol.replace([jm], key, {1: 1, 2: 2, 3: 3}, 4, rng, KB)
        msgs.append(m)
        dks.append(dk)
    return keys, msgs, dks, jm, rng


def test_even_dlog_modulus(gpu_ctx):
    keys, msgs, dks, jm, rng = _joins_setup("edge-dlog")
    ro, rg, ko, kg = _both(msgs, keys[1], dks[1], [jm], KB, gpu_ctx)
    assert ro is None and rg is None
    # a fresh joiner statement over N' = 16 N~ with valid proofs for both bases
    twos = 4
    ek_t, dk_t = paillier.keypair_with_modulus_size(KB, rng)
    phi = (dk_t.p - 1) * (dk_t.q - 1)
    Nt = ek_t.n
    N2 = Nt << twos
    g = rng.sample_below(Nt) | 1
    while True:
        xhi = rng.sample_below(phi)
        if bigint.mod_inv(xhi, phi) is not None:
            break
    xinv = pow(xhi, -1, phi)
    ni = pow(g, xhi, N2)
    s1 = DLogStatement(N2, g, ni)
    s2 = DLogStatement(N2, ni, g)

    def prove(stmt, secret):
        r = rng.sample_below((1 << 512) * stmt.N)
        x = pow(stmt.g, r, stmt.N)
        e = CompositeDLogProof.challenge(x, stmt)
        return CompositeDLogProof(x, r + e * secret)
    j2 = copy.deepcopy(jm)
    j2.dlog_statement = s1
    j2.composite_dlog_proof_base_h1 = prove(s1, phi - xhi)      # g^(r + e(phi - xhi)) * ni^e = g^r
    j2.composite_dlog_proof_base_h2 = prove(s2, phi - xinv)     # ni^(r + e(phi - xinv)) * g^e = ni^r
    assert j2.composite_dlog_proof_base_h1.verify(s1) and j2.composite_dlog_proof_base_h2.verify(s2)
    ro = _check(gpu_ctx, msgs, keys[1], dks[1], [j2])
    assert ro is None, ro
    j3 = copy.deepcopy(j2)                                       # x + N~: equal mod N~, differs mod 16
    p = j3.composite_dlog_proof_base_h2
    j3.composite_dlog_proof_base_h2 = CompositeDLogProof((p.x + Nt) % N2, p.y)
    _check(gpu_ctx, msgs, keys[1], dks[1], [j3], expect="DLogProofValidation")


# ------------------------------------------------ share recovery in the order --
def _bad_ck(msgs, k):
    m2 = copy.deepcopy(msgs)
    sv = m2[k].dk_correctness_proof.sigma_vec
    m2[k].dk_correctness_proof = NiCorrectKeyProof((sv[0] + 1,) + tuple(sv[1:]))
    return m2


def test_ciphertext_sum_panic_precedes_later_checks(gpu_ctx, dkr5):
    """get_ciphertext_sum (refresh_message.rs:367-373) runs after the ring-Pedersen
    checks and before the correct-key / moduli checks and the paillier_key_vec
    writes: with a broken correct-key proof AND a LocalKey whose VSS threshold asks
    for more messages than there are (refresh_messages[i] out of bounds), or whose
    own index is past the ciphertext vectors, the reference panics and writes no
    key.  Same on both orders of share recovery."""
    from fsdkr import refresh
    keys, msgs, dks, _ = dkr5
    m2 = _bad_ck(msgs, 2)
    k1 = keys[0].clone()
    k1.vss_scheme.threshold = len(msgs)
    assert _check(gpu_ctx, m2, k1, dks[0], expect="panic")
    k2 = keys[0].clone()
    k2.i = len(msgs) + 3
    assert _check(gpu_ctx, m2, k2, dks[0], expect="panic")
    for recovery in refresh.RECOVERY_MODES:
        kg = k1.clone()
        with pytest.raises(refresh.FsDkrPanic):
            refresh.collect(copy.deepcopy(m2), kg, dks[0], [], ctx=gpu_ctx, key_bits=KB, recovery=recovery)
        assert [k.n for k in kg.paillier_key_vec] == [k.n for k in k1.paillier_key_vec]
    # without the correct-key tamper the reference reaches the same panic
    _check(gpu_ctx, msgs, k1, dks[0], expect="panic")
    # a failing check BEFORE get_ciphertext_sum wins over its panic
    m3 = copy.deepcopy(msgs)
    p = m3[1].range_proofs[2]
    m3[1].range_proofs[2] = type(p)(**{**p.__dict__, "s2": p.s2 + 1})
    _check(gpu_ctx, m3, k1, dks[0], expect="RangeProof")


def test_degenerate_local_dk_fails_alone(gpu_ctx, dkr5):
    """A LocalKey whose Paillier dk the batched decryption refuses (p == q): that
    collect fails with a panic, the batch is not left in flight (the next collect
    runs), and in collect_all the other parties still get their keys."""
    from fsdkr import refresh
    from fsdkr.types import DecryptionKey
    keys, msgs, dks, _ = dkr5
    bad = keys[1].clone()
    bad.paillier_dk = DecryptionKey(keys[1].paillier_dk.p, keys[1].paillier_dk.p)
    with pytest.raises(refresh.FsDkrPanic):
        refresh.collect(copy.deepcopy(msgs), bad, dks[1], [], ctx=gpu_ctx, key_bits=KB)
    ok = keys[0].clone()
    refresh.collect(copy.deepcopy(msgs), ok, dks[0], [], ctx=gpu_ctx, key_bits=KB)
    ko = keys[0].clone()
    protocol.collect(copy.deepcopy(msgs), ko, dks[0], [], Rng("a8"), KB)
    _same_key(ko, ok)
    # (the failed collect above applied every new ek before its decryption panic,
    # as the reference does: a fresh copy of the degenerate key for collect_all)
    bad2 = keys[1].clone()
    bad2.paillier_dk = DecryptionKey(keys[1].paillier_dk.p, keys[1].paillier_dk.p)
    assert [k.n for k in bad.paillier_key_vec] == [m.ek.n for m in msgs]
    parties = [(keys[0].clone(), dks[0]), (bad2, dks[1]), (keys[2].clone(), dks[2])]
    out = refresh.collect_all(copy.deepcopy(msgs), parties, [], ctx=gpu_ctx, key_bits=KB)
    assert out[0] is None and out[2] is None and isinstance(out[1], refresh.FsDkrPanic)
    _same_key(ko, parties[0][0])


def test_recovery_orders_agree(gpu_ctx, dkr5):
    """recovery="after" (decrypt once the verdicts are in, refresh_message.rs:439)
    and the default speculative recovery give the same LocalKey and the same
    error with the same side effects, for collect, collect_all and collect_many."""
    from fsdkr import refresh
    keys, msgs, dks, _ = dkr5
    outs = {}
    for recovery in refresh.RECOVERY_MODES:
        k = keys[3].clone()
        refresh.collect(copy.deepcopy(msgs), k, dks[3], [], ctx=gpu_ctx, key_bits=KB, recovery=recovery)
        bad = keys[3].clone()
        e = None
        try:
            refresh.collect(_bad_ck(msgs, 4), bad, dks[3], [], ctx=gpu_ctx, key_bits=KB, recovery=recovery)
        except refresh.FsDkrError as x:
            e = (x.variant, x.fields)
        parties = [(keys[i].clone(), dks[i]) for i in range(3)]
        res = refresh.collect_all(copy.deepcopy(msgs), parties, [], ctx=gpu_ctx, key_bits=KB, recovery=recovery)
        sess = [(copy.deepcopy(msgs), keys[i].clone(), dks[i], []) for i in (0, 4)]
        many = refresh.collect_many(sess, ctx=gpu_ctx, key_bits=KB, recovery=recovery)
        outs[recovery] = (k, e, [p[0] for p in parties], res, [s[1] for s in sess], many,
                          [x.n for x in bad.paillier_key_vec])
    a, b = outs["speculative"], outs["after"]
    _same_key(a[0], b[0])
    assert a[1] == b[1] == ("PaillierVerificationError", {"party_index": 5})
    assert a[6] == b[6]
    for x, y in zip(a[2], b[2]):
        _same_key(x, y)
    assert a[3] == b[3] == [None] * 3
    for x, y in zip(a[4], b[4]):
        _same_key(x, y)
    assert a[5] == b[5] == [None, None]
    with pytest.raises(ValueError):
        refresh.collect(msgs, keys[0].clone(), dks[0], [], ctx=gpu_ctx, recovery="later")


def test_join_collect_non_unit_ciphertext(gpu_ctx):
    """JoinMessage::collect decrypts without a PDL check (add_party_message.rs:183-213),
    so a refresh message may carry, for the joiner, a ciphertext divisible by the
    joiner's p.  The reference decrypts Enc(0) * prod_k c_k^l_k once
    with kzen-paillier's CRT decryption: p divides the product, so the p half is
    L_p(0) h_p = 0 (truncating division); the product's per-half recovery
    (csrc/recover.cpp) and the oracle (oracle/paillier.decrypt) both follow it.
    The decomposition sum_k l_k Dec(c_k) would have kept the other messages'
    p halves.  (kzen-paillier's own source is not in the image: parity with it
    is pinned only by this restatement.)"""
    from fsdkr import join
    rng = Rng("edge-nonunit")
    t, n = 1, 4
    all_keys = protocol.simulate_keygen(t, n, rng, KB)
    keys = [k.clone() for k in all_keys[:3]]
    jm, kk = protocol.join_distribute(rng, KB)
    jm.set_party_index(4)
    msgs = [protocol.replace([jm], key, {1: 1, 2: 2, 3: 3}, 4, rng, KB)[0] for key in keys]
    honest = join.collect(jm, copy.deepcopy(msgs), kk, [], t, n, ctx=gpu_ctx, key_bits=KB, rng=Rng("jc"))
    m2 = copy.deepcopy(msgs)
    N2 = kk.ek.n * kk.ek.n
    m2[0].points_encrypted_vec[3] = m2[0].points_encrypted_vec[3] * kk.dk.p % N2
    lo = protocol.join_collect(jm, copy.deepcopy(m2), kk, [], t, n, Rng("jc"), KB)
    lg = join.collect(jm, copy.deepcopy(m2), kk, [], t, n, ctx=gpu_ctx, key_bits=KB, rng=Rng("jc"))
    assert (lo.x_i, lo.y, lo.pk_vec) == (lg.x_i, lg.y, lg.pk_vec)
    assert lg.x_i != honest.x_i


def test_ciphertext_wider_than_n_squared(gpu_ctx, dkr5):
    """A ciphertext c + k N^2 wider than 2^(64 nl).  In
    RefreshMessage::collect the PDL transcript hashes c itself, so the pair's
    proof fails (same error in the oracle and on the GPU, whose batch runs at the
    3072-bit width).  JoinMessage::collect has no PDL check: there Paillier::mul /
    add / decrypt reduce mod N^2, so the joiner recovers the same share as with c;
    the share recovery reduces the ciphertext mod N^2 before the C ABI (which
    takes values < 2^(64 nl))."""
    from fsdkr import join
    keys, msgs, dks, _ = dkr5
    i = 2
    N2 = keys[i].paillier_key_vec[i].n ** 2
    m2 = copy.deepcopy(msgs)
    m2[0].points_encrypted_vec[i] += N2 << 2100
    assert m2[0].points_encrypted_vec[i].bit_length() > 64 * 64
    ro = _check(gpu_ctx, m2, keys[i], dks[i])
    assert ro is not None and ro[0] == "PDLwSlackProof", ro
    # the join path
    rng = Rng("edge-wide-join")
    t, n = 1, 4
    all_keys = protocol.simulate_keygen(t, n, rng, KB)
    jm, kk = protocol.join_distribute(rng, KB)
    jm.set_party_index(4)
    jmsgs = [protocol.replace([jm], k.clone(), {1: 1, 2: 2, 3: 3}, 4, rng, KB)[0] for k in all_keys[:3]]
    honest = join.collect(jm, copy.deepcopy(jmsgs), kk, [], t, n, ctx=gpu_ctx, key_bits=KB, rng=Rng("jc"))
    j2 = copy.deepcopy(jmsgs)
    j2[0].points_encrypted_vec[3] += (kk.ek.n ** 2) << 2100
    lo = protocol.join_collect(jm, copy.deepcopy(j2), kk, [], t, n, Rng("jc"), KB)
    lg = join.collect(jm, copy.deepcopy(j2), kk, [], t, n, ctx=gpu_ctx, key_bits=KB, rng=Rng("jc"))
    assert (lo.x_i, lo.y, lo.pk_vec) == (lg.x_i, lg.y, lg.pk_vec) == (honest.x_i, honest.y, honest.pk_vec)
