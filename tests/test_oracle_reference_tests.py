"""The reference's own tests, restated against the oracle (CPU).

zk_pdl_with_slack.rs:205-266 / :268-331, range_proofs.rs:650-670,
ring_pedersen_proof.rs:166-178, test.rs:34-224 (GG20 signing replaced by
secret-reconstruction and public-key consistency checks; GG20 itself is out of
scope)."""
import pytest

from oracle import bigint, paillier, protocol, range_proofs, ring_pedersen
from oracle import secp256k1 as ec
from oracle import zk_pdl_with_slack as pdl
from oracle.rng import Rng
from oracle.zk_paillier import CompositeDLogProof, DLogStatement

KB = 2048


def _pdl_setup(rng, plus_one=False):
    """zk_pdl_with_slack.rs:207-253."""
    ek_t, dk_t = paillier.keypair_with_modulus_size(KB, rng)
    phi = (dk_t.p - 1) * (dk_t.q - 1)
    h1 = rng.sample_below(phi)
    xhi = rng.sample_below(1 << 256)
    h1_inv = bigint.mod_inv(h1, ek_t.n)
    h2 = bigint.mod_pow(h1_inv, xhi, ek_t.n)
    st_dlog = DLogStatement(ek_t.n, h1, h2)
    cdl = CompositeDLogProof.prove(st_dlog, xhi, rng)
    ek, _ = paillier.keypair_with_modulus_size(KB, rng)
    r = rng.sample_below(ek.n)
    x = rng.sample_below(ec.Q)
    Q = ec.mul(ec.G, x)
    c = paillier.encrypt_with_chosen_randomness(ek, x + (1 if plus_one else 0), r)
    st = pdl.PDLwSlackStatement(c, ek, Q, ec.G, h1, h2, ek_t.n)
    return st, st_dlog, cdl, x, r


def test_zk_pdl_with_slack():
    rng = Rng("test_zk_pdl_with_slack")
    st, st_dlog, cdl, x, r = _pdl_setup(rng)
    proof = pdl.prove(x, r, st, rng)
    assert cdl.verify(st_dlog)
    pdl.verify(proof, st)


def test_zk_pdl_with_slack_soundness():
    rng = Rng("test_zk_pdl_with_slack_soundness")
    st, st_dlog, cdl, x, r = _pdl_setup(rng, plus_one=True)
    proof = pdl.prove(x, r, st, rng)
    assert cdl.verify(st_dlog)
    with pytest.raises(pdl.PDLwSlackError) as ei:
        pdl.verify(proof, st)
    assert ei.value.flags == (True, False, True)    # only the Paillier relation breaks


def test_alice_zkp():
    """range_proofs.rs:626-670."""
    rng = Rng("alice_zkp")
    ek_t, dk_t = paillier.keypair_with_modulus_size(KB, rng)
    phi = (dk_t.p - 1) * (dk_t.q - 1)
    h1 = rng.sample_below(ek_t.n)
    while True:
        xhi = rng.sample_below(phi)
        if bigint.mod_inv(xhi, phi) is not None:
            break
    h2 = bigint.mod_pow(h1, xhi, ek_t.n)
    ek, _ = paillier.keypair_with_modulus_size(KB, rng)
    st = DLogStatement(ek_t.n, h1, h2)
    a = rng.sample_below(ec.Q)
    r = rng.from_modulo(ek.n)
    cipher = paillier.encrypt_with_chosen_randomness(ek, a, r)
    proof = range_proofs.generate(a, cipher, ek, st, r, rng)
    assert range_proofs.verify(proof, cipher, ek, st)
    bad = range_proofs.AliceProof(proof.z, proof.e, proof.s, proof.s1, proof.s2 + 1)
    assert not range_proofs.verify(bad, cipher, ek, st)


def test_ring_pedersen():
    rng = Rng("test_ring_pedersen")
    st, wit = ring_pedersen.generate(KB, rng)
    while True:
        try:
            proof = ring_pedersen.prove(wit, st, protocol.M_SECURITY, rng)
            break
        except bigint.PanicError:
            continue
    assert ring_pedersen.verify(proof, st, protocol.M_SECURITY)


# ---- protocol flows (small keys keep the CPU suite fast; flows are size-independent)
SMALL = 1024   # Paillier N must exceed (t+1)*q^2 for the decrypted share (refresh_message.rs:439)


def _simulate_dkr(keys, rng, key_bits=SMALL):
    """test.rs:311-334."""
    n = len(keys)
    msgs, dks = [], []
    for key in keys:
        m, dk = protocol.distribute(key.i, key, n, rng, key_bits)
        msgs.append(m)
        dks.append(dk)
    for i in range(n):
        protocol.collect(msgs, keys[i], dks[i], [], rng, key_bits)
    return msgs, dks


@pytest.mark.slow
def test1_refresh_preserves_secret():
    """test.rs:34-67 (t=3, n=6)."""
    rng = Rng("test1")
    t, n = 3, 6
    keys = protocol.simulate_keygen(t, n, rng, SMALL)
    old = [k.x_i for k in keys]
    _simulate_dkr(keys, rng)
    new = [k.x_i for k in keys]
    idx = list(range(t + 1))
    assert protocol.reconstruct(idx, old[:t + 1]) == protocol.reconstruct(idx, new[:t + 1])
    assert old != new


def test_sign_rotate_sign_without_signing():
    """test.rs:69-80 (t=2, n=5): two refreshes; every (t+1)-subset keeps
    reconstructing the same secret and y = G*x_i holds for every party."""
    rng = Rng("rotate")
    t, n = 2, 5
    keys = protocol.simulate_keygen(t, n, rng, SMALL)
    y0 = keys[0].y_sum_s
    secret = protocol.reconstruct([0, 1, 2], [k.x_i for k in keys[:3]])
    for _ in range(2):
        _simulate_dkr(keys, rng)
        for subset in ([1, 2, 3], [0, 2, 4]):
            assert protocol.reconstruct(subset, [keys[i].x_i for i in subset]) == secret
        for k in keys:
            assert k.y == ec.mul(ec.G, k.x_i)
            assert k.y_sum_s == y0
            assert k.pk_vec[k.i - 1] == k.y       # pk_vec insert quirk keeps the new keys first
    assert ec.mul(ec.G, secret) == y0


def test_remove_party_collect_fails():
    """test.rs:82-93,238-309: a removed party receives only its own message."""
    rng = Rng("remove")
    t, n = 2, 5
    keys = protocol.simulate_keygen(t, n, rng, SMALL)
    msgs, dks = [], []
    for key in keys:
        m, dk = protocol.distribute(key.i, key, n, rng, SMALL)
        msgs.append(m)
        dks.append(dk)
    with pytest.raises(protocol.FsDkrError) as ei:
        protocol.collect([msgs[0]], keys[0], dks[0], [], rng, SMALL)
    assert ei.value.variant == "PartiesThresholdViolation"
    assert ei.value.fields == {"threshold": 2, "refreshed_keys": 1}


@pytest.mark.slow
def test_add_party_with_permute():
    """test.rs:95-224 (t=2, n=7; parties 2 and 7 replaced by joiners)."""
    rng = Rng("permute")
    t, n = 2, 7
    all_keys = protocol.simulate_keygen(t, n, rng, SMALL)
    keys = [k.clone() for k in all_keys]
    del keys[6]
    del keys[1]
    old_to_new = {1: 4, 3: 1, 4: 3, 5: 6, 6: 5}
    joins, new_keys = [], []
    for pi in (2, 7):
        jm, kk = protocol.join_distribute(rng, SMALL)
        jm.set_party_index(pi)
        joins.append(jm)
        new_keys.append(kk)
    msgs, dks = [], []
    for key in keys:
        m, dk = protocol.replace(joins, key, old_to_new, len(keys) + len(joins), rng, SMALL)
        msgs.append(m)
        dks.append(dk)
    out = []
    for i in range(len(keys)):
        protocol.collect(msgs, keys[i], dks[i], joins, rng, SMALL)
        out.append((keys[i].i - 1, keys[i]))
    for jm, kk in zip(joins, new_keys):
        lk = protocol.join_collect(jm, msgs, kk, joins, t, n, rng, SMALL)
        out.append((jm.party_index - 1, lk))
    out.sort(key=lambda p: p[0])
    new_keys_sorted = [p[1] for p in out]
    secret_old = protocol.reconstruct([0, 1, 2], [k.x_i for k in all_keys[:3]])
    secret_new = protocol.reconstruct([0, 1, 2], [k.x_i for k in new_keys_sorted[:3]])
    assert secret_old == secret_new
    assert protocol.reconstruct([0, 1, 6], [new_keys_sorted[i].x_i for i in (0, 1, 6)]) == secret_old
