"""RefreshMessage::distribute on the GPU engine (fsdkr.distribute) against the
oracle's distribute (refresh_message.rs:51-145): with the same injected draws
the whole message -- encryptions (job 1), every PDL / Alice proof, Feldman
commitments, the new Paillier key and its correct-key proof, the ring-Pedersen
statement and proof -- and the decryption key are identical, and the
GPU-made messages pass the GPU collect()."""
import copy
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

import codec  # noqa: E402
from oracle import protocol  # noqa: E402
from oracle.rng import Rng  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kb,t,n", [(1024, 1, 3), (1024, 2, 5), (2048, 1, 2)])
def test_distribute_matches_oracle(gpu_ctx, kb, t, n):
    from fsdkr import distribute, refresh
    keys = protocol.simulate_keygen(t, n, Rng(f"dist-keys-{kb}-{n}"), kb)
    msgs, dks, kgs = [], [], []
    for key in keys[:n if kb == 1024 else 1]:
        ko, kg = key.clone(), key.clone()
        seed = f"dist-{kb}-{n}-{key.i}"
        mo, dko = protocol.distribute(ko.i, ko, n, Rng(seed), kb)
        mg, dkg = distribute.distribute(kg.i, kg, n, Rng(seed), ctx=gpu_ctx, key_bits=kb)
        assert codec.enc(mg) == codec.enc(mo)
        assert (dkg.p, dkg.q) == (dko.p, dko.q)
        assert codec.enc(kg.vss_scheme) == codec.enc(ko.vss_scheme)
        msgs.append(mg)
        dks.append(dkg)
        kgs.append(kg)
    if len(msgs) == n:   # the GPU-made messages verify on the GPU and refresh party 1's key
        k = kgs[0]
        refresh.collect(copy.deepcopy(msgs), k, dks[0], [], ctx=gpu_ctx, key_bits=kb)
        assert k.x_i != keys[0].x_i


def test_distribute_chosen_randomness_and_errors(gpu_ctx):
    from fsdkr import distribute, refresh
    keys = protocol.simulate_keygen(1, 3, Rng("dist-err"), 1024)
    rnd = Rng("dist-r")
    rs = [rnd.sample_below(e.n) for e in keys[0].paillier_key_vec]
    ko, kg = keys[0].clone(), keys[0].clone()
    mo, _ = protocol.distribute(1, ko, 3, Rng("dist-c"), 1024, randomness=rs)
    mg, _ = distribute.distribute(1, kg, 3, Rng("dist-c"), ctx=gpu_ctx, key_bits=1024, randomness=rs)
    assert mg.points_encrypted_vec == mo.points_encrypted_vec
    with pytest.raises(refresh.FsDkrPanic):           # assert!(t <= new_n / 2), refresh_message.rs:56
        distribute.distribute(1, keys[0].clone(), 1, Rng("x"), ctx=gpu_ctx, key_bits=1024)


def test_join_distribute_and_replace_match_oracle(gpu_ctx):
    """JoinMessage::distribute (add_party_message.rs:101-124) and
    RefreshMessage::replace (refresh_message.rs:239-319) against the oracle,
    then the GPU-made messages through RefreshMessage::collect (an old party)
    and JoinMessage::collect (the joiner) on the GPU."""
    from fsdkr import distribute, join, refresh
    kb, t, n = 1024, 1, 4
    all_keys = protocol.simulate_keygen(t, n, Rng("jd-keys"), kb)
    jo, jko = protocol.join_distribute(Rng("jd"), kb)
    jg, jkg = distribute.join_distribute(Rng("jd"), ctx=gpu_ctx, key_bits=kb)
    assert codec.enc(jg) == codec.enc(jo)
    assert (jkg.dk.p, jkg.dk.q) == (jko.dk.p, jko.dk.q)
    jg.party_index = 4
    old_to_new = {1: 1, 2: 2, 3: 3}
    msgs, dks, keys = [], [], []
    for key in all_keys[:3]:
        ko, kg = key.clone(), key.clone()
        jo2 = copy.deepcopy(jo)
        jo2.set_party_index(4)
        mo, dko = protocol.replace([jo2], ko, old_to_new, n, Rng(f"rep-{key.i}"), kb)
        mg, dkg = distribute.replace([jg], kg, old_to_new, n, Rng(f"rep-{key.i}"), ctx=gpu_ctx, key_bits=kb)
        assert codec.enc(mg) == codec.enc(mo)
        assert [e.n for e in kg.paillier_key_vec] == [e.n for e in ko.paillier_key_vec]
        msgs.append(mg)
        dks.append(dkg)
        keys.append(kg)
    k1 = keys[1]
    refresh.collect(copy.deepcopy(msgs), k1, dks[1], [copy.deepcopy(jg)], ctx=gpu_ctx, key_bits=kb)
    lk = join.collect(jg, copy.deepcopy(msgs), jkg, [], t, n, ctx=gpu_ctx)
    assert lk.i == 4 and lk.y_sum_s == msgs[0].public_key
    # both ends of the refresh agree on the joiner's public share
    assert k1.pk_vec[3] == lk.pk_vec[3]
    # a party with no message (party 3 here): JoinMessage::collect generates its
    # DLogStatement (add_party_message.rs:257-266) -- on the GPU, equal to the
    # oracle's generate_h1_h2_n_tilde under the same draws
    lk2 = join.collect(jg, copy.deepcopy(msgs[:2]), jkg, [], t, n, ctx=gpu_ctx, key_bits=kb, rng=Rng("miss"))
    n_tilde, h1, h2, _, _ = protocol.generate_h1_h2_n_tilde(kb, Rng("miss"))
    st = lk2.h1_h2_n_tilde_vec[2]
    assert (st.N, st.g, st.ni) == (n_tilde, h1, h2)
    assert [s.N for s in lk2.h1_h2_n_tilde_vec[:2]] == [s.N for s in lk.h1_h2_n_tilde_vec[:2]]
    assert lk2.x_i == lk.x_i and lk2.pk_vec == lk.pk_vec   # the first t+1 messages fix the share
    assert lk2.paillier_key_vec[2].n == 0                  # EncryptionKey(0, 0) for the missing party
