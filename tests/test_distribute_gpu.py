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
