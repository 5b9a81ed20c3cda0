"""The reference's own end-to-end scenarios (/root/reference/src/test.rs) through
the GPU path at the reference's PAILLIER_KEY_SIZE = 2048 (lib.rs:26), with every
party's LocalKey compared against the oracle's after every collect().

  test_sign_rotate_sign          test.rs:69-80   t=2 n=5, two consecutive refreshes
  test_remove_sign_rotate_sign   test.rs:82-93   t=2 n=5, parties {1} then {1,2} removed
  test_add_party_with_permute    test.rs:95-224  t=2 n=7, parties 2 and 7 replaced by
                                                 joiners, permuted old_to_new map

The messages are made by the GPU prover (fsdkr.distribute / replace /
join_distribute), which reproduces the oracle's messages bit for bit for the
same draws (tests/test_distribute_gpu.py; re-checked here for one party per
scenario).  Each collect() runs on the GPU (fsdkr.refresh.collect /
fsdkr.join.collect, the C ABI) and in the oracle on a copy of the same
LocalKey; the outcome and the whole updated LocalKey must be equal.

GG20 signing (multi-party-ecdsa OfflineStage / SignManual) is out of scope; in
its place every signing set of the reference test must reconstruct the
original secret from the refreshed shares, every party's y must equal G*x_i and
y_sum_s must stay the public key that secret gives."""
import copy
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

import codec  # noqa: E402
from oracle import protocol  # noqa: E402
from oracle import secp256k1 as ec  # noqa: E402
from oracle.rng import Rng  # noqa: E402

pytestmark = pytest.mark.gpu

KB = 2048   # PAILLIER_KEY_SIZE (lib.rs:26)


def _oracle_view(x):
    """GPU-made messages decoded into the oracle's types (the oracle verifies them itself)."""
    return codec.dec(codec.enc(x), codec.oracle_classes())


def _same_key(o, g):
    assert g.x_i == o.x_i
    assert g.y == o.y
    assert g.pk_vec == o.pk_vec
    assert [k.n for k in g.paillier_key_vec] == [k.n for k in o.paillier_key_vec]
    assert (g.paillier_dk.p, g.paillier_dk.q) == (o.paillier_dk.p, o.paillier_dk.q)
    assert [(s.N, s.g, s.ni) for s in g.h1_h2_n_tilde_vec] == [(s.N, s.g, s.ni) for s in o.h1_h2_n_tilde_vec]
    assert (g.i, g.t, g.n, g.y_sum_s) == (o.i, o.t, o.n, o.y_sum_s)


def _outcome(fn):
    from fsdkr import refresh
    try:
        fn()
    except (protocol.FsDkrError, refresh.FsDkrError) as e:
        return e.variant, e.fields
    except (refresh.FsDkrPanic, Exception) as e:   # the reference panics
        return "panic", None
    return None


def _collect_both(gpu_ctx, msgs, key, dk, joins=(), recovery="speculative"):
    """collect() of one party: the oracle on a clone of `key`, the GPU on `key`
    itself.  Returns (oracle outcome, GPU outcome, oracle's key)."""
    from fsdkr import refresh
    ko = key.clone()
    ro = _outcome(lambda: protocol.collect(_oracle_view(msgs), ko, dk, _oracle_view(list(joins)), Rng("a8"), KB))
    rg = _outcome(lambda: refresh.collect(copy.deepcopy(msgs), key, dk, copy.deepcopy(list(joins)), ctx=gpu_ctx,
                                          key_bits=KB, recovery=recovery))
    return ro, rg, ko


def _distribute_all(gpu_ctx, keys, new_n, tag):
    """test.rs:317-325 on the GPU prover; party 1's message re-checked against the oracle's."""
    from fsdkr import distribute
    msgs, dks = [], []
    for key in keys:
        seed = f"{tag}-{key.i}"
        if key is keys[0]:
            mo, dko = protocol.distribute(key.i, key.clone(), new_n, Rng(seed), KB)
        m, dk = distribute.distribute(key.i, key, new_n, Rng(seed), ctx=gpu_ctx, key_bits=KB)
        if key is keys[0]:
            assert codec.enc(m) == codec.enc(mo) and (dk.p, dk.q) == (dko.p, dko.q)
        msgs.append(m)
        dks.append(dk)
    return msgs, dks


def _signing_set_ok(keys, signers, secret, y0):
    """Stand-in for simulate_offline_stage + simulate_signing (test.rs:336-382):
    the signing set reconstructs the original secret and its public key."""
    idx = [s - 1 for s in signers]
    assert protocol.reconstruct(idx, [keys[i].x_i for i in idx]) == secret
    assert ec.mul(ec.G, secret) == y0
    for k in keys:
        assert k.y == ec.mul(ec.G, k.x_i)
        assert k.y_sum_s == y0


def test_sign_rotate_sign(gpu_ctx):
    """test.rs:69-80: sign with {1,2,3}, refresh, sign with {2,3,4}, refresh, sign with {1,3,5}.
    After each refresh every party's LocalKey equals the oracle's, including pk_vec, which
    grows by n entries per refresh (the insert at refresh_message.rs:455-464 keeps the new
    entries first).  Party 1 recovers its share after the verdicts (recovery="after",
    the reference's order, :439), the others speculatively: same keys either way."""
    t, n = 2, 5
    keys = protocol.simulate_keygen(t, n, Rng("ref-rotate"), KB)
    y0 = keys[0].y_sum_s
    secret = protocol.reconstruct([0, 1, 2], [k.x_i for k in keys[:3]])
    _signing_set_ok(keys, [1, 2, 3], secret, y0)
    old_shares = [k.x_i for k in keys]
    for rot, signers in enumerate(([2, 3, 4], [1, 3, 5])):
        msgs, dks = _distribute_all(gpu_ctx, keys, n, f"ref-rotate-{rot}")
        for i in range(n):
            ro, rg, ko = _collect_both(gpu_ctx, msgs, keys[i], dks[i], recovery="after" if i == 0 else "speculative")
            assert ro is None and rg is None, (ro, rg)
            _same_key(ko, keys[i])
            assert len(keys[i].pk_vec) == n * (rot + 2)
            assert keys[i].pk_vec[keys[i].i - 1] == keys[i].y
        assert all(k.pk_vec[:n] == keys[0].pk_vec[:n] for k in keys)
        _signing_set_ok(keys, signers, secret, y0)
    assert [k.x_i for k in keys] != old_shares


def test_remove_sign_rotate_sign(gpu_ctx):
    """test.rs:82-93 / :238-309 (simulate_dkr_removal), quirks included: each message
    carries remove_party_indices; a removed party receives only its own message and
    its collect (into keys[index], the NEXT party's key, with its own new dk) fails
    with PartiesThresholdViolation leaving that key untouched; the other parties
    collect into copies (party_key), so `keys` keeps its shares between the two
    removals and only the refreshed copies change."""
    t, n = 2, 5
    keys = protocol.simulate_keygen(t, n, Rng("ref-remove"), KB)
    y0 = keys[0].y_sum_s
    secret = protocol.reconstruct([0, 1, 2], [k.x_i for k in keys[:3]])
    _signing_set_ok(keys, [1, 2, 3], secret, y0)
    for rnd, (removed, signers) in enumerate((([1], [2, 3, 4]), ([1, 2], [3, 4, 5]))):
        msgs, dks = _distribute_all(gpu_ctx, keys, n, f"ref-remove-{rnd}")
        party_key = {m.party_index: keys[k].clone() for k, m in enumerate(msgs)}
        new_dks = {m.party_index: dks[k] for k, m in enumerate(msgs)}
        for m in msgs:
            m.remove_party_indices = [r for r in removed if r != m.party_index]
        buckets = {m.party_index: [] for m in msgs}
        for m in msgs:
            for p in buckets:
                if p not in m.remove_party_indices:
                    buckets[p].append(m)
        for r in removed:
            assert len(buckets[r]) == 1
        refreshed = []
        for p in sorted(party_key):
            if p in removed:
                continue
            ro, rg, ko = _collect_both(gpu_ctx, buckets[p], party_key[p], new_dks[p])
            assert ro is None and rg is None, (ro, rg)
            _same_key(ko, party_key[p])
            refreshed.append(party_key[p])
        for r in removed:
            before = keys[r].clone()
            ro, rg, ko = _collect_both(gpu_ctx, buckets[r], keys[r], new_dks[r])
            assert ro == rg == ("PartiesThresholdViolation", {"threshold": 2, "refreshed_keys": 1})
            _same_key(ko, keys[r])
            assert keys[r].x_i == before.x_i and keys[r].pk_vec == before.pk_vec
        by_index = {k.i: k for k in refreshed}
        idx = [s - 1 for s in signers]
        assert protocol.reconstruct(idx, [by_index[s].x_i for s in signers]) == secret
        for k in refreshed:
            assert k.y == ec.mul(ec.G, k.x_i) and k.y_sum_s == y0
        _signing_set_ok(keys, signers, secret, y0)   # `keys` itself was not refreshed


def test_add_party_with_permute(gpu_ctx):
    """test.rs:95-224: t=2, n=7; parties 2 and 7 leave, two joiners take indices 2 and 7,
    the remaining parties are renumbered by old_to_new {1:4, 3:1, 4:3, 5:6, 6:5}
    (RefreshMessage::replace), every old party collects with the join messages
    (RefreshMessage::collect) and each joiner runs JoinMessage::collect; all LocalKeys
    equal the oracle's, and the sorted new keys reconstruct the old secret from
    {1,2,3} and from the signing set {1,2,7}."""
    from fsdkr import distribute, join
    t, n = 2, 7
    all_keys = protocol.simulate_keygen(t, n, Rng("ref-permute"), KB)
    keys = [k.clone() for k in all_keys]
    del keys[6]
    del keys[1]
    old_to_new = {1: 4, 3: 1, 4: 3, 5: 6, 6: 5}
    joins, join_keys = [], []
    for pi in (2, 7):
        jm, kk = distribute.join_distribute(Rng(f"ref-join-{pi}"), ctx=gpu_ctx, key_bits=KB)
        if pi == 2:
            jo, kko = protocol.join_distribute(Rng(f"ref-join-{pi}"), KB)
            assert codec.enc(jm) == codec.enc(jo) and (kk.dk.p, kk.dk.q) == (kko.dk.p, kko.dk.q)
        jm.party_index = pi
        joins.append(jm)
        join_keys.append(kk)
    new_n = len(keys) + len(joins)
    msgs, dks = [], []
    for k, key in enumerate(keys):
        seed = f"ref-replace-{key.i}"
        if k == 0:
            ko = key.clone()
            mo, dko = protocol.replace(_oracle_view(joins), ko, old_to_new, new_n, Rng(seed), KB)
        m, dk = distribute.replace(joins, key, old_to_new, new_n, Rng(seed), ctx=gpu_ctx, key_bits=KB)
        if k == 0:
            assert codec.enc(m) == codec.enc(mo)
            assert [e.n for e in key.paillier_key_vec] == [e.n for e in ko.paillier_key_vec]
        msgs.append(m)
        dks.append(dk)
    out = []
    for k, key in enumerate(keys):
        ro, rg, ko = _collect_both(gpu_ctx, msgs, key, dks[k], joins)
        assert ro is None and rg is None, (ro, rg)
        _same_key(ko, key)
        out.append((key.i - 1, key))
    for jm, kk in zip(joins, join_keys):
        lo = protocol.join_collect(_oracle_view(jm), _oracle_view(msgs), _oracle_view(kk), _oracle_view(joins), t, n,
                                   Rng("jc"), KB)
        lg = join.collect(jm, copy.deepcopy(msgs), kk, copy.deepcopy(joins), t, n, ctx=gpu_ctx, key_bits=KB)
        _same_key(lo, lg)
        # the new VSS polynomial is random in both (curv VerifiableSS::share); its
        # constant term commits to the recovered share
        assert lg.vss_scheme.commitments[0] == ec.mul(ec.G, lg.x_i)
        out.append((jm.party_index - 1, lg))
    out.sort(key=lambda p: p[0])
    new_keys = [p[1] for p in out]
    assert [k.i for k in new_keys] == list(range(1, n + 1))
    secret_old = protocol.reconstruct([0, 1, 2], [k.x_i for k in all_keys[:3]])
    assert protocol.reconstruct([0, 1, 2], [k.x_i for k in new_keys[:3]]) == secret_old
    assert [k.x_i for k in new_keys] != [k.x_i for k in all_keys]
    _signing_set_ok(new_keys, [1, 2, 7], secret_old, all_keys[0].y_sum_s)
    # every party, old or new, holds the same public shares of the new sharing
    assert all(k.pk_vec[:n] == new_keys[0].pk_vec[:n] for k in new_keys)
