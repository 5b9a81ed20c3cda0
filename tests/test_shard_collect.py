"""End-to-end sharded RefreshMessage::collect (fsdkr.shard.collect, SURVEY §8e;
VERDICT r1 "do this" 5) on CPU: world_size 2 gloo processes each verify their
slice of the messages (an oracle-backed stand-in answers the device calls,
tests/oracle_device.py), all-reduce the verdict bytes, map them to the first
error on a header-only batch of the whole set and apply collect()'s side
effects + share recovery.  Every rank's outcome and LocalKey must equal the
single-process oracle collect(): valid messages, a tamper in rank 1's slice,
a correct-key tamper (partial paillier_key_vec writes) and a join transcript.
The GPU variant (two contexts, one per emulated rank) is in
test_shard_batch.py."""
import copy
import os
import socket
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _scenario(name, tamper):
    sys.path[:0] = [REPO, os.path.join(REPO, "fs-dkr_amd"), os.path.join(HERE, "golden"), HERE]
    import codec
    raw = codec.load_raw(name)
    cls = codec.oracle_classes()
    d = {k: codec.dec(raw[k], cls) for k in ("keys", "dks", "msgs", "joins")}
    msgs, joins = d["msgs"], d["joins"]
    if tamper == "pdl":          # message 3 lands in rank 1's slice of 5
        p = msgs[3].pdl_proof_vec[1]
        msgs[3].pdl_proof_vec[1] = type(p)(**{**p.__dict__, "s3": p.s3 + 1})
    elif tamper == "ck":
        sv = msgs[4].dk_correctness_proof.sigma_vec
        msgs[4].dk_correctness_proof = type(msgs[4].dk_correctness_proof)((sv[0] + 1,) + tuple(sv[1:]))
    party = 1 if joins else 0
    return msgs, joins, d["keys"][party], d["dks"][party], raw["meta"]["key_bits"]


def _outcome(fn):
    try:
        fn()
        return None
    except Exception as e:   # FsDkrError of either side carries variant + fields
        return (getattr(e, "variant", "panic"), getattr(e, "fields", {}))


def _summary(k):
    return (k.x_i, k.y, list(k.pk_vec), [e.n for e in k.paillier_key_vec])


class _WideDk:
    """a decryption key wider than the recovery's 6144-bit limit"""
    p = (1 << 3100) + 15
    q = (1 << 3100) + 27


class _NoDk:
    """a decryption key without its primes (AttributeError in the recovery plan)"""


def _worker(rank, world, port, name, tamper, q):
    sys.path[:0] = [REPO, os.path.join(REPO, "fs-dkr_amd"), HERE]
    import torch.distributed as dist
    from fsdkr import shard
    from oracle_device import OracleDevice
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    msgs, joins, key, dk, kb = _scenario(name, tamper)
    if tamper in ("dk_wide", "dk_noattr"):   # the local key's decryption key, not the new one
        key.paillier_dk = _WideDk() if tamper == "dk_wide" else _NoDk()
    k = key.clone()
    dev = OracleDevice(msgs, joins, k, world, rank)
    out = _outcome(lambda: shard.collect(dist, msgs, k, dk, joins, dev, key_bits=kb))
    dist.destroy_process_group()
    q.put((rank, out, _summary(k)))


@pytest.mark.parametrize("name,tamper", [("transcript_t2_n5_kb1024.json.gz", None),
                                         ("transcript_t2_n5_kb1024.json.gz", "pdl"),
                                         ("transcript_t2_n5_kb1024.json.gz", "ck"),
                                         ("transcript_join_t1_n4_kb1024.json.gz", None)])
def test_sharded_collect_equals_single_process(name, tamper):
    from oracle import protocol
    from oracle.rng import Rng
    msgs, joins, key, dk, kb = _scenario(name, tamper)
    ko = key.clone()
    want = _outcome(lambda: protocol.collect(copy.deepcopy(msgs), ko, dk, copy.deepcopy(joins), Rng("a8"), kb))
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 2
    ps = [ctx.Process(target=_worker, args=(r, world, port, name, tamper, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    for rank, out, summ in res:
        assert out == want, (rank, out, want)
        assert summ == _summary(ko), rank
    if tamper is None:
        assert want is None


@pytest.mark.parametrize("tamper", ["dk_wide", "dk_noattr"])
def test_sharded_recovery_panic_agrees_on_every_rank(tamper):
    """A decryption key the share recovery refuses (wider than 6144 bits, or
    without its primes) is checked on every rank, not only on the decrypting one:
    every rank raises the same panic and leaves the same LocalKey (the
    non-decrypting ranks used to apply share 0 while rank 0 panicked)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 2
    name = "transcript_t2_n5_kb1024.json.gz"
    ps = [ctx.Process(target=_worker, args=(r, world, port, name, tamper, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    outs = {out[0] if out else None for _, out, _ in res}
    assert outs == {"panic"}, res
    assert res[0][2] == res[1][2]
