"""The host gather of the batching layer (csrc/pack.c via fsdkr.batch): every
big integer lands in its u32-limb slot exactly as int.to_bytes(little) would put
it, on one worker or many, and out-of-range values raise UnsupportedInput."""
import random
from types import SimpleNamespace as NS

import numpy as np
import pytest

from fsdkr import _pack
from fsdkr.batch import UnsupportedInput, _Gather, pack, pack_attr, pack_points


def _expect(vals, limbs):
    raw = b"".join(v.to_bytes(4 * limbs, "little") for v in vals)
    return np.frombuffer(raw, dtype=np.uint32).reshape(len(vals), limbs)


def _vals(rnd, count, bits):
    # random widths up to `bits`, plus the edges: 0, 1, all ones, digit-boundary widths
    out = [0, 1, (1 << bits) - 1, 1 << (bits - 1), (1 << 30) - 1, 1 << 30, (1 << 60) + 7]
    out += [rnd.getrandbits(rnd.randint(1, bits)) for _ in range(count)]
    return [v for v in out if v.bit_length() <= bits]


@pytest.mark.parametrize("limbs", [1, 2, 8, 15, 16, 64, 72, 129])
def test_pack_matches_to_bytes(limbs):
    rnd = random.Random(limbs)
    vals = _vals(rnd, 300, 32 * limbs)
    assert np.array_equal(pack(vals, limbs), _expect(vals, limbs))


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_gather_convert_many_jobs(threads):
    rnd = random.Random(threads)
    G = _Gather()
    want, got = [], []
    for limbs in (64, 128, 8, 9, 33):
        objs = [NS(z=v) for v in _vals(rnd, 1500, 32 * limbs)]
        f = G.field(objs, "z")
        assert f[1] == max(o.z.bit_length() for o in objs)
        got.append(G.slot(f, limbs))
        want.append(_expect([o.z for o in objs], limbs))
    G.run()
    for g, w in zip(got, want):
        assert np.array_equal(g, w)
    # the same through the C entry point with an explicit worker count
    h, _ = _pack.gather([o for o in range(5000)], None)
    arr = np.empty((5000, 1), np.uint32)
    _pack.convert([(h, arr, 1)], threads)
    assert np.array_equal(arr[:, 0], np.arange(5000, dtype=np.uint32))


def test_overflow_and_negative():
    with pytest.raises(UnsupportedInput):
        pack([1 << 64], 2)
    with pytest.raises(UnsupportedInput):
        pack([5, -3], 2)
    with pytest.raises(UnsupportedInput):
        pack_attr([NS(z=(1 << 100) - 1), NS(z=1 << 100)], "z", 3)
    assert np.array_equal(pack([(1 << 96) - 1], 3), _expect([(1 << 96) - 1], 3))
    G = _Gather()
    G.slot(G.field([1, 2, 3]), 1)
    G.slot(G.field([1 << 40]), 1)   # the second job overflows its slot
    with pytest.raises(UnsupportedInput, match="job 1"):
        G.run()
    with pytest.raises(TypeError):
        _pack.gather([1, "x"], None)


def test_points():
    rnd = random.Random(7)
    pts = [(rnd.getrandbits(256), rnd.getrandbits(256)) for _ in range(50)] + [None, [3, 4], (0, 0)]
    arr = pack_points(pts)
    want = _expect([0 if p is None else p[0] | (p[1] << 256) for p in pts], 16)
    assert np.array_equal(arr, want)
    objs = [NS(u1=p) for p in pts]
    assert np.array_equal(pack_points(objs, "u1"), want)
    with pytest.raises(UnsupportedInput):
        pack_points([(1 << 256, 1)])
    with pytest.raises(UnsupportedInput):
        pack_points([(1, -1)])
