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


def _fake_collect(n=6, t=2, M=8, J=2, seed=3, big_ped=False):
    rnd = random.Random(seed)

    def r(b):
        return rnd.getrandbits(b) | 1

    def pt():
        return (rnd.getrandbits(255), rnd.getrandbits(255))

    def stmt():
        return NS(N=r(2048), g=r(2040), ni=r(2040))
    lk = NS(t=t, paillier_key_vec=[NS(n=r(2048)) for _ in range(n)], h1_h2_n_tilde_vec=[stmt() for _ in range(n)])

    def msg(i):
        return NS(party_index=i + 1,
                  pdl_proof_vec=[NS(z=r(3000 if big_ped and i == 1 and q == 2 else 2040), u1=pt(), u2=r(4090),
                                    u3=r(2040), s1=r(1024), s2=r(2040), s3=r(2300)) for q in range(n)],
                  points_committed_vec=[pt() for _ in range(n)], points_encrypted_vec=[r(4090) for _ in range(n)],
                  range_proofs=[NS(z=r(2040), e=r(256), s=r(2040), s1=r(1024), s2=r(2300)) for _ in range(n)],
                  coefficients_committed_vec=NS(commitments=[pt() for _ in range(t + 1)]),
                  ring_pedersen_statement=NS(N=r(2048), S=r(2040), T=r(2040)),
                  ring_pedersen_proof=NS(A=[r(2040) for _ in range(M)], Z=[r(2300) for _ in range(M)]),
                  ek=NS(n=r(2048)), dk_correctness_proof=NS(sigma_vec=[r(2040) for _ in range(11)]))
    msgs = [msg(i) for i in range(n - J)]
    joins = []
    for i in range(J):
        m = msg(n - J + i)
        m.dlog_statement = stmt()
        m.composite_dlog_proof_base_h1 = NS(x=r(2040), y=r(2300))
        m.composite_dlog_proof_base_h2 = NS(x=r(2040), y=r(2300))
        joins.append(m)
    return msgs, joins, lk


def _dump(b, M):
    """Every array of the C batch struct, by the shapes the C ABI documents."""
    c = b.c
    R, J, n = b.R, b.J, b.n
    P, Mt = R * n, R + J
    V = sum(len(m.coefficients_committed_vec.commitments) for m in b._msgs)
    rows = {"recv_n": (n, c.nl), "recv_ntilde": (n, c.nl), "recv_h1": (n, c.nl), "recv_h2": (n, c.nl),
            "enc": (P, 2 * c.nl), "commit": (P, 16), "pdl_z": (P, c.nl), "pdl_u1": (P, 16), "pdl_u2": (P, 2 * c.nl),
            "pdl_u3": (P, c.nl), "pdl_s1": (P, c.s1l), "pdl_s2": (P, c.nl), "pdl_s3": (P, c.s3l), "rp_z": (P, c.nl),
            "rp_e": (P, c.el), "rp_s": (P, c.nl), "rp_s1": (P, c.s1l), "rp_s2": (P, c.s3l), "vss": (V, 16),
            "ped_S": (Mt, c.nl), "ped_T": (Mt, c.nl), "ped_N": (Mt, c.nl), "ped_A": (Mt * M, c.nl),
            "ped_Z": (Mt * M, c.zl), "ck_n": (Mt, c.ckl), "ck_sigma": (Mt * 11, c.ckl), "dlog_N": (J, c.nl),
            "dlog_g": (J, c.nl), "dlog_ni": (J, c.nl), "dlog_x1": (J, c.nl), "dlog_x2": (J, c.nl),
            "dlog_y1": (J, c.yl), "dlog_y2": (J, c.yl)}
    out = {"widths": (c.nl, c.ckl, c.s1l, c.s3l, c.el, c.zl, c.yl)}
    for name, (r_, w) in rows.items():
        out[name] = np.ctypeslib.as_array(getattr(c, name), shape=(r_ * w,)).copy() if r_ * w else None
    return out


@pytest.mark.parametrize("big_ped", [False, True])
@pytest.mark.parametrize("split", [False, True])
def test_staged_batch_equals_one_shot(big_ped, split):
    """CollectBatch(staged=True) + complete() packs exactly what the one-shot
    constructor packs, also when stage 1's width is superseded (a 3000-bit PDL z,
    a stage-2 field, moves the batch to 3072-bit slots) and when stage 1 is split
    (GA's fields, then stage1b())."""
    from fsdkr.batch import CollectBatch
    M = 8
    msgs, joins, lk = _fake_collect(M=M, big_ped=big_ped)
    one = CollectBatch(msgs, lk, joins, M, 2048)
    st = CollectBatch(msgs, lk, joins, M, 2048, staged=True, split_stage1=split)
    assert st.ga_ready and st.c.nl == 64
    assert st.stage1b() == split and not st.stage1b()
    st.complete()
    one._msgs = st._msgs = msgs
    a, b = _dump(one, M), _dump(st, M)
    assert a["widths"] == b["widths"] and a["widths"][0] == (96 if big_ped else 64)
    for k in a:
        assert (a[k] is None and b[k] is None) or np.array_equal(a[k], b[k]), k


def test_session_set_equals_per_session_batches():
    """SessionSet (configs[4]: one gather across all sessions, per-session struct
    rows filled vectorised) points every regular session at exactly the arrays
    its own CollectBatch packs; irregular sessions keep their own batch, and a
    header-only session is not prepared."""
    from types import SimpleNamespace as NSp
    from fsdkr._native import CollectBatchC
    from fsdkr.batch import CollectBatch, SessionSet, _BATCH_DT
    M = 8
    sessions = []
    for s in range(5):
        msgs, joins, lk = _fake_collect(n=3, t=1, M=M, J=1 if s == 2 else 0, seed=10 + s)
        sessions.append((msgs, lk, joins))
    # irregular: a short range_proofs vector; header only: threshold (R <= t)
    m0 = sessions[3][0][0]
    m0.range_proofs = m0.range_proofs[:2]
    hm, hj, hl = _fake_collect(n=3, t=1, M=M, J=0, seed=99)
    sessions.append((hm[:1], hl, []))
    ss = SessionSet(sessions, M, 2048)
    assert ss.live == [0, 1, 2, 3, 4] and ss.batches[5].header_only and ss.batches[3] is not None
    for s in ss.live:
        one = CollectBatch(sessions[s][0], sessions[s][1], sessions[s][2], M, 2048)
        row = NSp(c=CollectBatchC.from_address(ss.structs.ctypes.data + ss.row[s] * _BATCH_DT.itemsize),
                  R=one.R, J=one.J, n=one.n, _msgs=sessions[s][0])
        one._msgs = sessions[s][0]
        a, b = _dump(one, M), _dump(row, M)
        if one.J == 0:   # yl (DLog y limbs) is the set's width, unused without joins
            a["widths"], b["widths"] = a["widths"][:-1], b["widths"][:-1]
        for k in a:
            assert (a[k] is None and b[k] is None) or np.array_equal(a[k], b[k]), (s, k)
        for f in ("n_refresh", "n_join", "t", "m_security", "key_bits", "n_recv", "recv_avail"):
            assert getattr(one.c, f) == getattr(row.c, f), (s, f)
        pi = np.ctypeslib.as_array(row.c.party_index, shape=(one.R + one.J,))
        assert list(pi) == [m.party_index for m in sessions[s][0]] + [j.party_index or 0 for j in sessions[s][2]]


def test_gather_rows_flattens_prefixes():
    """_pack.gather_rows(objs, attr, take) == gather of [v for o in objs for v in getattr(o, attr)[:take]]."""
    rnd = random.Random(5)
    objs = [NS(A=tuple(rnd.getrandbits(rnd.randint(1, 3072)) for _ in range(9))) for _ in range(40)]
    G = _Gather()
    f_rows = G.rows(objs, "A", 7)
    flat = [v for o in objs for v in o.A[:7]]
    assert f_rows[1] == max(v.bit_length() for v in flat) and f_rows[2] == len(flat)
    a = G.slot(f_rows, 96)
    G.run()
    assert np.array_equal(a, _expect(flat, 96))
    with pytest.raises(IndexError):
        _pack.gather_rows(objs, "A", 10)          # a row shorter than `take`
    with pytest.raises(UnsupportedInput):
        _Gather().rows([NS(A=(1, -2))], "A", 2)   # negative value
    with pytest.raises(TypeError):
        _pack.gather_rows([NS(A=(1, 2.0))], "A", 2)


def test_session_set_pool_reuse():
    """A collected SessionSet's large slot arrays are reused by the next set of
    the same shape, and the packed contents do not depend on the recycling."""
    import gc
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from pack_many_cpu import fake_sessions
    from fsdkr.batch import SessionSet, _POOL
    sess = fake_sessions(24, seed=3)
    first = SessionSet(sess, 256, 3072)
    snap = {k: np.array(v, copy=True) for k, v in enumerate(first._owned)}
    ids = {id(a) for a in first._owned if a.nbytes >= _POOL.MIN_BYTES}
    assert ids, "the fake sessions must produce pooled slots"
    del first
    gc.collect()
    second = SessionSet(sess, 256, 3072)
    assert ids & {id(a) for a in second._owned}
    for k, a in enumerate(second._owned):
        assert np.array_equal(a, snap[k])


def test_session_set_stage1_correct_key_rows():
    """Stage 1 of a staged SessionSet carries every message's ek.n and sigma_vec
    rows (fsdkr_collect_prestart_multi's correct-key job) at the width stage 2
    uses, row k of session s at the session's message offset."""
    import ctypes
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from pack_many_cpu import fake_sessions
    from fsdkr.batch import M2, SessionSet
    sess = fake_sessions(5, seed=4)
    ss = SessionSet(sess, 256, 3072, staged=True)
    assert int(ss._pre["ckl"][0]) == 0 and ss.stage1b() and not ss.stage1b()   # split: GA's fields first
    pre = ss._pre
    ckl = int(pre["ckl"][0])
    assert ckl == 96
    for s, (msgs, lk, joins) in enumerate(sess):
        for k, m in enumerate(msgs):
            row = np.ctypeslib.as_array(ctypes.cast(int(pre["ck_n"][s]) + k * ckl * 4, ctypes.POINTER(ctypes.c_uint32)),
                                        (ckl,))
            assert np.array_equal(row, _expect([m.ek.n], ckl)[0])
            for j in range(M2):
                at = int(pre["ck_sigma"][s]) + (k * M2 + j) * ckl * 4
                row = np.ctypeslib.as_array(ctypes.cast(at, ctypes.POINTER(ctypes.c_uint32)), (ckl,))
                assert np.array_equal(row, _expect([m.dk_correctness_proof.sigma_vec[j]], ckl)[0])
    ss.complete()
    assert int(ss.structs["ckl"][0]) == ckl


def test_session_set_stage_z_rows_reused_by_stage2():
    """Stage 1b (SessionSet.stage_z, fsdkr_collect_prestart_rp's input) packs every
    message's ring-Pedersen Z rows at the width stage 2 gives them; stage 2 then
    points ped_Z at the same rows, byte-identical to a one-shot set."""
    import ctypes
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from pack_many_cpu import fake_sessions
    from fsdkr.batch import SessionSet
    sess = fake_sessions(6, seed=7)
    M = 256
    one = SessionSet(sess, M, 3072)
    ss = SessionSet(sess, M, 3072, staged=True)
    assert ss.stage_z()
    zl = int(ss._pre["zl"][0])
    ss.complete()
    assert int(ss.structs["zl"][0]) == zl == int(one.structs["zl"][0])
    for s, (msgs, lk, joins) in enumerate(sess):
        assert int(ss._pre["ped_Z"][s]) == int(ss.structs["ped_Z"][ss.row[s]])
        rows = len(msgs + joins) * M
        a = np.ctypeslib.as_array(ctypes.cast(int(ss.structs["ped_Z"][ss.row[s]]), ctypes.POINTER(ctypes.c_uint32)),
                                  (rows * zl,))
        b = np.ctypeslib.as_array(ctypes.cast(int(one.structs["ped_Z"][one.row[s]]), ctypes.POINTER(ctypes.c_uint32)),
                                  (rows * zl,))
        assert np.array_equal(a, b)
        want = _expect([z for m in msgs + joins for z in m.ring_pedersen_proof.Z[:M]], zl).reshape(-1)
        assert np.array_equal(a, want)
