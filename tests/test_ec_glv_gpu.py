"""secp256k1 scalar multiplications on the GPU over the GLV split (vec.hip:
pdl_u1_kernel, four lanes per pair; ec_msm_term_kernel, Shamir over the two
128-bit halves) against the oracle's curve arithmetic: the PDL u1 equation
G*s1 + Q*(q-e) == u1 (zk_pdl_with_slack.rs:124-127, through fsdkr_pdl_u1_check)
and sum_j s_j P_j (fsdkr_ec_msm; pk_vec, refresh_message.rs:451-464), at edge
scalars (0, 1, q - 1, q, multiples of q, lambda, values past 2^256, the split's
boundary values) and random ones, with points at infinity."""
import random

import pytest

from oracle import secp256k1 as ec

from test_ec_glv import EDGE, LAM

pytestmark = pytest.mark.gpu
N = ec.Q


def _u1(s1, e, Q):
    a = ec.mul(ec.G, s1 % N)
    b = ec.mul(Q, (N - e % N) % N) if Q is not None else None
    return ec.add(a, b)


def test_pdl_u1_check_edges_vs_oracle(gpu_ctx):
    rnd = random.Random(11)
    pts = [ec.G, ec.neg(ec.G), None] + [ec.mul(ec.G, rnd.randrange(1, N)) for _ in range(5)]
    s1s, es, Qs, u1s, want = [], [], [], [], []
    scal = EDGE + [N, 2 * N + 5, 2 ** 300 + 17, 3 * N - 1]
    for k in range(len(scal) * 3):
        s1 = scal[k % len(scal)] if k < len(scal) else rnd.randrange(2 ** 260)
        e = scal[(k * 7) % len(scal)] % 2 ** 256 if k % 3 else rnd.randrange(2 ** 256)
        Q = pts[k % len(pts)]
        u = _u1(s1, e, Q)
        bad = k % 5 == 4
        if bad:   # off by G: must be rejected
            u = ec.add(u, ec.G)
        s1s.append(s1)
        es.append(e)
        Qs.append(Q)
        u1s.append(u)
        want.append(0 if bad else 1)
    got = gpu_ctx.pdl_u1_check(s1s, es, Qs, u1s)
    assert list(got) == want


def test_pdl_u1_check_random_batch(gpu_ctx):
    rnd = random.Random(12)
    count = 3000
    s1s = [rnd.randrange(2 ** 1100) for _ in range(count)]   # the PDL s1 is wider than q
    es = [rnd.randrange(2 ** 256) for _ in range(count)]
    Qs = [ec.mul(ec.G, rnd.randrange(1, N)) for _ in range(count)]
    u1s = [_u1(s, e, q) for s, e, q in zip(s1s, es, Qs)]
    flip = set(rnd.sample(range(count), 40))
    for i in flip:
        u1s[i] = ec.add(u1s[i], ec.G)
    got = gpu_ctx.pdl_u1_check(s1s, es, Qs, u1s)
    assert [i for i in range(count) if got[i] == 0] == sorted(flip)


def test_ec_msm_glv_vs_oracle(gpu_ctx):
    rnd = random.Random(13)
    pts = [ec.G, ec.neg(ec.G), None] + [ec.mul(ec.G, rnd.randrange(1, N)) for _ in range(9)]
    rows, scs, want = [], [], []
    scal = [k % 2 ** 256 for k in EDGE + [N, 2 ** 256 - 1, LAM * 2 % N]]
    for o in range(24):
        terms = [pts[(o + j) % len(pts)] for j in range(3)]
        ks = [scal[(o * 3 + j) % len(scal)] if o < 12 else rnd.randrange(2 ** 256) for j in range(3)]
        acc = None
        for pt, k in zip(terms, ks):
            acc = ec.add(acc, ec.mul(pt, k % N) if pt is not None else None)
        rows.append(terms)
        scs.append(ks)
        want.append(acc)
    assert gpu_ctx.ec_msm(rows, scs) == want
