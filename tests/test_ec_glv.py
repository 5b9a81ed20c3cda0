"""The GLV split behind the secp256k1 scalar multiplications (csrc/vec.hip:
scalar_split_lambda, the lattice decomposition of libsecp256k1's
secp256k1_scalar_split_lambda restated), checked on the CPU against the
oracle's curve arithmetic (oracle/secp256k1.py, the restatement of the curv /
libsecp256k1 group law the reference uses at zk_pdl_with_slack.rs:124-127):
lambda and beta are the cube roots with lambda * P = (beta x, y), every k splits
as k = s1 + s2 lambda (mod q) with |s1|, |s2| < 2^128, and the __constant__
limbs in vec.hip are these values."""
import os
import random
import re

from oracle import secp256k1 as ec

P, N = ec.P, ec.Q
LAM = 0x5363ad4cc05c30e0a5261c028812645a122e22ea20816678df02967c1b23bd72
BETA = 0x7ae96a2b657c07106e64479eac3434e99cf0497512f58995c1396c28719501ee
MB1 = 0xe4437ed6010e88286f547fa90abfe4c3
MB2 = 0xfffffffffffffffffffffffffffffffe8a280ac50774346dd765cda83db1562c
G1 = 0x3086d221a7d46bcde86c90e49284eb153daa8a1471e8ca7fe893209a45dbb031
G2 = 0xe4437ed6010e88286f547fa90abfe4c4221208ac9df506c61571b4ae8ac47f71
EDGE = [0, 1, 2, N - 1, N - 2, LAM, N - LAM, (N - 1) // 2, (N + 1) // 2, 2 ** 128, 2 ** 128 - 1, N - 2 ** 128,
        2 ** 255, MB1, G1 % N, G2 % N]


def split(k):
    """vec.hip scalar_split_lambda: c_i = round(k g_i / 2^384), r2 = c1 (-b1) + c2 (-b2),
    r1 = k - r2 lambda (mod q); signed by r > (q - 1) / 2."""
    def mul_shift(g):
        t = k * g
        return (t >> 384) + ((t >> 383) & 1)
    r2 = (mul_shift(G1) * MB1 + mul_shift(G2) * MB2) % N
    r1 = (k - r2 * LAM) % N
    return tuple(r if r <= (N - 1) // 2 else r - N for r in (r1, r2))


def test_endomorphism_constants():
    assert pow(LAM, 3, N) == 1 and LAM != 1
    assert pow(BETA, 3, P) == 1 and BETA != 1
    for k in (1, 7, 2 ** 200 + 5):
        pt = ec.mul(ec.G, k)
        assert ec.mul(pt, LAM) == ((BETA * pt[0]) % P, pt[1])


def test_split_bounds_and_identity():
    rnd = random.Random(7)
    for k in EDGE + [rnd.randrange(N) for _ in range(20000)]:
        s1, s2 = split(k)
        assert (s1 + s2 * LAM - k) % N == 0
        assert abs(s1) < 2 ** 128 and abs(s2) < 2 ** 128, k


def test_split_points_match_oracle_mul():
    rnd = random.Random(8)
    for k in EDGE[:10] + [rnd.randrange(N) for _ in range(6)]:
        pt = ec.mul(ec.G, rnd.randrange(1, N))
        s1, s2 = split(k)
        a = ec.mul(pt, abs(s1))
        a = ec.neg(a) if s1 < 0 and a is not None else a
        b = ec.mul(((BETA * pt[0]) % P, pt[1]), abs(s2))
        b = ec.neg(b) if s2 < 0 and b is not None else b
        assert ec.add(a, b) == ec.mul(pt, k)


def test_device_constants_are_these():
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fs-dkr_amd", "csrc",
                            "vec.hip")).read()

    def const(name):
        body = re.search(name + r"\[\d+\] = \{([^}]*)\}", src).group(1)
        limbs = [int(x.strip().rstrip("u"), 16) for x in body.split(",")]
        return sum(v << (32 * i) for i, v in enumerate(limbs))
    assert const("GLV_LAMBDA") == LAM and const("GLV_BETA") == BETA
    assert const("GLV_MB1") == MB1 and const("GLV_MB2") == MB2
    assert const("GLV_G1") == G1 and const("GLV_G2") == G2
    assert const("Q_HALF") == (N - 1) // 2
