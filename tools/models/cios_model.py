"""Pure-Python model of the lane-distributed CIOS Montgomery multiply used by
fs-dkr_amd/csrc/modexp.hip (G lanes per instance, L = K/G limbs per lane,
deferred cross-lane carries).  Used only to validate the carry/shift algebra
before it is written in HIP; not product code and not the oracle."""
import random

M32 = (1 << 32) - 1


def to_limbs(x, k):
    return [(x >> (32 * i)) & M32 for i in range(k)]


def from_limbs(v):
    return sum(l << (32 * i) for i, l in enumerate(v))


def montmul_model(a, b, n, K, G):
    L = K // G
    n0inv = (-pow(n, -1, 1 << 32)) & M32
    A = to_limbs(a, K)
    B = [to_limbs(b, K)[g * L:(g + 1) * L] for g in range(G)]
    N = [to_limbs(n, K)[g * L:(g + 1) * L] for g in range(G)]
    t = [[0] * L for _ in range(G)]
    x = [0] * G
    for i in range(K):
        ai = A[i]
        for g in range(G):                      # pass A
            C = 0
            for j in range(L):
                P = ai * B[g][j] + t[g][j] + C
                t[g][j] = P & M32
                C = P >> 32
            x[g] += C
        m = (t[0][0] * n0inv) & M32             # lane 0 of the group, broadcast
        v0 = [0] * G
        for g in range(G):                      # pass B with in-lane shift
            P = m * N[g][0] + t[g][0]
            v0[g] = P & M32
            C = P >> 32
            for j in range(1, L):
                P = m * N[g][j] + t[g][j] + C
                t[g][j - 1] = P & M32
                C = P >> 32
            x[g] += C
        assert v0[0] == 0
        for g in range(G):                      # cross-lane shift
            nv = v0[g + 1] if g + 1 < G else 0
            S = x[g] + nv
            t[g][L - 1] = S & M32
            x[g] = S >> 32
            assert x[g] < 8
    # resolve deferred carries: ripple G-1 rounds
    for _ in range(G - 1):
        y = [0] + x[:-1]
        x = [0] * (G - 1) + [x[-1]]
        for g in range(G):
            C = y[g]
            for j in range(L):
                S = t[g][j] + C
                t[g][j] = S & M32
                C = S >> 32
            if g < G - 1:
                x[g] += C
            else:
                x[g] += C
    T = from_limbs([l for g in range(G) for l in t[g]]) + (x[-1] << (32 * K))
    R = 1 << (32 * K)
    assert T == (a * b * pow(R, -1, n)) % n or T == (a * b * pow(R, -1, n)) % n + n, "bad"
    assert T < 2 * n
    return T - n if T >= n else T


if __name__ == "__main__":
    rnd = random.Random(1)
    for K, G in [(8, 1), (8, 2), (8, 4), (64, 2), (128, 4), (16, 4)]:
        for _ in range(200):
            n = rnd.getrandbits(32 * K) | 1 | (1 << (32 * K - 1))
            if rnd.random() < 0.3:
                n = (1 << (32 * K)) - 1 - 2 * rnd.getrandbits(8)  # near-max moduli stress carries
            a = rnd.randrange(n); b = rnd.randrange(n)
            if rnd.random() < 0.2:
                a = n - 1; b = n - 1
            r = montmul_model(a, b, n, K, G)
            assert r == a * b * pow(1 << (32 * K), -1, n) % n
    print("cios model ok")
