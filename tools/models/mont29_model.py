"""Python model of the radix-2^29 lane-distributed Montgomery multiply in
fs-dkr_amd/csrc/mont29.hpp (64-bit lazy column accumulators, rotating
register slots, partial normalisation).  Asserts the 64-bit no-overflow bound
at every step.  Development model only (not product code, not the oracle)."""
import random

B = 29
M = (1 << B) - 1
U64 = 1 << 64


def digits(x, kd):
    return [(x >> (B * i)) & M for i in range(kd)]


def value(ds):
    return sum(d << (B * i) for i, d in enumerate(ds))


def montmul(adig, bdig, n, KD, G, NORM_AT):
    L = KD // G
    ninv = (-pow(n, -1, 1 << B)) & M
    nd = digits(n, KD)
    Nl = [nd[g * L:(g + 1) * L] for g in range(G)]
    Bl = [bdig[g * L:(g + 1) * L] for g in range(G)]
    acc = [[0] * L for _ in range(G)]           # physical slots
    for cyc in range(G):
        for r in range(L):
            i = cyc * L + r
            ai = adig[i]
            sl = lambda j: (j + r) % L
            for g in range(G):
                for j in range(L):
                    acc[g][sl(j)] += ai * Bl[g][j]
                    assert acc[g][sl(j)] < U64
            m = ((acc[0][sl(0)] & 0xFFFFFFFF) * ninv) & M
            for g in range(G):
                for j in range(L):
                    acc[g][sl(j)] += m * Nl[g][j]
                    assert acc[g][sl(j)] < U64
            assert acc[0][sl(0)] & M == 0
            acc[0][sl(1)] += acc[0][sl(0)] >> B        # carry fold, lane 0 only
            nxt = [acc[g + 1][sl(0)] if g + 1 < G else 0 for g in range(G)]
            for g in range(G):
                acc[g][sl(0)] = nxt[g]
            if r in NORM_AT:
                rho = r + 1
                s2 = lambda j: (j + rho) % L
                cL = [acc[g][s2(L - 1)] >> B for g in range(G)]
                for g in range(G):
                    for j in range(L - 1, 0, -1):
                        acc[g][s2(j)] = (acc[g][s2(j)] & M) + (acc[g][s2(j - 1)] >> B)
                    acc[g][s2(0)] = (acc[g][s2(0)] & M) + (cL[g - 1] if g > 0 else 0)
                assert cL[G - 1] == 0
    # final 2-step partial normalisation
    for step in range(2):
        cL = [acc[g][L - 1] >> B for g in range(G)]
        for g in range(G):
            for j in range(L - 1, 0, -1):
                acc[g][j] = (acc[g][j] & M) + (acc[g][j - 1] >> B)
            acc[g][0] = (acc[g][0] & M) + (cL[g - 1] if g > 0 else 0)
        assert cL[G - 1] == 0
    out = [d for g in range(G) for d in acc[g]]
    assert max(out) <= M + 127, max(out) - M
    return out


if __name__ == "__main__":
    rnd = random.Random(5)
    for KD, G, nbits, NORM_AT in [(72, 2, 2048, (17, 35)), (144, 4, 4096, (17, 35)), (108, 4, 3072, (13, 26)),
                                  (216, 4, 6144, (17, 35, 53))]:
        R = 1 << (B * KD)
        for trial in range(40):
            n = rnd.getrandbits(nbits) | 1 | (1 << (nbits - 1))
            assert 4 * n < R
            # lazy inputs: value < 2n, digits up to M+127
            a = rnd.randrange(2 * n); b = rnd.randrange(2 * n)
            if trial % 5 == 0:
                a = 2 * n - 1; b = 2 * n - 1
            ad = digits(a, KD); bd = digits(b, KD)
            if trial % 3 == 0:   # redundant digits: borrow 1 from digit j+1, add 2^29 to digit j
                for j in range(KD - 1):
                    if ad[j + 1] > 0 and ad[j] <= 127:
                        ad[j + 1] -= 1; ad[j] += 1 << B
                        break
                ad = [min(d, d) for d in ad]
            assert value(ad) == a
            out = montmul(ad, bd, n, KD, G, NORM_AT)
            v = value(out)
            assert v % n == a * b * pow(R, -1, n) % n
            assert v < 2 * n, (v, n)
    print("mont29 model ok")
