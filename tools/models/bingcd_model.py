"""Model of the GPU modular inverse (fs-dkr_amd/csrc/inverse.hip): T. Pornin,
"Optimized Binary GCD for Modular Inversion" (eprint 2020/972, Alg. 2), with
k-1 = 31 inner steps on 64-bit approximations and u, v divided by 2^31 mod m
in Montgomery style each outer step.  Development model, not product code."""
import random

M31 = (1 << 31) - 1


def inverse(y, m):
    """y^-1 mod m (m odd, 0 <= y < m) or None."""
    L = m.bit_length()
    a, b, u, v = y, m, 1, 0
    minv = pow(m, -1, 1 << 31)
    mprime = (-minv) % (1 << 31)
    iters = (2 * L - 1 + 30) // 31
    for _ in range(iters):
        n = max(a.bit_length(), b.bit_length(), 64)
        ah = (a & M31) | ((a >> (n - 33)) << 31)
        bh = (b & M31) | ((b >> (n - 33)) << 31)
        f0, g0, f1, g1 = 1, 0, 0, 1
        for _ in range(31):
            if ah & 1:
                if ah < bh:
                    ah, bh = bh, ah
                    f0, g0, f1, g1 = f1, g1, f0, g0
                ah -= bh
                f0 -= f1
                g0 -= g1
            ah >>= 1
            f1 <<= 1
            g1 <<= 1
        assert abs(f0) + abs(g0) <= 1 << 31 and abs(f1) + abs(g1) <= 1 << 31
        na = a * f0 + b * g0
        nb = a * f1 + b * g1
        assert na % (1 << 31) == 0 and nb % (1 << 31) == 0
        na >>= 31
        nb >>= 31
        if na < 0:
            na, f0, g0 = -na, -f0, -g0
        if nb < 0:
            nb, f1, g1 = -nb, -f1, -g1
        a, b = na, nb

        def mdiv(t):
            q = ((t & M31) * mprime) & M31
            r = (t + q * m) >> 31
            if r < 0:
                r += m
            if r >= m:
                r -= m
            assert 0 <= r < m
            return r
        u, v = mdiv(u * f0 + v * g0), mdiv(u * f1 + v * g1)
    assert a == 0
    return v if b == 1 else None


if __name__ == "__main__":
    rnd = random.Random(1)
    for bits in (64, 255, 2048, 4096):
        for _ in range(60):
            m = rnd.getrandbits(bits) | 1 | (1 << (bits - 1))
            y = rnd.randrange(m)
            r = inverse(y, m)
            try:
                want = pow(y, -1, m)
            except ValueError:
                want = None
            assert r == want, (bits, y, m)
        # non-units
        p = 65537
        m = p * (rnd.getrandbits(bits - 17) | 1)
        assert inverse(p * 3 % m, m) is None
        assert inverse(0, m) is None
    print("bingcd model ok")
