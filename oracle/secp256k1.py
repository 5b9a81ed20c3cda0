"""secp256k1 group as used through curv `Point<Secp256k1>` / `Scalar<Secp256k1>`
(curv-kzen 0.10, secp256k1 backend [dep]) — TEST INFRASTRUCTURE ONLY.

Points are affine (x, y) tuples or None (the point at infinity)."""
P = 2**256 - 2**32 - 977
Q = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
GX = 0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798
GY = 0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8
G = (GX, GY)


def scalar(n: int) -> int:
    """curv Scalar::from(&BigInt): reduction mod q (negatives to [0,q))."""
    return n % Q


def is_on_curve(pt) -> bool:
    if pt is None:
        return True
    x, y = pt
    return 0 <= x < P and 0 <= y < P and (y * y - x * x * x - 7) % P == 0


def _to_jac(pt):
    return (pt[0], pt[1], 1)


def _from_jac(j):
    X, Y, Z = j
    if Z == 0:
        return None
    zi = pow(Z, -1, P)
    zi2 = zi * zi % P
    return (X * zi2 % P, Y * zi2 * zi % P)


def _jdbl(j):
    X, Y, Z = j
    if Z == 0 or Y == 0:
        return (0, 1, 0)
    S = 4 * X * Y * Y % P
    M = 3 * X * X % P
    X3 = (M * M - 2 * S) % P
    Y3 = (M * (S - X3) - 8 * Y ** 4) % P
    Z3 = 2 * Y * Z % P
    return (X3, Y3, Z3)


def _jadd(a, b):
    if a[2] == 0:
        return b
    if b[2] == 0:
        return a
    X1, Y1, Z1 = a
    X2, Y2, Z2 = b
    Z1s, Z2s = Z1 * Z1 % P, Z2 * Z2 % P
    U1, U2 = X1 * Z2s % P, X2 * Z1s % P
    S1, S2 = Y1 * Z2s * Z2 % P, Y2 * Z1s * Z1 % P
    if U1 == U2:
        if S1 != S2:
            return (0, 1, 0)
        return _jdbl(a)
    H = (U2 - U1) % P
    R = (S2 - S1) % P
    H2 = H * H % P
    H3 = H * H2 % P
    X3 = (R * R - H3 - 2 * U1 * H2) % P
    Y3 = (R * (U1 * H2 - X3) - S1 * H3) % P
    Z3 = H * Z1 * Z2 % P
    return (X3, Y3, Z3)


def add(a, b):
    if a is None:
        return b
    if b is None:
        return a
    return _from_jac(_jadd(_to_jac(a), _to_jac(b)))


def neg(a):
    return None if a is None else (a[0], (-a[1]) % P)


def mul(pt, k: int):
    """pt * Scalar::from(k)."""
    k = scalar(k)
    if pt is None or k == 0:
        return None
    acc = (0, 1, 0)
    base = _to_jac(pt)
    for bit in bin(k)[2:]:
        acc = _jdbl(acc)
        if bit == "1":
            acc = _jadd(acc, base)
    return _from_jac(acc)


def to_bytes_compressed(pt) -> bytes:
    """Point::to_bytes(true): SEC1 compressed; the zero point serialises as 33
    zero bytes in curv's secp256k1 backend [dep, unverified]."""
    if pt is None:
        return b"\x00" * 33
    return bytes([2 + (pt[1] & 1)]) + pt[0].to_bytes(32, "big")


def to_bigint_compressed(pt) -> int:
    """BigInt::from_bytes(&P.to_bytes(true)) as hashed in zk_pdl_with_slack.rs:88-92,115-119."""
    return int.from_bytes(to_bytes_compressed(pt), "big")
