"""curv-kzen 0.10 BigInt semantics with the default rust-gmp-kzen backend
(/root/reference/Cargo.toml:33,41-44) — TEST INFRASTRUCTURE ONLY.

Arithmetic is exact Python ints; mod_pow / mod_inv go through the system GMP
(libgmp.so.10, the library the reference links) when present, else Python's
pow.  Both are exact, so results are identical."""
import ctypes
import ctypes.util


class PanicError(Exception):
    """A condition on which the Rust reference panics (unwrap/assert/index)."""


# ---------------------------------------------------------------- encoding ----
def to_bytes(n: int) -> bytes:
    """curv Converter::to_bytes [dep, unverified]: rust-gmp `Vec<u8>::from(&Mpz)`
    = big-endian magnitude of (sizeinbase(2)+7)/8 bytes; zero -> b"\\x00"
    (mpz_sizeinbase(0,2) == 1); the sign is dropped (mpz_export)."""
    n = abs(n)
    return n.to_bytes(max(1, (n.bit_length() + 7) // 8), "big")


def from_bytes(b: bytes) -> int:
    """curv Converter::from_bytes: big-endian, non-negative."""
    return int.from_bytes(b, "big")


# ------------------------------------------------------------------ GMP -------
class _Mpz(ctypes.Structure):
    _fields_ = [("alloc", ctypes.c_int), ("size", ctypes.c_int), ("d", ctypes.c_void_p)]


def _load_gmp():
    for name in ("libgmp.so.10", ctypes.util.find_library("gmp")):
        if not name:
            continue
        try:
            g = ctypes.CDLL(name)
        except OSError:
            continue
        g.__gmpz_sizeinbase.restype = ctypes.c_size_t
        g.__gmpz_invert.restype = ctypes.c_int
        g.__gmpz_probab_prime_p.restype = ctypes.c_int
        return g
    return None


_gmp = _load_gmp()
if _gmp is not None:   # module-level handles (``__gmpz_*`` would be name-mangled inside classes)
    _g_init = getattr(_gmp, "__gmpz_init")
    _g_clear = getattr(_gmp, "__gmpz_clear")
    _g_import = getattr(_gmp, "__gmpz_import")
    _g_export = getattr(_gmp, "__gmpz_export")
    _g_sizeinbase = getattr(_gmp, "__gmpz_sizeinbase")
    _g_powm = getattr(_gmp, "__gmpz_powm")
    _g_prime = getattr(_gmp, "__gmpz_probab_prime_p")


class _Z:
    __slots__ = ("z",)

    def __init__(self, v=None):
        self.z = _Mpz()
        _g_init(ctypes.byref(self.z))
        if v is not None:
            self.set(v)

    def set(self, v):
        assert v >= 0
        b = v.to_bytes(max(1, (v.bit_length() + 7) // 8), "little")
        _g_import(ctypes.byref(self.z), ctypes.c_size_t(len(b)), -1, 1, 0, 0, b)
        return self

    def get(self):
        n = (_g_sizeinbase(ctypes.byref(self.z), 2) + 7) // 8
        buf = ctypes.create_string_buffer(n + 8)
        cnt = ctypes.c_size_t()
        _g_export(buf, ctypes.byref(cnt), -1, 1, 0, 0, ctypes.byref(self.z))
        return int.from_bytes(buf.raw[:cnt.value], "little")

    def __del__(self):
        try:
            _g_clear(ctypes.byref(self.z))
        except Exception:
            pass


def have_gmp() -> bool:
    return _gmp is not None


def _powm(b, e, m):
    if _gmp is None or m.bit_length() < 512:
        return pow(b, e, m)
    r, zb, ze, zm = _Z(), _Z(b % m), _Z(e), _Z(m)   # keep the wrappers alive across the call
    _g_powm(ctypes.byref(r.z), ctypes.byref(zb.z), ctypes.byref(ze.z), ctypes.byref(zm.z))
    return r.get()


# ----------------------------------------------------------- curv traits ------
def mod_pow(base: int, exponent: int, modulus: int) -> int:
    """curv BigInt::mod_pow -> GMP mpz_powm.  curv asserts a non-negative
    exponent [dep, unverified] (a panic in the reference)."""
    if exponent < 0:
        raise PanicError("mod_pow: negative exponent")
    if modulus <= 0:
        raise PanicError("mod_pow: non-positive modulus")
    if modulus == 1:
        return 0
    return _powm(base % modulus, exponent, modulus)


_POOL = None


def pool():
    """Shared thread pool for the oracle's independent checks: GMP mpz_powm runs
    through ctypes, which releases the GIL, so per-proof checks overlap.  The
    caller still consumes the results in the reference's order (the restated
    semantics -- which check fails or panics first -- are unchanged)."""
    global _POOL
    if _POOL is None:
        import os
        from concurrent.futures import ThreadPoolExecutor
        try:
            ncpu = len(os.sched_getaffinity(0))
        except AttributeError:
            ncpu = os.cpu_count() or 1
        _POOL = ThreadPoolExecutor(max_workers=max(1, min(16, ncpu)))
    return _POOL


def outcome(fn, *args):
    """Run fn(*args) and capture its result or exception: (True, value) / (False, exc)."""
    try:
        return True, fn(*args)
    except Exception as e:  # re-raised by settle() at the point the reference would reach it
        return False, e


def settle(res):
    ok, v = res
    if not ok:
        raise v
    return v


def mod_inv(a: int, modulus: int):
    """curv BigInt::mod_inv -> GMP mpz_invert; None when gcd(a, m) != 1."""
    if modulus < 1:
        raise PanicError("mod_inv: modulus must be >= 1")
    try:
        return pow(a, -1, modulus)
    except ValueError:
        return None


def mod_mul(a: int, b: int, modulus: int) -> int:
    """curv BigInt::mod_mul = (a mod m)(b mod m) mod m."""
    return (a % modulus) * (b % modulus) % modulus


def mod_add(a: int, b: int, modulus: int) -> int:
    return (a % modulus + b % modulus) % modulus


def gcd(a: int, b: int) -> int:
    import math
    return math.gcd(a, b)


def is_probable_prime(n: int, rounds: int = 30) -> bool:
    if n < 2:
        return False
    if _gmp is not None:
        zn = _Z(n)
        return _g_prime(ctypes.byref(zn.z), rounds) > 0
    small = (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37)
    for p in small:
        if n % p == 0:
            return n == p
    d, s = n - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    for a in small[:12]:
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(s - 1):
            x = x * x % n
            if x == n - 1:
                break
        else:
            return False
    return True
