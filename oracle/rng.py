"""Seeded randomness — TEST INFRASTRUCTURE ONLY.

The reference draws every random value from the OS RNG through curv
`BigInt::sample_below` / `sample_range` (rejection sampling on bit length,
[dep]) and has no seeding hook.  Bit-exact transcripts need
injected randomness, so the oracle uses a SHA-256 counter-mode stream with the
same sampling structure."""
import hashlib

from . import bigint


class Rng:
    def __init__(self, seed):
        self._key = hashlib.sha256(repr(seed).encode()).digest()
        self._ctr = 0

    def _block(self) -> bytes:
        self._ctr += 1
        return hashlib.sha256(self._key + self._ctr.to_bytes(8, "little")).digest()

    def bits(self, k: int) -> int:
        if k <= 0:
            return 0
        nbytes = (k + 7) // 8
        buf = b""
        while len(buf) < nbytes:
            buf += self._block()
        return int.from_bytes(buf[:nbytes], "big") >> (8 * nbytes - k)

    def sample_below(self, upper: int) -> int:
        """curv BigInt::sample_below: sample bit_length(upper) bits until < upper."""
        if upper <= 0:
            raise bigint.PanicError("sample_below: upper must be positive")
        k = upper.bit_length()
        while True:
            x = self.bits(k)
            if x < upper:
                return x

    def sample_range(self, lower: int, upper: int) -> int:
        """curv BigInt::sample_range(lower, upper) = lower + sample_below(upper - lower)."""
        return lower + self.sample_below(upper - lower)

    def from_modulo(self, n: int) -> int:
        """SampleFromMultiplicativeGroup::from_modulo (range_proofs.rs:599-607)."""
        while True:
            r = self.sample_below(n)
            if bigint.gcd(r, n) == 1:
                return r

    def prime(self, bits: int) -> int:
        """A `bits`-bit prime with the top two bits set (so p*q has exactly 2*bits bits)."""
        while True:
            c = self.bits(bits) | (3 << (bits - 2)) | 1
            # walk to the next probable prime from a random start
            for _ in range(4 * bits):
                if c >> bits:       # the walk stays below 2^bits
                    break
                if bigint.is_probable_prime(c):
                    return c
                c += 2
