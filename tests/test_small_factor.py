"""The correct-key primorial check's trial division (hbn::SmallFactorSieve,
fs-dkr_amd/csrc/hostbn.hpp) against Python trial division by every prime below
6370 (collect.hpp CK_ALPHA), and against the round-2 routine, on CPU: random
odd values of 64 to 192 limbs, values with one planted factor (each prime
class, including the largest below the bound), products of two primes just
above it, 0, 1 and 2."""
import os
import random
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PRIMES = [p for p in range(2, 6370) if all(p % q for q in range(2, int(p ** 0.5) + 1))]


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    out = tmp_path_factory.mktemp("sf") / "small_factor_host"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(REPO, "fs-dkr_amd", "csrc"),
                    os.path.join(REPO, "tests", "native", "small_factor_host.cpp"), "-o", str(out)], check=True)
    return str(out)


def _limbs(v, n):
    return [(v >> (32 * j)) & 0xFFFFFFFF for j in range(n)]


def test_sieve_matches_trial_division(exe):
    rnd = random.Random(11)
    vals = [0, 1, 2, 3, 6367 * 6361, 6373 * 6379, (1 << 6143) | 1]
    for bits in (2048, 3072, 4096, 6144):
        for _ in range(40):
            vals.append(rnd.getrandbits(bits) | 1 | (1 << (bits - 1)))
        for p in rnd.sample(PRIMES, 12) + [3, 5, 6367]:
            vals.append((rnd.getrandbits(bits - 14) | 1) * p)
        big = [q for q in range(6371, 8000, 2) if all(q % r for r in range(3, int(q ** 0.5) + 1, 2))]
        vals.append(big[0] * big[1] * (rnd.getrandbits(bits - 30) | 1))
    widths = [max(1, (v.bit_length() + 31) // 32) + random.Random(v).randint(0, 3) for v in vals]
    widths = [min(w, 192) for w in widths]
    inp = f"{len(vals)} " + " ".join(f"{w} " + " ".join(map(str, _limbs(v, w))) for v, w in zip(vals, widths))
    out = subprocess.run([exe], input=inp, capture_output=True, text=True, check=True).stdout.split("\n")
    for v, line in zip(vals, out):
        want = v == 0 or any(v % p == 0 for p in PRIMES)
        got_new, got_old = (bool(int(x)) for x in line.split())
        assert got_new == want and got_old == want, (v, got_new, got_old, want)
