"""The streaming SHA-256 of fs-dkr_amd/csrc/sha256.hpp (host + device code,
curv to_bytes absorption incl. unaligned word appends) against hashlib, on CPU."""
import hashlib
import os
import random
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def sha_exe(tmp_path_factory):
    out = tmp_path_factory.mktemp("sha") / "sha_host"
    subprocess.run(["hipcc", "-O1", "-std=c++17", "-I", os.path.join(REPO, "fs-dkr_amd", "csrc"),
                    os.path.join(REPO, "tests", "native", "sha_host.cpp"), "-o", str(out)], check=True)
    return str(out)


def _to_bytes(v):
    return v.to_bytes(max(1, (v.bit_length() + 7) // 8), "big")


def test_sha_matches_hashlib(sha_exe):
    rnd = random.Random(1)
    for trial in range(40):
        vals = []
        for _ in range(rnd.randint(1, 12)):
            bits = rnd.choice([0, 1, 7, 8, 9, 31, 32, 33, 255, 256, 257, 1000, 2048, 4096])
            vals.append(rnd.getrandbits(bits) if bits else 0)
        limbs = []
        for v in vals:
            n = max(1, (v.bit_length() + 31) // 32) + rnd.randint(0, 2)   # zero-padded widths
            limbs.append([(v >> (32 * j)) & 0xFFFFFFFF for j in range(n)])
        inp = f"{len(vals)} " + " ".join(f"{len(l)} " + " ".join(map(str, l)) for l in limbs)
        out = subprocess.run([sha_exe], input=inp, capture_output=True, text=True, check=True).stdout.split()
        got = sum(int(x) << (32 * i) for i, x in enumerate(out))
        want = int.from_bytes(hashlib.sha256(b"".join(_to_bytes(v) for v in vals)).digest(), "big")
        assert got == want, (trial, vals)
