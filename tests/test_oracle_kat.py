"""Known-answer tests pinning the oracle's primitives (CPU)."""
import hashlib
import random

from oracle import bigint, paillier
from oracle import secp256k1 as ec
from oracle.hashing import chain_bigint
from oracle.rng import Rng
from oracle.vss import VerifiableSS, map_share_to_new_params


def test_sha256_known_answer():
    assert hashlib.sha256(b"abc").hexdigest() == "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"
    # chain_bigint hashes the concatenated minimal big-endian encodings
    assert chain_bigint(0x616263) == int("ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad", 16)


def test_to_bytes_encoding():
    assert bigint.to_bytes(0) == b"\x00"
    assert bigint.to_bytes(1) == b"\x01"
    assert bigint.to_bytes(256) == b"\x01\x00"
    assert bigint.to_bytes(-5) == b"\x05"


def test_secp256k1_known_points():
    # 2G and 3G from the SEC2 test vectors
    two = ec.mul(ec.G, 2)
    assert two == (0xC6047F9441ED7D6D3045406E95C07CD85C778E4B8CEF3CA7ABAC09B95C709EE5,
                   0x1AE168FEA63DC339A3C58419466CEAEEF7F632653266D0E1236431A950CFE52A)
    assert ec.mul(ec.G, 3)[0] == 0xF9308A019258C31049344F85F89D5229B531C845836F99B08601F113BCE036F9
    assert ec.mul(ec.G, ec.Q) is None
    assert ec.mul(ec.G, ec.Q + 5) == ec.mul(ec.G, 5)
    assert ec.is_on_curve(ec.mul(ec.G, 123456789))
    assert ec.to_bytes_compressed(ec.G).hex() == "0279be667ef9dcbbac55a06295ce870b07029bfcdb2dce28d959f2815b16f81798"


def test_gmp_matches_python_pow():
    rnd = random.Random(3)
    for bits in (512, 2048, 4096):
        m = rnd.getrandbits(bits) | 1
        b, e = rnd.getrandbits(bits + 40), rnd.getrandbits(bits)
        assert bigint.mod_pow(b, e, m) == pow(b, e, m)
    assert bigint.mod_inv(6, 9) is None
    assert bigint.mod_inv(2, 9) == 5


def test_paillier_homomorphism():
    rng = Rng("paillier-kat")
    ek, dk = paillier.keypair_with_modulus_size(512, rng)
    c1 = paillier.encrypt_with_chosen_randomness(ek, 41, 7)
    c2 = paillier.encrypt(ek, 1, rng)
    assert paillier.decrypt(dk, paillier.add(ek, c1, c2)) == 42
    assert paillier.decrypt(dk, paillier.mul(ek, c1, 3)) == 123


def test_feldman_and_lagrange():
    rng = Rng("vss")
    vss, shares = VerifiableSS.share(2, 5, 1234, rng)
    for i in range(5):
        assert vss.validate_share_public(ec.mul(ec.G, shares[i]), i + 1)
    assert not vss.validate_share_public(ec.mul(ec.G, shares[0] + 1), 1)
    idx = [0, 2, 4]
    assert sum(map_share_to_new_params(i, idx) * shares[i] for i in idx) % ec.Q == 1234
