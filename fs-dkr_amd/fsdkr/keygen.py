"""Batched key generation on the MI355X engine.

Replaces, under the reference's unchanged API, what kzen-paillier 0.4.3 and
zk-paillier 0.4.4 compute for the refresh:
  Paillier::keypair_with_modulus_size   refresh_message.rs:118, ring_pedersen_proof.rs:50,
                                        add_party_message.rs:51
  NiCorrectKeyProof::proof              refresh_message.rs:119, add_party_message.rs:103

The prime walk (the same walk the oracle restates, oracle/keygen.py) is one
C-ABI call, fsdkr_sample_primes (csrc/keygen.cpp): a random start with the top
two bits and the low bit set, then the first probable prime among the next
4*bits odd numbers (else a new start): a sieve by the odd primes below 2000 on
the host, Miller-Rabin to base 2 on a window of survivors of every walk in one
GPU launch (fsdkr_miller_rabin), then 8 rounds to candidate-derived bases on each
walk's first passer.  Draw order: every walk's start first, in walk order; a
walk that ends without a prime draws a new start after every walk of its pass
is settled.  A batch of one is exactly the sequential walk, so single keys match
the oracle's keys for the same draws.  Nothing consumes draws besides the
starts."""
import hashlib

from .refresh import _ctx
from .types import DecryptionKey, EncryptionKey, NiCorrectKeyProof

SALT = bytes([75, 90, 101, 110])    # zk-paillier SALT_STRING [dep, unverified]
M2 = 11                             # NiCorrectKeyProof sigma_vec length


def sample_primes(ctx, rng, bits, count, window=None, span=None):
    """`count` primes of `bits` bits (top two bits set) by independent walks of
    `span` odd candidates (default 4*bits; shorter walks exercise the redraws);
    rng.bits(k) draws the starts."""
    if bits < 64:
        raise ValueError("sample_primes: bits >= 64")
    return _ctx(ctx).sample_primes(rng.bits, bits, count, window or 0, span or 0)


def prime(ctx, rng, bits):
    """One walk: the oracle's Rng.prime for the same draws."""
    return sample_primes(ctx, rng, bits, 1)[0]


def keypair_with_modulus_size(ctx, rng, bits):
    """Paillier::keypair_with_modulus_size (refresh_message.rs:118): p, then q,
    redrawn while equal (the oracle's sequential draw order)."""
    while True:
        p = prime(ctx, rng, bits // 2)
        q = prime(ctx, rng, bits // 2)
        if p != q:
            n = p * q
            return EncryptionKey(n, n * n), DecryptionKey(p, q)


def keypairs_with_modulus_size(ctx, rng, bits, count):
    """`count` keypairs from one batch of 2*count walks (pair k = primes 2k, 2k+1;
    a pair with p == q redraws q after the batch, pairs in order)."""
    primes = sample_primes(ctx, rng, bits // 2, 2 * count)
    out = []
    for k in range(count):
        p, q = primes[2 * k], primes[2 * k + 1]
        while p == q:
            q = prime(ctx, rng, bits // 2)
        n = p * q
        out.append((EncryptionKey(n, n * n), DecryptionKey(p, q)))
    return out


# ------------------------------------------------------- correct-key proofs ----
def _chain(*vals):
    h = hashlib.sha256()
    for v in vals:
        v = abs(v)
        h.update(v.to_bytes(max(1, (v.bit_length() + 7) // 8), "big"))
    return int.from_bytes(h.digest(), "big")


def correct_key_rho(n):
    """zk-paillier NiCorrectKeyProof rho_j = mask_generation(|n|, H(n, salt, j)) mod n [dep]."""
    salt = int.from_bytes(SALT, "big")
    klen = n.bit_length()
    out = []
    for j in range(M2):
        seed = _chain(n, salt, j)
        msk = sum(_chain(seed, k) << (256 * k) for k in range(klen // 256 + 1))
        out.append(msk % n)
    return out


def _width(bits):
    for w in (64, 96, 128, 192):
        if bits <= 32 * w:
            return w
    raise ValueError(f"{bits}-bit modulus")


def correct_key_proofs(ctx, dks):
    """NiCorrectKeyProof::proof for many keys (refresh_message.rs:119):
    sigma_j = rho_j^(n^-1 mod phi) mod n, all 11*len(dks) exponentiations in one
    GPU launch per modulus width."""
    ctx = _ctx(ctx)
    out = [None] * len(dks)
    by_w = {}
    for k, dk in enumerate(dks):
        by_w.setdefault(_width((dk.p * dk.q).bit_length()), []).append(k)
    for w, ks in by_w.items():
        bases, exps, mods, midx = [], [], [], []
        for m, k in enumerate(ks):
            dk = dks[k]
            n = dk.p * dk.q
            d = pow(n, -1, (dk.p - 1) * (dk.q - 1))
            bases += correct_key_rho(n)
            exps += [d] * M2
            mods.append(n)
            midx += [m] * M2
        sig = ctx.modexp_batch(bases, exps, mods, midx, w, secret=True)   # d = N^-1 mod phi is secret
        for m, k in enumerate(ks):
            out[k] = NiCorrectKeyProof(tuple(sig[M2 * m:M2 * m + M2]))
    return out


def refresh_keys(ctx, rng, bits, count):
    """The key material of `count` distribute() calls (refresh_message.rs:118-119):
    [(EncryptionKey, DecryptionKey, NiCorrectKeyProof)], two batched GPU rounds."""
    kps = keypairs_with_modulus_size(ctx, rng, bits, count)
    cks = correct_key_proofs(ctx, [dk for _, dk in kps])
    return [(ek, dk, ck) for (ek, dk), ck in zip(kps, cks)]
