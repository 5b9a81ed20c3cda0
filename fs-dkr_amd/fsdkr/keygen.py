"""Batched key generation on the MI355X engine.

Replaces, under the reference's unchanged API, what kzen-paillier 0.4.3 and
zk-paillier 0.4.4 compute for the refresh:
  Paillier::keypair_with_modulus_size   refresh_message.rs:118, ring_pedersen_proof.rs:50,
                                        add_party_message.rs:51
  NiCorrectKeyProof::proof              refresh_message.rs:119, add_party_message.rs:103

Prime walk (the same walk the oracle restates, oracle/keygen.py): a random
start with the top two bits and the low bit set, then the first probable prime
among the next 4*bits odd numbers (else a new start).  Per walk:
  * the host sieves the whole walk against the odd primes below 2000
    (numpy: one strided mark per prime);
  * the GPU runs a Miller–Rabin round to base 2 on a window of survivors of
    every walk at once (fsdkr_miller_rabin: b^d mod c on the batched modexp
    engine, witness squarings in prime.hip);
  * the first survivor passing base 2 gets MR_ROUNDS more rounds to
    candidate-derived bases (witness_bases), again one launch for all walks;
    a failure moves on to the walk's next base-2 passer.
Draw order: every walk's start first, in walk order; a walk that ends without
a prime draws a new start after every walk of its pass is settled.  A batch of
one is exactly the sequential walk, so single keys match the oracle's keys for
the same draws.  Nothing here consumes draws besides the starts."""
import hashlib

import numpy as np

from .refresh import _ctx
from .types import DecryptionKey, EncryptionKey, NiCorrectKeyProof

MR_ROUNDS = 8
SIEVE_LIMIT = 2000
MAX_PASSES = 1000
SALT = bytes([75, 90, 101, 110])    # zk-paillier SALT_STRING [dep, unverified]
M2 = 11                             # NiCorrectKeyProof sigma_vec length


def _odd_primes_below(n):
    flags = np.ones(n, dtype=bool)
    flags[:3] = False
    for i in range(2, int(n ** 0.5) + 1):
        if flags[i]:
            flags[i * i::i] = False
    flags[::2] = False
    return [int(p) for p in np.nonzero(flags)[0]]


_SMALL = _odd_primes_below(SIEVE_LIMIT)
_HALF = [pow(2, -1, p) for p in _SMALL]


def mr_width(bits):
    """u32 limbs of a candidate class: 1024-bit primes get their own 32-limb shape."""
    for w in (32, 64, 96):
        if bits <= 32 * w:
            return w
    raise ValueError(f"{bits}-bit candidate")


def sieve(start, span):
    """Offsets k in [0, span) with start + 2k divisible by no odd prime below 2000
    (start odd and far above 2000)."""
    keep = np.ones(span, dtype=bool)
    for p, h in zip(_SMALL, _HALF):
        keep[(-(start % p) * h) % p::p] = False
    return np.nonzero(keep)[0]


def witness_bases(c, rounds=MR_ROUNDS):
    """Bases of the extra rounds: 2 + (SHA-256("fsdkr-mr" | c | j | ctr) stream mod (c - 3))."""
    nb = (c.bit_length() + 7) // 8
    cb = c.to_bytes(nb, "big")
    out = []
    for j in range(rounds):
        stream = b""
        ctr = 0
        while len(stream) < nb + 8:
            stream += hashlib.sha256(b"fsdkr-mr" + cb + j.to_bytes(4, "little") + ctr.to_bytes(4, "little")).digest()
            ctr += 1
        out.append(2 + int.from_bytes(stream[:nb + 8], "big") % (c - 3))
    return out


def _mr(ctx, cands, bases):
    """One GPU launch per candidate width class."""
    out = [0] * len(cands)
    by_w = {}
    for k, c in enumerate(cands):
        by_w.setdefault(mr_width(c.bit_length()), []).append(k)
    for w, ks in by_w.items():
        v = ctx.miller_rabin([cands[k] for k in ks], [bases[k] for k in ks], w)
        for k, r in zip(ks, v):
            out[k] = r
    return out


class _Walk:
    __slots__ = ("start", "offs", "pos", "passers")

    def __init__(self, start, span):
        self.start = start
        self.offs = sieve(start, span)
        self.pos = 0
        self.passers = []   # base-2 passers of the current window, in walk order


def sample_primes(ctx, rng, bits, count, window=None, span=None):
    """`count` primes of `bits` bits (top two bits set) by independent walks of
    `span` odd candidates (default 4*bits; shorter walks exercise the redraws)."""
    if bits < 64:
        raise ValueError("sample_primes: bits >= 64")
    ctx = _ctx(ctx)
    window = window or max(32, bits // 8)
    span = span or 4 * bits
    draw = lambda: rng.bits(bits) | (3 << (bits - 2)) | 1   # noqa: E731
    walks = [_Walk(draw(), span) for _ in range(count)]
    out = [None] * count
    passes = 0
    while True:
        active = [w for w in range(count) if out[w] is None and walks[w].pos < len(walks[w].offs)]
        if not active:
            failed = [w for w in range(count) if out[w] is None]
            if not failed:
                return out
            passes += 1
            if passes > MAX_PASSES:   # never for a working test (a pass fails w.p. ~1e-5 at 4*bits)
                raise RuntimeError(f"sample_primes: no prime after {MAX_PASSES} walk passes (Miller-Rabin backend?)")
            for w in failed:                       # a new pass, in walk order
                walks[w] = _Walk(draw(), span)
            continue
        # base 2 on the next window of every unsettled walk
        cands, owner = [], []
        for w in active:
            wk = walks[w]
            for k in wk.offs[wk.pos:wk.pos + window]:
                cands.append(wk.start + 2 * int(k))
                owner.append(w)
            wk.pos += window
        v2 = _mr(ctx, cands, [2] * len(cands))
        for c, w, ok in zip(cands, owner, v2):
            if ok:
                walks[w].passers.append(c)
        # extra rounds on each walk's first passer; a failure tries the next
        while True:
            head = [w for w in active if walks[w].passers and out[w] is None]
            if not head:
                break
            cands, owner, bases = [], [], []
            for w in head:
                c = walks[w].passers[0]
                for b in witness_bases(c):
                    cands.append(c)
                    owner.append(w)
                    bases.append(b)
            v = _mr(ctx, cands, bases)
            verdict = {}
            for w, ok in zip(owner, v):
                verdict[w] = verdict.get(w, True) and bool(ok)
            for w in head:
                c = walks[w].passers.pop(0)
                if verdict[w]:
                    out[w] = c
                    walks[w].passers = []


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
