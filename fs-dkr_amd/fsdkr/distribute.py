"""Host-side mirror of RefreshMessage::distribute (/root/reference/src/refresh_message.rs:51-145)
on the MI355X engine: the prover side of the refresh and
job 1 (Paillier encryption of the new shares, :72-84).

Every exponentiation runs on the GPU in a few batched launches:
  round 1  job-1 encryptions (fsdkr_paillier_encrypt); the PDL / Alice
           commitments h1^x h2^rho, h1^alpha h2^gamma mod N~ and beta^N mod N^2
           (fsdkr_modexp_batch); G*share, G*a_k, G*alpha (fsdkr_ec_msm)
  round 2  r^e mod N for the PDL s2 and Alice s responses (after the challenges)
  keys     Paillier / ring-Pedersen moduli by the batched GPU Miller-Rabin prime
           walk (fsdkr/keygen.py), correct-key sigma_j = rho_j^(N^-1 mod phi),
           ring-Pedersen A_i = T^a_i.
Every exponentiation with a secret exponent (alpha, gamma, rho, the share x,
a_i, lambda, xhi, N^-1 mod phi, the DLog proof's r) runs through the
regular-access kernel (fsdkr_modexp_batch_ct: no exponent-dependent addresses).
Hashes, small-number arithmetic and the order of random draws are host work.

Randomness is injected: `rng` provides sample_below(n) and bits(k) (the
reference draws from the OS RNG through curv; SystemRng below is the
production default).  With the same draws this produces the oracle's
transcript bit for bit (tests/test_distribute_gpu.py).  Prime generation
follows the restated key generation of the oracle (a random start with the
top two bits set, then the next probable prime within 4*bits odd steps);
kzen-paillier's own keygen is a dependency whose output cannot be matched
without its RNG (parity unpinned)."""
import hashlib
import math
import secrets

from .refresh import GX, GY, Q, FsDkrError, FsDkrPanic, _ctx
from .types import (AliceProof, DecryptionKey, EncryptionKey, NiCorrectKeyProof, PDLwSlackProof, RefreshMessage,
                    RingPedersenProof, RingPedersenStatement, VerifiableSS)



class SystemRng:
    """OS randomness with the sampler interface the reference uses
    (curv BigInt::sample_below: rejection on bit length)."""

    def bits(self, k):
        return secrets.randbits(k) if k > 0 else 0

    def sample_below(self, upper):
        if upper <= 0:
            raise FsDkrPanic("sample_below: upper must be positive")
        k = upper.bit_length()
        while True:
            x = self.bits(k)
            if x < upper:
                return x


# ---------------------------------------------------------------- encodings ----
def _to_bytes(v):
    v = abs(v)
    return v.to_bytes(max(1, (v.bit_length() + 7) // 8), "big")


def chain_bigint(*vals):
    """curv DigestExt::chain_bigint / result_bigint with H = SHA-256."""
    h = hashlib.sha256()
    for v in vals:
        h.update(_to_bytes(v))
    return int.from_bytes(h.digest(), "big")


def _compressed(pt):
    if pt is None:
        return 0
    return int.from_bytes(bytes([2 + (pt[1] & 1)]) + pt[0].to_bytes(32, "big"), "big")


def _width(bits):
    for w in (64, 96, 128, 192):
        if bits <= 32 * w:
            return w
    raise ValueError(f"{bits}-bit modulus")


def _sample_range(rng, lo, hi):
    return lo + rng.sample_below(hi - lo)


def _from_modulo(rng, n):
    """SampleFromMultiplicativeGroup::from_modulo (range_proofs.rs:599-607)."""
    while True:
        r = rng.sample_below(n)
        if math.gcd(r, n) == 1:
            return r


# ---------------------------------------------------------- key generation ----
# Paillier keys, primes and correct-key proofs come from the batched key
# generation (fsdkr/keygen.py: GPU Miller-Rabin over the oracle's prime walk).
from .keygen import correct_key_rho, keypair_with_modulus_size, prime  # noqa: E402,F401
from .keygen import correct_key_proofs  # noqa: E402


def correct_key_proof(ctx, dk):
    """NiCorrectKeyProof::proof (refresh_message.rs:119): sigma_j = rho_j^(n^-1 mod phi) mod n."""
    return correct_key_proofs(ctx, [dk])[0]


def ring_pedersen_generate_and_prove(ctx, rng, key_bits, M):
    """RingPedersenStatement::generate + RingPedersenProof::prove (refresh_message.rs:121-124,
    ring_pedersen_proof.rs:48-124).  A challenge with a leading zero byte makes the
    reference prover panic (BitVec index); as in the oracle the statement is redrawn."""
    while True:
        ek, dk = keypair_with_modulus_size(ctx, rng, key_bits)
        N = ek.n
        phi = (dk.p - 1) * (dk.q - 1)
        r = rng.sample_below(N)
        lam = rng.sample_below(phi)
        T = r * r % N
        w = _width(N.bit_length())
        S = ctx.modexp_batch([T], [lam], [N], [0], w, secret=True)[0]
        a = [rng.sample_below(phi) for _ in range(M)]
        # secret a_i: the regular-access modexp (the fixed-base engine's digit sort
        # would order memory accesses by the exponent digits)
        A = ctx.modexp_batch([T] * M, a, [N], [0] * M, w, secret=True)
        eb = _to_bytes(chain_bigint(*A))
        if 8 * len(eb) < M:
            continue
        bits = [(eb[i >> 3] >> (i & 7)) & 1 for i in range(M)]
        Z = tuple((a[i] + bits[i] * lam) % phi for i in range(M))
        return RingPedersenStatement(S, T, N, phi, ek), RingPedersenProof(tuple(A), Z)


# -------------------------------------------------------------- distribute ----
def vss_share(ctx, t, n, secret, rng):
    """VerifiableSS::share (curv feldman_vss [dep]): degree-t polynomial with
    constant term `secret`, a non-zero top coefficient; shares f(1..n)."""
    if not t < n:
        raise FsDkrPanic("VerifiableSS::share: t < n")
    coeffs = [secret % Q] + [rng.sample_below(Q) for _ in range(t)]
    while t > 0 and coeffs[-1] == 0:
        coeffs[-1] = rng.sample_below(Q)
    shares = []
    for i in range(1, n + 1):
        acc = 0
        for c in reversed(coeffs):
            acc = (acc * i + c) % Q
        shares.append(acc)
    return coeffs, shares


def distribute(old_party_index, local_key, new_n, rng=None, ctx=None, key_bits=2048, m_security=256,
               randomness=None):
    """RefreshMessage::distribute (refresh_message.rs:51-145) -> (RefreshMessage, DecryptionKey).
    Rewrites local_key.vss_scheme as the reference does (:62-64).  `randomness`
    optionally fixes the Paillier r_i of :74 (encrypt_with_chosen_randomness)."""
    ctx = _ctx(ctx)
    rng = rng or SystemRng()
    t = local_key.t
    if not t <= new_n // 2:                                            # :56
        raise FsDkrPanic("distribute: assert!(t <= new_n / 2)")
    if new_n <= t:                                                     # :58-60
        raise FsDkrError("NewPartyUnassignedIndexError")
    coeffs, shares = vss_share(ctx, t, new_n, local_key.x_i, rng)     # :62
    n = len(shares)
    eks = local_key.paillier_key_vec[:n]
    sts = local_key.h1_h2_n_tilde_vec[:n]
    # ---- draws, in the reference's order: r_i (:74), PDL proofs (:86-98), Alice proofs (:100-112)
    rs = [randomness[i] if randomness is not None else rng.sample_below(eks[i].n) for i in range(n)]
    q3 = Q ** 3
    pd = []
    for i in range(n):
        Nt = sts[i].N
        pd.append(dict(alpha=rng.sample_below(q3), beta=_sample_range(rng, 1, eks[i].n - 1),
                       rho=rng.sample_below(Q * Nt), gamma=rng.sample_below(q3 * Nt)))
    ad = []
    for i in range(n):
        Nt = sts[i].N
        alpha = rng.sample_below(q3)
        beta = _from_modulo(rng, eks[i].n)
        gamma = rng.sample_below(q3 * Nt)
        ro = rng.sample_below(Q * Nt)
        ad.append(dict(alpha=alpha, beta=beta, gamma=gamma, ro=ro))
    # ---- round 1 on the GPU
    wN = _width(max(max(e.n.bit_length() for e in eks), max(s.N.bit_length() for s in sts)))
    enc = ctx.paillier_encrypt(shares, rs, [e.n for e in eks], list(range(n)), wN)       # job 1, :72-84
    bases, exps, mods = [], [], []
    for i in range(n):
        h1, h2, Nt = sts[i].g, sts[i].ni, sts[i].N
        for b, e in ((h1, shares[i]), (h2, pd[i]["rho"]), (h1, pd[i]["alpha"]), (h2, pd[i]["gamma"]),
                     (h1, shares[i]), (h2, ad[i]["ro"]), (h1, ad[i]["alpha"]), (h2, ad[i]["gamma"])):
            bases.append(b)
            exps.append(e)
            mods.append(Nt)
    nt = ctx.modexp_batch(bases, exps, mods, list(range(len(mods))), wN, secret=True)
    bn = ctx.modexp_batch([pd[i]["beta"] for i in range(n)] + [ad[i]["beta"] for i in range(n)],
                          [eks[i].n for i in range(n)] * 2, [eks[i].nn for i in range(n)] * 2,
                          list(range(2 * n)), 2 * wN)
    G = (GX, GY)
    pts = [[G] for _ in range(n + len(coeffs) + n)]
    scs = [[s] for s in shares] + [[c] for c in coeffs] + [[pd[i]["alpha"] % Q] for i in range(n)]
    ecr = ctx.ec_msm(pts, scs)
    committed, comms, u1s = ecr[:n], ecr[n:n + len(coeffs)], ecr[n + len(coeffs):]
    # ---- challenges (host), round 2 on the GPU
    e_pdl, e_al = [], []
    for i in range(n):
        N, NN, Nt = eks[i].n, eks[i].nn, sts[i].N
        x8 = nt[8 * i:8 * i + 8]
        d = pd[i]
        d["z"] = x8[0] * x8[1] % Nt                                    # zk_pdl_with_slack.rs:63-69
        d["u2"] = (1 + d["alpha"] * N) % NN * bn[i] % NN               # :71-77 ((N+1)^alpha = 1 + alpha N)
        d["u3"] = x8[2] * x8[3] % Nt                                   # :78-84
        d["e"] = chain_bigint(_compressed(G), _compressed(committed[i]), enc[i], d["z"],
                              _compressed(u1s[i]), d["u2"], d["u3"])
        a = ad[i]
        a["z"] = x8[4] * x8[5] % Nt                                    # range_proofs.rs:58-64
        a["u"] = (a["alpha"] * N + 1) * bn[n + i] % NN                 # :65-67
        a["w"] = x8[6] * x8[7] % Nt                                    # :68-72
        a["e"] = chain_bigint(N, N + 1, enc[i], a["z"], a["u"], a["w"])  # :183-190
        e_pdl.append(d["e"])
        e_al.append(a["e"])
    re = ctx.modexp_batch(rs + rs, e_pdl + e_al, [e.n for e in eks], list(range(n)) * 2, wN)
    pdl_vec, rng_vec = [], []
    for i in range(n):
        N = eks[i].n
        d, a = pd[i], ad[i]
        pdl_vec.append(PDLwSlackProof(z=d["z"], u1=u1s[i], u2=d["u2"], u3=d["u3"], s1=d["e"] * shares[i] + d["alpha"],
                                      s2=re[i] * d["beta"] % N, s3=d["e"] * d["rho"] + d["gamma"]))
        rng_vec.append(AliceProof(z=a["z"], e=a["e"], s=re[n + i] * a["beta"] % N, s1=a["e"] * shares[i] + a["alpha"],
                                  s2=a["e"] * a["ro"] + a["gamma"]))
    vss = VerifiableSS(threshold=t, share_count=new_n, commitments=list(comms))
    local_key.vss_scheme = VerifiableSS(threshold=t, share_count=new_n, commitments=list(comms))
    # ---- the party's new Paillier key, its correctness proof, ring-Pedersen (:118-124)
    ek, dk = keypair_with_modulus_size(ctx, rng, key_bits)
    ck = correct_key_proof(ctx, dk)
    rp_st, rp_pf = ring_pedersen_generate_and_prove(ctx, rng, key_bits, m_security)
    msg = RefreshMessage(old_party_index=old_party_index, party_index=local_key.i, pdl_proof_vec=pdl_vec,
                         range_proofs=rng_vec, coefficients_committed_vec=vss, points_committed_vec=list(committed),
                         points_encrypted_vec=list(enc), dk_correctness_proof=ck,
                         dlog_statement=local_key.h1_h2_n_tilde_vec[local_key.i - 1], ek=ek,
                         remove_party_indices=[], public_key=local_key.y_sum_s,
                         ring_pedersen_statement=rp_st, ring_pedersen_proof=rp_pf)
    return msg, dk


# ------------------------------------------------------------ join / replace ----
def generate_h1_h2_n_tilde(ctx, rng, key_bits):
    """add_party_message.rs:50-66: a fresh modulus N~ with h2 = h1^xhi, returns
    (N~, h1, h2, xhi, xhi_inv) with the reference's final negation mod phi."""
    ek, dk = keypair_with_modulus_size(ctx, rng, key_bits)
    phi = (dk.p - 1) * (dk.q - 1)
    h1 = rng.sample_below(ek.n)
    while True:
        xhi = rng.sample_below(phi)
        if math.gcd(xhi, phi) == 1:
            xhi_inv = pow(xhi, -1, phi)
            break
    h2 = ctx.modexp_batch([h1], [xhi], [ek.n], [0], _width(ek.n.bit_length()), secret=True)[0]
    return ek.n, h1, h2, phi - xhi, phi - xhi_inv


def join_distribute(rng=None, ctx=None, key_bits=2048, m_security=256):
    """JoinMessage::distribute (add_party_message.rs:101-124) -> (JoinMessage, Keys)."""
    from .types import DLogStatement, JoinMessage, Keys
    ctx = _ctx(ctx)
    rng = rng or SystemRng()
    ek, dk = keypair_with_modulus_size(ctx, rng, key_bits)
    Nt, h1, h2, xhi, xhi_inv = generate_h1_h2_n_tilde(ctx, rng, key_bits)
    st1, st2 = DLogStatement(Nt, h1, h2), DLogStatement(Nt, h2, h1)
    # the draws of the two composite proofs come one proof at a time in the reference
    p1 = _one_dlog_proof(ctx, rng, st1, xhi)
    p2 = _one_dlog_proof(ctx, rng, st2, xhi_inv)
    rp_st, rp_pf = ring_pedersen_generate_and_prove(ctx, rng, key_bits, m_security)
    msg = JoinMessage(ek=ek, dk_correctness_proof=correct_key_proof(ctx, dk), party_index=None, dlog_statement=st1,
                      composite_dlog_proof_base_h1=p1, composite_dlog_proof_base_h2=p2,
                      ring_pedersen_statement=rp_st, ring_pedersen_proof=rp_pf)
    return msg, Keys(ek, dk)


def _one_dlog_proof(ctx, rng, st, secret):
    from .types import CompositeDLogProof
    r = rng.sample_below((1 << (128 + 128 + 256)) * st.N)
    x = ctx.modexp_batch([st.g], [r], [st.N], [0], _width(st.N.bit_length()), secret=True)[0]
    return CompositeDLogProof(x, r + chain_bigint(x, st.g, st.N, st.ni) * secret)


def replace(join_messages, local_key, old_to_new, new_n, rng=None, ctx=None, key_bits=2048, m_security=256):
    """RefreshMessage::replace (refresh_message.rs:239-319): re-index the
    existing parties' keys by `old_to_new`, insert the joiners' keys, then
    distribute() under the party's new index.  The reference walks a HashMap
    (unspecified order); new indices are applied in ascending order here."""
    current_len = len(local_key.paillier_key_vec)
    remap = {old_to_new[old]: (local_key.paillier_key_vec[old - 1], local_key.h1_h2_n_tilde_vec[old - 1])
             for old in old_to_new}
    for new in sorted(remap):
        if new <= current_len:
            local_key.paillier_key_vec[new - 1], local_key.h1_h2_n_tilde_vec[new - 1] = remap[new]
        else:
            local_key.paillier_key_vec.insert(new - 1, remap[new][0])
            local_key.h1_h2_n_tilde_vec.insert(new - 1, remap[new][1])
    for jm in join_messages:
        if jm.party_index is None:
            raise FsDkrError("NewPartyUnassignedIndexError")
        pi = jm.party_index
        if pi <= current_len:
            local_key.paillier_key_vec[pi - 1] = jm.ek
            local_key.h1_h2_n_tilde_vec[pi - 1] = jm.dlog_statement
        else:
            local_key.paillier_key_vec.insert(pi - 1, jm.ek)
            local_key.h1_h2_n_tilde_vec.insert(pi - 1, jm.dlog_statement)
    old_party_index = local_key.i
    local_key.i = old_to_new[local_key.i]
    local_key.n = new_n
    return distribute(old_party_index, local_key, new_n, rng, ctx, key_bits, m_security)
