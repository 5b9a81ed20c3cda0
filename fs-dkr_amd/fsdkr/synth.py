"""Seeded synthetic collect() workloads for benchmarks, generated with the GPU
engine (a batched restatement of the prover side of distribute(),
refresh_message.rs:51-145, zk_pdl_with_slack.rs:53-111, range_proofs.rs:168-202,
ring_pedersen_proof.rs:48-124, add_party_message.rs:50-124).

Every exponentiation (prime tests, encryptions, commitments, proof responses,
ring-Pedersen A_i, correct-key sigma_j, composite-DLog x) runs through
Context.modexp_batch; every scalar multiplication through Context.ec_msm.
Randomness is a seeded PRNG (synthetic data, not a production prover); the
statistical shapes follow the reference's samplers."""
import hashlib
import math
import random

from .types import (AliceProof, CompositeDLogProof, DecryptionKey, DLogStatement, EncryptionKey, JoinMessage,
                    LocalKey, NiCorrectKeyProof, PDLwSlackProof, RefreshMessage, RingPedersenProof,
                    RingPedersenStatement, VerifiableSS)

Q = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
GX = 0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798
GY = 0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8
G = (GX, GY)
SALT = bytes([75, 90, 101, 110])
M2 = 11


def to_bytes(v):
    v = abs(v)
    return v.to_bytes(max(1, (v.bit_length() + 7) // 8), "big")


def H(*vals):
    h = hashlib.sha256()
    for v in vals:
        h.update(to_bytes(v))
    return int.from_bytes(h.digest(), "big")


def compressed(pt):
    if pt is None:
        return 0
    return int.from_bytes(bytes([2 + (pt[1] & 1)]) + pt[0].to_bytes(32, "big"), "big")


def _width(bits):
    for w in (64, 96, 128, 192):
        if bits <= 32 * w:
            return w
    raise ValueError(bits)


class Batch:
    """Collects modexp requests and runs them in as few GPU launches as possible."""

    def __init__(self, ctx):
        self.ctx = ctx
        self.req = []

    def add(self, b, e, m):
        self.req.append((b, e, m))
        return len(self.req) - 1

    def run(self):
        """Launch per (modulus width, exponent-length class); classes double in
        size so a launch never pays more than ~2x for its shortest exponent."""
        out = [None] * len(self.req)
        groups = {}
        for k, (b, e, m) in enumerate(self.req):
            cls = max(6, e.bit_length()).bit_length()
            groups.setdefault((_width(m.bit_length()), cls), []).append(k)
        for (w, _), ks in sorted(groups.items()):
            mods, midx, ix = [], [], {}
            for k in ks:
                m = self.req[k][2]
                if m not in ix:
                    ix[m] = len(mods)
                    mods.append(m)
                midx.append(ix[m])
            bases = [self.req[k][0] if self.req[k][0].bit_length() <= 32 * w else self.req[k][0] % self.req[k][2]
                     for k in ks]
            res = self.ctx.modexp_batch(bases, [self.req[k][1] for k in ks], mods, midx, w)
            for k, r in zip(ks, res):
                out[k] = r
        self.req = []
        return out


_SIEVE = None


def _primorial_16():
    """Product of the odd primes below 2^12: a gcd against it drops 87 % of odd
    candidates for 0.02 ms each (the 2^16 primorial drops 90 % for 0.27 ms: the
    n = 256 workload's 52 k candidates took 14 s of host time)."""
    global _SIEVE
    if _SIEVE is None:
        n = 1 << 12
        flags = bytearray([1]) * n
        flags[0:2] = b"\x00\x00"
        for i in range(2, int(n ** 0.5) + 1):
            if flags[i]:
                flags[i * i::i] = bytearray(len(flags[i * i::i]))
        p = 1
        for i in range(3, n):
            if flags[i]:
                p *= i
        _SIEVE = p
    return _SIEVE


def gen_primes(ctx, count, bits, rnd):
    """`count` distinct `bits`-bit primes (top two bits set): CPU gcd sieve,
    then Fermat tests to bases 2 and 3 as one GPU batch each."""
    prim = _primorial_16()
    out = []
    while len(out) < count:
        need = count - len(out)
        cands = []
        while len(cands) < need * 48:
            c = rnd.getrandbits(bits) | (3 << (bits - 2)) | 1
            if math.gcd(c, prim) == 1:
                cands.append(c)
        r2 = ctx.modexp_batch([2] * len(cands), [c - 1 for c in cands], cands, list(range(len(cands))),
                              _width(bits))
        surv = [c for c, r in zip(cands, r2) if r == 1]
        if not surv:
            continue
        r3 = ctx.modexp_batch([3] * len(surv), [c - 1 for c in surv], surv, list(range(len(surv))), _width(bits))
        for c, r in zip(surv, r3):
            if r == 1 and c not in out:
                out.append(c)
    return out[:count]


def _keypairs(primes):
    it = iter(primes)
    out = []
    for p in it:
        q = next(it)
        out.append((p, q, p * q))
    return out


def _mask(key_len, seed):
    msklen = key_len // 256 + 1
    return sum(H(seed, j) << (256 * j) for j in range(msklen))


def synth_collect_tiled(ctx, R, t, seed, unique, key_bits=2048, M=256):
    """A collect() batch of R refresh messages (no joins) over n = R receivers
    built from `unique` distinct messages: message k is a copy of message
    k mod unique under party index k+1.  Every copy is a valid message (its
    proofs are for the same receivers) and the verifier recomputes every pair
    independently, so the verification work equals that of R distinct
    messages; only the prover-side generation (CPU/GPU minutes at n = 256) is
    saved.  Used for the n = 256 measurement (BASELINE configs[3])."""
    import dataclasses
    msgs, joins, lk = synth_collect(ctx, unique, 0, t, seed, key_bits, M, n_recv=R)
    tiled = [dataclasses.replace(msgs[k % unique], party_index=k + 1, old_party_index=k + 1) for k in range(R)]
    return tiled, joins, lk


def _drive(B, gens):
    """Run session generators in lockstep: each yields when it needs the shared
    Batch run; one GPU pass serves every session's requests."""
    outs = [None] * len(gens)
    alive = {}
    for k, g in enumerate(gens):
        try:
            next(g)
            alive[k] = g
        except StopIteration as e:
            outs[k] = e.value
    while alive:
        res = B.run()
        nxt = {}
        for k, g in alive.items():
            try:
                g.send(res)
                nxt[k] = g
            except StopIteration as e:
                outs[k] = e.value
        alive = nxt
    return outs


def synth_collect(ctx, R, J, t, seed, key_bits=2048, M=256, n_recv=None):
    """Messages for one collect() with R refresh and J join messages (n = R+J
    receivers, or n_recv when J = 0): returns (refresh_messages,
    join_messages, local_key of party 1).  Party k (1-based) of the refresh set
    has party_index = old_party_index = k; joiners take indices R+1..n (the
    replace() layout)."""
    rnd = random.Random(seed)
    assert n_recv is None or J == 0
    n = n_recv or (R + J)
    Mt = R + J
    nk = 2 * n + 2 * Mt                     # receivers: Paillier + N~; messages: new ek + RP key
    kp = _keypairs(gen_primes(ctx, 2 * nk, key_bits // 2, rnd))
    B = Batch(ctx)
    return _drive(B, [_session(ctx, B, R, J, t, rnd, n, kp, M)])[0][:3]


def synth_sessions(ctx, count, n=3, t=1, seed=0, key_bits=3072, M=256):
    """`count` independent collect() sessions (BASELINE configs[4]: custody
    wallets, t=1 n=3, 3072-bit keys), generated in lockstep so each GPU pass
    serves all sessions.  Keys are products of distinct prime PAIRS drawn from a
    shared pool (every modulus distinct; the verifier's work is that of
    independent keys).  Returns [(refresh_messages, join_messages, local_key of
    party 1, a fresh DecryptionKey for collect's new_dk)]."""
    rnd = random.Random(seed)
    per = 2 * n + 2 * n                     # keys per session
    need = per * count
    pool = 16
    while pool * (pool - 1) // 2 < need + need // 4:
        pool += 16
    primes = gen_primes(ctx, pool, key_bits // 2, rnd)
    pairs = set()
    keys = []
    while len(keys) < need:
        a, b = rnd.sample(range(pool), 2)
        if (min(a, b), max(a, b)) in pairs:
            continue
        pairs.add((min(a, b), max(a, b)))
        p, q = primes[a], primes[b]
        keys.append((p, q, p * q))
    B = Batch(ctx)
    gens = [_session(ctx, B, n, 0, t, random.Random(rnd.getrandbits(64)), n, keys[s * per:(s + 1) * per], M)
            for s in range(count)]
    out = _drive(B, gens)
    return [(m, j, lk, dk) for (m, j, lk, dk) in out]


def _session(ctx, B, R, J, t, rnd, n, kp, M):
    """Generator body of one session (yields where the shared Batch must run)."""
    Mt = R + J
    recv_kp, nt_kp = kp[:n], kp[n:2 * n]
    ek_kp, rp_kp = kp[2 * n:2 * n + Mt], kp[2 * n + Mt:2 * n + 2 * Mt]
    # ---- receivers' DLog statements (generate_h1_h2_n_tilde, add_party_message.rs:50-66)
    h1s, xhis, xinvs = [], [], []
    for (p, q, Nt) in nt_kp:
        phi = (p - 1) * (q - 1)
        h1s.append(rnd.randrange(Nt))
        while True:
            x = rnd.randrange(phi)
            if math.gcd(x, phi) == 1:
                break
        xhis.append(x)
        xinvs.append(pow(x, -1, phi))
    h2_h = [B.add(h1s[i], xhis[i], nt_kp[i][2]) for i in range(n)]
    # ---- Feldman sharing of each refresh party's old share
    shares, coeffs = [], []
    for k in range(R):
        a = [rnd.randrange(Q) for _ in range(t + 1)]
        coeffs.append(a)
        shares.append([sum(a[j] * pow(i + 1, j, Q) for j in range(t + 1)) % Q for i in range(n)])
    # ---- per pair randomness (zk_pdl_with_slack.rs:54-62, range_proofs.rs:54-57)
    q3 = Q ** 3
    pr = {}
    for k in range(R):
        for i in range(n):
            N = recv_kp[i][2]
            Nt = nt_kp[i][2]
            d = dict(r=rnd.randrange(N), alpha=rnd.randrange(q3), beta=rnd.randrange(1, N - 1),
                     rho=rnd.randrange(Q * Nt), gamma=rnd.randrange(q3 * Nt), aalpha=rnd.randrange(q3),
                     abeta=rnd.randrange(1, N), agamma=rnd.randrange(q3 * Nt), arho=rnd.randrange(Q * Nt))
            NN = N * N
            h1, h2 = h1s[i], None
            s = shares[k][i]
            d["rN"] = B.add(d["r"], N, NN)
            d["h1x"] = B.add(h1, s, Nt)
            d["h1a"] = B.add(h1, d["alpha"], Nt)
            d["bN"] = B.add(d["beta"], N, NN)
            d["ah1a"] = B.add(h1, d["aalpha"], Nt)
            d["abN"] = B.add(d["abeta"], N, NN)
            pr[k, i] = d
    # ---- ring-Pedersen statements + correct-key sigma (need fresh keys only)
    rp = []
    for m in range(Mt):
        p, q, N = rp_kp[m]
        phi = (p - 1) * (q - 1)
        r = rnd.randrange(N)
        T = r * r % N
        lam = rnd.randrange(phi)
        rp.append(dict(N=N, phi=phi, T=T, lam=lam, S=B.add(T, lam, N),
                       a=[rnd.randrange(phi) for _ in range(M)]))
        rp[-1]["A"] = [B.add(T, a, N) for a in rp[-1]["a"]]
    # joiners' new ek is their receiver key (replace() writes join_message.ek into
    # paillier_key_vec, refresh_message.rs:299-313)
    new_ek = [ek_kp[m] for m in range(R)] + [recv_kp[R + j] for j in range(J)]
    ck = []
    for m in range(Mt):
        p, q, N = new_ek[m]
        phi = (p - 1) * (q - 1)
        dinv = pow(N, -1, phi)
        rho = [_mask(N.bit_length(), H(N, int.from_bytes(SALT, "big"), j)) % N for j in range(M2)]
        ck.append([B.add(r_, dinv, N) for r_ in rho])
    res = yield
    # h2 depends on round-1 results; second batch: h2^rho, h2^gamma etc.
    h2s = [res[h] for h in h2_h]
    for (k, i), d in pr.items():
        Nt = nt_kp[i][2]
        d["h2r"] = B.add(h2s[i], d["rho"], Nt)
        d["h2g"] = B.add(h2s[i], d["gamma"], Nt)
        d["ah2r"] = B.add(h2s[i], d["arho"], Nt)
        d["ah2g"] = B.add(h2s[i], d["agamma"], Nt)
    res2 = yield
    # ---- EC: committed points, commitments, u1 = G*alpha
    pts_sc = []
    for k in range(R):
        pts_sc += [[s] for s in shares[k]]
    for k in range(R):
        pts_sc += [[a] for a in coeffs[k]]
    for k in range(R):
        pts_sc += [[pr[k, i]["alpha"] % Q] for i in range(n)]   # Scalar::from(alpha) reduces mod q
    ecres = ctx.ec_msm([[G]] * len(pts_sc), pts_sc)
    committed = [ecres[k * n:(k + 1) * n] for k in range(R)]
    off = R * n
    comms = [ecres[off + k * (t + 1): off + (k + 1) * (t + 1)] for k in range(R)]
    off += R * (t + 1)
    u1s = {(k, i): ecres[off + k * n + i] for k in range(R) for i in range(n)}
    # ---- assemble round-1 values, challenges, round-2 exponentiations
    for (k, i), d in pr.items():
        N = recv_kp[i][2]
        NN = N * N
        Nt = nt_kp[i][2]
        s = shares[k][i]
        d["c"] = (s * N + 1) % NN * res[d["rN"]] % NN
        d["z"] = res[d["h1x"]] * res2[d["h2r"]] % Nt
        d["u2"] = (1 + d["alpha"] * N) % NN * res[d["bN"]] % NN
        d["u3"] = res[d["h1a"]] * res2[d["h2g"]] % Nt
        Qp = committed[k][i]
        d["e"] = H(compressed(G), compressed(Qp), d["c"], d["z"], compressed(u1s[k, i]), d["u2"], d["u3"])
        d["az"] = res[d["h1x"]] * res2[d["ah2r"]] % Nt
        d["au"] = (d["aalpha"] * N + 1) * res[d["abN"]] % NN
        d["aw"] = res[d["ah1a"]] * res2[d["ah2g"]] % Nt
        d["ae"] = H(N, N + 1, d["c"], d["az"], d["au"], d["aw"])
        d["re"] = B.add(d["r"], d["e"], N)
        d["rae"] = B.add(d["r"], d["ae"], N)
    # ring-Pedersen challenge bits; redraw a message whose challenge has a leading zero byte
    for m in range(Mt):
        while True:
            A = [res[h] for h in rp[m]["A"]]
            e = H(*A)
            eb = to_bytes(e)
            if 8 * len(eb) >= M:
                break
            rp[m]["a"] = [rnd.randrange(rp[m]["phi"]) for _ in range(M)]
            tmp = Batch(ctx)
            hs = [tmp.add(rp[m]["T"], a, rp[m]["N"]) for a in rp[m]["a"]]
            out = tmp.run()
            for j, h in enumerate(rp[m]["A"]):
                res[h] = out[hs[j]]
        bits = [(eb[j >> 3] >> (j & 7)) & 1 for j in range(M)]
        rp[m]["Av"] = A
        rp[m]["Z"] = [(rp[m]["a"][j] + bits[j] * rp[m]["lam"]) % rp[m]["phi"] for j in range(M)]
    # joiners' DLog statements + composite proofs (add_party_message.rs:69-92)
    jd = []
    for j in range(J):
        i = R + j
        Nt = nt_kp[i][2]
        phi = (nt_kp[i][0] - 1) * (nt_kp[i][1] - 1)
        xs, xi = phi - xhis[i], phi - xinvs[i]
        st1 = DLogStatement(Nt, h1s[i], h2s[i])
        st2 = DLogStatement(Nt, h2s[i], h1s[i])
        r1 = rnd.randrange((1 << 512) * Nt)
        r2 = rnd.randrange((1 << 512) * Nt)
        jd.append(dict(st1=st1, st2=st2, sec1=xs, sec2=xi, r1=r1, r2=r2, x1=B.add(st1.g, r1, Nt),
                       x2=B.add(st2.g, r2, Nt)))
    res3 = yield
    # ---- build messages
    msgs = []
    for k in range(R):
        pdl, rng_ = [], []
        for i in range(n):
            d = pr[k, i]
            N = recv_kp[i][2]
            s = shares[k][i]
            pdl.append(PDLwSlackProof(z=d["z"], u1=u1s[k, i], u2=d["u2"], u3=d["u3"], s1=d["e"] * s + d["alpha"],
                                      s2=res3[d["re"]] * d["beta"] % N, s3=d["e"] * d["rho"] + d["gamma"]))
            rng_.append(AliceProof(z=d["az"], e=d["ae"], s=res3[d["rae"]] * d["abeta"] % N,
                                   s1=d["ae"] * s + d["aalpha"], s2=d["ae"] * d["arho"] + d["agamma"]))
        p, q, Nek = ek_kp[k]
        rpm = rp[k]
        msgs.append(RefreshMessage(
            old_party_index=k + 1, party_index=k + 1, pdl_proof_vec=pdl, range_proofs=rng_,
            coefficients_committed_vec=VerifiableSS(t, n, comms[k]), points_committed_vec=committed[k],
            points_encrypted_vec=[pr[k, i]["c"] for i in range(n)],
            dk_correctness_proof=NiCorrectKeyProof(tuple(res[h] for h in ck[k])),
            dlog_statement=DLogStatement(nt_kp[k][2], h1s[k], h2s[k]), ek=EncryptionKey(Nek, Nek * Nek),
            remove_party_indices=[], public_key=None,
            ring_pedersen_statement=RingPedersenStatement(res[rpm["S"]], rpm["T"], rpm["N"], rpm["phi"],
                                                          EncryptionKey(rpm["N"], rpm["N"] ** 2)),
            ring_pedersen_proof=RingPedersenProof(tuple(rpm["Av"]), tuple(rpm["Z"]))))
    joins = []
    for j in range(J):
        m = R + j
        d = jd[j]
        Nt = d["st1"].N
        x1, x2 = res3[d["x1"]], res3[d["x2"]]
        e1 = H(x1, d["st1"].g, Nt, d["st1"].ni)
        e2 = H(x2, d["st2"].g, Nt, d["st2"].ni)
        p, q, Nek = new_ek[m]
        rpm = rp[m]
        joins.append(JoinMessage(
            ek=EncryptionKey(Nek, Nek * Nek), dk_correctness_proof=NiCorrectKeyProof(tuple(res[h] for h in ck[m])),
            party_index=m + 1, dlog_statement=d["st1"],
            composite_dlog_proof_base_h1=CompositeDLogProof(x1, d["r1"] + e1 * d["sec1"]),
            composite_dlog_proof_base_h2=CompositeDLogProof(x2, d["r2"] + e2 * d["sec2"]),
            ring_pedersen_statement=RingPedersenStatement(res[rpm["S"]], rpm["T"], rpm["N"], rpm["phi"],
                                                          EncryptionKey(rpm["N"], rpm["N"] ** 2)),
            ring_pedersen_proof=RingPedersenProof(tuple(rpm["Av"]), tuple(rpm["Z"]))))
    lk = LocalKey(paillier_dk=DecryptionKey(recv_kp[0][0], recv_kp[0][1]), pk_vec=[], x_i=0, y=None,
                  paillier_key_vec=[EncryptionKey(kk[2], kk[2] ** 2) for kk in recv_kp], y_sum_s=None,
                  h1_h2_n_tilde_vec=[DLogStatement(nt_kp[i][2], h1s[i], h2s[i]) for i in range(n)],
                  vss_scheme=VerifiableSS(t, n, []), i=1, t=t, n=n)
    return msgs, joins, lk, DecryptionKey(ek_kp[0][0], ek_kp[0][1])
