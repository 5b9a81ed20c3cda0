"""Batching layer: gathers the n x n proof instances of a collect() call into
the SoA little-endian limb buffers of `struct fsdkr_collect_batch`
(include/fsdkr/fsdkr.h).

North star job (4) places this layer in the Rust crate; with no Rust
toolchain in this image it is restated here and reads the reference's message
structures by field name (refresh_message.rs:31-48, add_party_message.rs:36-45,
zk_pdl_with_slack.rs:41-50, range_proofs.rs:101-108,
ring_pedersen_proof.rs:30-38,79-84).  Any object with those attributes works.

Shapes the reference accepts and the kernels represent per instance (instead
of rejecting the whole batch): commitment vectors of any length (Horner over
each message's own vector, refresh_message.rs:180-182), range_proofs / A / Z /
sigma_vec shorter than the loops index (the reference's index panic at that
check), a LocalKey with fewer keys than receivers (panic at the first pair
past them, :334-339), an ek.n wider than the batch's moduli (its correct-key
proof runs at its own width before ModuliTooSmall, :376-391), and negative
BigInts where the reference's outcome for that instance is a panic, an error,
a plain residue, an h2^-1 exponent or a hashed-and-reduced value (_Negatives:
PDL s1 / u2 / u3 / s2 / s3 / z, Alice s / s1 / s2 / e / z, the ciphertext c,
ring-Pedersen A / Z, DLog x / y).  Still outside the representable set
(UnsupportedInput): negative statement fields (keys, N~, h1, h2, ring-Pedersen
S / T / N, ek.n, sigma) and values wider than 3072 bits in a proof field (6144
bits for ek.n / sigma)."""
import ctypes
import math
import os
import threading
import weakref

import numpy as np

from . import _pack
from ._native import CollectBatchC, ErrorC, VerdictsC, lib

M2 = 11   # zk-paillier NiCorrectKeyProof sigma_vec length
_CK_WIDTHS = (64, 96, 128, 192)
_Q = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141   # secp256k1 group order


class UnsupportedInput(ValueError):
    """Input outside what the C ABI represents (negative BigInts, oversize values)."""


def _limbs_for(bits):
    return max(1, (bits + 31) // 32)


def host_threads():
    """Worker threads of the host gather (FSDKR_HOST_THREADS, else OMP_NUM_THREADS,
    else the visible cores, at most 16 -- the GPU box's CPU share)."""
    for k in ("FSDKR_HOST_THREADS", "OMP_NUM_THREADS"):
        v = os.environ.get(k)
        if v and v.isdigit() and int(v) > 0:
            return min(int(v), 64)
    try:
        cores = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        cores = os.cpu_count() or 1
    return max(1, min(cores, 16))


def _gather(objs, attr=None):
    try:
        return _pack.gather(objs, attr)
    except ValueError as e:
        raise UnsupportedInput(str(e)) from None


def _convert(jobs, threads=1):
    try:
        _pack.convert(jobs, threads)
    except OverflowError as e:
        raise UnsupportedInput(str(e)) from None


def pack_attr(objs, attr, limbs):
    """getattr(o, attr) (attr None: o) of every object -> (len, limbs) uint32,
    little-endian, written in place by the C extension; raises UnsupportedInput
    on negatives / overflow."""
    arr = np.empty((len(objs), limbs), dtype=np.uint32)
    h, _ = _gather(objs, attr)
    _convert([(h, arr, limbs)])
    return arr


def pack(values, limbs):
    """ints -> (len, limbs) uint32, little-endian; raises on negatives / overflow."""
    return pack_attr(values, None, limbs)


def pack_points(points, attr=None):
    """affine (x, y) or None (or their `attr`) -> (len, 16) uint32, (0,0) = infinity."""
    arr = np.empty((len(points), 16), dtype=np.uint32)
    try:
        _pack.points(points, attr, arr)
    except (ValueError, OverflowError) as e:
        raise UnsupportedInput(str(e)) from None
    return arr


class _HostPool:
    """Recycled host arrays for the large SoA slots of a SessionSet.  A configs[4]
    step converts ~0.6 GB of 3072-bit values; writing them into fresh arrays pays
    a first-touch page fault per 4 KiB, a quarter of the conversion on the GPU
    box (31 -> 23 ms, profiles/r03z_pack_host_only.jsonl).  A set's arrays return
    when the set is collected (weakref.finalize), keyed by exact shape, so the
    next call of the same shape reuses them; at most CAP_BYTES are kept."""
    MIN_BYTES = 1 << 20
    CAP_BYTES = 4 << 30

    def __init__(self):
        self._free = {}
        self._bytes = 0
        self._lock = threading.Lock()

    def empty(self, shape):
        shape = tuple(int(x) for x in shape)
        nbytes = int(np.prod(shape)) * 4
        if nbytes >= self.MIN_BYTES:
            with self._lock:
                lst = self._free.get(shape)
                if lst:
                    self._bytes -= nbytes
                    return lst.pop()
        return np.empty(shape, dtype=np.uint32)

    def give(self, arrays):
        with self._lock:
            for a in arrays:
                if a.dtype == np.uint32 and a.nbytes >= self.MIN_BYTES and a.flags.owndata and \
                        self._bytes + a.nbytes <= self.CAP_BYTES:
                    self._free.setdefault(a.shape, []).append(a)
                    self._bytes += a.nbytes


_POOL = _HostPool()


class _Gather:
    """Every big-integer field of one batch: gathered once (max bit lengths for the
    slot widths), converted together on host_threads() workers.  With `owned`
    (a list), the slots come from _POOL and are recorded there for its return."""

    def __init__(self, owned=None):
        self.jobs = []
        self.owned = owned

    def field(self, objs, attr=None):
        return _gather(objs, attr) + (len(objs),)

    def rows(self, objs, attr, take):
        """the first `take` values of every getattr(o, attr), flattened"""
        try:
            h, bits = _pack.gather_rows(objs, attr, take)
        except ValueError as e:
            raise UnsupportedInput(str(e)) from None
        return h, bits, len(objs) * take

    def slot(self, f, limbs):
        if self.owned is None:
            arr = np.empty((f[2], limbs), dtype=np.uint32)
        else:
            arr = _POOL.empty((f[2], limbs))
            self.owned.append(arr)
        self.jobs.append((f[0], arr, limbs))
        return arr

    def run(self):
        jobs, self.jobs = self.jobs, []
        _convert(jobs, host_threads())


def _ptr(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))


class _Negatives:
    """Per-instance outcomes of negative operands:
    the gather of a field that may hold a negative value falls back, only when
    the C gather rejects it, to a Python pass that packs a stand-in row and
    records the instance; decide() derives each instance's rule once the batch
    is gathered, and after the device pass apply() rewrites that
    instance's verdict to the reference's outcome.  The rest of the batch runs
    unchanged.

    Reference semantics (curv BigInt::mod_pow -> GMP mpz_powm: a negative
    exponent panics, a negative base is reduced; to_bytes hashes |v|):
    - PDL (zk_pdl_with_slack.rs:113-167): s1 < 0 panics in h^s1 (u2_test_tmp,
      :139) whatever else holds; u2 / u3 < 0 hash as |u| (the challenge, and so
      u1's check, is unchanged) and can never equal a residue (flag false);
      s2 < 0 is the base of s2^N mod N^2: packed as s2 mod N^2; s3 < 0 raises
      h2^-1 to |s3| (commitment_unknown_order, :177-184): mod_inv(h2).unwrap()
      panics when h2 is not a unit mod N~, else |s3| is packed with the pair's
      pdl_s3_neg flag and the device checks h1^s1 == u3 * z^e * h2^|s3|;
      z < 0 hashes as |z| and is the base of z^e mod N~ (GMP reduces it): |z|
      is packed with the pair's neg_bits bit, the device raises -|z| mod N~;
      the ciphertext c < 0 likewise (bit 2: |c| hashed by both proofs, -|c|
      mod N^2 in c^e, c^-1 and, on the host, the share decryption).
    - Alice (range_proofs.rs:112-164): s1 > q^3 -> false first; e < 0 panics
      in z^e; z^e not invertible -> false; then s1 / s2 < 0 panic in h1^s1 /
      h2^s2; s < 0 is the base of s^N mod N^2 (packed as s mod N^2); z < 0 as
      PDL's z (neg_bits bit 1).
    - ring-Pedersen (ring_pedersen_proof.rs:126-157): Z[i] < 0 panics at
      iteration i, after checks 0..i-1 -- exactly the short-Z mechanism
      (ped_lens: Z "ends" at its first negative entry); A[i] < 0 hashes as
      |A[i]| and mod_mul reduces it: |A[i]| packed with its ped_a_neg flag.
    - composite DLog (zk-paillier, joins :417-424): y < 0 panics in g^y once the
      N > 2^128 and gcd checks pass (else false); proof 2 runs only if proof 1
      holds; x < 0 (hashed as |x|) never equals mod_mul(g^y, ni^e) >= 0: that
      proof is false unless its y panics first.

    Provenance and parity: the sign rules of curv-kzen 0.10 (Cargo.toml:33;
    BigInt::mod_pow / mod_mul / to_bytes over rust-gmp, Cargo.toml:43) and the
    DLog verification order of zk-paillier 0.4.4 (Cargo.toml:32,
    CompositeDLogProof::verify) are restated from those published crates, which
    /root/reference does not vendor.  The GPU outcomes for negative operands are
    checked against the local oracle (oracle/), which encodes the same
    restatement, not against reference-produced fixtures: parity unpinned."""

    def __init__(self):
        self.rows = {}     # field -> rows packed with a stand-in
        self.pdl = {}      # pair -> (or-bits, and-mask)
        self.range = {}    # pair -> verdict (0 false, 2 panic)
        self.dlog = {}     # join -> "y1-panic" | "y1-false" | "y2"
        self.dlogx = {}    # join -> DLog verdict bits a negative x clears (1: proof 1, 2: proof 2)
        self.s3 = None     # [pairs] uint8 pdl_s3_neg flags (None: no negative s3)
        self.z = None      # [pairs] uint8 neg_bits flags: bit 0 PDL z, bit 1 Alice z, bit 2 c
        self.a = None      # [(R+J) * M] uint8 ped_a_neg flags (None: no negative A)

    def __bool__(self):
        return bool(self.rows)

    def field(self, G, name, objs, attr, fix):
        """G.field(objs, attr); a negative value at row k is packed as fix(k, v)"""
        try:
            return G.field(objs, attr)
        except UnsupportedInput:
            vals = [o if attr is None else getattr(o, attr) for o in objs]
            bad = [k for k, v in enumerate(vals) if isinstance(v, int) and v < 0]
            if not bad:
                raise
            for k in bad:
                vals[k] = fix(k, vals[k])
            self.rows[name] = bad
            return G.field(vals)

    def decide(self, msgs, joins, n, avail, pdl, rng, sts):
        """the verdict rules, once every field is gathered"""
        for p in self.rows.get("pdl_s1", ()):
            self.pdl[p] = (8, 0xFF)
        if self.rows.get("pdl_z") or self.rows.get("rp_z") or self.rows.get("enc"):
            self.z = np.zeros(len(pdl), np.uint8)
            for name, bit in (("pdl_z", 1), ("rp_z", 2), ("enc", 4)):
                for p in self.rows.get(name, ()):
                    self.z[p] |= bit
        if self.rows.get("pdl_s3"):
            self.s3 = np.zeros(len(pdl), np.uint8)
            for p in self.rows["pdl_s3"]:
                self.s3[p] = 1
                i = p % n
                if i < avail and math.gcd(sts[i].ni, sts[i].N) != 1:   # mod_inv(h2, N~).unwrap()
                    self.pdl[p] = (8, 0xFF)
        for name, bit in (("pdl_u2", 2), ("pdl_u3", 4)):
            for p in self.rows.get(name, ()):
                o, a = self.pdl.get(p, (0, 0xFF))
                self.pdl[p] = (o, a & ~bit)
        q3 = _Q ** 3
        for p in sorted(set().union(*(self.rows.get(x, ()) for x in ("rp_s1", "rp_s2", "rp_e")))):
            i = p % n
            if i >= avail:          # the pair panics at its statement (refresh_message.rs:334)
                continue
            a = rng[p]
            if a.s1 > q3:
                self.range[p] = 0
            elif a.e < 0:
                self.range[p] = 2
            elif a.e > 0 and math.gcd(a.z, sts[i].N) != 1:
                self.range[p] = 0
            else:                   # s1 or s2 < 0
                self.range[p] = 2
        for name, bit in (("dlog_x1", 1), ("dlog_x2", 2)):   # x < 0 never equals mod_mul(..) >= 0
            for j in self.rows.get(name, ()):
                self.dlogx[j] = self.dlogx.get(j, 0) | bit
        for j in sorted(set(self.rows.get("dlog_y1", ())) | set(self.rows.get("dlog_y2", ()))):
            st = joins[j].dlog_statement
            if joins[j].composite_dlog_proof_base_h1.y < 0:
                pre = st.N > (1 << 128) and math.gcd(st.g, st.N) == 1 and math.gcd(st.ni, st.N) == 1
                self.dlog[j] = "y1-panic" if pre else "y1-false"
            else:
                self.dlog[j] = "y2"

    def apply(self, pdl, rng, dlog):
        """rewrite the device verdicts (this batch's rows) to the reference's outcome"""
        for p, (o, a) in self.pdl.items():
            pdl[p] = (pdl[p] & a) | o
        for p, v in self.range.items():
            rng[p] = v
        for j, bits in self.dlogx.items():   # before the y rules: g^y's panic comes first
            dlog[j] &= ~bits & 0xFF
        for j, rule in self.dlog.items():
            if rule == "y1-panic" or (rule == "y2" and dlog[j] & 1):
                dlog[j] = 4
            elif rule == "y1-false":
                dlog[j] = 0


def _zero(k, v):
    return 0


def _magnitude(k, v):
    return -v


class Verdicts:
    def __init__(self, R, J, n):
        P = R * n
        self.feldman = np.zeros(P, np.uint8)
        self.pdl = np.zeros(P, np.uint8)
        self.range = np.zeros(P, np.uint8)
        self.ped = np.zeros(R + J, np.uint8)
        self.ck = np.zeros(R + J, np.uint8)
        self.dlog = np.zeros(max(J, 1), np.uint8)
        self._bind(P, R + J, J)

    def _bind(self, P, Mt, J):
        u8 = ctypes.POINTER(ctypes.c_uint8)
        arrs = [np.ascontiguousarray(a) for a in (self.feldman, self.pdl, self.range, self.ped, self.ck, self.dlog)]
        self._keep = arrs
        self.c = VerdictsC(*(a.ctypes.data_as(u8) for a in arrs), P, Mt, J)


class CollectBatch:
    """SoA view of (refresh_messages, local_key, join_messages) for one collect().

    `header_only` is set when validate_collect's threshold / size checks fail
    (refresh_message.rs:149-175), or when the caller asks for it (the rank that
    maps all-reduced shard verdicts): then only what fsdkr_collect_first_error
    reads is packed (counts, party indices, lengths, ek.n)."""

    def __init__(self, refresh_messages, local_key, join_messages, m_security=256, key_bits=2048, n_recv=None,
                 header_only=False, staged=False, ck_stage1=False, split_stage1=True):
        """n_recv: receivers (default R + J); a multi-GPU shard passes its slice of the
        messages together with the full receiver count.  staged: pack only the
        fields fsdkr_collect_prestart reads (recv_n, pdl s2, range-proof s; see
        ga_ready) and leave the rest to complete().  ck_stage1: stage 1 also packs
        ek.n and sigma, so the prestart runs the correct-key job beside GA (at
        n = 64 it competed with GA's chains: 56.2 -> 59.0 ms median,
        profiles/r04/r04a_ab_ck_j2j5_v0/v1).  split_stage1: stage 1 packs only
        GA's fields; stage1b() the table bases and exponents (complete() packs
        them if stage1b() never ran)."""
        msgs, joins = list(refresh_messages), list(join_messages)
        R, J = len(msgs), len(joins)
        n = n_recv if n_recv else R + J
        self.R, self.J, self.n = R, J, n
        self._keep = []
        c = CollectBatchC()
        c.n_refresh, c.n_join, c.t, c.m_security, c.key_bits = R, J, local_key.t, m_security, key_bits
        pidx = np.array([m.party_index for m in msgs] + [(j.party_index or 0) for j in joins], dtype=np.uint32)
        lens = np.array([[len(m.pdl_proof_vec), len(m.points_committed_vec), len(m.points_encrypted_vec)]
                         for m in msgs] or [[0, 0, 0]], dtype=np.uint32)
        c.party_index, c.msg_lens = self._k(pidx), self._k(lens)
        c.n_recv = n if n_recv else 0
        self.c = c
        ref = int(lens[0][0]) if R else 0
        self.ref_len = ref
        # the threshold check (refresh_message.rs:149) is about the whole message set: a
        # multi-GPU shard (n_recv given) holds a slice that may be <= t messages
        below_threshold = R <= local_key.t and not n_recv
        self.size_fail = below_threshold or R == 0 or any(tuple(l) != (ref, ref, ref) for l in lens[:R]) or ref < n
        self.header_only = header_only or self.size_fail
        all_m = msgs + joins
        M = m_security
        G = _Gather()
        k = self._k
        self._ga, self._pending, self._stage1b = None, None, None
        self.negs = _Negatives()
        if self.header_only:
            f_ckn = G.field([m.ek.n for m in all_m] or [0])
            ck_bits = max(1, f_ckn[1])
            ckl = next((w for w in _CK_WIDTHS if ck_bits <= 32 * w), None)
            if ckl is None:
                raise UnsupportedInput(f"{ck_bits}-bit Paillier key / correct-key proof")
            c.nl = 64 if ck_bits <= 2048 else 96
            c.ckl = max(ckl, c.nl)
            c.ck_n = k(G.slot(f_ckn, c.ckl))
            G.run()
            self.nl = c.nl
            return
        keys, sts = local_key.paillier_key_vec, local_key.h1_h2_n_tilde_vec
        avail = min(len(keys), len(sts), n)
        c.recv_avail = avail if avail < n else 0
        pdl = [m.pdl_proof_vec[i] for m in msgs for i in range(n)]
        if any(len(m.range_proofs) < n for m in msgs):
            # range_proofs[i] past the vector: placeholder rows, the reference panics there
            c.range_lens = k(np.array([len(m.range_proofs) for m in msgs], dtype=np.uint32))
            rng = [m.range_proofs[i] if i < len(m.range_proofs) else _ZERO_ALICE for m in msgs for i in range(n)]
        else:
            rng = [m.range_proofs[i] for m in msgs for i in range(n)]
        # receivers (placeholders past the keys the LocalKey holds: odd modulus 3)
        rst = list(sts[:avail]) + [None] * (n - avail)
        # gathered first: GA's fields and what sets stage 1's width; every other
        # field is gathered by _rest() (stage1b / complete), after GA has started
        rn = [x.n for x in keys[:avail]] + [3] * (n - avail)
        neg = self.negs

        def residue(k, v):   # a negative base of x^N mod N^2: GMP reduces it
            nn = rn[k % n] ** 2
            return v % nn if nn else 0
        F = {"recv_n": G.field(rn),
             "recv_ntilde": G.field([s.N if s else 3 for s in rst]),
             "recv_h1": G.field([s.g if s else 1 for s in rst]),
             "recv_h2": G.field([s.ni if s else 1 for s in rst]),
             "pdl_s2": neg.field(G, "pdl_s2", pdl, "s2", residue), "rp_s": neg.field(G, "rp_s", rng, "s", residue)}
        for a in ("T", "N"):
            F["ped_" + a] = G.field([m.ring_pedersen_statement for m in all_m], a)
        self._pending = dict(msgs=msgs, joins=joins, all_m=all_m, n=n, M=M, G=G, F=F, pdl=pdl, rng=rng,
                             t=local_key.t, rest=False, avail=avail, sts=sts)
        # stage 1: the fields fsdkr_collect_prestart reads (GA's bases and moduli, the
        # h1/h2 table bases and the exponents that size the tables), at the width they
        # need; stage 2 (complete) keeps them if the batch width agrees
        ga_bits = max(1, *(F[x][1] for x in ("recv_n", "recv_ntilde", "recv_h1", "recv_h2", "pdl_s2", "rp_s",
                                              "ped_T", "ped_N")))
        nl_ga = 64 if ga_bits <= 2048 else 96 if ga_bits <= 3072 else None
        if staged and nl_ga is not None:
            if not split_stage1 or ck_stage1:
                self._rest()   # stage 1 then packs more than GA's own fields
            Gs = _Gather()
            # GA's own fields first when split: GA starts after converting 2Rn + n
            # values instead of every stage-1 field (stage1b() packs the rest; n = 64
            # whole call 0.5-1.2 ms shorter, profiles/r04/r04g_*, r04h_*)
            names = ("recv_n", "pdl_s2", "rp_s") + (() if split_stage1 else _STAGE1B)
            self._stage1b = _STAGE1B if split_stage1 else None
            ga = {name: Gs.slot(F[name], _STAGE1_WIDTH.get(name, lambda c_: nl_ga)(c)) for name in names}
            # the correct-key job (sigma^n mod n) reads only ek.n and sigma: stage 1
            # packs them at the width complete() gives them, so the prestart runs
            # it beside GA (csrc/collect_prestart.cpp prestart_ck)
            st = self._pending
            ck_pre = ck_stage1 and not st["ck_short"] and not split_stage1
            if ck_pre:
                c.ckl = max(st["ckl"], nl_ga)
                ga["ck_n"] = Gs.slot(st["f_ckn"], c.ckl)
                ga["ck_sigma"] = Gs.slot(st["f_sig"], c.ckl)
            Gs.run()
            for name, arr in ga.items():
                setattr(c, name, k(arr))
            c.nl = nl_ga
            self._ga = (nl_ga, ga)
        if not staged:
            self.complete()

    def _rest(self):
        """The gathers stage 1 leaves for later (correct-key widths, the exponents
        and ring-Pedersen vectors): their bit lengths set the slot widths s1l, s3l,
        zl and ckl.  Runs once, from stage1b() or complete()."""
        st = self._pending
        if st is None or st["rest"]:
            return
        st["rest"] = True
        c, k, G, F, M = self.c, self._k, st["G"], st["F"], st["M"]
        all_m, pdl, rng = st["all_m"], st["pdl"], st["rng"]
        f_ckn = G.field([m.ek.n for m in all_m] or [0])
        dkp = [m.dk_correctness_proof for m in all_m]
        ck_short = any(len(d.sigma_vec) < M2 for d in dkp)
        sig = [list(d.sigma_vec[:M2]) for d in dkp] if ck_short else None
        if ck_short:   # short vectors: zero-padded rows (the verdict reports them)
            f_sig = G.field([s for row in sig for s in row + [0] * (M2 - len(row))])
        else:          # the common case: the first M2 of every vector, flattened in C
            f_sig = G.rows(dkp, "sigma_vec", M2)
        ck_bits = max(1, f_ckn[1], f_sig[1])
        ckl = next((w for w in _CK_WIDTHS if ck_bits <= 32 * w), None)
        if ckl is None:
            raise UnsupportedInput(f"{ck_bits}-bit Paillier key / correct-key proof")
        neg = self.negs
        F["pdl_s1"] = neg.field(G, "pdl_s1", pdl, "s1", _zero)
        F["pdl_s3"] = neg.field(G, "pdl_s3", pdl, "s3", _magnitude)
        for a in ("s1", "s2"):
            F["rp_" + a] = neg.field(G, "rp_" + a, rng, a, _zero)
        F["ped_S"] = G.field([m.ring_pedersen_statement for m in all_m], "S")
        rpp = [m.ring_pedersen_proof for m in all_m]
        short = any(len(r.A) < M or len(r.Z) < M for r in rpp)
        a_rows = short
        if not short:   # the first M of every vector, flattened in C
            try:
                F["ped_A"] = G.rows(rpp, "A", M)
            except UnsupportedInput:   # a negative A[i]: |A[i]| with its ped_a_neg flag
                a_rows = True
            try:
                F["ped_Z"] = G.rows(rpp, "Z", M)
            except UnsupportedInput:   # a negative Z[i]: Z "ends" there (see _Negatives)
                short = True
        if a_rows:   # short A vectors or a negative entry: zero-padded |A| rows
            A = [list(r.A[:M]) for r in rpp]
            neg_a = [[1 if isinstance(v, int) and v < 0 else 0 for v in row] + [0] * (M - len(row)) for row in A]
            if any(map(any, neg_a)):
                neg.a = np.array(neg_a, dtype=np.uint8).reshape(-1)
                neg.rows["ped_A"] = [k for k, v in enumerate(neg.a) if v]
            F["ped_A"] = G.field([abs(v) for row in A for v in row + [0] * (M - len(row))])
        if short:   # short vectors (or a negative Z entry): zero-padded rows
            Z = [list(r.Z[:M]) for r in rpp]
            zlen = [next((i for i, v in enumerate(row) if isinstance(v, int) and v < 0), len(row)) for row in Z]
            if any(zl < len(row) for zl, row in zip(zlen, Z)):
                neg.rows["ped_Z"] = [m for m, (zl, row) in enumerate(zip(zlen, Z)) if zl < len(row)]
                Z = [row[:zl] for zl, row in zip(zlen, Z)]
            c.ped_lens = k(np.array([[min(len(r.A), M), zl] for r, zl in zip(rpp, zlen)], dtype=np.uint32))
            F["ped_Z"] = G.field([v for row in Z for v in row + [0] * (M - len(row))])
        c.s1l = _limbs_for(max(F["pdl_s1"][1], F["rp_s1"][1], 1))
        c.s3l = _limbs_for(max(F["pdl_s3"][1], F["rp_s2"][1], 1))
        c.zl = _limbs_for(max(F["ped_Z"][1], 1))
        st.update(ckl=ckl, f_ckn=f_ckn, f_sig=f_sig, ck_short=ck_short, sig=sig)

    def complete(self):
        """Stage 2 of a staged batch (CollectBatch(..., staged=True)): every other field."""
        st = getattr(self, "_pending", None)
        if st is None:
            return self
        self._rest()
        self._pending = None
        c, k = self.c, self._k
        msgs, joins, all_m, n, M, G, F = (st[x] for x in ("msgs", "joins", "all_m", "n", "M", "G", "F"))
        J = len(joins)
        self._late(st)

        def bits(*names):
            return max([1] + [F[x][1] for x in names if x in F])

        one_bits = bits("pdl_z", "pdl_u3", "pdl_s2", "rp_z", "rp_s")
        two_bits = bits("enc", "pdl_u2")
        nl_bits = max(bits("recv_n", "recv_ntilde", "recv_h1", "recv_h2"), bits("ped_N", "ped_S", "ped_T", "ped_A"),
                      bits("dlog_N", "dlog_g", "dlog_ni", "dlog_x1", "dlog_x2"), one_bits, (two_bits + 1) // 2)
        nl = 64 if nl_bits <= 2048 else 96 if nl_bits <= 3072 else None
        if nl is None:
            raise UnsupportedInput(f"{nl_bits}-bit value in a 3072-bit slot")
        c.nl = nl
        c.ckl = max(st["ckl"], nl)
        c.el = _limbs_for(bits("rp_e"))
        c.yl = _limbs_for(bits("dlog_y1", "dlog_y2"))
        width = {"enc": 2 * nl, "pdl_u2": 2 * nl, "pdl_s1": c.s1l, "rp_s1": c.s1l, "pdl_s3": c.s3l, "rp_s2": c.s3l,
                 "rp_e": c.el, "ped_Z": c.zl, "dlog_y1": c.yl, "dlog_y2": c.yl}
        # stage-1 arrays: the nl-wide ones are kept if the batch width agrees, the
        # s1l / s3l-wide ones always (their widths do not depend on nl)
        keep = set()
        if self._ga is not None:
            keep = {x for x in self._ga[1] if self._ga[0] == nl or x in _STAGE1_WIDTH}
            if "rp_e" in keep and self._ga[1]["rp_e"].shape[1] != c.el:
                keep.discard("rp_e")
            for y in ("dlog_y1", "dlog_y2"):
                if y in keep and self._ga[1][y].shape[1] != c.yl:
                    keep.discard(y)
        for name, f in F.items():
            if name not in keep:
                setattr(c, name, k(G.slot(f, width.get(name, nl))))
        ga_arrs = self._ga[1] if self._ga is not None else {}
        if "ck_n" in ga_arrs and ga_arrs["ck_n"].shape[1] == c.ckl:   # stage 1 packed them at this width
            pass
        else:
            c.ck_n = k(G.slot(st["f_ckn"], c.ckl))
            c.ck_sigma = k(G.slot(st["f_sig"], c.ckl))
        if st["ck_short"]:
            c.ck_lens = k(np.array([len(x) for x in st["sig"]], dtype=np.uint32))
        G.run()
        self._points(st)
        if self.negs:
            self.negs.decide(msgs, joins, n, st["avail"], st["pdl"], st["rng"], st["sts"])
            for arr, attr in ((self.negs.s3, "pdl_s3_neg"), (self.negs.z, "neg_bits"), (self.negs.a, "ped_a_neg")):
                if arr is not None:
                    self._keep.append(arr)
                    setattr(c, attr, arr.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
        self.nl = nl
        return self

    def _late(self, st):
        """The gathers of the challenge jobs' fields (PDL transcript, Alice c / z / e,
        DLog proofs): from complete(), once."""
        if st.get("late"):
            return
        st["late"] = True
        F, G, pdl, rng, n = st["F"], st["G"], st["pdl"], st["rng"], st["n"]
        neg = self.negs
        F["enc"] = neg.field(G, "enc", [m.points_encrypted_vec[i] for m in st["msgs"] for i in range(n)], None,
                             _magnitude)
        F["pdl_z"] = neg.field(G, "pdl_z", pdl, "z", _magnitude)
        for a in ("u2", "u3"):
            F["pdl_" + a] = neg.field(G, "pdl_" + a, pdl, a, _magnitude)
        F["rp_z"] = neg.field(G, "rp_z", rng, "z", _magnitude)
        F["rp_e"] = neg.field(G, "rp_e", rng, "e", _zero)
        if st["joins"]:
            for name, attr in (("N", "N"), ("g", "g"), ("ni", "ni")):
                F["dlog_" + name] = G.field([j.dlog_statement for j in st["joins"]], attr)
            for name, which, attr in (("x1", 1, "x"), ("x2", 2, "x"), ("y1", 1, "y"), ("y2", 2, "y")):
                pf = [getattr(j, f"composite_dlog_proof_base_h{which}") for j in st["joins"]]
                F["dlog_" + name] = neg.field(G, "dlog_" + name, pf, attr, _zero)

    def _points(self, st):
        """secp256k1 points: the shares' commitments Q, PDL u1 and the VSS commitments"""
        c, k, n, msgs = self.c, self._k, st["n"], st["msgs"]
        c.commit = k(pack_points([m.points_committed_vec[i] for m in msgs for i in range(n)]))
        c.pdl_u1 = k(pack_points(st["pdl"], "u1"))
        com = [list(m.coefficients_committed_vec.commitments) for m in msgs]
        if any(len(x) != st["t"] + 1 for x in com):   # Horner over each message's own vector
            c.vss_len = k(np.array([len(x) for x in com], dtype=np.uint32))
        c.vss = k(pack_points([p for x in com for p in x] or [None]))

    def stage1b(self):
        """The rest of stage 1 (the fixed-base tables' bases and the exponents
        that size them) when GA's fields went first; True when it packed them
        (fsdkr_collect_prestart may then run again: GA keeps running and the
        tables start)."""
        if not self._stage1b or self._pending is None or self._ga is None:
            return False
        self._rest()
        F, c = self._pending["F"], self.c
        nl_ga, ga = self._ga
        Gs = _Gather()
        for name in self._stage1b:
            ga[name] = Gs.slot(F[name], _STAGE1_WIDTH.get(name, lambda c_: nl_ga)(c))
        Gs.run()
        for name in self._stage1b:
            setattr(c, name, self._k(ga[name]))
        self._stage1b = None
        return True

    @property
    def ga_ready(self):
        """Stage 1 packed the prestart fields (fsdkr_collect_prestart may run)."""
        return self._ga is not None

    def _k(self, arr):
        arr = np.ascontiguousarray(arr, dtype=np.uint32)
        self._keep.append(arr)
        return _ptr(arr)

    def settle(self, verdicts):
        """the device verdicts with the negative-operand instances' outcomes (_Negatives)"""
        if self.negs:
            self.negs.apply(verdicts.pdl, verdicts.range, verdicts.dlog)
        return verdicts

    def first_error(self, verdicts):
        err = ErrorC()
        rc = lib().fsdkr_collect_first_error(ctypes.byref(self.c),
                                             ctypes.byref(verdicts.c) if verdicts is not None else None,
                                             ctypes.byref(err))
        if rc != 0:
            raise RuntimeError(f"fsdkr_collect_first_error failed ({rc})")
        return err


# stage-1 fields after GA's own (recv_n, pdl_s2, rp_s): the fixed-base tables'
# bases and the exponents that size them
_STAGE1B = ("recv_ntilde", "recv_h1", "recv_h2", "ped_T", "ped_N", "pdl_s1", "rp_s1", "pdl_s3", "rp_s2", "ped_Z")

# stage-1 fields whose slot width does not depend on nl
_STAGE1_WIDTH = {"pdl_s1": lambda c: c.s1l, "rp_s1": lambda c: c.s1l, "pdl_s3": lambda c: c.s3l,
                 "rp_s2": lambda c: c.s3l, "ped_Z": lambda c: c.zl}


class _ZeroAlice:
    z = e = s = s1 = s2 = 0


_ZERO_ALICE = _ZeroAlice()


def _struct_dtype(cls):
    """numpy structured dtype with the exact layout of a ctypes Structure (pointers as u8)."""
    names, formats, offsets = [], [], []
    for name, typ in cls._fields_:
        names.append(name)
        formats.append(np.uint64 if ctypes.sizeof(typ) == 8 else np.uint32)
        offsets.append(getattr(cls, name).offset)
    return np.dtype({"names": names, "formats": formats, "offsets": offsets, "itemsize": ctypes.sizeof(cls)})


_BATCH_DT = _struct_dtype(CollectBatchC)
_VERD_DT = _struct_dtype(VerdictsC)


def _has_negative(session):
    """any negative integer among the proof / key fields of one session (the slow
    scan that runs only after a set-wide gather rejected a value)"""
    msgs, lk, joins = session

    def neg(*xs):
        return any(isinstance(x, int) and x < 0 for x in xs)

    def fields(o, names):
        return neg(*(getattr(o, a, 0) for a in names))
    for k in lk.paillier_key_vec:
        if fields(k, ("n",)):
            return True
    for s in lk.h1_h2_n_tilde_vec:
        if fields(s, ("N", "g", "ni")):
            return True
    for m in list(msgs) + list(joins):
        rp = m.ring_pedersen_proof
        if fields(m.ek, ("n",)) or fields(m.ring_pedersen_statement, ("S", "T", "N")) or neg(*rp.A) or \
                neg(*rp.Z) or neg(*m.dk_correctness_proof.sigma_vec):
            return True
    for m in msgs:
        if neg(*m.points_encrypted_vec) or \
                any(fields(p, ("z", "u2", "u3", "s1", "s2", "s3")) for p in m.pdl_proof_vec) or \
                any(fields(a, ("z", "e", "s", "s1", "s2")) for a in m.range_proofs):
            return True
    for j in joins:
        if fields(j.dlog_statement, ("N", "g", "ni")) or \
                fields(j.composite_dlog_proof_base_h1, ("x", "y")) or fields(j.composite_dlog_proof_base_h2, ("x", "y")):
            return True
    return False


def _regular(msgs, lk, joins, M):
    """The shape a SessionSet packs without per-session optional fields: every
    vector at full length, the LocalKey holding every receiver's keys, t+1
    commitments per message, and the threshold / size checks passing."""
    R, J = len(msgs), len(joins)
    n = R + J
    t = lk.t
    if R == 0 or R <= t or len(lk.paillier_key_vec) < n or len(lk.h1_h2_n_tilde_vec) < n:
        return False
    for m in msgs:
        if not (len(m.pdl_proof_vec) == len(m.points_committed_vec) == len(m.points_encrypted_vec) == n) or \
                len(m.range_proofs) < n or len(m.coefficients_committed_vec.commitments) != t + 1:
            return False
    for m in msgs + joins:
        if len(m.ring_pedersen_proof.A) < M or len(m.ring_pedersen_proof.Z) < M or \
                len(m.dk_correctness_proof.sigma_vec) < M2:
            return False
    return True


class SessionSet:
    """Many independent collect() sessions (BASELINE configs[4]) packed as ONE set
    of SoA arrays: every field is gathered across all regular sessions in one
    pass (one gather, one threaded conversion), and each session's
    fsdkr_collect_batch points at its rows (a numpy array with the C struct
    layout, filled vectorised).  Sessions of another shape get their own
    CollectBatch; header-only sessions (threshold / size failures) are not
    prepared.  `live` lists the prepared sessions, in `structs` row order."""

    def __init__(self, sessions, m_security=256, key_bits=2048, staged=False, split_stage1=True):
        """staged: gather only what fsdkr_collect_prestart_multi reads (recv_n, PDL
        s2, range-proof s of the regular sessions; prestart_array) and leave the
        rest to complete(), so the longest chains run while it packs."""
        M = m_security
        S = len(sessions)
        self.S = S
        self.batches = [None] * S
        reg = [s for s, (m, lk, j) in enumerate(sessions) if _regular(m, lk, j, M)]
        regset = set(reg)
        for s, (m, lk, j) in enumerate(sessions):
            if s not in regset:
                self.batches[s] = CollectBatch(m, lk, j, M, key_bits)
        self.live = [s for s in range(S) if s in regset or not self.batches[s].header_only]
        self.R = np.array([len(sessions[s][0]) for s in range(S)], dtype=np.int64)
        self.J = np.array([len(sessions[s][2]) for s in range(S)], dtype=np.int64)
        self.n = self.R + self.J
        self._keep = []
        self._owned = []   # pooled slot arrays, back to _POOL when the set is collected
        weakref.finalize(self, _POOL.give, self._owned)
        self.structs = np.zeros(len(self.live), dtype=_BATCH_DT)
        self.row = {s: r for r, s in enumerate(self.live)}
        self._pre, self.n_prestart = None, 0
        self._z = None   # stage 1b: (Z rows array, max bits), reused by stage 2
        self._pending = (sessions, reg, M, key_bits)
        # the prestart covers the set only when every prepared session is regular
        # (prepare_multi's session list must equal the prestart's)
        self._s1b = None   # a split stage 1's rest: (n, nl, M, its gathered fields)
        if staged and reg and len(reg) == len(self.live):
            self._stage1(sessions, reg, M, split_stage1)
        if not staged:
            self.complete()

    def complete(self):
        """Stage 2 of a staged set (SessionSet(..., staged=True)): every field."""
        if self._pending is None:
            return self
        sessions, reg, M, key_bits = self._pending
        self._pending = None
        if reg:
            try:
                self._pack_regular(sessions, reg, M, key_bits)
            except UnsupportedInput:
                # negative operands: those sessions get their own CollectBatch, whose
                # instances carry the reference's per-instance outcome (_Negatives)
                neg = [s for s in reg if _has_negative(sessions[s])]
                if not neg:
                    raise
                for s in neg:
                    self.batches[s] = CollectBatch(*sessions[s], M, key_bits)
                reg = [s for s in reg if s not in set(neg)]
                self._z = None   # (stage 1b's Z rows covered the old list)
                if reg:
                    self._pack_regular(sessions, reg, M, key_bits)
        regset = set(reg)
        for s in self.live:
            if s not in regset:
                b = self.batches[s]
                self.structs[self.row[s]] = np.frombuffer(ctypes.string_at(ctypes.addressof(b.c), ctypes.sizeof(b.c)),
                                                          dtype=_BATCH_DT)[0]
        return self

    def _stage1(self, sessions, reg, M, split=True):
        """The fields fsdkr_collect_prestart_multi reads: the GA chains' (receivers'
        N, PDL s2, range-proof s), the fixed-base tables' bases (receivers' N~,
        h1, h2; ring-Pedersen T and N) and the correct-key job's (ek.n, sigma).  The exponents stay in stage 2: the tables
        are sized by honest bounds (s1 < 2^770, s3 | s2 < 2^770 N~, Z < phi(N)),
        which prepare checks against the packed exponents.  split: GA's fields
        only, so GA starts after converting 2Rn + n values per session; stage1b()
        packs the rest for a second prestart call."""
        ses = [sessions[s] for s in reg]
        R = np.array([len(m) for m, lk, j in ses], dtype=np.int64)
        n = R + np.array([len(j) for m, lk, j in ses], dtype=np.int64)
        if any(len(lk.paillier_key_vec) < nn for (m, lk, j), nn in zip(ses, n)):
            return
        G = _Gather(self._owned)
        try:   # (a negative operand: no prestart; complete() moves its session out)
            f_rn = G.field([k for (ms, lk, js), nn in zip(ses, n) for k in lk.paillier_key_vec[:nn]], "n")
            f_s2 = G.field([m.pdl_proof_vec[i] for (ms, lk, js), nn in zip(ses, n) for m in ms for i in range(nn)],
                           "s2")
            f_s = G.field([m.range_proofs[i] for (ms, lk, js), nn in zip(ses, n) for m in ms for i in range(nn)],
                          "s")
            sts = [st for (ms, lk, js), nn in zip(ses, n) for st in lk.h1_h2_n_tilde_vec[:nn]]
            if len(sts) != int(n.sum()):
                return
            f_nt, f_h1, f_h2 = G.field(sts, "N"), G.field(sts, "g"), G.field(sts, "ni")
            am = [m for ms, lk, js in ses for m in ms + js]
            rps = [m.ring_pedersen_statement for m in am]
            f_T, f_N = G.field(rps, "T"), G.field(rps, "N")
        except UnsupportedInput:
            return
        bits = max(1, f_rn[1], f_s2[1], f_s[1], f_nt[1], f_h1[1], f_h2[1], f_T[1], f_N[1])
        nl = 64 if bits <= 2048 else 96 if bits <= 3072 else None
        if nl is None:
            return
        a_rn, a_s2, a_s = G.slot(f_rn, nl), G.slot(f_s2, nl), G.slot(f_s, nl)
        rest = (f_nt, f_h1, f_h2, f_T, f_N, am)
        if not split:
            self._stage1_rest(G, n, nl, M, *rest)
        G.run()

        def starts(counts):
            return np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.uint64)
        st = np.zeros(len(reg), dtype=_BATCH_DT)
        st["n_refresh"] = R
        st["n_join"] = n - R
        st["nl"] = nl
        st["recv_n"] = np.uint64(self._k(a_rn)) + starts(n) * np.uint64(nl * 4)
        st["pdl_s2"] = np.uint64(self._k(a_s2)) + starts(R * n) * np.uint64(nl * 4)
        st["rp_s"] = np.uint64(self._k(a_s)) + starts(R * n) * np.uint64(nl * 4)
        st["m_security"] = M
        st["s1l"], st["s3l"], st["zl"] = _limbs_for(770), nl + _limbs_for(770), nl
        self._pre, self.n_prestart = st, len(reg)
        if split:
            self._s1b = (n, nl, M) + rest
        else:
            self._stage1_fill()

    def _stage1_rest(self, G, n, nl, M, f_nt, f_h1, f_h2, f_T, f_N, am):
        """slots of the tables' bases and the correct-key inputs (converted by G.run)"""
        f_ckn = G.field([m.ek.n for m in am])
        f_sig = G.rows([m.dk_correctness_proof for m in am], "sigma_vec", M2)
        ckl = next((w for w in _CK_WIDTHS if max(1, f_ckn[1], f_sig[1]) <= 32 * w), None)
        arrs = {"recv_ntilde": G.slot(f_nt, nl), "recv_h1": G.slot(f_h1, nl), "recv_h2": G.slot(f_h2, nl),
                "ped_T": G.slot(f_T, nl), "ped_N": G.slot(f_N, nl)}
        if ckl is not None:
            ckl = max(ckl, nl)
            arrs["ck_n"], arrs["ck_sigma"] = G.slot(f_ckn, ckl), G.slot(f_sig, ckl)
        self._s1_arrs = (n, nl, ckl, arrs)

    def _stage1_fill(self):
        """point the prestart rows at _stage1_rest's converted arrays"""
        n, nl, ckl, arrs = self._s1_arrs
        st = self._pre

        def starts(counts):
            return np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.uint64)
        for name in ("recv_ntilde", "recv_h1", "recv_h2"):
            st[name] = np.uint64(self._k(arrs[name])) + starts(n) * np.uint64(nl * 4)
        for name in ("ped_T", "ped_N"):
            st[name] = np.uint64(self._k(arrs[name])) + starts(n) * np.uint64(nl * 4)   # R + J messages per session
        if ckl is not None:
            st["ckl"] = ckl
            st["ck_n"] = np.uint64(self._k(arrs["ck_n"])) + starts(n) * np.uint64(ckl * 4)
            st["ck_sigma"] = np.uint64(self._k(arrs["ck_sigma"])) + starts(n * M2) * np.uint64(ckl * 4)

    def stage1b(self):
        """The rest of a split stage 1 (the fixed-base tables' bases, the
        correct-key inputs) for a second fsdkr_collect_prestart_multi call (GA
        keeps running; the table chains and the correct-key job start).  True when
        it packed them."""
        if self._s1b is None or self._pre is None or self._pending is None:
            return False
        n, nl, M, *rest = self._s1b
        self._s1b = None
        G = _Gather(self._owned)
        try:
            self._stage1_rest(G, n, nl, M, *rest)
        except UnsupportedInput:
            return False
        G.run()
        self._stage1_fill()
        return True

    def stage_z(self):
        """Stage 1b of a staged set: the ring-Pedersen Z rows of every regular
        session (the largest field: 0.3 GB at configs[4]), packed at the width
        stage 2 gives them and reused there, for fsdkr_collect_prestart_rp.
        Returns whether the prestart rows now carry them."""
        if self._pre is None or self._pending is None:
            return False
        sessions, reg, M, key_bits = self._pending
        ses = [sessions[s] for s in reg]
        G = _Gather(self._owned)
        try:
            f_z = G.rows([m.ring_pedersen_proof for ms, lk, js in ses for m in ms + js], "Z", M)
        except UnsupportedInput:
            return False
        zl = _limbs_for(max(1, f_z[1]))
        a_z = G.slot(f_z, zl)
        G.run()
        n = self._pre["n_refresh"].astype(np.int64) + self._pre["n_join"].astype(np.int64)
        starts = np.concatenate([[0], np.cumsum(n * M)[:-1]]).astype(np.uint64)
        self._pre["ped_Z"] = np.uint64(self._k(a_z)) + starts * np.uint64(zl * 4)
        self._pre["zl"] = zl
        self._z = (a_z, f_z[1])
        return True

    def prestart_array(self):
        """fsdkr_collect_batch rows for fsdkr_collect_prestart_multi (None: nothing to start)."""
        if self._pre is None:
            return None
        return ctypes.cast(self._pre.ctypes.data, ctypes.POINTER(CollectBatchC))

    def _k(self, arr):
        arr = np.ascontiguousarray(arr, dtype=np.uint32)
        self._keep.append(arr)
        return arr.ctypes.data

    def _pack_regular(self, sessions, reg, M, key_bits):
        G = _Gather(self._owned)
        ses = [sessions[s] for s in reg]
        R = np.array([len(m) for m, lk, j in ses], dtype=np.int64)
        J = np.array([len(j) for m, lk, j in ses], dtype=np.int64)
        n = R + J
        Mt, P = R + J, R * n
        t = np.array([lk.t for m, lk, j in ses], dtype=np.int64)
        V = R * (t + 1)
        all_m = [m + j for m, lk, j in ses]
        pdl = [m.pdl_proof_vec[i] for (ms, lk, js), nn in zip(ses, n) for m in ms for i in range(nn)]
        rng = [m.range_proofs[i] for (ms, lk, js), nn in zip(ses, n) for m in ms for i in range(nn)]
        keys = [k for (ms, lk, js), nn in zip(ses, n) for k in lk.paillier_key_vec[:nn]]
        sts = [s for (ms, lk, js), nn in zip(ses, n) for s in lk.h1_h2_n_tilde_vec[:nn]]
        msgs = [m for ms, lk, js in ses for m in ms]
        joins = [j for ms, lk, js in ses for j in js]
        am = [m for row in all_m for m in row]
        F = {"recv_n": G.field(keys, "n"), "recv_ntilde": G.field(sts, "N"), "recv_h1": G.field(sts, "g"),
             "recv_h2": G.field(sts, "ni"),
             "enc": G.field([m.points_encrypted_vec[i] for (ms, lk, js), nn in zip(ses, n) for m in ms
                             for i in range(nn)])}
        for a in ("z", "u2", "u3", "s1", "s2", "s3"):
            F["pdl_" + a] = G.field(pdl, a)
        for a in ("z", "e", "s", "s1", "s2"):
            F["rp_" + a] = G.field(rng, a)
        for a in ("S", "T", "N"):
            F["ped_" + a] = G.field([m.ring_pedersen_statement for m in am], a)
        # regular sessions hold full-length vectors (_regular): flattened in C
        rpp = [m.ring_pedersen_proof for m in am]
        F["ped_A"] = G.rows(rpp, "A", M)
        if self._z is None:   # (stage 1b packed Z already: reused below)
            F["ped_Z"] = G.rows(rpp, "Z", M)
        f_ckn = G.field([m.ek.n for m in am])
        f_sig = G.rows([m.dk_correctness_proof for m in am], "sigma_vec", M2)
        if joins:
            for name, attr in (("N", "N"), ("g", "g"), ("ni", "ni")):
                F["dlog_" + name] = G.field([j.dlog_statement for j in joins], attr)
            for name, which, attr in (("x1", 1, "x"), ("x2", 2, "x"), ("y1", 1, "y"), ("y2", 2, "y")):
                F["dlog_" + name] = G.field([getattr(j, f"composite_dlog_proof_base_h{which}") for j in joins], attr)

        def bits(*names):
            return max([1] + [F[x][1] for x in names if x in F])

        ck_bits = max(1, f_ckn[1], f_sig[1])
        ckl = next((w for w in _CK_WIDTHS if ck_bits <= 32 * w), None)
        if ckl is None:
            raise UnsupportedInput(f"{ck_bits}-bit Paillier key / correct-key proof")
        nl_bits = max(bits("recv_n", "recv_ntilde", "recv_h1", "recv_h2"), bits("ped_N", "ped_S", "ped_T", "ped_A"),
                      bits("dlog_N", "dlog_g", "dlog_ni", "dlog_x1", "dlog_x2"),
                      bits("pdl_z", "pdl_u3", "pdl_s2", "rp_z", "rp_s"), (bits("enc", "pdl_u2") + 1) // 2)
        nl = 64 if nl_bits <= 2048 else 96 if nl_bits <= 3072 else None
        if nl is None:
            raise UnsupportedInput(f"{nl_bits}-bit value in a 3072-bit slot")
        z_bits = self._z[1] if self._z is not None else bits("ped_Z")
        W = {"nl": nl, "ckl": max(ckl, nl), "s1l": _limbs_for(bits("pdl_s1", "rp_s1")),
             "s3l": _limbs_for(bits("pdl_s3", "rp_s2")), "el": _limbs_for(bits("rp_e")),
             "zl": _limbs_for(max(1, z_bits)), "yl": _limbs_for(bits("dlog_y1", "dlog_y2"))}
        width = {"enc": 2 * nl, "pdl_u2": 2 * nl, "pdl_s1": W["s1l"], "rp_s1": W["s1l"], "pdl_s3": W["s3l"],
                 "rp_s2": W["s3l"], "rp_e": W["el"], "ped_Z": W["zl"], "dlog_y1": W["yl"], "dlog_y2": W["yl"]}
        arrs = {name: G.slot(f, width.get(name, nl)) for name, f in F.items()}
        if self._z is not None:
            arrs["ped_Z"] = self._z[0]
        arrs["ck_n"] = G.slot(f_ckn, W["ckl"])
        arrs["ck_sigma"] = G.slot(f_sig, W["ckl"])
        G.run()
        arrs["commit"] = pack_points([m.points_committed_vec[i] for (ms, lk, js), nn in zip(ses, n) for m in ms
                                      for i in range(nn)])
        arrs["pdl_u1"] = pack_points(pdl, "u1")
        arrs["vss"] = pack_points([p for m in msgs for p in m.coefficients_committed_vec.commitments])
        # party indices per session: refresh then joins (0 = unassigned)
        pidx = np.array([x for ms, lk, js in ses for x in [m.party_index for m in ms] +
                         [(j.party_index or 0) for j in js]], dtype=np.uint32)
        lens = np.repeat(n, R)[:, None].repeat(3, axis=1).astype(np.uint32)
        arrs["party_index"], arrs["msg_lens"] = pidx, lens
        # row offsets of every session, per row class
        def starts(counts):
            return np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.uint64)
        row_of = {"recv": starts(n), "pair": starts(P), "vss": starts(V), "msg": starts(Mt),
                  "rpm": starts(Mt * M), "sig": starts(Mt * M2), "join": starts(J), "pidx": starts(Mt),
                  "lens": starts(R)}
        klass = {"recv_n": "recv", "recv_ntilde": "recv", "recv_h1": "recv", "recv_h2": "recv", "enc": "pair",
                 "commit": "pair", "pdl_z": "pair", "pdl_u1": "pair", "pdl_u2": "pair", "pdl_u3": "pair",
                 "pdl_s1": "pair", "pdl_s2": "pair", "pdl_s3": "pair", "rp_z": "pair", "rp_e": "pair",
                 "rp_s": "pair", "rp_s1": "pair", "rp_s2": "pair", "vss": "vss", "ped_S": "msg", "ped_T": "msg",
                 "ped_N": "msg", "ped_A": "rpm", "ped_Z": "rpm", "ck_n": "msg", "ck_sigma": "sig",
                 "dlog_N": "join", "dlog_g": "join", "dlog_ni": "join", "dlog_x1": "join", "dlog_x2": "join",
                 "dlog_y1": "join", "dlog_y2": "join", "party_index": "pidx", "msg_lens": "lens"}
        row = {s: r for r, s in enumerate(self.live)}
        rows = np.array([row[s] for s in reg], dtype=np.int64)
        st = self.structs
        for f, v in (("n_refresh", R), ("n_join", J), ("t", t)):
            st[f][rows] = v
        for f, v in (("m_security", M), ("key_bits", key_bits)):
            st[f][rows] = v
        for f in ("nl", "s1l", "s3l", "el", "zl", "yl", "ckl"):
            st[f][rows] = W[f]
        for name, arr in arrs.items():
            stride = arr.shape[1] * 4 if arr.ndim == 2 else 4
            base = self._k(arr)
            st[name][rows] = np.uint64(base) + row_of[klass[name]] * np.uint64(stride)

    @property
    def c_array(self):
        """the fsdkr_collect_batch array (live sessions) as ctypes pointer"""
        return ctypes.cast(self.structs.ctypes.data, ctypes.POINTER(CollectBatchC))

    def verdicts(self):
        """Verdict arrays of the live sessions and their fsdkr_verdicts array."""
        return SetVerdicts(self)

    def settle(self, v):
        """CollectBatch.settle for the sessions packed on their own (the only ones
        that may carry negative operands)"""
        for s, b in enumerate(self.batches):
            if b is not None and b.negs and s in self.row:
                r = self.row[s]
                p, j = int(v.off["pair"][r]), int(v.off["join"][r])
                P, J = int(v.P[r]), int(v.Jn[r])
                b.negs.apply(v.pdl[p:p + P], v.range[p:p + P], v.dlog[j:j + J])
        return v

    def first_errors(self, verdicts):
        """{session: fsdkr_error} of every live session from ONE
        fsdkr_collect_first_error_multi call (1 024 per-session ctypes calls cost
        ~5 ms of a configs[4] step)"""
        n = len(self.live)
        errs = (ErrorC * n)()
        if n:
            bp = ctypes.cast(self.structs.ctypes.data, ctypes.POINTER(CollectBatchC))
            vp = ctypes.cast(verdicts.structs.ctypes.data, ctypes.POINTER(VerdictsC))
            rc = lib().fsdkr_collect_first_error_multi(bp, vp, n, errs)
            if rc != 0:
                raise RuntimeError(f"fsdkr_collect_first_error_multi failed ({rc})")
        return {s: errs[r] for s, r in self.row.items()}

    def first_error(self, s, verdicts):
        """fsdkr_collect_first_error of session s (live: its prepared verdicts; else header only)."""
        if s not in self.row:
            return self.batches[s].first_error(None)
        err = ErrorC()
        r = self.row[s]
        bp = ctypes.cast(self.structs.ctypes.data + r * _BATCH_DT.itemsize, ctypes.POINTER(CollectBatchC))
        vp = ctypes.cast(verdicts.structs.ctypes.data + r * _VERD_DT.itemsize, ctypes.POINTER(VerdictsC))
        rc = lib().fsdkr_collect_first_error(bp, vp, ctypes.byref(err))
        if rc != 0:
            raise RuntimeError(f"fsdkr_collect_first_error failed ({rc})")
        return err


class SetVerdicts:
    """Verdict bytes of every live session of a SessionSet, one array per kind,
    and the per-session fsdkr_verdicts rows pointing into them."""

    def __init__(self, sset):
        live = sset.live
        R, J, n = sset.R[live], sset.J[live], sset.n[live]
        P, Mt = R * n, R + J
        self.P, self.Mt, self.Jn = P, Mt, J

        def starts(c):
            return np.concatenate([[0], np.cumsum(c)[:-1]]).astype(np.uint64)
        self.feldman = np.zeros(max(int(P.sum()), 1), np.uint8)
        self.pdl = np.zeros_like(self.feldman)
        self.range = np.zeros_like(self.feldman)
        self.ped = np.zeros(max(int(Mt.sum()), 1), np.uint8)
        self.ck = np.zeros_like(self.ped)
        self.dlog = np.zeros(max(int(J.sum()), 1), np.uint8)
        self.off = {"pair": starts(P), "msg": starts(Mt), "join": starts(J)}
        st = np.zeros(len(live), dtype=_VERD_DT)
        for name, kind in (("feldman", "pair"), ("pdl", "pair"), ("range", "pair"), ("ped", "msg"), ("ck", "msg"),
                           ("dlog", "join")):
            st[name] = np.uint64(getattr(self, name).ctypes.data) + self.off[kind]
        st["cap_pairs"], st["cap_msgs"], st["cap_joins"] = P, Mt, J
        self.structs = st

    @property
    def c_array(self):
        return ctypes.cast(self.structs.ctypes.data, ctypes.POINTER(VerdictsC))
