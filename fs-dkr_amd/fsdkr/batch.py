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
proof runs at its own width before ModuliTooSmall, :376-391).  Still outside
the representable set (UnsupportedInput): negative BigInts and values wider
than 3072 bits in a proof field (6144 bits for ek.n / sigma)."""
import ctypes

import numpy as np

from . import _pack
from ._native import CollectBatchC, ErrorC, VerdictsC, lib

M2 = 11   # zk-paillier NiCorrectKeyProof sigma_vec length
_CK_WIDTHS = (64, 96, 128, 192)


class UnsupportedInput(ValueError):
    """Input outside what the C ABI represents (negative BigInts, oversize values)."""


def _limbs_for(bits):
    return max(1, (bits + 31) // 32)


def pack_attr(objs, attr, limbs):
    """getattr(o, attr) (attr None: o) of every object -> (len, limbs) uint32,
    little-endian, written in place by the C extension; raises UnsupportedInput
    on negatives / overflow."""
    arr = np.empty((len(objs), limbs), dtype=np.uint32)
    try:
        _pack.pack(objs, attr, arr, limbs)
    except ValueError as e:
        raise UnsupportedInput(str(e)) from None
    except OverflowError:
        raise UnsupportedInput(f"value exceeds the {32 * limbs}-bit slot") from None
    return arr


def pack(values, limbs):
    """ints -> (len, limbs) uint32, little-endian; raises on negatives / overflow."""
    return pack_attr(values, None, limbs)


def pack_points(points):
    """affine (x, y) or None -> (len, 16) uint32, (0,0) = infinity."""
    z = b"\x00" * 64
    raw = b"".join([z if pt is None else pt[0].to_bytes(32, "little") + pt[1].to_bytes(32, "little")
                    for pt in points])
    return np.frombuffer(raw, dtype=np.uint32).reshape(len(points), 16)


def _ptr(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))


def _bits(values, attr=None):
    """max bit length (>= 1) of the values (or of their `attr`); negatives -> UnsupportedInput."""
    try:
        return max(1, _pack.maxbits(values, attr))
    except ValueError as e:
        raise UnsupportedInput(str(e)) from None


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
                 header_only=False):
        """n_recv: receivers (default R + J); a multi-GPU shard passes its slice of the
        messages together with the full receiver count."""
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
        # ---- widths: nl covers every value of the nl / 2nl slots; ek.n and sigma get ckl
        ck_bits = _bits([m.ek.n for m in all_m] + [s for m in all_m for s in m.dk_correctness_proof.sigma_vec[:M2]])
        ckl = next((w for w in _CK_WIDTHS if ck_bits <= 32 * w), None)
        if ckl is None:
            raise UnsupportedInput(f"{ck_bits}-bit Paillier key / correct-key proof")
        if self.header_only:
            c.nl = 64 if ck_bits <= 2048 else 96
            c.ckl = max(ckl, c.nl)
            c.ck_n = self._k(pack([m.ek.n for m in all_m] or [0], c.ckl))
            self.nl = c.nl
            return
        keys, sts = local_key.paillier_key_vec, local_key.h1_h2_n_tilde_vec
        avail = min(len(keys), len(sts), n)
        c.recv_avail = avail if avail < n else 0
        pdl = [m.pdl_proof_vec[i] for m in msgs for i in range(n)]
        short_rng = any(len(m.range_proofs) < n for m in msgs)
        rng = [m.range_proofs[i] if i < len(m.range_proofs) else None for m in msgs for i in range(n)]
        rng_ok = [a for a in rng if a is not None]
        recv_vals = [k.n for k in keys[:avail]] + [v for s in sts[:avail] for v in (s.N, s.g, s.ni)]
        rp_vals = [v for m in all_m for v in (m.ring_pedersen_statement.N, m.ring_pedersen_statement.S,
                                             m.ring_pedersen_statement.T)] + \
                  [a for m in all_m for a in m.ring_pedersen_proof.A[:M]]
        dl_vals = [v for j in joins for v in (j.dlog_statement.N, j.dlog_statement.g, j.dlog_statement.ni,
                                             j.composite_dlog_proof_base_h1.x, j.composite_dlog_proof_base_h2.x)]
        enc = [m.points_encrypted_vec[i] for m in msgs for i in range(n)]
        one_bits = max(_bits(pdl, "z"), _bits(pdl, "u3"), _bits(pdl, "s2"), _bits(rng_ok, "z"), _bits(rng_ok, "s"))
        two_bits = max(_bits(enc), _bits(pdl, "u2"))
        nl_bits = max(_bits(recv_vals), _bits(rp_vals), _bits(dl_vals), one_bits, (two_bits + 1) // 2)
        nl = 64 if nl_bits <= 2048 else 96 if nl_bits <= 3072 else None
        if nl is None:
            raise UnsupportedInput(f"{nl_bits}-bit value in a 3072-bit slot")
        c.nl = nl
        c.ckl = max(ckl, nl)
        c.s1l = _limbs_for(max(_bits(pdl, "s1"), _bits(rng_ok, "s1")))
        c.s3l = _limbs_for(max(_bits(pdl, "s3"), _bits(rng_ok, "s2")))
        c.el = _limbs_for(_bits(rng_ok, "e"))
        c.zl = _limbs_for(_bits([z for m in all_m for z in m.ring_pedersen_proof.Z[:M]]))
        c.yl = _limbs_for(_bits([j.composite_dlog_proof_base_h1.y for j in joins] +
                                [j.composite_dlog_proof_base_h2.y for j in joins]))
        k = self._k
        # receivers (placeholders past the keys the LocalKey holds: odd modulus 3)
        rn = [x.n for x in keys[:avail]] + [3] * (n - avail)
        rst = list(sts[:avail]) + [None] * (n - avail)
        c.recv_n = k(pack(rn, nl))
        c.recv_ntilde = k(pack([s.N if s else 3 for s in rst], nl))
        c.recv_h1 = k(pack([s.g if s else 1 for s in rst], nl))
        c.recv_h2 = k(pack([s.ni if s else 1 for s in rst], nl))
        c.enc = k(pack(enc, 2 * nl))
        c.commit = k(pack_points([m.points_committed_vec[i] for m in msgs for i in range(n)]))
        c.pdl_z = k(pack_attr(pdl, "z", nl))
        c.pdl_u1 = k(pack_points([p.u1 for p in pdl]))
        c.pdl_u2 = k(pack_attr(pdl, "u2", 2 * nl))
        c.pdl_u3 = k(pack_attr(pdl, "u3", nl))
        c.pdl_s1 = k(pack_attr(pdl, "s1", c.s1l))
        c.pdl_s2 = k(pack_attr(pdl, "s2", nl))
        c.pdl_s3 = k(pack_attr(pdl, "s3", c.s3l))
        if short_rng:   # range_proofs[i] past the vector: placeholder rows, the reference panics there
            c.range_lens = k(np.array([len(m.range_proofs) for m in msgs], dtype=np.uint32))
            rng = [a if a is not None else _ZERO_ALICE for a in rng]
        c.rp_z = k(pack_attr(rng, "z", nl))
        c.rp_e = k(pack_attr(rng, "e", c.el))
        c.rp_s = k(pack_attr(rng, "s", nl))
        c.rp_s1 = k(pack_attr(rng, "s1", c.s1l))
        c.rp_s2 = k(pack_attr(rng, "s2", c.s3l))
        t = local_key.t
        com = [list(m.coefficients_committed_vec.commitments) for m in msgs]
        if any(len(x) != t + 1 for x in com):   # Horner over each message's own vector
            c.vss_len = k(np.array([len(x) for x in com], dtype=np.uint32))
        c.vss = k(pack_points([p for x in com for p in x] or [None]))
        c.ped_S = k(pack([m.ring_pedersen_statement.S for m in all_m], nl))
        c.ped_T = k(pack([m.ring_pedersen_statement.T for m in all_m], nl))
        c.ped_N = k(pack([m.ring_pedersen_statement.N for m in all_m], nl))
        A = [list(m.ring_pedersen_proof.A[:M]) for m in all_m]
        Z = [list(m.ring_pedersen_proof.Z[:M]) for m in all_m]
        if any(len(a) < M for a in A) or any(len(z) < M for z in Z):
            c.ped_lens = k(np.array([[len(a), len(z)] for a, z in zip(A, Z)], dtype=np.uint32))
            A = [a + [0] * (M - len(a)) for a in A]
            Z = [z + [0] * (M - len(z)) for z in Z]
        c.ped_A = k(pack([a for row in A for a in row], nl))
        c.ped_Z = k(pack([z for row in Z for z in row], c.zl))
        c.ck_n = k(pack([m.ek.n for m in all_m], c.ckl))
        sig = [list(m.dk_correctness_proof.sigma_vec[:M2]) for m in all_m]
        if any(len(x) < M2 for x in sig):
            c.ck_lens = k(np.array([len(x) for x in sig], dtype=np.uint32))
            sig = [x + [0] * (M2 - len(x)) for x in sig]
        c.ck_sigma = k(pack([s for row in sig for s in row], c.ckl))
        if J:
            c.dlog_N = k(pack([j.dlog_statement.N for j in joins], nl))
            c.dlog_g = k(pack([j.dlog_statement.g for j in joins], nl))
            c.dlog_ni = k(pack([j.dlog_statement.ni for j in joins], nl))
            c.dlog_x1 = k(pack([j.composite_dlog_proof_base_h1.x for j in joins], nl))
            c.dlog_x2 = k(pack([j.composite_dlog_proof_base_h2.x for j in joins], nl))
            c.dlog_y1 = k(pack([j.composite_dlog_proof_base_h1.y for j in joins], c.yl))
            c.dlog_y2 = k(pack([j.composite_dlog_proof_base_h2.y for j in joins], c.yl))
        self.nl = nl

    def _k(self, arr):
        arr = np.ascontiguousarray(arr, dtype=np.uint32)
        self._keep.append(arr)
        return _ptr(arr)

    def first_error(self, verdicts):
        err = ErrorC()
        rc = lib().fsdkr_collect_first_error(ctypes.byref(self.c),
                                             ctypes.byref(verdicts.c) if verdicts is not None else None,
                                             ctypes.byref(err))
        if rc != 0:
            raise RuntimeError(f"fsdkr_collect_first_error failed ({rc})")
        return err


class _ZeroAlice:
    z = e = s = s1 = s2 = 0


_ZERO_ALICE = _ZeroAlice()
