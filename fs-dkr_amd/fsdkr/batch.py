"""Batching layer: gathers the n x n proof instances of a collect() call into
the SoA little-endian limb buffers of `struct fsdkr_collect_batch`
(include/fsdkr/fsdkr.h).

North star job (4) places this layer in the Rust crate; with no Rust
toolchain in this image it is restated here and reads the reference's message
structures by field name (refresh_message.rs:31-48, add_party_message.rs:36-45,
zk_pdl_with_slack.rs:41-50, range_proofs.rs:101-108,
ring_pedersen_proof.rs:30-38,79-84).  Any object with those attributes works."""
import ctypes

import numpy as np

from ._native import CollectBatchC, ErrorC, VerdictsC, lib

M2 = 11   # zk-paillier NiCorrectKeyProof sigma_vec length


class UnsupportedInput(ValueError):
    """Input outside what the C ABI represents (negative BigInts, oversize moduli)."""


def _limbs_for(bits):
    return max(1, (bits + 31) // 32)


def pack(values, limbs):
    """ints -> (len, limbs) uint32, little-endian; raises on negatives / overflow."""
    nbytes = 4 * limbs
    parts = []
    for v in values:
        if v < 0:
            raise UnsupportedInput("negative big integer in a proof field")
        if v.bit_length() > 8 * nbytes:
            raise UnsupportedInput(f"value of {v.bit_length()} bits exceeds the {8 * nbytes}-bit slot")
        parts.append(v.to_bytes(nbytes, "little"))
    return np.frombuffer(b"".join(parts), dtype=np.uint32).reshape(len(values), limbs).copy()


def pack_points(points):
    """affine (x, y) or None -> (len, 16) uint32, (0,0) = infinity."""
    parts = []
    for pt in points:
        if pt is None:
            parts.append(b"\x00" * 64)
        else:
            parts.append(pt[0].to_bytes(32, "little") + pt[1].to_bytes(32, "little"))
    return np.frombuffer(b"".join(parts), dtype=np.uint32).reshape(len(points), 16).copy()


def _ptr(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))


class Verdicts:
    def __init__(self, R, J, n):
        P = R * n
        self.feldman = np.zeros(P, np.uint8)
        self.pdl = np.zeros(P, np.uint8)
        self.range = np.zeros(P, np.uint8)
        self.ped = np.zeros(R + J, np.uint8)
        self.ck = np.zeros(R + J, np.uint8)
        self.dlog = np.zeros(max(J, 1), np.uint8)
        u8 = ctypes.POINTER(ctypes.c_uint8)
        self.c = VerdictsC(*(a.ctypes.data_as(u8) for a in (self.feldman, self.pdl, self.range, self.ped, self.ck,
                                                            self.dlog)))


class CollectBatch:
    """SoA view of (refresh_messages, local_key, join_messages) for one collect().

    `header_only` is set when validate_collect's threshold / size checks fail
    (refresh_message.rs:149-175): then only the counts are filled and the
    first error is decided without the GPU."""

    def __init__(self, refresh_messages, local_key, join_messages, m_security=256, key_bits=2048, n_recv=None):
        """n_recv: receivers (default R + J); a multi-GPU shard passes its slice of
        the messages together with the full receiver count."""
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
        ref = lens[0][0] if R else 0
        # the threshold check (refresh_message.rs:149) is about the whole message set: a
        # multi-GPU shard (n_recv given) holds a slice that may be <= t messages
        below_threshold = R <= local_key.t and not n_recv
        self.header_only = (below_threshold or R == 0 or any(tuple(l) != (ref, ref, ref) for l in lens[:R])
                            or ref < n or any(len(m.range_proofs) < n for m in msgs))
        if self.header_only:
            return
        recv_keys = local_key.paillier_key_vec[:n]
        recv_dlog = local_key.h1_h2_n_tilde_vec[:n]
        mod_bits = max([k.n.bit_length() for k in recv_keys] + [s.N.bit_length() for s in recv_dlog] +
                       [m.ring_pedersen_statement.N.bit_length() for m in msgs + joins] +
                       [m.ek.n.bit_length() for m in msgs + joins] +
                       [j.dlog_statement.N.bit_length() for j in joins])
        nl = 64 if mod_bits <= 2048 else 96 if mod_bits <= 3072 else None
        if nl is None:
            raise UnsupportedInput(f"{mod_bits}-bit modulus")
        c.nl = nl
        pdl = [m.pdl_proof_vec[i] for m in msgs for i in range(n)]
        rng = [m.range_proofs[i] for m in msgs for i in range(n)]
        c.s1l = _limbs_for(max([p.s1.bit_length() for p in pdl] + [a.s1.bit_length() for a in rng]))
        c.s3l = _limbs_for(max([p.s3.bit_length() for p in pdl] + [a.s2.bit_length() for a in rng]))
        c.el = _limbs_for(max(a.e.bit_length() for a in rng))
        M = m_security
        for m in msgs + joins:
            if len(m.ring_pedersen_proof.A) < M or len(m.ring_pedersen_proof.Z) < M or \
                    len(m.dk_correctness_proof.sigma_vec) < M2:
                raise UnsupportedInput("short ring-Pedersen / correct-key vectors (the reference panics)")
        c.zl = _limbs_for(max(z.bit_length() for m in msgs + joins for z in m.ring_pedersen_proof.Z[:M]))
        c.yl = _limbs_for(max([j.composite_dlog_proof_base_h1.y.bit_length() for j in joins] +
                              [j.composite_dlog_proof_base_h2.y.bit_length() for j in joins] + [1]))
        k = self._k
        c.recv_n = k(pack([x.n for x in recv_keys], nl))
        c.recv_ntilde = k(pack([s.N for s in recv_dlog], nl))
        c.recv_h1 = k(pack([s.g for s in recv_dlog], nl))
        c.recv_h2 = k(pack([s.ni for s in recv_dlog], nl))
        c.enc = k(pack([m.points_encrypted_vec[i] for m in msgs for i in range(n)], 2 * nl))
        c.commit = k(pack_points([m.points_committed_vec[i] for m in msgs for i in range(n)]))
        c.pdl_z = k(pack([p.z for p in pdl], nl))
        c.pdl_u1 = k(pack_points([p.u1 for p in pdl]))
        c.pdl_u2 = k(pack([p.u2 for p in pdl], 2 * nl))
        c.pdl_u3 = k(pack([p.u3 for p in pdl], nl))
        c.pdl_s1 = k(pack([p.s1 for p in pdl], c.s1l))
        c.pdl_s2 = k(pack([p.s2 for p in pdl], nl))
        c.pdl_s3 = k(pack([p.s3 for p in pdl], c.s3l))
        c.rp_z = k(pack([a.z for a in rng], nl))
        c.rp_e = k(pack([a.e for a in rng], c.el))
        c.rp_s = k(pack([a.s for a in rng], nl))
        c.rp_s1 = k(pack([a.s1 for a in rng], c.s1l))
        c.rp_s2 = k(pack([a.s2 for a in rng], c.s3l))
        t = local_key.t
        vss = []
        for m in msgs:
            com = list(m.coefficients_committed_vec.commitments)
            if len(com) != t + 1:
                raise UnsupportedInput("commitment vector length != t+1")
            vss += com
        c.vss = k(pack_points(vss))
        all_m = msgs + joins
        c.ped_S = k(pack([m.ring_pedersen_statement.S for m in all_m], nl))
        c.ped_T = k(pack([m.ring_pedersen_statement.T for m in all_m], nl))
        c.ped_N = k(pack([m.ring_pedersen_statement.N for m in all_m], nl))
        c.ped_A = k(pack([a for m in all_m for a in m.ring_pedersen_proof.A[:M]], nl))
        c.ped_Z = k(pack([z for m in all_m for z in m.ring_pedersen_proof.Z[:M]], c.zl))
        c.ck_n = k(pack([m.ek.n for m in all_m], nl))
        c.ck_sigma = k(pack([s for m in all_m for s in m.dk_correctness_proof.sigma_vec[:M2]], nl))
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
