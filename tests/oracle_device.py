"""An oracle-backed stand-in for the GPU context (TEST INFRASTRUCTURE ONLY).

CPU tests of the host orchestration around the C ABI (sharding, verdict
all-reduce, first-error mapping, side effects, speculative share recovery:
fsdkr.shard.collect) run without a GPU by giving that code this object in
place of fsdkr.Context.  It answers each device call with the oracle's
restatement of the reference: collect_finish returns the verdicts the oracle
computes for the prepared slice, paillier_decrypt_many / ec_msm /
feldman_check compute with oracle.paillier / oracle.secp256k1 / oracle.vss.
The product never sees it; GPU tests exercise the real kernels."""
import numpy as np

from oracle import bigint, paillier, range_proofs, ring_pedersen
from oracle import secp256k1 as ec
from oracle import zk_pdl_with_slack as pdl
from oracle.vss import VerifiableSS
from oracle.zk_paillier import CompositeDLogProof, DLogStatement, NiCorrectKeyProof

M = 256


class OracleDevice:
    def __init__(self, msgs, joins, lk, world=1, rank=0):
        self.msgs, self.joins, self.lk = list(msgs), list(joins), lk
        self.world, self.rank = world, rank
        self._batch = None

    # ---- collect pipeline --------------------------------------------------
    def collect_prepare(self, batch):
        self._batch = batch

    def collect_launch(self):
        assert self._batch is not None

    def collect_finish(self, batch):
        from fsdkr.batch import Verdicts
        from fsdkr.shard import shard_range
        R, J = len(self.msgs), len(self.joins)
        n = R + J
        r0, r1 = shard_range(R, self.world, self.rank)
        j0, j1 = shard_range(J, self.world, self.rank)
        sm, sj = self.msgs[r0:r1], self.joins[j0:j1]
        v = Verdicts(len(sm), len(sj), n)
        lk = self.lk
        for k, m in enumerate(sm):
            vss = VerifiableSS(lk.t, n, list(m.coefficients_committed_vec.commitments))
            for i in range(n):
                p = k * n + i
                v.feldman[p] = 1 if vss.validate_share_public(m.points_committed_vec[i], i + 1) else 0
                st = pdl.PDLwSlackStatement(m.points_encrypted_vec[i], lk.paillier_key_vec[i],
                                            m.points_committed_vec[i], ec.G, lk.h1_h2_n_tilde_vec[i].g,
                                            lk.h1_h2_n_tilde_vec[i].ni, lk.h1_h2_n_tilde_vec[i].N)
                try:
                    pdl.verify(m.pdl_proof_vec[i], st)
                    bits = 7
                except pdl.PDLwSlackError as e:
                    bits = (1 if e.flags[0] else 0) | (2 if e.flags[1] else 0) | (4 if e.flags[2] else 0)
                v.pdl[p] = bits
                v.range[p] = 1 if range_proofs.verify(m.range_proofs[i], st.ciphertext, st.ek,
                                                      lk.h1_h2_n_tilde_vec[i]) else 0
        for q, m in enumerate(sm + sj):
            try:
                v.ped[q] = 1 if ring_pedersen.verify(m.ring_pedersen_proof, m.ring_pedersen_statement, M) else 0
            except bigint.PanicError:
                v.ped[q] = 2
            v.ck[q] = 1 if NiCorrectKeyProof(tuple(m.dk_correctness_proof.sigma_vec)).verify(m.ek.n) else 0
        for q, j in enumerate(sj):
            st = DLogStatement(j.dlog_statement.N, j.dlog_statement.g, j.dlog_statement.ni)
            st2 = DLogStatement(st.N, st.ni, st.g)
            a = CompositeDLogProof(j.composite_dlog_proof_base_h1.x, j.composite_dlog_proof_base_h1.y).verify(st)
            b = CompositeDLogProof(j.composite_dlog_proof_base_h2.x, j.composite_dlog_proof_base_h2.y).verify(st2)
            v.dlog[q] = (1 if a else 0) | (2 if b else 0)
        self._batch = None
        return v

    # ---- share recovery ----------------------------------------------------
    def paillier_decrypt_many(self, cts, key_idx, ps, qs, nl):
        return [paillier.decrypt(paillier.DecryptionKey(ps[k], qs[k]), c) for c, k in zip(cts, key_idx)]

    def collect_recover(self, jobs):
        """fsdkr_collect_recover restated: Lagrange weights (oracle.vss), the
        oracle's decryption, share = sum l_k m_k mod N mod q, y and pk_vec."""
        from oracle.vss import map_share_to_new_params
        out = []
        for j in jobs:
            idx = [x - 1 for x in j["old_index"]]
            li = [map_share_to_new_params(idx[k], idx) for k in range(len(idx))]
            pk = self.ec_msm(j["points"], [li[:len(row)] for row in j["points"]])
            status = 1 if j["t_key"] > j["t_vss"] else 0
            if j.get("flags", 0) & 1:   # FSDKR_RECOVER_NO_DECRYPT: the pk_vec rows only
                out.append((status, 0, None, pk))
                continue
            dk = paillier.DecryptionKey(j["p"], j["q"])
            ms = [paillier.decrypt(dk, c) for c in j["cts"]]
            share = sum(l * m for l, m in zip(li, ms)) % (j["p"] * j["q"]) % ec.Q
            out.append((status, share, ec.mul(ec.G, share), pk))
        return out

    def collect_recover_launch(self, jobs):
        return list(jobs)

    def collect_recover_finish(self, handle):
        return self.collect_recover(handle)

    def ec_msm(self, rows, scs):
        out = []
        for row, sc in zip(rows, scs):
            acc = None
            for pt, s in zip(row, sc):
                if pt is not None:
                    acc = ec.add(acc, ec.mul(pt, s % ec.Q))
            out.append(acc)
        return out

    def feldman_check(self, vss, commit, n, t):
        out = np.zeros(len(commit), np.uint8)
        for k, com in enumerate(vss):
            v = VerifiableSS(t, n, list(com))
            for i in range(n):
                out[k * n + i] = 1 if v.validate_share_public(commit[k * n + i], i + 1) else 0
        return out
