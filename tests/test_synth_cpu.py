"""Host logic of the synthetic workload generator (fsdkr.synth) on the CPU:
the generator is driven through a stand-in context whose modexp / MSM calls
are answered by the oracle, and the oracle then verifies every generated
proof.  (The GPU run of the same generator is tests/test_synth_gpu.py.)"""
import pytest

from oracle import bigint
from oracle import secp256k1 as ec


class OracleCtx:
    """Same call surface as fsdkr.Context for the methods synth uses (test only)."""

    def modexp_batch(self, bases, exps, mods, mod_idx, mod_limbs):
        return [bigint.mod_pow(b, e, mods[i]) for b, e, i in zip(bases, exps, mod_idx)]

    def ec_msm(self, points, scalars):
        out = []
        for row_p, row_s in zip(points, scalars):
            acc = None
            for p, s in zip(row_p, row_s):
                assert 0 <= s < 1 << 256
                if p is not None:
                    acc = ec.add(acc, ec.mul(p, s))
            out.append(acc)
        return out


def _verify_all(msgs, joins, lk, M=256):
    from oracle import protocol, range_proofs, ring_pedersen, zk_pdl_with_slack as pdl
    from oracle.vss import VerifiableSS
    from oracle.zk_paillier import CompositeDLogProof, DLogStatement, NiCorrectKeyProof
    n = len(msgs) + len(joins)
    for m in msgs:
        v = m.coefficients_committed_vec
        m.coefficients_committed_vec = VerifiableSS(v.threshold, v.share_count, list(v.commitments))
    protocol.validate_collect(msgs, lk.t, n)
    for m in msgs:
        for i in range(n):
            st = pdl.PDLwSlackStatement(m.points_encrypted_vec[i], lk.paillier_key_vec[i], m.points_committed_vec[i],
                                        ec.G, lk.h1_h2_n_tilde_vec[i].g, lk.h1_h2_n_tilde_vec[i].ni,
                                        lk.h1_h2_n_tilde_vec[i].N)
            pdl.verify(m.pdl_proof_vec[i], st)
            assert range_proofs.verify(m.range_proofs[i], st.ciphertext, st.ek, lk.h1_h2_n_tilde_vec[i])
    for m in msgs + joins:
        assert ring_pedersen.verify(m.ring_pedersen_proof, m.ring_pedersen_statement, M)
        assert NiCorrectKeyProof(m.dk_correctness_proof.sigma_vec).verify(m.ek.n)
    for j in joins:
        st = DLogStatement(j.dlog_statement.N, j.dlog_statement.g, j.dlog_statement.ni)
        assert CompositeDLogProof(j.composite_dlog_proof_base_h1.x, j.composite_dlog_proof_base_h1.y).verify(st)
        st2 = DLogStatement(st.N, st.ni, st.g)
        assert CompositeDLogProof(j.composite_dlog_proof_base_h2.x, j.composite_dlog_proof_base_h2.y).verify(st2)


@pytest.mark.parametrize("R,J,t", [(3, 0, 1), (3, 1, 1)])
def test_synth_host_logic(R, J, t):
    from fsdkr import synth
    msgs, joins, lk = synth.synth_collect(OracleCtx(), R=R, J=J, t=t, seed=11, key_bits=1024)
    assert len(msgs) == R and len(joins) == J
    _verify_all(msgs, joins, lk)
