"""The GPU-generated synthetic workload (fsdkr.synth, used by bench.py) is a
valid collect() input: the oracle accepts every proof and the GPU verifier
returns no error."""
import pytest

from oracle import protocol
from oracle.vss import VerifiableSS as OracleVSS

pytestmark = pytest.mark.gpu


def _to_oracle(msgs):
    for m in msgs:
        v = m.coefficients_committed_vec
        m.coefficients_committed_vec = OracleVSS(v.threshold, v.share_count, list(v.commitments))
    return msgs


def test_synth_collect_valid(gpu_ctx):
    from fsdkr import refresh, synth
    msgs, joins, lk = synth.synth_collect(gpu_ctx, R=4, J=1, t=1, seed=7, key_bits=1024)
    err, applied, _ = refresh.verify(msgs, lk, joins, ctx=gpu_ctx, key_bits=1024)
    assert err is None and applied == 5
    # the oracle's verification half of collect() accepts the same messages
    om = _to_oracle(msgs)
    protocol.validate_collect(om, lk.t, 5)
    from oracle import range_proofs, ring_pedersen, zk_pdl_with_slack as pdl
    from oracle import secp256k1 as ec
    for m in om:
        for i in range(5):
            st = pdl.PDLwSlackStatement(m.points_encrypted_vec[i], lk.paillier_key_vec[i], m.points_committed_vec[i],
                                        ec.G, lk.h1_h2_n_tilde_vec[i].g, lk.h1_h2_n_tilde_vec[i].ni,
                                        lk.h1_h2_n_tilde_vec[i].N)
            pdl.verify(m.pdl_proof_vec[i], st)
            assert range_proofs.verify(m.range_proofs[i], st.ciphertext, st.ek, lk.h1_h2_n_tilde_vec[i])
    for m in om + joins:
        assert ring_pedersen.verify(m.ring_pedersen_proof, m.ring_pedersen_statement, 256)
        assert m.dk_correctness_proof.__class__.__name__ == "NiCorrectKeyProof"
    from oracle.zk_paillier import CompositeDLogProof, DLogStatement, NiCorrectKeyProof
    for m in om + joins:
        assert NiCorrectKeyProof(m.dk_correctness_proof.sigma_vec).verify(m.ek.n)
    j = joins[0]
    st = DLogStatement(j.dlog_statement.N, j.dlog_statement.g, j.dlog_statement.ni)
    assert CompositeDLogProof(j.composite_dlog_proof_base_h1.x, j.composite_dlog_proof_base_h1.y).verify(st)
    st2 = DLogStatement(st.N, st.ni, st.g)
    assert CompositeDLogProof(j.composite_dlog_proof_base_h2.x, j.composite_dlog_proof_base_h2.y).verify(st2)
