"""The C++ CPU baseline (oracle/cpu_baseline.cpp, bench.py's cpu_baseline leg)
agrees with the Python oracle instance by instance on the golden transcripts,
valid and tampered (CPU only: it reads the product's packed batch)."""
import copy
import dataclasses
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "golden"), HERE]

import codec  # noqa: E402


def _lib_or_skip():
    from oracle import cpu_baseline as cb
    try:
        cb.lib()
    except (ImportError, OSError) as e:
        pytest.skip(f"C++ baseline unavailable: {e}")
    return cb


@pytest.mark.parametrize("name", ["transcript_t2_n5_kb1024.json.gz", "transcript_join_t1_n4_kb1024.json.gz"])
def test_cpu_baseline_matches_oracle(name):
    cb = _lib_or_skip()
    from fsdkr.batch import CollectBatch
    from oracle_device import OracleDevice
    raw = codec.load_raw(name)
    d = {k: codec.dec(raw[k], codec.product_classes()) for k in ("keys", "msgs", "joins")}
    kb = raw["meta"]["key_bits"]
    msgs, joins = copy.deepcopy(d["msgs"]), d["joins"]
    key = d["keys"][1 if joins else 0]
    p = msgs[1].pdl_proof_vec[2]
    msgs[1].pdl_proof_vec[2] = dataclasses.replace(p, s3=p.s3 + 1)
    a = msgs[2].range_proofs[0]
    msgs[2].range_proofs[0] = dataclasses.replace(a, s2=a.s2 + 1)
    msgs[0].points_committed_vec[1] = msgs[0].points_committed_vec[2]
    b = CollectBatch(msgs, key, joins, 256, kb)
    R, J, n = b.R, b.J, b.n
    v, secs = cb.verify(b, R * n, R + J, J, R * n, 4)
    ocls = codec.oracle_classes()
    od = {k: codec.dec(raw[k], ocls) for k in ("keys",)}
    import tamper
    om = tamper.to_oracle(msgs, joins) if joins else (tamper.to_oracle(msgs), [])
    want = OracleDevice(om[0], om[1], od["keys"][1 if joins else 0]).collect_finish(None)
    assert np.array_equal(v["pdl"][:R * n], want.pdl)
    assert np.array_equal(v["range"][:R * n], want.range)
    assert np.array_equal(v["feldman"][:R * n], want.feldman)
    assert np.array_equal(v["ped"][:R + J], want.ped)
    assert np.array_equal(v["ck"][:R + J], want.ck)
    if J:
        assert np.array_equal(v["dlog"][:J], want.dlog[:J])
    assert want.pdl[1 * n + 2] != 7 and want.range[2 * n + 0] == 0 and want.feldman[1] == 0
