#!/usr/bin/env python3
"""Key generation throughput: `count` 2048-bit Paillier keypairs
plus their NiCorrectKeyProof in one batched call (fsdkr.keygen.refresh_keys),
and single-key latency (keypair_with_modulus_size, the distribute() path).
CPU side for context: the oracle's walk over GMP (1 thread)."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fs-dkr_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bits", type=int, default=2048)
    ap.add_argument("--count", type=int, default=64)
    ap.add_argument("--cpu-keys", type=int, default=2)
    a = ap.parse_args()
    import torch  # noqa: F401
    from fsdkr import Context, keygen
    from oracle import keygen as ok
    from oracle.rng import Rng
    ctx = Context()
    keygen.refresh_keys(ctx, Rng("warm"), a.bits, 2)
    t0 = time.perf_counter()
    keys = keygen.refresh_keys(ctx, Rng("batch"), a.bits, a.count)
    batch_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    for k in range(4):
        keygen.keypair_with_modulus_size(ctx, Rng(("one", k)), a.bits)
    single_s = (time.perf_counter() - t0) / 4
    t0 = time.perf_counter()
    ok.keypairs_with_modulus_size(Rng("cpu"), a.bits, a.cpu_keys)
    cpu_s = (time.perf_counter() - t0) / a.cpu_keys
    assert len(keys) == a.count and all(ek.n.bit_length() == a.bits for ek, _, _ in keys)
    print(json.dumps({"keygen_bits": a.bits, "batch_keys": a.count, "batch_s": batch_s,
                      "batch_keys_per_s": a.count / batch_s, "single_keypair_s": single_s,
                      "cpu_oracle_keypair_s_1t": cpu_s,
                      "note": "batch = keypairs + correct-key proofs (refresh_keys); single = one keypair (distribute path)"}))


if __name__ == "__main__":
    main()
