"""CPU restatement of Leo-Li009/fs-dkr's key-refresh hot path — TEST INFRASTRUCTURE ONLY.

This package is the parity oracle.  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import it, and only as the checker / the CPU
baseline — never as the thing measured or shipped.  The product path
(fs-dkr_amd/) never imports it and has no CPU fallback.

Each module restates one reference file (cited file:line, reference mounted
read-only at /root/reference) or one un-vendored dependency whose published
algorithm is restated from the pinned version named in the module header:

  bigint.py            curv-kzen 0.10 BigInt (GMP backend) semantics
  hashing.py           curv DigestExt::chain_bigint / zk-paillier compute_digest
  rng.py               seeded replacement for curv sample_below / sample_range (OS RNG in the reference)
  secp256k1.py         curv Point/Scalar<Secp256k1>
  paillier.py          kzen-paillier 0.4.3
  vss.py               curv VerifiableSS (Feldman) + Lagrange map
  zk_paillier.py       zk-paillier 0.4.4 NiCorrectKeyProof, CompositeDLogProof
  zk_pdl_with_slack.py src/zk_pdl_with_slack.rs
  range_proofs.py      src/range_proofs.rs (AliceProof)
  ring_pedersen.py     src/ring_pedersen_proof.rs
  protocol.py          src/refresh_message.rs, src/add_party_message.rs, src/error.rs

Parity status: the reference (Rust) cannot be built here (no cargo/rustc, no
network, dependencies un-vendored) and its tests hold no golden
vectors, so byte-level encodings of the third-party crates are PARITY UNPINNED
(marked [dep, unverified] where they occur).  The restatement is pinned against
the reference's own tests (round-trip acceptance + the x+1 soundness vector,
tests/test_oracle_reference_tests.py) and against GMP / hashlib / secp256k1
known answers (tests/test_oracle_kat.py).
"""
