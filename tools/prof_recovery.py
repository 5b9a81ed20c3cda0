#!/usr/bin/env python3
"""Where the share recovery of collect_many goes for S sessions (configs[4]):
recovery plans (host), batched GPU decryption (fsdkr_paillier_decrypt_multi),
the combine + pk_vec MSM (fsdkr_ec_msm).  Diagnostics for DESIGN.md."""
import copy
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fs-dkr_amd")]


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    import torch  # noqa: F401
    from fsdkr import Context, synth
    from fsdkr import refresh as rf
    ctx = Context()
    sess = synth.synth_sessions(ctx, S, n=3, t=1, seed=9, key_bits=3072)
    jobs = [(m, copy.deepcopy(lk), len(m) + len(j)) for (m, j, lk, dk) in sess]
    for rep in range(3):
        t0 = time.perf_counter()
        plans = [rf._recovery_plan(m, lk, nn) for m, lk, nn in jobs]
        t1 = time.perf_counter()
        cts, kidx, ps, qs = [], [], [], []
        for p, (m, lk, nn) in zip(plans, jobs):
            for c in p["cts"]:
                cts.append(c)
                kidx.append(len(ps))
            ps.append(lk.paillier_dk.p)
            qs.append(lk.paillier_dk.q)
        sig = ctx.paillier_decrypt_many(cts, kidx, ps, qs, 96)
        t2 = time.perf_counter()
        sig_of, at = {}, 0
        for j, p in enumerate(plans):
            sig_of[j] = sig[at:at + len(p["cts"])]
            at += len(p["cts"])
        rf._finish_recovery(ctx, plans, sig_of)
        t3 = time.perf_counter()
        t4 = time.perf_counter()
        rf._speculative(ctx, jobs)
        t5 = time.perf_counter()
        print(json.dumps({"sessions": S, "plans_ms": (t1 - t0) * 1e3, "decrypt_ms": (t2 - t1) * 1e3,
                          "combine_msm_ms": (t3 - t2) * 1e3, "speculative_ms": (t5 - t4) * 1e3}), flush=True)


if __name__ == "__main__":
    main()
