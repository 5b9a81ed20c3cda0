#!/usr/bin/env python3
"""How the share recovery (aux stream) overlaps the collect() device pipeline
at BASELINE configs[2]: device pipeline alone, launch+finish without recovery,
with overlapped recovery, recovery alone (decrypt / MSM split), whole collect().
Diagnostics for DESIGN.md; prints one JSON line per measurement."""
import argparse
import copy
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fs-dkr_amd")]
os.environ["GPU_MAX_HW_QUEUES"] = str(max(12, int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=64)
    ap.add_argument("--t", type=int, default=32)
    ap.add_argument("--joins", type=int, default=4)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch  # noqa: F401
    from fsdkr import Context, synth
    from fsdkr.batch import CollectBatch
    from fsdkr.refresh import _speculative, collect
    ctx = Context()
    R, J = a.n - a.joins, a.joins
    msgs, joins, lk = synth.synth_collect(ctx, R, J, a.t, 2024)
    job = [(msgs, lk, a.n)]
    b = CollectBatch(msgs, lk, joins, 256, 2048)
    ctx.collect_prepare(b)
    ctx.collect_run(b)
    _speculative(ctx, job)

    def ms(f, reps=a.reps):
        out = []
        for _ in range(reps):
            t0 = time.perf_counter()
            f()
            out.append((time.perf_counter() - t0) * 1e3)
        return round(min(out), 2)

    res = {"hw_queues": os.environ["GPU_MAX_HW_QUEUES"]}
    res["device_pipeline_ms"] = ms(lambda: ctx.collect_run(b))

    def no_rec():
        ctx.collect_launch()
        ctx.collect_finish(b)
    res["launch_finish_no_recovery_ms"] = ms(no_rec)

    def with_rec():
        ctx.collect_launch()
        _speculative(ctx, job)
        ctx.collect_finish(b)
    res["launch_recovery_finish_ms"] = ms(with_rec)

    def rec_after():
        ctx.collect_launch()
        ctx.collect_finish(b)
        _speculative(ctx, job)
    res["launch_finish_then_recovery_ms"] = ms(rec_after)
    res["recovery_alone_ms"] = ms(lambda: _speculative(ctx, job))
    import fsdkr.refresh as rf
    plans = [rf._recovery_plan(msgs, lk, a.n)]
    dk = lk.paillier_dk
    w = rf._dk_limbs(dk)
    res["decrypt_alone_ms"] = ms(lambda: ctx.paillier_decrypt_many(plans[0]["cts"], [0] * len(plans[0]["cts"]),
                                                                     [dk.p], [dk.q], w))
    sig = {0: ctx.paillier_decrypt_many(plans[0]["cts"], [0] * len(plans[0]["cts"]), [dk.p], [dk.q], w)}
    res["msm_and_combine_alone_ms"] = ms(lambda: rf._finish_recovery(ctx, [dict(plans[0])], sig))
    ks = [copy.deepcopy(lk) for _ in range(a.reps)]
    it = iter(ks)
    res["collect_ms"] = ms(lambda: collect(msgs, next(it), lk.paillier_dk, joins, ctx=ctx))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
