"""Interleaved A/B of the metric-2 modexp launch: fixed windows over per-instance
exponent rows (fsdkr_modexp_batch_device) against the keyed sliding-window launch
(fsdkr_modexp_keyed_device).  One JSON line per measurement."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from fsdkr import Context  # noqa: E402


def main():
    count = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    import torch
    torch.cuda.set_device(0)   # torch's HIP runtime first (bench.py's order), then the context
    ctx = Context(device=0, timing=True)
    for r in range(rounds):
        for keyed in (False, True):
            out = bench.modexp_roofline(ctx, count, 3, keyed=keyed)
            out["round"] = r
            out["achieved_frac"] = out["achieved_mac_per_s"] / bench.PEAK_MAC
            out["issued_frac"] = out["issued_mac_per_s"] / bench.PEAK_MAC
            print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
