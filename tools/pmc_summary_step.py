#!/usr/bin/env python3
"""Counter totals per collect() call from a rocprofv3 --pmc pass over
tools/pmc_step.py (every dispatch belongs to one of CALLS collect() calls):
per counter the sum over all dispatches / CALLS, plus the per-kernel split of
SQ_INSTS_VALU_INT64.  With --ms (the call's wall time, e.g. bench.py's
ms_per_step) it adds the counter-based issue fraction
    pmc_issued_frac = SQ_INSTS_VALU_INT64 x 64 lanes / (ms x 3.40e13 lane-MAC/s)
i.e. the 64-bit integer VALU lane-operations the chip issued per call
(v_mad_u64_u32 MACs plus the few 64-bit carry shifts/adds of each Montgomery
row) against the measured v_mad_u64_u32 peak (profiles/r01_intrates.jsonl).
With --mac-share (tools/mac_share.py's JSON for the SAME libfsdkr.so) it adds
the MAC count: pmc_mac_per_call = sum over kernels of SQ_INSTS_VALU_INT64 x
that kernel's v_mad_u64_u32 share of its INT64 instructions (kernels absent
from the file are not credited).
Usage: pmc_summary_step.py COUNTER_CSV CALLS [--ms MS] [--label L] [--mac-share F]"""
import argparse
import collections
import csv
import json

PEAK = 3.40e13


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("calls", type=int)
    ap.add_argument("--ms", type=float, default=0.0)
    ap.add_argument("--label", default="")
    ap.add_argument("--mac-share", default="")
    a = ap.parse_args()
    tot = collections.defaultdict(float)
    per_kernel = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = set()
    for r in csv.DictReader(open(a.csv)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("fsdkr::", "")
        v = float(r["Counter_Value"])
        tot[r["Counter_Name"]] += v
        per_kernel[k][r["Counter_Name"]] += v
        disp.add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
    out = {"label": a.label, "source": a.csv, "calls": a.calls, "dispatches_per_call": len(disp) / a.calls,
           "per_call": {c: v / a.calls for c, v in sorted(tot.items())}}
    i64 = tot.get("SQ_INSTS_VALU_INT64", 0.0) / a.calls
    valu = tot.get("SQ_INSTS_VALU", 0.0) / a.calls
    if valu:
        out["int64_share_of_valu"] = i64 / valu
    if a.ms and i64:
        out["ms_per_call"] = a.ms
        out["pmc_issued_lane_ops"] = i64 * 64
        out["pmc_issued_frac"] = i64 * 64 / (a.ms * 1e-3 * PEAK)
    if "SQ_INSTS_VALU_INT64" in tot:
        ks = sorted(per_kernel.items(), key=lambda kv: -kv[1].get("SQ_INSTS_VALU_INT64", 0.0))
        out["int64_by_kernel"] = {k: {"int64_per_call": c.get("SQ_INSTS_VALU_INT64", 0.0) / a.calls,
                                      "int64_share": (c.get("SQ_INSTS_VALU_INT64", 0.0) / c["SQ_INSTS_VALU"])
                                      if c.get("SQ_INSTS_VALU") else None}
                                  for k, c in ks}
        if a.mac_share:
            ms = json.load(open(a.mac_share))["kernels"]
            mac = 0.0
            for k, c in out["int64_by_kernel"].items():
                r = ms.get(k, {}).get("mac_share_of_int64", 0.0)
                c["mac_share_of_int64"] = r
                mac += c["int64_per_call"] * r
            out["mac_share_source"] = a.mac_share
            out["pmc_mac_per_call"] = mac
            out["mac_share_of_int64"] = mac / i64 if i64 else None
            if a.ms:
                out["pmc_mac_frac"] = mac * 64 / (a.ms * 1e-3 * PEAK)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
