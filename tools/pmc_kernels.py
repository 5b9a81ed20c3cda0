#!/usr/bin/env python3
"""Per-kernel summary of one rocprofv3 --pmc pass over a collect() pipeline run
(tools/gpu_r03o.sh): per dispatch of each kernel, the SQ counters averaged, and
the derived issue split (VALU instructions, 64-bit integer share, time issuing
vs waiting on instruction dependencies)."""
import collections
import csv
import json
import sys


def main(path):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("fsdkr::", "")
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    out = {}
    for k, c in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        n = max(1, len(disp[k]))
        d = {name: v / n for name, v in c.items()}
        wc = d.get("SQ_WAVE_CYCLES", 0) or 1
        valu = d.get("SQ_INSTS_VALU", 0) or 1
        out[k] = {"dispatches": n, "waves": d.get("SQ_WAVES"), "valu_insts": d.get("SQ_INSTS_VALU"),
                  "int64_share": d.get("SQ_INSTS_VALU_INT64", 0) / valu,
                  "active_valu_frac": d.get("SQ_ACTIVE_INST_VALU", 0) / wc,
                  "wait_inst_frac": d.get("SQ_WAIT_INST_ANY", 0) / wc,
                  "busy_cycles": d.get("SQ_BUSY_CYCLES")}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
