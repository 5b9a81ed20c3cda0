#!/usr/bin/env python3
"""Summarise the rocprofv3 --pmc passes of tools/pmc.sh into one JSON object per
kernel (per-launch values: sums over the dispatches of that kernel / dispatch
count).  HBM traffic follows /opt/skills/guides/MI355X_MICROARCH.md (HBM
section): FETCH_SIZE and WRITE_SIZE come from separate passes, both in KiB;
on gfx950 FETCH_SIZE reports half the bytes of wide reads, so it is doubled
(the guide's correction; our table reads are 4 B/lane, an access width the
guide leaves uncalibrated, so the raw value is kept beside it)."""
import argparse
import collections
import csv
import json
import os


def load(pass_dir, kernel_sub):
    vals = collections.defaultdict(float)
    dispatches = collections.defaultdict(set)
    names = set()
    for r in csv.DictReader(open(os.path.join(pass_dir, "run_counter_collection.csv"))):
        if kernel_sub not in r["Kernel_Name"]:
            continue
        names.add(r["Kernel_Name"].split("(")[0].replace("void ", ""))
        vals[r["Counter_Name"]] += float(r["Counter_Value"])
        dispatches[r["Counter_Name"]].add(r["Dispatch_Id"])
    return {k: v / max(1, len(dispatches[k])) for k, v in vals.items()}, names


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="modexp_kernel<144, 4, 128, false>")
    ap.add_argument("--instances", type=int, default=65536)
    ap.add_argument("--macs-per-instance", type=float, default=80.86e6)
    a = ap.parse_args()
    per = {}
    names = set()
    for p in sorted(os.listdir(a.dir)):
        d = os.path.join(a.dir, p)
        if os.path.isdir(d) and os.path.exists(os.path.join(d, "run_counter_collection.csv")):
            v, nm = load(d, a.kernel)
            per.update(v)
            names |= nm
    fetch_raw = per.get("FETCH_SIZE", 0.0) * 1024
    write = per.get("WRITE_SIZE", 0.0) * 1024
    out = {"kernel": sorted(names), "instances": a.instances, "per_launch": per,
           "hbm_fetch_bytes_raw": fetch_raw, "hbm_fetch_bytes_corrected_x2": 2 * fetch_raw,
           "hbm_write_bytes": write, "hbm_traffic_bytes": 2 * fetch_raw + write}
    if "SQ_INSTS_VALU" in per:
        out["valu_insts_per_launch"] = per["SQ_INSTS_VALU"]
        out["int64_valu_fraction"] = per.get("SQ_INSTS_VALU_INT64", 0) / per["SQ_INSTS_VALU"]
        out["issued_mad_wave_insts"] = per.get("SQ_INSTS_VALU_INT64", 0)
    if "SQ_WAVE_CYCLES" in per:
        wc = per["SQ_WAVE_CYCLES"]
        out["wave_time_split"] = {"active_any": per.get("SQ_ACTIVE_INST_ANY", 0) / wc,
                                  "wait_inst_any": per.get("SQ_WAIT_INST_ANY", 0) / wc,
                                  "wait_any": per.get("SQ_WAIT_ANY", 0) / wc}
    if "TCC_HIT_sum" in per:
        out["l2_hit_rate"] = per["TCC_HIT_sum"] / max(1.0, per["TCC_HIT_sum"] + per["TCC_MISS_sum"])
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
