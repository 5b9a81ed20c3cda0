#!/usr/bin/env python3
"""MAC share of each kernel's 64-bit integer VALU instructions, from the gfx950
disassembly of libfsdkr.so.

SQ_INSTS_VALU_INT64 counts every 64-bit integer VALU instruction: the
v_mad_u64_u32 MACs of the Montgomery rows and also their 64-bit carry shifts
and adds (v_lshrrev_b64, v_lshl_add_u64, v_lshlrev_b64).  The PMC cannot tell
them apart, the disassembly can: a product's VALU work is its cycle loop
(mont29.hpp product(): G trips of L unrolled CIOS rows, or KR/L trips in the
wave shape), so the MAC share of a kernel's INT64 instructions is the share in
its cycle loops -- every innermost loop holding >= 8 v_mad_u64_u32.  A kernel
has several (squaring cycles issue fewer a*b MACs than multiply cycles); the
SMALLEST loop share is taken, a lower bound for any mix of them.  The INT64
work outside the cycle loops (finish(), window steps) is < 1 % of a product's
(GA's slide kernel: 18 of 2338 INT64 instructions per 4096-bit squaring), and
is not credited; neither are the long-lane shapes' rolling-normalisation folds
(L > 30: one v_mad_u64_u32 by 8 per fold point and row, folds_per_cycle).
Kernels with no cycle loop (inverses, secp256k1, hashing) get their
whole-body share of v_mad_u64_u32 among INT64 instructions.

    pmc_mac = sum_k  SQ_INSTS_VALU_INT64[k] x mac_share[k]   (x 64 lanes)

Usage: mac_share.py [--lib fs-dkr_amd/fsdkr/libfsdkr.so] [--out FILE.json]"""
import argparse
import collections
import glob
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
INT64 = ("v_mad_u64_u32", "v_lshl_add_u64", "v_lshrrev_b64", "v_lshlrev_b64", "v_ashrrev_i64", "v_mad_i64_i32")
MAC = "v_mad_u64_u32"


def disassemble(lib):
    """{mangled kernel name: [(address, opcode, line)]} of every gfx950 code object in lib"""
    tmp = tempfile.mkdtemp(prefix="macshare")
    try:
        shutil.copy(lib, os.path.join(tmp, "lib.so"))
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", "lib.so"], cwd=tmp, check=True,
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        funcs = {}
        for co in sorted(glob.glob(os.path.join(tmp, "*gfx950"))):
            txt = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True,
                                 capture_output=True, text=True).stdout
            cur = None
            for line in txt.splitlines():
                m = re.match(r"^([0-9a-f]+) <(.+)>:", line)
                if m:
                    cur = m.group(2)
                    funcs[cur] = []
                    continue
                m = re.match(r"^\s+(\S+)(.*?)//\s*([0-9A-F]+):", line)
                if cur is not None and m:
                    funcs[cur].append((int(m.group(3), 16), m.group(1), line))
        return funcs
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def loops(ins):
    """(start index, end index) of every backward branch's body"""
    where = {a: k for k, (a, _, _) in enumerate(ins)}
    out = []
    for k, (a, op, line) in enumerate(ins):
        if not (op.startswith("s_cbranch") or op == "s_branch"):
            continue
        m = re.search(r"<[^+>]+\+0x([0-9a-f]+)>", line)
        if not m:
            continue
        tgt = ins[0][0] + int(m.group(1), 16)
        if tgt < a and tgt in where:
            out.append((where[tgt], k))
    return out


GROUP_KERNELS = ("modexp_kernel", "modexp_slide_kernel", "modexp_tail_kernel", "comb_build_kernel", "comb_exp_kernel",
                 "fb_exp_kernel", "fb_table_kernel", "eq_check_kernel", "prod3_kernel")


def folds_per_cycle(name):
    """v_mad_u64_u32 of a cycle loop that are NOT products: the rolling
    normalisation of long lanes (mont29.hpp NORM_IN_CYCLE: L > 30, NROLL folds per
    row, a multiply by 8 that moves a column's high word) -- L rows per cycle"""
    m = re.match(r"(\w+)<(\d+), (\d+)", name)
    if not m or m.group(1) not in GROUP_KERNELS:
        return 0
    L = int(m.group(2)) // int(m.group(3))
    return L * ((L + 17) // 18 - 1) if L > 30 else 0


def share(ins, name=""):
    """(mac share of INT64, how, per-loop detail)"""
    fold = folds_per_cycle(name)
    cyc = []
    lp = loops(ins)
    for s, e in lp:
        inner = any(s <= s2 and e2 <= e and (s2, e2) != (s, e) for s2, e2 in lp)
        c = collections.Counter(op for _, op, _ in ins[s:e + 1])
        if c[MAC] >= 8 and not inner:
            i64 = sum(c[x] for x in INT64)
            cyc.append({"v_mad_u64_u32": c[MAC], "roll_folds": fold, "int64": i64,
                        "valu": sum(v for k, v in c.items() if k.startswith("v_")), "share": (c[MAC] - fold) / i64})
    if cyc:
        return min(x["share"] for x in cyc), "min over cycle loops", cyc
    c = collections.Counter(op for _, op, _ in ins)
    i64 = sum(c[x] for x in INT64)
    return (c[MAC] / i64 if i64 else 0.0), "whole body", []


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
    return dict(zip(names, out))


def short(d):
    return d.replace("void ", "").replace("fsdkr::", "").split("(")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(REPO, "fs-dkr_amd", "fsdkr", "libfsdkr.so"))
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    funcs = disassemble(a.lib)
    dm = demangle(list(funcs))
    res = {}
    for name, ins in funcs.items():
        if not ins or name.startswith("__"):
            continue
        s, how, cyc = share(ins, short(dm[name]))
        res[short(dm[name])] = {"mac_share_of_int64": round(s, 4), "how": how,
                                "cycle_loops": [{k: (round(v, 4) if isinstance(v, float) else v) for k, v in x.items()}
                                                for x in cyc]}
    out = {"lib": os.path.relpath(a.lib, REPO), "int64_opcodes": list(INT64), "kernels": dict(sorted(res.items()))}
    txt = json.dumps(out, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")
    else:
        sys.stdout.write(txt + "\n")


if __name__ == "__main__":
    main()
