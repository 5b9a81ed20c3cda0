"""group_by_exponent (fs-dkr_amd/csrc/ctx.hpp) on the CPU: the regrouping that
lays a modexp job out receiver-major so every wave's instances share their
exponent (GA's sliding windows, job 1).  Its output must be the stable order by
exponent address, each run of one exponent padded to whole waves when a pad row
is given (pads repeat the run's last instance and write the pad row, or their
own row for kPadSelf), and `aligned` must say whether every run fills whole
waves.  Checked against a Python restatement on random jobs."""
import os
import random
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NO_PAD, PAD_SELF = 0xFFFFFFFF, 0xFFFFFFFE


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    out = tmp_path_factory.mktemp("gbe") / "group_by_exponent_host"
    subprocess.run(["g++", "-O2", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I", "/opt/rocm/include",
                    "-I", os.path.join(REPO, "fs-dkr_amd", "csrc"),
                    os.path.join(REPO, "tests", "native", "group_by_exponent_host.cpp"), "-o", str(out)], check=True)
    return str(out)


def expected(per_wave, pad, inst):
    """(aligned, [(src, row, key)]) -- the restatement"""
    order = sorted(range(len(inst)), key=lambda k: inst[k][0])   # stable by address
    runs, s = [], 0
    while s < len(order):
        e = s
        while e < len(order) and inst[order[e]] == inst[order[s]]:
            e += 1
        runs.append(order[s:e])
        s = e
    aligned = per_wave > 0
    if pad == NO_PAD:
        aligned = aligned and all(len(r) % per_wave == 0 for r in runs)
    out = []
    for r in runs:
        out += [(k, k, inst[k][0]) for k in r]
        if aligned and pad != NO_PAD:
            q = len(r)
            while q % per_wave:
                last = r[-1]
                out.append((last, last if pad == PAD_SELF else pad, inst[last][0]))
                q += 1
    return aligned, out


def run(exe, per_wave, pad, inst):
    txt = f"{per_wave} {pad} {len(inst)}\n" + "\n".join(f"{k} {l}" for k, l in inst) + "\n"
    r = subprocess.run([exe], input=txt, capture_output=True, text=True, check=True)
    lines = r.stdout.split("\n")
    return lines[0] == "1", [tuple(int(x) for x in ln.split()) for ln in lines[1:] if ln.strip()]


@pytest.mark.parametrize("seed", range(6))
def test_matches_restatement(exe, seed):
    rnd = random.Random(seed)
    keys = [0x7F0000000000 + 4096 * rnd.randrange(1, 10_000) for _ in range(rnd.choice([1, 3, 64, 300]))]
    for per_wave, pad in ((4, 999_999), (16, PAD_SELF), (8, NO_PAD), (0, NO_PAD), (4, NO_PAD)):
        n = rnd.choice([1, 7, 120, 4000])
        if pad == NO_PAD and per_wave and seed % 2:   # whole runs: aligned
            inst = [(keys[k // per_wave % len(keys)], 64) for k in range(per_wave * max(1, n // per_wave))]
            rnd.shuffle(inst)
        else:
            inst = [(rnd.choice(keys), rnd.choice([64, 64, 64, 32])) for _ in range(n)]
        assert run(exe, per_wave, pad, inst) == expected(per_wave, pad, inst), (seed, per_wave, pad)
