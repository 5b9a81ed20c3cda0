"""tools/mac_share.py (the MAC share of each kernel's 64-bit VALU instructions,
from the gfx950 disassembly) on the built libfsdkr.so: the product cycle loops
are found and their v_mad_u64_u32 counts match mont29.hpp's row structure
(squaring rows: (L+1)/2 or L/2+1 a*b MACs + L m*n MACs + the long lanes'
rolling folds, which are not credited)."""
import importlib.util
import os
import shutil

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "fs-dkr_amd", "fsdkr", "libfsdkr.so")


def _tool():
    spec = importlib.util.spec_from_file_location("mac_share", os.path.join(REPO, "tools", "mac_share.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.fixture(scope="module")
def shares():
    if not os.path.exists(LIB) or not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump") or not shutil.which("c++filt"):
        pytest.skip("needs the built library and the ROCm llvm-objdump")
    t = _tool()
    funcs = t.disassemble(LIB)
    dm = t.demangle(list(funcs))
    return {t.short(dm[k]): t.share(v, t.short(dm[k])) for k, v in funcs.items() if v}


def _rows(KD, G, sq):
    L = KD // G
    ab = ((L + 1) // 2 if L % 2 else L // 2 + 1) if sq else L
    fold = ((L + 17) // 18 - 1) if L > 24 else 0
    return L * (ab + L + fold), L * fold


@pytest.mark.parametrize("kernel,KD,G", [("modexp_slide_kernel<144, 16, 128, true>", 144, 16),
                                          ("modexp_kernel<72, 8, 64, false, true>", 72, 8),
                                          ("modexp_kernel<144, 4, 128, false, true>", 144, 4)])
def test_cycle_loops_match_row_structure(shares, kernel, KD, G):
    s, how, cyc = shares[kernel]
    assert how == "min over cycle loops"
    mads = {c["v_mad_u64_u32"] for c in cyc}
    sq, fold = _rows(KD, G, True)
    mul, _ = _rows(KD, G, False)
    assert mul in mads
    assert sq in mads or sq + 1 in mads     # (+1: a loop-carried address MAC in one variant)
    for c in cyc:
        assert c["roll_folds"] == fold
    assert 0.8 < s < 1.0


def test_no_credit_above_the_mac_count(shares):
    for k, (s, how, cyc) in shares.items():
        assert 0.0 <= s <= 1.0, k
