"""GPU parity of the batched modexp kernel against Python's exact pow()
(the arithmetic curv's BigInt::mod_pow performs via GMP mpz_powm)."""
import random

import pytest

pytestmark = pytest.mark.gpu

WIDTHS = [64, 96, 128, 192]


def _odd(rnd, bits):
    return rnd.getrandbits(bits) | 1 | (1 << (bits - 1))


@pytest.mark.parametrize("limbs", WIDTHS)
def test_modexp_random(gpu_ctx, limbs):
    rnd = random.Random(limbs)
    bits = 32 * limbs
    mods = [_odd(rnd, bits) for _ in range(5)] + [_odd(rnd, bits - 1), _odd(rnd, bits - 37)]
    count = 300
    idx = [rnd.randrange(len(mods)) for _ in range(count)]
    bases = [rnd.getrandbits(bits) for _ in range(count)]          # not reduced: may exceed N
    exps = [rnd.getrandbits(rnd.choice([1, 7, 64, 256, 769, 2048])) for _ in range(count)]
    got = gpu_ctx.modexp_batch(bases, exps, mods, idx, limbs)
    want = [pow(b, e, mods[i]) for b, e, i in zip(bases, exps, idx)]
    bad = [k for k in range(count) if got[k] != want[k]]
    assert not bad, f"{len(bad)} mismatches, first at {bad[0]}"


@pytest.mark.parametrize("limbs", [64, 128])
def test_modexp_edges(gpu_ctx, limbs):
    rnd = random.Random(7 + limbs)
    bits = 32 * limbs
    N = _odd(rnd, bits)
    NN = (1 << bits) - 1                     # all-ones modulus stresses carries
    mods = [N, NN, 3, (1 << (bits - 1)) + 1]
    cases = [(0, 0, 0), (0, 5, 0), (1, 0, 0), (N - 1, 2, 0), (N, 3, 0), (N + 5, 3, 0), ((1 << bits) - 1, 65537, 0),
             (NN - 1, NN, 1), (2, 1000, 2), (5, 0, 2), (12345, 1 << 2047, 3), (N - 1, (1 << 2048) - 1, 0)]
    bases = [c[0] for c in cases]
    exps = [c[1] for c in cases]
    idx = [c[2] for c in cases]
    got = gpu_ctx.modexp_batch(bases, exps, mods, idx, limbs)
    want = [pow(b, e, mods[i]) for b, e, i in zip(bases, exps, idx)]
    assert got == want


def test_modexp_paillier_shape(gpu_ctx):
    """r^N mod N^2 — the Paillier encryption shape (refresh_message.rs:72-84)."""
    rnd = random.Random(99)
    Ns = [_odd(rnd, 2048) for _ in range(4)]
    mods = [n * n for n in Ns]
    idx = [k % 4 for k in range(256)]
    bases = [rnd.randrange(Ns[i]) for i in idx]
    exps = [Ns[i] for i in idx]
    got = gpu_ctx.modexp_batch(bases, exps, mods, idx, 128)
    assert got == [pow(b, e, mods[i]) for b, e, i in zip(bases, exps, idx)]


@pytest.mark.parametrize("limbs,group", [(64, 2), (64, 4), (64, 8), (128, 4), (128, 8), (128, 16), (128, 32), (128, 64),
                                         (192, 4), (192, 8)])
def test_modexp_every_group_size(gpu_ctx, limbs, group):
    """Each lanes-per-instance variant (mont29.hpp DPP paths for G = 2..32; G = 64 the
    one-instance-per-wave kernel with v_readlane rows) is exact,
    including the all-ones modulus and exponent-length spread in one launch."""
    rnd = random.Random(1000 * limbs + group)
    bits = 32 * limbs
    mods = [_odd(rnd, bits) for _ in range(3)] + [(1 << bits) - 1, _odd(rnd, bits - 61)]
    count = 200
    idx = [rnd.randrange(len(mods)) for _ in range(count)]
    bases = [rnd.getrandbits(bits) for _ in range(count)]
    exps = [rnd.getrandbits(rnd.choice([1, 30, 256, 1000, 2048])) for _ in range(count)]
    gpu_ctx.set_modexp_group(group)
    try:
        got = gpu_ctx.modexp_batch(bases, exps, mods, idx, limbs)
    finally:
        gpu_ctx.set_modexp_group(0)
    want = [pow(b, e, mods[i]) for b, e, i in zip(bases, exps, idx)]
    bad = [k for k in range(count) if got[k] != want[k]]
    assert not bad, f"G={group}: {len(bad)} mismatches, first at {bad[0]}"


@pytest.mark.parametrize("limbs,group", [(64, 8), (128, 8), (128, 16), (128, 32), (192, 8)])
@pytest.mark.parametrize("kind", ["zero", "zero_one"])
def test_modexp_one_window_quotient_scaled(gpu_ctx, limbs, group, kind):
    """The quotient-scaled group shapes (modexp_kernel QS, 8-32 lanes) on launches
    whose exponents all fit one window (all 0, or all 0/1: w = 1, nwin = 1): the
    ladder start T[d0] is loaded after the table build (it used to return the last
    table row, base^(2^w - 1), instead of base^e)."""
    rnd = random.Random(77 * limbs + group + len(kind))
    bits = 32 * limbs
    mods = [_odd(rnd, bits) for _ in range(3)] + [(1 << bits) - 1]
    count = 96
    idx = [rnd.randrange(len(mods)) for _ in range(count)]
    bases = [rnd.getrandbits(bits) for _ in range(count)]
    exps = [0] * count if kind == "zero" else [rnd.getrandbits(1) for _ in range(count)]
    gpu_ctx.set_modexp_group(group)
    try:
        got = gpu_ctx.modexp_batch(bases, exps, mods, idx, limbs)
    finally:
        gpu_ctx.set_modexp_group(0)
    want = [pow(b, e, mods[i]) for b, e, i in zip(bases, exps, idx)]
    bad = [k for k in range(count) if got[k] != want[k]]
    assert not bad, f"G={group}: {len(bad)} mismatches, first at {bad[0]}"


@pytest.mark.parametrize("limbs", [32, 64, 96, 128])
def test_modexp_regular_access_equals_plain(gpu_ctx, limbs):
    """fsdkr_modexp_batch_ct (secret exponents: table scans, uniform window count)
    returns exactly fsdkr_modexp_batch's results, including tiny exponents mixed
    with full-width ones (one-window instances) and exponent 0."""
    rnd = random.Random(100 + limbs)
    bits = 32 * limbs
    mods = [_odd(rnd, bits) for _ in range(3)] + [_odd(rnd, bits - 61)]
    count = 120
    idx = [rnd.randrange(len(mods)) for _ in range(count)]
    bases = [rnd.getrandbits(bits) for _ in range(count)]
    exps = [rnd.getrandbits(rnd.choice([1, 3, 6, 64, 700, bits])) for _ in range(count)]
    exps[:4] = [0, 1, 2, (1 << bits) - 1]
    got = gpu_ctx.modexp_batch(bases, exps, mods, idx, limbs, secret=True)
    assert got == [pow(b, e, mods[i]) for b, e, i in zip(bases, exps, idx)]
    assert got == gpu_ctx.modexp_batch(bases, exps, mods, idx, limbs)


@pytest.mark.parametrize("group", [4, 8, 16, 32])
def test_modexp_joint_split_chains(gpu_ctx, group):
    """collect()'s GA chains split into a head (the exponent's bits >= 256) and a
    joint tail that multiplies base2^exp2 in along the tail's squarings
    (fsdkr_modexp_joint_batch): bit-exact against Python for s^N * (c^-1)^e mod N^2
    shapes, exponents N shared per modulus (waves padded), exp2 = 0 / 1 / full 256
    bits, base2 = 1, bases above N^2, and exponents shorter than the split point
    (E < 2^256, E = 0: the head only builds the table or nothing).  32 lanes: the
    KD = 160 shape small launches (multi-GPU shards) take."""
    rnd = random.Random(4242 + group)
    Ns = [_odd(rnd, 2048) for _ in range(4)]
    mods = [n * n for n in Ns]
    exps = [Ns[0], Ns[1], Ns[2], rnd.getrandbits(200) | 1]   # the last one below 2^256
    mods.append(_odd(rnd, 4090))
    exps.append(0)
    count = 150
    idx = [rnd.randrange(len(mods)) for _ in range(count)]
    bases = [rnd.getrandbits(4096) for _ in range(count)]
    bases2 = [rnd.randrange(mods[i]) for i in idx]
    e2 = [rnd.getrandbits(256) for _ in range(count)]
    e2[:6] = [0, 1, 15, 16, (1 << 256) - 1, 1 << 255]
    bases2[6] = 1
    gpu_ctx.set_modexp_group(group)
    try:
        got = gpu_ctx.modexp_joint_batch(bases, bases2, e2, mods, exps, idx)
    finally:
        gpu_ctx.set_modexp_group(0)
    want = [pow(b, exps[i], mods[i]) * pow(y, f, mods[i]) % mods[i] for b, y, f, i in zip(bases, bases2, e2, idx)]
    bad = [k for k in range(count) if got[k] != want[k]]
    assert not bad, f"G={group}: {len(bad)} mismatches, first at {bad[0]}"


def _keyed(ctx, bases, exps, mods, idx, limbs, exp_limbs):
    """fsdkr_modexp_keyed_device on device-resident operands (exps: one per modulus),
    staged through the HIP runtime libfsdkr already loaded (hipMalloc / hipMemcpy)."""
    import ctypes
    import numpy as np
    from fsdkr._native import ints_to_limbs, limbs_to_ints
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    held = []

    def put(a):
        a = np.ascontiguousarray(a, dtype=np.uint32)
        p = ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(p), max(a.nbytes, 4)) == 0
        held.append(p)
        assert hip.hipMemcpy(p, a.ctypes.data, a.nbytes, 1) == 0   # hipMemcpyHostToDevice
        return p.value

    try:
        out = np.full((len(bases), limbs), 0xffffffff, dtype=np.uint32)
        d_o = put(out)
        ebits = max(1, max(e.bit_length() for e in exps))
        ctx.check(ctx._lib.fsdkr_modexp_keyed_device(ctx.handle, limbs, len(bases), put(ints_to_limbs(bases, limbs)),
                                                     put(ints_to_limbs(exps, exp_limbs)), exp_limbs, ebits,
                                                     put(np.asarray(idx, dtype=np.uint32)),
                                                     put(ints_to_limbs(mods, limbs)), len(mods), d_o))
        assert hip.hipMemcpy(out.ctypes.data, d_o, out.nbytes, 2) == 0   # hipMemcpyDeviceToHost
        return limbs_to_ints(out)
    finally:
        for p in held:
            hip.hipFree(p)


@pytest.mark.parametrize("count", [150, 3000, 30000])
def test_modexp_keyed_sliding_windows(gpu_ctx, count):
    """One exponent per modulus (fsdkr_modexp_keyed_device, the r^N mod N^2 shape of
    Paillier encryption): instances regrouped by key into waves that share their
    exponent, ragged runs padded with copies that rewrite their own row, sliding
    windows.  Counts cover the 16-, 8- and 4-lane launches; shuffled key order, a key
    with one instance, an exponent of 0 and one of 1, bases above N^2."""
    rnd = random.Random(5150 + count)
    Ns = [_odd(rnd, 2048) for _ in range(5)]
    mods = [n * n for n in Ns] + [_odd(rnd, 4096), _odd(rnd, 4001)]
    exps = Ns + [0, 1]
    idx = [rnd.choice([0, 0, 1, 2, 3, 5, 6]) for _ in range(count)]
    idx[rnd.randrange(count)] = 4                    # the only instance of key 4
    bases = [rnd.getrandbits(4096) for _ in range(count)]
    got = _keyed(gpu_ctx, bases, exps, mods, idx, 128, 64)
    # Python's pow takes ~0.1 s per 4096-bit chain: a sample of the full chains,
    # the single-instance key, and every exponent-0 / exponent-1 instance
    check = sorted(set(rnd.sample(range(count), 30)) | {idx.index(4)} | {k for k in range(count) if idx[k] >= 5})
    bad = [k for k in check if got[k] != pow(bases[k], exps[idx[k]], mods[idx[k]])]
    assert not bad, f"{len(bad)} mismatches, first at {bad[0]}"


@pytest.mark.parametrize("limbs", [64, 192])
def test_modexp_keyed_other_widths(gpu_ctx, limbs):
    """Widths without a sliding-window shape keep fixed windows (per-instance exponent
    pointers into the per-key rows); out-of-range key indices are refused."""
    from fsdkr._native import FsdkrError
    rnd = random.Random(limbs)
    bits = 32 * limbs
    mods = [_odd(rnd, bits) for _ in range(3)]
    exps = [rnd.getrandbits(bits) for _ in range(3)]
    idx = [rnd.randrange(3) for _ in range(100)]
    bases = [rnd.getrandbits(bits) for _ in range(100)]
    got = _keyed(gpu_ctx, bases, exps, mods, idx, limbs, limbs)
    assert got == [pow(b, exps[i], mods[i]) for b, i in zip(bases, idx)]
    idx[7] = 3
    with pytest.raises(FsdkrError):
        _keyed(gpu_ctx, bases, exps, mods, idx, limbs, limbs)
