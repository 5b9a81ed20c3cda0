"""ctypes binding of libfsdkr.so (include/fsdkr/fsdkr.h).

The product path is the HIP library: loading fails loudly if it is missing,
and there is no CPU fallback anywhere in this package."""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# FSDKR_LIB: alternative build of the same library (A/B timing tools only)
LIB_PATH = os.environ.get("FSDKR_LIB") or os.path.join(_HERE, "libfsdkr.so")

FSDKR_OK = 0
FSDKR_E_ARG = -1
FSDKR_E_HIP = -2
FSDKR_E_OOM = -3
FSDKR_E_UNSUPPORTED = -4
FSDKR_CFG_TIMING = 1
# algorithm switches (parity tests, A/B runs; results identical under each)
FSDKR_CFG_FB_BGMW = 2    # fixed-base exponentiations by BGMW windows only
FSDKR_CFG_FB_COMB = 4    # a Lim-Lee comb wherever one fits
FSDKR_CFG_INV_EACH = 8   # one inverse per element (no simultaneous inversion)

u32p = ctypes.POINTER(ctypes.c_uint32)


class FsdkrError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"fsdkr error {code}: {msg}")
        self.code = code


class _Cfg(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("flags", ctypes.c_uint32)]


class CollectBatchC(ctypes.Structure):
    """struct fsdkr_collect_batch (include/fsdkr/fsdkr.h)."""
    _fields_ = [(f, ctypes.c_uint32) for f in ("n_refresh", "n_join", "t", "m_security", "key_bits", "nl",
                                               "s1l", "s3l", "el", "zl", "yl")] + \
               [(f, u32p) for f in ("party_index", "msg_lens", "recv_n", "recv_ntilde", "recv_h1", "recv_h2",
                                    "enc", "commit", "pdl_z", "pdl_u3", "pdl_s2", "pdl_u1", "pdl_u2", "pdl_s1",
                                    "pdl_s3", "rp_z", "rp_s", "rp_e", "rp_s1", "rp_s2", "vss", "ped_S", "ped_T",
                                    "ped_N", "ped_A", "ped_Z", "ck_n", "ck_sigma", "dlog_N", "dlog_g", "dlog_ni",
                                    "dlog_x1", "dlog_x2", "dlog_y1", "dlog_y2")] + [("n_recv", ctypes.c_uint32)] + \
               [("vss_len", u32p), ("range_lens", u32p), ("ckl", ctypes.c_uint32), ("recv_avail", ctypes.c_uint32),
                ("ped_lens", u32p), ("ck_lens", u32p), ("pdl_s3_neg", ctypes.POINTER(ctypes.c_uint8)),
                ("neg_bits", ctypes.POINTER(ctypes.c_uint8)), ("ped_a_neg", ctypes.POINTER(ctypes.c_uint8))]


u8p = ctypes.POINTER(ctypes.c_uint8)


class VerdictsC(ctypes.Structure):
    _fields_ = [(f, u8p) for f in ("feldman", "pdl", "range", "ped", "ck", "dlog")] + \
               [(f, ctypes.c_uint32) for f in ("cap_pairs", "cap_msgs", "cap_joins")]


class RecoverJobC(ctypes.Structure):
    _fields_ = [("nl", ctypes.c_uint32), ("t_vss", ctypes.c_uint32), ("t_key", ctypes.c_uint32),
                ("n_new", ctypes.c_uint32), ("old_index", u32p), ("cts", u32p), ("p", u32p), ("q", u32p),
                ("points", u32p), ("flags", ctypes.c_uint32)]


class RecoveredC(ctypes.Structure):
    _fields_ = [("share", ctypes.c_uint32 * 8), ("y", ctypes.c_uint32 * 16), ("pk_vec", u32p),
                ("status", ctypes.c_int32)]


def _struct_dtype(cls):
    """numpy structured dtype with the exact layout of a ctypes Structure (pointers as u8)."""
    names, formats, offsets = [], [], []
    for name, typ in cls._fields_:
        names.append(name)
        formats.append(np.uint64 if ctypes.sizeof(typ) == 8 else np.uint32)
        offsets.append(getattr(cls, name).offset)
    return np.dtype({"names": names, "formats": formats, "offsets": offsets, "itemsize": ctypes.sizeof(cls)})


_RECOVER_DT = _struct_dtype(RecoverJobC)
_RECOVERED_DT = np.dtype({"names": ["pk_vec", "status"], "formats": [np.uint64, np.int32],
                          "offsets": [RecoveredC.pk_vec.offset, RecoveredC.status.offset],
                          "itemsize": ctypes.sizeof(RecoveredC)})
RECOVER_OK, RECOVER_PANIC_LI, RECOVER_PANIC_DECRYPT = 0, 1, 2
RECOVER_NO_DECRYPT = 1   # fsdkr_recover_job.flags
DRAW_BITS_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32),
                                ctypes.c_uint32)


class ErrorC(ctypes.Structure):
    _fields_ = [("variant", ctypes.c_int32), ("panic", ctypes.c_int32), ("f", ctypes.c_uint32 * 4),
                ("keys_applied", ctypes.c_uint32)]


_lib = None


def lib():
    """Load libfsdkr.so.  Raises (never falls back) if the HIP library is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} missing: run __graft_entry__.build() (no CPU fallback exists)")
    L = ctypes.CDLL(LIB_PATH)
    vp = ctypes.c_void_p
    L.fsdkr_ctx_create.argtypes = [ctypes.POINTER(_Cfg), ctypes.POINTER(vp)]
    L.fsdkr_ctx_create.restype = ctypes.c_int
    L.fsdkr_collect_recover.argtypes = [vp, ctypes.POINTER(RecoverJobC), ctypes.c_uint32,
                                        ctypes.POINTER(RecoveredC)]
    L.fsdkr_collect_recover.restype = ctypes.c_int
    L.fsdkr_collect_recover_launch.argtypes = [vp, ctypes.POINTER(RecoverJobC), ctypes.c_uint32]
    L.fsdkr_collect_recover_launch.restype = ctypes.c_int
    L.fsdkr_collect_recover_finish.argtypes = [vp, ctypes.POINTER(RecoveredC)]
    L.fsdkr_collect_recover_finish.restype = ctypes.c_int
    L.fsdkr_sample_primes.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                      DRAW_BITS_FN, vp, u32p, ctypes.c_uint32]
    L.fsdkr_sample_primes.restype = ctypes.c_int
    L.fsdkr_ctx_destroy.argtypes = [vp]
    L.fsdkr_ctx_destroy.restype = None
    L.fsdkr_last_error.argtypes = [vp]
    L.fsdkr_last_error.restype = ctypes.c_char_p
    L.fsdkr_device_available.argtypes = []
    L.fsdkr_device_available.restype = ctypes.c_int
    L.fsdkr_modexp_batch.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, u32p, u32p, ctypes.c_uint32, u32p, u32p,
                                     ctypes.c_uint32, u32p]
    L.fsdkr_modexp_batch.restype = ctypes.c_int
    L.fsdkr_modexp_batch_ct.argtypes = L.fsdkr_modexp_batch.argtypes
    L.fsdkr_modexp_joint_batch.argtypes = [vp, ctypes.c_uint32, u32p, u32p, u32p, u32p, u32p, u32p, ctypes.c_uint32,
                                           ctypes.c_uint32, u32p]
    L.fsdkr_modexp_joint_batch.restype = ctypes.c_int
    L.fsdkr_modexp_batch_ct.restype = ctypes.c_int
    L.fsdkr_modexp_batch_device.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, vp, vp, ctypes.c_uint32,
                                            ctypes.c_uint32, vp, vp, ctypes.c_uint32, vp]
    L.fsdkr_modexp_batch_device.restype = ctypes.c_int
    L.fsdkr_modexp_keyed_device.argtypes = L.fsdkr_modexp_batch_device.argtypes
    L.fsdkr_modexp_keyed_device.restype = ctypes.c_int
    L.fsdkr_kernel_time.argtypes = [vp, ctypes.c_char_p, ctypes.POINTER(ctypes.c_double),
                                    ctypes.POINTER(ctypes.c_uint32)]
    L.fsdkr_kernel_time.restype = ctypes.c_int
    L.fsdkr_kernel_time_reset.argtypes = [vp]
    L.fsdkr_kernel_time_reset.restype = None
    L.fsdkr_verify_collect.argtypes = [vp, ctypes.POINTER(CollectBatchC), ctypes.POINTER(VerdictsC)]
    L.fsdkr_verify_collect.restype = ctypes.c_int
    L.fsdkr_collect_prepare.argtypes = [vp, ctypes.POINTER(CollectBatchC)]
    L.fsdkr_collect_prepare.restype = ctypes.c_int
    L.fsdkr_collect_run.argtypes = [vp, ctypes.POINTER(VerdictsC)]
    L.fsdkr_collect_run.restype = ctypes.c_int
    L.fsdkr_collect_launch.argtypes = [vp]
    L.fsdkr_collect_launch.restype = ctypes.c_int
    L.fsdkr_collect_prestart.argtypes = [vp, ctypes.POINTER(CollectBatchC)]
    L.fsdkr_collect_prestart.restype = ctypes.c_int
    L.fsdkr_collect_last_span_ms.argtypes = [vp]
    L.fsdkr_collect_last_span_ms.restype = ctypes.c_double
    L.fsdkr_collect_reuse_mask.argtypes = [vp]
    L.fsdkr_collect_reuse_mask.restype = ctypes.c_uint32
    L.fsdkr_collect_finish.argtypes = [vp, ctypes.POINTER(VerdictsC)]
    L.fsdkr_collect_finish.restype = ctypes.c_int
    L.fsdkr_collect_prepare_multi.argtypes = [vp, ctypes.POINTER(CollectBatchC), ctypes.c_uint32]
    L.fsdkr_collect_prepare_multi.restype = ctypes.c_int
    L.fsdkr_collect_prestart_multi.argtypes = [vp, ctypes.POINTER(CollectBatchC), ctypes.c_uint32]
    L.fsdkr_collect_prestart_multi.restype = ctypes.c_int
    L.fsdkr_collect_prestart_rp.argtypes = [vp, ctypes.POINTER(CollectBatchC), ctypes.c_uint32]
    L.fsdkr_collect_prestart_rp.restype = ctypes.c_int
    L.fsdkr_collect_finish_multi.argtypes = [vp, ctypes.POINTER(VerdictsC), ctypes.c_uint32]
    L.fsdkr_collect_finish_multi.restype = ctypes.c_int
    L.fsdkr_verify_collect_multi.argtypes = [vp, ctypes.POINTER(CollectBatchC), ctypes.c_uint32,
                                             ctypes.POINTER(VerdictsC)]
    L.fsdkr_verify_collect_multi.restype = ctypes.c_int
    L.fsdkr_paillier_decrypt_multi.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, u32p, u32p, u32p, u32p,
                                               ctypes.c_uint32, u32p]
    L.fsdkr_paillier_decrypt_multi.restype = ctypes.c_int
    L.fsdkr_collect_first_error.argtypes = [ctypes.POINTER(CollectBatchC), ctypes.POINTER(VerdictsC),
                                            ctypes.POINTER(ErrorC)]
    L.fsdkr_collect_first_error.restype = ctypes.c_int
    L.fsdkr_paillier_decrypt.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, u32p, u32p, u32p, u32p]
    L.fsdkr_paillier_decrypt.restype = ctypes.c_int
    L.fsdkr_paillier_encrypt.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, u32p, ctypes.c_uint32, u32p, u32p,
                                         u32p, ctypes.c_uint32, u32p]
    L.fsdkr_paillier_encrypt.restype = ctypes.c_int
    L.fsdkr_ctx_set_modexp_group.argtypes = [vp, ctypes.c_uint32]
    L.fsdkr_ctx_set_modexp_group.restype = ctypes.c_int
    L.fsdkr_ctx_set_timing.argtypes = [vp, ctypes.c_int]
    L.fsdkr_ctx_set_cu_split.argtypes = [vp, ctypes.c_uint32]
    L.fsdkr_ctx_set_cu_split.restype = ctypes.c_int
    L.fsdkr_ctx_set_timing.restype = ctypes.c_int
    L.fsdkr_ctx_set_flags.argtypes = [vp, ctypes.c_uint32]
    L.fsdkr_ctx_set_flags.restype = ctypes.c_int
    L.fsdkr_mod_inverse.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, u32p, u32p, u32p, u32p]
    L.fsdkr_mod_inverse.restype = ctypes.c_int
    L.fsdkr_miller_rabin.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, u32p, u32p, u32p]
    L.fsdkr_miller_rabin.restype = ctypes.c_int
    L.fsdkr_ec_msm.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, u32p, u32p, u32p]
    L.fsdkr_ec_msm.restype = ctypes.c_int
    L.fsdkr_fixed_base_modexp.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, u32p, u32p, u32p, ctypes.c_uint32,
                                          ctypes.c_uint32, u32p, u32p, ctypes.c_uint32, u32p]
    L.fsdkr_fixed_base_modexp.restype = ctypes.c_int
    L.fsdkr_feldman_check.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, u32p, u32p, u8p]
    L.fsdkr_feldman_check.restype = ctypes.c_int
    L.fsdkr_pdl_u1_check.argtypes = [vp, ctypes.c_uint32, u32p, ctypes.c_uint32, u32p, u32p, u32p, u8p]
    L.fsdkr_pdl_u1_check.restype = ctypes.c_int
    L.fsdkr_ring_pedersen_verify.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                             u32p, u32p, u32p, u32p, u32p, u8p]
    L.fsdkr_ring_pedersen_verify.restype = ctypes.c_int
    _lib = L
    return L


def _ptr(a):
    return a.ctypes.data_as(u32p)


def ints_to_limbs(values, limbs):
    """list of non-negative ints -> (len, limbs) uint32 little-endian array
    (csrc/pack.c digit re-slicing); ValueError if a value is negative or too wide."""
    from . import _pack
    out = np.empty((len(values), limbs), dtype=np.uint32)
    try:
        _pack.pack(values, None, out, limbs)
    except OverflowError:
        raise ValueError(f"a value does not fit {limbs} limbs") from None
    return out


def limbs_to_ints(arr):
    arr = np.ascontiguousarray(arr, dtype=np.uint32)
    b = arr.tobytes()
    n = arr.shape[1] * 4
    return [int.from_bytes(b[i * n:(i + 1) * n], "little") for i in range(arr.shape[0])]


class Context:
    """Owns one fsdkr_ctx (HIP stream + device buffers)."""

    def __init__(self, device=-1, timing=False):
        L = lib()
        cfg = _Cfg(device, FSDKR_CFG_TIMING if timing else 0)
        h = ctypes.c_void_p()
        rc = L.fsdkr_ctx_create(ctypes.byref(cfg), ctypes.byref(h))
        if rc != FSDKR_OK:
            raise FsdkrError(rc, "fsdkr_ctx_create failed (no HIP device?)")
        self._h = h
        self._lib = L
        self._flags = cfg.flags

    @property
    def handle(self):
        return self._h

    def close(self):
        if self._h:
            self._lib.fsdkr_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def check(self, rc):
        if rc != FSDKR_OK:
            raise FsdkrError(rc, self._lib.fsdkr_last_error(self._h).decode())

    def kernel_time(self, name):
        ms = ctypes.c_double()
        n = ctypes.c_uint32()
        self.check(self._lib.fsdkr_kernel_time(self._h, name.encode(), ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def kernel_time_reset(self):
        self._lib.fsdkr_kernel_time_reset(self._h)

    def modexp_batch(self, bases, exps, mods, mod_idx, mod_limbs, secret=False):
        """[base_i ^ exp_i mod mods[mod_idx_i]] computed on the GPU.  secret=True:
        regular-access kernel (fsdkr_modexp_batch_ct) for secret exponents."""
        count = len(bases)
        if count == 0:
            return []
        emax = max(1, max(e.bit_length() for e in exps))
        exp_limbs = (emax + 31) // 32
        B = ints_to_limbs(bases, mod_limbs)
        E = ints_to_limbs(exps, exp_limbs)
        Mo = ints_to_limbs(mods, mod_limbs)
        I = np.ascontiguousarray(np.asarray(mod_idx, dtype=np.uint32))
        O = np.zeros((count, mod_limbs), dtype=np.uint32)
        fn = self._lib.fsdkr_modexp_batch_ct if secret else self._lib.fsdkr_modexp_batch
        self.check(fn(self._h, mod_limbs, count, _ptr(B), _ptr(E), exp_limbs, _ptr(I), _ptr(Mo), len(mods), _ptr(O)))
        return limbs_to_ints(O)

    def modexp_joint_batch(self, bases, bases2, exps2, mods, mod_exps, mod_idx):
        """[bases[i] ^ mod_exps[k] * bases2[i] ^ exps2[i] mod mods[k]], k = mod_idx[i],
        4096-bit moduli, exps2 < 2^256, bases2 reduced: collect()'s split GA chains
        (fsdkr_modexp_joint_batch)."""
        count = len(bases)
        if count == 0:
            return []
        exp_limbs = max(1, (max(e.bit_length() for e in mod_exps) + 31) // 32)
        B = ints_to_limbs(bases, 128)
        B2 = ints_to_limbs(bases2, 128)
        E2 = ints_to_limbs(exps2, 8)
        Mo = ints_to_limbs(mods, 128)
        ME = ints_to_limbs(mod_exps, exp_limbs)
        I = np.ascontiguousarray(np.asarray(mod_idx, dtype=np.uint32))
        O = np.zeros((count, 128), dtype=np.uint32)
        self.check(self._lib.fsdkr_modexp_joint_batch(self._h, count, _ptr(B), _ptr(B2), _ptr(E2), _ptr(I), _ptr(Mo),
                                                      _ptr(ME), exp_limbs, len(mods), _ptr(O)))
        return limbs_to_ints(O)

    def fixed_base_modexp(self, bases, base_mod_idx, mods, base_idx, exps, mod_limbs):
        """[bases[base_idx[i]] ^ exps[i] mod mods[base_mod_idx[base_idx[i]]]] via the fixed-base engine."""
        count = len(exps)
        if count == 0:
            return []
        exp_limbs = max(1, (max(e.bit_length() for e in exps) + 31) // 32)
        B = ints_to_limbs(bases, mod_limbs)
        Bm = np.ascontiguousarray(np.asarray(base_mod_idx, dtype=np.uint32))
        Mo = ints_to_limbs(mods, mod_limbs)
        Bi = np.ascontiguousarray(np.asarray(base_idx, dtype=np.uint32))
        E = ints_to_limbs(exps, exp_limbs)
        O = np.zeros((count, mod_limbs), dtype=np.uint32)
        self.check(self._lib.fsdkr_fixed_base_modexp(self._h, mod_limbs, len(bases), _ptr(B), _ptr(Bm), _ptr(Mo),
                                                     len(mods), count, _ptr(Bi), _ptr(E), exp_limbs, _ptr(O)))
        return limbs_to_ints(O)

    def set_modexp_group(self, lanes):
        """Force the lanes per modexp instance (0 = automatic)."""
        self.check(self._lib.fsdkr_ctx_set_modexp_group(self._h, lanes))

    def set_cu_split(self, ga_cus):
        """Multi-GPU shards: GA chains on `ga_cus` CUs, everything else on the rest (0 = off)."""
        self.check(self._lib.fsdkr_ctx_set_cu_split(self._h, ga_cus))

    def set_timing(self, on):
        """Per-kernel HIP-event timing on/off (kernel_time needs it on)."""
        self.check(self._lib.fsdkr_ctx_set_timing(self._h, 1 if on else 0))
        self._flags = (self._flags | FSDKR_CFG_TIMING) if on else (self._flags & ~FSDKR_CFG_TIMING)

    def set_flags(self, flags):
        """Replace the fsdkr_cfg flags (FSDKR_CFG_*); returns the previous ones."""
        old = self._flags
        self.check(self._lib.fsdkr_ctx_set_flags(self._h, flags))
        self._flags = flags
        return old

    @property
    def flags(self):
        return self._flags

    def mod_inverse(self, ys, ms, mod_limbs):
        """[(y^-1 mod m or None)] on the GPU (None where gcd(y, m) != 1)."""
        count = len(ys)
        if count == 0:
            return []
        Y = ints_to_limbs(ys, mod_limbs)
        M = ints_to_limbs(ms, mod_limbs)
        O = np.zeros((count, mod_limbs), dtype=np.uint32)
        U = np.zeros(count, dtype=np.uint32)
        self.check(self._lib.fsdkr_mod_inverse(self._h, mod_limbs, count, _ptr(Y), _ptr(M), _ptr(O), _ptr(U)))
        return [v if u else None for v, u in zip(limbs_to_ints(O), U.tolist())]

    def miller_rabin(self, cands, bases, mod_limbs):
        """[1 if cands[i] is a strong probable prime to base bases[i] else 0] on the GPU."""
        count = len(cands)
        if count == 0:
            return []
        C = ints_to_limbs(cands, mod_limbs)
        B = ints_to_limbs(bases, mod_limbs)
        V = np.zeros(count, dtype=np.uint32)
        self.check(self._lib.fsdkr_miller_rabin(self._h, mod_limbs, count, _ptr(C), _ptr(B), _ptr(V)))
        return V.tolist()

    def sample_primes(self, draw_bits, bits, count, window=0, span=0):
        """fsdkr_sample_primes: `count` primes of `bits` bits by the batched prime
        walk; draw_bits(k) supplies the k-bit random starts (the caller's RNG)."""
        limbs = (bits + 31) // 32
        errs = []

        def cb(_user, nbits, out, nl):
            try:
                v = draw_bits(nbits)
                for k in range(nl):
                    out[k] = (v >> (32 * k)) & 0xFFFFFFFF
                return 0
            except Exception as e:   # re-raised below, after the C call returns
                errs.append(e)
                return 1
        fn = DRAW_BITS_FN(cb)
        O = np.zeros((max(1, count), limbs), dtype=np.uint32)
        rc = self._lib.fsdkr_sample_primes(self._h, bits, count, window, span, fn, None, _ptr(O), limbs)
        if errs:
            raise errs[0]
        self.check(rc)
        return limbs_to_ints(O[:count])

    # ---- collect() verification -------------------------------------------
    def verify_collect(self, batch):
        """Run fsdkr_verify_collect on a fsdkr.batch.CollectBatch; returns a Verdicts."""
        from .batch import Verdicts
        v = Verdicts(batch.R, batch.J, batch.n)
        self.check(self._lib.fsdkr_verify_collect(self._h, ctypes.byref(batch.c), ctypes.byref(v.c)))
        return batch.settle(v)

    def collect_prepare(self, batch):
        """Host pre-pass + one upload of the batch image (device-resident afterwards)."""
        self.check(self._lib.fsdkr_collect_prepare(self._h, ctypes.byref(batch.c)))

    def collect_run(self, batch):
        """Kernel pipeline on the prepared batch; returns Verdicts."""
        from .batch import Verdicts
        v = Verdicts(batch.R, batch.J, batch.n)
        self.check(self._lib.fsdkr_collect_run(self._h, ctypes.byref(v.c)))
        return batch.settle(v)

    def collect_prestart(self, batch):
        """Start the s^N mod N^2 chains of a batch whose GA fields are packed
        (CollectBatch(..., staged=True)); the next prepare of it reuses them."""
        self.check(self._lib.fsdkr_collect_prestart(self._h, ctypes.byref(batch.c)))

    def collect_last_span_ms(self):
        """Device span of the last finished collect() call (HIP events: first
        device work -> the pipeline's last kernel), -1 before any."""
        return float(self._lib.fsdkr_collect_last_span_ms(self._h))

    REUSE = {"ga": 1, "tables": 2, "ck": 4, "tz": 8}

    def collect_reuse(self):
        """Names of the prestarted parts the last prepare reused (fsdkr_collect_reuse_mask)."""
        m = int(self._lib.fsdkr_collect_reuse_mask(self._h))
        return {k for k, bit in self.REUSE.items() if m & bit}

    def collect_launch(self):
        """Enqueue the kernel pipeline of the prepared batch (returns at once)."""
        self.check(self._lib.fsdkr_collect_launch(self._h))

    def collect_finish(self, batch):
        """Wait for the launched pipeline; returns Verdicts."""
        from .batch import Verdicts
        v = Verdicts(batch.R, batch.J, batch.n)
        self.check(self._lib.fsdkr_collect_finish(self._h, ctypes.byref(v.c)))
        return batch.settle(v)

    def collect_prepare_many(self, batches):
        """Prepare many sessions (fsdkr.batch.CollectBatch each) as ONE device image."""
        arr = (CollectBatchC * len(batches))(*[b.c for b in batches])
        self._many = arr   # keep the array alive until finish
        self.check(self._lib.fsdkr_collect_prepare_multi(self._h, arr, len(batches)))

    def collect_prestart_set(self, sset):
        """Start the GA chains of every regular session of a staged SessionSet."""
        arr = sset.prestart_array()
        if arr is not None:
            self._prestart_keep = sset
            self.check(self._lib.fsdkr_collect_prestart_multi(self._h, arr, sset.n_prestart))

    def collect_prestart_rp_set(self, sset):
        """Start the ring-Pedersen T^Z exponents of a SessionSet whose stage 1b
        (SessionSet.stage_z) packed Z, behind the prestarted T tables."""
        arr = sset.prestart_array()
        if arr is not None:
            self.check(self._lib.fsdkr_collect_prestart_rp(self._h, arr, sset.n_prestart))

    def collect_prepare_set(self, sset):
        """Prepare every live session of a fsdkr.batch.SessionSet as ONE device image."""
        self._many = sset   # keep the struct rows alive until finish
        self.check(self._lib.fsdkr_collect_prepare_multi(self._h, sset.c_array, len(sset.live)))

    def collect_finish_set(self, sset):
        """Wait for the launched multi-session pipeline; SetVerdicts of the live sessions."""
        v = sset.verdicts()
        self.check(self._lib.fsdkr_collect_finish_multi(self._h, v.c_array, len(sset.live)))
        return sset.settle(v)

    def collect_finish_many(self, batches):
        """Wait for the launched multi-session pipeline; one Verdicts per session."""
        from .batch import Verdicts
        vs = [Verdicts(b.R, b.J, b.n) for b in batches]
        arr = (VerdictsC * len(vs))(*[v.c for v in vs])
        self.check(self._lib.fsdkr_collect_finish_multi(self._h, arr, len(vs)))
        return [b.settle(v) for b, v in zip(batches, vs)]

    def paillier_decrypt(self, cts, p, q, nl):
        """Decrypt ciphertexts under dk = (p, q) on the GPU (CRT form)."""
        C = ints_to_limbs(cts, 2 * nl)
        Pp = ints_to_limbs([p], nl)
        Qq = ints_to_limbs([q], nl)
        O = np.zeros((len(cts), nl), dtype=np.uint32)
        self.check(self._lib.fsdkr_paillier_decrypt(self._h, nl, len(cts), _ptr(C), _ptr(Pp), _ptr(Qq), _ptr(O)))
        return limbs_to_ints(O)

    def paillier_decrypt_many(self, cts, key_idx, ps, qs, nl):
        """Decrypt cts[k] under key (ps[key_idx[k]], qs[key_idx[k]]) on the GPU."""
        if not cts:
            return []
        C = ints_to_limbs(cts, 2 * nl)
        I = np.ascontiguousarray(np.asarray(key_idx, dtype=np.uint32))
        Pp = ints_to_limbs(ps, nl)
        Qq = ints_to_limbs(qs, nl)
        O = np.zeros((len(cts), nl), dtype=np.uint32)
        self.check(self._lib.fsdkr_paillier_decrypt_multi(self._h, nl, len(cts), _ptr(C), _ptr(I), _ptr(Pp),
                                                          _ptr(Qq), len(ps), _ptr(O)))
        return limbs_to_ints(O)

    def paillier_encrypt(self, ms, rs, ns, n_idx, nl):
        """Job 1: [(1 + m N) r^N mod N^2] for N = ns[n_idx[k]]."""
        ml = max(1, (max(m.bit_length() for m in ms) + 31) // 32)
        Mm = ints_to_limbs(ms, ml)
        Rr = ints_to_limbs(rs, nl)
        Nn = ints_to_limbs(ns, nl)
        I = np.ascontiguousarray(np.asarray(n_idx, dtype=np.uint32))
        O = np.zeros((len(ms), 2 * nl), dtype=np.uint32)
        self.check(self._lib.fsdkr_paillier_encrypt(self._h, nl, len(ms), _ptr(Mm), ml, _ptr(Rr), _ptr(I), _ptr(Nn),
                                                    len(ns), _ptr(O)))
        return limbs_to_ints(O)

    def pdl_u1_check(self, s1s, es, Qs, u1s):
        """[G*(s1 mod q) + Q*(q - e mod q) == u1] per pair (uint8 0/1)."""
        from .batch import pack_points
        sl = max(1, (max(s.bit_length() for s in s1s) + 31) // 32)
        S = ints_to_limbs(s1s, sl)
        E = ints_to_limbs(es, 8)
        Qp, Up = pack_points(Qs), pack_points(u1s)
        out = np.zeros(len(s1s), dtype=np.uint8)
        self.check(self._lib.fsdkr_pdl_u1_check(self._h, len(s1s), _ptr(S), sl, _ptr(E), _ptr(Qp), _ptr(Up),
                                                out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))))
        return out

    def feldman_check(self, vss, commit, n, t):
        """vss: [n_msgs][t+1] points, commit: [n_msgs*n] points -> uint8 verdicts [n_msgs*n]."""
        from .batch import pack_points
        V = pack_points([p for row in vss for p in row])
        Cm = pack_points(commit)
        out = np.zeros(len(commit), dtype=np.uint8)
        self.check(self._lib.fsdkr_feldman_check(self._h, len(vss), n, t, _ptr(V), _ptr(Cm),
                                                 out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))))
        return out

    def ring_pedersen_verify(self, statements, proofs, m_security, nl):
        """[(statement, proof)] -> uint8 verdicts (bit0 ok, bit1 the reference panics)."""
        from .batch import pack
        M = m_security
        zl = max(1, (max(z.bit_length() for p in proofs for z in p.Z[:M]) + 31) // 32)
        S = pack([s.S for s in statements], nl)
        T = pack([s.T for s in statements], nl)
        N = pack([s.N for s in statements], nl)
        A = pack([a for p in proofs for a in p.A[:M]], nl)
        Z = pack([z for p in proofs for z in p.Z[:M]], zl)
        out = np.zeros(len(proofs), dtype=np.uint8)
        self.check(self._lib.fsdkr_ring_pedersen_verify(self._h, nl, len(proofs), M, zl, _ptr(S), _ptr(T), _ptr(N),
                                                        _ptr(A), _ptr(Z),
                                                        out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))))
        return out

    def collect_recover(self, jobs):
        """fsdkr_collect_recover: jobs = [dict(nl, t_vss, t_key, old_index, cts, p, q, points[, flags])],
        points[i] = the first min(t_key, t_vss)+1 committed points for new party i
        (flags RECOVER_NO_DECRYPT: those pk_vec rows only, share and y zero).
        Returns per job (status, share, y, pk_vec); a ciphertext wider than N^2
        raises ValueError (ints_to_limbs)."""
        return self.collect_recover_finish(self.collect_recover_launch(jobs))

    def collect_recover_launch(self, jobs):
        """fsdkr_collect_recover_launch: the recovery's GPU work is enqueued and
        runs while the caller goes on; returns the handle collect_recover_finish takes.
        Every job's ciphertexts, keys, indices and points are packed into one array
        per field (one conversion each, however many jobs; the rows of job k at
        its offsets), and the fsdkr_recover_job rows are filled vectorised."""
        from . import _pack
        J = len(jobs)
        nls = np.array([j["nl"] for j in jobs], dtype=np.int64)
        T = np.array([len(j["cts"]) for j in jobs], dtype=np.int64)
        tp = np.array([min(j["t_key"], j["t_vss"]) + 1 for j in jobs], dtype=np.int64)
        n_new = np.array([len(j["points"]) for j in jobs], dtype=np.int64)
        for j, t in zip(jobs, T):
            assert t == j["t_vss"] + 1
        idx = np.ascontiguousarray(np.fromiter((i for j in jobs for i in j["old_index"]), dtype=np.uint32,
                                               count=int(T.sum())))
        Pt = np.zeros((max(1, int((n_new * tp).sum())), 16), dtype=np.uint32)
        pts = [pt for j in jobs for row in j["points"] for pt in row]
        if pts:
            _pack.points(pts, None, Pt)
        if J and (nls != nls[0]).any():   # rows at each job's own width
            C2, PQ2 = [], []
            for k, j in enumerate(jobs):
                C2.append(ints_to_limbs(j["cts"], 2 * j["nl"]))
                PQ2.append(ints_to_limbs([j["p"], j["q"]], j["nl"]))
            c_ptr = np.array([a.ctypes.data for a in C2], dtype=np.uint64)
            p_ptr = np.array([a.ctypes.data for a in PQ2], dtype=np.uint64)
            q_ptr = p_ptr + (nls * 4).astype(np.uint64)
            keep = (C2, PQ2)
        else:   # one width: one array per field
            W = int(nls[0]) if J else 1
            C = ints_to_limbs([c for j in jobs for c in j["cts"]], 2 * W)
            PQ = ints_to_limbs([v for j in jobs for v in (j["p"], j["q"])], W)

            def starts(c):
                return np.concatenate([[0], np.cumsum(c)[:-1]]).astype(np.uint64)
            c_ptr = np.uint64(C.ctypes.data) + starts(T) * np.uint64(2 * W * 4)
            p_ptr = np.uint64(PQ.ctypes.data) + np.arange(J, dtype=np.uint64) * np.uint64(2 * W * 4)
            q_ptr = p_ptr + np.uint64(W * 4)
            keep = (C, PQ)
        rows = np.zeros(J, dtype=_RECOVER_DT)
        rows["nl"] = nls
        rows["t_vss"] = [j["t_vss"] for j in jobs]
        rows["t_key"] = [j["t_key"] for j in jobs]
        rows["n_new"] = n_new
        off = np.concatenate([[0], np.cumsum(T)[:-1]]).astype(np.uint64)
        rows["old_index"] = np.uint64(idx.ctypes.data) + off * np.uint64(4)
        rows["cts"], rows["p"], rows["q"] = c_ptr, p_ptr, q_ptr
        poff = np.concatenate([[0], np.cumsum(n_new * tp)[:-1]]).astype(np.uint64)
        rows["points"] = np.uint64(Pt.ctypes.data) + poff * np.uint64(64)
        rows["flags"] = [j.get("flags", 0) for j in jobs]
        # the launch reads every host array before it returns (keep, idx, Pt, rows live until then)
        self.check(self._lib.fsdkr_collect_recover_launch(
            self._h, ctypes.cast(rows.ctypes.data, ctypes.POINTER(RecoverJobC)), J))
        del keep
        return [int(x) for x in n_new]

    def collect_recover_finish(self, handle):
        """Waits for the launched recovery; per job (status, share, y, pk_vec).
        Every job's pk_vec rows land in one array (job k's at its offset) and the
        results are converted in one pass each (no per-job allocations)."""
        n_new = np.asarray(handle, dtype=np.int64)
        J = len(n_new)
        outs = (RecoveredC * J)()
        PK = np.zeros((max(1, int(n_new.sum())), 16), dtype=np.uint32)
        rows = np.frombuffer(outs, dtype=_RECOVERED_DT, count=J) if J else None
        if J:
            off = np.concatenate([[0], np.cumsum(n_new)[:-1]]).astype(np.uint64)
            rows["pk_vec"] = np.uint64(PK.ctypes.data) + off * np.uint64(64)
        self.check(self._lib.fsdkr_collect_recover_finish(self._h, outs))
        if not J:
            return []

        def point(v):
            return None if v == 0 else (v & ((1 << 256) - 1), v >> 256)
        raw = np.frombuffer(outs, dtype=np.uint8).reshape(J, ctypes.sizeof(RecoveredC))
        o_sh, o_y = RecoveredC.share.offset, RecoveredC.y.offset
        shares = limbs_to_ints(raw[:, o_sh:o_sh + 32].copy().view(np.uint32))
        ys = [point(v) for v in limbs_to_ints(raw[:, o_y:o_y + 64].copy().view(np.uint32))]
        pks = [point(v) for v in limbs_to_ints(PK[:int(n_new.sum())])] if n_new.sum() else []
        res, at = [], 0
        for k in range(J):
            n = int(n_new[k])
            res.append((int(rows["status"][k]), shares[k], ys[k], pks[at:at + n]))
            at += n
        return res

    def ec_msm(self, points, scalars):
        """points/scalars: lists (count) of equal-length lists; points are (x, y) or None."""
        from . import _pack
        count, terms = len(points), len(points[0])
        Pt = np.empty((count * terms, 16), dtype=np.uint32)
        _pack.points([pt for row in points for pt in row], None, Pt)
        Sc = ints_to_limbs([s for row in scalars for s in row], 8)
        O = np.zeros((count, 16), dtype=np.uint32)
        self.check(self._lib.fsdkr_ec_msm(self._h, count, terms, _ptr(Pt), _ptr(Sc), _ptr(O)))
        out = []
        for v in limbs_to_ints(O):
            x, y = v & ((1 << 256) - 1), v >> 256
            out.append(None if (x == 0 and y == 0) else (x, y))
        return out
