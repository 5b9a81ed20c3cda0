"""ctypes binding of libfsdkr.so (include/fsdkr/fsdkr.h).

The product path is the HIP library: loading fails loudly if it is missing,
and there is no CPU fallback anywhere in this package."""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libfsdkr.so")

FSDKR_OK = 0
FSDKR_E_ARG = -1
FSDKR_E_HIP = -2
FSDKR_E_OOM = -3
FSDKR_E_UNSUPPORTED = -4
FSDKR_CFG_TIMING = 1

u32p = ctypes.POINTER(ctypes.c_uint32)


class FsdkrError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"fsdkr error {code}: {msg}")
        self.code = code


class _Cfg(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("flags", ctypes.c_uint32)]


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
    L.fsdkr_ctx_destroy.argtypes = [vp]
    L.fsdkr_ctx_destroy.restype = None
    L.fsdkr_last_error.argtypes = [vp]
    L.fsdkr_last_error.restype = ctypes.c_char_p
    L.fsdkr_device_available.argtypes = []
    L.fsdkr_device_available.restype = ctypes.c_int
    L.fsdkr_modexp_batch.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, u32p, u32p, ctypes.c_uint32, u32p, u32p,
                                     ctypes.c_uint32, u32p]
    L.fsdkr_modexp_batch.restype = ctypes.c_int
    L.fsdkr_modexp_batch_device.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, vp, vp, ctypes.c_uint32,
                                            ctypes.c_uint32, vp, vp, ctypes.c_uint32, vp]
    L.fsdkr_modexp_batch_device.restype = ctypes.c_int
    L.fsdkr_kernel_time.argtypes = [vp, ctypes.c_char_p, ctypes.POINTER(ctypes.c_double),
                                    ctypes.POINTER(ctypes.c_uint32)]
    L.fsdkr_kernel_time.restype = ctypes.c_int
    L.fsdkr_kernel_time_reset.argtypes = [vp]
    L.fsdkr_kernel_time_reset.restype = None
    _lib = L
    return L


def _ptr(a):
    return a.ctypes.data_as(u32p)


def ints_to_limbs(values, limbs):
    """list of non-negative ints -> (len, limbs) uint32 little-endian array."""
    out = np.zeros((len(values), limbs), dtype=np.uint32)
    nbytes = 4 * limbs
    buf = bytearray(nbytes * len(values))
    for i, v in enumerate(values):
        if v < 0 or v.bit_length() > 32 * limbs:
            raise ValueError(f"value {i} does not fit {limbs} limbs")
        buf[i * nbytes:(i + 1) * nbytes] = v.to_bytes(nbytes, "little")
    out[:] = np.frombuffer(bytes(buf), dtype=np.uint32).reshape(len(values), limbs)
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

    def modexp_batch(self, bases, exps, mods, mod_idx, mod_limbs):
        """[base_i ^ exp_i mod mods[mod_idx_i]] computed on the GPU."""
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
        self.check(self._lib.fsdkr_modexp_batch(self._h, mod_limbs, count, _ptr(B), _ptr(E), exp_limbs, _ptr(I),
                                                _ptr(Mo), len(mods), _ptr(O)))
        return limbs_to_ints(O)
