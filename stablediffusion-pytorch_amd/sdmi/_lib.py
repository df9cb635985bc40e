"""ctypes binding of the C ABI declared in include/sdmi.h (libsdmi.so, built in-tree for gfx950).

The product path has no fallback: if the library is missing or fails to load, every op raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libsdmi.so")

# ---- enums (include/sdmi.h) ----
A_ROWMAJOR, A_CONV, A_COLMAJOR = 0, 1, 2
B_NK, B_KN, B_KN_CONV = 0, 1, 2


class ConvGeom(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in
                ("ih", "iw", "cin", "ldx", "kh", "kw", "oh_log2", "ow_log2", "sy", "sx", "oy0", "ox0")]


class GemmDesc(ctypes.Structure):
    _fields_ = [
        ("m", ctypes.c_int), ("n", ctypes.c_int), ("k", ctypes.c_int),
        ("a_mode", ctypes.c_int), ("b_mode", ctypes.c_int),
        ("a", ctypes.c_void_p), ("lda", ctypes.c_int),
        ("b", ctypes.c_void_p), ("ldb", ctypes.c_int),
        ("geom", ConvGeom),
        ("c", ctypes.c_void_p), ("ldc", ctypes.c_int), ("c_f32", ctypes.c_int),
        ("bias", ctypes.c_void_p),
        ("rowbias", ctypes.c_void_p), ("rb_ld", ctypes.c_int), ("rb_shift", ctypes.c_int),
        ("resid", ctypes.c_void_p), ("ldr", ctypes.c_int),
        ("alpha", ctypes.c_float),
        ("act", ctypes.c_int),
        ("remap", ctypes.c_int), ("r_gh_log2", ctypes.c_int), ("r_gw_log2", ctypes.c_int),
        ("r_oh", ctypes.c_int), ("r_ow", ctypes.c_int), ("r_sy", ctypes.c_int), ("r_sx", ctypes.c_int),
        ("r_oy", ctypes.c_int), ("r_ox", ctypes.c_int),
        ("perm", ctypes.c_int), ("p_cin", ctypes.c_int), ("p_taps", ctypes.c_int),
    ]


_lib = None

# (name, argtypes) of every exported entry point; used for loading and for the export test.
_P, _I, _F, _L = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_longlong
SIGNATURES = {
    "sdmi_gemm_plan": [ctypes.POINTER(GemmDesc), ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_size_t)],
    "sdmi_gemm": [ctypes.POINTER(GemmDesc), _P, ctypes.c_size_t, _P],
}


def lib():
    """Load libsdmi.so once (raises if absent: there is no CPU fallback on the product path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libsdmi.so not built ({LIB_PATH}); run __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH)
        for name, argt in SIGNATURES.items():
            fn = getattr(L, name)
            fn.argtypes = argt
            fn.restype = ctypes.c_int
        _lib = L
    return _lib


class SdmiError(RuntimeError):
    pass


def check(rc, what):
    if rc != 0:
        raise SdmiError(f"{what} failed with status {rc}")
