"""ctypes binding of the C ABI declared in include/sdmi.h (libsdmi.so, built in-tree for gfx950).

The product path has no fallback: if the library is missing or fails to load, every op raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
DEFAULT_LIB_PATH = os.path.join(_HERE, "libsdmi.so")
# SDMI_LIB_PATH: A/B timing of two builds only. It is announced on stderr when it takes effect, and the test suite
# refuses to run under it (tests/conftest.py), so a leaked variable cannot make the parity tests bind a stale library.
LIB_PATH = os.environ.get("SDMI_LIB_PATH") or DEFAULT_LIB_PATH

# ---- enums (include/sdmi.h) ----
A_ROWMAJOR, A_CONV, A_COLMAJOR = 0, 1, 2
B_NK, B_KN, B_KN_CONV = 0, 1, 2


class ConvGeom(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in
                ("ih", "iw", "cin", "ldx", "kh", "kw", "oh", "ow", "sy", "sx", "oy0", "ox0")]


class GemmDesc(ctypes.Structure):
    _fields_ = [
        ("m", ctypes.c_int), ("n", ctypes.c_int), ("k", ctypes.c_int),
        ("a_mode", ctypes.c_int), ("b_mode", ctypes.c_int),
        ("a", ctypes.c_void_p), ("lda", ctypes.c_int),
        ("b", ctypes.c_void_p), ("ldb", ctypes.c_int),
        ("geom", ConvGeom),
        ("c", ctypes.c_void_p), ("ldc", ctypes.c_int), ("c_f32", ctypes.c_int),
        ("bias", ctypes.c_void_p),
        ("rowbias", ctypes.c_void_p), ("rb_ld", ctypes.c_int), ("rb_div", ctypes.c_int),
        ("resid", ctypes.c_void_p), ("ldr", ctypes.c_int),
        ("alpha", ctypes.c_float),
        ("act", ctypes.c_int),
        ("remap", ctypes.c_int), ("r_gh", ctypes.c_int), ("r_gw", ctypes.c_int),
        ("r_oh", ctypes.c_int), ("r_ow", ctypes.c_int), ("r_sy", ctypes.c_int), ("r_sx", ctypes.c_int),
        ("r_oy", ctypes.c_int), ("r_ox", ctypes.c_int),
        ("perm", ctypes.c_int), ("p_cin", ctypes.c_int), ("p_taps", ctypes.c_int), ("p_cvalid", ctypes.c_int),
        ("m_store", ctypes.c_int), ("n_store", ctypes.c_int),
        ("a2", ctypes.c_void_p), ("lda2", ctypes.c_int), ("k_split", ctypes.c_int),
        ("bias2", ctypes.c_void_p),
        ("rb_mod", ctypes.c_int),
        ("aux", ctypes.c_void_p), ("ld_aux", ctypes.c_int),
        ("splits_hint", ctypes.c_int),
        ("tile_n_hint", ctypes.c_int),
        ("sum_out", ctypes.c_void_p), ("sum_out2", ctypes.c_void_p), ("gsum_out", ctypes.c_void_p),
        ("gsum_ld", ctypes.c_int), ("sum_group", ctypes.c_int),
        ("variant_hint", ctypes.c_int),
        ("gn_x", ctypes.c_void_p), ("gn_ldx", ctypes.c_int),
        ("gn_tab", ctypes.c_void_p),
        ("gn_part", ctypes.c_void_p),
        ("gn_P", ctypes.c_int), ("gn_rb", ctypes.c_int), ("gn_silu", ctypes.c_int),
    ]


_lib = None

# (name, argtypes) of every exported entry point; used for loading and for the export test.
_P, _I, _F, _L = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_longlong
_SZ = ctypes.c_size_t


class GnRowsJob(ctypes.Structure):
    _fields_ = [("rows", ctypes.c_void_p), ("dgamma", ctypes.c_void_p), ("dbeta", ctypes.c_void_p),
                ("B", ctypes.c_int), ("C", ctypes.c_int)]


GN_ROWS_GROUP_MAX = 16


class TPackDesc(ctypes.Structure):
    _fields_ = [("src", ctypes.c_void_p), ("dst", ctypes.c_void_p)] + [(n, ctypes.c_int) for n in (
        "O", "I", "taps", "src_ld", "src_tap", "dst_ld", "dst_tap")] + [("smap", ctypes.c_byte * 16)]


class PackDesc(ctypes.Structure):
    _fields_ = [("src", ctypes.c_void_p), ("dst", ctypes.c_void_p),
                ("so", ctypes.c_longlong), ("si", ctypes.c_longlong), ("skh", ctypes.c_longlong),
                ("skw", ctypes.c_longlong)] + [(n, ctypes.c_int) for n in
                                                ("O", "I", "Ipad", "KH", "KW", "kh_off", "kh_mul", "kw_off", "kw_mul",
                                                 "dst_ld")]


SIGNATURES = {
    "sdmi_gemm_plan": ([ctypes.POINTER(GemmDesc), ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_size_t)], _I),
    "sdmi_gemm": ([ctypes.POINTER(GemmDesc), _P, _SZ, _P], _I),
    "sdmi_gemm_grouped_plan": ([ctypes.POINTER(GemmDesc), _I, ctypes.POINTER(ctypes.c_int),
                                ctypes.POINTER(ctypes.c_size_t)], _I),
    "sdmi_gemm_grouped": ([ctypes.POINTER(GemmDesc), _I, _P, _SZ, _P], _I),
    "sdmi_gemm_kernel_info": ([ctypes.POINTER(GemmDesc), ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)],
                              _I),
    "sdmi_attn_fwd": ([_P, _I, _P, _I, _P, _I, _P, _I, _P, _I, _I, _I, _I, _I, _P], _I),
    "sdmi_attn_bwd": ([_P, _I, _P, _I, _P, _I, _P, _I, _P, _I, _P, _P, _P, _I, _P, _I, _P, _I,
                       _I, _I, _I, _I, _I, _P], _I),
    "sdmi_attn_bwd_workspace": ([_I, _I, _I, _I, _I], _SZ),
    "sdmi_attn_bwd_fused": ([_P, _I, _P, _I, _P, _I, _P, _I, _P, _I, _P, _P, _P, _SZ, _P, _I, _P, _I, _P, _I,
                             _I, _I, _I, _I, _I, _P], _I),
    "sdmi_chan_reduce_workspace": ([_I, _I, _I], _SZ),
    "sdmi_gn_stats": ([_P, _I, _I, _I, _I, _I, _F, _P, _P, _P, _P, _P], _I),
    "sdmi_gn_apply": ([_P, _I, _P, _I, _P, _I, _I, _I, _I, _P], _I),
    "sdmi_gn_fwd": ([_P, _I, _P, _I, _I, _I, _I, _I, _F, _P, _P, _I, _P, _P, _P], _I),
    "sdmi_gn_bwd": ([_P, _I, _P, _I, _P, _I, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _I, _P], _I),
    "sdmi_gn_bwd_part": ([_P, _I, _P, _I, _P, _I, _P, _P, _I, _I, _I, _I, _I, _P, _I, _P, _P, _P, _P, _I, _P], _I),
    "sdmi_gn_bwd_rows": ([_P, _I, _P, _I, _P, _I, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _I, _P], _I),
    "sdmi_gn_bwd_part_rows": ([_P, _I, _P, _I, _P, _I, _P, _P, _I, _I, _I, _I, _I, _P, _I, _P, _P, _P, _I, _P], _I),
    "sdmi_gn_rows_sum": ([_P, _I, _I, _P, _P, _P], _I),
    "sdmi_gn_rows_sum_grouped": ([_P, _I, _P], _I),
    "sdmi_chan_sum": ([_P, _I, _I, _I, _I, _P, _P, _I, _P, _P, _I, _P], _I),
    "sdmi_prep_input": ([_P, _I, _I, _I, _I, _P, _I, _I, _I, _P, _I, _P, _I, _P, _P], _I),
    "sdmi_cond_wgrad": ([_P, _I, _I, _I, _I, _I, _P, _I, _I, _I, _I, _P, _P, _P], _I),
    "sdmi_prep_input_cmap": ([_P, _I, _I, _I, _I, _P, _I, _I, _I, _P, _I, _P, _I, _P, _P], _I),
    "sdmi_cond_wgrad_cmap": ([_P, _I, _I, _I, _I, _I, _P, _I, _I, _I, _I, _P, _P, _P], _I),
    "sdmi_nhwc_to_nchw": ([_P, _I, _I, _I, _I, _I, _P, _P], _I),
    "sdmi_nchw_to_nhwc_bf16": ([_P, _I, _I, _I, _P, _I, _P], _I),
    "sdmi_add_noise": ([_P, _P, _P, _P, _P, _I, _L, _P, _P], _I),
    "sdmi_mse_workspace": ([], _SZ),
    "sdmi_mse": ([_P, _I, _P, _I, _I, _I, _F, _P, _P, _P, _P, _P], _I),
    "sdmi_time_embedding": ([_P, _I, _I, _I, _P, _I, _P, _P], _I),
    "sdmi_silu": ([_P, _P, _P, _L, _P], _I),
    "sdmi_copy_slice": ([_P, _I, _P, _I, _L, _I, _I, _P], _I),
    "sdmi_pack_chunk": ([], _I),
    "sdmi_pack_weights": ([_P, _P, _I, _P], _I),
    "sdmi_pack_transpose": ([_P, _P, _I, _P], _I),
    "sdmi_optim_workspace": ([], _SZ),
    "sdmi_clip_unscale": ([_P, _L, _F, _P, _P, _I, _I, _F, _P], _I),
    "sdmi_optim_workspace_for": ([_L], _SZ),
    "sdmi_clip_unscale_ws": ([_P, _L, _F, _P, _P, _SZ, _I, _I, _F, _P], _I),
    "sdmi_loss_flag": ([_P, _P, _I, _P], _I),
    "sdmi_clip_finalize": ([_P, _I, _F, _P, _I, _I, _F, _P], _I),
    "sdmi_norm_block": ([], _L),
    "sdmi_sumsq_blocks": ([_P, _L, _P, _P], _I),
    "sdmi_widen_bf16_sumsq": ([_P, _P, _L, _P, _P], _I),
    "sdmi_adam_ema": ([_P, _P, _P, _P, _P, _L, _P, _F, _F, _F, _F, _F, _F, _P], _I),
    "sdmi_adam_ema_bf16": ([_P, _P, _P, _P, _P, _L, _P, _F, _F, _F, _F, _F, _F, _P, _P], _I),
    "sdmi_cast_bf16": ([_P, _P, _L, _P], _I),
    "sdmi_resize_nearest": ([_P, _I, _I, _I, _P, _I, _I, _P], _I),
    "sdmi_chan_copy": ([_P, _I, _I, _P, _I, _I, _I, _I, _L, _P], _I),
    "sdmi_modulate_fwd": ([_P, _P, _P, _P, _I, _F, _P, _I, _I, _I, _P], _I),
    "sdmi_modulate_bwd": ([_P, _P, _P, _I, _F, _P, _P, _P, _I, _I, _I, _P], _I),
    "sdmi_attn_map": ([_P, _I, _P, _I, _I, _I, _I, _I, _I, _F, _I, _P, _P], _I),
    "sdmi_ln_chunk_rows": ([_I], _I),
    "sdmi_ln_mod_fwd": ([_P, _I, _P, _I, _P, _P, _I, _P, _P, _I, _P, _I, _P, _P, _I, _I, _I, _F, _I, _P], _I),
    "sdmi_ln_mod_bwd": ([_P, _I, _P, _P, _P, _I, _P, _I, _P, _I, _P, _I, _P, _P, _I, _P, _P, _I, _P, _I, _P,
                         _I, _I, _I, _I, _P, _I, _P], _I),
    "sdmi_mod_finalize": ([_P, _I, _I, _I, _I, _P, _I, _P], _I),
    "sdmi_tokens_to_nchw": ([_P, _I, _I, _I, _I, _I, _I, _I, _P, _P], _I),
    "sdmi_nchw_to_tokens_bf16": ([_P, _I, _I, _I, _I, _I, _P, _I, _P], _I),
    "sdmi_vq_workspace": ([_L], _SZ),
    "sdmi_vq_quantize": ([_P, _I, _P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P], _I),
    "sdmi_pointwise_in": ([_P, _I, _I, _I, _P, _P, _I, _P, _I, _P], _I),
    "sdmi_ddpm_prev": ([_P, _P, _P, _L, _P, _P, _P, _P, _P, _P, _P, _I, _P], _I),
    "sdmi_ddim_prev": ([_P, _P, _P, _L, _F, _F, _F, _P, _P], _I),
    "sdmi_ddim_prev_dev": ([_P, _P, _P, _L, _P, _P, _P, _P, _P, _F, _P, _I, _P], _I),
    "sdmi_affine_step": ([_P, _P, _P, _L, _F, _F, _F, _P, _P], _I),
    "sdmi_mse_patch": ([_P, _I, _P, _I, _I, _I, _I, _I, _F, _P, _P, _P, _P, _P], _I),
    "sdmi_randn": ([_P, _L, ctypes.c_ulonglong, _P, _I, _P], _I),
    "sdmi_step_draw": ([_P, _L, _P, _I, _I, _P, _P, _P, _L, ctypes.c_float, _P, ctypes.c_float, ctypes.c_ulonglong,
                        ctypes.c_ulonglong, _P], _I),
    "sdmi_relu": ([_P, _P, _P, _L, _P], _I),
    "sdmi_vq_bwd_workspace": ([], _SZ),
    "sdmi_vq_bwd": ([_P, _I, _P, _P, _P, _P, _P, _I, _P, _I, _P, _I, _I, _I, _F, _F, _P, _I, _P, _P, _P, _P, _P, _P,
                     _P, _P, _P], _I),
    "sdmi_plan_begin": ([], _I),
    "sdmi_plan_end": ([ctypes.POINTER(ctypes.c_void_p)], _I),
    "sdmi_plan_recording": ([], _I),
    "sdmi_plan_note_event": ([_P, _P], _I),
    "sdmi_plan_note_wait": ([_P, _P], _I),
    "sdmi_plan_note_callout": ([_I], _I),
    "sdmi_plan_info": ([_P, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)], _I),
    "sdmi_plan_replay": ([_P, _I, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)], _I),
    "sdmi_plan_destroy": ([_P], _I),
    "sdmi_plan_op_stream": ([_P, _I, ctypes.POINTER(ctypes.c_void_p)], _I),
    "sdmi_plan_op_info": ([_P, _I, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_char_p),
                           ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)], _I),
    "sdmi_plan_time_op": ([_P, _I, _I, _I, ctypes.POINTER(ctypes.c_float)], _I),
    "sdmi_comm_load": ([ctypes.c_char_p], _I),
    "sdmi_comm_unique_id": ([_P], _I),
    "sdmi_comm_init": ([_P, _I, _I, ctypes.POINTER(ctypes.c_void_p)], _I),
    "sdmi_allreduce": ([_P, _P, _L, _I, _P], _I),
    "sdmi_comm_destroy": ([_P], _I),
}


class _Lib:
    """libsdmi.so with argument / result types set on every entry point of include/sdmi.h. Launches made while a
    native plan records (sdmi.plan.StepPlan) are captured inside the library itself (csrc/plan.hip)."""

    def __init__(self, cdll):
        self._cdll = cdll
        ab = bool(os.environ.get("SDMI_LIB_PATH"))  # A/B timing against an older library: newer entry points may lack
        for name, (argt, rest) in SIGNATURES.items():
            if ab and not hasattr(cdll, name):
                continue
            fn = getattr(cdll, name)
            fn.argtypes = argt
            fn.restype = rest
            setattr(self, name, fn)


def lib():
    """Load libsdmi.so once (raises if absent: there is no CPU fallback on the product path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libsdmi.so not built ({LIB_PATH}); run __graft_entry__.build()")
        # torch must bring in its HIP runtime first: libsdmi.so's libamdhip64.so.7 dependency then binds
        # to that same (already loaded, same SONAME) runtime instead of loading a second copy.
        import torch  # noqa: F401
        if os.path.abspath(LIB_PATH) != DEFAULT_LIB_PATH:
            import sys
            print(f"sdmi: SDMI_LIB_PATH override in effect, loading {LIB_PATH} (A/B timing only)", file=sys.stderr)
        _lib = _Lib(ctypes.CDLL(LIB_PATH))
    return _lib


class SdmiError(RuntimeError):
    pass


def check(rc, what):
    if rc != 0:
        raise SdmiError(f"{what} failed with status {rc}")
