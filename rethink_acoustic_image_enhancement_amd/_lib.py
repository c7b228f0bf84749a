"""ctypes binding of libkdlae.so (the C ABI declared in include/kdlae.h).

The product path has no CPU fallback: if the shared library is missing or a call fails, a
RuntimeError is raised.  Build it with ``make -C rethink_acoustic_image_enhancement_amd/csrc``
(or ``python -c 'import __graft_entry__ as g; g.build()'``).
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# KDLAE_LIB overrides the library (kernel A/B builds under tools/); default: the in-tree build
LIB_PATH = os.environ.get("KDLAE_LIB") or os.path.join(_HERE, "libkdlae.so")

c_int, c_int64, c_double, c_void_p, c_char_p = (ctypes.c_int, ctypes.c_int64, ctypes.c_double,
                                                ctypes.c_void_p, ctypes.c_char_p)

ERRORS = {0: "OK", 1: "EINVAL_SHAPE", 2: "EINVAL_CONFIG", 3: "EHIP", 4: "EPARAM", 5: "ENOTIMPL",
          6: "ESTATE"}

# Every entry point include/kdlae.h declares (checked by tests/test_abi.py).
EXPORTS = (
    "kdlae_last_error", "kdlae_abi_version",
    "kdlae_t_create", "kdlae_t_destroy", "kdlae_t_num_params", "kdlae_t_param_info",
    "kdlae_t_set_param", "kdlae_t_commit_params", "kdlae_t_params_numel", "kdlae_t_prepare", "kdlae_t_pack_device",
    "kdlae_t_workspace_bytes", "kdlae_t_forward",
    "kdlae_t_probe_arm", "kdlae_t_probe_read",
    "kdlae_t_debug_tap_count", "kdlae_t_debug_tap_info", "kdlae_t_debug_taps",
    "kdlae_s_create", "kdlae_s_destroy", "kdlae_s_num_params", "kdlae_s_param_info",
    "kdlae_s_set_param", "kdlae_s_commit_params", "kdlae_s_params_numel", "kdlae_s_prepare", "kdlae_s_pack_device",
    "kdlae_s_workspace_bytes", "kdlae_s_forward",
    "asdqe_create", "asdqe_destroy", "asdqe_num_params", "asdqe_param_info", "asdqe_set_param",
    "asdqe_commit_params", "asdqe_params_numel", "asdqe_prepare", "asdqe_pack_device", "asdqe_workspace_bytes", "asdqe_forward",
    "kdlae_padded_size", "kdlae_preprocess_u8", "kdlae_frames_preprocess_u8", "kdlae_postprocess_u8",
    "kdlae_tt_create", "kdlae_tt_destroy", "kdlae_tt_num_params", "kdlae_tt_param_info", "kdlae_tt_num_floats",
    "kdlae_tt_workspace_bytes", "kdlae_tt_forward", "kdlae_tt_backward", "kdlae_tt_backward_marked",
    "kdlae_tt_mark_count", "kdlae_tt_mark_lo", "kdlae_tt_mark_wait", "kdlae_tt_mark_sync",
    "kdlae_train_l1sr_scratch_floats", "kdlae_train_l1sr", "kdlae_train_adamw_scratch_floats",
    "kdlae_train_clip_adamw", "kdlae_train_mixup", "kdlae_train_ema",
    "kdlae_st_create", "kdlae_st_destroy", "kdlae_st_num_params", "kdlae_st_param_info", "kdlae_st_num_floats",
    "kdlae_st_workspace_bytes", "kdlae_st_forward", "kdlae_st_backward",
    "kdlae_train_l1frames_scratch_floats", "kdlae_train_l1frames",
    "kdlae_debug_tgemm",
    "kdlae_debug_gemm",
    "kdlae_debug_gemm_variant",
    "kdlae_debug_gram",
    "kdlae_debug_ln",
    "kdlae_debug_small_in",
)


class TConfig(ctypes.Structure):
    """kdlae_t_config (include/kdlae.h) = KDLAE_teacher ctor kwargs (KDLAE_model.py:205-218)."""

    _fields_ = [
        ("inp_channels", c_int), ("out_channels", c_int), ("dim", c_int),
        ("num_blocks", c_int * 4), ("num_refinement_blocks", c_int), ("heads", c_int * 4),
        ("ffn_expansion_factor", c_double), ("bias", c_int), ("layernorm_biasfree", c_int),
        ("dual_pixel_task", c_int), ("static_train", c_int), ("params_cat", c_int),
    ]


class SConfig(ctypes.Structure):
    """kdlae_s_config (include/kdlae.h) = KDLAE_student ctor kwargs (KDLAE_model.py:341-342)."""

    _fields_ = [
        ("inp_channels", c_int), ("out_channels", c_int), ("residual", c_int), ("num_hidden", c_int),
        ("hidden_channels", c_int * 8), ("kernel_size", c_int),
    ]


class AConfig(ctypes.Structure):
    """asdqe_config (include/kdlae.h) = DenoiseRatePredictor ctor kwargs (ASDQE_model.py:127)."""

    _fields_ = [("in_channels", c_int), ("dim", c_int)]


_lib = None


def lib() -> ctypes.CDLL:
    """Load libkdlae.so once; raise loudly if it is missing (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} is missing: the KDLAE HIP path has no CPU fallback. Build it with "
            "`make -C rethink_acoustic_image_enhancement_amd/csrc` (hipcc, gfx950).")
    L = ctypes.CDLL(LIB_PATH)
    L.kdlae_last_error.restype = c_char_p
    L.kdlae_abi_version.restype = c_int
    L.kdlae_t_create.argtypes = [ctypes.POINTER(TConfig), c_int, ctypes.POINTER(c_void_p)]
    L.kdlae_t_destroy.argtypes = [c_void_p]
    L.kdlae_t_num_params.argtypes = [c_void_p]
    L.kdlae_t_param_info.argtypes = [c_void_p, c_int, ctypes.POINTER(c_char_p), ctypes.POINTER(c_int64)]
    L.kdlae_t_set_param.argtypes = [c_void_p, c_char_p, c_void_p, c_int64]
    L.kdlae_t_commit_params.argtypes = [c_void_p, c_void_p]
    for pre in ("kdlae_t", "kdlae_s", "asdqe"):
        getattr(L, pre + "_params_numel").argtypes = [c_void_p]
        getattr(L, pre + "_params_numel").restype = c_int64
        getattr(L, pre + "_pack_device").argtypes = [c_void_p, c_void_p, c_int64, c_void_p]
        getattr(L, pre + "_prepare").argtypes = [c_void_p]
    L.kdlae_t_workspace_bytes.argtypes = [c_void_p, c_int, c_int, c_int]
    L.kdlae_t_workspace_bytes.restype = c_int64
    L.kdlae_t_forward.argtypes = [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p,
                                  c_void_p, c_int64, c_void_p]
    L.kdlae_t_probe_arm.argtypes = [c_void_p, c_int, c_int]
    L.kdlae_t_probe_read.argtypes = [c_void_p, ctypes.POINTER(c_double), ctypes.POINTER(c_int64),
                                     ctypes.POINTER(c_double), ctypes.POINTER(c_double)]
    L.kdlae_t_debug_tap_count.argtypes = [c_void_p]
    L.kdlae_t_debug_tap_info.argtypes = [c_void_p, c_int, c_char_p, c_int, ctypes.POINTER(c_int),
                                         ctypes.POINTER(c_int), ctypes.POINTER(c_int)]
    L.kdlae_t_debug_taps.argtypes = [c_void_p, c_int, ctypes.POINTER(c_void_p)]
    L.kdlae_s_create.argtypes = [ctypes.POINTER(SConfig), c_int, ctypes.POINTER(c_void_p)]
    L.kdlae_s_destroy.argtypes = [c_void_p]
    L.kdlae_s_num_params.argtypes = [c_void_p]
    L.kdlae_s_param_info.argtypes = [c_void_p, c_int, ctypes.POINTER(c_char_p), ctypes.POINTER(c_int64)]
    L.kdlae_s_set_param.argtypes = [c_void_p, c_char_p, c_void_p, c_int64]
    L.kdlae_s_commit_params.argtypes = [c_void_p, c_void_p]
    L.kdlae_s_workspace_bytes.argtypes = [c_void_p, c_int, c_int, c_int, c_int]
    L.kdlae_s_workspace_bytes.restype = c_int64
    L.kdlae_s_forward.argtypes = [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int64,
                                  c_void_p]
    L.asdqe_create.argtypes = [ctypes.POINTER(AConfig), c_int, ctypes.POINTER(c_void_p)]
    L.asdqe_destroy.argtypes = [c_void_p]
    L.asdqe_num_params.argtypes = [c_void_p]
    L.asdqe_param_info.argtypes = [c_void_p, c_int, ctypes.POINTER(c_char_p), ctypes.POINTER(c_int64)]
    L.asdqe_set_param.argtypes = [c_void_p, c_char_p, c_void_p, c_int64]
    L.asdqe_commit_params.argtypes = [c_void_p, c_void_p]
    L.asdqe_workspace_bytes.argtypes = [c_void_p, c_int, c_int, c_int]
    L.asdqe_workspace_bytes.restype = c_int64
    L.asdqe_forward.argtypes = [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                c_int64, c_void_p]
    L.kdlae_padded_size.argtypes = [c_int, c_int, c_int, ctypes.POINTER(c_int), ctypes.POINTER(c_int)]
    L.kdlae_padded_size.restype = None
    L.kdlae_preprocess_u8.argtypes = [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                                      c_void_p, c_void_p]
    L.kdlae_frames_preprocess_u8.argtypes = [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p,
                                             c_void_p]
    L.kdlae_postprocess_u8.argtypes = [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int,
                                       c_void_p, c_void_p]
    L.kdlae_tt_create.argtypes = [ctypes.POINTER(TConfig), c_int, ctypes.POINTER(c_void_p)]
    L.kdlae_tt_destroy.argtypes = [c_void_p]
    L.kdlae_tt_num_params.argtypes = [c_void_p]
    L.kdlae_tt_param_info.argtypes = [c_void_p, c_int, ctypes.POINTER(c_char_p), ctypes.POINTER(c_int64),
                                      ctypes.POINTER(c_int64)]
    L.kdlae_tt_num_floats.argtypes = [c_void_p]
    L.kdlae_tt_num_floats.restype = c_int64
    L.kdlae_tt_workspace_bytes.argtypes = [c_void_p, c_int, c_int, c_int]
    L.kdlae_tt_workspace_bytes.restype = c_int64
    L.kdlae_tt_forward.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p,
                                   c_void_p, c_void_p, ctypes.c_size_t, c_void_p]
    L.kdlae_tt_backward.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_size_t,
                                    c_void_p]
    L.kdlae_tt_backward_marked.argtypes = L.kdlae_tt_backward.argtypes
    L.kdlae_tt_mark_count.argtypes = [c_void_p]
    L.kdlae_tt_mark_lo.argtypes = [c_void_p, c_int]
    L.kdlae_tt_mark_lo.restype = c_int64
    L.kdlae_tt_mark_wait.argtypes = [c_void_p, c_int, c_void_p]
    L.kdlae_tt_mark_sync.argtypes = [c_void_p, c_int]
    L.kdlae_train_l1sr_scratch_floats.argtypes = []
    L.kdlae_train_l1sr_scratch_floats.restype = c_int64
    L.kdlae_train_l1sr.argtypes = [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_void_p, c_void_p,
                                   c_void_p, c_void_p, c_void_p]
    L.kdlae_train_adamw_scratch_floats.argtypes = []
    L.kdlae_train_adamw_scratch_floats.restype = c_int64
    c_float = ctypes.c_float
    L.kdlae_train_clip_adamw.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_float, c_float,
                                         c_float, c_float, c_float, c_float, c_float, c_int, c_void_p, c_int, c_void_p,
                                         c_void_p]
    L.kdlae_train_mixup.argtypes = [c_void_p, c_void_p, c_int, c_int64, c_void_p, c_float, c_void_p]
    L.kdlae_train_ema.argtypes = [c_void_p, c_void_p, c_int64, c_float, c_void_p]
    L.kdlae_st_create.argtypes = [ctypes.POINTER(SConfig), c_int, ctypes.POINTER(c_void_p)]
    L.kdlae_st_destroy.argtypes = [c_void_p]
    L.kdlae_st_num_params.argtypes = [c_void_p]
    L.kdlae_st_param_info.argtypes = [c_void_p, c_int, ctypes.POINTER(c_char_p), ctypes.POINTER(c_int64),
                                      ctypes.POINTER(c_int64)]
    L.kdlae_st_num_floats.argtypes = [c_void_p]
    L.kdlae_st_num_floats.restype = c_int64
    L.kdlae_st_workspace_bytes.argtypes = [c_void_p, c_int, c_int, c_int, c_int]
    L.kdlae_st_workspace_bytes.restype = c_int64
    L.kdlae_st_forward.argtypes = [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                                   c_int64, c_void_p]
    L.kdlae_st_backward.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p]
    L.kdlae_train_l1frames_scratch_floats.argtypes = []
    L.kdlae_train_l1frames_scratch_floats.restype = c_int64
    L.kdlae_train_l1frames.argtypes = [c_void_p, c_void_p, c_int, c_int, c_int64, ctypes.c_float, ctypes.c_float,
                                       ctypes.c_float, c_int, c_void_p, c_void_p, c_void_p, c_void_p]
    L.kdlae_debug_tgemm.argtypes = [c_void_p, c_void_p]
    for f in ("kdlae_debug_gemm", "kdlae_debug_gram", "kdlae_debug_ln", "kdlae_debug_small_in"):
        getattr(L, f).argtypes = [c_void_p, c_void_p]
    L.kdlae_debug_gemm_variant.argtypes = [c_int, c_int, ctypes.POINTER(c_int)]
    for name in EXPORTS:
        if not name.endswith(("_last_error", "_abi_version", "_workspace_bytes", "_padded_size", "_num_floats",
                              "_scratch_floats", "_params_numel", "_mark_lo")):
            getattr(L, name).restype = c_int
    _lib = L
    return L


def last_error() -> str:
    msg = lib().kdlae_last_error()
    return msg.decode() if msg else ""


def check(rc: int, what: str) -> None:
    if rc != 0:
        err = last_error()
        code = ERRORS.get(rc, str(rc))
        if rc == 5:
            raise NotImplementedError(f"{what}: {err}")
        raise RuntimeError(f"{what} failed ({code}): {err}")
