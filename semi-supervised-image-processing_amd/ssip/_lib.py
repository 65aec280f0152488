"""ctypes binding of libssip_hip.so (the C ABI declared in include/ssip.h).

This is the only place Python touches the native library.  Every call
checks the returned status and raises ``RuntimeError`` with
``ssip_last_error()``; a missing library raises at first use — there is
no CPU fallback in the product path.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

_HERE = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("SSIP_LIB", _HERE / "libssip_hip.so"))
HEADER = _HERE.parents[1] / "include" / "ssip.h"


def abi_version_expected() -> int:
    """SSIP_ABI_VERSION as include/ssip.h declares it (the one source of truth
    for build() and the tests).  Falls back to the compiled-in value of this
    binding when the header is not shipped next to the package."""
    import re

    try:
        m = re.search(r"^#define\s+SSIP_ABI_VERSION\s+(\d+)", HEADER.read_text(), re.M)
    except OSError:
        m = None
    return int(m.group(1)) if m else ABI_VERSION


ABI_VERSION = 14  # must equal include/ssip.h SSIP_ABI_VERSION (tests/test_cpu_abi.py)

F32 = 0
BF16 = 1

_c_int = ctypes.c_int
_c_i64 = ctypes.c_int64
_c_f = ctypes.c_float
_vp = ctypes.c_void_p


class ConvDesc(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("N", "H", "W", "C", "K", "R", "S", "stride", "pad", "P", "Q")]


WPREP_MAX = 32


class WPrep(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("K", "C", "R", "S", "Cp", "Sp")] + [
        ("w_kcrs", ctypes.c_void_p), ("w_krsc", ctypes.c_void_p), ("w_crsk", ctypes.c_void_p),
        ("kscale", ctypes.c_void_p)]


class AugParam(ctypes.Structure):
    _fields_ = [
        ("flip", ctypes.c_int32),
        ("rotate", ctypes.c_int32),
        ("a0", ctypes.c_int32),
        ("a1", ctypes.c_int32),
        ("a3", ctypes.c_int32),
        ("a4", ctypes.c_int32),
        ("xo", ctypes.c_int32),
        ("yo", ctypes.c_int32),
        ("photometric", ctypes.c_int32),
        ("brightness", ctypes.c_float),
        ("contrast", ctypes.c_float),
        ("cut_x0", ctypes.c_int32),
        ("cut_y0", ctypes.c_int32),
        ("cut_x1", ctypes.c_int32),
        ("cut_y1", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
    ]


_PD = ctypes.POINTER(ConvDesc)

# name -> (restype, argtypes)
_SIGS = {
    "ssip_last_error": (ctypes.c_char_p, []),
    "ssip_version": (_c_int, []),
    "ssip_conv_fwd_partial_floats": (_c_i64, [_PD]),
    "ssip_conv_fwd_partial_tiles": (_c_int, [_PD, _c_int]),
    "ssip_conv_fwd": (_c_int, [_PD, _c_int, _vp, _vp, _vp, _vp, _vp]),
    "ssip_conv_dgrad": (_c_int, [_PD, _c_int, _vp, _vp, _vp, _vp, _vp]),
    "ssip_conv_dgrad_ds": (_c_int, [_PD, _c_int, _vp, _vp, _vp, _vp, _vp, _vp]),
    "ssip_conv_fwd_ds_partial_tiles": (_c_int, [_PD, _PD, _c_int]),
    "ssip_conv_fwd_ds": (_c_int, [_PD, _PD, _c_int] + [_vp] * 8),
    "ssip_conv_fwd_bias": (_c_int, [_PD, _c_int, _vp, _vp, _vp, _vp, _c_int, _vp, _vp]),
    "ssip_conv_dgrad_bn_partial_floats": (_c_i64, [_PD]),
    "ssip_conv_dgrad_bn_partial_tiles": (_c_int, [_PD, _c_int]),
    "ssip_conv_dgrad_bn": (_c_int, [_PD, _c_int] + [_vp] * 13),
    "ssip_conv_wgrad_workspace_bytes": (_c_i64, [_PD]),
    "ssip_conv_wgrad_workspace_bytes_budget": (_c_i64, [_PD, _c_int]),
    "ssip_conv_wgrad": (_c_int, [_PD, _c_int, _vp, _vp, _vp, _c_int, _c_int, _c_int, _vp, _c_i64, _vp]),
    "ssip_conv_wgrad_budget": (_c_int, [_PD, _c_int, _vp, _vp, _vp, _c_int, _c_int, _c_int, _vp, _c_i64, _c_int, _vp]),
    "ssip_conv_bnrelu_in_supported": (_c_int, [_PD, _c_int]),
    "ssip_conv_fwd_bnrelu_in": (_c_int, [_PD, _c_int] + [_vp] * 8),
    "ssip_conv_wgrad_bnrelu_in": (_c_int, [_PD, _c_int] + [_vp] * 5 + [_c_int, _vp, _c_i64, _c_int, _vp]),
    "ssip_stem_bwd_wgrad_supported": (_c_int, [_PD, _c_int]),
    "ssip_conv_kernel_name": (_c_int, [_c_int, _PD, _c_int, ctypes.c_char_p, _c_int]),
    "ssip_conv_kernel_name_budget": (_c_int, [_c_int, _PD, _c_int, _c_int, ctypes.c_char_p, _c_int]),
    "ssip_stem_bwd_wgrad": (_c_int, [_PD, _c_int] + [_vp] * 8 + [_c_int] * 3 + [_vp, _c_i64, _vp]),
    "ssip_bn_finalize_scratch_floats": (_c_i64, [_c_int, _c_int]),
    "ssip_bn_finalize": (_c_int, [_c_int, _c_int, _vp, _vp, _vp, _vp, _vp, _c_f, _c_f, _c_int, _vp, _vp, _vp, _vp, _vp]),
    "ssip_bn_eval_coeffs": (_c_int, [_c_int, _vp, _vp, _vp, _vp, _c_f, _vp, _vp, _vp, _vp, _vp]),
    "ssip_bn_apply": (_c_int, [_c_int, _c_i64, _c_int, _vp, _vp, _vp, _vp, _c_int, _vp, _vp, _vp]),
    "ssip_bn_apply2": (_c_int, [_c_int, _c_i64, _c_int, _vp, _vp, _vp, _vp, _vp, _vp, _c_int, _vp, _vp, _vp]),
    "ssip_bn_bwd_dual_partial_floats": (_c_i64, [_c_i64, _c_int]),
    "ssip_bn_bwd_dual": (_c_int, [_c_int, _c_i64, _c_int] + [_vp] * 15 + [_c_int, _vp, _vp, _vp, _vp, _vp]),
    "ssip_bn_bwd_partial_floats": (_c_i64, [_c_i64, _c_int]),
    "ssip_bn_bwd": (_c_int, [_c_int, _c_i64, _c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _c_int, _vp, _vp, _vp, _vp, _vp]),
    "ssip_bn_relu_bwd": (_c_int, [_c_int, _c_i64, _c_int] + [_vp] * 9 + [_c_int, _vp, _vp, _vp, _vp]),
    "ssip_bn_bwd_from_partials": (_c_int, [_c_int, _c_i64, _c_int, _c_int] + [_vp] * 8 + [_c_int, _vp, _vp, _vp]),
    "ssip_relu_bwd": (_c_int, [_c_int, _c_i64, _vp, _vp, _vp, _vp]),
    "ssip_stem_bn_pool_fwd": (_c_int, [_c_int] * 8 + [_vp] * 7),
    "ssip_stem_bn_pool_kernel_name": (_c_int, [_c_int] * 9 + [ctypes.c_char_p, _c_int]),
    "ssip_stem_pool_bn_bwd_partial_floats": (_c_i64, [_c_int] * 4),
    "ssip_stem_pool_bn_bwd": (_c_int, [_c_int] * 8 + [_vp] * 11 + [_c_int] + [_vp] * 4),
    "ssip_maxpool_fwd": (_c_int, [_c_int] * 8 + [_vp, _vp, _vp, _vp]),
    "ssip_maxpool_bwd": (_c_int, [_c_int] * 8 + [_vp, _vp, _vp, _vp]),
    "ssip_avgpool_fc_fwd": (_c_int, [_c_int] * 5 + [_vp] * 6),
    "ssip_avgpool_fc_bwd": (_c_int, [_c_int] * 5 + [_vp] * 6 + [_c_int, _vp]),
    "ssip_cross_entropy": (_c_int, [_c_int, _c_int, _vp, _vp, _c_f, _vp, _vp, _vp, _vp]),
    "ssip_semi_loss": (_c_int, [_c_int, _c_int, _c_int, _vp, _vp, _vp, _vp, _c_f, _c_f, _vp, _vp, _vp, _vp, _vp, _vp]),
    "ssip_softmax_select": (_c_int, [_c_int, _c_int, _vp, _c_f, _c_int, _vp, _vp, _vp, _vp, _vp, _vp]),
    "ssip_resize_h_u8": (_c_int, [_c_int, _vp, _c_i64, _c_int, _c_int, _c_int, _c_int, _vp, _vp, _vp, _vp]),
    "ssip_augment_u8": (
        _c_int,
        [_c_int, _c_int, _vp, _c_i64] + [_c_int] * 9 + [_vp, _vp, _vp, _vp, _vp, _c_int, _vp, _vp],
    ),
    "ssip_nchw_to_nhwc": (_c_int, [_c_int] * 7 + [_vp, _vp, _vp]),
    "ssip_adamw": (_c_int, [_c_i64, _vp, _vp, _vp, _vp, _c_f, _c_f, _c_f, _c_f, _c_f, _c_i64, _c_f, _vp]),
    "ssip_adamw_sched_step": (_c_int, [_vp, _c_f, _c_f, _vp]),
    "ssip_adamw_dev": (_c_int, [_c_i64, _vp, _vp, _vp, _vp, _vp, _c_f, _c_f, _c_f, _c_f, _c_f, _c_int, _vp]),
    "ssip_weight_prep": (_c_int, [_c_int] * 7 + [_vp, _vp, _vp, _vp]),
    "ssip_weight_prep_batch": (_c_int, [_c_int, _c_int, ctypes.POINTER(WPrep), _vp]),
    "ssip_counters_add": (_c_int, [_c_int, _vp, _c_i64, _vp]),
    # launch plans (ssip/plan.py)
    "ssip_plan_create": (_vp, []),
    "ssip_plan_destroy": (None, [_vp]),
    "ssip_plan_fn_index": (_c_int, [ctypes.c_char_p]),
    "ssip_plan_add_call": (_c_int, [_vp, _c_int, _c_int, _vp, _vp, _vp]),
    "ssip_plan_add_event": (_c_int, [_vp, _vp]),
    "ssip_plan_add_wait": (_c_int, [_vp, _vp, _c_int]),
    "ssip_plan_add_marker": (_c_int, [_vp]),
    "ssip_plan_segments": (_c_int, [_vp]),
    "ssip_plan_num_ops": (_c_i64, [_vp]),
    "ssip_plan_run": (_c_int, [_vp, _c_int]),
}

EXPORTED_SYMBOLS = tuple(_SIGS)

_lib = None


def lib() -> ctypes.CDLL:
    """Load (once) and return the native library; raise if it is missing."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise RuntimeError(
                f"ssip native library not found at {LIB_PATH}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)"
            )
        handle = ctypes.CDLL(str(LIB_PATH))
        for name, (res, args) in _SIGS.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    return _lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().ssip_last_error().decode("utf-8", "replace")
        raise RuntimeError(f"{what} failed ({rc}): {msg}")


# int-returning queries (not status codes)
_NOT_STATUS = ("ssip_version", "ssip_conv_fwd_partial_tiles", "ssip_conv_fwd_ds_partial_tiles", "ssip_conv_dgrad_bn_partial_tiles",
               "ssip_stem_bwd_wgrad_supported", "ssip_plan_fn_index", "ssip_plan_segments")

# Active launch-plan recorder (ssip.plan.PlanRecorder) or None.  While set,
# every stream-ordered call made through `call` is also appended to the plan,
# and every tensor whose pointer is taken through `ptr` is kept alive by it.
RECORDER = None


def call(name: str, *args) -> int:
    fn = getattr(lib(), name)
    rc = fn(*args)
    if _SIGS[name][0] is _c_int and name not in _NOT_STATUS:
        check(rc, name)
    if RECORDER is not None:
        RECORDER.on_call(name, args)
    return rc


def ptr(t) -> int:
    """Device pointer of tensor t (kept alive by an active recorder)."""
    if RECORDER is not None:
        RECORDER.keep.append(t)
    return t.data_ptr()
