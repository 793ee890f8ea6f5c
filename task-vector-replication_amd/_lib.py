"""ctypes binding of ``libtvr.so`` (the C ABI declared in include/tvr.h).

The reference is Python, so its binding to a native engine is a ctypes stub
(INTEGRATION.md).  The compute entry points (clean forward, patch sweep, head
projection, logits) are called as torch.library operators ``torch.ops.tvr.*``
registered by ``_tvr_ops.so`` (csrc/torch_ops.cpp, over the same C ABI:
load_ops); handle lifetime, GEMM mode, traces and profiling stay on ctypes.
Loading fails loudly: there is no CPU fallback anywhere in the product path.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

LIB_NAME = "libtvr.so"
OPS_NAME = "_tvr_ops.so"
# TVR_LIB: another in-tree build of the engine (same-box A/B of two builds)
LIB_PATH = Path(os.environ["TVR_LIB"]).resolve() if os.environ.get("TVR_LIB") else Path(__file__).resolve().parent / LIB_NAME

# enum tvr_status
TVR_OK = 0
TVR_ERR_INVALID = -1
TVR_ERR_HIP = -2
TVR_ERR_NOMEM = -3
TVR_ERR_UNSUPPORTED = -4
TVR_ERR_RANGE = -5
TVR_ERR_INTERNAL = -6

# enum tvr_trace_hook
TRACE_RESID_PRE = 0
TRACE_Z = 1

# enum tvr_site_kind
SITE_NONE = 0
SITE_REPLACE_HEAD_ALLPOS = 1
SITE_ADD_ATTN_OUT_LASTPOS = 2
SITE_SET_RESID_PRE_POS = 3

c_f32p = ctypes.c_void_p
c_i32p = ctypes.c_void_p


class CLayerWeights(ctypes.Structure):
    _fields_ = [("w1", ctypes.c_void_p), ("b1", ctypes.c_void_p),
                ("w2", ctypes.c_void_p), ("b2", ctypes.c_void_p)]


class CExact16Layer(ctypes.Structure):
    _fields_ = [("w1", ctypes.c_void_p), ("w2", ctypes.c_void_p), ("g1", ctypes.c_void_p), ("g2", ctypes.c_void_p)]


class CSite(ctypes.Structure):
    _fields_ = [("seq", ctypes.c_int32), ("kind", ctypes.c_int32), ("layer", ctypes.c_int32),
                ("head", ctypes.c_int32), ("pos", ctypes.c_int32), ("src_seq", ctypes.c_int32),
                ("src_pos", ctypes.c_int32), ("vec", ctypes.c_int32), ("target", ctypes.c_int32)]


SITE_FIELDS = [f for f, _ in CSite._fields_]


class CKernelStats(ctypes.Structure):
    _fields_ = [("gemm_launches", ctypes.c_int64 * 3), ("gemm_flops", ctypes.c_double * 3),
                ("gemm_ms", ctypes.c_double * 3), ("gemm_bytes", ctypes.c_double * 3)]


GEMM_VARIANTS = ("unembed", "qkv_mlpin", "o_mlpout")


class CHbmStats(ctypes.Structure):
    _fields_ = [("launches", ctypes.c_int64 * 6), ("ms", ctypes.c_double * 6), ("bytes", ctypes.c_double * 6)]


# include/tvr.h enum tvr_hbm_kind
HBM_KINDS = ("entry", "capture", "lnpre", "attention", "row_stats", "lin_entry")

# name -> (restype, argtypes); every symbol include/tvr.h declares.
ABI_VERSION = 11  # include/tvr.h TVR_ABI_VERSION

# include/tvr.h enum tvr_gemm_mode
GEMM_MODES = {"f32": 0, "x3bf16": 1, "x2f16": 2, "bf16": 3}
GEMM_NAMES = {v: k for k, v in GEMM_MODES.items()}

SIGNATURES = {
    "tvr_version": (ctypes.c_char_p, []),
    "tvr_abi_version": (ctypes.c_int32, []),
    "tvr_last_error": (ctypes.c_char_p, []),
    "tvr_model_create": (ctypes.c_int, [ctypes.c_void_p, c_f32p, ctypes.POINTER(CLayerWeights),
                                        c_f32p, c_f32p, ctypes.POINTER(ctypes.c_void_p)]),
    "tvr_model_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "tvr_trace_create": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                                        ctypes.POINTER(ctypes.c_void_p)]),
    "tvr_trace_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "tvr_trace_flush": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "tvr_trace_read": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, c_f32p,
                                      ctypes.c_void_p]),
    "tvr_trace_num_tokens": (ctypes.c_int32, [ctypes.c_void_p]),
    "tvr_forward_clean": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, c_i32p, c_i32p, ctypes.c_int32,
                                         c_i32p, c_f32p, c_i32p, ctypes.c_int32, c_f32p, c_f32p,
                                         ctypes.c_void_p]),
    "tvr_forward_clean_deferred": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, c_i32p, c_i32p, ctypes.c_int32,
                                                  c_i32p, c_f32p, c_i32p, ctypes.c_int32, ctypes.c_void_p]),
    "tvr_forward_logits": (ctypes.c_int, [ctypes.c_void_p, c_i32p, c_f32p, ctypes.c_int32, c_i32p, ctypes.c_int32,
                                          c_f32p, ctypes.c_void_p]),
    "tvr_patch_sweep": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32,
                                       c_f32p, ctypes.c_int32, c_f32p, c_i32p, ctypes.c_int32, c_f32p,
                                       ctypes.c_void_p]),
    "tvr_project_heads": (ctypes.c_int, [ctypes.c_void_p, c_f32p, c_f32p, ctypes.c_void_p]),
    "tvr_gemm_f32": (ctypes.c_int, [c_f32p, ctypes.c_int32, c_f32p, ctypes.c_int32, c_f32p, c_f32p,
                                    ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                    ctypes.c_void_p]),
    "tvr_lnpre_f32": (ctypes.c_int, [c_f32p, ctypes.c_int32, c_f32p, ctypes.c_int32, ctypes.c_int32,
                                     ctypes.c_int32, ctypes.c_float, ctypes.c_void_p]),
    "tvr_workspace_bytes": (ctypes.c_size_t, [ctypes.c_void_p]),
    "tvr_model_set_gemm": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]),
    "tvr_model_set_exact16": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "tvr_model_set_exact16_unembed": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "tvr_model_get_gemm": (ctypes.c_int32, [ctypes.c_void_p]),
    "tvr_split_planes": (ctypes.c_int, [c_f32p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "tvr_gemm_x3bf16": (ctypes.c_int, [c_f32p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32,
                                       ctypes.c_size_t, c_f32p, c_f32p, ctypes.c_int32, ctypes.c_int32,
                                       ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p]),
    "tvr_model_range_status": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "tvr_weight_planes": (ctypes.c_int, [ctypes.c_int32, c_f32p, ctypes.c_float, ctypes.c_void_p, ctypes.c_size_t,
                                         ctypes.c_void_p]),
    "tvr_gemm_x2f16": (ctypes.c_int, [c_f32p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32,
                                      ctypes.c_size_t, ctypes.c_float, c_f32p, c_f32p, ctypes.c_int32,
                                      ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                      ctypes.c_void_p]),
    "tvr_act_rows": (ctypes.c_int, [ctypes.c_int32, c_f32p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32,
                                    ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p]),
    "tvr_gemm_planar": (ctypes.c_int, [ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                       ctypes.c_int32, ctypes.c_size_t, ctypes.c_float, c_f32p, c_f32p,
                                       ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                       ctypes.c_void_p]),
    "tvr_profile_enable": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32]),
    "tvr_profile_read": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(CKernelStats)]),
    "tvr_profile_read_hbm": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(CHbmStats)]),
    "tvr_gemm_plan": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                     ctypes.c_void_p]),
}

OPS_PATH = LIB_PATH.parent / OPS_NAME
# the torch.library operators _tvr_ops.so registers (csrc/torch_ops.cpp)
OPS = ("forward_clean", "patch_sweep", "project_heads", "forward_logits")

_LIB = None
_OPS_LOADED = False


class EngineError(RuntimeError):
    pass


class RangeError(EngineError):
    """TVR_ERR_RANGE: an x2f16 GEMM input left the fp16 split's range (the
    results since the last check are not fp32-accurate).  The experiment
    functions retry on a path without that limit (``Model.range_fallback``)."""


def load(path: os.PathLike | str | None = None) -> ctypes.CDLL:
    """Load libtvr.so (cached).  Raises if it is missing: build it with
    ``python __graft_entry__.py`` or ``make -C task-vector-replication_amd/csrc``."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    p = Path(path) if path else LIB_PATH
    if not p.exists():
        raise EngineError(f"{p} not found: the HIP engine is not built (no CPU fallback exists); "
                          "run `make -C task-vector-replication_amd/csrc`")
    lib = ctypes.CDLL(str(p))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.tvr_abi_version() != ABI_VERSION:
        raise EngineError("libtvr ABI mismatch")
    if path is None:
        _LIB = lib
    return lib


def load_ops():
    """Register the ``torch.ops.tvr`` operators (once; after libtvr.so, which
    they link from their own directory).  Raises if the extension is missing."""
    global _OPS_LOADED
    import torch
    load()
    if not _OPS_LOADED:
        if not OPS_PATH.exists():
            raise EngineError(f"{OPS_PATH} not found: the torch operator extension is not built (no CPU fallback "
                              "exists); run `make -C task-vector-replication_amd/csrc`")
        torch.ops.load_library(str(OPS_PATH))
        _OPS_LOADED = True
    return torch.ops.tvr


def check(rc: int, what: str) -> None:
    """Status code → exception, with the reference's error types: invalid
    shapes raise ValueError (scratch2.py:172-175), the rest RuntimeError."""
    if rc == TVR_OK:
        return
    msg = (load().tvr_last_error() or b"").decode(errors="replace")
    if rc == TVR_ERR_INVALID:
        raise ValueError(f"{what}: {msg}")
    if rc == TVR_ERR_RANGE:
        raise RangeError(f"{what} failed ({rc}): {msg}")
    raise EngineError(f"{what} failed ({rc}): {msg}")


def ptr(t) -> int:
    """Device pointer of a torch tensor (None → NULL)."""
    return 0 if t is None else t.data_ptr()
