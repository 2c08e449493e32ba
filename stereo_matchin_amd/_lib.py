"""ctypes binding of the C-ABI in ``include/asw.h`` (``libasw_hip.so``).

The library is the product: hand-written gfx950 HIP kernels.  There is no CPU
fallback — if the shared object is missing or does not load, every entry point
raises :class:`AswLibraryError`.

``torch`` is imported before the library is opened so that the HIP runtime
already mapped by torch (``libamdhip64.so.7``) is the one the kernels link
against; device pointers and ``hipStream_t`` handles from torch are then valid
arguments.
"""
from __future__ import annotations

import ctypes
import os
import re

import torch  # noqa: F401  (must precede loading libasw_hip.so, see module doc)

_HERE = os.path.dirname(os.path.abspath(__file__))
# ASW_LIB overrides the library path (kernel experiments: tools/ builds variants
# of the same sources into another file); the default is the in-tree build.
LIB_PATH = os.environ.get("ASW_LIB") or os.path.join(_HERE, "libasw_hip.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "asw.h")

ASW_OK = 0
ASW_E_INVALID = -1
ASW_E_HIP = -2
ASW_E_NOMEM = -3
ASW_E_UNSUPPORTED = -4
ASW_E_COMM = -5
DISP16_INVALID = 0xFFFF
COMM_ID_BYTES = 128
# the asw_outputs / asw_timings layouts mirrored below (ASW_ABI_VERSION of include/asw.h):
# a library of another revision would write past them, so _load() refuses it
ABI_VERSION = 4

DIR_V = 0
DIR_H = 1
DEN_NONE, DEN_WRITE, DEN_READ = 0, 1, 2  # ASW_DEN_* (cached aggregation denominator)
COLOR_RGB = 0
COLOR_LAB = 1
LR_U8 = 0
LR_NATIVE = 1
# asw_params.flags (ASW_FLAG_*): frame-API context options (ABI 4)
FLAG_COMM_LOCAL = 0x20
FLAG_RAW_F32 = 0x40


class AswLibraryError(RuntimeError):
    """The HIP library is missing or failed to load (no fallback exists)."""


class AswError(RuntimeError):
    def __init__(self, status: int, where: str):
        self.status = status
        msg = f"{where}: {strerror(status)} ({status})"
        if status == ASW_E_HIP:
            msg += f", hipError={_lib_or_raise().asw_last_hip_error()}"
        super().__init__(msg)


class AswParams(ctypes.Structure):
    """Mirror of ``asw_params`` (include/asw.h)."""

    _fields_ = [
        ("width", ctypes.c_int), ("height", ctypes.c_int),
        ("ndisp", ctypes.c_int), ("taps", ctypes.c_int), ("iters", ctypes.c_int),
        ("gamma_c", ctypes.c_float), ("gamma_g", ctypes.c_float),
        ("color_space", ctypes.c_int), ("tad_tau", ctypes.c_float),
        ("lr_check", ctypes.c_int), ("lr_mode", ctypes.c_int),
        ("d_begin", ctypes.c_int), ("d_end", ctypes.c_int),
        ("flags", ctypes.c_int),
    ]

    def copy(self) -> "AswParams":
        p = AswParams()
        ctypes.pointer(p)[0] = self
        return p

    def as_dict(self) -> dict:
        return {f: getattr(self, f) for f, _ in self._fields_}

    @property
    def d_stop(self) -> int:
        return self.ndisp if self.d_end < 0 else self.d_end


class AswOutputs(ctypes.Structure):
    _fields_ = [
        ("d_ref", ctypes.c_void_p), ("d_tar", ctypes.c_void_p),
        ("conf_ref", ctypes.c_void_p), ("conf_tar", ctypes.c_void_p),
        ("disp_rgba", ctypes.c_void_p), ("lr_rgba", ctypes.c_void_p),
        ("lr_red_rgba", ctypes.c_void_p), ("cost", ctypes.c_void_p),
        ("final_rgba", ctypes.c_void_p), ("post_red_rgba", ctypes.c_void_p),
        ("disp16", ctypes.c_void_p), ("lr16", ctypes.c_void_p),
    ]


class AswRefineParams(ctypes.Structure):
    """Mirror of ``asw_refine_params`` (include/asw.h)."""

    _fields_ = [("iters", ctypes.c_int), ("taps", ctypes.c_int), ("gamma_c", ctypes.c_float),
                ("gamma_g", ctypes.c_float), ("alpha", ctypes.c_float)]


class AswTimings(ctypes.Structure):
    _fields_ = [(n, ctypes.c_double) for n in (
        "raw_cost", "support", "v_pass_mean", "h_pass_mean", "aggregation_total", "wta",
        "consistency", "total", "h2d", "d2h", "refine", "exchange")]


_lib = None
_load_error: Exception | None = None

P = ctypes.c_void_p
PP = ctypes.POINTER(AswParams)
RP = ctypes.POINTER(AswRefineParams)
I = ctypes.c_int

# name -> (restype, argtypes).  Every function declared in include/asw.h.
SIGNATURES = {
    "asw_params_default": (None, [PP]),
    "asw_params_check": (I, [PP]),
    "asw_strerror": (ctypes.c_char_p, [I]),
    "asw_last_hip_error": (I, []),
    "asw_abi_version": (I, []),
    "asw_disp_pitch": (I, [PP]),
    "asw_tap_pitch": (I, [PP]),
    "asw_cost_bytes": (ctypes.c_size_t, [PP]),
    "asw_support_bytes": (ctypes.c_size_t, [PP]),
    "asw_lut_bytes": (ctypes.c_size_t, [PP]),
    "asw_raw_cost": (I, [PP, P, P, P, P]),
    "asw_support_lut": (I, [PP, P, P]),
    "asw_support": (I, [PP, I, P, P, P, P]),
    "asw_support_all": (I, [PP, P, P, P, P, P, P, P, P]),
    "asw_lab_bytes": (ctypes.c_size_t, [PP]),
    "asw_lab": (I, [PP, P, P, P]),
    "asw_support_lab": (I, [PP, I, P, P, P]),
    "asw_aggregate_pass": (I, [PP, I, P, P, P, P, P]),
    "asw_aggregate_pass_den": (I, [PP, I, P, P, P, P, P, I, P]),
    "asw_raw_cost16": (I, [PP, P, P, P, P]),
    "asw_aggregate_pass_den16": (I, [PP, P, P, P, P, P, I, P]),
    "asw_raw16_supported": (I, [PP]),
    "asw_aggregate": (I, [PP, P, P, P, P, P, P, P]),
    "asw_aggregate_den": (I, [PP, P, P, P, P, P, P, P, P, P]),
    "asw_wta": (I, [PP, P, P, P, P, P, P, P, P]),
    "asw_consistency": (I, [PP, P, P, P, P, P, P, P, P, P]),
    "asw_wta_local": (I, [PP, P, P, P, P, P]),
    "asw_wta_target_local": (I, [PP, P, P, P, P, P, P]),
    "asw_wta_second": (I, [PP, P, P, P, P, P, P]),
    "asw_wta_finalize": (I, [PP, P, P, P, P, P, P, P, P, P, P, P]),
    "asw_wta_ref_local": (I, [PP, P, P, P, P, P, P]),
    "asw_wta_ref_target_local": (I, [PP, P, P, P, P, P, P, P]),
    "asw_wta_ref_finalize": (I, [PP, P, P, P, P, P, P, P, P, P]),
    "asw_refine_params_default": (None, [RP]),
    "asw_refine_params_check": (I, [PP, RP]),
    "asw_refine_lut_bytes": (ctypes.c_size_t, [RP]),
    "asw_refine_lut": (I, [PP, RP, P, P]),
    "asw_ref_v": (I, [PP, RP, P, P, I, P, P, P, P]),
    "asw_ref_h": (I, [PP, RP, P, P, P, P, P, P]),
    "asw_wta_ref": (I, [PP, P, P, P, P, P, P, P, P, P]),
    "asw_median3": (I, [PP, P, I, P, P]),
    "asw_refine_workspace_bytes": (ctypes.c_size_t, [PP, RP]),
    "asw_refine": (I, [PP, RP, P, P, P, P, P, P, P, P, P, P, P, P, P]),
    "asw_set_refine": (I, [P, RP]),
    "asw_set_graph": (I, [P, I]),
    "asw_tune_set": (I, [I, I]),
    "asw_pass_kernel": (I, [I, I, ctypes.c_char_p, I]),
    "asw_device_name": (I, [I, ctypes.c_char_p, I]),
    "asw_create": (I, [PP, I, ctypes.POINTER(P)]),
    "asw_destroy": (I, [P]),
    "asw_match": (I, [P, P, P, ctypes.POINTER(AswOutputs), ctypes.POINTER(AswTimings)]),
    "asw_create_multi": (I, [PP, ctypes.POINTER(I), I, ctypes.POINTER(P)]),
    "asw_comm_unique_id": (I, [ctypes.c_char_p]),
    "asw_create_rank": (I, [PP, I, I, I, ctypes.c_char_p, ctypes.POINTER(P)]),
    "asw_ctx_shard": (I, [P, I, ctypes.POINTER(I), ctypes.POINTER(I), ctypes.POINTER(I)]),
    "asw_match_batch": (I, [P, P, P, I, ctypes.POINTER(AswOutputs), ctypes.POINTER(AswTimings)]),
}


def header_functions(path: str = HEADER_PATH) -> list[str]:
    """Names of every function the C header declares."""
    with open(path) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(asw_[a-z0-9_]+)\s*\(", text)) - {"asw_params", "asw_ctx"})


def _load():
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        _load_error = AswLibraryError(
            f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(there is no CPU fallback)")
        raise _load_error
    try:
        L = ctypes.CDLL(LIB_PATH)
    except OSError as e:  # pragma: no cover - depends on the environment
        _load_error = AswLibraryError(f"failed to load {LIB_PATH}: {e}")
        raise _load_error from e
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    got = L.asw_abi_version()
    if got != ABI_VERSION:
        _load_error = AswLibraryError(
            f"{LIB_PATH} has ABI revision {got}, this binding mirrors revision {ABI_VERSION} "
            "(asw_outputs / asw_timings layouts differ): rebuild the library")
        raise _load_error
    _lib = L
    return L


def _lib_or_raise():
    return _load()


def lib():
    return _load()


def strerror(status: int) -> str:
    return _load().asw_strerror(status).decode()


def check(status: int, where: str) -> None:
    if status != ASW_OK:
        raise AswError(status, where)


def default_params(width: int = 0, height: int = 0, **kw) -> AswParams:
    p = AswParams()
    _load().asw_params_default(ctypes.byref(p))
    p.width, p.height = width, height
    for k, v in kw.items():
        if not hasattr(p, k):
            raise TypeError(f"unknown asw_params field {k!r}")
        setattr(p, k, v)
    return p


def default_refine_params(**kw) -> AswRefineParams:
    """Reference refinement settings (k = 6, 33 taps, 10.94 / 118.78, 0.085), overridable."""
    rp = AswRefineParams()
    _load().asw_refine_params_default(ctypes.byref(rp))
    for k, v in kw.items():
        if not hasattr(rp, k):
            raise TypeError(f"unknown asw_refine_params field {k!r}")
        setattr(rp, k, v)
    return rp


def disp_pitch(p: AswParams) -> int:
    return _load().asw_disp_pitch(ctypes.byref(p))


def tap_pitch(p: AswParams) -> int:
    return _load().asw_tap_pitch(ctypes.byref(p))


def params_check(p: AswParams) -> int:
    return _load().asw_params_check(ctypes.byref(p))
