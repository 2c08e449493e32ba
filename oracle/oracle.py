"""ORACLE — test infrastructure only.

ctypes/numpy front end of ``asw_oracle.c``, the CPU restatement of the
reference ASW path (stereo_matching/kernels/asw_*.cl, consist.cl, driven by
stereo_matching/main.cpp:413-537).  Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg import this module, and only as the
checker / the timed CPU baseline — never as the product path.

All volumes here are plane-major ``[plane][y][x]`` like the reference.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))

# fp policy ids (asw_oracle.c): the product uses FMA_NUM (DESIGN.md §FP policy)
FMA_NONE, FMA_NUM, FMA_ALL = 0, 1, 2

# reference constants (K/asw_vsupport.cl:22,24; main.cpp:177)
GAMMA_C = 30.91
GAMMA_G = 28.21

_lib = None


def _host_has_v3() -> bool:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("flags"):
                    fl = set(line.split())
                    return {"avx2", "fma", "bmi2"} <= fl
    except OSError:
        pass
    return False


def build(force: bool = False) -> None:
    """Compile the oracle shared objects with the committed Makefile."""
    need = force or not (os.path.exists(os.path.join(_HERE, "liboracle.so"))
                         and os.path.exists(os.path.join(_HERE, "liboracle_v3.so")))
    if need:
        subprocess.check_call(["make", "-s", "-C", _HERE, "all"])


# refinement contraction policy (asw_oracle.c, oracle_refine): chosen against the
# reference's device PNGs by tests/test_oracle_golden.py::test_refinement_policy
REF_POL = 0


def lib():
    global _lib
    if _lib is not None:
        return _lib
    build()
    name = "liboracle_v3.so" if _host_has_v3() else "liboracle.so"
    L = ctypes.CDLL(os.path.join(_HERE, name))
    P = ctypes.c_void_p
    i, f = ctypes.c_int, ctypes.c_float
    L.oracle_version.restype = i
    L.oracle_set_threads.argtypes = [i]
    L.oracle_set_threads.restype = i
    L.oracle_raw_cost.argtypes = [P, P, i, i, i, P]
    L.oracle_support_weight.argtypes = [i, i, f, f]
    L.oracle_support_weight.restype = f
    L.oracle_support.argtypes = [P, i, i, i, i, f, f, P]
    L.oracle_pass.argtypes = [P, P, P, P, i, i, i, i, i, i, i, i]
    L.oracle_wta.argtypes = [P, i, i, i, P, P, P, P]
    L.oracle_code_u8.argtypes = [i, i]
    L.oracle_code_u8.restype = i
    L.oracle_consistency.argtypes = [P, P, P, P, i, i, i, P, P]
    L.oracle_match.argtypes = [P, P, i, i, i, i, i, f, f, i, P, P, P, P, P, P, P]
    L.oracle_match.restype = i
    L.oracle_match_ex.argtypes = [P, P, i, i, i, i, i, f, f, i, i, f, P, P, P, P, P, P, P]
    L.oracle_match_ex.restype = i
    L.oracle_raw_cost_tad.argtypes = [P, P, i, i, i, f, P]
    L.oracle_lab.argtypes = [P, i, i, P]
    L.oracle_refine.argtypes = [P, P, i, i, i, i, i, i, P, P, P, P, P, P, P, P, P]
    L.oracle_refine.restype = i
    L.oracle_support_lab.argtypes = [P, i, i, i, i, f, f, P]
    _lib = L
    return L


def _p(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.c_void_p)


def set_threads(n: int) -> int:
    return lib().oracle_set_threads(int(n))


def raw_cost(L: np.ndarray, R: np.ndarray, D: int) -> np.ndarray:
    H, W = L.shape[:2]
    out = np.empty((D, H, W), np.float32)
    lib().oracle_raw_cost(_p(L), _p(R), W, H, D, _p(out))
    return out


def support_weight(sad: int, dist: int, gc: float = GAMMA_C, gg: float = GAMMA_G) -> float:
    return lib().oracle_support_weight(int(sad), int(dist), gc, gg)


def support(img: np.ndarray, T: int, direction: int, gc: float = GAMMA_C, gg: float = GAMMA_G) -> np.ndarray:
    H, W = img.shape[:2]
    out = np.empty((T, H, W), np.float32)
    lib().oracle_support(_p(img), W, H, T, direction, gc, gg, _p(out))
    return out


def raw_cost_tad(L: np.ndarray, R: np.ndarray, D: int, tau: float) -> np.ndarray:
    H, W = L.shape[:2]
    C = np.empty((D, H, W), np.float32)
    lib().oracle_raw_cost_tad(_p(L), _p(R), W, H, D, tau, _p(C))
    return C


def lab(img: np.ndarray) -> np.ndarray:
    """CIELab (D65) of an RGBA8 image: float32 [H][W][4] = (L*, a*, b*, 0)."""
    img = np.ascontiguousarray(img, np.uint8)
    H, W = img.shape[:2]
    out = np.empty((H, W, 4), np.float32)
    lib().oracle_lab(_p(img), W, H, _p(out))
    return out


def support_lab(lab_img: np.ndarray, T: int, direction: int, gc: float = GAMMA_C, gg: float = GAMMA_G):
    H, W = lab_img.shape[:2]
    out = np.empty((T, H, W), np.float32)
    lib().oracle_support_lab(_p(np.ascontiguousarray(lab_img, np.float32)), W, H, T, direction, gc, gg, _p(out))
    return out


def aggregate_pass(sL, sR, cin, T: int, direction: int, d0: int = 0, d1: int | None = None,
                   plane_base: int = 0, fma_mode: int = FMA_NUM) -> np.ndarray:
    n, H, W = cin.shape
    if d1 is None:
        d1 = plane_base + n
    out = np.zeros_like(cin)
    lib().oracle_pass(_p(sL), _p(sR), _p(cin), _p(out), W, H, T, direction, d0, d1, plane_base, fma_mode)
    return out


def wta(C: np.ndarray):
    D, H, W = C.shape
    dr = np.empty((H, W), np.int32)
    dt = np.empty((H, W), np.int32)
    cr = np.empty((H, W), np.float32)
    ct = np.empty((H, W), np.float32)
    lib().oracle_wta(_p(C), W, H, D, _p(dr), _p(cr), _p(dt), _p(ct))
    return dr, cr, dt, ct


def code_u8(d, D: int):
    d = np.asarray(d, np.int64)
    if D <= 1:
        return np.zeros(d.shape, np.uint8)
    return np.clip((510 * d + (D - 2)) // (2 * (D - 1)), 0, 255).astype(np.uint8)


def consistency(code_ref, code_tar, conf_ref, conf_tar, D: int):
    H, W = code_ref.shape
    conf_ref = np.ascontiguousarray(conf_ref, np.float32).copy()
    conf_tar = np.ascontiguousarray(conf_tar, np.float32).copy()
    o = np.empty((H, W, 4), np.uint8)
    r = np.empty((H, W, 4), np.uint8)
    lib().oracle_consistency(_p(np.ascontiguousarray(code_ref, np.uint8)),
                             _p(np.ascontiguousarray(code_tar, np.uint8)),
                             _p(conf_ref), _p(conf_tar), W, H, D, _p(o), _p(r))
    return o, r, conf_ref, conf_tar


def match(L: np.ndarray, R: np.ndarray, D: int, T: int, iters: int = 7, gc: float = GAMMA_C,
          gg: float = GAMMA_G, fma_mode: int = FMA_NUM, want_cost: bool = False, color_space: int = 0,
          tad_tau: float = 765.0, refine_iters: int = 0, refine_taps: int = 33, ref_pol: int = REF_POL) -> dict:
    """Full reference ASW pipeline (main.cpp:463-537) on host RGBA8 images [H][W][4]."""
    L = np.ascontiguousarray(L, np.uint8)
    R = np.ascontiguousarray(R, np.uint8)
    H, W = L.shape[:2]
    out = {
        "d_ref": np.empty((H, W), np.int32), "conf_ref": np.empty((H, W), np.float32),
        "d_tar": np.empty((H, W), np.int32), "conf_tar": np.empty((H, W), np.float32),
        "lr_rgba": np.empty((H, W, 4), np.uint8), "lr_red_rgba": np.empty((H, W, 4), np.uint8),
    }
    cost = np.empty((D, H, W), np.float32) if want_cost else None
    if refine_iters and cost is None:
        cost = np.empty((D, H, W), np.float32)
    rc = lib().oracle_match_ex(_p(L), _p(R), W, H, D, T, iters, gc, gg, fma_mode, color_space, tad_tau,
                            _p(out["d_ref"]), _p(out["conf_ref"]), _p(out["d_tar"]), _p(out["conf_tar"]),
                            _p(out["lr_rgba"]), _p(out["lr_red_rgba"]),
                            _p(cost) if cost is not None else None)
    if rc != 0:
        raise MemoryError("oracle_match failed to allocate")
    if refine_iters:
        out.update(refine(L, R, D, cost, out, refine_iters, refine_taps, ref_pol))
    if want_cost:
        out["cost"] = cost
    return out


def refine(L, R, D: int, cost, pre: dict, k: int, taps: int = 33, pol: int = REF_POL) -> dict:
    """Refinement loop + 3x3 median (main.cpp:540-623) after a match() result `pre`."""
    H, W = L.shape[:2]
    conf_ref = np.ascontiguousarray(pre["conf_ref"], np.float32).copy()
    conf_tar = np.ascontiguousarray(pre["conf_tar"], np.float32).copy()
    est_left = np.ascontiguousarray(pre["lr_rgba"][..., 0])
    est_right = code_u8(pre["d_tar"], D)
    res = {"post_red_rgba": np.empty((H, W, 4), np.uint8), "final_rgba": np.empty((H, W, 4), np.uint8),
           "ref_d_ref": np.empty((H, W), np.int32), "ref_d_tar": np.empty((H, W), np.int32)}
    rc = lib().oracle_refine(_p(L), _p(R), W, H, D, k, taps, pol, _p(cost), _p(est_left), _p(est_right),
                             _p(conf_ref), _p(conf_tar), _p(res["post_red_rgba"]), _p(res["final_rgba"]),
                             _p(res["ref_d_ref"]), _p(res["ref_d_tar"]))
    if rc != 0:
        raise MemoryError("oracle_refine failed to allocate")
    res["ref_conf_ref"], res["ref_conf_tar"] = conf_ref, conf_tar
    return res
