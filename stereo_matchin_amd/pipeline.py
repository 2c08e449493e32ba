"""The ASW sequence of main.cpp:463-537 on one GPU, over the HIP C-ABI.

:class:`StereoMatcher` owns the device buffers of one image size / parameter
set (the reference re-creates every ``cl_mem`` per run, main.cpp:243-457; here
they are allocated once and reused across frames) and runs

    asw_Aggr -> 4 x support -> r x (V pass, H pass) -> asw_WTA -> Constistency

on torch's current stream.  ``match()`` takes device-resident RGBA8 images.
:func:`match_frame` is the host-pointer frame API (``asw_match``) used by the
CLI path.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from . import kernels as K
from ._lib import COLOR_LAB, DIR_H, DIR_V, AswParams


def make_params(width: int, height: int, ndisp: int = 61, taps: int = 33, iters: int = 7, **kw) -> AswParams:
    """asw_params with the reference defaults (include/asw.h) and the given overrides."""
    return _lib.default_params(width, height, ndisp=ndisp, taps=taps, iters=iters, **kw)


@dataclass
class MatchResult:
    d_ref: torch.Tensor       # int32 [H][W] left-view disparity index
    conf_ref: torch.Tensor    # float32 [H][W]
    d_tar: torch.Tensor       # int32 [H][W] right-view (target) index
    conf_tar: torch.Tensor
    code_ref: torch.Tensor    # u8 [H][W] 8-bit image codes (asw_left_wta)
    code_tar: torch.Tensor
    lr_rgba: torch.Tensor | None       # consistency_error
    lr_red_rgba: torch.Tensor | None   # consistency_error_red (asw_consistency_pre-reff.png)
    cost: torch.Tensor        # final aggregated volume [H][W][Dp]


class StereoMatcher:
    """One GPU, one disparity shard: the buffers of main.cpp:434-457, allocated once.

    ``den_cache`` (default on for r >= 2): keep the two aggregation denominators
    (V, H) as volumes — written by the first pass of each direction, read by the
    other r-1 (ASW_DEN_*); bit-identical results, 2 more cost-sized buffers."""

    def __init__(self, params: AswParams, device="cuda", den_cache: bool = True):
        st = _lib.params_check(params)
        if st != _lib.ASW_OK:
            raise _lib.AswError(st, "asw_params_check")
        self.p = params.copy()
        self.device = torch.device(device)
        dev = self.device
        self.lut = torch.empty(K.lut_shape(self.p), dtype=torch.float32, device=dev)
        self.wvl, self.wvr, self.whl, self.whr = (K.new_support(self.p, dev) for _ in range(4))
        self.c0 = K.new_cost(self.p, dev)
        self.c1 = K.new_cost(self.p, dev)
        # the raw costs as uint16 in c0's first half (asw_raw_cost16 + the first V pass
        # asw_aggregate_pass_den16: half the bytes of asw_Aggr's write and that pass's read,
        # bit-identical); ASW_FLAG_RAW_F32 keeps the float volume
        self.raw16 = not params.flags & _lib.FLAG_RAW_F32 and K.raw16_supported(self.p)
        self.c0_16 = K.cost16_view(self.c0) if self.raw16 else None
        self.den_v = self.den_h = None
        if den_cache and self.p.iters >= 2 and K.cost_shape(self.p)[2] != 32:
            # a 32-plane shard's passes recompute den (C4 / 8: k_vpass32 den-none 0.24
            # against den-read 0.28 ms, k_hpass32 0.30-0.33 against 0.36,
            # profiles/r04/h32_variants_r11d.log; asw_frame.cpp the same)
            self.den_v = K.new_cost(self.p, dev)
            self.den_h = K.new_cost(self.p, dev)
        # the WTA's local scan (key, m1, m2) of c0 when a pass already produced it (None:
        # asw_WTA / asw_wta_local scan the volume); read by match() and the d-sharded protocol
        self.local = None

    # -- stages ---------------------------------------------------------------
    def raw_and_support(self, left: torch.Tensor, right: torch.Tensor):
        """asw_Aggr into c0 and the four support arrays."""
        p = self.p
        if self.raw16:
            K.asw_Aggr16(p, left, right, out=self.c0_16)
        else:
            K.asw_Aggr(p, left, right, out=self.c0)
        if p.color_space == COLOR_LAB:
            lab_l, lab_r = K.lab_image(p, left), K.lab_image(p, right)
            K.support_lab(p, DIR_V, lab_l, out=self.wvl)
            K.support_lab(p, DIR_H, lab_l, out=self.whl)
            K.support_lab(p, DIR_V, lab_r, out=self.wvr)
            K.support_lab(p, DIR_H, lab_r, out=self.whr)
            return
        K.support_lut(p, self.device, out=self.lut)
        # asw_vSupport / asw_hSupport of both images (main.cpp:469-484) in one launch
        K.support_all(p, left, right, self.lut, self.wvl, self.whl, self.wvr, self.whr)

    def aggregate(self, events: list | None = None):
        """r x (V: c0 -> c1, H: c1 -> c0); the result is in c0 (main.cpp:486-515)."""
        p = self.p
        self.local = None
        for it in range(p.iters):
            dmv = _lib.DEN_NONE if self.den_v is None else (_lib.DEN_WRITE if it == 0 else _lib.DEN_READ)
            dm = _lib.DEN_NONE if self.den_h is None else (_lib.DEN_WRITE if it == 0 else _lib.DEN_READ)
            if it == 0 and self.raw16:
                K.asw_vCostAggregation16(p, self.wvl, self.wvr, self.c0_16, out=self.c1, den=self.den_v, den_mode=dmv)
            else:
                K.asw_vCostAggregation(p, self.wvl, self.wvr, self.c0, out=self.c1, den=self.den_v, den_mode=dmv)
            if events is not None:
                events.append(("v", _record()))
            K.asw_hCostAggregation(p, self.whl, self.whr, self.c1, out=self.c0, den=self.den_h, den_mode=dm)
            if events is not None:
                events.append(("h", _record()))
        return self.c0

    def match(self, left: torch.Tensor, right: torch.Tensor, lr_check: bool | None = None,
              events: list | None = None) -> MatchResult:
        p = self.p
        if events is not None:
            events.append(("start", _record()))
        self.raw_and_support(left, right)
        if events is not None:
            events.append(("support", _record()))
        cost = self.aggregate(events)
        if self.local is not None:  # the own scan ran in the last pass: the target scan and finalize
            d_ref, conf_ref, d_tar, conf_tar, code_ref, code_tar = K.wta_from_local(p, cost, *self.local)
        else:
            d_ref, conf_ref, d_tar, conf_tar, code_ref, code_tar = K.asw_WTA(p, cost)
        if events is not None:
            events.append(("wta", _record()))
        lr = red = None
        if p.lr_check if lr_check is None else lr_check:
            lr, red = K.Constistency(p, d_ref, d_tar, code_ref, code_tar, conf_ref, conf_tar)
        if events is not None:
            events.append(("consistency", _record()))
        return MatchResult(d_ref, conf_ref, d_tar, conf_tar, code_ref, code_tar, lr, red, cost)

    def refine(self, res: MatchResult, left: torch.Tensor, right: torch.Tensor, rp=None) -> dict:
        """The refinement loop + median (main.cpp:540-623) after ``match`` (needs its LR
        check).  ``res``'s lr image, target codes and confidences are refined in place
        like the reference's buffers; returns post_red_rgba (asw_consistency_post-reff),
        final_rgba (asw_disparity.png) and the last asw_WTA_REF maps."""
        if res.lr_rgba is None:
            raise ValueError("refinement starts from the consistency image: match() with lr_check")
        rp = _lib.default_refine_params() if rp is None else rp
        return K.refine(self.p, rp, left, right, res.cost, res.lr_rgba, res.code_tar, res.conf_ref, res.conf_tar)


def _record():
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    return e


def to_rgba(img: np.ndarray) -> np.ndarray:
    """RGB or RGBA u8 [H][W][C] -> contiguous RGBA8 (alpha 255), what lodepng::decode yields."""
    img = np.asarray(img, np.uint8)
    if img.ndim == 2:
        img = np.repeat(img[..., None], 3, axis=2)
    if img.shape[2] == 4:
        return np.ascontiguousarray(img)
    a = np.full(img.shape[:2] + (1,), 255, np.uint8)
    return np.ascontiguousarray(np.concatenate([img[..., :3], a], axis=2))


class FrameContext:
    """The FRAME API (``asw_create`` / ``asw_create_multi`` / ``asw_create_rank`` +
    ``asw_match`` / ``asw_match_batch``): host RGBA8 in, host maps out, buffers
    allocated once and reused pair after pair.

    ``devices``: HIP ordinals of the shards driven by this process (one = one GPU;
    several = the disparity range split across them, RCCL when distinct, a
    device-local reduction when an ordinal repeats).  ``rank``/``nranks``/``comm_id``:
    one process per GPU (``asw_create_rank``), ``comm_id`` from :func:`comm_unique_id`.
    """

    def __init__(self, params: AswParams, devices=(0,), rank: int | None = None, nranks: int | None = None,
                 comm_id: bytes | None = None, refine=None, graph: bool = False):
        self.L = _lib.lib()
        self.p = params.copy()
        self.ctx = ctypes.c_void_p()
        devices = list(devices)
        if rank is not None:
            if len(devices) != 1 or comm_id is None or nranks is None:
                raise ValueError("rank mode: one device, nranks and comm_id")
            _lib.check(self.L.asw_create_rank(ctypes.byref(self.p), devices[0], rank, nranks, comm_id,
                                              ctypes.byref(self.ctx)), "asw_create_rank")
        elif len(devices) == 1:
            _lib.check(self.L.asw_create(ctypes.byref(self.p), devices[0], ctypes.byref(self.ctx)), "asw_create")
        else:
            arr = (ctypes.c_int * len(devices))(*devices)
            _lib.check(self.L.asw_create_multi(ctypes.byref(self.p), arr, len(devices), ctypes.byref(self.ctx)),
                       "asw_create_multi")
        self.refine = refine is not None
        if refine is not None:  # an AswRefineParams: main.cpp:540-623 inside asw_match
            _lib.check(self.L.asw_set_refine(self.ctx, ctypes.byref(refine)), "asw_set_refine")
        if graph:  # asw_set_graph: capture the device work into HIP graphs, replay them
            _lib.check(self.L.asw_set_graph(self.ctx, 1), "asw_set_graph")

    def shards(self) -> list[tuple[int, int]]:
        n, b, e = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        self.L.asw_ctx_shard(self.ctx, 0, ctypes.byref(n), None, None)
        out = []
        for i in range(n.value):
            _lib.check(self.L.asw_ctx_shard(self.ctx, i, None, ctypes.byref(b), ctypes.byref(e)), "asw_ctx_shard")
            out.append((b.value, e.value))
        return out

    def _outputs(self, want_cost: bool, want16: bool):
        H, W = self.p.height, self.p.width
        out = {
            "d_ref": np.empty((H, W), np.int32), "d_tar": np.empty((H, W), np.int32),
            "conf_ref": np.empty((H, W), np.float32), "conf_tar": np.empty((H, W), np.float32),
            "disp_rgba": np.empty((H, W, 4), np.uint8), "lr_rgba": np.empty((H, W, 4), np.uint8),
            "lr_red_rgba": np.empty((H, W, 4), np.uint8),
        }
        if want_cost:
            out["cost"] = np.zeros((H, W, _lib.disp_pitch(self.p)), np.float32)
        if self.refine:
            out["final_rgba"] = np.empty((H, W, 4), np.uint8)
            out["post_red_rgba"] = np.empty((H, W, 4), np.uint8)
        if want16:
            out["disp16"] = np.empty((H, W), np.uint16)
            out["lr16"] = np.empty((H, W), np.uint16)
        o = _lib.AswOutputs(*[out[k].ctypes.data if k in out else None for k, _ in _lib.AswOutputs._fields_])
        return out, o

    def match(self, left_rgba: np.ndarray, right_rgba: np.ndarray, want_cost: bool = False,
              want16: bool = False) -> dict:
        return self.match_batch(left_rgba[None], right_rgba[None], want_cost, want16)[0]

    def match_batch(self, lefts: np.ndarray, rights: np.ndarray, want_cost: bool = False,
                    want16: bool = False) -> list[dict]:
        """``asw_match_batch``: lefts / rights are [B][H][W][4] (or RGB) stacks."""
        H, W = self.p.height, self.p.width
        lefts = np.ascontiguousarray(np.stack([to_rgba(x) for x in lefts]))
        rights = np.ascontiguousarray(np.stack([to_rgba(x) for x in rights]))
        B = lefts.shape[0]
        assert lefts.shape == (B, H, W, 4) and rights.shape == (B, H, W, 4)
        outs, os_ = zip(*[self._outputs(want_cost, want16) for _ in range(B)]) if B else ((), ())
        oarr = (_lib.AswOutputs * B)(*os_)
        tarr = (_lib.AswTimings * B)()
        _lib.check(self.L.asw_match_batch(self.ctx, lefts.ctypes.data, rights.ctypes.data, B, oarr, tarr),
                   "asw_match_batch")
        for b in range(B):
            outs[b]["timings"] = \
                {f: getattr(tarr[b], f) for f, _ in tarr[b]._fields_}
        return list(outs)

    def close(self):
        if self.ctx:
            self.L.asw_destroy(self.ctx)
            self.ctx = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass


def comm_unique_id() -> bytes:
    """``asw_comm_unique_id`` (ncclGetUniqueId) for :class:`FrameContext` rank mode."""
    buf = ctypes.create_string_buffer(_lib.COMM_ID_BYTES)
    _lib.check(_lib.lib().asw_comm_unique_id(buf), "asw_comm_unique_id")
    return buf.raw


def match_frame(params: AswParams, left_rgba: np.ndarray, right_rgba: np.ndarray, device: int = 0,
                want_cost: bool = False, refine=None, devices=None, want16: bool = False) -> dict:
    """Frame API (``asw_create`` + ``asw_match``): host RGBA8 in, host maps out."""
    with FrameContext(params, devices=devices if devices is not None else (device,), refine=refine) as fc:
        return fc.match(left_rgba, right_rgba, want_cost=want_cost, want16=want16)
