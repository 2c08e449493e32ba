"""Reference-named operators on torch device tensors.

One function per OpenCL kernel the reference enqueues on the ASW path
(stereo_matching/main.cpp:463-537), with the same argument meaning, each a
thin call into the HIP C-ABI (``include/asw.h``) on torch's current stream:

=========================  ====================================  ==========================
reference kernel           reference launch (main.cpp)           here
=========================  ====================================  ==========================
``asw_Aggr``               :463-466                               :func:`asw_Aggr`
``asw_vSupport``           :469-472, :477-480                     :func:`asw_vSupport`
``asw_hSupport``           :473-476, :481-484                     :func:`asw_hSupport`
``asw_vCostAggregation``   :494-500 (x r)                         :func:`asw_vCostAggregation`
``asw_hCostAggregation``   :503-509 (x r)                         :func:`asw_hCostAggregation`
``asw_WTA``                :517-526                               :func:`asw_WTA`
``Constistency``           :529-537                               :func:`Constistency`
=========================  ====================================  ==========================

Layouts are the MI355X ones of include/asw.h: images ``uint8 [H][W][4]``; cost
volumes ``float32 [H][W][Dp]`` (pixel-major, disparity fastest); supports
``float32 [H][W][Tp]``.  Errors raise :class:`~stereo_matchin_amd._lib.AswError`
(the reference printed the cl_int and carried on, main.cpp:27-30).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import DIR_H, DIR_V, AswParams


def _ptr(t: torch.Tensor | None):
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError("ASW operators take device tensors (the HIP path has no CPU fallback)")
    if not t.is_contiguous():
        raise ValueError("ASW operators take contiguous tensors")
    return ctypes.c_void_p(t.data_ptr())


def _stream(device: torch.device | None = None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _expect(t: torch.Tensor, shape, dtype, name: str):
    if tuple(t.shape) != tuple(shape) or t.dtype != dtype:
        raise ValueError(f"{name}: expected {dtype} {tuple(shape)}, got {t.dtype} {tuple(t.shape)}")


def cost_shape(p: AswParams):
    return (p.height, p.width, _lib.disp_pitch(p))


def support_shape(p: AswParams):
    return (p.height, p.width, _lib.tap_pitch(p))


def lut_shape(p: AswParams):
    return (p.taps // 2 + 1, 766)


def new_cost(p: AswParams, device) -> torch.Tensor:
    return torch.empty(cost_shape(p), dtype=torch.float32, device=device)


def new_support(p: AswParams, device) -> torch.Tensor:
    return torch.empty(support_shape(p), dtype=torch.float32, device=device)


# --------------------------------------------------------------------------- stages

def asw_Aggr(p: AswParams, left: torch.Tensor, right: torch.Tensor, out: torch.Tensor | None = None):
    """Raw per-disparity cost (K/asw_aggr.cl:3-23) for planes [d_begin, d_end)."""
    _expect(left, (p.height, p.width, 4), torch.uint8, "left")
    _expect(right, (p.height, p.width, 4), torch.uint8, "right")
    if out is None:
        out = new_cost(p, left.device)
    _expect(out, cost_shape(p), torch.float32, "out")
    _lib.check(_lib.lib().asw_raw_cost(ctypes.byref(p), _ptr(left), _ptr(right), _ptr(out), _stream(left.device)),
               "asw_raw_cost")
    return out


def raw16_supported(p: AswParams) -> bool:
    """asw_raw16_supported: the uint16 raw-cost volume (asw_raw_cost16) and the first V
    pass over it (asw_aggregate_pass_den16) are built for p."""
    return bool(_lib.lib().asw_raw16_supported(ctypes.byref(p)))


def cost16_view(cost: torch.Tensor) -> torch.Tensor:
    """The first half of a float cost volume's bytes as the [H][W][Dp] uint16 raw-cost
    volume (int16 storage) that asw_Aggr16 writes and the first V pass reads."""
    H, W, Dp = cost.shape
    return cost.view(-1).view(torch.int16)[:H * W * Dp].view(H, W, Dp)


def asw_Aggr16(p: AswParams, left: torch.Tensor, right: torch.Tensor, out: torch.Tensor | None = None):
    """The raw costs of asw_Aggr (K/asw_aggr.cl:3-23) as uint16 (asw_raw_cost16: integers
    <= 765), in int16 storage [H][W][Dp]: half the bytes of the float volume."""
    _expect(left, (p.height, p.width, 4), torch.uint8, "left")
    _expect(right, (p.height, p.width, 4), torch.uint8, "right")
    if out is None:
        out = torch.empty(cost_shape(p), dtype=torch.int16, device=left.device)
    _expect(out, cost_shape(p), torch.int16, "out")
    _lib.check(_lib.lib().asw_raw_cost16(ctypes.byref(p), _ptr(left), _ptr(right), _ptr(out), _stream(left.device)),
               "asw_raw_cost16")
    return out


def asw_vCostAggregation16(p: AswParams, supp_left, supp_right, cost16, out=None, den=None, den_mode: int = 0):
    """The first vertical pass (K/asw_vcost_aggregation.cl:11-44) over the uint16 raw
    costs of asw_Aggr16 (asw_aggregate_pass_den16; den_mode NONE or WRITE): the same
    result as asw_vCostAggregation over asw_Aggr's float volume."""
    _expect(supp_left, support_shape(p), torch.float32, "supp_left")
    _expect(supp_right, support_shape(p), torch.float32, "supp_right")
    _expect(cost16, cost_shape(p), torch.int16, "cost16")
    if out is None:
        out = new_cost(p, cost16.device)
    _expect(out, cost_shape(p), torch.float32, "out")
    if den is not None:
        _expect(den, cost_shape(p), torch.float32, "den")
    _lib.check(_lib.lib().asw_aggregate_pass_den16(ctypes.byref(p), _ptr(supp_left), _ptr(supp_right), _ptr(cost16),
                                                   _ptr(out), _ptr(den), den_mode, _stream(cost16.device)),
               "asw_aggregate_pass_den16")
    return out


def support_lut(p: AswParams, device, out: torch.Tensor | None = None) -> torch.Tensor:
    """(R+1) x 766 table of exp(-sad/gamma_c - dist/gamma_g) (K/asw_vsupport.cl:22-25)."""
    if out is None:
        out = torch.empty(lut_shape(p), dtype=torch.float32, device=device)
    _expect(out, lut_shape(p), torch.float32, "lut")
    _lib.check(_lib.lib().asw_support_lut(ctypes.byref(p), _ptr(out), _stream(out.device)), "asw_support_lut")
    return out


def _support(p: AswParams, direction: int, img: torch.Tensor, lut: torch.Tensor | None, out):
    _expect(img, (p.height, p.width, 4), torch.uint8, "image")
    if lut is None:
        lut = support_lut(p, img.device)
    if out is None:
        out = new_support(p, img.device)
    _expect(out, support_shape(p), torch.float32, "out")
    _lib.check(_lib.lib().asw_support(ctypes.byref(p), direction, _ptr(img), _ptr(lut), _ptr(out),
                                      _stream(img.device)), "asw_support")
    return out


def support_all(p: AswParams, left: torch.Tensor, right: torch.Tensor, lut: torch.Tensor, wvl: torch.Tensor,
                whl: torch.Tensor, wvr: torch.Tensor, whr: torch.Tensor) -> None:
    """asw_vSupport + asw_hSupport of both images in one launch (``asw_support_all``)."""
    for img in (left, right):
        _expect(img, (p.height, p.width, 4), torch.uint8, "image")
    for w in (wvl, whl, wvr, whr):
        _expect(w, support_shape(p), torch.float32, "out")
    _lib.check(_lib.lib().asw_support_all(ctypes.byref(p), _ptr(left), _ptr(right), _ptr(lut), _ptr(wvl), _ptr(whl),
                                          _ptr(wvr), _ptr(whr), _stream(left.device)), "asw_support_all")


def lab_image(p: AswParams, img: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """CIELab (D65) of an RGBA8 image, float32 [H][W][4] = (L*, a*, b*, 0) (north-star extension)."""
    _expect(img, (p.height, p.width, 4), torch.uint8, "image")
    if out is None:
        out = torch.empty((p.height, p.width, 4), dtype=torch.float32, device=img.device)
    _expect(out, (p.height, p.width, 4), torch.float32, "out")
    _lib.check(_lib.lib().asw_lab(ctypes.byref(p), _ptr(img), _ptr(out), _stream(img.device)), "asw_lab")
    return out


def support_lab(p: AswParams, direction: int, lab: torch.Tensor, out=None) -> torch.Tensor:
    """Support weights of a CIELab context (Euclidean L*a*b* colour term)."""
    _expect(lab, (p.height, p.width, 4), torch.float32, "lab")
    if out is None:
        out = new_support(p, lab.device)
    _expect(out, support_shape(p), torch.float32, "out")
    _lib.check(_lib.lib().asw_support_lab(ctypes.byref(p), direction, _ptr(lab), _ptr(out), _stream(lab.device)),
               "asw_support_lab")
    return out


def asw_vSupport(p: AswParams, img: torch.Tensor, lut: torch.Tensor | None = None, out=None):
    """Vertical support weights (K/asw_vsupport.cl:3-27)."""
    return _support(p, DIR_V, img, lut, out)


def asw_hSupport(p: AswParams, img: torch.Tensor, lut: torch.Tensor | None = None, out=None):
    """Horizontal support weights (K/asw_hsupport.cl:3-28)."""
    return _support(p, DIR_H, img, lut, out)


def _pass(p: AswParams, direction: int, supp_left, supp_right, cost_in, out, den=None, den_mode: int = 0):
    _expect(supp_left, support_shape(p), torch.float32, "supp_left")
    _expect(supp_right, support_shape(p), torch.float32, "supp_right")
    _expect(cost_in, cost_shape(p), torch.float32, "cost_in")
    if out is None:
        out = torch.empty_like(cost_in)
    _expect(out, cost_shape(p), torch.float32, "out")
    if out.data_ptr() == cost_in.data_ptr():
        raise ValueError("aggregation passes are out of place (cost_in != out)")
    if den_mode:
        _expect(den, cost_shape(p), torch.float32, "den")
    _lib.check(_lib.lib().asw_aggregate_pass_den(ctypes.byref(p), direction, _ptr(supp_left), _ptr(supp_right),
                                                 _ptr(cost_in), _ptr(out), _ptr(den), den_mode,
                                                 _stream(cost_in.device)),
               "asw_aggregate_pass_den")
    return out


def pass_kernel(direction: int, den_mode: int) -> str | None:
    """Name of the kernel instantiation the latest aggregation-pass launch of
    (direction, den_mode) in this process ran (asw_pass_kernel), or None."""
    import ctypes
    buf = ctypes.create_string_buffer(128)
    if _lib.lib().asw_pass_kernel(direction, den_mode, buf, len(buf)) != 0:
        return None
    return buf.value.decode()


def asw_vCostAggregation(p: AswParams, supp_left, supp_right, cost_in, out=None, den=None, den_mode: int = 0):
    """One vertical weighted-aggregation pass (K/asw_vcost_aggregation.cl:11-44).

    ``den``/``den_mode`` (DEN_WRITE / DEN_READ): the cached-denominator volume, the
    live form of the reference's write-only ``denom`` argument (``:38``)."""
    return _pass(p, DIR_V, supp_left, supp_right, cost_in, out, den, den_mode)


def asw_hCostAggregation(p: AswParams, supp_left, supp_right, cost_in, out=None, den=None, den_mode: int = 0):
    """One horizontal weighted-aggregation pass (K/asw_hcost_aggregation.cl:12-44)."""
    return _pass(p, DIR_H, supp_left, supp_right, cost_in, out, den, den_mode)


def wta_from_local(p: AswParams, cost, key, m1, m2):
    """asw_WTA's outputs on a whole-range volume from its local scan (key, m1, m2): the
    one-shard case of the d-sharded protocol, the target scan and the finalize (one
    shard's second minima are its own)."""
    tkey, t1, t2 = wta_target_local(p, cost, key)
    return wta_finalize(p, key, m2, tkey, t2)


def asw_WTA(p: AswParams, cost: torch.Tensor):
    """Winner-take-all + target map (K/asw_wta.cl:12-82).

    Returns ``(d_ref, conf_ref, d_tar, conf_tar, code_ref, code_tar)``: int32 index
    maps, float32 confidences and the u8 codes the reference writes into its
    ``asw_left_wta`` / ``asw_right_wta`` images.
    """
    _expect(cost, cost_shape(p), torch.float32, "cost")
    H, W = p.height, p.width
    dev = cost.device
    d_ref = torch.empty((H, W), dtype=torch.int32, device=dev)
    d_tar = torch.empty_like(d_ref)
    conf_ref = torch.empty((H, W), dtype=torch.float32, device=dev)
    conf_tar = torch.empty_like(conf_ref)
    code_ref = torch.empty((H, W), dtype=torch.uint8, device=dev)
    code_tar = torch.empty_like(code_ref)
    _lib.check(_lib.lib().asw_wta(ctypes.byref(p), _ptr(cost), _ptr(d_ref), _ptr(conf_ref), _ptr(d_tar),
                                  _ptr(conf_tar), _ptr(code_ref), _ptr(code_tar), _stream(dev)), "asw_wta")
    return d_ref, conf_ref, d_tar, conf_tar, code_ref, code_tar


def Constistency(p: AswParams, d_ref, d_tar, code_ref, code_tar, conf_ref, conf_tar, want_rgba: bool = True):
    """Left-right consistency (K/consist.cl:3-34).  Zeroes confidences in place.

    Returns ``(output_rgba, output_red_rgba)`` — ``consistency_error`` and
    ``consistency_error_red`` (the latter is asw_consistency_pre-reff.png).
    """
    H, W = p.height, p.width
    dev = d_ref.device
    out = torch.empty((H, W, 4), dtype=torch.uint8, device=dev) if want_rgba else None
    red = torch.empty((H, W, 4), dtype=torch.uint8, device=dev) if want_rgba else None
    _lib.check(_lib.lib().asw_consistency(ctypes.byref(p), _ptr(d_ref), _ptr(d_tar), _ptr(code_ref),
                                          _ptr(code_tar), _ptr(conf_ref), _ptr(conf_tar), _ptr(out), _ptr(red),
                                          _stream(dev)), "asw_consistency")
    return out, red


# ----------------------------------------------------------- sharded WTA primitives

def wta_local(p: AswParams, cost):
    H, W = p.height, p.width
    dev = cost.device
    key = torch.empty((H, W), dtype=torch.int64, device=dev)
    m1 = torch.empty((H, W), dtype=torch.float32, device=dev)
    m2 = torch.empty_like(m1)
    _lib.check(_lib.lib().asw_wta_local(ctypes.byref(p), _ptr(cost), _ptr(key), _ptr(m1), _ptr(m2), _stream(dev)),
               "asw_wta_local")
    return key, m1, m2


def wta_target_local(p: AswParams, cost, key_ref):
    H, W = p.height, p.width
    dev = cost.device
    tkey = torch.empty((H, W), dtype=torch.int64, device=dev)
    t1 = torch.empty((H, W), dtype=torch.float32, device=dev)
    t2 = torch.empty_like(t1)
    _lib.check(_lib.lib().asw_wta_target_local(ctypes.byref(p), _ptr(cost), _ptr(key_ref), _ptr(tkey), _ptr(t1),
                                               _ptr(t2), _stream(dev)), "asw_wta_target_local")
    return tkey, t1, t2


def wta_second(p: AswParams, key_global, key_local, m1, m2):
    out = torch.empty_like(m1)
    _lib.check(_lib.lib().asw_wta_second(ctypes.byref(p), _ptr(key_global), _ptr(key_local), _ptr(m1), _ptr(m2),
                                         _ptr(out), _stream(m1.device)), "asw_wta_second")
    return out


def wta_finalize(p: AswParams, key, m2, tkey, t2):
    H, W = p.height, p.width
    dev = key.device
    d_ref = torch.empty((H, W), dtype=torch.int32, device=dev)
    d_tar = torch.empty_like(d_ref)
    conf_ref = torch.empty((H, W), dtype=torch.float32, device=dev)
    conf_tar = torch.empty_like(conf_ref)
    code_ref = torch.empty((H, W), dtype=torch.uint8, device=dev)
    code_tar = torch.empty_like(code_ref)
    _lib.check(_lib.lib().asw_wta_finalize(ctypes.byref(p), _ptr(key), _ptr(m2), _ptr(tkey), _ptr(t2), _ptr(d_ref),
                                           _ptr(conf_ref), _ptr(d_tar), _ptr(conf_tar), _ptr(code_ref),
                                           _ptr(code_tar), _stream(dev)), "asw_wta_finalize")
    return d_ref, conf_ref, d_tar, conf_tar, code_ref, code_tar


# --------------------------------------------------------------------------- refinement
# main.cpp:540-623: k x (asw_ref_v, asw_ref_h on both views, asw_WTA_REF,
# Constistency), then Median.  Estimates are [2][H][W] f32 (value plane, den plane).

def refine_lut(p: AswParams, rp, device) -> torch.Tensor:
    """Weight table of asw_ref_v / asw_ref_h (refinement falloffs 10.94 / 118.78)."""
    lut = torch.empty((rp.taps // 2 + 1, 766), dtype=torch.float32, device=device)
    _lib.check(_lib.lib().asw_refine_lut(ctypes.byref(p), ctypes.byref(rp), _ptr(lut), _stream(device)),
               "asw_refine_lut")
    return lut


def asw_ref_v(p: AswParams, rp, img: torch.Tensor, est: torch.Tensor, conf: torch.Tensor, lut: torch.Tensor,
              out: torch.Tensor | None = None):
    """Vertical refinement (K/asw_refinement_v.cl:13-51).  ``est``: u8 codes [H][W]
    or an RGBA8 image [H][W][4] (channel 0 is read, like read_imagef(...).x)."""
    H, W = p.height, p.width
    stride = 4 if est.dim() == 3 else 1
    _expect(est, (H, W, 4) if stride == 4 else (H, W), torch.uint8, "est")
    _expect(conf, (H, W), torch.float32, "conf")
    if out is None:
        out = torch.empty((2, H, W), dtype=torch.float32, device=img.device)
    _expect(out, (2, H, W), torch.float32, "out")
    _lib.check(_lib.lib().asw_ref_v(ctypes.byref(p), ctypes.byref(rp), _ptr(img), _ptr(est), stride, _ptr(conf),
                                    _ptr(lut), _ptr(out), _stream(img.device)), "asw_ref_v")
    return out


def asw_ref_h(p: AswParams, rp, img: torch.Tensor, conf: torch.Tensor, est_v: torch.Tensor, lut: torch.Tensor,
              out: torch.Tensor | None = None):
    """Horizontal refinement (K/asw_refinement_h.cl:16-53) of asw_ref_v's output."""
    H, W = p.height, p.width
    _expect(est_v, (2, H, W), torch.float32, "est_v")
    if out is None:
        out = torch.empty_like(est_v)
    _lib.check(_lib.lib().asw_ref_h(ctypes.byref(p), ctypes.byref(rp), _ptr(img), _ptr(conf), _ptr(est_v),
                                    _ptr(lut), _ptr(out), _stream(img.device)), "asw_ref_h")
    return out


def asw_WTA_REF(p: AswParams, cost: torch.Tensor, ref_l: torch.Tensor, ref_r: torch.Tensor, conf_ref: torch.Tensor):
    """Penalised WTA (K/asw_wta_ref.cl:2-68).  Writes the TARGET confidence into
    ``conf_ref`` (the reference's second store to ``confidence``); returns
    ``(d_ref, d_tar, code_ref, code_tar)``."""
    _expect(cost, cost_shape(p), torch.float32, "cost")
    H, W = p.height, p.width
    dev = cost.device
    d_ref = torch.empty((H, W), dtype=torch.int32, device=dev)
    d_tar = torch.empty_like(d_ref)
    code_ref = torch.empty((H, W), dtype=torch.uint8, device=dev)
    code_tar = torch.empty_like(code_ref)
    _lib.check(_lib.lib().asw_wta_ref(ctypes.byref(p), _ptr(cost), _ptr(ref_l), _ptr(ref_r), _ptr(d_ref),
                                      _ptr(d_tar), _ptr(conf_ref), _ptr(code_ref), _ptr(code_tar), _stream(dev)),
               "asw_wta_ref")
    return d_ref, d_tar, code_ref, code_tar


def Median(p: AswParams, codes: torch.Tensor) -> torch.Tensor:
    """3x3 median (K/median.cl:58-88) of u8 codes [H][W] or of channel 0 of RGBA8 [H][W][4]."""
    stride = 4 if codes.dim() == 3 else 1
    out = torch.empty((p.height, p.width, 4), dtype=torch.uint8, device=codes.device)
    _lib.check(_lib.lib().asw_median3(ctypes.byref(p), _ptr(codes), stride, _ptr(out), _stream(codes.device)),
               "asw_median3")
    return out


def refine(p: AswParams, rp, left, right, cost, est_left_rgba, code_tar, conf_ref, conf_tar) -> dict:
    """The whole loop (asw_refine).  est_left_rgba, code_tar, conf_ref, conf_tar are
    updated in place like the reference's buffers; returns the outputs."""
    H, W = p.height, p.width
    dev = cost.device
    ws = torch.empty(int(_lib.lib().asw_refine_workspace_bytes(ctypes.byref(p), ctypes.byref(rp))),
                     dtype=torch.uint8, device=dev)
    if ws.numel() == 0:
        _lib.check(_lib.lib().asw_refine_params_check(ctypes.byref(p), ctypes.byref(rp)), "asw_refine_params_check")
    post = torch.zeros((H, W, 4), dtype=torch.uint8, device=dev)
    final = torch.empty((H, W, 4), dtype=torch.uint8, device=dev)
    d_ref = torch.empty((H, W), dtype=torch.int32, device=dev)
    d_tar = torch.empty_like(d_ref)
    _lib.check(_lib.lib().asw_refine(ctypes.byref(p), ctypes.byref(rp), _ptr(left), _ptr(right), _ptr(cost),
                                     _ptr(est_left_rgba), _ptr(code_tar), _ptr(conf_ref), _ptr(conf_tar), _ptr(ws),
                                     _ptr(post), _ptr(final), _ptr(d_ref), _ptr(d_tar), _stream(dev)), "asw_refine")
    return {"post_red_rgba": post, "final_rgba": final, "d_ref": d_ref, "d_tar": d_tar}
