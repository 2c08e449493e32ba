"""Parity of the HIP path (through the C-ABI) with the CPU oracle — run on an MI355X.

Bit-exact for every integer output (disparity indices, 8-bit codes, LR images)
and, because the HIP kernels replay the oracle's exact fp32 operation sequence
(DESIGN.md §FP policy), bit-exact on the float cost volumes and confidences too;
the north-star tolerance for the aggregated cost, |a-b| <= 1e-4 * max(1,|b|),
is asserted alongside as the contractual bar.
"""
import ctypes

import numpy as np
import pytest

from conftest import load_scene, pixel_major, plane_major

pytestmark = pytest.mark.gpu

COST_TOL = 1e-4  # north star: "within 1e-4 on the float aggregated cost" (relative to max(1,|b|))


def _t(a, dev):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _np(t):
    return t.detach().cpu().numpy()


def _params(W, H, D, T, iters=7, **kw):
    from stereo_matchin_amd import make_params
    return make_params(W, H, ndisp=D, taps=T, iters=iters, **kw)


def assert_cost_close(got, want):
    err = np.abs(got.astype(np.float64) - want.astype(np.float64)) / np.maximum(1.0, np.abs(want))
    assert err.max() <= COST_TOL, err.max()


def _rand_pair(seed, H, W, shift=4):
    rng = np.random.default_rng(seed)
    L = rng.integers(0, 256, (H, W, 4), dtype=np.uint8)
    R = np.roll(L, -shift, axis=1).copy()
    R[..., :3] = np.clip(R[..., :3].astype(int) + rng.integers(-5, 6, (H, W, 3)), 0, 255).astype(np.uint8)
    L[..., 3] = 255
    R[..., 3] = 255
    return np.ascontiguousarray(L), np.ascontiguousarray(R)


# ------------------------------------------------------------------ stage parity

def test_support_lut_exhaustive(gpu, oracle):
    import stereo_matchin_amd.kernels as K
    for T in (3, 33, 35, 51):
        p = _params(8, 8, 16, T)
        lut = _np(K.support_lut(p, gpu))
        want = np.array([[oracle.support_weight(s, d) for s in range(766)] for d in range(T // 2 + 1)], np.float32)
        bad = np.argwhere(lut.view(np.uint32) != want.view(np.uint32))
        assert bad.size == 0, f"T={T}: {len(bad)} LUT entries differ, first {bad[:5]}"


@pytest.mark.parametrize("D,d_begin,d_end", [(61, 0, 61), (64, 0, 64), (100, 37, 100), (16, 0, 16)])
def test_raw_cost(gpu, oracle, D, d_begin, d_end):
    import stereo_matchin_amd.kernels as K
    Lh, Rh, _ = load_scene("tsukuba")
    p = _params(Lh.shape[1], Lh.shape[0], D, 33, d_begin=d_begin, d_end=d_end)
    c = _np(K.asw_Aggr(p, _t(Lh, gpu), _t(Rh, gpu)))
    want = oracle.raw_cost(Lh, Rh, D)[d_begin:d_end]
    assert np.array_equal(plane_major(c, d_end - d_begin), want)
    assert (c[:, :, d_end - d_begin:] == 0).all()


def test_raw_cost_truncated(gpu, oracle):
    import stereo_matchin_amd.kernels as K
    Lh, Rh = _rand_pair(3, 20, 30)
    p = _params(30, 20, 10, 5, tad_tau=40.0)
    c = plane_major(_np(K.asw_Aggr(p, _t(Lh, gpu), _t(Rh, gpu))), 10)
    assert np.array_equal(c, np.minimum(oracle.raw_cost(Lh, Rh, 10), np.float32(40.0)))


# the alpha byte never enters the cost (K/asw_aggr.cl sums the three colour channels):
# random alpha in both images, float and uint16 forms, a plain, a truncating and a
# non-integral tau (float form only), ragged widths and a d-shard
@pytest.mark.parametrize("W,H,D,d0,d1,tau", [(97, 13, 70, 0, 70, 765.0), (150, 9, 200, 64, 160, 90.0),
                                             (40, 7, 64, 0, 64, 30.5), (333, 5, 256, 96, 128, 765.0)])
def test_raw_cost_random_alpha(gpu, oracle, W, H, D, d0, d1, tau):
    import torch

    import stereo_matchin_amd.kernels as K
    rng = np.random.default_rng(W + H + D)
    Lh = rng.integers(0, 256, (H, W, 4), dtype=np.uint8)
    Rh = np.roll(Lh, -5, axis=1)
    Rh = np.ascontiguousarray(np.clip(Rh.astype(int) + rng.integers(-40, 41, Rh.shape), 0, 255).astype(np.uint8))
    p = _params(W, H, D, 5, d_begin=d0, d_end=d1, tad_tau=tau)
    want = np.minimum(oracle.raw_cost(Lh, Rh, D)[d0:d1], np.float32(tau))
    L, R = _t(Lh, gpu), _t(Rh, gpu)
    c = _np(K.asw_Aggr(p, L, R))
    assert np.array_equal(plane_major(c, d1 - d0), want)
    assert (c[:, :, d1 - d0:] == 0).all()
    if K.raw16_supported(p):
        c16 = K.asw_Aggr16(p, L, R)
        assert torch.equal(c16.to(torch.int32).to(torch.float32), torch.from_numpy(c).to(gpu))
    else:
        assert tau != int(tau)


# every unrolled k_support<Q>, Q = Tp/4 (T 1, 3 -> 1; 5 -> 3; 17 -> 5; 33, 35 -> 9; 41 -> 11;
# 51 -> 13; 57 -> 15; 65 -> 17; Q = 7 runs end to end at T = 25) and T = 71, the generic float4-per-thread kernel past them; the random
# pair is ragged (W not a multiple of 64, H of 4)
@pytest.mark.parametrize("T", [1, 3, 5, 17, 33, 35, 41, 51, 57, 65, 71])
@pytest.mark.parametrize("scene", ["tsukuba", "ragged"])
def test_support(gpu, oracle, T, scene):
    import stereo_matchin_amd.kernels as K
    if scene == "tsukuba":
        Lh, Rh, _ = load_scene("tsukuba")
    else:
        Lh, Rh = _rand_pair(T, 45, 67)
    p = _params(Lh.shape[1], Lh.shape[0], 16, T)
    Tp = K.support_shape(p)[2]
    for img in (Lh, Rh):
        for fn, direction in ((K.asw_vSupport, 0), (K.asw_hSupport, 1)):
            w = _np(fn(p, _t(img, gpu)))
            want = oracle.support(img, T, direction)
            assert np.array_equal(np.transpose(w[:, :, :T], (2, 0, 1)), want), (T, direction)
            assert (w[:, :, T:Tp] == 0).all()
    # the four arrays in one launch (asw_support_all)
    L, R = _t(Lh, gpu), _t(Rh, gpu)
    ws = [K.new_support(p, gpu) for _ in range(4)]
    K.support_all(p, L, R, K.support_lut(p, gpu), *ws)
    for w, img, direction in zip(ws, (Lh, Lh, Rh, Rh), (0, 1, 0, 1)):
        assert np.array_equal(np.transpose(_np(w)[:, :, :T], (2, 0, 1)), oracle.support(img, T, direction))


# 1, 11, 21, 37: no ring kernel, the generic pass (asw_aggregate_any.hip)
@pytest.mark.parametrize("T", [1, 3, 5, 7, 9, 11, 15, 21, 33, 35, 37, 51])
@pytest.mark.parametrize("direction", [0, 1])
def test_single_pass_bit_exact(gpu, oracle, T, direction):
    import stereo_matchin_amd.kernels as K
    H, W, D = 45, 83, 70
    Lh, Rh = _rand_pair(T * 7 + direction, H, W)
    p = _params(W, H, D, T)
    Dp = K.cost_shape(p)[2]
    rng = np.random.default_rng(T)
    cin = (rng.random((D, H, W)) * 700).astype(np.float32)
    sl = oracle.support(Lh, T, direction)
    sr = oracle.support(Rh, T, direction)
    want = oracle.aggregate_pass(sl, sr, cin, T, direction)
    f = K.asw_vSupport if direction == 0 else K.asw_hSupport
    wl, wr = f(p, _t(Lh, gpu)), f(p, _t(Rh, gpu))
    g = K.asw_vCostAggregation if direction == 0 else K.asw_hCostAggregation
    got = plane_major(_np(g(p, wl, wr, _t(pixel_major(cin, Dp), gpu))), D)
    assert_cost_close(got, want)
    assert np.array_equal(got, want), f"max abs diff {np.abs(got - want).max()}"


@pytest.mark.parametrize("direction", [0, 1])
def test_single_pass_sharded_planes(gpu, oracle, direction):
    import stereo_matchin_amd.kernels as K
    H, W, D, T = 40, 300, 200, 33
    d0, d1 = 70, 135
    Lh, Rh = _rand_pair(11, H, W, shift=9)
    p = _params(W, H, D, T, d_begin=d0, d_end=d1)
    Dp = K.cost_shape(p)[2]
    rng = np.random.default_rng(5)
    cin = (rng.random((d1 - d0, H, W)) * 700).astype(np.float32)
    sl, sr = oracle.support(Lh, T, direction), oracle.support(Rh, T, direction)
    want = oracle.aggregate_pass(sl, sr, cin, T, direction, d0=d0, d1=d1, plane_base=d0)
    f = K.asw_vSupport if direction == 0 else K.asw_hSupport
    g = K.asw_vCostAggregation if direction == 0 else K.asw_hCostAggregation
    got = plane_major(_np(g(p, f(p, _t(Lh, gpu)), f(p, _t(Rh, gpu)), _t(pixel_major(cin, Dp), gpu))), d1 - d0)
    assert np.array_equal(got, want)


# cached denominators: a DEN_WRITE pass on one cost volume, then a DEN_READ pass on
# another with the same supports, each bit-exact against the oracle's full pass
@pytest.mark.parametrize("T", [3, 5, 7, 9, 11, 15, 33, 35, 51])
@pytest.mark.parametrize("direction", [0, 1])
@pytest.mark.parametrize("H,W,D,d0,d1", [(37, 91, 70, 0, 70), (23, 150, 200, 70, 135)])
def test_den_cache_write_then_read(gpu, oracle, T, direction, H, W, D, d0, d1):
    import torch

    import stereo_matchin_amd.kernels as K
    from stereo_matchin_amd import _lib
    Lh, Rh = _rand_pair(T * 3 + direction + W, H, W, shift=6)
    p = _params(W, H, D, T, d_begin=d0, d_end=d1)
    Dp = K.cost_shape(p)[2]
    rng = np.random.default_rng(T + D)
    sl, sr = oracle.support(Lh, T, direction), oracle.support(Rh, T, direction)
    f = K.asw_vSupport if direction == 0 else K.asw_hSupport
    g = K.asw_vCostAggregation if direction == 0 else K.asw_hCostAggregation
    wl, wr = f(p, _t(Lh, gpu)), f(p, _t(Rh, gpu))
    den = torch.full(K.cost_shape(p), float("nan"), dtype=torch.float32, device=gpu)
    for mode in (_lib.DEN_WRITE, _lib.DEN_READ):
        cin = (rng.random((d1 - d0, H, W)) * 700).astype(np.float32)
        want = oracle.aggregate_pass(sl, sr, cin, T, direction, d0=d0, d1=d1, plane_base=d0)
        out = g(p, wl, wr, _t(pixel_major(cin, Dp), gpu), den=den, den_mode=mode)
        got = plane_major(_np(out), d1 - d0)
        assert np.array_equal(got, want), (mode, np.argwhere(got != want)[:5])


# the raw costs as uint16 (asw_raw_cost16) and the first V pass over them
# (asw_aggregate_pass_den16, the matcher's and the frame API's default since round 5):
# the uint16 volume holds exactly asw_raw_cost's floats, and the pass equals the float
# pass bit for bit (64-lane k_vpass10 and, for a shard of <= 32 planes, k_vpass32),
# incl. padding planes, truncated AD at an integral tau, both den modes
@pytest.mark.parametrize("T", [5, 9, 33, 35, 51])
@pytest.mark.parametrize("H,W,D,d0,d1,tau", [(37, 91, 70, 0, 70, 765.0), (23, 150, 200, 70, 135, 765.0),
                                              (40, 77, 64, 0, 64, 90.0), (3, 5, 9, 0, 9, 765.0),
                                              (150, 70, 64, 0, 64, 765.0), (233, 37, 200, 10, 140, 90.0),
                                              (41, 131, 256, 96, 128, 765.0), (150, 70, 256, 224, 256, 30.0)])
def test_raw16_first_v_pass(gpu, T, H, W, D, d0, d1, tau):
    import torch

    import stereo_matchin_amd.kernels as K
    from stereo_matchin_amd import _lib
    Lh, Rh = _rand_pair(T * 3 + W + D, H, W, shift=6)
    p = _params(W, H, D, T, d_begin=d0, d_end=d1, tad_tau=tau)
    assert K.raw16_supported(p)
    L, R = _t(Lh, gpu), _t(Rh, gpu)
    c0 = K.asw_Aggr(p, L, R)
    c16 = K.asw_Aggr16(p, L, R)
    assert torch.equal(c16.to(torch.int32).to(torch.float32), c0)  # every plane, the padding zeros too
    wl, wr = K.asw_vSupport(p, L), K.asw_vSupport(p, R)
    kern = "k_vpass32_c16<" if K.cost_shape(p)[2] == 32 else "k_vpass10_c16<"
    for mode in (_lib.DEN_NONE, _lib.DEN_WRITE):
        den_a = torch.full(K.cost_shape(p), float("nan"), dtype=torch.float32, device=gpu)
        den_b = den_a.clone()
        want = K.asw_vCostAggregation(p, wl, wr, c0, den=den_a, den_mode=mode)
        got = K.asw_vCostAggregation16(p, wl, wr, c16, den=den_b, den_mode=mode)
        assert K.pass_kernel(0, mode).startswith(kern + f"T={T},"), K.pass_kernel(0, mode)
        n = d1 - d0
        assert torch.equal(got[..., :n], want[..., :n]), (mode, torch.nonzero(got[..., :n] != want[..., :n])[:5])
        if mode == _lib.DEN_WRITE:
            assert torch.equal(den_b[..., :n], den_a[..., :n])


def test_raw16_rejects(gpu):
    """A non-integral tau truncates the costs to non-integers: no uint16 form
    (ASW_E_UNSUPPORTED), and the matcher keeps the float volume; den-read is no first pass."""
    import torch

    import stereo_matchin_amd.kernels as K
    from stereo_matchin_amd import _lib
    from stereo_matchin_amd.pipeline import StereoMatcher
    p = _params(40, 16, 64, 9, tad_tau=30.5)
    assert not K.raw16_supported(p)
    img = torch.zeros((16, 40, 4), dtype=torch.uint8, device=gpu)
    with pytest.raises(_lib.AswError) as e:
        K.asw_Aggr16(p, img, img)
    assert e.value.status == _lib.ASW_E_UNSUPPORTED
    assert not StereoMatcher(p, gpu).raw16
    q = _params(40, 16, 64, 9)
    assert StereoMatcher(q, gpu).raw16 and not StereoMatcher(_params(40, 16, 64, 9, flags=_lib.FLAG_RAW_F32), gpu).raw16
    w = K.new_support(q, gpu)
    c16 = torch.zeros(K.cost_shape(q), dtype=torch.int16, device=gpu)
    with pytest.raises(_lib.AswError) as e:
        K.asw_vCostAggregation16(q, w, w, c16, den=K.new_cost(q, gpu), den_mode=_lib.DEN_READ)
    assert e.value.status == _lib.ASW_E_INVALID


# V pass (k_vpass10) on images tall enough for its unclamped interior chunks
# (rows well past 2T + the look-ahead), every den mode, a shard with padding planes
@pytest.mark.parametrize("T", [5, 9, 35, 51])
@pytest.mark.parametrize("H,W,D,d0,d1", [(150, 70, 64, 0, 64), (233, 37, 200, 10, 140)])
def test_vpass_v10_bit_exact(gpu, oracle, T, H, W, D, d0, d1):
    import torch

    import stereo_matchin_amd.kernels as K
    from stereo_matchin_amd import _lib
    Lh, Rh = _rand_pair(T * 7 + W, H, W, shift=5)
    p = _params(W, H, D, T, d_begin=d0, d_end=d1)
    Dp = K.cost_shape(p)[2]
    rng = np.random.default_rng(T + H)
    sl, sr = oracle.support(Lh, T, 0), oracle.support(Rh, T, 0)
    wl, wr = K.asw_vSupport(p, _t(Lh, gpu)), K.asw_vSupport(p, _t(Rh, gpu))
    den = torch.full(K.cost_shape(p), float("nan"), dtype=torch.float32, device=gpu)
    for mode in (_lib.DEN_NONE, _lib.DEN_WRITE, _lib.DEN_READ):
        cin = (rng.random((d1 - d0, H, W)) * 700).astype(np.float32)
        want = oracle.aggregate_pass(sl, sr, cin, T, 0, d0=d0, d1=d1, plane_base=d0)
        out = K.asw_vCostAggregation(p, wl, wr, _t(pixel_major(cin, Dp), gpu), den=den, den_mode=mode)
        got = plane_major(_np(out), d1 - d0)
        assert np.array_equal(got, want), (mode, np.argwhere(got != want)[:5])


# H pass k_hpass11 (one right-weight LDS ring per block of 4, 2 or 1 plane blocks:
# Dp = 256, 512 / 128 / 192, 64), every den mode, several segments per row, a shard
# whose first plane is not 0; T = 33 and the 1-wave blocks refill 4 entries per batch
@pytest.mark.parametrize("T", [5, 33, 35, 51])
@pytest.mark.parametrize("H,W,D,d0,d1", [(7, 530, 256, 0, 256), (3, 300, 520, 4, 516), (4, 290, 300, 40, 296),
                                          (5, 410, 128, 0, 128), (6, 333, 200, 8, 200), (3, 150, 64, 0, 50)])
def test_hpass_h11_bit_exact(gpu, oracle, T, H, W, D, d0, d1):
    import torch

    import stereo_matchin_amd.kernels as K
    from stereo_matchin_amd import _lib
    Lh, Rh = _rand_pair(T * 5 + W, H, W, shift=7)
    p = _params(W, H, D, T, d_begin=d0, d_end=d1)
    Dp = K.cost_shape(p)[2]
    rng = np.random.default_rng(T + W)
    sl, sr = oracle.support(Lh, T, 1), oracle.support(Rh, T, 1)
    wl, wr = K.asw_hSupport(p, _t(Lh, gpu)), K.asw_hSupport(p, _t(Rh, gpu))
    den = torch.full(K.cost_shape(p), float("nan"), dtype=torch.float32, device=gpu)
    old = _lib.lib().asw_tune_set(1, 4096)  # k_hpass11 below its frame-size threshold too
    try:
        for mode in (_lib.DEN_NONE, _lib.DEN_WRITE, _lib.DEN_READ):
            cin = (rng.random((d1 - d0, H, W)) * 700).astype(np.float32)
            want = oracle.aggregate_pass(sl, sr, cin, T, 1, d0=d0, d1=d1, plane_base=d0)
            out = K.asw_hCostAggregation(p, wl, wr, _t(pixel_major(cin, Dp), gpu), den=den, den_mode=mode)
            got = plane_major(_np(out), d1 - d0)
            assert np.array_equal(got, want), (mode, np.argwhere(got != want)[:5])
    finally:
        _lib.lib().asw_tune_set(1, old)


# every compiled pass variant (asw_tune_set): H block shapes (128: k_hpass9 always;
# 4096: k_hpass11 at any size, 512: with 2-chunk segments), on shapes that hit
# segment / row edges
@pytest.mark.parametrize("variant", [0, 128, 4096, 4096 + 512])
@pytest.mark.parametrize("H,W,D,d0,d1", [(9, 331, 256, 0, 256), (6, 47, 128, 0, 128), (5, 161, 300, 40, 168),
                                          (4, 400, 256, 128, 256)])
def test_pass_variants_bit_exact(gpu, oracle, variant, H, W, D, d0, d1):
    import stereo_matchin_amd.kernels as K
    from stereo_matchin_amd import _lib
    T = 35
    Lh, Rh = _rand_pair(variant * 31 + W, H, W, shift=5)
    p = _params(W, H, D, T, d_begin=d0, d_end=d1)
    Dp = K.cost_shape(p)[2]
    rng = np.random.default_rng(W + variant)
    cin = (rng.random((d1 - d0, H, W)) * 700).astype(np.float32)
    old = _lib.lib().asw_tune_set(1, variant)
    try:
        for direction in (0, 1):
            sl, sr = oracle.support(Lh, T, direction), oracle.support(Rh, T, direction)
            want = oracle.aggregate_pass(sl, sr, cin, T, direction, d0=d0, d1=d1, plane_base=d0)
            f = K.asw_vSupport if direction == 0 else K.asw_hSupport
            g = K.asw_vCostAggregation if direction == 0 else K.asw_hCostAggregation
            out = g(p, f(p, _t(Lh, gpu)), f(p, _t(Rh, gpu)), _t(pixel_major(cin, Dp), gpu))
            got = plane_major(_np(out), d1 - d0)
            assert np.array_equal(got, want), (variant, direction, np.argwhere(got != want)[:5])
    finally:
        _lib.lib().asw_tune_set(1, old)


def test_wta_and_consistency_on_oracle_volume(gpu, oracle):
    import stereo_matchin_amd.kernels as K
    Lh, Rh, _ = load_scene("tsukuba")
    H, W = Lh.shape[:2]
    ref = oracle.match(Lh, Rh, 61, 33, 7, want_cost=True)
    p = _params(W, H, 61, 33)
    cost = _t(pixel_major(ref["cost"], 64), gpu)
    d_ref, conf_ref, d_tar, conf_tar, code_ref, code_tar = K.asw_WTA(p, cost)
    assert np.array_equal(_np(d_ref), ref["d_ref"])
    assert np.array_equal(_np(d_tar), ref["d_tar"])
    out, red = K.Constistency(p, d_ref, d_tar, code_ref, code_tar, conf_ref, conf_tar)
    assert np.array_equal(_np(red), ref["lr_red_rgba"])
    assert np.array_equal(_np(out), ref["lr_rgba"])
    assert np.array_equal(_np(conf_ref), ref["conf_ref"])
    assert np.array_equal(_np(conf_tar), ref["conf_tar"])


# ------------------------------------------------------------------ end to end

def _run(gpu, Lh, Rh, D, T, iters, **kw):
    from stereo_matchin_amd import StereoMatcher
    p = _params(Lh.shape[1], Lh.shape[0], D, T, iters, **kw)
    m = StereoMatcher(p, gpu)
    return p, m.match(_t(Lh, gpu), _t(Rh, gpu))


def _compare_e2e(res, ref, D):
    assert np.array_equal(_np(res.d_ref), ref["d_ref"])
    assert np.array_equal(_np(res.d_tar), ref["d_tar"])
    assert np.array_equal(_np(res.lr_red_rgba), ref["lr_red_rgba"])
    assert np.array_equal(_np(res.lr_rgba), ref["lr_rgba"])
    assert np.array_equal(_np(res.conf_ref), ref["conf_ref"])
    assert np.array_equal(_np(res.conf_tar), ref["conf_tar"])
    cost = plane_major(_np(res.cost), D)
    assert_cost_close(cost, ref["cost"])
    assert np.array_equal(cost, ref["cost"])


def test_e2e_tsukuba_reference_params(gpu, oracle):
    """D=61, T=33, r=7: the reference's own configuration (main.cpp:176-177)."""
    Lh, Rh, dev_red = load_scene("tsukuba")
    _, res = _run(gpu, Lh, Rh, 61, 33, 7)
    ref = oracle.match(Lh, Rh, 61, 33, 7, want_cost=True)
    _compare_e2e(res, ref, 61)
    # and therefore the committed device PNG, exactly
    assert np.array_equal(_np(res.lr_red_rgba)[..., :3], dev_red)


@pytest.mark.parametrize("raw_f32", [False, True])
def test_e2e_c1_tsukuba_d16_t5(gpu, oracle, raw_f32):
    from stereo_matchin_amd import _lib
    Lh, Rh, _ = load_scene("tsukuba")
    _, res = _run(gpu, Lh, Rh, 16, 5, 7, flags=_lib.FLAG_RAW_F32 if raw_f32 else 0)
    _compare_e2e(res, oracle.match(Lh, Rh, 16, 5, 7, want_cost=True), 16)


@pytest.mark.parametrize("scene", ["cones", "teddy"])
def test_e2e_c2_c3_d64_t35(gpu, oracle, scene):
    Lh, Rh, _ = load_scene(scene)
    _, res = _run(gpu, Lh, Rh, 64, 35, 7)
    _compare_e2e(res, oracle.match(Lh, Rh, 64, 35, 7, want_cost=True), 64)


@pytest.mark.parametrize("scene", ["laundry", "art", "cones"])
def test_e2e_device_png_agreement(gpu, oracle, scene):
    Lh, Rh, dev_red = load_scene(scene)
    _, res = _run(gpu, Lh, Rh, 61, 33, 7)
    ref = oracle.match(Lh, Rh, 61, 33, 7)
    assert np.array_equal(_np(res.lr_red_rgba), ref["lr_red_rgba"])
    frac = (_np(res.lr_red_rgba)[..., :3] != dev_red).any(-1).mean()
    assert frac <= 0.0025


@pytest.mark.parametrize("H,W,D,T,iters", [
    (1, 1, 1, 3, 1), (1, 1, 4, 5, 2), (2, 3, 5, 9, 2), (7, 5, 12, 33, 1), (5, 70, 3, 51, 1),
    (33, 2, 7, 35, 2), (17, 19, 65, 15, 1), (9, 130, 129, 7, 2), (31, 47, 64, 35, 0),
    (24, 61, 40, 11, 2), (20, 90, 70, 25, 2)])
def test_e2e_edge_shapes(gpu, oracle, H, W, D, T, iters):
    Lh, Rh = _rand_pair(H * 1000 + W * 10 + D, H, W, shift=min(3, W - 1))
    _, res = _run(gpu, Lh, Rh, D, T, iters)
    _compare_e2e(res, oracle.match(Lh, Rh, D, T, iters, want_cost=True), D)


def test_lr_native_mode(gpu, oracle):
    Lh, Rh, _ = load_scene("teddy")
    _, res = _run(gpu, Lh, Rh, 64, 35, 2, lr_mode=1)
    ref = oracle.match(Lh, Rh, 64, 35, 2)
    d_ref, d_tar = ref["d_ref"], ref["d_tar"]
    assert np.array_equal(_np(res.d_ref), d_ref) and np.array_equal(_np(res.d_tar), d_tar)
    cons = np.abs(d_ref - d_tar) <= 1
    code = oracle.code_u8(d_ref, 64)
    grey = np.stack([code, code, code, np.full_like(code, 255)], -1)
    want = np.where(cons[..., None], grey, np.array([255, 0, 0, 255], np.uint8))
    assert np.array_equal(_np(res.lr_red_rgba), want)


def test_frame_api_equals_stage_pipeline(gpu, oracle):
    from stereo_matchin_amd import match_frame
    Lh, Rh, _ = load_scene("tsukuba")
    p, res = _run(gpu, Lh, Rh, 61, 33, 7)
    out = match_frame(p, Lh, Rh, device=0, want_cost=True)
    assert np.array_equal(out["d_ref"], _np(res.d_ref))
    assert np.array_equal(out["d_tar"], _np(res.d_tar))
    assert np.array_equal(out["lr_red_rgba"], _np(res.lr_red_rgba))
    assert np.array_equal(out["cost"], _np(res.cost))
    disp = out["disp_rgba"]
    assert np.array_equal(disp[..., 0], oracle.code_u8(out["d_ref"], 61)) and (disp[..., 3] == 255).all()
    t = out["timings"]
    assert t["total"] > 0 and t["aggregation_total"] > 0


# ------------------------------------------------------------------ sharding

def _simulated_shards(gpu, Lh, Rh, D, T, iters, G):
    """Run G d-shards one after another on one GPU and combine with torch.minimum,
    exercising the exact protocol of stereo_matchin_amd.distributed.sharded_wta."""
    import torch
    from stereo_matchin_amd import StereoMatcher
    from stereo_matchin_amd.distributed import HipShardOps, shard_range
    import stereo_matchin_amd.kernels as K
    H, W = Lh.shape[:2]
    L_, R_ = _t(Lh, gpu), _t(Rh, gpu)
    shards = []
    for g in range(G):
        p = _params(W, H, D, T, iters)
        p.d_begin, p.d_end = shard_range(D, g, G)
        m = StereoMatcher(p, gpu)
        m.raw_and_support(L_, R_)
        shards.append((p, HipShardOps(p), m.aggregate().clone()))
    loc = [ops.local(c) for _, ops, c in shards]
    key_g = torch.stack([k for k, _, _ in loc]).amin(0)
    m2_g = torch.stack([ops.second(key_g, k, a, b) for (_, ops, _), (k, a, b) in zip(shards, loc)]).amin(0)
    tl = [ops.target_local(c, key_g) for _, ops, c in shards]
    tkey_g = torch.stack([k for k, _, _ in tl]).amin(0)
    t2_g = torch.stack([ops.second(tkey_g, k, a, b) for (_, ops, _), (k, a, b) in zip(shards, tl)]).amin(0)
    return shards[0][1].finalize(key_g, m2_g, tkey_g, t2_g)


@pytest.mark.parametrize("G", [2, 3, 8])
def test_sharded_equals_unsharded(gpu, G):
    Lh, Rh, _ = load_scene("cones")
    D, T, iters = 64, 35, 2
    _, res = _run(gpu, Lh, Rh, D, T, iters)
    d_ref, conf_ref, d_tar, conf_tar, code_ref, code_tar = _simulated_shards(gpu, Lh, Rh, D, T, iters, G)
    assert np.array_equal(_np(d_ref), _np(res.d_ref))
    assert np.array_equal(_np(d_tar), _np(res.d_tar))
    assert np.array_equal(_np(code_ref), _np(res.code_ref))
    assert np.array_equal(_np(code_tar), _np(res.code_tar))
    # res confidences were zeroed by the consistency stage; compare before it
    from stereo_matchin_amd.kernels import asw_WTA
    p = _params(Lh.shape[1], Lh.shape[0], D, T, iters)
    _, cr, _, ct, _, _ = asw_WTA(p, res.cost)
    assert np.array_equal(_np(conf_ref), _np(cr))
    assert np.array_equal(_np(conf_tar), _np(ct))


# ------------------------------------------------------------------ full-size parity (C4, C5 band)

def _pass_kernels():
    from stereo_matchin_amd.kernels import pass_kernel
    return {(d, m): pass_kernel(d, m) for d in (0, 1) for m in (1, 2)}


def _cost_equal_on_gpu(gpu, cost_hwdp, ref_dhw):
    """bit-exact compare of a device [H][W][Dp] volume with the oracle's [D][H][W], on the GPU"""
    import torch
    D = ref_dhw.shape[0]
    want = torch.from_numpy(ref_dhw).to(gpu).permute(1, 2, 0)
    got = cost_hwdp[:, :, :D]
    rel = ((got.double() - want.double()).abs() / want.double().abs().clamp_min(1.0)).max().item()
    assert rel <= COST_TOL, rel
    neq = int((got != want).sum())
    assert neq == 0, f"{neq} voxels differ"


def test_c4_full_frame_oracle_parity(gpu, oracle):
    """C4 as benched: 1920x1080, D=256, T=35, r=7 + LR check on a synthetic pair, the
    WHOLE frame bit-exact against the oracle (maps, confidences, LR images and the
    float volume; K/asw_vcost_aggregation.cl:33-43, K/asw_hcost_aggregation.cl:34-41,
    K/asw_wta.cl:22-80).  The volume is past 256 MB and the H grid past 8192 waves, so
    the shipped nt / row-segment instantiations run: asserted by name."""
    import torch
    from stereo_matchin_amd import StereoMatcher
    from stereo_matchin_amd.synthetic import make_pair
    W, H, D, T = 1920, 1080, 256, 35
    Lh, Rh, gt = make_pair(W, H, D, 0)
    p, res = _run(gpu, Lh, Rh, D, T, 7)  # the matcher's default (as benched)
    names = _pass_kernels()
    print("C4 pass kernels:", names)
    m = StereoMatcher(p, gpu)
    raw16 = m.raw16  # the first V pass: k_vpass10_c16 (uint16 raw costs)
    del m
    for dm in (1, 2):
        v = "k_vpass10_c16" if raw16 and dm == 1 else "k_vpass10"
        assert names[(0, dm)].startswith(f"{v}<T={T},NW=16,DM={dm}") and names[(0, dm)].endswith(",nt>"), names
        assert names[(1, dm)].startswith(f"k_hpass11<T={T},NKW=4,DM={dm}") and names[(1, dm)].endswith(",nt>"), \
            names
    ref = oracle.match(Lh, Rh, D, T, 7, want_cost=True)
    for k in ("d_ref", "d_tar", "conf_ref", "conf_tar", "lr_rgba", "lr_red_rgba"):
        assert np.array_equal(_np(getattr(res, k)), ref[k]), k
    _cost_equal_on_gpu(gpu, res.cost, ref.pop("cost"))
    # determinism, and quality sanity on the synthetic ground truth (non-occluded interior)
    res2 = StereoMatcher(p, gpu).match(_t(Lh, gpu), _t(Rh, gpu))
    assert torch.equal(res.cost, res2.cost) and torch.equal(res.d_tar, res2.d_tar)
    inner = np.s_[40:-40, 300:-40]
    assert (np.abs(_np(res.d_ref)[inner] - gt[inner]) <= 1).mean() > 0.6


C5_H_NKW = 2  # plane blocks per k_hpass11 block at T = 51 (launch_dm)


def test_c5_band_oracle_parity(gpu, oracle):
    """A full-width C5 band: 3840x270, D=512, T=51, r=7, native LR check, bit-exact
    against the oracle.  2.1 GB volume (> 256 MB: nt streams) and 38880 H waves
    (> 8192: the row-segment k_hpass11), the instantiations the C5 bench runs."""
    import torch
    from stereo_matchin_amd.synthetic import make_pair
    W, H, D, T = 3840, 2160, 512, 51
    Lh, Rh, _ = make_pair(W, H, D, 3)
    Ls, Rs = np.ascontiguousarray(Lh[900:1170]), np.ascontiguousarray(Rh[900:1170])
    del Lh, Rh
    p, res = _run(gpu, Ls, Rs, D, T, 7, lr_mode=1)
    names = _pass_kernels()
    print("C5 band pass kernels:", names)
    from stereo_matchin_amd.kernels import raw16_supported
    raw16 = raw16_supported(p)  # the matcher's default (p.flags = 0): uint16 raw costs
    for dm in (1, 2):
        v = "k_vpass10_c16" if raw16 and dm == 1 else "k_vpass10"
        # 12-column blocks in 3 phases; on this 3840-wide band in XCD-round tiles of 4 plane
        # blocks (v12_tiles in asw_aggregate_impl.h)
        assert names[(0, dm)] == f"{v}<T={T},NW=12,NPH=3,TK=4,DM={dm},nt>", names
        # (den-read: the deeper cost prefetch, PX = 24, round 6)
        h = f"k_hpass11<T={T},NKW={C5_H_NKW}" + (",PX=24" if dm == 2 else "") + f",DM={dm}"
        assert names[(1, dm)].startswith(h) and names[(1, dm)].endswith(",nt>"), names
    ref = oracle.match(Ls, Rs, D, T, 7, want_cost=True)
    dr, dt = ref["d_ref"], ref["d_tar"]
    assert np.array_equal(_np(res.d_ref), dr) and np.array_equal(_np(res.d_tar), dt)
    assert dr.max() > 256  # past the 8-bit code range
    # native LR check (the oracle's match() applies the 8-bit rule): red exactly where
    # |d_ref - d_tar| > 1, confidences = the oracle WTA's, zeroed there
    bad = np.abs(dr - dt) > 1
    red = _np(res.lr_red_rgba)
    assert np.array_equal((red[..., 0] == 255) & (red[..., 1] == 0) & (red[..., 2] == 0), bad)
    _, cr, _, ct = oracle.wta(ref["cost"])
    assert np.array_equal(_np(res.conf_ref), np.where(bad, np.float32(0), cr))
    assert np.array_equal(_np(res.conf_tar), np.where(bad, np.float32(0), ct))
    _cost_equal_on_gpu(gpu, res.cost, ref.pop("cost"))
    del res
    torch.cuda.empty_cache()


# ------------------------------------------------------------------ full-size properties (C5)

def test_c5_full_size_properties(gpu, oracle):
    """3840x2160, D=512, T=51, r=7 (C5, one pair) with the native LR check: parity on a
    full-width strip against the oracle, size-independent properties on the whole frame."""
    import torch
    from stereo_matchin_amd import StereoMatcher
    from stereo_matchin_amd.synthetic import make_pair
    W, H, D, T = 3840, 2160, 512, 51
    Lh, Rh, gt = make_pair(W, H, D, 3)
    p = _params(W, H, D, T, 7, lr_mode=1)
    m = StereoMatcher(p, gpu)
    L, R = _t(Lh, gpu), _t(Rh, gpu)
    res = m.match(L, R)
    d_ref, d_tar = res.d_ref.clone(), res.d_tar.clone()
    dr = _np(d_ref)
    assert dr.min() >= 0 and dr.max() < D and dr.max() > 256  # past the 8-bit code range
    # the index map is the first argmin of the returned volume (row blocks bound memory)
    for y0 in range(0, H, 270):
        c = res.cost[y0:y0 + 270, :, :D]
        mn = c.amin(-1, keepdim=True)
        first = (c == mn).to(torch.uint8).argmax(-1)
        assert torch.equal(first.int(), d_ref[y0:y0 + 270]), y0
        del c, mn, first
    # native LR check: red exactly where |d_ref - d_tar| > 1
    red = _np(res.lr_red_rgba)
    bad = (red[..., 0] == 255) & (red[..., 1] == 0) & (red[..., 2] == 0)
    assert np.array_equal(bad, np.abs(dr - _np(d_tar)) > 1)
    # determinism: the same context again gives the same bits
    cost_sum = float(res.cost[:, :, :D].double().sum())
    res2 = m.match(L, R)
    assert torch.equal(res2.d_ref, d_ref) and torch.equal(res2.d_tar, d_tar)
    assert float(res2.cost[:, :, :D].double().sum()) == cost_sum
    # quality sanity on the synthetic ground truth (non-occluded interior)
    inner = np.s_[60:-60, 600:-60]
    assert (np.abs(dr[inner] - gt[inner]) <= 1).mean() > 0.6
    del m, res, res2
    torch.cuda.empty_cache()
    # bit-exact parity on a full-width strip (3840 x 24 rows, r = 2 to bound the oracle)
    Ls, Rs = np.ascontiguousarray(Lh[1000:1024]), np.ascontiguousarray(Rh[1000:1024])
    _, rs = _run(gpu, Ls, Rs, D, T, 2, lr_mode=1)
    want = oracle.match(Ls, Rs, D, T, 2, want_cost=True)
    assert np.array_equal(_np(rs.d_ref), want["d_ref"]) and np.array_equal(_np(rs.d_tar), want["d_tar"])
    got = plane_major(_np(rs.cost), D)
    assert_cost_close(got, want["cost"])
    assert np.array_equal(got, want["cost"])
