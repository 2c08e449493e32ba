"""Parity of the HIP refinement loop (main.cpp:540-623: asw_ref_v, asw_ref_h,
asw_WTA_REF, Constistency, Median) and of the lane-per-pixel WTA scan with the
CPU oracle (oracle_refine, pinned to the reference's asw_disparity.png /
asw_consistency_post-reff.png — tsukuba exact).  Run on an MI355X; bit-exact on
every output (indices, codes, images, confidences, refined estimates)."""
import numpy as np
import pytest

from conftest import GOLDEN, load_scene, pixel_major

pytestmark = pytest.mark.gpu


def _t(a, dev):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _np(t):
    return t.detach().cpu().numpy()


def _params(W, H, D, T, iters=7, **kw):
    from stereo_matchin_amd import make_params
    return make_params(W, H, ndisp=D, taps=T, iters=iters, **kw)


def _rand_pair(seed, H, W, shift=4):
    rng = np.random.default_rng(seed)
    L = rng.integers(0, 256, (H, W, 4), dtype=np.uint8)
    R = np.roll(L, -shift, axis=1).copy()
    R[..., :3] = np.clip(R[..., :3].astype(int) + rng.integers(-5, 6, (H, W, 3)), 0, 255).astype(np.uint8)
    L[..., 3] = 255
    R[..., 3] = 255
    return np.ascontiguousarray(L), np.ascontiguousarray(R)


def _gpu_refine(gpu, Lh, Rh, D, T, iters, k, Tr=33):
    from stereo_matchin_amd import StereoMatcher, _lib
    p = _params(Lh.shape[1], Lh.shape[0], D, T, iters)
    m = StereoMatcher(p, gpu)
    L, R = _t(Lh, gpu), _t(Rh, gpu)
    res = m.match(L, R)
    out = m.refine(res, L, R, _lib.default_refine_params(iters=k, taps=Tr))
    return res, out


def _compare(res, out, ref):
    assert np.array_equal(_np(out["final_rgba"]), ref["final_rgba"]), "asw_disparity.png"
    assert np.array_equal(_np(out["post_red_rgba"]), ref["post_red_rgba"]), "asw_consistency_post-reff.png"
    assert np.array_equal(_np(out["d_ref"]), ref["ref_d_ref"])
    assert np.array_equal(_np(out["d_tar"]), ref["ref_d_tar"])
    assert np.array_equal(_np(res.conf_ref), ref["ref_conf_ref"])
    assert np.array_equal(_np(res.conf_tar), ref["ref_conf_tar"])


def test_refine_tsukuba_reference_params(gpu, oracle):
    """D=61, T=33, r=7, k=6: the reference run; equals the oracle bit for bit and
    therefore the committed device PNGs asw_disparity.png / post-reff exactly."""
    Lh, Rh, _ = load_scene("tsukuba")
    res, out = _gpu_refine(gpu, Lh, Rh, 61, 33, 7, 6)
    ref = oracle.match(Lh, Rh, 61, 33, 7, refine_iters=6)
    _compare(res, out, ref)
    z = np.load(f"{GOLDEN}/tsukuba.npz")
    assert np.array_equal(_np(out["final_rgba"])[..., :3], z["disp_final"])
    assert np.array_equal(_np(out["post_red_rgba"])[..., :3], z["lr_post_red"])


@pytest.mark.parametrize("scene", ["cones", "teddy"])
def test_refine_c2_c3(gpu, oracle, scene):
    Lh, Rh, _ = load_scene(scene)
    res, out = _gpu_refine(gpu, Lh, Rh, 64, 35, 7, 6)
    _compare(res, out, oracle.match(Lh, Rh, 64, 35, 7, refine_iters=6))


@pytest.mark.parametrize("H,W,D,T,iters,k,Tr", [
    (1, 1, 2, 3, 1, 1, 3), (3, 5, 7, 5, 1, 2, 5), (17, 40, 16, 5, 2, 3, 9), (40, 23, 61, 9, 1, 2, 33),
    (9, 130, 100, 7, 1, 1, 51), (20, 70, 256, 5, 1, 2, 15), (12, 31, 16, 5, 1, 0, 33)])
def test_refine_edge_shapes(gpu, oracle, H, W, D, T, iters, k, Tr):
    Lh, Rh = _rand_pair(H * 131 + W + D, H, W, shift=min(5, W - 1))
    res, out = _gpu_refine(gpu, Lh, Rh, D, T, iters, k, Tr)
    pre = oracle.match(Lh, Rh, D, T, iters, want_cost=True)
    ref = oracle.refine(Lh, Rh, D, pre["cost"], pre, k, Tr)
    assert np.array_equal(_np(out["final_rgba"]), ref["final_rgba"])
    if k > 0:
        _compare(res, out, ref)


def test_refine_stages_one_iteration(gpu, oracle):
    """asw_ref_v -> asw_ref_h -> asw_WTA_REF -> Constistency -> Median called one by
    one through the stage API equal the asw_refine loop (k = 1)."""
    import stereo_matchin_amd.kernels as K
    from stereo_matchin_amd import StereoMatcher, _lib
    Lh, Rh, _ = load_scene("tsukuba")
    p = _params(Lh.shape[1], Lh.shape[0], 61, 33)
    rp = _lib.default_refine_params(iters=1)
    m = StereoMatcher(p, gpu)
    L, R = _t(Lh, gpu), _t(Rh, gpu)
    res = m.match(L, R)
    est, ct = res.lr_rgba.clone(), res.code_tar.clone()
    cr, cf = res.conf_ref.clone(), res.conf_tar.clone()
    lut = K.refine_lut(p, rp, gpu)
    vl = K.asw_ref_v(p, rp, L, est, cr, lut)
    vr = K.asw_ref_v(p, rp, R, ct, cf, lut)
    hl = K.asw_ref_h(p, rp, L, cr, vl, lut)
    hr = K.asw_ref_h(p, rp, R, cf, vr, lut)
    d_ref, d_tar, k_ref, k_tar = K.asw_WTA_REF(p, res.cost, hl, hr, cr)
    o1, o2 = K.Constistency(p, d_ref, d_tar, k_ref, k_tar, cr, cf)
    fin = K.Median(p, o1)
    out = m.refine(res, L, R, rp)
    assert np.array_equal(_np(fin), _np(out["final_rgba"]))
    assert np.array_equal(_np(o2), _np(out["post_red_rgba"]))
    assert np.array_equal(_np(d_ref), _np(out["d_ref"]))
    assert np.array_equal(_np(cr), _np(res.conf_ref)) and np.array_equal(_np(cf), _np(res.conf_tar))


def test_frame_api_refine(gpu, oracle):
    from stereo_matchin_amd import _lib, match_frame
    Lh, Rh, dev_red = load_scene("tsukuba")
    p = _params(Lh.shape[1], Lh.shape[0], 61, 33)
    out = match_frame(p, Lh, Rh, device=0, refine=_lib.default_refine_params())
    ref = oracle.match(Lh, Rh, 61, 33, 7, refine_iters=6)
    assert np.array_equal(out["final_rgba"], ref["final_rgba"])
    assert np.array_equal(out["post_red_rgba"], ref["post_red_rgba"])
    # lr outputs stay the pre-refinement images
    assert np.array_equal(out["lr_red_rgba"][..., :3], dev_red)
    assert np.array_equal(out["lr_rgba"], ref["lr_rgba"])
    assert out["timings"]["refine"] > 0


@pytest.mark.parametrize("variant", [0, 2])
@pytest.mark.parametrize("H,W,D", [(1, 1, 1), (5, 67, 61), (13, 129, 256), (3, 200, 300), (7, 64, 33),
                                   (2, 700, 128), (4, 1000, 256), (3, 63, 200), (2, 300, 2)])
def test_wta_variants_on_random_volume(gpu, oracle, variant, H, W, D):
    """asw_WTA: the lane-per-pixel scan (variant 0) and the row sweep (2: Dp 64 / 128 /
    256, the scan elsewhere; round 1's wave-per-pixel form is checked by
    tools/exp/exp_forms.py) against the oracle on
    volumes with many exact ties (rows longer than the 255-plane diagonals, the clamped
    first points of pixels x < md, rows not a multiple of 64 pixels)."""
    import stereo_matchin_amd.kernels as K
    from stereo_matchin_amd import _lib
    rng = np.random.default_rng(H * W + D)
    cost = rng.integers(1, 9, (D, H, W)).astype(np.float32)  # small integers: ties everywhere
    p = _params(W, H, D, 3)
    want = oracle.wta(cost)
    old = _lib.lib().asw_tune_set(2, variant)
    try:
        got = K.asw_WTA(p, _t(pixel_major(cost, K.cost_shape(p)[2]), gpu))
    finally:
        _lib.lib().asw_tune_set(2, old)
    for i, (g, w) in enumerate(zip(got[:4], want[:4])):
        assert np.array_equal(_np(g), w), (i, np.argwhere(_np(g) != w)[:5])
