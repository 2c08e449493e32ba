"""CIELab extension (north star).  The reference has no colour
conversion, so nothing in it pins this row: the conversion is pinned by
colorimetric known answers (sRGB D65 primaries, white, black, greys) and the HIP
kernels by bit-exact agreement with the oracle's restatement of the same IEEE
double sequence ("parity unpinned" with respect to the reference itself).
"""
import numpy as np
import pytest

from conftest import load_scene

# published CIE L*a*b* (D65, 2 deg) of the sRGB primaries / neutrals
KNOWN = {
    (255, 255, 255): (100.0, 0.0, 0.0),
    (0, 0, 0): (0.0, 0.0, 0.0),
    (255, 0, 0): (53.2408, 80.0925, 67.2032),
    (0, 255, 0): (87.7347, -86.1827, 83.1793),
    (0, 0, 255): (32.2970, 79.1875, -107.8602),
    (128, 128, 128): (53.5850, 0.0, 0.0),
    (255, 255, 0): (97.1393, -21.5537, 94.4780),
}


def _img(colors):
    a = np.array([[list(c) + [255] for c in colors]], np.uint8)
    return np.ascontiguousarray(a)


def test_oracle_lab_known_answers(oracle):
    cols = list(KNOWN)
    lab = oracle.lab(_img(cols))[0]
    for c, got in zip(cols, lab):
        np.testing.assert_allclose(got[:3], KNOWN[c], atol=2e-3, err_msg=str(c))
        assert got[3] == 0.0


def test_oracle_lab_grey_ramp_monotone_and_neutral(oracle):
    grey = _img([(v, v, v) for v in range(256)])
    lab = oracle.lab(grey)[0]
    assert np.all(np.diff(lab[:, 0]) > 0)
    assert np.abs(lab[:, 1:3]).max() < 1e-3


def test_oracle_support_lab_centre_tap_is_one(oracle):
    L, _, _ = load_scene("tsukuba")
    lab = oracle.lab(L[:40, :50])
    for T, direction in ((5, 0), (33, 1)):
        w = oracle.support_lab(lab, T, direction)
        assert np.all(w[T // 2] == 1.0)
        assert np.all((w > 0) & (w <= 1.0))


@pytest.mark.gpu
def test_lab_exhaustive_bit_exact(gpu, oracle):
    """Every one of the 2^24 RGB colours, HIP vs oracle, bit for bit."""
    import torch
    from stereo_matchin_amd import kernels as K, make_params
    v = np.arange(1 << 24, dtype=np.uint32)
    img = np.empty((4096, 4096, 4), np.uint8)
    img[..., 0] = (v >> 16).reshape(4096, 4096)
    img[..., 1] = ((v >> 8) & 255).reshape(4096, 4096)
    img[..., 2] = (v & 255).reshape(4096, 4096)
    img[..., 3] = 255
    p = make_params(4096, 4096, color_space=1)
    got = K.lab_image(p, torch.from_numpy(img).to(gpu)).cpu().numpy()
    want = oracle.lab(img)
    bad = np.argwhere(got.view(np.uint32) != want.view(np.uint32))
    assert bad.size == 0, f"{len(bad)} differing components, first {bad[:4]}"


@pytest.mark.gpu
@pytest.mark.parametrize("T", [5, 33, 35])
def test_support_lab_bit_exact(gpu, oracle, T):
    import torch
    from stereo_matchin_amd import kernels as K, make_params
    L, R, _ = load_scene("cones")
    H, W = L.shape[:2]
    p = make_params(W, H, ndisp=64, taps=T, color_space=1)
    for img in (L, R):
        lab = K.lab_image(p, torch.from_numpy(img).to(gpu))
        lab_ref = oracle.lab(img)
        for direction in (0, 1):
            got = K.support_lab(p, direction, lab).cpu().numpy()[:, :, :T]
            want = np.transpose(oracle.support_lab(lab_ref, T, direction), (1, 2, 0))
            assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), (T, direction)


@pytest.mark.gpu
def test_rgb_support_entry_rejects_lab_context(gpu):
    import torch
    from stereo_matchin_amd import kernels as K, make_params
    from stereo_matchin_amd._lib import AswError
    p = make_params(16, 8, ndisp=8, taps=5, color_space=1)
    img = torch.zeros((8, 16, 4), dtype=torch.uint8, device=gpu)
    with pytest.raises(AswError):
        K.asw_vSupport(p, img)


@pytest.mark.gpu
@pytest.mark.parametrize("scene,D,T,tau", [("tsukuba", 16, 5, 765.0), ("teddy", 64, 35, 60.0)])
def test_e2e_lab_tad_bit_exact(gpu, oracle, scene, D, T, tau):
    """Full pipeline with the CIELab colour term (and truncated AD) vs the oracle."""
    import torch
    from conftest import plane_major
    from stereo_matchin_amd import StereoMatcher, make_params
    L, R, _ = load_scene(scene)
    H, W = L.shape[:2]
    p = make_params(W, H, ndisp=D, taps=T, iters=3, color_space=1, tad_tau=tau, gamma_c=7.0)
    res = StereoMatcher(p, gpu).match(torch.from_numpy(L).to(gpu), torch.from_numpy(R).to(gpu))
    ref = oracle.match(L, R, D, T, 3, gc=7.0, want_cost=True, color_space=1, tad_tau=tau)
    assert np.array_equal(res.d_ref.cpu().numpy(), ref["d_ref"])
    assert np.array_equal(res.d_tar.cpu().numpy(), ref["d_tar"])
    assert np.array_equal(res.lr_red_rgba.cpu().numpy(), ref["lr_red_rgba"])
    assert np.array_equal(plane_major(res.cost.cpu().numpy(), D), ref["cost"])


@pytest.mark.gpu
def test_frame_api_lab(gpu, oracle):
    """asw_match of a LAB context (the frame API allocates and converts itself)."""
    import ctypes
    from stereo_matchin_amd import _lib, make_params
    L, R, _ = load_scene("tsukuba")
    H, W = L.shape[:2]
    p = make_params(W, H, ndisp=16, taps=5, iters=2, color_space=1, gamma_c=7.0)
    lib = _lib.lib()
    ctx = ctypes.c_void_p()
    _lib.check(lib.asw_create(ctypes.byref(p), 0, ctypes.byref(ctx)), "asw_create")
    try:
        d_ref = np.empty((H, W), np.int32)
        red = np.empty((H, W, 4), np.uint8)
        out = _lib.AswOutputs()
        out.d_ref = d_ref.ctypes.data
        out.lr_red_rgba = red.ctypes.data
        _lib.check(lib.asw_match(ctx, L.ctypes.data, R.ctypes.data, ctypes.byref(out), None), "asw_match")
    finally:
        lib.asw_destroy(ctx)
    ref = oracle.match(L, R, 16, 5, 2, gc=7.0, color_space=1)
    assert np.array_equal(d_ref, ref["d_ref"])
    assert np.array_equal(red, ref["lr_red_rgba"])
