"""The 32-plane shard passes (k_vpass32 / k_hpass32, asw_pass32.h) — run on an MI355X.

A d-shard of at most 32 planes (the C4 frame split over 8 GPUs: 32 of 256 planes per
GPU) has pitch Dp = 32 and runs passes that hold two pixels per wave.  Every pass is
compared bit for bit with the oracle's pass (the reference's tap sequence,
K/asw_vcost_aggregation.cl:33-40, K/asw_hcost_aggregation.cl:34-41) over the shard's
planes, in all three denominator modes, on shapes that hit the image edges (W < 32,
odd heights, a row pair cut by the bottom), for every ring tap count.
"""
import numpy as np
import pytest

from conftest import pixel_major, plane_major

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


def test_pitch_of_small_shards():
    import stereo_matchin_amd.kernels as K
    assert K.cost_shape(_params(40, 20, 256, 35, d_begin=224, d_end=256))[2] == 32
    assert K.cost_shape(_params(40, 20, 256, 35, d_begin=0, d_end=32))[2] == 32
    assert K.cost_shape(_params(40, 20, 100, 35, d_begin=40, d_end=57))[2] == 32
    assert K.cost_shape(_params(40, 20, 256, 35, d_begin=0, d_end=33))[2] == 64
    assert K.cost_shape(_params(40, 20, 16, 5))[2] == 64  # a whole (unsharded) range keeps 64


# every ring tap count (other odd T run k_pass_any, pitch 32 too), both directions,
# a DEN_NONE, a DEN_WRITE and a DEN_READ pass each bit-exact against the oracle
@pytest.mark.parametrize("T", [3, 5, 7, 9, 11, 15, 33, 35, 51])
@pytest.mark.parametrize("direction", [0, 1])
@pytest.mark.parametrize("H,W,D,d0,d1", [(37, 91, 70, 38, 70), (23, 150, 200, 70, 87), (8, 20, 64, 0, 32),
                                          (9, 331, 256, 224, 256)])
def test_pass32_bit_exact(gpu, oracle, T, direction, H, W, D, d0, d1):
    import torch

    import stereo_matchin_amd.kernels as K
    from stereo_matchin_amd import _lib
    Lh, Rh = _rand_pair(T * 5 + direction + W, H, W, shift=6)
    p = _params(W, H, D, T, d_begin=d0, d_end=d1)
    Dp = K.cost_shape(p)[2]
    assert Dp == 32
    rng = np.random.default_rng(T + D + H)
    sl, sr = oracle.support(Lh, T, direction), oracle.support(Rh, T, direction)
    f = K.asw_vSupport if direction == 0 else K.asw_hSupport
    g = K.asw_vCostAggregation if direction == 0 else K.asw_hCostAggregation
    wl, wr = f(p, _t(Lh, gpu)), f(p, _t(Rh, gpu))
    den = torch.full(K.cost_shape(p), float("nan"), dtype=torch.float32, device=gpu)
    for mode in (_lib.DEN_NONE, _lib.DEN_WRITE, _lib.DEN_READ):
        cin = (rng.random((d1 - d0, H, W)) * 700).astype(np.float32)
        want = oracle.aggregate_pass(sl, sr, cin, T, direction, d0=d0, d1=d1, plane_base=d0)
        out = g(p, wl, wr, _t(pixel_major(cin, Dp), gpu), den=den, den_mode=mode)
        got = plane_major(_np(out), d1 - d0)
        assert np.array_equal(got, want), (mode, np.argwhere(got != want)[:5])
        name = K.pass_kernel(direction, mode)
        if T in (3, 5, 7, 9, 15, 33, 35, 51):
            assert name.startswith(("k_vpass32<" if direction == 0 else "k_hpass32<") + f"T={T},"), name
        else:
            assert name.startswith("k_pass_any<"), name


# the V pass with both weights on the fly (asw_aggregate_pass_otf_v): the
# oracle's pass over its support arrays, bit for bit, for every ring tap count <= 35 on the
# edge shapes of the float tests, in both cache policies
@pytest.mark.parametrize("T", [3, 5, 7, 9, 15, 33, 35])
@pytest.mark.parametrize("H,W,D,d0,d1", [(37, 91, 70, 38, 70), (23, 150, 200, 70, 87), (8, 20, 64, 0, 32),
                                          (9, 331, 256, 224, 256), (150, 70, 256, 96, 128)])
def test_pass32_otf_v_bit_exact(gpu, oracle, tune_variant, T, H, W, D, d0, d1):
    import stereo_matchin_amd.kernels as K
    Lh, Rh = _rand_pair(T * 11 + W, H, W, shift=6)
    p = _params(W, H, D, T, d_begin=d0, d_end=d1)
    assert K.otf_v_supported(p)
    rng = np.random.default_rng(T + D + H + 1)
    sl, sr = oracle.support(Lh, T, 0), oracle.support(Rh, T, 0)
    L, R = _t(Lh, gpu), _t(Rh, gpu)
    lut = K.support_lut(p, gpu)
    for flip in (False, True):
        if flip:
            tune_variant(1 << 26)
        cin = (rng.random((d1 - d0, H, W)) * 700).astype(np.float32)
        want = oracle.aggregate_pass(sl, sr, cin, T, 0, d0=d0, d1=d1, plane_base=d0)
        out = K.asw_vCostAggregation_otf_v(p, L, R, lut, _t(pixel_major(cin, 32), gpu))
        assert K.pass_kernel(0, 0).startswith(f"k_vpass32_otf<T={T},"), K.pass_kernel(0, 0)
        got = plane_major(_np(out), d1 - d0)
        assert np.array_equal(got, want), (flip, np.argwhere(got != want)[:5])


def test_pass32_otf_v_supported_shapes(gpu):
    import stereo_matchin_amd.kernels as K
    from stereo_matchin_amd import _lib
    assert not K.otf_v_supported(_params(64, 16, 256, 51, d_begin=224, d_end=256))  # T > 35
    assert not K.otf_v_supported(_params(64, 16, 256, 11, d_begin=224, d_end=256))  # no ring kernel
    assert not K.otf_v_supported(_params(64, 16, 256, 35, d_begin=192, d_end=256))  # pitch 64
    assert not K.otf_v_supported(_params(64, 16, 256, 35, d_begin=224, d_end=256, color_space=_lib.COLOR_LAB))


# the other forms behind variant bits (asw_pass32.h): bit 26 = the nt cache policy flipped
# (both passes), bit 24 = the 4-wave-block H form
@pytest.mark.parametrize("variant", [1 << 26, 1 << 24])
@pytest.mark.parametrize("T", [9, 35])
@pytest.mark.parametrize("H,W,D,d0,d1", [(37, 91, 70, 38, 70), (9, 331, 256, 224, 256)])
def test_pass32_h_variants_bit_exact(gpu, oracle, tune_variant, variant, T, H, W, D, d0, d1):
    tune_variant(variant)
    for direction in ((0, 1) if variant == 1 << 26 else (1,)):
        test_pass32_bit_exact(gpu, oracle, T, direction, H, W, D, d0, d1)


# the lean H form's left weights: from DPP rows (DL, the default; T <= 35) and from the
# LDS ring (variant bit 27): every ring tap count, all den modes, on the edge shapes, in
# both cache policies; the V pass and T = 51 have one form
@pytest.mark.parametrize("T", [3, 5, 7, 9, 15, 33, 35, 51])
@pytest.mark.parametrize("lds_left", [False, True])
def test_pass32_dl_bit_exact(gpu, oracle, tune_variant, T, lds_left):
    import stereo_matchin_amd.kernels as K
    from stereo_matchin_amd import _lib
    for flip in (False, True):
        tune_variant((1 << 27 if lds_left else 0) | (1 << 26 if flip else 0))
        for direction in (0, 1):
            for H, W, D, d0, d1 in ((37, 91, 70, 38, 70), (8, 20, 64, 0, 32), (9, 331, 256, 224, 256),
                                    (150, 70, 256, 96, 128)):
                test_pass32_bit_exact(gpu, oracle, T, direction, H, W, D, d0, d1)
                name = K.pass_kernel(direction, _lib.DEN_READ)
                assert (",DL" in name) == (direction == 1 and T <= 35 and not lds_left), name


def test_pass32_rejects_fused_raw_and_otf(gpu):
    import torch

    import stereo_matchin_amd.kernels as K
    from stereo_matchin_amd import _lib
    p = _params(64, 16, 256, 35, d_begin=224, d_end=256)
    assert not K.otf_supported(p)
    x = torch.zeros(K.cost_shape(p), dtype=torch.float32, device=gpu)
    w = torch.zeros(K.support_shape(p), dtype=torch.float32, device=gpu)
    img = torch.zeros((16, 64, 4), dtype=torch.uint8, device=gpu)
    with pytest.raises(_lib.AswError) as e:
        K.asw_vCostAggregation_raw(p, w, w, img, img, out=x)
    assert e.value.status == _lib.ASW_E_UNSUPPORTED


# the full-size C4 shard (1920 x 1080 x 32 x 4 B = 253 MiB, just under the 256 MiB nt
# threshold) in both cache-policy instantiations of both passes (variant bit 26 flips
# the policy; ADVICE r04: no smaller test shape reaches the nt ones): one den-none V and
# one den-none H pass, as the shard's frame runs them, against the oracle over the
# whole shard
@pytest.mark.parametrize("flip", [False, True])
def test_c4_shard_full_size_passes(gpu, oracle, tune_variant, flip):
    import stereo_matchin_amd.kernels as K
    from stereo_matchin_amd import _lib
    from stereo_matchin_amd.synthetic import make_pair
    W, H, D, T = 1920, 1080, 256, 35
    d0, d1 = 96, 128
    Lh, Rh, _ = make_pair(W, H, D, 5)
    p = _params(W, H, D, T, iters=7, d_begin=d0, d_end=d1)
    assert K.cost_shape(p) == (H, W, 32) and H * W * 32 * 4 < 256 << 20
    if flip:
        tune_variant(1 << 26)
    rng = np.random.default_rng(11)
    cin = (rng.random((d1 - d0, H, W)) * 700).astype(np.float32)
    for direction in (0, 1):
        sl, sr = oracle.support(Lh, T, direction), oracle.support(Rh, T, direction)
        want = oracle.aggregate_pass(sl, sr, cin, T, direction, d0=d0, d1=d1, plane_base=d0)
        f = K.asw_vSupport if direction == 0 else K.asw_hSupport
        g = K.asw_vCostAggregation if direction == 0 else K.asw_hCostAggregation
        out = g(p, f(p, _t(Lh, gpu)), f(p, _t(Rh, gpu)), _t(pixel_major(cin, 32), gpu), den_mode=_lib.DEN_NONE)
        name = K.pass_kernel(direction, _lib.DEN_NONE)
        assert name.startswith(("k_vpass32<" if direction == 0 else "k_hpass32<") + f"T={T},") and \
            name.endswith(",nt>") == flip, name
        got = plane_major(_np(out), d1 - d0)
        assert np.array_equal(got, want), (direction, np.argwhere(got != want)[:5])
        cin = want  # the H pass aggregates the V pass's output, as in the frame


# the C4 shard of the 8-way split: one rank's 32 planes of a 1920-column D256 T35
# frame through the whole r = 7 pass sequence, on a full-width band of 215 rows (the
# oracle's passes over all 1080 rows take minutes), against the oracle on that band
def test_c4_shard_band_r7(gpu, oracle):
    import stereo_matchin_amd.kernels as K
    from stereo_matchin_amd import _lib
    from stereo_matchin_amd.pipeline import StereoMatcher
    from stereo_matchin_amd.synthetic import make_pair
    W, H, D, T, r = 1920, 1080, 256, 35, 7
    Lh, Rh, _ = make_pair(W, H, D, 0)
    band = 96 + r * (T // 2)
    d0, d1 = 96, 128  # rank 3 of 8
    Lb, Rb = np.ascontiguousarray(Lh[:band]), np.ascontiguousarray(Rh[:band])
    p = _params(W, band, D, T, iters=r, d_begin=d0, d_end=d1)
    cost = oracle.raw_cost(Lb, Rb, D)[d0:d1]
    sv = (oracle.support(Lb, T, 0), oracle.support(Rb, T, 0))
    sh = (oracle.support(Lb, T, 1), oracle.support(Rb, T, 1))
    for _ in range(r):
        cost = oracle.aggregate_pass(*sv, cost, T, 0, d0=d0, d1=d1, plane_base=d0)
        cost = oracle.aggregate_pass(*sh, cost, T, 1, d0=d0, d1=d1, plane_base=d0)
    # float supports (the default), index-form supports (opt-in), and
    # float supports with the H denominators cached (ASW_FLAG_SHARD_DEN_H), and the V
    # weights on the fly (ASW_FLAG_OTF_V: no V support arrays)
    for index, denh, otfv in ((None, "0", False), (True, "0", False), (None, "1", False), (None, "0", True)):
        p.flags = (_lib.FLAG_SHARD_DEN_H if denh == "1" else 0) | (_lib.FLAG_OTF_V if otfv else 0)
        m = StereoMatcher(p, gpu, support_index=index)
        assert m.otfv == otfv and (m.wvl is None) == otfv
        m.raw_and_support(_t(Lb, gpu), _t(Rb, gpu))
        got = plane_major(_np(m.aggregate()), d1 - d0)
        # (a 32-plane shard recomputes the denominators of both directions by default)
        tag = ",IDX" if index else ""
        assert m.vidx == m.hidx == bool(index)
        assert K.pass_kernel(0, 0).startswith(("k_vpass32_otf" if otfv else "k_vpass32") + "<T=35,NW=16,NPH=4" + tag), \
            K.pass_kernel(0, 0)
        assert (m.den_h is not None) == (denh == "1")
        assert K.pass_kernel(1, 2 if denh == "1" else 0).startswith(
            "k_hpass32<T=35,NWB=" + ("8,NPH=4,IDX" if index else "1,NPH=4")), K.pass_kernel(1, 0)
        assert np.array_equal(got, cost), (index, denh, np.argwhere(got != cost)[:5])
        del m


# ---------------------------------------------------------------------------
# index-form supports (asw_support_all_fmt / asw_aggregate_pass_index):
# uint16 LUT indices in place of the float weights of a 32-plane shard's V passes


@pytest.mark.parametrize("T", [3, 9, 35, 51])
@pytest.mark.parametrize("H,W", [(37, 91), (8, 20), (70, 150)])
def test_support_index_form_is_lut_index(gpu, T, H, W):
    """lut[index] equals the float weight asw_support writes, bit for bit, in all four
    arrays (clamped edges included: the index carries the clamped distance); padding
    taps hold index 0."""
    import torch

    import stereo_matchin_amd.kernels as K
    Lh, Rh = _rand_pair(T + H + W, H, W)
    p = _params(W, H, 256, T)
    L, R = _t(Lh, gpu), _t(Rh, gpu)
    lut = K.support_lut(p, gpu)
    wf = [K.new_support(p, gpu) for _ in range(4)]
    wi = [K.new_support_index(p, gpu) for _ in range(4)]
    K.support_all(p, L, R, lut, *wf)
    K.support_all(p, L, R, lut, *wi)
    # mixed formats in one launch (what a 32-plane shard computes: V index, H float)
    wm = [wi[0].clone().zero_(), K.new_support(p, gpu), wi[2].clone().zero_(), K.new_support(p, gpu)]
    K.support_all(p, L, R, lut, *wm)
    flat = lut.reshape(-1)
    for j in range(4):
        idx = wi[j].to(torch.int32) & 0xFFFF
        assert int(idx.max()) < flat.numel()
        got = flat[idx.reshape(-1).long()].reshape(wf[j].shape)
        got[..., T:] = 0.0
        assert torch.equal(got.view(torch.int32), wf[j].view(torch.int32)), j
        assert int(idx[..., T:].abs().sum()) == 0
    assert torch.equal(wm[0], wi[0]) and torch.equal(wm[2], wi[2])
    assert torch.equal(wm[1], wf[1]) and torch.equal(wm[3], wf[3])


@pytest.mark.parametrize("T", [3, 5, 7, 9, 15, 33, 35])
@pytest.mark.parametrize("H,W,D,d0,d1", [(37, 91, 70, 38, 70), (23, 150, 200, 70, 87), (8, 20, 64, 0, 32),
                                          (9, 331, 256, 224, 256)])
@pytest.mark.parametrize("direction", [0, 1])
def test_pass32_index_bit_exact(gpu, oracle, T, direction, H, W, D, d0, d1):
    """The passes over index-form supports equal the oracle's pass (and so the float
    form) bit for bit: V in den mode NONE, H in all three."""
    import torch

    import stereo_matchin_amd.kernels as K
    from stereo_matchin_amd import _lib
    Lh, Rh = _rand_pair(T * 7 + W + direction, H, W, shift=6)
    p = _params(W, H, D, T, d_begin=d0, d_end=d1)
    Dp = K.cost_shape(p)[2]
    assert Dp == 32 and K.index_supported(p, direction, 0)
    L, R = _t(Lh, gpu), _t(Rh, gpu)
    lut = K.support_lut(p, gpu)
    iw = [K.new_support_index(p, gpu) for _ in range(4)]
    K.support_all(p, L, R, lut, *iw)
    il, ir = (iw[0], iw[2]) if direction == 0 else (iw[1], iw[3])
    sl, sr = oracle.support(Lh, T, direction), oracle.support(Rh, T, direction)
    rng = np.random.default_rng(T + D + H)
    den = torch.full(K.cost_shape(p), float("nan"), dtype=torch.float32, device=gpu)
    modes = (_lib.DEN_NONE,) if direction == 0 else (_lib.DEN_NONE, _lib.DEN_WRITE, _lib.DEN_READ)
    for mode in modes:
        cin = (rng.random((d1 - d0, H, W)) * 700).astype(np.float32)
        want = oracle.aggregate_pass(sl, sr, cin, T, direction, d0=d0, d1=d1, plane_base=d0)
        out = K.aggregate_pass_index(p, direction, il, ir, lut, _t(pixel_major(cin, Dp), gpu), den=den,
                                     den_mode=mode)
        got = plane_major(_np(out), d1 - d0)
        assert np.array_equal(got, want), (mode, np.argwhere(got != want)[:5])
        name = K.pass_kernel(direction, mode)
        assert name.startswith(("k_vpass32<" if direction == 0 else "k_hpass32<") + f"T={T},") and ",IDX" in name


def test_pass_index_supported_shapes(gpu):
    import torch

    import stereo_matchin_amd.kernels as K
    from stereo_matchin_amd import _lib
    shard = dict(d_begin=224, d_end=256)
    assert K.index_supported(_params(64, 16, 256, 35, **shard), 0, 0)
    assert all(K.index_supported(_params(64, 16, 256, 35, **shard), 1, dm) for dm in (0, 1, 2))
    assert not K.index_supported(_params(64, 16, 256, 35, **shard), 0, 2)       # V: den mode NONE only
    assert not K.index_supported(_params(64, 16, 256, 51, **shard), 0, 0)       # LUT + slab exceed the LDS
    assert not K.index_supported(_params(64, 16, 256, 11, **shard), 0, 0)       # no ring kernel
    assert not K.index_supported(_params(64, 16, 256, 35), 0, 0)                # pitch 64
    assert not K.index_supported(_params(64, 16, 256, 35, color_space=1, **shard), 0, 0)
    p = _params(64, 16, 256, 35)
    x = torch.zeros(K.cost_shape(p), dtype=torch.float32, device=gpu)
    w = torch.zeros(K.support_shape(p), dtype=torch.int16, device=gpu)
    lut = K.support_lut(p, gpu)
    with pytest.raises(_lib.AswError) as e:
        K.aggregate_pass_index(p, 0, w, w, lut, x, out=x.clone())
    assert e.value.status == _lib.ASW_E_UNSUPPORTED
    # a StereoMatcher on a full range keeps float supports; on a shard: on request
    from stereo_matchin_amd.pipeline import StereoMatcher
    assert not StereoMatcher(p, gpu, support_index=True).vidx
    assert StereoMatcher(_params(64, 16, 256, 35, **shard), gpu, support_index=True).vidx
    assert not StereoMatcher(_params(64, 16, 256, 35, **shard), gpu).vidx
    m = StereoMatcher(_params(64, 16, 256, 35, **shard), gpu, support_index="v")
    assert m.vidx and not m.hidx
