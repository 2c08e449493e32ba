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


# the lean H form (T <= 35: left weights from DPP rows, "DL") and the 2-wave form
# (T = 51), and the V pass, in both cache policies (variant bit 26 flips the nt policy):
# every ring tap count, all den modes, on the edge shapes
@pytest.mark.parametrize("T", [3, 5, 7, 9, 15, 33, 35, 51])
def test_pass32_dl_bit_exact(gpu, oracle, tune_variant, T):
    import stereo_matchin_amd.kernels as K
    from stereo_matchin_amd import _lib
    for flip in (False, True):
        tune_variant(1 << 26 if flip else 0)
        for direction in (0, 1):
            for H, W, D, d0, d1 in ((37, 91, 70, 38, 70), (8, 20, 64, 0, 32), (9, 331, 256, 224, 256),
                                    (150, 70, 256, 96, 128)):
                test_pass32_bit_exact(gpu, oracle, T, direction, H, W, D, d0, d1)
                name = K.pass_kernel(direction, _lib.DEN_READ)
                assert (",DL" in name) == (direction == 1 and T <= 35), name


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
    # both raw-cost forms (uint16, the default; ASW_FLAG_RAW_F32)
    for flags in (0, _lib.FLAG_RAW_F32):
        p.flags = flags
        m = StereoMatcher(p, gpu)
        m.raw_and_support(_t(Lb, gpu), _t(Rb, gpu))
        got = plane_major(_np(m.aggregate()), d1 - d0)
        # (a 32-plane shard recomputes the denominators of both directions)
        assert m.den_v is None and m.den_h is None
        assert K.pass_kernel(0, 0).startswith("k_vpass32<T=35,NW=16,NPH=4"), K.pass_kernel(0, 0)
        assert K.pass_kernel(1, 0).startswith("k_hpass32<T=35,NWB=1,NPH=4,DL"), K.pass_kernel(1, 0)
        assert np.array_equal(got, cost), (flags, np.argwhere(got != cost)[:5])
        del m
