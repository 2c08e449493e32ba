"""The WTA's own scan fused into the last H pass (asw_aggregate_pass_wta_local,
k_hpass11_wl) — run on an MI355X.

The fused pass must write the same volume as the den-read H pass and the same
(key, m1, m2) as asw_wta_local on that volume (K/asw_wta.cl:34-47: strict '<' in plane
order, the first argmin, the second minimum of the multiset, the 100000 sentinels),
bit for bit: on random and tie-heavy volumes, ragged widths (a last batch cut by the
segment end), padding planes (nloc < pitch), d-shards (global indices) and both block
shapes (pitch 256: 4 plane blocks per block; 128: 2).  End to end, a frame with the
fused pass equals the unfused one and asw_WTA.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

H11_ANY_SIZE = 4096  # pass variant bit: k_hpass11 at any frame size (small test shapes)


def _params(W, H, D, T, **kw):
    from stereo_matchin_amd import make_params
    return make_params(W, H, ndisp=D, taps=T, iters=7, **kw)


def _pair(seed, H, W):
    rng = np.random.default_rng(seed)
    L = rng.integers(0, 256, (H, W, 4), dtype=np.uint8)
    R = np.roll(L, -5, axis=1)
    R = np.clip(R.astype(int) + rng.integers(-6, 7, R.shape), 0, 255).astype(np.uint8)
    L[..., 3] = 255
    R[..., 3] = 255
    return np.ascontiguousarray(L), np.ascontiguousarray(R)


@pytest.mark.parametrize("W,H,D,d0,d1,fill", [
    (500, 9, 256, 0, 256, "rand"),      # pitch 256, 3 segments, a ragged last batch
    (333, 7, 256, 0, 256, "const"),     # tie-heavy output: equal minima across blocks and chunks
    (241, 5, 100, 0, 100, "rand"),      # pitch 128 (2 plane blocks), 28 padding planes
    (300, 6, 256, 64, 190, "const"),    # a d-shard (global indices), pitch 128
    (97, 4, 256, 0, 256, "rand"),       # one segment narrower than U
    (150, 3, 256, 0, 256, "sentinel"),  # no value below the 100000 sentinel: no key
])
def test_fused_pass_equals_pass_and_local_scan(gpu, tune_variant, W, H, D, d0, d1, fill):
    import torch

    import stereo_matchin_amd.kernels as K
    from stereo_matchin_amd import _lib
    tune_variant(H11_ANY_SIZE)
    T = 35
    p = _params(W, H, D, T, d_begin=d0, d_end=d1)
    assert K.wta_local_fused_supported(p)
    Lh, Rh = _pair(W + H + D, H, W)
    L, R = torch.from_numpy(Lh).to(gpu), torch.from_numpy(Rh).to(gpu)
    wl, wr = K.asw_hSupport(p, L), K.asw_hSupport(p, R)
    rng = np.random.default_rng(W * H)
    shape = K.cost_shape(p)
    if fill == "const":  # outputs num/den of a constant: many exactly equal
        cin = torch.full(shape, 7.0, dtype=torch.float32, device=gpu)
    elif fill == "sentinel":
        cin = torch.full(shape, 2.0e5, dtype=torch.float32, device=gpu)
    else:
        cin = torch.from_numpy((rng.random(shape) * 700).astype(np.float32)).to(gpu)
    den = torch.empty_like(cin)
    ref = K.asw_hCostAggregation(p, wl, wr, cin, den=den, den_mode=_lib.DEN_WRITE)  # den_h
    ref = K.asw_hCostAggregation(p, wl, wr, cin, den=den, den_mode=_lib.DEN_READ)
    want = K.wta_local(p, ref)
    out, key, m1, m2 = K.asw_hCostAggregation_wta_local(p, wl, wr, cin, den)
    assert torch.equal(out, ref)
    if fill == "sentinel":
        assert bool((key == 0x7fffffffffffffff).all())
    for name, a, b in (("key", key, want[0]), ("m1", m1, want[1]), ("m2", m2, want[2])):
        assert torch.equal(a.view(torch.int32) if a.dtype == torch.float32 else a,
                           b.view(torch.int32) if b.dtype == torch.float32 else b), \
            (name, torch.nonzero(a != b)[:5].tolist())


def test_fused_supported_shapes(gpu, tune_variant):
    import stereo_matchin_amd.kernels as K
    assert not K.wta_local_fused_supported(_params(500, 9, 256, 51))          # T > 35
    assert not K.wta_local_fused_supported(_params(500, 9, 512, 35))          # pitch 512: 8 plane blocks
    assert not K.wta_local_fused_supported(_params(500, 9, 256, 35, d_begin=224, d_end=256))  # pitch 32
    assert not K.wta_local_fused_supported(_params(500, 9, 256, 11))          # no ring kernel
    assert not K.wta_local_fused_supported(_params(500, 9, 256, 35))          # small: the H pass is k_hpass9
    assert K.wta_local_fused_supported(_params(1920, 1080, 256, 35))          # C4
    tune_variant(H11_ANY_SIZE)
    assert K.wta_local_fused_supported(_params(500, 9, 256, 35))


@pytest.mark.parametrize("lr", [False, True])
def test_frame_fused_equals_unfused(gpu, tune_variant, lr):
    """A whole frame with the fused last pass + target scan equals the unfused frame
    (asw_WTA) in every output, and the fused path really ran."""
    import torch

    from stereo_matchin_amd.pipeline import StereoMatcher
    tune_variant(H11_ANY_SIZE)
    W, H, D = 257, 40, 128
    Lh, Rh = _pair(7, H, W)
    L, R = torch.from_numpy(Lh).to(gpu), torch.from_numpy(Rh).to(gpu)
    p = _params(W, H, D, 35)
    a = StereoMatcher(p, gpu, wta_fused=True)
    b = StereoMatcher(p, gpu)  # (the default: opt-in by ASW_FLAG_WTA_FUSED)
    assert a.wta_fused and not b.wta_fused
    ra, rb = a.match(L, R, lr_check=lr), b.match(L, R, lr_check=lr)
    assert a.local is not None and b.local is None
    for k in ("d_ref", "conf_ref", "d_tar", "conf_tar", "code_ref", "code_tar", "lr_rgba", "lr_red_rgba", "cost"):
        x, y = getattr(ra, k), getattr(rb, k)
        if x is None:
            assert y is None
            continue
        assert torch.equal(x, y), k


def test_pipelined_fused_equals_match(gpu, tune_variant):
    """PipelinedMatcher with ASW_FLAG_WTA_FUSED (the one-shard protocol's target scan and
    finalize on the side stream, from the last pass's local scan) equals StereoMatcher.match
    frame after frame."""
    import torch

    from stereo_matchin_amd import _lib
    from stereo_matchin_amd.distributed import PipelinedMatcher
    from stereo_matchin_amd.pipeline import StereoMatcher
    tune_variant(H11_ANY_SIZE)
    W, H, D = 257, 40, 128
    p = _params(W, H, D, 35)
    p.flags = _lib.FLAG_WTA_FUSED
    pm = PipelinedMatcher(p, device=gpu)
    assert pm.sets[0].wta_fused
    ref = StereoMatcher(_params(W, H, D, 35), gpu)
    got, want = [], []
    for seed in (1, 2, 3):
        Lh, Rh = _pair(seed, H, W)
        L, R = torch.from_numpy(Lh).to(gpu), torch.from_numpy(Rh).to(gpu)
        torch.cuda.synchronize()
        got.append(pm.submit(L, R))
        want.append(ref.match(L, R))
    pm.flush()
    torch.cuda.synchronize()
    for a, b in zip(got, want):
        for k in ("d_ref", "conf_ref", "d_tar", "conf_tar", "code_ref", "code_tar", "lr_rgba", "lr_red_rgba"):
            assert torch.equal(getattr(a, k), getattr(b, k)), k
