"""The symmetry rule behind half-size supports (asw_pass32.h
hs_index), pinned on the CPU oracle: the support weight is symmetric in its pixel
pair (K/asw_vsupport.cl:19-25, K/asw_hsupport.cl:19-26), so taps R..2R of every pixel
determine taps 0..R-1 of every pixel, the clamped border included.  The GPU form
(k_vpass32<HS>, tools/exp/hs_bench.py) was measured not faster and is not shipped;
this test keeps the rule its DESIGN entry states checked."""
import numpy as np
import pytest

from conftest import load_scene


def rebuild(half, T, direction):
    """full [T][H][W] from half [R+1][H][W] (half[u] = tap R+u)"""
    R = T // 2
    _, H, W = half.shape
    full = np.empty((T, H, W), np.float32)
    full[R:] = half
    for u in range(1, R + 1):
        if direction == 0:  # V: the pixel u rows up, else row 0 at tap R+y
            full[R - u, u:] = half[u, :H - u]
            for y in range(min(u, H)):
                full[R - u, y] = half[y, 0]
        else:  # H: the pixel u columns left, else column 0 at tap R+x
            full[R - u, :, u:] = half[u, :, :W - u]
            for x in range(min(u, W)):
                full[R - u, :, x] = half[x, :, 0]
    return full


@pytest.mark.parametrize("T", [5, 33, 35])
@pytest.mark.parametrize("direction", [0, 1])
def test_half_supports_rebuild_full(oracle, T, direction):
    L, Rimg, _ = load_scene("tsukuba")
    for img in (L, Rimg):
        full = oracle.support(img, T, direction)
        R = T // 2
        got = rebuild(full[R:].copy(), T, direction)
        assert np.array_equal(got, full)
