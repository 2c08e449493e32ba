"""Deterministic synthetic stereo pairs for the C4/C5 workloads.

There are no 1080p/4K scenes in the reference (its inputs are the five
Middlebury pairs); the benchmark configurations use synthetic pairs:

* PRNG: splitmix64, seed = 0x5EED0000 + pair_index (no RNG-library dependence);
* ground-truth disparity: 24 slanted planar rectangles painted in order, integer
  d in [0, D-1];
* left image: per-region base colour + 3-octave value noise (amplitude 40) +
  per-pixel uniform +-3 LSB, clamped to 0..255, alpha 255;
* right image: forward warp Right(x - d, y) = Left(x, y), larger d wins;
  holes filled with fresh noise.
"""
from __future__ import annotations

import numpy as np

_M64 = (1 << 64) - 1


class SplitMix64:
    def __init__(self, seed: int):
        self.state = np.uint64(seed & _M64)

    def next_u64(self, n: int) -> np.ndarray:
        with np.errstate(over="ignore"):
            idx = np.arange(1, n + 1, dtype=np.uint64)
            z = self.state + idx * np.uint64(0x9E3779B97F4A7C15)
            self.state = self.state + np.uint64(n) * np.uint64(0x9E3779B97F4A7C15)
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            return z ^ (z >> np.uint64(31))

    def uniform(self, n: int) -> np.ndarray:
        return (self.next_u64(n) >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))

    def integers(self, lo: int, hi: int, n: int) -> np.ndarray:
        return lo + (self.next_u64(n) % np.uint64(hi - lo)).astype(np.int64)


def _value_noise(rng: SplitMix64, W: int, H: int, cell: int) -> np.ndarray:
    gw, gh = W // cell + 2, H // cell + 2
    g = rng.uniform(gw * gh * 3).reshape(gh, gw, 3) * 2.0 - 1.0
    xs = np.arange(W) / cell
    ys = np.arange(H) / cell
    x0 = np.floor(xs).astype(np.int64)
    y0 = np.floor(ys).astype(np.int64)
    fx = (xs - x0)[None, :, None]
    fy = (ys - y0)[:, None, None]
    a = g[y0][:, x0]
    b = g[y0][:, x0 + 1]
    c = g[y0 + 1][:, x0]
    d = g[y0 + 1][:, x0 + 1]
    return (a * (1 - fx) + b * fx) * (1 - fy) + (c * (1 - fx) + d * fx) * fy


def make_pair(width: int, height: int, ndisp: int, pair_index: int = 0, regions: int = 24):
    """Return ``(left_rgba, right_rgba, gt_disparity)`` as numpy arrays."""
    W, H, D = width, height, ndisp
    rng = SplitMix64(0x5EED0000 + pair_index)
    disp = np.zeros((H, W), np.float64)
    base = np.zeros((H, W, 3), np.float64)
    bg = rng.uniform(3) * 255.0
    base[:] = bg
    disp[:] = rng.uniform(1)[0] * (D - 1) * 0.25
    for _ in range(regions):
        u = rng.uniform(9)
        rw, rh = max(8, int(u[0] * W * 0.5)), max(8, int(u[1] * H * 0.5))
        x0, y0 = int(u[2] * (W - rw)), int(u[3] * (H - rh))
        d0 = u[4] * (D - 1)
        ax = (u[5] - 0.5) * 0.2
        ay = (u[6] - 0.5) * 0.2
        col = rng.uniform(3) * 255.0
        yy, xx = np.mgrid[y0:y0 + rh, x0:x0 + rw]
        disp[y0:y0 + rh, x0:x0 + rw] = d0 + ax * (xx - x0 - rw / 2) + ay * (yy - y0 - rh / 2)
        base[y0:y0 + rh, x0:x0 + rw] = col
    gt = np.clip(np.rint(disp), 0, D - 1).astype(np.int32)
    noise = sum(_value_noise(rng, W, H, c) * (40.0 / 2 ** o) for o, c in enumerate((64, 16, 4)))
    jitter = rng.integers(-3, 4, H * W * 3).reshape(H, W, 3)
    left = np.clip(np.rint(base + noise) + jitter, 0, 255).astype(np.uint8)

    # forward warp, larger disparity wins: write in ascending-d order
    right = np.clip(rng.integers(0, 256, H * W * 3).reshape(H, W, 3), 0, 255).astype(np.uint8)
    ys, xs = np.mgrid[0:H, 0:W]
    xr = xs - gt
    ok = xr >= 0
    order = np.argsort(gt[ok], kind="stable")
    src_y, src_x, dst_x = ys[ok][order], xs[ok][order], xr[ok][order]
    right[src_y, dst_x] = left[src_y, src_x]

    alpha = np.full((H, W, 1), 255, np.uint8)
    return (np.ascontiguousarray(np.concatenate([left, alpha], 2)),
            np.ascontiguousarray(np.concatenate([right, alpha], 2)), gt)
