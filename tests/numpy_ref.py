"""Independent pure-numpy restatement of the reference ASW path (test infrastructure).

Used only to cross-check the C oracle (oracle/asw_oracle.c) on small inputs; it
restates the same reference lines (cited per function) with numpy vector ops
over (plane, y, x).  numpy has no fused multiply-add, so ``fma32`` evaluates
a*b+c in float64 (a*b is exact there) and rounds once more to float32; a
double-rounding difference is possible in principle (probability ~2^-29 per op)
and has not been observed on these sizes.
"""
from __future__ import annotations

import math

import numpy as np

f32 = np.float32


def fma32(a, b, c):
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(np.float32)


def raw_cost(L, R, D):
    """K/asw_aggr.cl:12-21"""
    H, W = L.shape[:2]
    Lf = L[..., :3].astype(np.float32)
    out = np.empty((D, H, W), np.float32)
    xs = np.arange(W)
    for d in range(D):
        Rs = R[:, np.maximum(xs - d, 0), :3].astype(np.float32)
        a = np.abs(Lf - Rs)
        out[d] = (a[..., 0] + a[..., 1]) + a[..., 2]
    return out


def support(img, T, direction, gc=30.91, gg=28.21):
    """K/asw_vsupport.cl:19-25 / K/asw_hsupport.cl:19-25"""
    H, W = img.shape[:2]
    R = T // 2
    im = img[..., :3].astype(np.int64)
    out = np.empty((T, H, W), np.float32)
    ys, xs = np.arange(H), np.arange(W)
    for i in range(T):
        if direction == 0:
            qy = np.clip(ys + i - R, 0, H - 1)
            q = im[qy]
            dist = np.abs(ys - qy)[:, None].repeat(W, 1)
        else:
            qx = np.clip(xs + i - R, 0, W - 1)
            q = im[:, qx]
            dist = np.abs(xs - qx)[None, :].repeat(H, 0)
        sad = np.abs(im - q).sum(-1)
        c_diff = (-sad).astype(np.float32) / f32(gc)
        g_dist = dist.astype(np.float32) / f32(gg)
        arg = (c_diff - g_dist).astype(np.float32)
        out[i] = np.vectorize(lambda v: f32(math.exp(float(v))), otypes=[np.float32])(arg)
    return out


def aggregate_pass(sL, sR, cin, T, direction):
    """K/asw_vcost_aggregation.cl:23-42 / K/asw_hcost_aggregation.cl:24-43, fp policy FMA_NUM."""
    D, H, W = cin.shape
    R = T // 2
    out = np.empty_like(cin)
    xs, ys = np.arange(W), np.arange(H)
    for d in range(D):
        xr = np.maximum(xs - d, 0)
        num = np.full((H, W), f32(1e-5), np.float32)
        den = np.full((H, W), f32(1e-5), np.float32)
        for i in range(T):
            a = sL[i]
            b = sR[i][:, xr]
            if direction == 0:
                c = cin[d][np.clip(ys + i - R, 0, H - 1)]
            else:
                c = cin[d][:, np.clip(xs + i - R, 0, W - 1)]
            ww = (a * b).astype(np.float32)
            num = fma32(ww, c, num)
            den = (den + ww).astype(np.float32)
        out[d] = num / den
    return out


def wta(C):
    """K/asw_wta.cl:22-80, sequential strict-'<' scans restated per pixel."""
    D, H, W = C.shape
    dr = np.zeros((H, W), np.int32)
    dt = np.zeros((H, W), np.int32)
    cr = np.zeros((H, W), np.float32)
    ct = np.zeros((H, W), np.float32)
    for y in range(H):
        for x in range(W):
            m1 = m2 = f32(100000.0)
            idx = 0
            for d in range(D):
                t = C[d, y, x]
                m2 = t if t < m2 else m2
                if t < m1:
                    idx = d
                m2 = m1 if t < m1 else m2
                m1 = t if t < m1 else m1
            t1 = t2 = f32(100000.0)
            mdr = idx
            for i in range(idx):
                xq = max(0, x - i)
                b = idx + xq - x
                t = C[b, y, xq]
                t2 = t if t < t2 else t2
                if t < t1:
                    mdr = b
                t2 = t1 if t < t1 else t2
                t1 = t if t < t1 else t1
            dr[y, x], dt[y, x] = idx, mdr
            cr[y, x] = (m2 - m1) / m2
            ct[y, x] = (t2 - t1) / t2
    return dr, cr, dt, ct


def match(L, R, D, T, iters):
    C = raw_cost(L, R, D)
    vl, hl = support(L, T, 0), support(L, T, 1)
    vr, hr = support(R, T, 0), support(R, T, 1)
    for _ in range(iters):
        C = aggregate_pass(vl, vr, C, T, 0)
        C = aggregate_pass(hl, hr, C, T, 1)
    return C, wta(C)
