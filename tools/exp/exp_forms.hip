// Measured-negative forms moved out of libasw_hip.so: each is
// bit-exact and was slower than the shipped form on MI355X, so the product no longer
// carries it; they stay here, buildable and checked by tools/exp/exp_forms.py against
// the library's shipped forms.  Not part of the product.
//   * k_support_expd: asw_vSupport / asw_hSupport (K/asw_vsupport.cl:19-25,
//     K/asw_hsupport.cl:19-27) with each weight computed as k_support_lut computes the
//     table entry, (float)exp_d((double)(c_diff[SAD] - g_dist[dist])), instead of
//     gathered from the LUT.  C4: 0.63 vs 0.39 ms, C5: 3.48 vs 1.98 ms
//     (profiles/r04/support_expd_r10j.log).
//   * k_wta_wave: asw_WTA (K/asw_wta.cl:12-82) with one wave per pixel (lanes over d,
//     then a shuffle reduction of the top-2 states), the round-1 form; the shipped
//     lane-per-pixel scan (asw_refine.hip) replaced it (0.84 -> 0.62 ms at C4, DESIGN.md
//     §Side kernels).
// Build: make -C tools/exp libforms.so
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

namespace {

constexpr int kLutWidth = 766;  // SAD 0..765 (include/asw.h LUT layout)

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// the library's exp sequence (asw_kernels.hip exp_d): Cody-Waite + degree-14 Horner in double
__device__ double exp_d(double x) {
    const double inv_ln2 = 1.44269504088896338700e+00;
    const double ln2_hi = 6.93147180369123816490e-01;
    const double ln2_lo = 1.90821492927058770002e-10;
    const double k = rint(x * inv_ln2);
    double r = fma(-k, ln2_hi, x);
    r = fma(-k, ln2_lo, r);
    double p = 1.0 / 87178291200.0;
    p = fma(p, r, 1.0 / 6227020800.0);
    p = fma(p, r, 1.0 / 479001600.0);
    p = fma(p, r, 1.0 / 39916800.0);
    p = fma(p, r, 1.0 / 3628800.0);
    p = fma(p, r, 1.0 / 362880.0);
    p = fma(p, r, 1.0 / 40320.0);
    p = fma(p, r, 1.0 / 5040.0);
    p = fma(p, r, 1.0 / 720.0);
    p = fma(p, r, 1.0 / 120.0);
    p = fma(p, r, 1.0 / 24.0);
    p = fma(p, r, 1.0 / 6.0);
    p = fma(p, r, 0.5);
    p = fma(p, r, 1.0);
    p = fma(p, r, 1.0);
    return ldexp(p, (int)k);
}

// one pixel per lane, Q float4 groups (Tp = 4Q taps) per pixel, transposed through LDS
// so each store is one coalesced 1-KB wave access (the shipped k_support's shape)
template <int Q>
__global__ __launch_bounds__(256) void k_support_expd(const uchar4 *__restrict__ img, float *__restrict__ w, int W,
                                                      int H, int T, int dir, float gamma_c, float gamma_g) {
    using f4 = float __attribute__((ext_vector_type(4)));
    __shared__ f4 stg[4][64 * Q];
    __shared__ float cd_s[kLutWidth], gd_s[2 * Q + 1];
    for (int t = threadIdx.x; t < kLutWidth; t += 256) cd_s[t] = (float)(-t) / gamma_c;  // K/asw_vsupport.cl:22
    for (int t = threadIdx.x; t <= T / 2; t += 256) gd_s[t] = (float)t / gamma_g;        // :24
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int x0 = blockIdx.x * 64;
    const int y = blockIdx.y * 4 + wv;
    if (y >= H) return;
    const int x = min(x0 + lane, W - 1);
    const int R = T / 2;
    const uchar4 a = img[y * W + x];
    uchar4 b[4 * Q];
#pragma unroll
    for (int k = 0; k < 4 * Q; ++k) {
        const int qx = dir == 0 ? x : clampi(x + k - R, 0, W - 1);
        const int qy = dir == 0 ? clampi(y + k - R, 0, H - 1) : y;
        b[k] = img[qy * W + qx];
    }
    f4 v[Q];
#pragma unroll
    for (int k = 0; k < 4 * Q; ++k) {
        int dist;
        if (dir == 0) {
            const int qy = clampi(y + k - R, 0, H - 1);
            dist = y > qy ? y - qy : qy - y;
        } else {
            const int qx = clampi(x + k - R, 0, W - 1);
            dist = x > qx ? x - qx : qx - x;
        }
        const int sad = abs((int)a.x - (int)b[k].x) + abs((int)a.y - (int)b[k].y) + abs((int)a.z - (int)b[k].z);
        v[k / 4][k % 4] = k < T ? (float)exp_d((double)(cd_s[sad] - gd_s[dist])) : 0.0f;
    }
    f4 *st = stg[wv];
#pragma unroll
    for (int g = 0; g < Q; ++g) st[lane * Q + g] = v[g];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int nval = min(64, W - x0) * Q;
    f4 *out = reinterpret_cast<f4 *>(w + ((long long)y * W + x0) * (4 * Q));
#pragma unroll
    for (int g = 0; g < Q; ++g) {
        const int e = g * 64 + lane;
        if (e < nval) out[e] = st[e];
    }
}

// ---- the wave-per-pixel asw_WTA: top-2 states combined by shuffles ----
struct Top2 {
    float m1, m2;
    int idx;
};
constexpr float kInit = 100000.0f;  // K/asw_wta.cl:25-26

__device__ __forceinline__ void top2_update(Top2 &s, float t, int d) {
    s.m2 = t < s.m2 ? t : s.m2;
    s.idx = t < s.m1 ? d : s.idx;
    s.m2 = t < s.m1 ? s.m1 : s.m2;
    s.m1 = t < s.m1 ? t : s.m1;
}

// partial states over disjoint index sets combine exactly: m1 = lexicographic min of
// (value, index); m2 = min(max(m1a, m1b), m2a, m2b)
__device__ __forceinline__ void top2_combine(Top2 &a, float om1, float om2, int oidx) {
    const float nm2 = fminf(fmaxf(a.m1, om1), fminf(a.m2, om2));
    const bool take = (om1 < a.m1) || (om1 == a.m1 && oidx < a.idx);
    a.m1 = take ? om1 : a.m1;
    a.idx = take ? oidx : a.idx;
    a.m2 = nm2;
}

__device__ __forceinline__ void top2_wave_reduce(Top2 &s) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const float om1 = __shfl_xor(s.m1, off, 64);
        const float om2 = __shfl_xor(s.m2, off, 64);
        const int oidx = __shfl_xor(s.idx, off, 64);
        top2_combine(s, om1, om2, oidx);
    }
}

__global__ __launch_bounds__(256) void k_wta_wave(const float *__restrict__ cost, int W, int H, int Dp, int D,
                                                  int bpx, int32_t *__restrict__ d_ref, float *__restrict__ conf_ref,
                                                  int32_t *__restrict__ d_tar, float *__restrict__ conf_tar) {
    const int lane = threadIdx.x & 63;
    const int xcd = blockIdx.x & 7, m = blockIdx.x >> 3;
    const long long p = ((long long)xcd * bpx + m) * 4 + (threadIdx.x >> 6);
    if (p >= (long long)W * H) return;
    const int x = (int)(p % W), y = (int)(p / W);
    const float *cp = cost + p * Dp;
    Top2 s{kInit, kInit, INT_MAX};
    for (int d = lane; d < D; d += 64) top2_update(s, cp[d], d);
    top2_wave_reduce(s);
    const int md = s.idx == INT_MAX ? 0 : s.idx;
    // target scan (K/asw_wta.cl:50-67): i < md, xq = max(0, x-i), b = md + xq - x
    Top2 t{kInit, kInit, INT_MAX};
    for (int i = lane; i < md; i += 64) {
        const int xq = x - i < 0 ? 0 : x - i;
        top2_update(t, cost[((long long)y * W + xq) * Dp + (md + xq - x)], i);
    }
    top2_wave_reduce(t);
    if (lane == 0) {
        const int mdr = t.idx == INT_MAX ? md : md + (x - t.idx < 0 ? 0 : x - t.idx) - x;
        d_ref[p] = md;
        conf_ref[p] = (s.m2 - s.m1) / s.m2;
        d_tar[p] = mdr;
        conf_tar[p] = (t.m2 - t.m1) / t.m2;
    }
}

}  // namespace

extern "C" {

// w: [H][W][Tp] float32 (Tp = 4Q, Q = 9 for T 33/35, 13 for T 51), img: RGBA8 [H][W]
int forms_support_expd(const void *img, float *w, int W, int H, int T, int dir, float gamma_c, float gamma_g,
                       void *stream) {
    const dim3 grid((unsigned)((W + 63) / 64), (unsigned)((H + 3) / 4));
    const uchar4 *im = static_cast<const uchar4 *>(img);
    if (T == 33 || T == 35)
        hipLaunchKernelGGL(k_support_expd<9>, grid, dim3(256), 0, (hipStream_t)stream, im, w, W, H, T, dir, gamma_c,
                           gamma_g);
    else if (T == 51)
        hipLaunchKernelGGL(k_support_expd<13>, grid, dim3(256), 0, (hipStream_t)stream, im, w, W, H, T, dir, gamma_c,
                           gamma_g);
    else
        return -4;
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// cost: [H][W][Dp] float32, the whole range D
int forms_wta_wave(const float *cost, int W, int H, int Dp, int D, int32_t *d_ref, float *conf_ref, int32_t *d_tar,
                   float *conf_tar, void *stream) {
    const long long n = (long long)W * H;
    const int bpx = (int)(((n + 3) / 4 + 7) / 8);
    hipLaunchKernelGGL(k_wta_wave, dim3((unsigned)(8 * bpx)), dim3(256), 0, (hipStream_t)stream, cost, W, H, Dp, D,
                       bpx, d_ref, conf_ref, d_tar, conf_tar);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // extern "C"
