// asw_kernels.hip — hand-written gfx950 (CDNA4) kernels of the ASW stereo hot path
// and the STAGE half of the C-ABI declared in include/asw.h.
//
// Every kernel restates one reference OpenCL kernel (file:line in its comment)
// with the same arithmetic, re-laid-out for MI355X:
//   * cost volumes are PIXEL-major [H][W][Dp] (d fastest): a wave's 64 lanes are
//     64 consecutive disparities of one pixel, so every cost load/store is one
//     coalesced 256-byte access;
//   * in an aggregation pass the left-image support weight of a tap is the same
//     for the whole wave (one pixel) and comes from scalar loads (SGPR operand),
//     while the right-image weight (column x-d differs per lane) is staged
//     through LDS and read with ds_read_b128 (4 taps per read);
//   * the 1-D cost window lives in VGPRs and rotates: each step loads ONE new
//     cost element per lane and emits one output (no re-reads of the window).
// FP policy (DESIGN.md §FP policy): per tap ww = wl*wr; num = fma(ww, c, num);
// den = den + ww; taps in order i = 0..T-1; IEEE division num/den.
// Compiled with -ffp-contract=off so the compiler adds no other contraction.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "asw_common.h"
#include "asw_srgb_table.h"

namespace asw {

static thread_local int g_last_hip_error = 0;
void set_hip_error(hipError_t e) { g_last_hip_error = (int)e; }

namespace {

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// ---------------------------------------------------------------------------
// Support-weight table.  w(sad, dist) = exp((-sad)/gamma_c - dist/gamma_g)
// (K/asw_vsupport.cl:22-25): the weight depends only on the integer SAD and the
// integer tap distance, so it is tabulated once per context.  exp is computed in
// double with a fixed Cody-Waite + degree-14 Horner sequence and rounded to
// float: correctly rounded on this domain (checked exhaustively against the
// oracle by tests/test_gpu_parity.py::test_support_lut_exhaustive).
// ---------------------------------------------------------------------------
__device__ double exp_d(double x) {
    const double inv_ln2 = 1.44269504088896338700e+00;
    const double ln2_hi = 6.93147180369123816490e-01;
    const double ln2_lo = 1.90821492927058770002e-10;
    const double k = rint(x * inv_ln2);
    double r = fma(-k, ln2_hi, x);
    r = fma(-k, ln2_lo, r);
    double p = 1.0 / 87178291200.0;  // 1/14!
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

__global__ void k_support_lut(float *lut, int rows, float gamma_c, float gamma_g) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= rows * kLutWidth) return;
    const int dist = t / kLutWidth, sad = t % kLutWidth;
    const float c_diff = (float)(-sad) / gamma_c;  // (-1)*(sum)/30.91f
    const float g_dist = (float)dist / gamma_g;    // distance(p,q)/28.21f
    const float arg = c_diff - g_dist;
    lut[t] = (float)exp_d((double)arg);
}

// ---------------------------------------------------------------------------
// asw_Aggr (K/asw_aggr.cl:3-23): per-disparity absolute-difference cost.
// Block = 4 waves on row blockIdx.y, 4*PPW consecutive pixels; the right-image
// pixels they reach (columns x - d) are staged once in LDS, so each lane's four
// planes d = 4q..4q+3 read LDS instead of four gathers; the wave's 16 left pixels
// are one load.  The cost |dR|+|dG|+|dB| of 8-bit channels is an integer below 766,
// so the reference's float sum of three fabs equals v_sad_u8 of the alpha-cleared
// pixels exactly (one instruction instead of six conversions, three subtractions and
// two adds).  Every store is a float4 per lane (1 KB per wave-instruction).
// U16 (asw_raw_cost16): the same costs as uint16 (an integer AD <= 765, or its
// truncation at an integral tau), a 4 x uint16 store per lane: half the bytes.
// ---------------------------------------------------------------------------
constexpr int kRawPPW = 16;                       // pixels per wave
constexpr int kRawSpan = 4 * kRawPPW;              // pixels per block
template <bool U16>
__global__ __launch_bounds__(256) void k_raw_cost(const uchar4 *__restrict__ L, const uchar4 *__restrict__ R,
                                                   void *__restrict__ cost_v, int W, int Dp, int nloc, int d_begin,
                                                   float tau) {
    using f4 = float __attribute__((ext_vector_type(4)));
    using u4 = unsigned short __attribute__((ext_vector_type(4)));
    // R[y][xr], xr in [xlo, x0 + kRawSpan), in 4 phases: element t at (t & 3) * s4 +
    // (t >> 2).  The lanes of a read are 4 elements apart (planes 4q..4q+3 of lane q),
    // so they read consecutive dwords of one phase (a linear row: 4-way conflicts), and
    // s4 = 8 (mod 32) spreads the staging writes of 32 consecutive t over 32 banks.
    extern __shared__ unsigned rrow[];
    const int s4 = ((kRawSpan + Dp - 1 + 3) / 4 + 31) / 32 * 32 + 8;
    auto slot = [s4](int t) __attribute__((always_inline)) { return (t & 3) * s4 + (t >> 2); };
    const int y = blockIdx.y;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const unsigned *Lrow = reinterpret_cast<const unsigned *>(L + (long long)y * W);
    const unsigned *Rrow = reinterpret_cast<const unsigned *>(R + (long long)y * W);
    const int x0 = blockIdx.x * kRawSpan;
    const int xlo = x0 - (d_begin + Dp - 1);  // smallest x - d of the block (staged clamped to [0, W-1])
    const int nr = kRawSpan + Dp - 1;
    // (alpha cleared: v_sad_u8 then sums |dR| + |dG| + |dB|)
    for (int t = threadIdx.x; t < nr; t += 256) {
        const int xr = xlo + t;
        rrow[slot(t)] = Rrow[xr < 0 ? 0 : (xr >= W ? W - 1 : xr)] & 0xFFFFFFu;
    }
    const int xa = x0 + wave * kRawPPW;
    const int xb = min(xa + kRawPPW, W);
    // the wave's 16 left pixels in one load (lane i: pixel xa + i), each taken by the
    // lanes that need it through a lane permute
    const unsigned lw = Lrow[min(xa + (lane & (kRawPPW - 1)), W - 1)] & 0xFFFFFFu;
    // an integral tau below 765 clamps the integer cost (the uint16 form's domain,
    // raw16_exact); the float form clamps the exact float sum, as fminf(sum, tau)
    const unsigned tau_u = tau >= 765.0f ? 765u : (unsigned)tau;
    __syncthreads();
    const int nq = Dp >> 2;
    // Dp < 256 (narrow shards): 64/nq pixels per wave iteration, so no lane idles
    const int ppi = (nq < 64 && 64 % nq == 0) ? 64 / nq : 1;
    const int lpp = ppi > 1 ? nq : 64;  // lanes per pixel
    // (a uniform trip count: the permute reads lanes that must all be active; Dp is 32
    // or a multiple of 64, so ppi <= 8 divides kRawPPW)
    for (int it = 0; it < kRawPPW / ppi; ++it) {
        const int x = xa + lane / lpp + it * ppi;
        const unsigned l = (unsigned)__shfl((int)lw, min(x - xa, kRawPPW - 1));
        if (x >= xb) continue;
        const long long e0 = ((long long)y * W + x) * Dp;  // first element of pixel x
        for (int q = lane % lpp; q < nq; q += lpp) {
            unsigned c[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int k = 4 * q + j;
                const unsigned r = rrow[slot(x - (d_begin + k) - xlo)];  // = R(max(x-d, 0), y): the stage clamps
                c[j] = k < nloc ? __builtin_amdgcn_sad_u8(l, r, 0u) : 0u;  // exact integer AD, <= 765
            }
            if constexpr (U16) {
                u4 h;
#pragma unroll
                for (int j = 0; j < 4; ++j) h[j] = (unsigned short)min(c[j], tau_u);
                __builtin_nontemporal_store(h, &reinterpret_cast<u4 *>(static_cast<unsigned short *>(cost_v) + e0)[q]);
            } else {
                f4 v;
#pragma unroll
                for (int j = 0; j < 4; ++j) v[j] = 4 * q + j < nloc ? fminf((float)c[j], tau) : 0.0f;
                __builtin_nontemporal_store(v, &reinterpret_cast<f4 *>(static_cast<float *>(cost_v) + e0)[q]);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// asw_vSupport / asw_hSupport (K/asw_vsupport.cl:3-27, K/asw_hsupport.cl:3-28).
// w[y][x][i] = LUT[|delta|][SAD(p,q)], q the i-th tap of p's 1-D window.
// One thread = one pixel, lanes = 64 consecutive x of one row: the neighbour of
// tap i is one coalesced 256-B load per wave (V: row y+i-R; H: the row shifted by
// i-R), the LUT row of tap i is one dist (except at clamped edges), so its gather
// stays inside 3 KB of L1.  All Q groups of a pixel are computed before its Q
// float4 stores (the loads of every tap in flight together); blockIdx.z selects one
// of up to four (image, direction) jobs, so the four arrays of a frame are one
// launch.  (Round 2's float4-per-thread form: 0.67 ms at C4.)
// ---------------------------------------------------------------------------
struct SupportJobs {
    const uchar4 *img[4];
    float *w[4];
    int dir[4];
};
// (Round 4's EXPD form, each weight's exp computed instead of gathered, measured
// slower and moved to tools/exp/exp_forms.hip.)
template <int Q>
__global__ __launch_bounds__(256) void k_support(SupportJobs jobs, const float *__restrict__ lut, int W, int H,
                                                 int T) {
    using f4 = float __attribute__((ext_vector_type(4)));
    // 4 waves x 64 pixels x Q float4 = 4 KiB per Q: Q = 17 (T 65-68) takes 68 KiB,
    // which only the 160 KiB LDS of gfx950 holds (the build targets gfx950 only)
    static_assert(4 * 64 * Q * 16 <= 160 * 1024, "k_support staging tile exceeds the gfx950 LDS");
    __shared__ f4 stg[4][64 * Q];  // per wave: its 64 pixels' Q float4, in output order
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int x0 = blockIdx.x * 64;
    const int y0 = blockIdx.y * 4;
    const int y = y0 + wv;
    const bool live = y < H;  // (a wave past the bottom row still loads and syncs, stores nothing)
    const int x = min(x0 + lane, W - 1);  // lanes past the right edge recompute column W-1, not stored
    const unsigned *__restrict__ img = reinterpret_cast<const unsigned *>(jobs.img[blockIdx.z]);
    const int dir = jobs.dir[blockIdx.z];
    const int R = T / 2;
    // The block's image window, loaded once into LDS (aliasing the staging tile, which
    // is written only after every wave has read its neighbours): V rows y0-R .. y0+3+R of
    // its 64 columns, [4Q+3][64]; H columns x0-R .. x0+63+R of its 4 rows, [4][64+4Q-1].
    // About 10 (V) or 2 (H) coalesced loads per thread instead of 4Q neighbour loads per
    // lane: the vector-memory pipe is left to the 4Q LUT gathers and the stores.
    // (Alpha cleared: v_sad_u8 then sums |dR| + |dG| + |dB|, the reference's exact integer.)
    unsigned *win = reinterpret_cast<unsigned *>(&stg[0][0]);
    constexpr int NV = (4 * Q + 3) * 64, HW = 64 + 4 * Q - 1, NH = 4 * HW;
    static_assert(NV <= 4 * 64 * 4 * Q && NH <= 4 * 64 * 4 * Q, "window inside the staging tile");
    if (dir == ASW_DIR_V) {
        for (int t = threadIdx.x; t < NV; t += 256)
            win[t] = img[clampi(y0 - R + (t >> 6), 0, H - 1) * W + min(x0 + (t & 63), W - 1)] & 0xFFFFFFu;
    } else {
        for (int t = threadIdx.x; t < NH; t += 256) {
            const int r = t / HW, c = t - r * HW;
            win[t] = img[min(y0 + r, H - 1) * W + clampi(x0 - R + c, 0, W - 1)] & 0xFFFFFFu;
        }
    }
    __syncthreads();
    // centre (x, y) and tap k of this lane: V window row wv + k, H window column lane + k
    const int wbase = dir == ASW_DIR_V ? wv * 64 + lane : wv * HW + lane;
    const int wstep = dir == ASW_DIR_V ? 64 : 1;
    const unsigned a = win[wbase + R * wstep];
    {
        constexpr int NG = Q;
        unsigned b[4 * NG];
#pragma unroll
        for (int k = 0; k < 4 * NG; ++k) b[k] = win[wbase + k * wstep];
        __syncthreads();  // every wave holds its neighbours: the tile is the staging tile again
        if (!live) return;
        f4 v[NG];
#pragma unroll
        for (int k = 0; k < 4 * NG; ++k) {
            int dist;
            if (dir == ASW_DIR_V) {
                const int qy = clampi(y + k - R, 0, H - 1);
                dist = y > qy ? y - qy : qy - y;
            } else {
                const int qx = clampi(x + k - R, 0, W - 1);
                dist = x > qx ? x - qx : qx - x;
            }
            const int sad = (int)__builtin_amdgcn_sad_u8(a, b[k], 0u);
            v[k / 4][k % 4] = k < T ? lut[dist * kLutWidth + sad] : 0.0f;
        }
        // The wave's 64 pixels are one contiguous 64*Q-float4 run of the output:
        // transposed through LDS (Q odd: the 144-B lane stride of the writes is
        // bank-conflict-free), every store is then one coalesced 1-KB wave access
        // instead of 64 float4 at a 16Q-byte stride.
        f4 *st = stg[wv];
#pragma unroll
        for (int g = 0; g < NG; ++g) st[lane * Q + g] = v[g];
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int nval = min(64, W - x0) * Q;
        f4 *out = reinterpret_cast<f4 *>(jobs.w[blockIdx.z] + ((long long)y * W + x0) * (4 * Q));
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            const int e = g * 64 + lane;
            if (e < nval) __builtin_nontemporal_store(st[e], &out[e]);  // (nt: write-once stream)
        }
    }
}

// any tap count (Q past the unrolled forms): one float4 group per thread
__global__ __launch_bounds__(256) void k_support_any(SupportJobs jobs, const float *__restrict__ lut, int W, int H,
                                                 int T, int Tp) {
    using f4 = float __attribute__((ext_vector_type(4)));
    const int y = blockIdx.y;
    const int Q = Tp >> 2;
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= W * Q) return;
    const int x = t / Q, q = t - x * Q;
    const uchar4 *__restrict__ img = jobs.img[blockIdx.z];
    const int dir = jobs.dir[blockIdx.z];
    const int R = T / 2;
    const uchar4 a = img[y * W + x];
    f4 v;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int i = 4 * q + j;
        int qx = x, qy = y, dist;
        if (dir == ASW_DIR_V) {
            qy = clampi(y + i - R, 0, H - 1);
            dist = y > qy ? y - qy : qy - y;
        } else {
            qx = clampi(x + i - R, 0, W - 1);
            dist = x > qx ? x - qx : qx - x;
        }
        const uchar4 b = img[qy * W + qx];
        const int sad = abs((int)a.x - (int)b.x) + abs((int)a.y - (int)b.y) + abs((int)a.z - (int)b.z);
        v[j] = i < T ? lut[dist * kLutWidth + sad] : 0.0f;
    }
    reinterpret_cast<f4 *>(jobs.w[blockIdx.z] + (long long)y * W * Tp)[t] = v;
}

template <int Q>
void launch_support_q(const asw_params *p, const SupportJobs &jobs, int njobs, const float *lut,
                             hipStream_t st) {
    const dim3 grid((unsigned)((p->width + 63) / 64), (unsigned)((p->height + 3) / 4), (unsigned)njobs);
    hipLaunchKernelGGL((k_support<Q>), grid, dim3(256), 0, st, jobs, lut, p->width, p->height, p->taps);
}

// ---------------------------------------------------------------------------
// CIELab extension (north star, no reference counterpart).
// sRGB (D65) 8-bit -> L*a*b*: linear light from the generated table
// (asw_srgb_table.h), the IEC 61966-2-1 matrix, white (0.95047, 1, 1.08883),
// f(t) = cbrt(t) above (6/29)^3 else (kappa t + 16)/116.  A fixed sequence of
// IEEE double operations (the cube root is 12 Newton steps from 1.0, no libm),
// compiled with -ffp-contract=off: identical to oracle_lab bit for bit.
// ---------------------------------------------------------------------------
__device__ double cbrt_newton(double t) {
    double y = 1.0;
#pragma unroll 1
    for (int k = 0; k < 12; ++k) y = (2.0 * y + t / (y * y)) / 3.0;
    return y;
}

__device__ double lab_f(double t) {
    const double eps = 216.0 / 24389.0, kappa = 24389.0 / 27.0;
    return t > eps ? cbrt_newton(t) : (kappa * t + 16.0) / 116.0;
}

__global__ void k_lab(const uchar4 *__restrict__ img, float4 *__restrict__ lab, long long n) {
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uchar4 c = img[p];
    const double r = kSrgbLinear[c.x], g = kSrgbLinear[c.y], b = kSrgbLinear[c.z];
    const double X = (0.4124564 * r + 0.3575761 * g) + 0.1804375 * b;
    const double Y = (0.2126729 * r + 0.7151522 * g) + 0.0721750 * b;
    const double Z = (0.0193339 * r + 0.1191920 * g) + 0.9503041 * b;
    const double fx = lab_f(X / 0.95047), fy = lab_f(Y / 1.0), fz = lab_f(Z / 1.08883);
    lab[p] = make_float4((float)(116.0 * fy - 16.0), (float)(500.0 * (fx - fy)), (float)(200.0 * (fy - fz)), 0.0f);
}

// Support weights with the colour term on CIELab: the formula of
// K/asw_vsupport.cl:19-25 with the RGB SAD replaced by the Euclidean distance
// dc = sqrt((dL^2 + da^2) + db^2) (float sums; the double sqrt rounded to float
// is the correctly rounded float sqrt), exp as exp_d.
__global__ __launch_bounds__(256) void k_support_lab(const float4 *__restrict__ lab, float *__restrict__ w, int W,
                                                     int H, int T, int Tp, int dir, float gamma_c, float gamma_g) {
    const int y = blockIdx.y;
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= W * Tp) return;
    const int x = t / Tp, i = t - x * Tp;
    const int R = T / 2;
    float v = 0.0f;
    if (i < T) {
        int qx = x, qy = y, dist;
        if (dir == ASW_DIR_V) {
            qy = clampi(y + i - R, 0, H - 1);
            dist = y > qy ? y - qy : qy - y;
        } else {
            qx = clampi(x + i - R, 0, W - 1);
            dist = x > qx ? x - qx : qx - x;
        }
        const float4 a = lab[y * W + x];
        const float4 b = lab[qy * W + qx];
        const float dL = a.x - b.x, da = a.y - b.y, db = a.z - b.z;
        float s2 = dL * dL + da * da;
        s2 = s2 + db * db;
        const float dc = (float)sqrt((double)s2);
        const float c_diff = (-dc) / gamma_c;
        const float g_dist = (float)dist / gamma_g;
        v = (float)exp_d((double)(c_diff - g_dist));
    }
    w[(long long)y * W * Tp + t] = v;
}

// ---------------------------------------------------------------------------
// WTA: first minimum m1 (index idx) and the second smallest m2 of the multiset,
// strict '<' in scan order (K/asw_wta.cl:43-46); the scans are lane-per-pixel
// (asw_refine.hip).  (The wave-per-pixel WTA kernels of round 1, which combined
// partial states by shuffles, are in tools/exp/exp_forms.hip.)
// ---------------------------------------------------------------------------
constexpr float kInit = 100000.0f;  // K/asw_wta.cl:25-26

constexpr long long kNoKey = 0x7fffffffffffffffLL;

// second-smallest contribution: the shard that owns the global minimum offers
// its own second smallest, every other shard its minimum.
__global__ void k_wta_second(long long n, const long long *__restrict__ key_global,
                             const long long *__restrict__ key_local, const float *__restrict__ m1,
                             const float *__restrict__ m2, float *__restrict__ contrib) {
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    contrib[p] = key_local[p] == key_global[p] ? m2[p] : m1[p];
}

__global__ void k_wta_finalize(int W, int H, int D, const long long *__restrict__ key, const float *__restrict__ m2,
                               const long long *__restrict__ tkey, const float *__restrict__ t2,
                               int32_t *__restrict__ d_ref, float *__restrict__ conf_ref,
                               int32_t *__restrict__ d_tar, float *__restrict__ conf_tar,
                               uint8_t *__restrict__ code_ref, uint8_t *__restrict__ code_tar) {
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= (long long)W * H) return;
    const int x = (int)(p % W);
    const long long k = key[p], tk = tkey[p];
    const int md = k == kNoKey ? 0 : (int)(unsigned)(k & 0xffffffffLL);
    const float m1 = k == kNoKey ? kInit : __uint_as_float((unsigned)((unsigned long long)k >> 32));
    int mdr = md;
    float tm1 = kInit;
    if (tk != kNoKey) {
        const int i = (int)(unsigned)(tk & 0xffffffffLL);
        mdr = md + (x - i < 0 ? 0 : x - i) - x;
        tm1 = __uint_as_float((unsigned)((unsigned long long)tk >> 32));
    }
    d_ref[p] = md;
    conf_ref[p] = (m2[p] - m1) / m2[p];
    d_tar[p] = mdr;
    conf_tar[p] = (t2[p] - tm1) / t2[p];
    if (code_ref) code_ref[p] = (uint8_t)code_u8(md, D);
    if (code_tar) code_tar[p] = (uint8_t)code_u8(mdr, D);
}

// asw_WTA_REF finalize (K/asw_wta_ref.cl:59-68): indices and codes as asw_WTA; the
// kernel's `confidence` receives the left and then the TARGET confidence, so conf_ref
// = the target confidence and the left second minimum is not needed.
__global__ void k_wta_ref_finalize(int W, int H, int D, const long long *__restrict__ key,
                                   const long long *__restrict__ tkey, const float *__restrict__ t2,
                                   int32_t *__restrict__ d_ref, int32_t *__restrict__ d_tar,
                                   float *__restrict__ conf_ref, uint8_t *__restrict__ code_ref,
                                   uint8_t *__restrict__ code_tar) {
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= (long long)W * H) return;
    const int x = (int)(p % W);
    const long long k = key[p], tk = tkey[p];
    const int md = k == kNoKey ? 0 : (int)(unsigned)(k & 0xffffffffLL);
    int mdr = md;
    float tm1 = kInit;
    if (tk != kNoKey) {
        const int i = (int)(unsigned)(tk & 0xffffffffLL);
        mdr = md + (x - i < 0 ? 0 : x - i) - x;
        tm1 = __uint_as_float((unsigned)((unsigned long long)tk >> 32));
    }
    d_ref[p] = md;
    d_tar[p] = mdr;
    conf_ref[p] = (t2[p] - tm1) / t2[p];
    if (code_ref) code_ref[p] = (uint8_t)code_u8(md, D);
    if (code_tar) code_tar[p] = (uint8_t)code_u8(mdr, D);
}

// Constistency (K/consist.cl:3-34).  The reference reads its 8-bit disparity
// images back as q = (code/255)*60 and calls a pixel consistent iff
// |q_tar - q_ref| < 1.001f; writing q/60 back to UNORM8 returns the code.
__global__ void k_consistency(long long n, int D, int mode, const int32_t *__restrict__ d_ref,
                              const int32_t *__restrict__ d_tar, const uint8_t *__restrict__ code_ref,
                              const uint8_t *__restrict__ code_tar, float *__restrict__ conf_ref,
                              float *__restrict__ conf_tar, uchar4 *__restrict__ out,
                              uchar4 *__restrict__ out_red) {
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint8_t cr = code_ref[p], ct = code_tar[p];
    bool cons;
    if (mode == ASW_LR_U8) {
        const float scale = (float)(D - 1);
        const float qr = ((float)cr / 255.0f) * scale;
        const float qt = ((float)ct / 255.0f) * scale;
        cons = fabsf(qt - qr) < 1.001f;
    } else {
        const int dd = d_ref[p] - d_tar[p];
        cons = dd <= 1 && dd >= -1;
    }
    if (!cons) {
        conf_ref[p] = 0.0f;
        conf_tar[p] = 0.0f;
    }
    if (out) out[p] = cons ? make_uchar4(cr, cr, cr, 255) : make_uchar4(ct, ct, ct, 255);
    if (out_red) out_red[p] = cons ? make_uchar4(cr, cr, cr, 255) : make_uchar4(255, 0, 0, 255);
}

// ---------------------------------------------------------------------------
// launch helpers
// ---------------------------------------------------------------------------
inline int finish_launch() {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_hip_error(e);
        return ASW_E_HIP;
    }
    return ASW_OK;
}


}  // namespace
}  // namespace asw

using namespace asw;

// ===========================================================================
// C-ABI: parameters and layout
// ===========================================================================
namespace asw {
// asw_wta_sweep.hip: asw_WTA as a row sweep (ASW_E_UNSUPPORTED for pitches it is not built for)
int launch_wta_sweep(const asw_params *p, const float *cost, int32_t *d_ref, float *conf_ref, int32_t *d_tar,
                     float *conf_tar, uint8_t *code_ref, uint8_t *code_tar, hipStream_t st);
}  // namespace asw

extern "C" {

// 2: asw_outputs gained disp16 / lr16 and asw_timings gained exchange (round 2);
// asw_create rejects shapes the pass kernels cannot address (ASW_E_UNSUPPORTED)
// 3: asw_params.flags (round 5)
// 4: the measured-negative forms and their flags removed (round 6)
int asw_abi_version(void) { return ASW_ABI_VERSION; }

// 0: lane-per-pixel scans (default), 2: asw_WTA by the row sweep (asw_wta_sweep.hip;
// the sharded halves keep the lane-per-pixel scans).  1 (round 1's wave per pixel) is
// no longer built (tools/exp/exp_forms.hip)
static int g_wta_variant = 0;

int asw_tune_set(int key, int value) {
    if (key == ASW_TUNE_PASS_VARIANT) {
        // only bits that select a compiled form (launch_dm): a stale bit would time the
        // default kernel under another name
        // (+ bits 16-23: strip / segment counts, and bit 26: the nt policy flip of the
        // 32-plane shard passes, asw_pass32.h)
        if (value & ~(asw::kPassVariantBits | 0xFF0000 | (1 << 26))) return ASW_E_INVALID;
        return asw::set_pass_variant(value);
    }
    if (key == ASW_TUNE_WTA_VARIANT) {
        if (value != 0 && value != 2) return ASW_E_INVALID;
        const int old = g_wta_variant;
        g_wta_variant = value;
        return old;
    }
    return ASW_E_INVALID;
}

void asw_params_default(asw_params *p) {
    if (!p) return;
    p->width = 0;
    p->height = 0;
    p->ndisp = 61;
    p->taps = 33;
    p->iters = 7;
    p->gamma_c = 30.91f;
    p->gamma_g = 28.21f;
    p->color_space = ASW_COLOR_RGB;
    p->tad_tau = 765.0f;
    p->lr_check = 1;
    p->lr_mode = ASW_LR_U8;
    p->d_begin = 0;
    p->d_end = -1;  // -1: = ndisp
    p->flags = 0;
}

static inline int d_end_of(const asw_params *p) { return p->d_end < 0 ? p->ndisp : p->d_end; }

int asw_params_check(const asw_params *p) {
    if (!p) return ASW_E_INVALID;
    if (p->width < 1 || p->height < 1 || p->ndisp < 1 || p->taps < 1 || (p->taps & 1) == 0) return ASW_E_INVALID;
    if (p->iters < 0 || !(p->gamma_c > 0.0f) || !(p->gamma_g > 0.0f)) return ASW_E_INVALID;
    if (p->d_begin < 0 || d_end_of(p) > p->ndisp || p->d_begin >= d_end_of(p)) return ASW_E_INVALID;
    if (p->color_space != ASW_COLOR_RGB && p->color_space != ASW_COLOR_LAB) return ASW_E_INVALID;
    if (p->lr_mode != ASW_LR_U8 && p->lr_mode != ASW_LR_NATIVE) return ASW_E_INVALID;
    if ((long long)p->width * p->height > (1LL << 31) / 64) return ASW_E_INVALID;
    if (p->flags & ~ASW_FLAG_ALL) return ASW_E_INVALID;
    return ASW_OK;
}

const char *asw_strerror(int s) {
    switch (s) {
        case ASW_OK: return "ok";
        case ASW_E_INVALID: return "invalid parameter";
        case ASW_E_HIP: return "HIP runtime error";
        case ASW_E_NOMEM: return "out of memory";
        case ASW_E_UNSUPPORTED: return "unsupported parameter combination";
        case ASW_E_COMM: return "collective (RCCL) error";
        default: return "unknown status";
    }
}

int asw_last_hip_error(void) { return g_last_hip_error; }

int asw_disp_pitch(const asw_params *p) {
    const int n = d_end_of(p) - p->d_begin;
    // a d-shard of at most 32 planes (the C4 frame over 8 GPUs): pitch 32, the
    // half-wave passes of asw_pass32.h; otherwise whole 64-plane blocks
    if (n <= 32 && (p->d_begin > 0 || d_end_of(p) < p->ndisp)) return 32;
    return round_up(n, 64);
}
int asw_tap_pitch(const asw_params *p) { return tap_pitch(p->taps); }
size_t asw_cost_bytes(const asw_params *p) {
    return (size_t)p->width * p->height * (size_t)asw_disp_pitch(p) * sizeof(float);
}
size_t asw_support_bytes(const asw_params *p) {
    return (size_t)p->width * p->height * (size_t)asw_tap_pitch(p) * sizeof(float);
}
size_t asw_lab_bytes(const asw_params *p) { return p ? (size_t)p->width * p->height * 16 : 0; }

size_t asw_lut_bytes(const asw_params *p) { return (size_t)(p->taps / 2 + 1) * kLutWidth * sizeof(float); }

// ===========================================================================
// C-ABI: stage API
// ===========================================================================
#define ASW_CHECK_PARAMS(p)                  \
    do {                                     \
        const int _s = asw_params_check(p);  \
        if (_s != ASW_OK) return _s;         \
    } while (0)

static int launch_raw_cost(bool u16, const asw_params *p, const uint8_t *left, const uint8_t *right, void *cost,
                           void *stream) {
    const int Dp = asw_disp_pitch(p);
    const dim3 grid((unsigned)((p->width + kRawSpan - 1) / kRawSpan), (unsigned)p->height);
    const size_t lds = (size_t)4 * (((kRawSpan + Dp - 1 + 3) / 4 + 31) / 32 * 32 + 8) * 4;  // 4 phases of s4
    if (lds > 64 * 1024) return ASW_E_UNSUPPORTED;
    const uchar4 *l = reinterpret_cast<const uchar4 *>(left), *r = reinterpret_cast<const uchar4 *>(right);
    if (u16)
        hipLaunchKernelGGL(k_raw_cost<true>, grid, dim3(256), lds, (hipStream_t)stream, l, r, cost, p->width, Dp,
                           d_end_of(p) - p->d_begin, p->d_begin, p->tad_tau);
    else
        hipLaunchKernelGGL(k_raw_cost<false>, grid, dim3(256), lds, (hipStream_t)stream, l, r, cost, p->width, Dp,
                           d_end_of(p) - p->d_begin, p->d_begin, p->tad_tau);
    return finish_launch();
}

int asw_raw_cost(const asw_params *p, const uint8_t *left, const uint8_t *right, float *cost, void *stream) {
    ASW_CHECK_PARAMS(p);
    if (!left || !right || !cost) return ASW_E_INVALID;
    return launch_raw_cost(false, p, left, right, cost, stream);
}

// the raw costs are integers (AD <= 765) unless a non-integral tau truncates them
static bool raw16_exact(const asw_params *p) { return p->tad_tau >= 765.0f || p->tad_tau == floorf(p->tad_tau); }

int asw_raw16_supported(const asw_params *p) {
    if (!p || asw_params_check(p) != ASW_OK) return 0;
    // exact, and read by a ring-kernel first V pass (asw_aggregate_pass_den16)
    return raw16_exact(p) && p->tad_tau >= 0.0f && p->iters >= 1 && asw::ring_taps(p->taps) ? 1 : 0;
}

int asw_raw_cost16(const asw_params *p, const uint8_t *left, const uint8_t *right, uint16_t *cost, void *stream) {
    ASW_CHECK_PARAMS(p);
    if (!left || !right || !cost) return ASW_E_INVALID;
    if (!raw16_exact(p) || p->tad_tau < 0.0f) return ASW_E_UNSUPPORTED;
    return launch_raw_cost(true, p, left, right, cost, stream);
}

int asw_support_lut(const asw_params *p, float *lut, void *stream) {
    ASW_CHECK_PARAMS(p);
    if (!lut) return ASW_E_INVALID;
    const int rows = p->taps / 2 + 1;
    const int n = rows * kLutWidth;
    hipLaunchKernelGGL(k_support_lut, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, lut, rows,
                       p->gamma_c, p->gamma_g);
    return finish_launch();
}

static int launch_support(const asw_params *p, const SupportJobs &jobs, int njobs, const float *lut, void *stream) {
    const hipStream_t st = (hipStream_t)stream;
    switch (asw_tap_pitch(p) / 4) {  // Tp = 4Q, Q odd past 1 (tap_pitch)
        case 1: launch_support_q<1>(p, jobs, njobs, lut, st); break;
        case 3: launch_support_q<3>(p, jobs, njobs, lut, st); break;
        case 5: launch_support_q<5>(p, jobs, njobs, lut, st); break;
        case 7: launch_support_q<7>(p, jobs, njobs, lut, st); break;
        case 9: launch_support_q<9>(p, jobs, njobs, lut, st); break;
        case 11: launch_support_q<11>(p, jobs, njobs, lut, st); break;
        case 13: launch_support_q<13>(p, jobs, njobs, lut, st); break;
        case 15: launch_support_q<15>(p, jobs, njobs, lut, st); break;
        case 17: launch_support_q<17>(p, jobs, njobs, lut, st); break;
        default: {
            const int Tp = asw_tap_pitch(p);
            const dim3 grid((unsigned)((p->width * (Tp / 4) + 255) / 256), (unsigned)p->height, (unsigned)njobs);
            hipLaunchKernelGGL(k_support_any, grid, dim3(256), 0, st, jobs, lut, p->width, p->height, p->taps, Tp);
        }
    }
    return finish_launch();
}

int asw_support(const asw_params *p, int dir, const uint8_t *img, const float *lut, float *w, void *stream) {
    ASW_CHECK_PARAMS(p);
    if (!img || !lut || !w || (dir != ASW_DIR_V && dir != ASW_DIR_H)) return ASW_E_INVALID;
    if (p->color_space != ASW_COLOR_RGB) return ASW_E_INVALID;  // LAB contexts: asw_support_lab
    SupportJobs jobs{};
    jobs.img[0] = reinterpret_cast<const uchar4 *>(img);
    jobs.w[0] = w;
    jobs.dir[0] = dir;
    return launch_support(p, jobs, 1, lut, stream);
}

int asw_support_all(const asw_params *p, const uint8_t *left, const uint8_t *right, const float *lut, float *wvl,
                    float *whl, float *wvr, float *whr, void *stream) {
    ASW_CHECK_PARAMS(p);
    if (!left || !right || !lut || !wvl || !whl || !wvr || !whr) return ASW_E_INVALID;
    if (p->color_space != ASW_COLOR_RGB) return ASW_E_INVALID;
    SupportJobs jobs{};
    const uchar4 *img[4] = {reinterpret_cast<const uchar4 *>(left), reinterpret_cast<const uchar4 *>(left),
                            reinterpret_cast<const uchar4 *>(right), reinterpret_cast<const uchar4 *>(right)};
    float *w[4] = {wvl, whl, wvr, whr};
    for (int j = 0; j < 4; ++j) {
        jobs.img[j] = img[j];
        jobs.w[j] = w[j];
        jobs.dir[j] = (j & 1) ? ASW_DIR_H : ASW_DIR_V;
    }
    return launch_support(p, jobs, 4, lut, stream);
}

int asw_lab(const asw_params *p, const uint8_t *img, float *lab, void *stream) {
    ASW_CHECK_PARAMS(p);
    if (!img || !lab) return ASW_E_INVALID;
    const long long n = (long long)p->width * p->height;
    hipLaunchKernelGGL(k_lab, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const uchar4 *>(img), reinterpret_cast<float4 *>(lab), n);
    return finish_launch();
}

int asw_support_lab(const asw_params *p, int dir, const float *lab, float *w, void *stream) {
    ASW_CHECK_PARAMS(p);
    if (!lab || !w || (dir != ASW_DIR_V && dir != ASW_DIR_H)) return ASW_E_INVALID;
    if (p->color_space != ASW_COLOR_LAB) return ASW_E_INVALID;
    const int Tp = asw_tap_pitch(p);
    const dim3 grid((unsigned)((p->width * Tp + 255) / 256), (unsigned)p->height);
    hipLaunchKernelGGL(k_support_lab, grid, dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const float4 *>(lab), w, p->width, p->height, p->taps, Tp, dir, p->gamma_c,
                       p->gamma_g);
    return finish_launch();
}

int asw_aggregate_pass(const asw_params *p, int dir, const float *wl, const float *wr, const float *cin,
                       float *cout, void *stream) {
    ASW_CHECK_PARAMS(p);
    if (!wl || !wr || !cin || !cout || cin == cout || (dir != ASW_DIR_V && dir != ASW_DIR_H))
        return ASW_E_INVALID;
    return asw::launch_pass(p, dir, wl, wr, cin, cout, nullptr, ASW_DEN_NONE, (hipStream_t)stream);
}

int asw_aggregate_pass_den(const asw_params *p, int dir, const float *wl, const float *wr, const float *cin,
                           float *cout, float *den, int den_mode, void *stream) {
    ASW_CHECK_PARAMS(p);
    if (!wl || !wr || !cin || !cout || cin == cout || (dir != ASW_DIR_V && dir != ASW_DIR_H)) return ASW_E_INVALID;
    if (den_mode < ASW_DEN_NONE || den_mode > ASW_DEN_READ) return ASW_E_INVALID;
    if (den_mode != ASW_DEN_NONE && (!den || den == cin || den == cout)) return ASW_E_INVALID;
    return asw::launch_pass(p, dir, wl, wr, cin, cout, den, den_mode, (hipStream_t)stream);
}

int asw_aggregate_pass_den16(const asw_params *p, const float *wvl, const float *wvr, const uint16_t *cin16,
                             float *cout, float *den, int den_mode, void *stream) {
    ASW_CHECK_PARAMS(p);
    if (!wvl || !wvr || !cin16 || !cout || (const void *)cin16 == (const void *)cout) return ASW_E_INVALID;
    if (den_mode != ASW_DEN_NONE && den_mode != ASW_DEN_WRITE) return ASW_E_INVALID;  // a first pass
    if (den_mode != ASW_DEN_NONE && (!den || den == cout)) return ASW_E_INVALID;
    if (!asw_raw16_supported(p)) return ASW_E_UNSUPPORTED;
    const asw::RawSrc raw{cin16};
    return asw::launch_pass(p, ASW_DIR_V, wvl, wvr, nullptr, cout, den, den_mode, (hipStream_t)stream, &raw);
}

int asw_aggregate(const asw_params *p, const float *wvl, const float *wvr, const float *whl, const float *whr,
                  float *c0, float *c1, void *stream) {
    return asw_aggregate_den(p, wvl, wvr, whl, whr, c0, c1, nullptr, nullptr, stream);
}

int asw_aggregate_den(const asw_params *p, const float *wvl, const float *wvr, const float *whl, const float *whr,
                      float *c0, float *c1, float *den_v, float *den_h, void *stream) {
    ASW_CHECK_PARAMS(p);
    const bool cached = den_v && den_h;
    for (int it = 0; it < p->iters; ++it) {
        const int dm = !cached ? ASW_DEN_NONE : (it == 0 ? ASW_DEN_WRITE : ASW_DEN_READ);
        int s = asw_aggregate_pass_den(p, ASW_DIR_V, wvl, wvr, c0, c1, den_v, dm, stream);
        if (s != ASW_OK) return s;
        s = asw_aggregate_pass_den(p, ASW_DIR_H, whl, whr, c1, c0, den_h, dm, stream);
        if (s != ASW_OK) return s;
    }
    return ASW_OK;
}

int asw_wta(const asw_params *p, const float *cost, int32_t *d_ref, float *conf_ref, int32_t *d_tar,
            float *conf_tar, uint8_t *code_ref, uint8_t *code_tar, void *stream) {
    ASW_CHECK_PARAMS(p);
    if (p->d_begin != 0 || d_end_of(p) != p->ndisp) return ASW_E_INVALID;  // sharded: use asw_wta_local & co.
    if (!cost || !d_ref || !conf_ref || !d_tar || !conf_tar) return ASW_E_INVALID;
    if (g_wta_variant == 2) {  // the row sweep (asw_wta_sweep.hip) where built for the pitch: opt-in,
        // measured 2.21 ms against the scan's 0.57 at C4 (one wave per row: latency-bound)
        const int s = asw::launch_wta_sweep(p, cost, d_ref, conf_ref, d_tar, conf_tar, code_ref, code_tar,
                                            (hipStream_t)stream);
        if (s != ASW_E_UNSUPPORTED) return s;
    }
    return asw::launch_wta_scan(p, 0, cost, nullptr, nullptr, d_ref, conf_ref, d_tar, conf_tar, code_ref, code_tar,
                                    (hipStream_t)stream);
}

int asw_wta_local(const asw_params *p, const float *cost, int64_t *key, float *m1, float *m2, void *stream) {
    ASW_CHECK_PARAMS(p);
    if (!cost || !key || !m1 || !m2) return ASW_E_INVALID;
    return asw::launch_wta_local_scan(p, cost, nullptr, reinterpret_cast<long long *>(key), m1, m2,
                                          (hipStream_t)stream);
}

int asw_wta_target_local(const asw_params *p, const float *cost, const int64_t *key_ref, int64_t *tkey, float *t1,
                         float *t2, void *stream) {
    ASW_CHECK_PARAMS(p);
    if (!cost || !key_ref || !tkey || !t1 || !t2) return ASW_E_INVALID;
    return asw::launch_wta_target_local_scan(p, cost, reinterpret_cast<const long long *>(key_ref), nullptr,
                                                 reinterpret_cast<long long *>(tkey), t1, t2, (hipStream_t)stream);
}

int asw_wta_ref_local(const asw_params *p, const float *cost, const float *ref_l, int64_t *key, float *m1, float *m2,
                      void *stream) {
    ASW_CHECK_PARAMS(p);
    if (!cost || !ref_l || !key || !m1 || !m2) return ASW_E_INVALID;
    return asw::launch_wta_local_scan(p, cost, ref_l, reinterpret_cast<long long *>(key), m1, m2,
                                          (hipStream_t)stream);
}

int asw_wta_ref_target_local(const asw_params *p, const float *cost, const float *ref_r, const int64_t *key_ref,
                             int64_t *tkey, float *t1, float *t2, void *stream) {
    ASW_CHECK_PARAMS(p);
    if (!cost || !ref_r || !key_ref || !tkey || !t1 || !t2) return ASW_E_INVALID;
    return asw::launch_wta_target_local_scan(p, cost, reinterpret_cast<const long long *>(key_ref), ref_r,
                                                 reinterpret_cast<long long *>(tkey), t1, t2, (hipStream_t)stream);
}

int asw_wta_ref_finalize(const asw_params *p, const int64_t *key, const int64_t *tkey, const float *t2,
                         int32_t *d_ref, int32_t *d_tar, float *conf_ref, uint8_t *code_ref, uint8_t *code_tar,
                         void *stream) {
    ASW_CHECK_PARAMS(p);
    if (!key || !tkey || !t2 || !d_ref || !d_tar || !conf_ref) return ASW_E_INVALID;
    const long long n = (long long)p->width * p->height;
    hipLaunchKernelGGL(k_wta_ref_finalize, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       p->width, p->height, p->ndisp, reinterpret_cast<const long long *>(key),
                       reinterpret_cast<const long long *>(tkey), t2, d_ref, d_tar, conf_ref, code_ref, code_tar);
    return finish_launch();
}

int asw_wta_second(const asw_params *p, const int64_t *key_global, const int64_t *key_local, const float *m1,
                   const float *m2, float *m2_contrib, void *stream) {
    ASW_CHECK_PARAMS(p);
    if (!key_global || !key_local || !m1 || !m2 || !m2_contrib) return ASW_E_INVALID;
    const long long n = (long long)p->width * p->height;
    hipLaunchKernelGGL(k_wta_second, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, n,
                       reinterpret_cast<const long long *>(key_global), reinterpret_cast<const long long *>(key_local),
                       m1, m2, m2_contrib);
    return finish_launch();
}

int asw_wta_finalize(const asw_params *p, const int64_t *key, const float *m2, const int64_t *tkey, const float *t2,
                     int32_t *d_ref, float *conf_ref, int32_t *d_tar, float *conf_tar, uint8_t *code_ref,
                     uint8_t *code_tar, void *stream) {
    ASW_CHECK_PARAMS(p);
    if (!key || !m2 || !tkey || !t2 || !d_ref || !conf_ref || !d_tar || !conf_tar) return ASW_E_INVALID;
    const long long n = (long long)p->width * p->height;
    hipLaunchKernelGGL(k_wta_finalize, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       p->width, p->height, p->ndisp, reinterpret_cast<const long long *>(key), m2,
                       reinterpret_cast<const long long *>(tkey), t2, d_ref, conf_ref, d_tar, conf_tar, code_ref,
                       code_tar);
    return finish_launch();
}

int asw_consistency(const asw_params *p, const int32_t *d_ref, const int32_t *d_tar, const uint8_t *code_ref,
                    const uint8_t *code_tar, float *conf_ref, float *conf_tar, uint8_t *out_rgba,
                    uint8_t *out_red_rgba, void *stream) {
    ASW_CHECK_PARAMS(p);
    if (!d_ref || !d_tar || !code_ref || !code_tar || !conf_ref || !conf_tar) return ASW_E_INVALID;
    const long long n = (long long)p->width * p->height;
    hipLaunchKernelGGL(k_consistency, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, n,
                       p->ndisp, p->lr_mode, d_ref, d_tar, code_ref, code_tar, conf_ref, conf_tar,
                       reinterpret_cast<uchar4 *>(out_rgba), reinterpret_cast<uchar4 *>(out_red_rgba));
    return finish_launch();
}

}  // extern "C"
