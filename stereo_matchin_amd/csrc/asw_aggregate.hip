// asw_aggregate.hip — the iterated weighted-aggregation passes, the hot kernels of
// the ASW path (reference: K/asw_vcost_aggregation.cl:11-44 and
// K/asw_hcost_aggregation.cl:12-44, 2*r launches per frame at main.cpp:492-515,
// 94 % of the reference's ASW time).
//
// Per voxel (x, y, d) and tap i = 0..T-1, in order (FP policy):
//     ww = wl_i(x,y) * wr_i(max(x-d,0), y);  num = fma(ww, c_i, num);  den = den + ww
// with num = den = 1e-5f on entry and out = num / den (IEEE).  c_i is the cost
// of plane d at the i-th vertical (V) or horizontal (H) neighbour, clamped.
//
// MI355X mapping (both passes):
//   * lanes = 64 consecutive disparities of one pixel; cost volumes are
//     [H][W][Dp], so the single cost load and the single store of a step are one
//     coalesced 256-B access per wave;
//   * the wave sweeps along the aggregation axis; the T-tap cost window lives in a
//     rotating VGPR ring of U = T+P registers and the next element is loaded P
//     steps ahead (the ring is indexed statically: the sweep loop is unrolled by U);
//   * wl_i(x,y) is the same for the whole wave: scalar loads (SGPR operands).  Its
//     lines are pulled into L2 PS steps ahead by a one-VGPR vector "warm" load so
//     the s_load finds them there;
//   * wr_i(x-d,y) differs per lane: the support rows of every x-d the block needs
//     are staged in LDS ([xr][Tp] with Tp/4 odd => conflict-free ds_read_b128,
//     4 taps per read).  H pass: one slab per row segment, staged once.  V pass:
//     one slab per row, double-buffered, loads issued PS steps ahead through a
//     VGPR ring, one barrier per row.
// Per voxel-tap the VALU work is the 3 instructions above; everything else is
// amortised over the T taps of a step.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "asw_common.h"

namespace asw {
namespace {

// native 4-float vector (the HIP f4 struct/union blocks SROA of small arrays)
using f4 = float __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

__device__ __forceinline__ void tap(float wl, float wr, float c, float &num, float &den) {
    const float ww = wl * wr;
    num = __builtin_fmaf(ww, c, num);
    den = den + ww;
}

// keep a prefetch load alive without using its value (the compiler would drop it)
__device__ __forceinline__ void keep(float v) { asm volatile("" ::"v"(v)); }

// C prefetch distance P: smallest P >= 3 with (T + P) % 4 == 0, so that the
// 4-deep staging/warm rings (PS = 4) divide the unroll period U = T + P.
constexpr int pf_dist(int T) {
    int P = 3;
    while ((T + P) % 4 != 0) ++P;
    return P;
}
constexpr int kPS = 4;

// Compile-time loop: f(integral_constant<int, I>) for I in [B, E).  Used for the
// U-step sweep so every ring index is a constant expression from the start
// (a #pragma-unrolled loop left the staging ring in scratch memory).
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F &&f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

// All T taps of one output: wl from scalar memory (uniform), wr from an LDS slab
// entry (per lane), c from the window ring.
template <int T, int U>
__device__ __forceinline__ float aggregate_taps(const float *__restrict__ wlrow, const f4 *srow,
                                                const float (&win)[U], int s) {
    constexpr int Q = tap_pitch(T) / 4;
    float num = 1e-5f, den = 1e-5f;
#pragma unroll
    for (int i4 = 0; i4 < Q; ++i4) {
        if (4 * i4 >= T) break;
        const f4 r4 = srow[i4];
        const f4 l4 = *reinterpret_cast<const f4 *>(wlrow + 4 * i4);
        tap(l4.x, r4.x, win[(s + 4 * i4 + 0) % U], num, den);
        if (4 * i4 + 1 < T) tap(l4.y, r4.y, win[(s + 4 * i4 + 1) % U], num, den);
        if (4 * i4 + 2 < T) tap(l4.z, r4.z, win[(s + 4 * i4 + 2) % U], num, den);
        if (4 * i4 + 3 < T) tap(l4.w, r4.w, win[(s + 4 * i4 + 3) % U], num, den);
    }
    return num / den;
}

// ---------------------------------------------------------------------------
// V pass.  Block = NW waves = NW consecutive columns x0..x0+NW-1, one 64-plane
// block, a strip of rows [y_begin, y_end).  Window slot of row q:
// (q - (y_begin - R)) mod U; at step y the row y+R+P is loaded into the slot of
// row y-R-1 (consumed at step y-1).
// ---------------------------------------------------------------------------
template <int T, int NW>
__global__ __launch_bounds__(NW * 64) void k_vpass(const float *__restrict__ wl, const float *__restrict__ wr,
                                                   const float *__restrict__ cin, float *__restrict__ cout,
                                                   int W, int H, int Dp, int d_begin, int rows_per_strip) {
    constexpr int R = T / 2;
    constexpr int TP = tap_pitch(T);
    constexpr int Q = TP / 4;
    constexpr int P = pf_dist(T);
    constexpr int U = T + P;
    constexpr int PS = kPS;
    static_assert(U % PS == 0 && U % 2 == 0, "ring periods must divide the unroll period");
    constexpr int SLAB = NW + 63;
    constexpr int NQ = SLAB * Q;
    constexpr int NSTAGE = (NQ + NW * 64 - 1) / (NW * 64);
    __shared__ f4 slab[2][NQ];

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int x0 = blockIdx.x * NW;
    const int kb = blockIdx.y * 64;
    const int y_begin = blockIdx.z * rows_per_strip;
    if (y_begin >= H) return;  // uniform for the block
    const int y_end = min(H, y_begin + rows_per_strip);
    const bool xvalid = x0 + wave < W;
    const int x = min(x0 + wave, W - 1);
    const int k = kb + lane;
    const int dabs0 = d_begin + kb;
    const int slab_base = x0 - dabs0 - 63;  // virtual xr of slab entry 0
    const f4 *my_slab0 = &slab[0][((x - x0) + 63 - lane) * Q];
    const long long rowstride = (long long)W * Dp;
    const float *cbase = cin + (long long)x * Dp + k;
    const float *wlcol = wl + (long long)x * TP;        // + y*W*TP
    const long long wlrowstride = (long long)W * TP;
    const int warm_off = lane < TP ? lane : 0;

    // per-thread share of a slab row (at most 2 f4 per thread): entry e,
    // quad q; surplus lanes redo the last entry (same value, same place)
    static_assert(NSTAGE <= 2, "slab row larger than two f4 per thread");
    const int t0 = min((int)threadIdx.x, NQ - 1);
    const int t1 = min((int)threadIdx.x + NW * 64, NQ - 1);
    const int off0 = clampi(slab_base + t0 / Q, 0, W - 1) * TP + 4 * (t0 % Q);
    const int off1 = clampi(slab_base + t1 / Q, 0, W - 1) * TP + 4 * (t1 % Q);
    const float *wrrows = wr;
    const long long wrrowstride = (long long)W * TP;

    float win[U];
    f4 sa[PS], sb[PS];
    float warm[PS];
#pragma unroll
    for (int j = 0; j < T - 1 + P; ++j) win[j] = cbase[clampi(y_begin - R + j, 0, H - 1) * rowstride];
#pragma unroll
    for (int j = 0; j < PS; ++j) {
        const float *row = wrrows + (long long)clampi(y_begin + j, 0, H - 1) * wrrowstride;
        sa[j] = *reinterpret_cast<const f4 *>(row + off0);
        if constexpr (NSTAGE > 1) sb[j] = *reinterpret_cast<const f4 *>(row + off1);
        warm[j] = wlcol[(long long)clampi(y_begin + j, 0, H - 1) * wlrowstride + warm_off];
    }
    slab[0][t0] = sa[0];
    if constexpr (NSTAGE > 1) slab[0][t1] = sb[0];
    __syncthreads();

    for (int ys = y_begin; ys < y_end; ys += U) {
        static_for<0, U>([&](auto sc) __attribute__((always_inline)) {
            constexpr int s = decltype(sc)::value;
            const int y = ys + s;
            if (y >= y_end) return;
            win[(s + U - 1) % U] = cbase[clampi(y + R + P, 0, H - 1) * rowstride];
            keep(warm[s % PS]);
            warm[s % PS] = wlcol[(long long)clampi(y + PS, 0, H - 1) * wlrowstride + warm_off];
            const float *wlrow = wlcol + (long long)y * wlrowstride;
            const f4 *srow = my_slab0 + (s & 1) * NQ;
            const float v = aggregate_taps<T, U>(wlrow, srow, win, s);
            if (xvalid) cout[(long long)y * rowstride + (long long)x * Dp + k] = v;
            slab[(s + 1) & 1][t0] = sa[(s + 1) % PS];
            if constexpr (NSTAGE > 1) slab[(s + 1) & 1][t1] = sb[(s + 1) % PS];
            {
                const float *row = wrrows + (long long)clampi(y + PS, 0, H - 1) * wrrowstride;
                sa[s % PS] = *reinterpret_cast<const f4 *>(row + off0);
                if constexpr (NSTAGE > 1) sb[s % PS] = *reinterpret_cast<const f4 *>(row + off1);
            }
            __syncthreads();
        });
    }
}

// ---------------------------------------------------------------------------
// H pass.  Block = NW waves on row y and a segment of SEG = NW*XW columns; the
// right-support slab for every xr the segment needs (SEG+63 entries) is staged
// once.  Wave w sweeps columns [xs + w*XW, +XW).  Window slot of column q:
// (q - (xw0 - R)) mod U.
// ---------------------------------------------------------------------------
template <int T, int NW, int XW>
__global__ __launch_bounds__(NW * 64) void k_hpass(const float *__restrict__ wl, const float *__restrict__ wr,
                                                   const float *__restrict__ cin, float *__restrict__ cout,
                                                   int W, int H, int Dp, int d_begin) {
    constexpr int R = T / 2;
    constexpr int TP = tap_pitch(T);
    constexpr int Q = TP / 4;
    constexpr int P = pf_dist(T);
    constexpr int U = T + P;
    constexpr int PS = kPS;
    static_assert(U % PS == 0, "ring period must divide the unroll period");
    constexpr int SEG = NW * XW;
    constexpr int SLAB = SEG + 63;
    constexpr int NQ = SLAB * Q;
    __shared__ f4 slab[NQ];

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int xs = blockIdx.x * SEG;
    const int y = blockIdx.y;
    const int kb = blockIdx.z * 64;
    const int k = kb + lane;
    const int dabs0 = d_begin + kb;
    const int slab_base = xs - dabs0 - 63;

    const float *wrrow = wr + (long long)y * W * TP;
    for (int t = threadIdx.x; t < NQ; t += NW * 64) {
        const int e = t / Q, q = t - e * Q;
        slab[t] = *reinterpret_cast<const f4 *>(wrrow + clampi(slab_base + e, 0, W - 1) * TP + 4 * q);
    }
    __syncthreads();

    const int xw0 = xs + wave * XW;
    if (xw0 >= W) return;
    const int xw1 = min(xw0 + XW, W);
    const float *cbase = cin + (long long)y * W * Dp + k;
    const float *wlrow0 = wl + (long long)y * W * TP;
    const int warm_off = lane < TP ? lane : 0;

    float win[U];
    float warm[PS];
#pragma unroll
    for (int j = 0; j < T - 1 + P; ++j) win[j] = cbase[(long long)clampi(xw0 - R + j, 0, W - 1) * Dp];
#pragma unroll
    for (int j = 0; j < PS; ++j) warm[j] = wlrow0[clampi(xw0 + j, 0, W - 1) * TP + warm_off];

    for (int xb = xw0; xb < xw1; xb += U) {
        static_for<0, U>([&](auto sc) __attribute__((always_inline)) {
            constexpr int s = decltype(sc)::value;
            const int x = xb + s;
            if (x >= xw1) return;
            win[(s + U - 1) % U] = cbase[(long long)clampi(x + R + P, 0, W - 1) * Dp];
            keep(warm[s % PS]);
            warm[s % PS] = wlrow0[clampi(x + PS, 0, W - 1) * TP + warm_off];
            const f4 *srow = &slab[((x - xs) + 63 - lane) * Q];
            const float v = aggregate_taps<T, U>(wlrow0 + x * TP, srow, win, s);
            cout[((long long)y * W + x) * Dp + k] = v;
        });
    }
}

template <int T>
int launch_pass_t(const asw_params *p, int dir, const float *wl, const float *wr, const float *cin, float *cout,
                  hipStream_t st) {
    const int W = p->width, H = p->height;
    const int Dp = asw_disp_pitch(p);
    const int nkb = Dp / 64;
    if (dir == ASW_DIR_V) {
        constexpr int NW = 16;
        const int nxb = (W + NW - 1) / NW;
        // enough blocks to fill 256 CUs several times; strips >= 2T rows keep
        // the window prologue (T-1+P row loads per strip) a small overhead.
        int nstrip = (int)((2048LL + (long long)nxb * nkb - 1) / ((long long)nxb * nkb));
        const int max_strip = H / (2 * T) > 1 ? H / (2 * T) : 1;
        if (nstrip > max_strip) nstrip = max_strip;
        if (nstrip < 1) nstrip = 1;
        const int rows = (H + nstrip - 1) / nstrip;
        nstrip = (H + rows - 1) / rows;
        hipLaunchKernelGGL((k_vpass<T, NW>), dim3(nxb, nkb, nstrip), dim3(NW * 64), 0, st, wl, wr, cin, cout, W, H,
                           Dp, p->d_begin, rows);
    } else {
        constexpr int NW = 4;
        constexpr int XW = (T > 41) ? 32 : 64;
        constexpr int SEG = NW * XW;
        const int nseg = (W + SEG - 1) / SEG;
        hipLaunchKernelGGL((k_hpass<T, NW, XW>), dim3(nseg, H, nkb), dim3(NW * 64), 0, st, wl, wr, cin, cout, W, H,
                           Dp, p->d_begin);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_hip_error(e);
        return ASW_E_HIP;
    }
    return ASW_OK;
}

}  // namespace

int launch_pass(const asw_params *p, int dir, const float *wl, const float *wr, const float *cin, float *cout,
                hipStream_t st) {
    switch (p->taps) {
#define ASW_CASE(TT) \
    case TT:         \
        return launch_pass_t<TT>(p, dir, wl, wr, cin, cout, st);
        ASW_CASE(3)
        ASW_CASE(5)
        ASW_CASE(7)
        ASW_CASE(9)
        ASW_CASE(15)
        ASW_CASE(33)
        ASW_CASE(35)
        ASW_CASE(51)
#undef ASW_CASE
        default:
            return ASW_E_UNSUPPORTED;
    }
}

}  // namespace asw
