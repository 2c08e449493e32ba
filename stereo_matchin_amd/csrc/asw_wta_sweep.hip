// asw_wta_sweep.hip — asw_WTA (K/asw_wta.cl:12-82) as a row sweep: the left
// first-argmin and the bresenham target scan of every pixel of a row in ONE pass
// over the row's volume, with no per-pixel gathers.
//
// Target scan (K/asw_wta.cl:50-67) of pixel x with left disparity md: for i < md,
// xq = max(0, x-i), b = md + xq - x, value C[b][y][xq].  For i <= x the points
// (xq, b) = (x-i, md-i) lie on the diagonal k = xq - b = x - md; for i > x the
// point clamps to (0, md-x), the diagonal's first point, repeated md-1-x more
// times.  So the scan of pixel x is the diagonal k = x - md over its points with
// b >= max(1, -k) and xq <= x, plus those repeats.
//   The sweep walks x left to right with one state (m1, m2, argmin b) per diagonal,
// stored at the plane b = x - k the diagonal reaches in column x: lane l holds
// planes PPL*l .. PPL*l+PPL-1 of the column (one PPL-dword load per lane and
// column), so from column x to x+1 every state moves up one plane: inside a lane
// by renaming registers (the unrolled steps rotate which register holds which
// plane), across lanes by one shuffle of the top plane's state.  Column x then
// adds its voxel C[b][y][x] to the state at plane b (b >= 1: b = 0 is no target
// point), and pixel x reads the state at plane md.
//   Ties: the reference scans i upward with strict '<', so the FIRST i (the largest
// b) wins; the sweep meets b upward and keeps the LAST with '<='.  The multiset
// second minimum (m1, m2 of the sequential loop) does not depend on the order; the
// md-1-x repeats of the first point (0, md-x) enter it as m2 = min(m2, C[md-x][y][0]).
//   Left scan (K/asw_wta.cl:25-47): each lane scans its PPL planes in order (strict
// '<'), then a butterfly over the 64 lanes combines (m1, m2, index) with ties to
// the smaller index (the first argmin).
// One wave per image row; results of 64 consecutive pixels are gathered into
// lanes and stored coalesced.  Bit-identical to k_wta_scan<0> (asw_refine.hip).
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>
#include <type_traits>

#include "asw_common.h"

namespace asw {
namespace {

constexpr float kSent = 100000.0f;  // K/asw_wta.cl:25-26

template <int B, int E, class F>
__device__ __forceinline__ void sfor(F &&f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        sfor<B + 1, E>(f);
    }
}

struct Top2 {
    float m1, m2;
    int idx;
};

// combine two partial scans of disjoint plane sets: first argmin (ties -> smaller
// index), multiset second minimum
__device__ __forceinline__ Top2 combine(const Top2 &a, float om1, float om2, int oidx) {
    Top2 r;
    r.m2 = fminf(fmaxf(a.m1, om1), fminf(a.m2, om2));
    const bool take = (om1 < a.m1) || (om1 == a.m1 && oidx < a.idx);
    r.m1 = take ? om1 : a.m1;
    r.idx = take ? oidx : a.idx;
    return r;
}

// PPL planes per lane (Dp = 64 PPL); PF columns of loads in flight
template <int PPL, int PF>
__global__ __launch_bounds__(64) void k_wta_sweep(const float *__restrict__ cost, int W, int H, int D,
                                                  int32_t *__restrict__ d_ref, float *__restrict__ conf_ref,
                                                  int32_t *__restrict__ d_tar, float *__restrict__ conf_tar,
                                                  uint8_t *__restrict__ code_ref, uint8_t *__restrict__ code_tar) {
    constexpr int Dp = 64 * PPL;
    static_assert(PF % PPL == 0, "register rotation period");
    const int y = blockIdx.x;
    if (y >= H) return;
    const int lane = threadIdx.x;
    const float *row = cost + (long long)y * W * Dp + PPL * lane;
    auto load = [&](int x, float (&v)[PPL]) __attribute__((always_inline)) {
        const float *pp = row + (long long)min(x, W - 1) * Dp;
#pragma unroll
        for (int j = 0; j < PPL; ++j) v[j] = pp[j];
    };
    float ring[PF][PPL];
#pragma unroll
    for (int s = 0; s < PF; ++s) load(s, ring[s]);
    float col0[PPL];  // column 0: the clamped first points of the negative diagonals
#pragma unroll
    for (int j = 0; j < PPL; ++j) col0[j] = ring[0][j];

    // diagonal states; physical register p holds plane slot (p + x) mod PPL at column x
    float sm1[PPL], sm2[PPL];
    int sb[PPL];
#pragma unroll
    for (int j = 0; j < PPL; ++j) {
        sm1[j] = kSent;
        sm2[j] = kSent;
        sb[j] = -1;
    }
    // per-pixel results gathered into lane (x & 63)
    int o_md = 0, o_tb = 0;
    float o_m1 = kSent, o_m2 = kSent, o_t1 = kSent, o_t2 = kSent;
    const long long rbase = (long long)y * W;
    auto flush = [&](int xbase, int n) __attribute__((always_inline)) {
        if (lane < n) {
            const long long p = rbase + xbase + lane;
            d_ref[p] = o_md;
            d_tar[p] = o_tb;
            conf_ref[p] = (o_m2 - o_m1) / o_m2;
            conf_tar[p] = (o_t2 - o_t1) / o_t2;
            if (code_ref) code_ref[p] = (uint8_t)code_u8(o_md, D);
            if (code_tar) code_tar[p] = (uint8_t)code_u8(o_tb, D);
        }
    };

    auto step = [&](auto sc, int x) __attribute__((always_inline)) {
        constexpr int s = decltype(sc)::value;
        float v[PPL];
#pragma unroll
        for (int j = 0; j < PPL; ++j) v[j] = ring[s][j];
        load(x + PF, ring[s]);
        // ---- left scan of column x
        Top2 t{kSent, kSent, INT_MAX};
#pragma unroll
        for (int j = 0; j < PPL; ++j) {
            const int d = PPL * lane + j;
            const float c = d < D ? v[j] : __builtin_inff();
            t.m2 = c < t.m2 ? c : t.m2;
            t.idx = c < t.m1 ? d : t.idx;
            t.m2 = c < t.m1 ? t.m1 : t.m2;
            t.m1 = c < t.m1 ? c : t.m1;
        }
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) t = combine(t, __shfl_xor(t.m1, o), __shfl_xor(t.m2, o), __shfl_xor(t.idx, o));
        const int md = __builtin_amdgcn_readfirstlane(t.idx == INT_MAX ? 0 : t.idx);
        // ---- diagonal states: move up one plane (column x-1 -> x).  The physical
        // register of the top plane slot becomes plane slot 0, fed by the lane below.
        // (x = s mod PPL: the sweep runs in PF-column periods, PF a multiple of PPL)
        constexpr int ptop = ((-s) % PPL + PPL) % PPL;  // top slot at column x-1 = slot 0 at column x
        {
            const float a = __shfl_up(sm1[ptop], 1), b2 = __shfl_up(sm2[ptop], 1);
            const int bi = __shfl_up(sb[ptop], 1);
            sm1[ptop] = lane == 0 ? kSent : a;
            sm2[ptop] = lane == 0 ? kSent : b2;
            sb[ptop] = lane == 0 ? -1 : bi;
        }
        // ---- add column x's voxels: plane slot j lives in physical ((j - s) mod PPL)
#pragma unroll
        for (int j = 0; j < PPL; ++j) {
            const int p = ((j - s) % PPL + PPL) % PPL;
            const int b = PPL * lane + j;
            const float c = (b >= 1 && b < D) ? v[j] : __builtin_inff();
            const bool le = c <= sm1[p];
            sm2[p] = le ? sm1[p] : fminf(sm2[p], c);
            sb[p] = le ? b : sb[p];
            sm1[p] = le ? c : sm1[p];
        }
        // ---- the target scan of pixel x: the state at plane md
        float t1 = kSent, t2 = kSent;
        int tb = md;
        if (md >= 1) {
            const int ln = md / PPL, slot = md - ln * PPL;
            const int p = ((slot - s) % PPL + PPL) % PPL;
            float a1 = sm1[0], a2 = sm2[0];
            int ab = sb[0];
#pragma unroll
            for (int q = 1; q < PPL; ++q) {
                a1 = p == q ? sm1[q] : a1;
                a2 = p == q ? sm2[q] : a2;
                ab = p == q ? sb[q] : ab;
            }
            t1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, a1), ln));
            t2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, a2), ln));
            tb = __builtin_amdgcn_readlane(ab, ln);
            if (md - x >= 2) {  // the repeats of the clamped first point (0, md - x)
                const int b0 = md - x, l0 = b0 / PPL, j0 = b0 - l0 * PPL;
                float c0 = col0[0];
#pragma unroll
                for (int q = 1; q < PPL; ++q) c0 = j0 == q ? col0[q] : c0;
                const float v0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, c0), l0));
                t2 = fminf(t2, v0);
            }
        }
        if (lane == (x & 63)) {
            o_md = md;
            o_m1 = t.m1;
            o_m2 = t.m2;
            o_tb = tb;
            o_t1 = t1;
            o_t2 = t2;
        }
        if ((x & 63) == 63) flush(x - 63, 64);
    };
    int x = 0;
    for (; x + PF <= W; x += PF) sfor<0, PF>([&](auto sc) __attribute__((always_inline)) { step(sc, x + decltype(sc)::value); });
    for (int xr = x; xr < W; xr += PF) {  // the last partial period
        sfor<0, PF>([&](auto sc) __attribute__((always_inline)) {
            if (xr + decltype(sc)::value < W) step(sc, xr + decltype(sc)::value);
        });
    }
    if (W & 63) flush(W - (W & 63), W & 63);
}

}  // namespace

// asw_WTA of a whole-range context (d_begin = 0) through the row sweep; Dp = 64..256.
// ASW_E_UNSUPPORTED for other pitches (the caller then runs k_wta_scan).
int launch_wta_sweep(const asw_params *p, const float *cost, int32_t *d_ref, float *conf_ref, int32_t *d_tar,
                     float *conf_tar, uint8_t *code_ref, uint8_t *code_tar, hipStream_t st) {
    const int Dp = asw_disp_pitch(p);
    const dim3 grid((unsigned)p->height), block(64);
#define ASW_SWEEP(PPL, PF)                                                                                         \
    hipLaunchKernelGGL((k_wta_sweep<PPL, PF>), grid, block, 0, st, cost, p->width, p->height, p->ndisp, d_ref,    \
                       conf_ref, d_tar, conf_tar, code_ref, code_tar)
    switch (Dp) {
        case 64: ASW_SWEEP(1, 16); break;
        case 128: ASW_SWEEP(2, 16); break;
        case 256: ASW_SWEEP(4, 16); break;
        default: return ASW_E_UNSUPPORTED;
    }
#undef ASW_SWEEP
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_hip_error(e);
        return ASW_E_HIP;
    }
    return ASW_OK;
}

}  // namespace asw
