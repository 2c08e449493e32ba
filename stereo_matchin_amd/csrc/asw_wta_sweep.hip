// asw_wta_sweep.hip — asw_WTA (K/asw_wta.cl:12-82) of a whole-range context as a
// row sweep: the left first-argmin AND the bresenham target scan of every pixel of a
// row from ONE pass over the row's volume, with no per-pixel gathers.
//
// Target scan (K/asw_wta.cl:50-67) of pixel x with left disparity md: for i < md,
// xq = max(0, x-i), b = md + xq - x, value C[b][y][xq].  For i <= x the points
// (xq, b) = (x-i, md-i) lie on the diagonal k = xq - b = x - md; for i > x the point
// clamps to (0, md-x), the diagonal's first point, repeated md-1-x more times.  So
// the scan of pixel x is diagonal k = x - md over its points with b >= max(1, -k)
// and xq <= x, plus those repeats.
//   Diagonal states (m1, m2, argmin b) live in lanes: slot j (= wave*64 + lane, Dp
// slots) holds the diagonals k = -j (mod Dp), which at column x are at plane
// b = (x + j) mod Dp.  Column x adds C[b][y][x] to every slot (b = 0 starts the
// slot's next diagonal, which has no point there), and pixel x takes the state of
// the one slot whose plane is then md(x) (slot (md - x) mod Dp), which writes it to
// LDS.  No state ever moves between lanes: each slot reads its own plane of the
// column, and a wave's 64 slots read 64 consecutive planes.
//   Ties: the reference scans i upward with strict '<' (the FIRST i, i.e. the largest
// b, wins); the slots meet b upward and keep the LAST with '<='.  (m1, m2) is the
// multiset's two smallest whatever the order; the md-1-x repeats of the first point
// enter as m2 = min(m2, C[md-x][y][0]).
//   Left scan (K/asw_wta.cl:25-47): lane = pixel, wave w scans planes [64w, 64w+64)
// of the tile's 64 pixels in order with strict '<'; the NW partials combine in plane
// order (ties to the smaller index: the first argmin).
// Block = NW = Dp/64 waves, one image row; the row is staged 64 columns at a time in
// LDS ([column][plane], pitch Dp+4: lane-per-pixel ds_read_b128 and slot ds_read_b32
// both conflict-free), the next tile loaded into registers while the current one is
// swept.  Bit-identical to k_wta_scan<0> (asw_refine.hip).
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "asw_common.h"

namespace asw {
namespace {

constexpr float kSent = 100000.0f;  // K/asw_wta.cl:25-26
constexpr int kTC = 64;             // columns per tile

template <int NW>
__global__ __launch_bounds__(NW * 64) void k_wta_tile(const float *__restrict__ cost, int W, int H, int D,
                                                      int32_t *__restrict__ d_ref, float *__restrict__ conf_ref,
                                                      int32_t *__restrict__ d_tar, float *__restrict__ conf_tar,
                                                      uint8_t *__restrict__ code_ref, uint8_t *__restrict__ code_tar) {
    using f4 = float __attribute__((ext_vector_type(4)));
    constexpr int Dp = 64 * NW;
    constexpr int PITCH = Dp + 4;
    constexpr int NQ = Dp / 4;                   // float4 per column
    constexpr int SPT = kTC * NQ / (NW * 64);    // staged float4 per thread (16)
    __shared__ float tile[kTC * PITCH];
    __shared__ float part_m1[NW][64], part_m2[NW][64];
    __shared__ int part_idx[NW][64];
    __shared__ float res_t1[kTC], res_t2[kTC];  // the target scan of each pixel of the tile
    __shared__ int res_tb[kTC];

    const int y = blockIdx.x;
    if (y >= H) return;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int j = wave * 64 + lane;  // diagonal slot
    const float *rowp = cost + (long long)y * W * Dp;
    const long long rbase = (long long)y * W;

    f4 stage[SPT];
    auto load_tile = [&](int x0) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < SPT; ++i) {
            const int f = (int)threadIdx.x + i * NW * 64;
            const int c = f / NQ, g = f - c * NQ;
            stage[i] = *reinterpret_cast<const f4 *>(rowp + (long long)min(x0 + c, W - 1) * Dp + 4 * g);
        }
    };
    auto write_tile = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < SPT; ++i) {
            const int f = (int)threadIdx.x + i * NW * 64;
            const int c = f / NQ, g = f - c * NQ;
            *reinterpret_cast<f4 *>(&tile[c * PITCH + 4 * g]) = stage[i];
        }
    };

    load_tile(0);
    write_tile();
    __syncthreads();
    const float first_v = tile[j];  // C[j][y][0]: the first point of slot j's diagonal k = -j
    float sm1 = kSent, sm2 = kSent;
    int sb = -1;

    for (int x0 = 0; x0 < W; x0 += kTC) {
        const int nc = min(kTC, W - x0);
        if (x0 + kTC < W) load_tile(x0 + kTC);  // in flight while this tile is swept
        // ---- left scan, lane = pixel x0 + lane, this wave's 64 planes
        {
            // four independent sequential scans of 16 planes each (latency: the chains
            // interleave), combined in plane order
            float m1[4], m2[4];
            int idx[4];
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                m1[h] = kSent;
                m2[h] = kSent;
                idx[h] = INT_MAX;
            }
            const float *pp = &tile[lane * PITCH + 64 * wave];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
#pragma unroll
                for (int h = 0; h < 4; ++h) {
                    const f4 v = *reinterpret_cast<const f4 *>(pp + 16 * h + 4 * q);
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int d = 64 * wave + 16 * h + 4 * q + e;
                        const float c = d < D ? v[e] : __builtin_inff();
                        m2[h] = c < m2[h] ? c : m2[h];
                        idx[h] = c < m1[h] ? d : idx[h];
                        m2[h] = c < m1[h] ? m1[h] : m2[h];
                        m1[h] = c < m1[h] ? c : m1[h];
                    }
                }
            }
            float a1 = m1[0], a2 = m2[0];
            int ai = idx[0];
#pragma unroll
            for (int h = 1; h < 4; ++h) {  // higher planes: ties keep the smaller index
                a2 = fminf(fmaxf(a1, m1[h]), fminf(a2, m2[h]));
                const bool take = m1[h] < a1;
                a1 = take ? m1[h] : a1;
                ai = take ? idx[h] : ai;
            }
            part_m1[wave][lane] = a1;
            part_m2[wave][lane] = a2;
            part_idx[wave][lane] = ai;
        }
        __syncthreads();
        float M1 = part_m1[0][lane], M2 = part_m2[0][lane];
        int MI = part_idx[0][lane];
#pragma unroll
        for (int w = 1; w < NW; ++w) {  // higher planes: ties keep the smaller index
            const float om1 = part_m1[w][lane], om2 = part_m2[w][lane];
            const int oi = part_idx[w][lane];
            M2 = fminf(fmaxf(M1, om1), fminf(M2, om2));
            const bool take = om1 < M1;
            M1 = take ? om1 : M1;
            MI = take ? oi : MI;
        }
        const int md_lane = MI == INT_MAX ? 0 : MI;
        if (wave == 0 && lane < nc) {
            const long long p = rbase + x0 + lane;
            d_ref[p] = md_lane;
            conf_ref[p] = (M2 - M1) / M2;
            if (code_ref) code_ref[p] = (uint8_t)code_u8(md_lane, D);
        }
        // ---- diagonal sweep of the tile's columns.  Pixel x's target scan is the slot
        // whose plane at column x is md(x) (slot (md - x) mod Dp): that lane alone sees
        // b == md and records its state for the pixel (res_*; md = 0: the defaults).
        if (wave == 0) {
            res_t1[lane] = kSent;
            res_t2[lane] = kSent;
            res_tb[lane] = 0;
        }
        __syncthreads();
        constexpr int CH = 16;  // columns per batch of tile reads
        for (int c0 = 0; c0 < nc; c0 += CH) {
            float tv[CH];
#pragma unroll
            for (int k = 0; k < CH; ++k) {
                const int b = (x0 + c0 + k + j) & (Dp - 1);
                tv[k] = tile[(c0 + k) * PITCH + b];
            }
#pragma unroll
            for (int k = 0; k < CH; ++k) {
                const int c = c0 + k;
                if (c < nc) {  // uniform (the last tile of a row may be partial)
                    const int x = x0 + c;
                    const int b = (x + j) & (Dp - 1);
                    if (b == 0) {  // slot j starts diagonal k = x (no point at b = 0)
                        sm1 = kSent;
                        sm2 = kSent;
                        sb = -1;
                    } else {
                        const float t = b < D ? tv[k] : __builtin_inff();
                        const bool le = t <= sm1;
                        sm2 = le ? sm1 : fminf(sm2, t);
                        sb = le ? b : sb;
                        sm1 = le ? t : sm1;
                    }
                    const int md = __builtin_amdgcn_readlane(md_lane, c);
                    if (b == md && md >= 1) {  // one lane of the block, if any
                        res_t1[c] = sm1;
                        res_t2[c] = md - x >= 2 ? fminf(sm2, first_v) : sm2;  // the clamped repeats
                        res_tb[c] = sb;
                    }
                }
            }
        }
        __syncthreads();
        if (wave == 0 && lane < nc) {
            const long long p = rbase + x0 + lane;
            const float t1 = res_t1[lane], t2 = res_t2[lane];
            const int tb = res_tb[lane];
            d_tar[p] = tb;
            conf_tar[p] = (t2 - t1) / t2;
            if (code_tar) code_tar[p] = (uint8_t)code_u8(tb, D);
        }
        __syncthreads();  // every read of this tile is done
        if (x0 + kTC < W) {
            write_tile();
            __syncthreads();
        }
    }
}

}  // namespace

// asw_WTA of a whole-range context through the row sweep; Dp = 64, 128 or 256
// (ASW_E_UNSUPPORTED otherwise: the caller then runs k_wta_scan).
int launch_wta_sweep(const asw_params *p, const float *cost, int32_t *d_ref, float *conf_ref, int32_t *d_tar,
                     float *conf_tar, uint8_t *code_ref, uint8_t *code_tar, hipStream_t st) {
    const int Dp = asw_disp_pitch(p);
    const dim3 grid((unsigned)p->height);
    switch (Dp) {
        case 64:
            hipLaunchKernelGGL(k_wta_tile<1>, grid, dim3(64), 0, st, cost, p->width, p->height, p->ndisp, d_ref,
                               conf_ref, d_tar, conf_tar, code_ref, code_tar);
            break;
        case 128:
            hipLaunchKernelGGL(k_wta_tile<2>, grid, dim3(128), 0, st, cost, p->width, p->height, p->ndisp, d_ref,
                               conf_ref, d_tar, conf_tar, code_ref, code_tar);
            break;
        case 256:
            hipLaunchKernelGGL(k_wta_tile<4>, grid, dim3(256), 0, st, cost, p->width, p->height, p->ndisp, d_ref,
                               conf_ref, d_tar, conf_tar, code_ref, code_tar);
            break;
        default:
            return ASW_E_UNSUPPORTED;
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_hip_error(e);
        return ASW_E_HIP;
    }
    return ASW_OK;
}

}  // namespace asw
