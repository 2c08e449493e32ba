// Experimental pass kernels behind a tiny C interface, driven by tools/exp/exp_bench.py
// on the real C4 inputs (the production library computes raw cost and supports and the
// reference pass; this library only has the instantiations under test, so it builds in
// minutes).  Not part of the product.
#include <hip/hip_runtime.h>

#include "asw_aggregate_impl.h"
#include "asw_vpass12.h"

namespace asw {
namespace agg {
int g_pass_variant = 0;
}
void note_pass_kernel(int, int, const char *, int, const char *, bool) {}
}  // namespace asw

using namespace asw::agg;

// the launchers call these library helpers; local copies keep this library stand-alone
extern "C" __attribute__((visibility("hidden"))) int asw_disp_pitch(const asw_params *p) {
    return asw::round_up(asw::d_end_of_p(p) - p->d_begin, 64);
}

#ifdef EXP_V12
// one k_vpass12 instantiation per build: -DV12_NW=.. -DV12_NPH=.. -DV12_PS=..
#ifndef V12_PS
#define V12_PS 4
#endif
extern "C" int exp_v12(int shape, int dm, int nstrip, const asw_params *p, const float *wl, const float *wr,
                       const float *cin, float *cout, float *den, void *stream) {
    hipStream_t st = (hipStream_t)stream;
    if (p->taps != 35 || dm != V12_DM) return -4;
    (void)shape;
    launch_v12<35, V12_NW, V12_DM, 2, V12_PS, V12_NPH, kCPStream>(p, wl, wr, cin, cout, den, st, nstrip);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
#endif

#ifdef EXP_C5
// C5 (T = 51) V shapes: shape = NW * 100 + NPH * 10 + RB (PS = 2 when RB = 1, else 4)
extern "C" int exp_c5(int dir, int shape, int dm, const asw_params *p, const float *wl, const float *wr,
                      const float *cin, float *cout, float *den, void *stream) {
    hipStream_t st = (hipStream_t)stream;
    if (p->taps != 51 || dm != 2 || dir != 0) return -4;
#ifndef C5_TK
#define C5_TK 0
#endif
    // (C5_TK: the XCD-round tile order of the shipped C5 V pass, round 6)
    if (shape == C5_NW * 100 + C5_NPH * 10 + C5_RB)
        launch_v10<51, C5_NW, DM_READ, C5_RB, kCPStream, kCPStream, C5_RB == 1 ? 2 : 4, C5_NPH, false, C5_TK>(
            p, wl, wr, cin, cout, den, st);
    else
        return -4;
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
#endif

#ifdef EXP_VPX
// k_vpass10 at T = 35, den-read: block shape / occupancy experiments
//   -DEXP_VPX=<extra prefetch> -DVNW=<columns> -DVNPH=<phases> -DVRB=<rows per barrier> -DVPS=<staging rows> -DVWPE=<waves/EU>
#ifndef VNW
#define VNW 16
#define VNPH 2
#define VRB 2
#define VPS 4
#define VWPE 0
#endif
extern "C" int exp_vpx(int dm, const asw_params *p, const float *wl, const float *wr, const float *cin, float *cout,
                       float *den, void *stream) {
    hipStream_t st = (hipStream_t)stream;
    if (p->taps != 35 || dm != 2) return -4;
    constexpr int U = pf9_period(35) + EXP_VPX;
    const int W = p->width, H = p->height, Dp = asw_disp_pitch(p), nkb = Dp / 64, nxb = (W + VNW - 1) / VNW;
    int nstrip = (int)((2048LL + (long long)nxb * nkb - 1) / ((long long)nxb * nkb));
    const int max_strip = H / 70 > 1 ? H / 70 : 1;
    if (nstrip > max_strip) nstrip = max_strip;
    const int rows = ((H + nstrip - 1) / nstrip + U - 1) / U * U;
    nstrip = (H + rows - 1) / rows;
    const int per_xcd = (nxb + 7) / 8;
    hipLaunchKernelGGL((k_vpass10<35, VNW, DM_READ, VRB, kCPStream, kCPStream, 2, VPS, 0, VNPH, EXP_VPX, VWPE>),
                       dim3(8 * per_xcd * nkb * nstrip), dim3(VNW * 64), 0, st, wl, wr, cin, cout, den, W, H, Dp,
                       p->d_begin, rows, nxb, nstrip, per_xcd);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
#endif

#ifdef EXP_VTILE
// k_vpass10 den-read in XCD-round tiles (round 5): TK plane blocks x 32/TK column groups
// per round of 32 blocks, so a round shares its left-weight columns across its plane
// blocks and a band of right-weight entries.  T = 35 (C4
// shape, 16 columns) or 51 (C5 shape, 12 columns, 3 phases).
extern "C" int exp_vtile(int tk, const asw_params *p, const float *wl, const float *wr, const float *cin, float *cout,
                         float *den, void *stream) {
    hipStream_t st = (hipStream_t)stream;
    const int T = p->taps;
    if (T != 35 && T != 51) return -4;
    const int NW = T == 35 ? 16 : 12;
    const int U = T == 35 ? pf9_period(35) : pf9_period(51);
    const int W = p->width, H = p->height, Dp = asw_disp_pitch(p), nkb = Dp / 64, nxb = (W + NW - 1) / NW;
    int nstrip = (int)((2048LL + (long long)nxb * nkb - 1) / ((long long)nxb * nkb));
    const int max_strip = H / (2 * T) > 1 ? H / (2 * T) : 1;
    if (nstrip > max_strip) nstrip = max_strip;
    if (nstrip < 1) nstrip = 1;
    const int rows = ((H + nstrip - 1) / nstrip + U - 1) / U * U;
    nstrip = (H + rows - 1) / rows;
    const int per_xcd = (nxb + 7) / 8;
    auto grid = [&](int TKv) {
        const int tcg = 32 / TKv;
        return dim3(8 * 32 * ((nkb + TKv - 1) / TKv) * ((per_xcd + tcg - 1) / tcg) * nstrip);
    };
#define VT(TKV)                                                                                                      \
    if (tk == TKV) {                                                                                                 \
        if (T == 35)                                                                                                 \
            hipLaunchKernelGGL((k_vpass10<35, 16, DM_READ, 2, kCPStream, kCPStream, 2, 4, TKV, 2>), grid(TKV),       \
                               dim3(16 * 64), 0, st, wl, wr, cin, cout, den, W, H, Dp, p->d_begin, rows, nxb, nstrip, \
                               per_xcd);                                                                             \
        else                                                                                                         \
            hipLaunchKernelGGL((k_vpass10<51, 12, DM_READ, 2, kCPStream, kCPStream, 2, 4, TKV, 3>), grid(TKV),       \
                               dim3(12 * 64), 0, st, wl, wr, cin, cout, den, W, H, Dp, p->d_begin, rows, nxb, nstrip, \
                               per_xcd);                                                                             \
        return hipGetLastError() == hipSuccess ? 0 : -2;                                                             \
    }
    VT(1) VT(2) VT(4) VT(8)
#undef VT
    return -4;
}
#endif

#ifdef EXP_C5S
// C5 (T = 51) V den-read with an explicit row-strip count and dispatch order (round 4):
// whether strips short enough for the Infinity Cache to hold a strip's support rows
// while all plane blocks pass over it (the plane blocks re-fetch the support rows:
// 81 GB per launch against 54 compulsory, profiles/r04/pmc_c5_r09d.json) pay for their
// window prologue.  kbi = 1: the plane blocks of a column group adjacent in dispatch.
extern "C" int exp_c5s(int nstrip, int kbi, const asw_params *p, const float *wl, const float *wr, const float *cin,
                       float *cout, float *den, void *stream) {
    hipStream_t st = (hipStream_t)stream;
    if (p->taps != 51) return -4;
    constexpr int T = 51, NW = 12;
    constexpr int U = pf9_period(T);
    const int W = p->width, H = p->height, Dp = asw_disp_pitch(p), nkb = Dp / 64, nxb = (W + NW - 1) / NW;
    const int rows = ((H + nstrip - 1) / nstrip + U - 1) / U * U;
    nstrip = (H + rows - 1) / rows;
    const int per_xcd = (nxb + 7) / 8;
    if (kbi)
        hipLaunchKernelGGL((k_vpass10<T, NW, DM_READ, 2, kCPStream, kCPStream, 2, 4, 4, 3>),
                           dim3(8 * per_xcd * nkb * nstrip), dim3(NW * 64), 0, st, wl, wr, cin, cout, den, W, H, Dp,
                           p->d_begin, rows, nxb, nstrip, per_xcd);
    else
        hipLaunchKernelGGL((k_vpass10<T, NW, DM_READ, 2, kCPStream, kCPStream, 2, 4, 0, 3>),
                           dim3(8 * per_xcd * nkb * nstrip), dim3(NW * 64), 0, st, wl, wr, cin, cout, den, W, H, Dp,
                           p->d_begin, rows, nxb, nstrip, per_xcd);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
#endif

#ifdef EXP_H32
// k_hpass32 (C4 8-way shard, T = 35, DL left weights) occupancy (round 5, VERDICT r04
// item 2): the shipped form keeps the conflict-free 48-entry right ring (13.5 KB of LDS
// per wave: 11 waves per CU; 138 VGPRs would admit 12).  The minimal 40-entry ring
// (11.25 KB: 14 by LDS) with 3 or 4 waves per SIMD requested: form 0 = shipped (48, WPE 3),
// 1 = ring 40 / WPE 3, 2 = ring 40 / WPE 4, 3 = ring 48 / WPE 4.  nseg: segments per
// row pair (the work items; 0 = the shipped 256 x 11 wave-slot rule).
#include "asw_pass32.h"
extern "C" int exp_h32(int form, int nseg, int dm, const asw_params *p, const float *wl, const float *wr,
                       const float *cin, float *cout, float *den, void *stream) {
    hipStream_t st = (hipStream_t)stream;
    if (p->taps != 35 || dm != DM_NONE) return -4;
    constexpr int T = 35;
    const int U = pf9_period(35) + (form == 4 ? 8 : form == 5 ? 16 : 0);
    const int pairs = (p->height + 1) / 2;
    const int slots = form == 0 || form >= 3 ? 256 * 11 : 256 * (form == 1 ? 12 : 14);
    if (nseg <= 0) nseg = (slots + pairs / 2) / (pairs > 0 ? pairs : 1);
    int seg = ((p->width + nseg - 1) / nseg + U - 1) / U * U;
    if (seg < 2 * U) seg = 2 * U;
    if (form == 0) launch_h32<T, 1, DM_NONE, 0, 4, true, 3, 0, true>(p, wl, wr, cin, cout, den, st, seg);
    else if (form == 1) launch_h32<T, 1, DM_NONE, 0, 4, false, 3, 0, true>(p, wl, wr, cin, cout, den, st, seg);
    else if (form == 2) launch_h32<T, 1, DM_NONE, 0, 4, false, 4, 0, true>(p, wl, wr, cin, cout, den, st, seg);
    else if (form == 3) launch_h32<T, 1, DM_NONE, 0, 4, true, 4, 0, true>(p, wl, wr, cin, cout, den, st, seg);
    // round 6: the shipped form with a deeper cost prefetch (PX more steps: the newest
    // window element requested P = 5 + PX steps ahead; k_hpass32 waits on vmcnt, not LDS)
    else if (form == 4) launch_h32<T, 1, DM_NONE, 0, 4, true, 3, 0, true, 8>(p, wl, wr, cin, cout, den, st, seg);
    else if (form == 5) launch_h32<T, 1, DM_NONE, 0, 4, true, 3, 0, true, 16>(p, wl, wr, cin, cout, den, st, seg);
    else return -4;
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
#endif

#ifdef EXP_VPROBE
// k_vpass10 resource probes (round 6, asw_vprobe.h): probe 0 is bit-exact, every other
// probe removes one resource and is wrong by design (timed only)
#include "asw_vprobe.h"
extern "C" int exp_vprobe(int probe, int dm, const asw_params *p, const float *wl, const float *wr, const float *cin,
                          float *cout, float *den, void *stream) {
    hipStream_t st = (hipStream_t)stream;
    if (p->taps != 35) return -4;
#define VP(DMV, PR)                                                                                                  \
    if (dm == DMV && probe == PR) {                                                                                  \
        launch_vprobe<35, DMV, PR>(p, wl, wr, cin, cout, den, st);                                                  \
        return hipGetLastError() == hipSuccess ? 0 : -2;                                                             \
    }
    VP(0, 0) VP(0, 8)
    VP(2, 0) VP(2, 4) VP(2, 8) VP(2, 79)
    VP(0, 128) VP(1, 128) VP(2, 128)
#undef VP
    return -4;
}
// the production den-read V pass with a deeper den prefetch ring (KDV rows; 2 ships)
extern "C" int exp_vkd(int kd, const asw_params *p, const float *wl, const float *wr, const float *cin, float *cout,
                       float *den, void *stream) {
    hipStream_t st = (hipStream_t)stream;
    if (p->taps != 35) return -4;
    constexpr int U = pf9_period(35);
    const int W = p->width, H = p->height, Dp = asw_disp_pitch(p), nkb = Dp / 64, nxb = (W + 15) / 16;
    int nstrip = (int)((2048LL + (long long)nxb * nkb - 1) / ((long long)nxb * nkb));
    const int max_strip = H / 70 > 1 ? H / 70 : 1;
    if (nstrip > max_strip) nstrip = max_strip;
    if (nstrip < 1) nstrip = 1;
    const int rows = ((H + nstrip - 1) / nstrip + U - 1) / U * U;
    nstrip = (H + rows - 1) / rows;
    const int per_xcd = (nxb + 7) / 8;
#define VK(KDV)                                                                                                      \
    if (kd == KDV) {                                                                                                 \
        hipLaunchKernelGGL((k_vpass10<35, 16, DM_READ, 2, kCPStream, kCPStream, KDV>), dim3(8 * per_xcd * nkb * nstrip), \
                           dim3(1024), 0, st, wl, wr, cin, cout, den, W, H, Dp, p->d_begin, rows, nxb, nstrip, per_xcd); \
        return hipGetLastError() == hipSuccess ? 0 : -2;                                                             \
    }
    VK(4) VK(5) VK(8)
#undef VK
    return -4;
}
#endif

#ifdef EXP_VDMA
// the LDS-DMA-staged V pass (round 6, asw_vdma.h), every den mode; form = LEADS * 10 + NBUF / 2
#include "asw_vdma.h"
extern "C" int exp_vdma(int form, int dm, const asw_params *p, const float *wl, const float *wr, const float *cin,
                        float *cout, float *den, void *stream) {
    hipStream_t st = (hipStream_t)stream;
    if (p->taps != 35) return -4;
#define VD(F, LE, NB)                                                                                                \
    if (form == F) {                                                                                                 \
        if (dm == 0) launch_vdma<35, DM_NONE, LE, 2, NB>(p, wl, wr, cin, cout, den, st);                             \
        else if (dm == 1) launch_vdma<35, DM_WRITE, LE, 2, NB>(p, wl, wr, cin, cout, den, st);                       \
        else launch_vdma<35, DM_READ, LE, 2, NB>(p, wl, wr, cin, cout, den, st);                                     \
        return hipGetLastError() == hipSuccess ? 0 : -2;                                                             \
    }
    VD(64, 6, 8)
#undef VD
    return -4;
}
#endif

#ifdef EXP_HWTA
// the last H pass with the WTA's own scan fused by DPP reductions (round 6, asw_hwta.h)
#include "asw_hwta.h"
extern "C" int exp_hwta(int vg, const asw_params *p, const float *wl, const float *wr, const float *cin, float *cout,
                        float *den, long long *key, float *m1, float *m2, void *stream) {
    if (p->taps != 35) return -4;
    const int Dp = asw_disp_pitch(p);
    constexpr int U = pf9_period(35);
    const int seg = ((240 + U / 2) / U) * U;
    hipStream_t st = (hipStream_t)stream;
    if (Dp == 256 && vg == 0) launch_h11_wr<35, 4, 0>(p, wl, wr, cin, cout, den, key, m1, m2, st, seg);
    else if (Dp == 256 && vg == 1) launch_h11_wr<35, 4, 1>(p, wl, wr, cin, cout, den, key, m1, m2, st, seg);
    else if (Dp == 128 && vg == 0) launch_h11_wr<35, 2, 0>(p, wl, wr, cin, cout, den, key, m1, m2, st, seg);
    else return -4;
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
#endif

#ifdef EXP_HS
// Half-size tap-major supports on the 32-plane shard V pass:
// exp_hs_convert writes the [H][R+1][W] half of a full [H][W][Tp] V support array,
// exp_hs_expand rebuilds a full array from a half one through hs_index (the symmetry
// and border rule, checked element for element by tools/exp/hs_bench.py), exp_v32hs
// runs k_vpass32 on the full (hs 0) or half (hs 1) arrays.
#include "asw_pass32.h"
__global__ void k_hs_convert(const float *__restrict__ full, float *__restrict__ half, int W, int H) {
    constexpr int T = 35, R = T / 2, TP = asw::tap_pitch(T);
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y, u = blockIdx.z;
    if (x >= W) return;
    half[((long long)y * (R + 1) + u) * W + x] = full[((long long)y * W + x) * TP + R + u];
}
__global__ void k_hs_expand(const float *__restrict__ half, float *__restrict__ full, int W, int H) {
    constexpr int T = 35, TP = asw::tap_pitch(T);
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y, t = blockIdx.z;
    if (x >= W) return;
    full[((long long)y * W + x) * TP + t] = t < T ? half[hs_index<T>(y, t, x, W)] : 0.0f;
}
extern "C" int exp_hs_convert(int expand, const float *src, float *dst, int W, int H, void *stream) {
    constexpr int T = 35, R = T / 2;
    const dim3 grid((W + 255) / 256, H, expand ? asw::tap_pitch(T) : R + 1);
    if (expand) hipLaunchKernelGGL(k_hs_expand, grid, dim3(256), 0, (hipStream_t)stream, src, dst, W, H);
    else hipLaunchKernelGGL(k_hs_convert, grid, dim3(256), 0, (hipStream_t)stream, src, dst, W, H);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
extern "C" int exp_v32hs(int hs, const asw_params *p, const float *wl, const float *wr, const float *cin, float *cout,
                         void *stream) {
    hipStream_t st = (hipStream_t)stream;
    if (p->taps != 35) return -4;
    if (hs) launch_v32<35, 16, DM_NONE, 0, 4, false, true>(p, wl, wr, cin, cout, nullptr, st);
    else launch_v32<35, 16, DM_NONE, 0, 4, false, false>(p, wl, wr, cin, cout, nullptr, st);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
#endif

#ifdef EXP_HPX
// k_hpass11 den-read with a deeper cost prefetch (PX more steps) and other segment
// lengths (round 6; the 32-plane H pass gained from PX = 8).  form: T = 51 (C5, 2 plane
// blocks per block) 0 = shipped (PX 0, 224-column segments), 1 = PX 8 / 256, 2 = PX 0 /
// 256, 3 = PX 8 / 192, 4 = PX 16 / 288; T = 35 (C4, 4 plane blocks) 10 = shipped
// (PX 0 / 240), 11 = PX 8 / 240.
extern "C" int exp_hpx(int form, const asw_params *p, const float *wl, const float *wr, const float *cin, float *cout,
                       float *den, void *stream) {
    hipStream_t st = (hipStream_t)stream;
    if (form < 10 && p->taps == 51) {
        constexpr int T = 51;
        if (form == 0) launch_h11<T, 2, DM_READ, kCPStream, kCPStream, 0>(p, wl, wr, cin, cout, den, st, 224);
        else if (form == 1) launch_h11<T, 2, DM_READ, kCPStream, kCPStream, 8>(p, wl, wr, cin, cout, den, st, 256);
        else if (form == 2) launch_h11<T, 2, DM_READ, kCPStream, kCPStream, 0>(p, wl, wr, cin, cout, den, st, 256);
        else if (form == 3) launch_h11<T, 2, DM_READ, kCPStream, kCPStream, 8>(p, wl, wr, cin, cout, den, st, 192);
        else if (form == 4) launch_h11<T, 2, DM_READ, kCPStream, kCPStream, 16>(p, wl, wr, cin, cout, den, st, 288);
        else if (form == 5) launch_h11<T, 2, DM_READ, kCPStream, kCPStream, 16, 8>(p, wl, wr, cin, cout, den, st, 288);
        else if (form == 6) launch_h11<T, 2, DM_READ, kCPStream, kCPStream, 24>(p, wl, wr, cin, cout, den, st, 320);
        else if (form == 7) launch_h11<T, 2, DM_READ, kCPStream, kCPStream, 0, 8>(p, wl, wr, cin, cout, den, st, 224);
        else if (form == 8) launch_h11<T, 2, DM_READ, kCPStream, kCPStream, 16>(p, wl, wr, cin, cout, den, st, 216);
        else return -4;
    } else if (form >= 10 && p->taps == 35) {
        constexpr int T = 35;
        if (form == 10) launch_h11<T, 4, DM_READ, kCPStream, kCPStream, 0>(p, wl, wr, cin, cout, den, st, 240);
        else if (form == 11) launch_h11<T, 4, DM_READ, kCPStream, kCPStream, 8>(p, wl, wr, cin, cout, den, st, 240);
        else return -4;
    } else {
        return -4;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
#endif

#ifdef EXP_C5VPX
// C5 (T = 51) V den-read, the shipped 12-column tiled shape, with a deeper cost prefetch
// (PX more steps; round 6, after the H passes gained from it) and / or one barrier per
// row (RB = 1: a 2-row staging ring, 16 fewer VGPRs; the shipped form spills 11 at the
// 168-VGPR cap of 3 waves per SIMD).  form = PX * 10 + RB.
template <int PX, int RB>
static void c5v_px(const asw_params *p, const float *wl, const float *wr, const float *cin, float *cout, float *den,
                   hipStream_t st) {
    constexpr int T = 51, NW = 12, TK = 4, U = pf9_period(T) + PX, PS = RB == 1 ? 2 : 4;
    const int W = p->width, H = p->height, Dp = asw_disp_pitch(p), nkb = Dp / 64, nxb = (W + NW - 1) / NW;
    int nstrip = (int)((2048LL + (long long)nxb * nkb - 1) / ((long long)nxb * nkb));
    const int max_strip = H / (2 * T) > 1 ? H / (2 * T) : 1;
    if (nstrip > max_strip) nstrip = max_strip;
    if (nstrip < 1) nstrip = 1;
    const int rows = ((H + nstrip - 1) / nstrip + U - 1) / U * U;
    nstrip = (H + rows - 1) / rows;
    const int per_xcd = (nxb + 7) / 8;
    constexpr int TCG = 32 / TK;
    const int nblocks = 8 * 32 * ((nkb + TK - 1) / TK) * ((per_xcd + TCG - 1) / TCG) * nstrip;
    hipLaunchKernelGGL((k_vpass10<T, NW, DM_READ, RB, kCPStream, kCPStream, 2, PS, TK, 3, PX>), dim3(nblocks),
                       dim3(NW * 64), 0, st, wl, wr, cin, cout, den, W, H, Dp, p->d_begin, rows, nxb, nstrip, per_xcd);
}
extern "C" int exp_c5vpx(int form, const asw_params *p, const float *wl, const float *wr, const float *cin,
                         float *cout, float *den, void *stream) {
    hipStream_t st = (hipStream_t)stream;
    if (p->taps != 51) return -4;
    if (form == 2) c5v_px<0, 2>(p, wl, wr, cin, cout, den, st);
    else if (form == 1) c5v_px<0, 1>(p, wl, wr, cin, cout, den, st);
    else if (form == 81) c5v_px<8, 1>(p, wl, wr, cin, cout, den, st);
    else return -4;
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
#endif

#ifdef EXP_HPXW
// C5 (T = 51) den-write H pass with the deeper cost prefetch of the shipped den-read form
// (round 6): form 20 = shipped (PX 0, 224), 21 = PX 24 / 320, 22 = PX 16 / 288
extern "C" int exp_hpxw(int form, const asw_params *p, const float *wl, const float *wr, const float *cin,
                        float *cout, float *den, void *stream) {
    hipStream_t st = (hipStream_t)stream;
    if (p->taps != 51) return -4;
    constexpr int T = 51;
    if (form == 20) launch_h11<T, 2, DM_WRITE, kCPStream, kCPStream, 0>(p, wl, wr, cin, cout, den, st, 224);
    else if (form == 21) launch_h11<T, 2, DM_WRITE, kCPStream, kCPStream, 24>(p, wl, wr, cin, cout, den, st, 320);
    else if (form == 22) launch_h11<T, 2, DM_WRITE, kCPStream, kCPStream, 16>(p, wl, wr, cin, cout, den, st, 288);
    else return -4;
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
#endif
