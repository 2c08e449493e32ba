// asw_vpass11.h — V aggregation pass with column pairs sharing their right weights
// (K/asw_vcost_aggregation.cl:11-44; one launch of main.cpp:494-500).
//
// Why: in k_vpass10 every voxel-tap reads its right weight wr_i(x-d, y) from LDS
// (4 B per voxel-tap, ds_read_b128 for 4 taps) and the per-row slab staging adds
// ~26 % on top; with the den cache a voxel-tap costs 2 VALU, so the LDS pipe, not the
// VALU nor HBM, paced the pass (tools/ubench/vexp.hip, profiles/r03).  Voxels
// (x, d) and (x+1, d+1) share the entry x-d, so here a wave owns TWO columns:
//   A = (xa, kb + l), B = (xa + 1, kb + l + 1), lane l,
// and one set of right-weight registers serves both: half the LDS reads per voxel.
// B's planes run [kb+1, kb+64]: plane Dp (lane 63 of the last plane block) does not
// exist and plane 0 of column xa+1 is not covered, so that lane computes plane 0
// instead, with its own right-weight entry (xa + 1 - d_begin) from a per-wave
// "special" slab entry: the waves of the last plane block re-read their right
// weights for the B phases (lane 63 at the special entry), the others reuse A's.
//
// Per step (one row y) a wave runs four phases, each with its weights requested one
// phase ahead (one lgkmcnt(0) per phase; SMEM and LDS share the counter):
//     A taps [0,TA) | A taps [TA,T) | B taps [0,TA) | B taps [TA,T)
// left weights wl_A / wl_B: SGPRs (two buffers of TA and TB floats alternate);
// right weights: wra (taps [0,TA)) serves phases 1 and 3, wrb phases 2 and 4.
//
// The slab rows reach LDS by LDS-DMA (buffer_load_dwordx4 ... lds, issued from
// inline asm so the compiler adds no vmcnt(0) before every LDS read): row y + LEAD is
// requested at step y, LEAD = RB + 1 + P rows ahead, into a ring of NBUF buffers.
// A wave knows its own DMAs have landed when the window element loaded P steps
// after them has (vmcnt retires in issue order); the block barrier every RB rows
// then publishes the rows to every wave.  No VGPR staging.
//
// Same FP sequence as every other pass (DESIGN.md §FP policy): bit-identical.
#pragma once
#include <cstdint>

#include "asw_aggregate_impl.h"

namespace asw {
namespace agg {

// LDS byte address of a __shared__ object (the low 32 bits of its flat address)
__device__ __forceinline__ unsigned lds_addr(const void *p) { return (unsigned)(uintptr_t)p; }

// one 1-KB LDS-DMA per wave: lane i's 16 bytes at rsrc + voff_i + soff land at
// LDS m0 + 16 i (exec-masked lanes write nothing)
__device__ __forceinline__ void dma16(unsigned lds, int voff, rsrc_t r, int soff) {
    asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds" ::"s"(lds), "v"(voff), "s"(r),
                 "s"(soff)
                 : "memory");
}

// float4 per slab row of k_vpass11: the 2 NW + 63 shared entries and NW special
// ones, padded to whole 1-KB DMA pieces
constexpr int v11_nq(int T, int NW) { return ((2 * NW + 63 + NW) * (tap_pitch(T) / 4) + 63) / 64 * 64; }

template <int T, int NW, int DM, int RB, int CP, int CPS, bool LK>
__device__ __forceinline__ void vpass11_body(const float *__restrict__ wl, const float *__restrict__ wr,
                                             const float *__restrict__ cin, float *__restrict__ cout,
                                             float *__restrict__ den, int W, int H, int Dp, int d_begin, int x0,
                                             int y_begin, int y_end, int kb, f4 (*slab)[v11_nq(T, NW)],
                                             f4 *wdump) {
    constexpr int R = T / 2;
    constexpr int TP = tap_pitch(T);
    constexpr int Q = TP / 4;
    constexpr int U = pf9_period(T);
    constexpr int P = U - T;
    constexpr int KD = 2;  // den prefetch ring (rows)
    constexpr int LEAD = RB + 1 + P;
    constexpr int NBUF = ring_div(U, LEAD + RB);
    constexpr int NC = 2 * NW;
    constexpr int SLAB = NC + 63;
    constexpr int NQ = v11_nq(T, NW);
    constexpr int NR = (NQ + NW * 64 - 1) / (NW * 64);
    constexpr int LA = cmax(cmax(R + P, LEAD), KD);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // A = column xa (clamped: a wave past the right edge recomputes column W-1, like
    // k_vpass10, storing the same values again); when xa + 1 is past the edge, B := A
    // (the same voxel, stored twice)
    const int xa = min(x0 + 2 * wave, W - 1);
    const bool b_live = x0 + 2 * wave + 1 < W;
    const int xb = b_live ? xa + 1 : xa;
    const int slab_base = x0 - (d_begin + kb) - 63;  // virtual xr of slab entry 0
    const int my_entry = ((xa - x0) + 63 - lane) * Q;
    // B's right weights: A's, except lane 63 of the last plane block (plane 0 of xb)
    const int b_entry = LK && b_live && lane == 63 ? (SLAB + wave) * Q : my_entry;
    const long long rowstride = (long long)W * Dp;
    const int rowbytes = (int)(rowstride * 4);  // U+LA rows < 2 GiB: checked by the launcher
    // one buffer resource per volume and chunk, based at column xa plane 0; B's
    // voxels are (xb - xa) columns further (SGPR budget: no second descriptor)
    const long long colA = (long long)xa * Dp;
    const int voffA = (kb + lane) * 4;
    const int kB = kb + lane + 1;
    const int voffB = b_live ? ((xb - xa) * Dp + (kB == Dp ? 0 : kB)) * 4  // lane 63 of the last plane block: plane 0
                             : voffA;
    const int wrow = W * TP;
    const int wrow_b = wrow * 4;
    const rsrc_t rwr = make_rsrc(wr);
    const float *wlA = wl + (long long)xa * TP;
    const float *wlB = wl + (long long)xb * TP;
    auto rsrc_at = [&](const float *base, int row) __attribute__((always_inline)) {
        return make_rsrc(base + (long long)row * rowstride + colA);
    };

    // LDS-DMA of a slab row: 64 NW float4 (one 1-KB piece per wave) and the rest (NQ
    // - 64 NW: the special entries, padding to whole pieces) by the first waves as a
    // second piece; every lane live (no exec masking), reading valid (clamped) entries.
    // The left-weight rows the scalar loads will read (wl of columns [x0, x0 + NC),
    // contiguous) are pulled into L2 LEAD rows ahead by the last waves' second piece,
    // into a scratch LDS tile nobody reads: no VGPR ring, no wait (k_vpass10's "warm"
    // loads).  One VGPR per lane and piece: the second piece's meaning is per wave.
    static_assert(NQ <= 2 * 64 * NW, "at most two slab pieces per wave");
    constexpr int WLP = (NC * TP * 4 + 1023) / 1024;  // 1-KB pieces of a wl row chunk
    constexpr int N2 = (NQ - 64 * NW) / 64;             // second slab pieces (waves [0, N2))
    static_assert(N2 + WLP <= NW, "second pieces: slab remainder and wl prefetch");
    auto slab_src = [&](int t) __attribute__((always_inline)) {
        const int e = t / Q, q = t - (t / Q) * Q;
        int src;
        if (e < SLAB) src = clampi(slab_base + e, 0, W - 1);
        else src = clampi(x0 + 2 * min(e - SLAB, NW - 1) + 1 - d_begin, 0, W - 1);
        return (src * TP + 4 * q) * 4;
    };
    const int dvoff0 = slab_src(threadIdx.x);
    const int wl_piece = NW - 1 - wave;  // waves [NW - WLP, NW): the wl prefetch
    const bool has2 = wave < N2 || wl_piece < WLP;  // wave-uniform
    const int dvoff1 = wave < N2 ? slab_src(threadIdx.x + 64 * NW)
                                 : min(x0 * TP * 4 + wl_piece * 1024 + lane * 16, (W * TP - 4) * 4);
    const rsrc_t r2 = make_rsrc(wave < N2 ? wr : wl);
    const unsigned lds1 = wave < N2 ? 0u : lds_addr(wdump);  // + the slab buffer's piece for the first waves
    auto dma_row = [&](int buf, int row) __attribute__((always_inline)) {
        const int soff = row * wrow_b;
        dma16(lds_addr(&slab[buf][wave * 64]), dvoff0, rwr, soff);
        if (has2) dma16(wave < N2 ? lds_addr(&slab[buf][(NW + wave) * 64]) : lds1, dvoff1, r2, soff);
    };

#ifdef V11_PROBE_WL0  // diagnostic builds only (tools/exp): left weights always from row 0, results WRONG
#define V11_WO(x) 0
#else
#define V11_WO(x) (x)
#endif
    using HV = Halves<T>;
    float winA[U], winB[U];
    float wlx[HV::NA], wly[HV::NB];
    f4 wra[HV::MA], wrb[HV::MB];
    float dringA[KD], dringB[KD];
    {
        const int r0 = max(0, y_begin - R);
        const rsrc_t ra = rsrc_at(cin, r0);
#pragma unroll
        for (int j = 0; j < U - 1; ++j) {
            const int o = (clampi(y_begin - R + j, 0, H - 1) - r0) * rowbytes;
            winA[j] = bload<CP>(ra, voffA, o);
            winB[j] = bload<CP>(ra, voffB, o);
        }
    }
    if constexpr (DM == DM_READ) {
        const rsrc_t ra = rsrc_at(den, y_begin);
#pragma unroll
        for (int j = 0; j < KD; ++j) {
            const int o = (min(y_begin + j, H - 1) - y_begin) * rowbytes;
            dringA[j] = bload<CP>(ra, voffA, o);
            dringB[j] = bload<CP>(ra, voffB, o);
        }
    }
#pragma unroll
    for (int j = 0; j < LEAD; ++j) dma_row(j, min(y_begin + j, H - 1));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    load_wl<0, HV::TA>(wlx, wlA + (long long)y_begin * wrow);
    read_wr<T, 0, HV::QA>(wra, &slab[0][my_entry]);

    auto chunk = [&](auto clamp_c, int ys) __attribute__((always_inline)) {
        constexpr bool CLAMP = decltype(clamp_c)::value;
        const int cb = min(ys + R + P, H - 1);
        const rsrc_t rc = rsrc_at(cin, cb);
        const rsrc_t ro = rsrc_at(cout, ys);
        const rsrc_t rd = rsrc_at(den, ys);
        int so = 0;              // (y - ys) * rowbytes
        int wo = ys * wrow;      // left weights of row y
        static_for<0, U>([&](auto sc) __attribute__((always_inline)) {
            constexpr int s = decltype(sc)::value;
            const int y = ys + s;
            if constexpr (CLAMP) {
                if (y >= y_end) return;
            }
            constexpr int bcur = s % NBUF, bnext = (s + 1) % NBUF, bput = (s + LEAD) % NBUF;
            // phase A1's weights (wlx = wl_A[0,TA), wra) are in; rows up to y+RB in LDS
            if constexpr (s % RB == 0) __syncthreads();
            else wait_lgkm0();
            asm volatile("" ::"v"(winA[(s + T - 1) % U]), "v"(winB[(s + T - 1) % U]));
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (HV::TB > 0) {
                load_wl<HV::TA, T>(wly, wlA + V11_WO(wo));
                read_wr<T, HV::QA, HV::QT>(wrb, &slab[bcur][my_entry]);
            }
            dma_row(bput, CLAMP ? min(y + LEAD, H - 1) : y + LEAD);
            __builtin_amdgcn_sched_barrier(0);
            float numA = 1e-5f, dnA = 1e-5f, numB = 1e-5f, dnB = 1e-5f;
            taps<U, s, 0, HV::TA, DM != DM_READ>(numA, dnA, wlx, wra, winA);  // A1
            __builtin_amdgcn_sched_barrier(0);
            wait_lgkm0();
            __builtin_amdgcn_sched_barrier(0);
            load_wl<0, HV::TA>(wlx, wlB + V11_WO(wo));
            if constexpr (LK) read_wr<T, 0, HV::QA>(wra, &slab[bcur][b_entry]);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (HV::TB > 0) taps<U, s, HV::TA, T, DM != DM_READ>(numA, dnA, wly, wrb, winA);  // A2
            __builtin_amdgcn_sched_barrier(0);
            wait_lgkm0();
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (HV::TB > 0) {
                load_wl<HV::TA, T>(wly, wlB + V11_WO(wo));
                if constexpr (LK) read_wr<T, HV::QA, HV::QT>(wrb, &slab[bcur][b_entry]);
            }
            __builtin_amdgcn_sched_barrier(0);
            taps<U, s, 0, HV::TA, DM != DM_READ>(numB, dnB, wlx, wra, winB);  // B1
            __builtin_amdgcn_sched_barrier(0);
            wait_lgkm0();
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (CLAMP) {
                wo = min(y + 1, H - 1) * wrow;
            } else {
                wo += wrow;
                asm volatile("" : "+s"(wo));
            }
            load_wl<0, HV::TA>(wlx, wlA + V11_WO(wo));
            read_wr<T, 0, HV::QA>(wra, &slab[bnext][my_entry]);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (HV::TB > 0) taps<U, s, HV::TA, T, DM != DM_READ>(numB, dnB, wly, wrb, winB);  // B2
            if constexpr (DM == DM_READ) {
                dnA = dringA[s % KD];
                dnB = dringB[s % KD];
                const int o = CLAMP ? (min(y + KD, H - 1) - ys) * rowbytes : so + KD * rowbytes;
                dringA[s % KD] = bload<CP>(rd, voffA, o);
                dringB[s % KD] = bload<CP>(rd, voffB, o);
            } else if constexpr (DM == DM_WRITE) {
                bstore<CPS>(dnA, rd, voffA, so);
                bstore<CPS>(dnB, rd, voffB, so);
            }
            bstore<CPS>(div_pos(numA, dnA), ro, voffA, so);
            bstore<CPS>(div_pos(numB, dnB), ro, voffB, so);
            {
                const int o = CLAMP ? (min(y + R + P, H - 1) - cb) * rowbytes : so;
                winA[(s + U - 1) % U] = bload<CP>(rc, voffA, o);
                winB[(s + U - 1) % U] = bload<CP>(rc, voffB, o);
            }
            so += rowbytes;
            asm volatile("" : "+s"(so));
        });
    };
    int ys = y_begin;
    for (; ys + U <= y_end && ys + U - 1 + LA <= H - 1; ys += U) chunk(std::false_type{}, ys);
    for (; ys < y_end; ys += U) {
        asm volatile("" : "+s"(ys));
        chunk(std::true_type{}, ys);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA outlives the block
}

template <int T, int NW, int DM, int RB, int CP, int CPS = CP>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(NW * 64 / 256))) void k_vpass11(
    const float *__restrict__ wl, const float *__restrict__ wr, const float *__restrict__ cin, float *__restrict__ cout,
    float *__restrict__ den, int W, int H, int Dp, int d_begin, int rows_per_strip, int nxb, int nstrip,
    int xg_per_xcd) {
    constexpr int U = pf9_period(T);
    constexpr int LEAD = RB + 1 + (U - T);
    constexpr int NBUF = ring_div(U, LEAD + RB);
    constexpr int NQ = v11_nq(T, NW);
    static_assert(U % 4 == 0 && U % 2 == 0 && U % RB == 0 && U % NBUF == 0, "ring periods");
    static_assert(NBUF * NQ * 16 + 1024 <= 160 * 1024, "slab ring exceeds the gfx950 LDS");
    __shared__ f4 slab[NBUF][NQ];
    __shared__ f4 wdump[64];  // L2-prefetch sink of the wl row DMAs (never read)

    const int nkb = Dp / 64;
    const int xcd = blockIdx.x & 7, m = blockIdx.x >> 3;
    const int xg = xcd * xg_per_xcd + m % xg_per_xcd;
    const int rest = m / xg_per_xcd;
    const int kbi = rest % nkb, strip = rest / nkb;
    if (xg >= nxb || strip >= nstrip) return;  // padding block (uniform)
    const int x0 = xg * 2 * NW;
    const int y_begin = strip * rows_per_strip;
    if (y_begin >= H) return;
    const int y_end = min(H, y_begin + rows_per_strip);
    const int kb = kbi * 64;
    if (kbi == nkb - 1) vpass11_body<T, NW, DM, RB, CP, CPS, true>(wl, wr, cin, cout, den, W, H, Dp, d_begin, x0,
                                                                     y_begin, y_end, kb, slab, wdump);
    else vpass11_body<T, NW, DM, RB, CP, CPS, false>(wl, wr, cin, cout, den, W, H, Dp, d_begin, x0, y_begin, y_end,
                                                    kb, slab, wdump);
}

template <int T, int NW, int DM, int RB, int CP, int CPS = CP>
void launch_v11(const asw_params *p, const float *wl, const float *wr, const float *cin, float *cout, float *den,
                hipStream_t st, int nstrip_req = 0) {
    constexpr int U = pf9_period(T);
    constexpr int NC = 2 * NW;
    const int W = p->width, H = p->height;
    const int Dp = round_up(d_end_of_p(p) - p->d_begin, 64);
    const int nkb = Dp / 64;
    const int nxb = (W + NC - 1) / NC;
    int nstrip = nstrip_req;
    if (nstrip <= 0) {  // about 2048 blocks, strips >= 2T rows (as k_vpass10)
        nstrip = (int)((2048LL + (long long)nxb * nkb - 1) / ((long long)nxb * nkb));
        const int max_strip = H / (2 * T) > 1 ? H / (2 * T) : 1;
        if (nstrip > max_strip) nstrip = max_strip;
        if (nstrip < 1) nstrip = 1;
    }
    const int rows = ((H + nstrip - 1) / nstrip + U - 1) / U * U;
    nstrip = (H + rows - 1) / rows;
    const int per_xcd = (nxb + 7) / 8;
    const int nblocks = 8 * per_xcd * nkb * nstrip;
    hipLaunchKernelGGL((k_vpass11<T, NW, DM, RB, CP, CPS>), dim3(nblocks), dim3(NW * 64), 0, st, wl, wr, cin, cout,
                       den, W, H, Dp, p->d_begin, rows, nxb, nstrip, per_xcd);
}

}  // namespace agg
}  // namespace asw
