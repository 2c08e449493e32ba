// Diagnostic copy of k_vpass10 (the C4 shape: NPH = 2, no raw / uint16 input, default
// block order) with probe switches that remove one resource at a time.  Results are
// WRONG by design for every probe but 0; only the time is measured
// (tools/exp/exp_bench.py --vprobe).  Round 6: which resource serialises the den-none
// V pass (1.94 ms against ~0.9 ms of VALU issue and ~0.9 ms of compulsory HBM).
//   PROBE bits  1: cost window loads from the chunk's first row (L2-resident)
//               2: output stores to the chunk's first row
//               4: slab rows staged from support row 0
//               8: left weights from support row 0
//              16: 4 taps per half computed (VALU cut to ~1/4)
//              32: no barrier in the sweep (LDS races)
//              64: den loads from the chunk's first row (den-read)
//             128: NOT a probe, bit-exact: waves 8-15 cross each barrier half a step later
//                  in their step than waves 0-7 (after their half-A taps), so the two
//                  groups run half a step apart and one group's LDS requests and waits
//                  overlap the other's taps; NBUF = 8 (a put then overwrites a row whose
//                  last readers passed an earlier barrier of both groups)
#pragma once
#include "asw_aggregate_impl.h"

namespace asw {
namespace agg {

template <int T, int DM, int PROBE>
__global__ __launch_bounds__(16 * 64) __attribute__((amdgpu_waves_per_eu(4))) void k_vprobe(
    const float *__restrict__ wl, const float *__restrict__ wr, const float *__restrict__ cin, float *__restrict__ cout,
    float *__restrict__ den, int W, int H, int Dp, int d_begin, int rows_per_strip, int nxb, int nstrip,
    int xg_per_xcd) {
    constexpr int NW = 16, RB = 2, CP = kCPStream, CPS = kCPStream;
    constexpr bool PC = PROBE & 1, PO = PROBE & 2, PSL = PROBE & 4, PWL = PROBE & 8, PV = PROBE & 16,
                   PNB = PROBE & 32, PD = PROBE & 64, STAG = PROBE & 128;
    constexpr int R = T / 2;
    constexpr int TP = tap_pitch(T);
    constexpr int Q = TP / 4;
    constexpr int U = pf9_period(T);
    constexpr int P = U - T;
    constexpr int PS = 4, PW = 4, KD = 2;
    constexpr int LEAD = RB + 1;
    constexpr int NBUF = STAG ? ring_div(U, 3 * RB + 2) : ring_div(U, 2 * RB + 1);
    constexpr int LA = cmax(cmax(R + P, LEAD + PS), cmax(PW, KD));
    constexpr int SLAB = NW + 63;
    constexpr int NQ = SLAB * Q;
    static_assert(NQ <= NW * 64, "one float4 per thread");
    __shared__ f4 slab[NBUF][NQ];

    const int nkb = Dp / 64;
    const int xcd = blockIdx.x & 7, m = blockIdx.x >> 3;
    const int xg = xcd * xg_per_xcd + m % xg_per_xcd;
    const int rest = m / xg_per_xcd;
    const int kbi = rest % nkb;
    const int strip = rest / nkb;
    if (xg >= nxb || strip >= nstrip) return;
    const int x0 = xg * NW;
    const int y_begin = strip * rows_per_strip;
    if (y_begin >= H) return;
    const int y_end = min(H, y_begin + rows_per_strip);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool late = STAG && wave >= NW / 2;  // (uniform) the group that crosses barriers mid-step
    const int kb = kbi * 64;
    const int x = min(x0 + wave, W - 1);
    const int slab_base = x0 - (d_begin + kb) - 63;
    const int my_entry = ((x - x0) + 63 - lane) * Q;
    const long long rowstride = (long long)W * Dp;
    const int rowbytes = (int)(rowstride * 4);
    const long long colbase = (long long)x * Dp + kb;
    const int voff = lane * 4;
    const int wrow = W * TP;
    const int wrow_b = wrow * 4;
    const rsrc_t rwr = make_rsrc(wr);
    const rsrc_t rwl = make_rsrc(wl + (long long)x * TP);
    const float *wlcol = wl + (long long)x * TP;
    auto rsrc_at = [&](const float *base, int row) __attribute__((always_inline)) {
        return make_rsrc(base + (long long)row * rowstride + colbase);
    };
    const int warm_voff = (lane < TP ? lane : 0) * 4;
    const int t0 = min((int)threadIdx.x, NQ - 1);
    const int sv0 = (clampi(slab_base + t0 / Q, 0, W - 1) * TP + 4 * (t0 % Q)) * 4;
    auto stage = [&](f4 &a, int roff) __attribute__((always_inline)) { a = bload4(rwr, sv0, PSL ? 0 : roff); };
    auto put = [&](int buf, const f4 &a) __attribute__((always_inline)) { slab[buf][t0] = a; };

    using HV = Halves<T>;
    float win[U];
    f4 sa[PS];
    float warm[PW];
    float sink = 0.0f;
    float wla[HV::NA], wlb[HV::NB];
    f4 wra[HV::MA], wrb[HV::MB];
    float dring[KD];
    {
        const int r0 = max(0, y_begin - R);
        const rsrc_t rp = rsrc_at(cin, r0);
#pragma unroll
        for (int j = 0; j < U - 1; ++j) win[j] = bload<CP>(rp, voff, (clampi(y_begin - R + j, 0, H - 1) - r0) * rowbytes);
    }
    if constexpr (DM == DM_READ) {
        const rsrc_t rp = rsrc_at(den, y_begin);
#pragma unroll
        for (int j = 0; j < KD; ++j) dring[j] = bload<CP>(rp, voff, (min(y_begin + j, H - 1) - y_begin) * rowbytes);
    }
#pragma unroll
    for (int j = 0; j < PS; ++j) stage(sa[j], min(y_begin + j, H - 1) * wrow_b);
#pragma unroll
    for (int j = 0; j < PW; ++j) warm[j] = bload(rwl, warm_voff, min(y_begin + j, H - 1) * wrow_b);
#pragma unroll
    for (int j = 0; j < LEAD; ++j) put(j, sa[j]);
#pragma unroll
    for (int j = 0; j < LEAD; ++j) stage(sa[j], min(y_begin + PS + j, H - 1) * wrow_b);
    __syncthreads();
    load_wl<0, HV::TA>(wla, wlcol + (PWL ? 0 : (long long)y_begin * wrow));
    read_wr<T, 0, HV::QA>(wra, &slab[0][my_entry]);

    constexpr int TAE = PV ? 4 : HV::TA;
    constexpr int TBE = PV ? HV::TA + 4 : T;
    auto chunk = [&](auto mode_c, int ys) __attribute__((always_inline)) {
        constexpr bool CLAMP = decltype(mode_c)::value >= 1;
        constexpr bool PART = decltype(mode_c)::value == 2;
        const int cb = min(ys + R + P, H - 1);
        const rsrc_t rc = rsrc_at(cin, cb);
        const rsrc_t ro = rsrc_at(cout, ys);
        const rsrc_t rdn = rsrc_at(den, min(ys + KD, H - 1));
        int so = 0;
        int wo = PWL ? 0 : ys * wrow;
        int woff = (ys + PW) * wrow_b;
        int soff = (ys + LEAD + PS) * wrow_b;
        static_for<0, U>([&](auto sc) __attribute__((always_inline)) {
            constexpr int s = decltype(sc)::value;
            const int y = ys + s;
            if constexpr (PART) {
                if (y >= y_end) return;
            }
            constexpr int bcur = s % NBUF, bnext = (s + 1) % NBUF, bput = (s + LEAD) % NBUF;
            float num = 1e-5f, dn = 1e-5f;
            if constexpr (s % RB == 0 && !PNB) {
                if (late) wait_lgkm0();
                else __syncthreads();
            } else {
                wait_lgkm0();
            }
            asm volatile("" ::"v"(win[(s + T - 1) % U]));
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (HV::TB > 0) {
                load_wl<HV::TA, T>(wlb, wlcol + wo);
                read_wr<T, HV::QA, HV::QT>(wrb, &slab[bcur][my_entry]);
            }
            put(bput, sa[(s + LEAD) % PS]);
            stage(sa[(s + LEAD) % PS], CLAMP ? min(y + LEAD + PS, H - 1) * wrow_b : soff);
            __builtin_amdgcn_sched_barrier(0);
            taps<U, s, 0, TAE, DM != DM_READ>(num, dn, wla, wra, win);
            __builtin_amdgcn_sched_barrier(0);
            wait_lgkm0();
            if constexpr (STAG && s % RB == 0) {
                if (late) __syncthreads();
            }
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (!PWL) {
                if constexpr (CLAMP) {
                    wo = min(y + 1, H - 1) * wrow;
                } else {
                    wo += wrow;
                    asm volatile("" : "+s"(wo));
                }
            }
            load_wl<0, HV::TA>(wla, wlcol + wo);
            read_wr<T, 0, HV::QA>(wra, &slab[bnext][my_entry]);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (HV::TB > 0) taps<U, s, HV::TA, TBE, DM != DM_READ>(num, dn, wlb, wrb, win);
            if constexpr (DM == DM_READ) {
                dn = dring[s % KD];
                dring[s % KD] = bload<CP>(rdn, voff,
                                          PD ? 0 : CLAMP ? (min(y + KD, H - 1) - min(ys + KD, H - 1)) * rowbytes : so);
            }
            bstore<CPS>(div_pos(num, dn), ro, voff, PO ? 0 : so);
            win[(s + U - 1) % U] = bload<CP>(rc, voff, PC ? 0 : CLAMP ? (min(y + R + P, H - 1) - cb) * rowbytes : so);
            sink += warm[s % PW];
            warm[s % PW] = bload(rwl, warm_voff, PWL ? 0 : CLAMP ? min(y + PW, H - 1) * wrow_b : woff);
            so += rowbytes;
            woff += wrow_b;
            soff += wrow_b;
            asm volatile("" : "+s"(so), "+s"(woff), "+s"(soff));
        });
    };
    int ys = y_begin;
    for (; ys + U <= y_end && ys + U - 1 + LA <= H - 1; ys += U) chunk(std::integral_constant<int, 0>{}, ys);
    for (; ys + U <= y_end; ys += U) {
        asm volatile("" : "+s"(ys));
        chunk(std::integral_constant<int, 1>{}, ys);
    }
    if (ys < y_end) chunk(std::integral_constant<int, 2>{}, ys);
    if (sink == -1.0f) cout[kb + lane] = sink;
}

template <int T, int DM, int PROBE>
void launch_vprobe(const asw_params *p, const float *wl, const float *wr, const float *cin, float *cout, float *den,
                   hipStream_t st) {
    constexpr int NW = 16;
    constexpr int U = pf9_period(T);
    const int W = p->width, H = p->height;
    const int Dp = round_up(d_end_of_p(p) - p->d_begin, 64);
    const int nkb = Dp / 64;
    const int nxb = (W + NW - 1) / NW;
    int nstrip = (int)((2048LL + (long long)nxb * nkb - 1) / ((long long)nxb * nkb));
    const int max_strip = H / (2 * T) > 1 ? H / (2 * T) : 1;
    if (nstrip > max_strip) nstrip = max_strip;
    if (nstrip < 1) nstrip = 1;
    const int rows = ((H + nstrip - 1) / nstrip + U - 1) / U * U;
    nstrip = (H + rows - 1) / rows;
    const int per_xcd = (nxb + 7) / 8;
    hipLaunchKernelGGL((k_vprobe<T, DM, PROBE>), dim3(8 * per_xcd * nkb * nstrip), dim3(NW * 64), 0, st, wl, wr, cin,
                       cout, den, W, H, Dp, p->d_begin, rows, nxb, nstrip, per_xcd);
}

}  // namespace agg
}  // namespace asw
