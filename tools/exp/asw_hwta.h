// Experimental (round 6): the last H pass of a frame with the WTA's
// own scan fused (K/asw_wta.cl:34-47, k_wta_local_scan's key / m1 / m2), the partial
// scan of each wave (64 planes of pixel x) by two DPP min reductions per step, in
// registers: no LDS tile (round 5's fused form took 9 KB of tiles per block and fell
// from 4 to 3 blocks per CU).  The block's NKW waves hold every plane of the volume
// (NKW * 64 = Dp); their partials merge in plane order one batch later.
#pragma once
#include "asw_aggregate_impl.h"

namespace asw {
namespace agg {

constexpr float kWtaSentinel = 100000.0f;  // K/asw_wta.cl:25-26

// min over the 64 lanes (DPP: row_shr 1, 2, 4, 8, then row_bcast 15 / 31; lane 63 holds
// it), one v_min_f32 with a DPP source per level: a lane the DPP gives no source keeps
// its own value (bound_ctrl off, dst = src1).  (The builtin mov_dpp + min form does not
// fold: 12 instructions instead of 6.)  s_nop 1: the two wait states between a VALU
// write of a VGPR and its DPP read.
#define ASW_DPP_MIN(CTRL) asm volatile("s_nop 1\n\tv_min_f32_dpp %0, %0, %0 " CTRL : "+v"(v))
__device__ __forceinline__ float wave_min64(float v) {
    ASW_DPP_MIN("row_shr:1 row_mask:0xf bank_mask:0xf");
    ASW_DPP_MIN("row_shr:2 row_mask:0xf bank_mask:0xf");
    ASW_DPP_MIN("row_shr:4 row_mask:0xf bank_mask:0xf");
    ASW_DPP_MIN("row_shr:8 row_mask:0xf bank_mask:0xf");
    ASW_DPP_MIN("row_bcast:15 row_mask:0xa bank_mask:0xf");
    ASW_DPP_MIN("row_bcast:31 row_mask:0xc bank_mask:0xf");
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
#undef ASW_DPP_MIN
// merge of two partial sequential scans (a then b in plane order)
__device__ __forceinline__ void wta_merge(float &cur, float &last, int &md, float c2, float l2, int m2) {
    const bool take = c2 < cur || (c2 == cur && (unsigned)m2 < (unsigned)md);
    last = fminf(fmaxf(cur, c2), fminf(last, l2));
    md = take ? m2 : md;
    cur = take ? c2 : cur;
}

template <int T, int NKW, int VG = 0>
__global__ __launch_bounds__(64 * NKW) __attribute__((amdgpu_waves_per_eu(4))) void k_hpass11_wr(
    const float *__restrict__ wl, const float *__restrict__ wr, const float *__restrict__ cin,
    float *__restrict__ cout, float *__restrict__ den, int W, int H, int Dp, int d_begin, int nseg, int seg_len,
    int groups_per_xcd, int ngroups, int ring_off, int kbg0, int nkbg, long long *__restrict__ wkey,
    float *__restrict__ wm1, float *__restrict__ wm2, int nloc) {
    constexpr int DM = DM_READ, CP = kCPStream, CPS = kCPStream;
    constexpr int R = T / 2;
    constexpr int TP = tap_pitch(T);
    constexpr int Q = TP / 4;
    constexpr int U = pf9_period(T);
    constexpr int P = U - T;
    constexpr int PW = VG ? 2 : 4;
    constexpr int KD = VG ? 2 : 4;  // den prefetch ring (steps); VG = 1: shallower rings (fewer VGPRs)
    constexpr int NT = 64 * NKW;        // threads, and entries of the block at one x
    constexpr int K = h11_batch(T, NKW);
    constexpr int RING = h11_ring(T, NKW);
    constexpr int EB = Q * 16;          // bytes per ring entry
    constexpr int RB = RING * EB;       // ring bytes
    static_assert(U % K == 0 && RING >= NT + 2 * K && RING % 16 == 0, "ring geometry");
    static_assert(K * Q <= NT, "one staged float4 per thread per batch");
    __shared__ f4 ring[RING * Q];
    // the waves' partial scans of a batch (double-buffered by batch parity)
    __shared__ float wpc[2 * K * NKW], wpl[2 * K * NKW];
    __shared__ int wpm[2 * K * NKW];

    // plane-block groups [kbg0, kbg0 + nkbg) of the Dp-pitched volume (the whole range
    // in production: kbg0 = 0, nkbg = Dp / NT)
    const int xcd = blockIdx.x & 7, m = blockIdx.x >> 3;
    const int gl = m / nkbg;
    const int g = xcd * groups_per_xcd + gl;
    if (gl >= groups_per_xcd || g >= ngroups) return;  // padding block (uniform)
    const int kbg = kbg0 + m - gl * nkbg;
    const int y = g / nseg;
    const int xs = (g - y * nseg) * seg_len;
    const int xe = min(xs + seg_len, W);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int d0 = d_begin + kbg * NT;
    const int kb = kbg * NT + wave * 64;
    const float *wrrow = wr + (long long)y * W * TP;
    // batch bb's pixels (first column xb0): the waves' partials merged in plane order
    // (first argmin = the smaller index of equal minima; second minimum of the union =
    // min(max(m1a, m1b), min(m2a, m2b))), written as k_wta_local_scan writes them
    auto wr_combine = [&](int bb, int xb0) __attribute__((always_inline)) {
        if (wave == 0 && lane < K && xb0 + lane < xe) {
            const int base = ((bb & 1) * K + lane) * NKW;
            float cur = wpc[base], last = wpl[base];
            int md = wpm[base];
#pragma unroll
            for (int w = 1; w < NKW; ++w) wta_merge(cur, last, md, wpc[base + w], wpl[base + w], wpm[base + w]);
            const long long pix = (long long)y * W + xb0 + lane;
            wkey[pix] = md < 0 ? 0x7fffffffffffffffLL
                               : (long long)(((unsigned long long)__float_as_uint(cur) << 32) | (unsigned)md);
            wm1[pix] = cur;
            wm2[pix] = last;
        }
    };

    // the ring before batch 0: entries [xs - d0 - (NT - 1), xs + K - d0]
    {
        const int e0 = xs - d0 - (NT - 1);
        for (int t = threadIdx.x; t < (NT + K) * Q; t += NT) {
            const int e = t / Q, q = t - e * Q;
            const int xr = e0 + e;
            ring[((xr + ring_off) % RING) * Q + q] =
                *reinterpret_cast<const f4 *>(wrrow + clampi(xr, 0, W - 1) * TP + 4 * q);
        }
    }
    // staging: thread t owns float4 q of entry e of every batch's K new entries,
    // t = min(threadIdx, K*Q-1) (surplus threads repeat the last: same value, same
    // place; no branch)
    const int st_t = min((int)threadIdx.x, K * Q - 1);
    const int st_e = st_t / Q, st_q = st_t - st_e * Q;
    int st_xr = xs + K + 1 - d0 + st_e;                              // batch 1's entry
    int st_addr = ((st_xr + ring_off) % RING) * EB + st_q * 16;      // its LDS byte address
    f4 stg = *reinterpret_cast<const f4 *>(wrrow + clampi(st_xr, 0, W - 1) * TP + 4 * st_q);
    __syncthreads();

    const long long rowoff = (long long)y * W * Dp + kb;
    const rsrc_t rc = make_rsrc(cin + rowoff);
    const rsrc_t ro = make_rsrc(cout + rowoff);
    const rsrc_t rd = make_rsrc(den + rowoff);
    const int voff = lane * 4;
    const int xstride = Dp * 4;  // bytes per column
    const float *wlrow = wl + (long long)y * W * TP;
    const int warm_off = lane < TP ? lane : 0;
    // LDS byte address of this lane's entry at step x (xr = x - d0 - 64*wave - lane)
    int ra = ((xs - d0 - wave * 64 - lane + ring_off) % RING) * EB;
    auto ring_next = [](int a) __attribute__((always_inline)) {
        const unsigned t = (unsigned)a + EB, u = t - (unsigned)RB;
        return (int)(t < u ? t : u);
    };
    auto at = [&](int a) __attribute__((always_inline)) {
        return reinterpret_cast<const f4 *>(reinterpret_cast<const char *>(ring) + a);
    };

    using HV = Halves<T>;
    float win[U];
    float wla[HV::NA], wlb[HV::NB];
    f4 wra[HV::MA], wrb[HV::MB];
    float warm[PW];
    float dring[KD];
    float sink = 0.0f;
#pragma unroll
    for (int j = 0; j < U - 1; ++j) win[j] = bload<CP>(rc, voff, clampi(xs - R + j, 0, W - 1) * xstride);
    if constexpr (DM == DM_READ) {
#pragma unroll
        for (int j = 0; j < KD; ++j) dring[j] = bload<CP>(rd, voff, min(xs + j, W - 1) * xstride);
    }
#pragma unroll
    for (int j = 0; j < PW; ++j) warm[j] = wlrow[min(xs + 1 + j, W - 1) * TP + warm_off];
    load_wl<0, HV::TA>(wla, wlrow + xs * TP);
    read_wr<T, 0, HV::QA>(wra, at(ra));

    auto body = [&](auto sc, auto chk, int xb) __attribute__((always_inline)) {
        constexpr int s = decltype(sc)::value;
        constexpr bool CHK = decltype(chk)::value;
        const int x = xb + s;
        if constexpr (CHK) {
            if (x >= xe) return;  // the same x for all waves: the barriers stay matched
        }
        const float *wlx = wlrow + xb * TP + s * TP;
        if constexpr (s % K == 0) {
            // top of a batch: every wave is done with the previous batch, and the
            // entries written at its top are visible
            __syncthreads();
            {
                const int b = (x - xs) / K;
                if (b >= 1) wr_combine(b - 1, x - K);
            }
            *reinterpret_cast<f4 *>(reinterpret_cast<char *>(ring) + st_addr) = stg;
            st_xr += K;
            st_addr += K * EB;
            st_addr = st_addr >= RB ? st_addr - RB : st_addr;
            stg = *reinterpret_cast<const f4 *>(wrrow + clampi(st_xr, 0, W - 1) * TP + 4 * st_q);
        } else {
            wait_lgkm0();  // half A's weights
        }
        asm volatile("" ::"v"(win[(s + T - 1) % U]));  // newest window element: one vmcnt wait per step
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (HV::TB > 0) {
            load_wl<HV::TA, T>(wlb, wlx);
            read_wr<T, HV::QA, HV::QT>(wrb, at(ra));
        }
        __builtin_amdgcn_sched_barrier(0);
        float num = 1e-5f, dn = 1e-5f;
        taps<U, s, 0, HV::TA, DM != DM_READ>(num, dn, wla, wra, win);
        __builtin_amdgcn_sched_barrier(0);
        wait_lgkm0();  // half B's weights
        __builtin_amdgcn_sched_barrier(0);
        ra = ring_next(ra);
        {
            const float *pn;
            if constexpr (CHK || s == U - 1) pn = wlrow + min(x + 1, W - 1) * TP;
            else pn = wlx + TP;
            load_wl<0, HV::TA>(wla, pn);
            read_wr<T, 0, HV::QA>(wra, at(ra));
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (HV::TB > 0) taps<U, s, HV::TA, T, DM != DM_READ>(num, dn, wlb, wrb, win);
        const int xo = x * xstride;
        if constexpr (DM == DM_READ) {
            dn = dring[s % KD];
            dring[s % KD] = bload<CP>(rd, voff, min(x + KD, W - 1) * xstride);
        } else if constexpr (DM == DM_WRITE) {
            bstore<CPS>(dn, rd, voff, xo);
        }
        const float o = div_pos(num, dn);
        bstore<CPS>(o, ro, voff, xo);
        win[(s + U - 1) % U] = bload<CP>(rc, voff, min(x + R + P, W - 1) * xstride);
        {
            // this wave's partial scan of pixel x over its 64 planes (padding planes +inf)
            const float v = kb + lane < nloc ? o : __builtin_inff();
            const float m = wave_min64(v);
            const unsigned long long eq = __ballot(v == m);
            const int f = __builtin_ctzll(eq);
            const float m2 = wave_min64(lane == f ? __builtin_inff() : v);
            if (lane == 0) {
                const int slot = ((((x - xs) / K) & 1) * K + s % K) * NKW + wave;
                wpc[slot] = fminf(m, kWtaSentinel);
                wpl[slot] = fminf(m2, kWtaSentinel);
                wpm[slot] = m < kWtaSentinel ? d_begin + kb + f : -1;
            }
        }
        sink += warm[s % PW];
        warm[s % PW] = wlrow[min(x + 1 + PW, W - 1) * TP + warm_off];
    };
    int xb = xs;
    for (; xb + U <= xe; xb += U)
        static_for<0, U>([&](auto sc) __attribute__((always_inline)) { body(sc, std::false_type{}, xb); });
    if (xb < xe)
        static_for<0, U>([&](auto sc) __attribute__((always_inline)) { body(sc, std::true_type{}, xb); });
    {  // the last batch
        const int nb = (xe - xs + K - 1) / K;
        __syncthreads();
        wr_combine(nb - 1, xs + (nb - 1) * K);
    }
    if (sink == -1.0f) cout[rowoff] = sink;  // never true (weights > 0): keeps the warm loads
}

// the launcher (k_hpass11's geometry; NKW = Dp / 64: one block over every plane)
template <int T, int NKW, int VG = 0>
void launch_h11_wr(const asw_params *p, const float *wl, const float *wr, const float *cin, float *cout,
                   float *den, long long *key, float *m1, float *m2, hipStream_t st, int seg_len) {
    constexpr int RING = h11_ring(T, NKW);
    const int W = p->width, H = p->height;
    const int Dp = round_up(d_end_of_p(p) - p->d_begin, 64);
    const int nkbg = Dp / (64 * NKW);
    const int nseg = (W + seg_len - 1) / seg_len;
    const int ngroups = H * nseg;
    const int per_xcd = (ngroups + 7) / 8;
    const int ring_off = ((p->d_begin + Dp) / RING + 1) * RING;
    hipLaunchKernelGGL((k_hpass11_wr<T, NKW, VG>), dim3(8 * per_xcd * nkbg), dim3(64 * NKW), 0, st, wl, wr, cin, cout, den,
                       W, H, Dp, p->d_begin, nseg, seg_len, per_xcd, ngroups, ring_off, 0, nkbg, key, m1, m2,
                       d_end_of_p(p) - p->d_begin);
}

}  // namespace agg
}  // namespace asw
