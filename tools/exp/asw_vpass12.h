// asw_vpass12.h — V aggregation pass, two diagonal columns per wave sharing their
// right weights (K/asw_vcost_aggregation.cl:11-44; one launch of main.cpp:494-500).
//
// Why: k_vpass10 reads every voxel-tap's right weight wr_i(x-d, y) from LDS (one
// ds_read_b128 per 4 taps) and stages a 79-entry slab row per 16 columns; with the
// den cache that LDS traffic is as large as the VALU work (PMC: SQ_WAIT_INST_LDS 14 %
// of wave cycles against 3 % in the H pass, profiles/r03/pmc_r08c.json).  Voxels
// (x, d) and (x+1, d+1) read the SAME entry x-d, so a wave here owns two columns,
//   A = (xa, kb + l),  B = (xa + 1, kb + l + 1),   lane l,
// and one set of right-weight registers serves both chains, interleaved tap by tap
// (two independent FMA chains per lane).  LDS reads per voxel halve, and the
// per-step waits, barriers and address work are paid once per two voxels.
//
// Plane Dp of column xa+1 (lane 63 of the LAST plane block) does not exist and plane 0
// of every B column is covered by no pair: that lane computes plane 0 instead, whose
// entry xa+1-d_begin is a per-wave "special" slab entry.  The last plane block's waves
// (LK) therefore run A's taps and then B's with B's right weights read separately
// (lane 63 at the special entry); every other wave shares them.
//
// Per step (row y) the taps run in NPH phases of about T/NPH taps; each phase's
// weights (left: SGPRs from scalar loads, right: ds_read_b128) are requested one
// phase ahead, with one lgkmcnt(0) wait per phase.  Slab rows are staged through a
// VGPR ring PS rows ahead into an NBUF-buffer LDS ring with one barrier per RB rows,
// cost / den / output go through buffer instructions with one running SGPR offset per
// U-row chunk — the k_vpass10 schedule.
//
// Same FP sequence as every other pass (DESIGN.md §FP policy): bit-identical outputs.
//
// STATUS: experiment, not in the product (tools/exp/exp_bench.py --v).  Bit-exact, but
// two cost windows and two left-weight sets do not fit 4 waves per SIMD: with 2 tap
// phases it spills ~450 VGPRs (each scratch reload a vmcnt(0)); with 5 phases (no
// spills, 3 waves/SIMD, 12 waves x 2 columns) it measured 2.02 ms den-read against
// k_vpass10's 1.60, den-none 1.86 vs 1.74, den-write 2.32 vs 1.82
// (profiles/r03/vpass12_r08d.log): the pass is latency-bound and loses more to the
// lower occupancy than it gains from halving the LDS reads.
#include "asw_aggregate_impl.h"

namespace asw {
namespace agg {

// taps [B, E) of the A and B chains, interleaved tap by tap; wl*/wr hold taps from B
template <int U, int S, int B, int E, bool DEN, int N, int M>
__device__ __forceinline__ void taps2(float &numA, float &denA, float &numB, float &denB, const float (&wlA)[N],
                                      const float (&wlB)[N], const f4 (&wr)[M], const float (&winA)[U],
                                      const float (&winB)[U]) {
#pragma unroll
    for (int i = B; i < E; ++i) {
        const float r = wr[(i - B) / 4][(i - B) % 4];
        const float wwA = wlA[i - B] * r;
        const float wwB = wlB[i - B] * r;
        numA = __builtin_fmaf(wwA, winA[(S + i) % U], numA);
        numB = __builtin_fmaf(wwB, winB[(S + i) % U], numB);
        if constexpr (DEN) {
            denA = denA + wwA;
            denB = denB + wwB;
        }
    }
}

// slab row of k_vpass12: SLAB = 2 NW + 62 shared entries, then NW special ones
constexpr int v12_slab(int NW) { return 2 * NW + 62; }

template <int T, int NW, int DM, int RB, int PS, int NPH, int CP, int CPS, bool LK>
__device__ __forceinline__ void vpass12_body(const float *__restrict__ wl, const float *__restrict__ wr,
                                             const float *__restrict__ cin, float *__restrict__ cout,
                                             float *__restrict__ den, int W, int H, int Dp, int d_begin, int x0,
                                             int y_begin, int y_end, int kb,
                                             f4 (*slab)[(v12_slab(NW) + NW) * (tap_pitch(T) / 4)]) {
    constexpr int R = T / 2;
    constexpr int TP = tap_pitch(T);
    constexpr int Q = TP / 4;
    constexpr int U = pf9_period(T);
    constexpr int P = U - T;
    constexpr int KD = 2;  // den prefetch ring (rows)
    constexpr int PW = 4;  // left-weight L2 warm distance (rows)
    constexpr int LEAD = RB + 1;
    constexpr int NBUF = ring_div(U, 2 * RB + 1);
    constexpr int SLAB = v12_slab(NW);
    // the special entries are staged by the LK blocks only (a wave-uniform extent)
    constexpr int NQ = (LK ? SLAB + NW : SLAB) * Q;
    constexpr int NTH = NW * 64;
    constexpr bool NS2 = NQ > NTH;  // a second staged float4 per thread
    static_assert(NQ <= 2 * NTH, "slab row larger than two float4 per thread");
    static_assert(U % PS == 0 && U % KD == 0 && U % PW == 0 && U % RB == 0 && U % NBUF == 0, "ring periods");
    static_assert(LEAD <= PS, "staging ring too short for the barrier period");
    constexpr int LA = cmax(cmax(R + P, LEAD + PS), cmax(KD, PW));
    using PH = Phases<T, NPH>;
    // phase j of a step: LK: A phases 0..NPH-1 then B phases; else NPH joint phases
    constexpr int NP = LK ? 2 * NPH : NPH;

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // A = column xa (a wave past the right edge recomputes column W-1 and stores the
    // same values again); when xa + 1 is past the edge, B := A (same voxel, same
    // weights, stored twice)
    const int xa = min(x0 + 2 * wave, W - 1);
    const bool b_live = x0 + 2 * wave + 1 < W;  // wave-uniform
    const int xb = b_live ? xa + 1 : xa;
    const int slab_base = x0 - (d_begin + kb) - 63;  // virtual xr of slab entry 0
    const int my_entry = ((xa - x0) + 63 - lane) * Q;
    const int b_entry = LK && b_live && lane == 63 ? (SLAB + wave) * Q : my_entry;
    const long long rowstride = (long long)W * Dp;
    const int rowbytes = (int)(rowstride * 4);  // U+LA rows < 2 GiB: checked by the launcher
    const long long colA = (long long)xa * Dp;
    const int voffA = (kb + lane) * 4;
    const int kB = kb + lane + 1;
    const int voffB = b_live ? ((xb - xa) * Dp + (kB == Dp ? 0 : kB)) * 4 : voffA;
    const int wrow = W * TP;
    const int wrow_b = wrow * 4;
    const rsrc_t rwr = make_rsrc(wr);
    const float *wlA = wl + (long long)xa * TP;
    const float *wlB = wl + (long long)xb * TP;
    // "warm" loads: one dword per lane pulls the left-weight rows of both columns (2 TP
    // contiguous floats) into L2 PW rows before their scalar loads
    const rsrc_t rwl = make_rsrc(wlA);
    const int warm_voff = min(2 * lane, 2 * TP - 1) * 4;
    auto rsrc_at = [&](const float *base, int row) __attribute__((always_inline)) {
        return make_rsrc(base + (long long)row * rowstride + colA);
    };

    // per-thread share of a slab row (<= 2 float4 per thread); surplus threads redo
    // the last entry (same value, same place: no branch)
    auto slab_src = [&](int t) __attribute__((always_inline)) {
        const int e = t / Q, q = t - (t / Q) * Q;
        const int src = e < SLAB ? clampi(slab_base + e, 0, W - 1)
                                 : clampi(x0 + 2 * (e - SLAB) + 1 - d_begin, 0, W - 1);
        return (src * TP + 4 * q) * 4;
    };
    const int t0 = min((int)threadIdx.x, NQ - 1);
    const int t1 = min((int)threadIdx.x + NTH, NQ - 1);
    const int sv0 = slab_src(t0), sv1 = slab_src(t1);
    auto stage = [&](f4 &a, f4 &b, int roff) __attribute__((always_inline)) {
        a = bload4(rwr, sv0, roff);
        if constexpr (NS2) b = bload4(rwr, sv1, roff);
    };
    auto put = [&](int buf, const f4 &a, const f4 &b) __attribute__((always_inline)) {
        slab[buf][t0] = a;
        if constexpr (NS2) slab[buf][t1] = b;
    };

    float winA[U], winB[U];
    f4 sa[PS], sb[PS];
    float dringA[KD], dringB[KD];
    float warm[PW];
    float sink = 0.0f;
    // weight sets of phase j (compile-time indices; at most two are live)
    float wlx[NP][PH::NT], wly[NP][PH::NT];
    f4 wrs[NP][PH::NG];
    {
        const int r0 = max(0, y_begin - R);
        const rsrc_t rp = rsrc_at(cin, r0);
#pragma unroll
        for (int j = 0; j < U - 1; ++j) {
            const int o = (clampi(y_begin - R + j, 0, H - 1) - r0) * rowbytes;
            winA[j] = bload<CP>(rp, voffA, o);
            winB[j] = bload<CP>(rp, voffB, o);
        }
    }
    if constexpr (DM == DM_READ) {
        const rsrc_t rp = rsrc_at(den, y_begin);
#pragma unroll
        for (int j = 0; j < KD; ++j) {
            const int o = (min(y_begin + j, H - 1) - y_begin) * rowbytes;
            dringA[j] = bload<CP>(rp, voffA, o);
            dringB[j] = bload<CP>(rp, voffB, o);
        }
    }
#pragma unroll
    for (int j = 0; j < PS; ++j) stage(sa[j], sb[j], min(y_begin + j, H - 1) * wrow_b);
#pragma unroll
    for (int j = 0; j < PW; ++j) warm[j] = bload(rwl, warm_voff, min(y_begin + j, H - 1) * wrow_b);
#pragma unroll
    for (int j = 0; j < LEAD; ++j) put(j, sa[j], sb[j]);
#pragma unroll
    for (int j = 0; j < LEAD; ++j) stage(sa[j], sb[j], min(y_begin + PS + j, H - 1) * wrow_b);
    __syncthreads();

    // requests of phase j's weights for row offset wo (floats) from slab buffer buf
    auto request = [&](auto jc, int wo, int buf) __attribute__((always_inline)) {
        constexpr int j = decltype(jc)::value;
        constexpr int k = j % NPH;
        constexpr bool isB = LK && j >= NPH;
        constexpr int b0 = PH::tb(k), b1 = PH::tb(k + 1);
        constexpr int g0 = PH::gb(k), g1 = PH::gb(k + 1);
        if constexpr (!LK || !isB) load_wl<b0, b1>(wlx[j], wlA + wo);
        if constexpr (!LK || isB) load_wl<b0, b1>(wly[j], wlB + wo);
        read_wr<T, g0, g1>(wrs[j], &slab[buf][isB ? b_entry : my_entry]);
    };
    request(std::integral_constant<int, 0>{}, y_begin * wrow, 0);

    auto chunk = [&](auto clamp_c, int ys) __attribute__((always_inline)) {
        constexpr bool CLAMP = decltype(clamp_c)::value;
        const int cb = min(ys + R + P, H - 1);
        const rsrc_t rc = rsrc_at(cin, cb);
        const rsrc_t ro = rsrc_at(cout, ys);
        const rsrc_t rd = rsrc_at(den, ys);
        const rsrc_t rdn = rsrc_at(den, min(ys + KD, H - 1));
        int so = 0;                          // (y - ys) * rowbytes
        int wo = ys * wrow;                  // left weights of row y (floats)
        int soff = (ys + LEAD + PS) * wrow_b;  // staged slab row y + LEAD + PS
        int woff = (ys + PW) * wrow_b;         // warm row y + PW
        static_for<0, U>([&](auto sc) __attribute__((always_inline)) {
            constexpr int s = decltype(sc)::value;
            const int y = ys + s;
            if constexpr (CLAMP) {
                if (y >= y_end) return;
            }
            constexpr int bcur = s % NBUF, bnext = (s + 1) % NBUF, bput = (s + LEAD) % NBUF;
            float numA = 1e-5f, dnA = 1e-5f, numB = 1e-5f, dnB = 1e-5f;
            static_for<0, NP>([&](auto jc) __attribute__((always_inline)) {
                constexpr int j = decltype(jc)::value;
                constexpr int k = j % NPH;
                constexpr int b0 = PH::tb(k), b1 = PH::tb(k + 1);
                // phase j's weights are in (lgkmcnt 0); at j = 0 every RB rows, also the
                // slab rows up to y + RB
                if constexpr (j == 0 && s % RB == 0) __syncthreads();
                else wait_lgkm0();
                if constexpr (j == 0) asm volatile("" ::"v"(winA[(s + T - 1) % U]), "v"(winB[(s + T - 1) % U]));
                __builtin_amdgcn_sched_barrier(0);
                if constexpr (j + 1 < NP) {
                    request(std::integral_constant<int, j + 1>{}, wo, bcur);
                } else {
                    if constexpr (CLAMP) {
                        wo = min(y + 1, H - 1) * wrow;
                    } else {
                        wo += wrow;
                        asm volatile("" : "+s"(wo));
                    }
                    request(std::integral_constant<int, 0>{}, wo, bnext);
                }
                if constexpr (j == 0) {
                    put(bput, sa[(s + LEAD) % PS], sb[(s + LEAD) % PS]);
                    stage(sa[(s + LEAD) % PS], sb[(s + LEAD) % PS], CLAMP ? min(y + LEAD + PS, H - 1) * wrow_b : soff);
                }
                __builtin_amdgcn_sched_barrier(0);
                if constexpr (!LK) {
                    taps2<U, s, b0, b1, DM != DM_READ>(numA, dnA, numB, dnB, wlx[j], wly[j], wrs[j], winA, winB);
                } else if constexpr (j < NPH) {
                    taps<U, s, b0, b1, DM != DM_READ>(numA, dnA, wlx[j], wrs[j], winA);
                } else {
                    taps<U, s, b0, b1, DM != DM_READ>(numB, dnB, wly[j], wrs[j], winB);
                }
                __builtin_amdgcn_sched_barrier(0);
            });
            if constexpr (DM == DM_READ) {
                dnA = dringA[s % KD];
                dnB = dringB[s % KD];
                const int o = CLAMP ? (min(y + KD, H - 1) - min(ys + KD, H - 1)) * rowbytes : so;
                dringA[s % KD] = bload<CP>(rdn, voffA, o);
                dringB[s % KD] = bload<CP>(rdn, voffB, o);
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
            sink += warm[s % PW];
            warm[s % PW] = bload(rwl, warm_voff, CLAMP ? min(y + PW, H - 1) * wrow_b : woff);
            so += rowbytes;
            soff += wrow_b;
            woff += wrow_b;
            asm volatile("" : "+s"(so), "+s"(soff), "+s"(woff));
        });
    };
    int ys = y_begin;
    for (; ys + U <= y_end && ys + U - 1 + LA <= H - 1; ys += U) chunk(std::false_type{}, ys);
    // the chunks that reach the image bottom, and the partial last chunk
    for (; ys < y_end; ys += U) {
        asm volatile("" : "+s"(ys));
        chunk(std::true_type{}, ys);
    }
    if (sink == -1.0f) cout[kb + lane] = sink;  // never true (weights > 0): keeps the warm loads
}

#ifndef V12_LK_ON
#define V12_LK_ON 1
#endif
// waves per SIMD the block size allows at one block per CU (NW <= 16)
constexpr int v12_waves_per_eu(int NW) { return NW >= 13 ? 4 : NW >= 9 ? 3 : 2; }

template <int T, int NW, int DM, int RB, int PS, int NPH, int CP, int CPS = CP>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(v12_waves_per_eu(NW)))) void k_vpass12(
    const float *__restrict__ wl, const float *__restrict__ wr, const float *__restrict__ cin, float *__restrict__ cout,
    float *__restrict__ den, int W, int H, int Dp, int d_begin, int rows_per_strip, int nxb, int nstrip,
    int xg_per_xcd) {
    constexpr int U = pf9_period(T);
    constexpr int NBUF = ring_div(U, 2 * RB + 1);
    constexpr int NQMAX = (v12_slab(NW) + NW) * (tap_pitch(T) / 4);
    static_assert(NBUF * NQMAX * 16 <= 160 * 1024, "slab ring exceeds the gfx950 LDS");
    __shared__ f4 slab[NBUF][NQMAX];

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
    if (V12_LK_ON && kbi == nkb - 1)
        vpass12_body<T, NW, DM, RB, PS, NPH, CP, CPS, true>(wl, wr, cin, cout, den, W, H, Dp, d_begin, x0, y_begin,
                                                             y_end, kb, slab);
    else
        vpass12_body<T, NW, DM, RB, PS, NPH, CP, CPS, false>(wl, wr, cin, cout, den, W, H, Dp, d_begin, x0, y_begin,
                                                              y_end, kb, slab);
}

template <int T, int NW, int DM, int RB, int PS, int NPH, int CP, int CPS = CP>
void launch_v12(const asw_params *p, const float *wl, const float *wr, const float *cin, float *cout, float *den,
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
    hipLaunchKernelGGL((k_vpass12<T, NW, DM, RB, PS, NPH, CP, CPS>), dim3(nblocks), dim3(NW * 64), 0, st, wl, wr, cin,
                       cout, den, W, H, Dp, p->d_begin, rows, nxb, nstrip, per_xcd);
}

}  // namespace agg
}  // namespace asw
