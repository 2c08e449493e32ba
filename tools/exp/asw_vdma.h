// k_vdma: the V aggregation pass (K/asw_vcost_aggregation.cl:11-44, main.cpp:494-500)
// with every global read staged by LDS-DMA (buffer_load ... lds) several rows ahead, so
// a wave's only VMEM result it waits for is in LDS and its registers hold no staging data
// (the den-none V pass ran its VALU and memory one after the other).
//
// Block = 16 waves = 16 columns x 64 planes (k_vpass10's C4 shape).  Per row step y:
//   * the right-weight slab row (79 entries x Q float4, 12 KB) is split in 12 pieces of
//     64 float4: waves 0..11 each DMA one piece of row y + LEADS into the slab ring
//     (NBUF rows), one raw s_barrier per RB rows publishes them;
//   * each wave DMAs its own column's cost element of row y + R + PC (64 planes, 256 B)
//     into a wave-private ring (NC slots), and (den-read) its den row y + PC likewise;
//     both are read back with one ds_read_b32 the step they are used;
//   * the left weights stay scalar loads (SGPR operands at the full VALU rate); each
//     wave DMAs its column's next-PW-row entry into a junk LDS slot, which only pulls
//     the line into L2 ahead of the scalar loads (the "warm" of k_vpass10);
//   * output (and, den-write, den) stores are the only other VMEM operations.
// Every VMEM operation is issued in a fixed order per step, so the waits are counted:
// vmcnt(N) with N = the operations issued after the one a step needs (vmcnt counts
// loads and stores in order on gfx9).  No ordinary VMEM load is in flight during the
// sweep (the window prologue is drained before the first DMA), so the compiler inserts
// no vmcnt wait of its own.  The FP sequence per voxel is k_vpass10's: bit-identical.
#pragma once
#include "asw_aggregate_impl.h"

namespace asw {
namespace agg {

// s_waitcnt vmcnt(N) (gfx9 encoding: vmcnt bits [3:0] and [15:14]; expcnt, lgkmcnt max)
template <int N>
__device__ __forceinline__ void wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt field");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

using lds_ptr_t = __attribute__((address_space(3))) void *;
// one buffer -> LDS DMA: lane l's `size` bytes at rsrc + voff + soff land at lds + size * l
template <int SIZE, int CP = 0>
__device__ __forceinline__ void dma(rsrc_t r, lds_ptr_t lds, int voff, int soff) {
    static_assert(SIZE == 4 || SIZE == 16, "dword or dwordx4");
    if constexpr (SIZE == 16) __builtin_amdgcn_raw_ptr_buffer_load_lds(r, lds, 16, voff, soff, 0, CP);
    else __builtin_amdgcn_raw_ptr_buffer_load_lds(r, lds, 4, voff, soff, 0, CP);
}

template <int T, int DM, int LEADS = 6, int RB = 2, int NBUF = 8, int NC = 5>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4))) void k_vdma(
    const float *__restrict__ wl, const float *__restrict__ wr, const float *__restrict__ cin, float *__restrict__ cout,
    float *__restrict__ den, int W, int H, int Dp, int d_begin, int rows_per_strip, int nxb, int nstrip,
    int xg_per_xcd) {
    constexpr int NW = 16;
    constexpr int CP = kCPStream, CPS = kCPStream;
    constexpr int R = T / 2;
    constexpr int TP = tap_pitch(T);
    constexpr int Q = TP / 4;
    constexpr int U = pf9_period(T);
    constexpr int L = LEADS - RB;  // cost / den lead (steps) = the slab's slack at a barrier
    constexpr int PC = L;
    constexpr int PW = 4;
    constexpr int SLAB = NW + 63;
    constexpr int NQ = SLAB * Q;
    constexpr int NPIECE = (NQ + 63) / 64;  // slab pieces of 64 float4 (one DMA each)
    constexpr int SROW = NPIECE * 64;       // float4 per slab ring row (padded)
    static_assert(NPIECE <= NW, "one slab piece per wave at most");
    static_assert(LEADS <= NBUF - RB && L >= 1, "slab ring: a row is overwritten only after its last reader's barrier");
    static_assert(NC >= PC + 1, "cost ring");
    static_assert(U % NBUF == 0 && U % NC == 0 && U % RB == 0 && U % PW == 0, "compile-time ring slots");
    // one LDS array (the staged rows): slab ring | cost ring | den ring | junk
    constexpr int CROW = NW * 16;  // float4 per cost ring slot (16 waves x 64 floats)
    constexpr int OFF_C = NBUF * SROW;
    constexpr int OFF_D = OFF_C + NC * CROW;
    constexpr int OFF_J = OFF_D + (DM == DM_READ ? NC * CROW : 0);
    __shared__ f4 lds[OFF_J + 16];

    const int nkb = Dp / 64;
    const int xcd = blockIdx.x & 7, m = blockIdx.x >> 3;
    const int xg = xcd * xg_per_xcd + m % xg_per_xcd;
    const int rest = m / xg_per_xcd;
    const int kbi = rest % nkb;
    const int strip = rest / nkb;
    if (xg >= nxb || strip >= nstrip) return;  // padding block (uniform)
    const int x0 = xg * NW;
    const int y_begin = strip * rows_per_strip;
    if (y_begin >= H) return;
    const int y_end = min(H, y_begin + rows_per_strip);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool slab_wave = wave < NPIECE;  // (uniform)
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
    // this wave's slab piece: float4 t = 64 wave + lane of a row (padding lanes re-load
    // the last float4 into the padding slots)
    const int st = min(wave * 64 + lane, NQ - 1);
    const int sv = (clampi(slab_base + st / Q, 0, W - 1) * TP + 4 * (st % Q)) * 4;
    const int warm_voff = (lane < TP ? lane : TP - 1) * 4;
    auto lp = [&](int f4_index) __attribute__((always_inline)) { return (lds_ptr_t)(lds + f4_index); };
    // VMEM operations per step of a wave (fixed order, the counted waits depend on it):
    //   [slab piece] cost [den] warm ... store [den store]
    constexpr int NST = 1 + (DM == DM_WRITE ? 1 : 0);  // stores
    constexpr int NDN = DM == DM_READ ? 1 : 0;
    // sslot: slab ring row (compile-time); srow_b / coff / doff / warm_b: source offsets
    auto issue = [&](int sslot, int srow_b, int cslot, rsrc_t rc, int coff, rsrc_t rdl, int doff, int warm_b)
                     __attribute__((always_inline)) {
        if (slab_wave) dma<16>(rwr, lp(sslot * SROW + wave * 64), sv, srow_b);
        dma<4, CP>(rc, lp(OFF_C + cslot * CROW + wave * 16), voff, coff);
        if constexpr (DM == DM_READ) dma<4, CP>(rdl, lp(OFF_D + cslot * CROW + wave * 16), voff, doff);
        dma<4>(rwl, lp(OFF_J), warm_voff, warm_b);
    };
    // counted waits at the top of step s: all operations up to the den (den-read) or the
    // cost element (else) of step s, issued PC steps before; that covers the slab row
    // y + RB of a barrier step (issued first in the same step).  N = the operations
    // issued after the needed one.
    constexpr int NA = 1 + 1 + NDN + 1 + NST;  // slab waves
    constexpr int NB = 1 + NDN + 1 + NST;      // other waves
    constexpr int WA = PC * NA - 2 - NDN;
    constexpr int WB = PC * NB - 1 - NDN;
    auto wait_step = [&]() __attribute__((always_inline)) {
        if (slab_wave) wait_vm<WA>();
        else wait_vm<WB>();
    };

    using HV = Halves<T>;
    float win[U];
    float wla[HV::NA], wlb[HV::NB];
    f4 wra[HV::MA], wrb[HV::MB];
    // window prologue: rows y_begin - R .. y_begin + R - 1, ordinary loads, drained
    {
        const int r0 = max(0, y_begin - R);
        const rsrc_t rp = rsrc_at(cin, r0);
#pragma unroll
        for (int j = 0; j < T - 1; ++j) win[j] = bload<CP>(rp, voff, (clampi(y_begin - R + j, 0, H - 1) - r0) * rowbytes);
        asm volatile("" ::: "memory");
        wait_vm<0>();  // (no ordinary load is in flight once the DMAs start)
        asm volatile("" ::: "memory");
    }
    // virtual steps -LEADS .. -1: the operations of a sweep step (a second warm DMA stands
    // in for each store), so the steady-state counts hold from step 0 (y_begin, a strip
    // start, is a multiple of U: ring slots are step indices)
    {
        const int c0 = min(max(0, y_begin + R - LEADS + PC), H - 1);
        const int d0r = min(max(0, y_begin - LEADS + PC), H - 1);
        const rsrc_t rcp = rsrc_at(cin, c0);
        const rsrc_t rdp = rsrc_at(den, d0r);
#pragma unroll
        for (int v = -LEADS; v < 0; ++v) {
            const int cr = clampi(y_begin + R + v + PC, 0, H - 1);
            const int dr = clampi(y_begin + v + PC, 0, H - 1);
            const int wb = min(y_begin + v + PW + 1, H - 1) * wrow_b;
            issue((v + LEADS) % NBUF, min(y_begin + v + LEADS, H - 1) * wrow_b, ((v + PC) % NC + NC) % NC, rcp,
                  (cr - c0) * rowbytes, rdp, (dr - d0r) * rowbytes, wb);
#pragma unroll
            for (int k = 0; k < NST; ++k) dma<4>(rwl, lp(OFF_J), warm_voff, wb);
        }
    }
    // slab rows y_begin .. y_begin + RB landed (the wait of step 0), then published
    wait_step();
    wait_lgkm0();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    load_wl<0, HV::TA>(wla, wlcol + (long long)y_begin * wrow);
    read_wr<T, 0, HV::QA>(wra, &lds[(y_begin % NBUF) * SROW + my_entry]);

    auto chunk = [&](auto mode_c, int ys) __attribute__((always_inline)) {
        constexpr bool CLAMP = decltype(mode_c)::value >= 1;
        constexpr bool PART = decltype(mode_c)::value == 2;
        const int cb = min(ys + R + PC, H - 1);
        const int db = min(ys + PC, H - 1);
        const rsrc_t rc = rsrc_at(cin, cb);
        const rsrc_t rdl = rsrc_at(den, db);
        const rsrc_t ro = rsrc_at(cout, ys);
        const rsrc_t rd = rsrc_at(den, ys);
        int so = 0;                      // (y - ys) * rowbytes
        int wo = ys * wrow;              // left weights of row y
        int sb = (ys + LEADS) * wrow_b;  // slab row y + LEADS
        int wb = (ys + PW + 1) * wrow_b; // warm row y + PW + 1
        static_for<0, U>([&](auto sc) __attribute__((always_inline)) {
            constexpr int s = decltype(sc)::value;
            const int y = ys + s;
            if constexpr (PART) {
                if (y >= y_end) return;
            }
            constexpr int bcur = s % NBUF, bnext = (s + 1) % NBUF;
            // (ys % NBUF == 0 and ys % NC == 0: strips and chunks start at multiples of U)
            float num = 1e-5f, dn = 1e-5f;
            wait_step();
            wait_lgkm0();  // half A's weights
            if constexpr (s % RB == 0) {
                asm volatile("" ::: "memory");
                __builtin_amdgcn_s_barrier();
                asm volatile("" ::: "memory");
            }
            const float *cl = reinterpret_cast<const float *>(lds + OFF_C + (s % NC) * CROW + wave * 16);
            win[(s + T - 1) % U] = cl[lane];  // row y + R
            if constexpr (DM == DM_READ) dn = reinterpret_cast<const float *>(lds + OFF_D + (s % NC) * CROW + wave * 16)[lane];
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (HV::TB > 0) {
                load_wl<HV::TA, T>(wlb, wlcol + wo);
                read_wr<T, HV::QA, HV::QT>(wrb, &lds[bcur * SROW + my_entry]);
            }
            issue((s + LEADS) % NBUF, CLAMP ? min(y + LEADS, H - 1) * wrow_b : sb, (s + PC) % NC, rc,
                  CLAMP ? (min(y + R + PC, H - 1) - cb) * rowbytes : so, rdl,
                  CLAMP ? (min(y + PC, H - 1) - db) * rowbytes : so, CLAMP ? min(y + PW + 1, H - 1) * wrow_b : wb);
            __builtin_amdgcn_sched_barrier(0);
            taps<U, s, 0, HV::TA, DM != DM_READ>(num, dn, wla, wra, win);
            __builtin_amdgcn_sched_barrier(0);
            wait_lgkm0();  // half B's weights, the window element (and den)
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (CLAMP) {
                wo = min(y + 1, H - 1) * wrow;
            } else {
                wo += wrow;
                asm volatile("" : "+s"(wo));
            }
            load_wl<0, HV::TA>(wla, wlcol + wo);
            read_wr<T, 0, HV::QA>(wra, &lds[bnext * SROW + my_entry]);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (HV::TB > 0) taps<U, s, HV::TA, T, DM != DM_READ>(num, dn, wlb, wrb, win);
            bstore<CPS>(div_pos(num, dn), ro, voff, so);
            if constexpr (DM == DM_WRITE) bstore<CPS>(dn, rd, voff, so);
            so += rowbytes;
            sb += wrow_b;
            wb += wrow_b;
            asm volatile("" : "+s"(so), "+s"(sb), "+s"(wb));
        });
    };
    int ys = y_begin;
    for (; ys + U <= y_end && ys + U - 1 + LEADS + R <= H - 1; ys += U) chunk(std::integral_constant<int, 0>{}, ys);
    for (; ys + U <= y_end; ys += U) {
        asm volatile("" : "+s"(ys));
        chunk(std::integral_constant<int, 1>{}, ys);
    }
    if (ys < y_end) chunk(std::integral_constant<int, 2>{}, ys);
    wait_vm<0>();  // no DMA may land after the block's LDS is released
}

template <int T, int DM, int LEADS = 6, int RB = 2, int NBUF = 8, int NC = 5>
void launch_vdma(const asw_params *p, const float *wl, const float *wr, const float *cin, float *cout, float *den,
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
    hipLaunchKernelGGL((k_vdma<T, DM, LEADS, RB, NBUF, NC>), dim3(8 * per_xcd * nkb * nstrip), dim3(NW * 64), 0, st,
                       wl, wr, cin, cout, den, W, H, Dp, p->d_begin, rows, nxb, nstrip, per_xcd);
}

}  // namespace agg
}  // namespace asw
