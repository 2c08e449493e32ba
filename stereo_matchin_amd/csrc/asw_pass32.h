// asw_pass32.h — the aggregation passes for a disparity shard of at most 32 planes
// (pitch Dp = 32; asw_disp_pitch).  The C4 frame d-sharded over 8 GPUs gives each
// GPU 32 of its 256 planes (BASELINE.json config 4); the 64-lane passes
// of asw_aggregate_impl.h would pad that shard to 64 planes and move twice its cost
// bytes.  Same tap sequence as every other pass (K/asw_vcost_aggregation.cl:33-40,
// K/asw_hcost_aggregation.cl:34-41; FP policy in DESIGN.md): bit-identical outputs.
//
// A wave holds 32 planes of TWO pixels: lane l is plane p = l & 31 of pixel half
// h = l >> 5.  The left weight wl_i of a voxel is then per HALF, not per wave, so it
// cannot be a scalar operand as in the 64-lane passes: the block stages the left
// support entries it needs in LDS beside the right ones, and each lane reads its
// half's entry with ds_read_b128 (the 16-lane groups of a b128 read lie inside one
// half, so a read is a broadcast: as cheap as a right-weight read).
//   k_vpass32: 16 waves = 32 columns; wave w holds columns x0+w (h=0) and x0+w+16
//              (h=1), sweeping rows.  One slab per row: the 63 right entries
//              xr = x0-d0-31 .. x0+31-d0 and the 32 left entries, in an LDS ring
//              of rows as k_vpass10.
//   k_hpass32: a wave holds rows y (h=0) and y+1 (h=1) of one row segment, sweeping
//              x; its right and left entries live in a wave-private LDS ring per row
//              (no block barrier: the waves of a block share nothing).
//              DL: the left entries never enter LDS.  Each lane loads float4 q =
//              lane & 15 of its row's left entry straight into VGPRs, a window-prefetch
//              ahead, and tap i takes wl_i from lane i/4 of its 16-lane DPP row
//              (row_newbcast, the DPP operand of the tap's v_mul_f32: no extra
//              instruction).  Half the LDS reads of a step, and 13.8 instead of 16.7 KB
//              of LDS per wave: 11 waves per CU instead of 9.
#pragma once
#include <cstdio>

#include "asw_aggregate_impl.h"

namespace asw {
namespace agg {

constexpr int kPlanes32 = 32;

// Half-size tap-major supports (odd T, R = T/2).  The weight is symmetric in its pixel
// pair (K/asw_vsupport.cl:19-25, K/asw_hsupport.cl:19-26: |p - q| per channel and the
// distance), so w(p, tap R - u) is the weight of the pixel u steps back at tap R + u,
// and at the clamped border (p - u before the first pixel: the neighbour clamps to
// pixel 0 at distance p) that of pixel 0 at tap R + p.  An array holds taps R..2R only,
// as [line][u][pos] (u = tap - R; line = row for V / column... the pass axis is pos for
// H); element index of tap t of the entry at (line, pos) along the pass axis `a`:
//   V: line = y (pass axis), pos = x;   t >= R: (y, t-R, x);  t < R, u = R-t:
//      (y-u, u, x) if y >= u, else (0, y, x).
// hs_index<T>(a, t, c, W): V form (a = row, c = column); taps >= T are padding (never
// read by the taps, the load is kept in range).
template <int T>
__device__ __forceinline__ int hs_index(int a, int t, int c, int W) {
    constexpr int R = T / 2, RH = R + 1;
    if (t >= T) t = R;  // padding: any in-range element
    if (t >= R) return (a * RH + (t - R)) * W + c;
    const int u = R - t;
    return a >= u ? ((a - u) * RH + u) * W + c : a * W + c;
}

// taps [B, E) of a phase with per-lane left weights (wl, wr hold taps from B)
template <int U, int S, int B, int E, bool DEN, int M>
__device__ __forceinline__ void taps32(float &num, float &den, const f4 (&wl)[M], const f4 (&wr)[M],
                                       const float (&win)[U]) {
#pragma unroll
    for (int i = B; i < E; ++i) {
        const float ww = wl[(i - B) / 4][(i - B) % 4] * wr[(i - B) / 4][(i - B) % 4];
        num = __builtin_fmaf(ww, win[(S + i) % U], num);
        if constexpr (DEN) den = den + ww;
    }
}

// DL: value v of lane N of each 16-lane row, as the DPP operand of its user
template <int N>
__device__ __forceinline__ float row_bcast(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x150 + N, 0xF, 0xF, true));
}

// taps [B, E) with the left weights in DPP rows (DL): wl = this lane's float4 of the
// left entry, tap i's weight in component i % 4 of lane i / 4 of the row
template <int U, int S, int B, int E, bool DEN, int M>
__device__ __forceinline__ void taps32_dl(float &num, float &den, const f4 &wl, const f4 (&wr)[M],
                                          const float (&win)[U]) {
    static_for<B, E>([&](auto ic) __attribute__((always_inline)) {
        constexpr int i = decltype(ic)::value;
        const float ww = row_bcast<i / 4>(wl[i % 4]) * wr[(i - B) / 4][(i - B) % 4];
        num = __builtin_fmaf(ww, win[(S + i) % U], num);
        if constexpr (DEN) den = den + ww;
    });
}

// ---------------------------------------------------------------------------
// k_vpass32: V pass over a 32-plane shard.  Block = NW waves = 2*NW columns
// [x0, x0 + 2 NW): wave w holds column x0 + w in lanes 0-31 and x0 + w + NW in
// lanes 32-63.  Rows are swept as in k_vpass10 (U-row chunks, running offsets, an
// NBUF-deep LDS ring of row slabs written LEAD rows ahead, one barrier per RB rows,
// weights in NPH phases with two phases' sets live).
// ---------------------------------------------------------------------------
// C16: the first V pass over the uint16 raw costs (asw_raw_cost16), as k_vpass10<C16>.
// HS: wl / wr are half-size tap-major supports (hs_index below): each staged float4 of
// an entry is assembled from 4 dwords, the slab in LDS is the same as from the full
// arrays, so the taps and the outputs are unchanged.
template <int T, int NW, int DM, int CP, int NPH, int RB = 2, int PS = 4, bool C16 = false, bool HS = false>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(NW >= 16 ? 4 : 2))) void k_vpass32(
    const float *__restrict__ wl, const float *__restrict__ wr, const float *__restrict__ cin, float *__restrict__ cout,
    float *__restrict__ den, int W, int H, int d_begin, int rows_per_strip, int nxb, int nstrip, int xg_per_xcd) {
    constexpr int R = T / 2;
    constexpr int TP = tap_pitch(T);
    constexpr int Q = TP / 4;
    constexpr int U = pf9_period(T);
    constexpr int P = U - T;
    constexpr int KD = 2;  // den prefetch ring (rows)
    constexpr int LEAD = RB + 1;
    constexpr int NBUF = ring_div(U, 2 * RB + 1);
    static_assert(U % PS == 0 && U % KD == 0 && U % RB == 0 && U % NBUF == 0, "ring periods");
    static_assert(LEAD <= PS, "staging ring too short for the barrier period");
    constexpr int LA = cmax(cmax(R + P, LEAD + PS), KD);  // rows past y a step touches
    constexpr int NC = 2 * NW;                             // columns per block
    constexpr int NER = NC + 31;                           // right entries per row
    constexpr int NE = NER + NC;                           // + the left entries
    constexpr int NQ = NE * Q;
    constexpr int NSTAGE = (NQ + NW * 64 - 1) / (NW * 64);
    static_assert(NSTAGE <= 2, "slab row larger than two float4 per thread");
    __shared__ f4 slab[NBUF][NQ];

    const int xcd = blockIdx.x & 7, m = blockIdx.x >> 3;
    const int xg = xcd * xg_per_xcd + m % xg_per_xcd;
    const int strip = m / xg_per_xcd;
    if (xg >= nxb || strip >= nstrip) return;  // padding block (uniform)
    const int x0 = xg * NC;
    const int y_begin = strip * rows_per_strip;
    if (y_begin >= H) return;
    const int y_end = min(H, y_begin + rows_per_strip);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int half = lane >> 5, pl = lane & 31;
    const int xc = min(x0 + wave + NW * half, W - 1);  // columns past the right edge recompute W-1
    const int my_wr = ((xc - x0) + 31 - pl) * Q;       // entry xr = xc - d_begin - pl
    const int my_wl = (NER + (xc - x0)) * Q;
    const long long rowstride = (long long)W * kPlanes32;
    const int rowbytes = (int)(rowstride * 4);  // U+LA rows < 2 GiB: checked by the launcher
    const long long colbase = (long long)x0 * kPlanes32;
    const int voff = ((xc - x0) * kPlanes32 + pl) * 4;
    const long long wrow = (long long)W * TP;  // floats per support row
    auto rsrc_at = [&](const float *base, int row) __attribute__((always_inline)) {
        return make_rsrc(base + (long long)row * rowstride + colbase);
    };
    auto cin_at = [&](int row) __attribute__((always_inline)) {
        if constexpr (C16) return make_rsrc(reinterpret_cast<const uint16_t *>(cin) + (long long)row * rowstride + colbase);
        else return rsrc_at(cin, row);
    };
    auto cload = [&](rsrc_t r, int off) __attribute__((always_inline)) {  // off: bytes of the float volume
        if constexpr (C16) return bload16<CP>(r, voff >> 1, off >> 1);
        else return bload<CP>(r, voff, off);
    };
    // C16: window elements in flight stay integers (a P-deep ring), converted the step
    // they enter the window, as k_vpass10<C16>
    auto cload_raw = [&](rsrc_t r, int off) __attribute__((always_inline)) {
        return (unsigned)__builtin_amdgcn_raw_buffer_load_b16(r, voff >> 1, off >> 1, CP);
    };
    constexpr int PR = ring_div(U, P);  // (a divisor of U: compile-time slots in every chunk)
    unsigned r16[C16 ? PR : 1];         // the load of step s sits in slot s mod PR until step s + P

    // slab row staging: thread share t0 (t1) = float4 q of entry e; entries < NER are
    // right weights of xr = x0 - d_begin - 31 + e, the rest left weights of column
    // x0 + e - NER (both clamped into the row); surplus threads redo the last one
    const int t0 = min((int)threadIdx.x, NQ - 1);
    const int t1 = min((int)threadIdx.x + NW * 64, NQ - 1);
    // element offset of share t's float4 in its (row 0) support row: right weights of
    // entries < NER, else left
    auto src_of = [&](int t) __attribute__((always_inline)) {
        const int e = t / Q, q = t - e * Q;
        if (e < NER) return clampi(x0 - d_begin - 31 + e, 0, W - 1) * TP + 4 * q;
        return min(x0 + e - NER, W - 1) * TP + 4 * q;
    };
    const int o0 = src_of(t0), o1 = src_of(t1);
    const bool r0 = t0 / Q < NER, r1 = t1 / Q < NER;
    const float *src0 = (r0 ? wr : wl) + o0;
    const float *src1 = (r1 ? wr : wl) + o1;
    // HS: threads [0, NSR) stage the right entries, [NSR, NSR + NER... ) the left ones
    // (wave-uniform array: one buffer resource per wave), q-major inside each part so the
    // lanes of a dword load are consecutive columns of one tap row (coalesced), and the
    // b128 slab write of consecutive entries keeps its odd-Q stride (conflict-free)
    constexpr int NSR = (NER * Q + 63) / 64 * 64;
    static_assert(!HS || (NSR + NC * Q <= NW * 64 && NSTAGE == 1), "HS: one share per thread");
    const int th = (int)threadIdx.x;
    const bool hs_right = th < NSR;
    const int hs_n = hs_right ? NER : NC;
    const int hs_t = hs_right ? min(th, NER * Q - 1) : min(th - NSR, NC * Q - 1);
    const int hs_e = hs_t % hs_n, hs_q = hs_t / hs_n;
    const int hs_col = hs_right ? clampi(x0 - d_begin - 31 + hs_e, 0, W - 1) : min(x0 + hs_e, W - 1);
    const int hs_slot = ((hs_right ? 0 : NER) + hs_e) * Q + hs_q;
    const rsrc_t hs_rs = make_rsrc(__builtin_amdgcn_readfirstlane((int)hs_right) ? wr : wl);
    // rows >= R (all but the first R of the image): element offset of tap 4q+j = (row -
    // R) * (R+1) * W (scalar) + hs_off[j], its offset at row R (the vector offset stays
    // non-negative: the buffer range check takes it as unsigned)
    int hs_off[HS ? 4 : 1];
    if constexpr (HS) {
#pragma unroll
        for (int j = 0; j < 4; ++j) hs_off[j] = hs_index<T>(R, 4 * hs_q + j, hs_col, W);
    }
    auto stage = [&](f4 &a, f4 &b, int row) __attribute__((always_inline)) {
        if constexpr (HS) {
            if (row >= R) {
                const int so = (row - R) * (R + 1) * W * 4;
#pragma unroll
                for (int j = 0; j < 4; ++j) a[j] = bload(hs_rs, hs_off[j] * 4, so);
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    a[j] = bload(hs_rs, hs_index<T>(row, 4 * hs_q + j, hs_col, W) * 4, 0);
            }
        } else {
            a = *reinterpret_cast<const f4 *>(src0 + row * wrow);
            if constexpr (NSTAGE > 1) b = *reinterpret_cast<const f4 *>(src1 + row * wrow);
        }
    };
    auto put = [&](int buf, const f4 &a, const f4 &b) __attribute__((always_inline)) {
        if constexpr (HS) {
            slab[buf][hs_slot] = a;
        } else {
            slab[buf][t0] = a;
            if constexpr (NSTAGE > 1) slab[buf][t1] = b;
        }
    };

    using PH = Phases<T, NPH>;
    float win[U];
    f4 sa[PS], sb[PS];
    f4 wlp[NPH][PH::NG], wrp[NPH][PH::NG];
    float dring[KD];
    {
        const int r0 = max(0, y_begin - R);
        const rsrc_t rp = cin_at(r0);
#pragma unroll
        for (int j = 0; j < U - 1; ++j) {
            const int off = (clampi(y_begin - R + j, 0, H - 1) - r0) * rowbytes;
            if constexpr (C16) {
                if (j < T - 1) win[j] = cload(rp, off);
                else r16[(j - (T - 1) - P + PR) % PR] = cload_raw(rp, off);  // "loaded" at step j-(T-1)-P
            } else {
                win[j] = cload(rp, off);
            }
        }
    }
    if constexpr (DM == DM_READ) {
        const rsrc_t rp = rsrc_at(den, y_begin);
#pragma unroll
        for (int j = 0; j < KD; ++j) dring[j] = bload<CP>(rp, voff, (min(y_begin + j, H - 1) - y_begin) * rowbytes);
    }
#pragma unroll
    for (int j = 0; j < PS; ++j) stage(sa[j], sb[j], min(y_begin + j, H - 1));
#pragma unroll
    for (int j = 0; j < LEAD; ++j) put(j, sa[j], sb[j]);
#pragma unroll
    for (int j = 0; j < LEAD; ++j) stage(sa[j], sb[j], min(y_begin + PS + j, H - 1));
    __syncthreads();
    auto request = [&](auto kc, int buf) __attribute__((always_inline)) {
        constexpr int k = decltype(kc)::value;
        read_wr<T, PH::gb(k), PH::gb(k + 1)>(wlp[k], &slab[buf][my_wl]);
        read_wr<T, PH::gb(k), PH::gb(k + 1)>(wrp[k], &slab[buf][my_wr]);
    };
    (void)r1;
    request(std::integral_constant<int, 0>{}, 0);

    // mode 0: interior chunk; 1: clamped row addresses; 2: clamped and partial (rows >= y_end skipped)
    auto chunk = [&](auto mode_c, int ys) __attribute__((always_inline)) {
        constexpr bool CLAMP = decltype(mode_c)::value >= 1;
        constexpr bool PART = decltype(mode_c)::value == 2;
        const int cb = min(ys + R + P, H - 1);
        const rsrc_t rc = cin_at(cb);
        const rsrc_t ro = rsrc_at(cout, ys);
        const rsrc_t rd = rsrc_at(den, ys);
        const rsrc_t rdn = rsrc_at(den, min(ys + KD, H - 1));
        int so = 0;  // (y - ys) * rowbytes
        static_for<0, U>([&](auto sc) __attribute__((always_inline)) {
            constexpr int s = decltype(sc)::value;
            const int y = ys + s;
            if constexpr (PART) {
                if (y >= y_end) return;
            }
            constexpr int bcur = s % NBUF, bnext = (s + 1) % NBUF, bput = (s + LEAD) % NBUF;
            float num = 1e-5f, dn = 1e-5f;
            if constexpr (C16) win[(s + T - 1) % U] = (float)r16[(s - P + PR) % PR];  // row y+R, loaded P steps ago
            static_for<0, NPH>([&](auto kc) __attribute__((always_inline)) {
                constexpr int k = decltype(kc)::value;
                // (lgkmcnt 0) phase k's weights are in; at k = 0 every RB rows, also the
                // slab rows up to y + RB (barrier)
                if constexpr (k == 0 && s % RB == 0) __syncthreads();
                else wait_lgkm0();
                if constexpr (k == 0) asm volatile("" ::"v"(win[(s + T - 1) % U]));  // one vmcnt wait per step
                __builtin_amdgcn_sched_barrier(0);
                if constexpr (k + 1 < NPH) request(std::integral_constant<int, k + 1>{}, bcur);
                else request(std::integral_constant<int, 0>{}, bnext);
                if constexpr (k == 0) {
                    put(bput, sa[(s + LEAD) % PS], sb[(s + LEAD) % PS]);
                    stage(sa[(s + LEAD) % PS], sb[(s + LEAD) % PS], min(y + LEAD + PS, H - 1));
                }
                __builtin_amdgcn_sched_barrier(0);
                taps32<U, s, PH::tb(k), PH::tb(k + 1), DM != DM_READ>(num, dn, wlp[k], wrp[k], win);
                __builtin_amdgcn_sched_barrier(0);
            });
            if constexpr (DM == DM_READ) {
                dn = dring[s % KD];
                dring[s % KD] = bload<CP>(rdn, voff, CLAMP ? (min(y + KD, H - 1) - min(ys + KD, H - 1)) * rowbytes : so);
            } else if constexpr (DM == DM_WRITE) {
                bstore<CP>(dn, rd, voff, so);
            }
            bstore<CP>(div_pos(num, dn), ro, voff, so);
            if constexpr (C16) r16[s % PR] = cload_raw(rc, CLAMP ? (min(y + R + P, H - 1) - cb) * rowbytes : so);
            else win[(s + U - 1) % U] = cload(rc, CLAMP ? (min(y + R + P, H - 1) - cb) * rowbytes : so);
            so += rowbytes;
            asm volatile("" : "+s"(so));
        });
    };
    int ys = y_begin;
    for (; ys + U <= y_end && ys + U - 1 + LA <= H - 1; ys += U) chunk(std::integral_constant<int, 0>{}, ys);
    // whole chunks that reach the image bottom, then the partial last one (k_vpass10)
    for (; ys + U <= y_end; ys += U) {
        asm volatile("" : "+s"(ys));
        chunk(std::integral_constant<int, 1>{}, ys);
    }
    if (ys < y_end) chunk(std::integral_constant<int, 2>{}, ys);
}

// ---------------------------------------------------------------------------
// k_hpass32: H pass over a 32-plane shard.  A wave = rows y (lanes 0-31) and y+1
// (lanes 32-63) of one row segment [xs, xe), sweeping x; block = NWB such waves
// (independent).  Per row the wave keeps a private LDS ring of right entries
// (slot = xr mod RING; at step x lane p reads xr = x - d_begin - p) and of left
// entries (slot = x mod LRING), refilled K entries at a time from one float4 per
// lane loaded a batch ahead.  The wave reads only what it wrote itself, in program
// order (LDS operations of a wave complete in order): no barrier.
//   Batch b (steps [xb, xb+K)) reads right entries [xb-d0-31, xb+K-d0] and left
//   entries [xb, xb+K] (the last ones: half A... phase 0 of the next step); its top
//   writes batch b+1's new ones: right [xb+K+1-d0, xb+2K-d0], left [xb+K+1, xb+2K].
// ---------------------------------------------------------------------------
constexpr int h32_batch(int T) { return tap_pitch(T) / 4 * 8 <= 64 * 4 ? 4 : 2; }

// RING16: right ring of a multiple of 16 entries (conflict-free across the wrap) or
// the minimal 32 + 2K (a 2-way conflict where a read wraps; less LDS, more waves)
// KB: the refill batch (0: h32_batch).
// (Round 5: the weights requested two phases ahead instead of one measured 0.3115
// against 0.3173 ms per pass and the same shard frame, profiles/r05/pd2_nt_r12c.log;
// not kept.)
// PX: extra cost-prefetch steps (tools/exp; the left-weight ring then keeps a 5-step lead)
template <int T, int NWB, int DM, int CP, int NPH, bool RING16 = true, int WPE = 2, int KB = 0, bool DL = false,
          int PX = 0>
__global__ __launch_bounds__(NWB * 64) __attribute__((amdgpu_waves_per_eu(WPE))) void k_hpass32(
    const float *__restrict__ wl, const float *__restrict__ wr, const float *__restrict__ cin, float *__restrict__ cout,
    float *__restrict__ den, int W, int H, int d_begin, int nseg, int seg_len, int npairs, int pairs_per_xcd) {
    constexpr int R = T / 2;
    constexpr int TP = tap_pitch(T);
    constexpr int Q = TP / 4;
    constexpr int U = pf9_period(T) + PX;
    constexpr int P = U - T;
    constexpr int KD = 4;  // den prefetch ring (steps)
    constexpr int K = KB ? KB : h32_batch(T);
    constexpr int RING = RING16 ? (32 + 2 * K + 15) / 16 * 16 : 32 + 2 * K;  // right entries per row
    constexpr int LRING = DL ? 0 : 2 * K + 2;          // left entries per row (not DL)
    constexpr int ROWE = RING + LRING;                 // ring entries per row
    static_assert(U % K == 0, "the batch top must be a compile-time step");
    static_assert(!DL || (T + 3) / 4 <= 16, "DL: taps in one DPP row");
    // staged per batch: 2 rows x (K right + K left entries, DL: K right) x Q float4 over 64 lanes
    constexpr int NK = DL ? 1 : 2;
    constexpr int NST = 2 * NK * K * Q;
    constexpr int SPL = (NST + 63) / 64;  // float4 per lane
    __shared__ f4 ring_all[NWB][2 * ROWE * Q];

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // work item = (row pair, segment); XCD-aware: consecutive items on one XCD
    const int xcd = blockIdx.x & 7, m = blockIdx.x >> 3;
    const int item_l = m * NWB + wave;
    if (item_l >= pairs_per_xcd) return;  // whole wave
    const int item = xcd * pairs_per_xcd + item_l;
    if (item >= npairs) return;
    const int pr = item / nseg;
    const int xs = (item - pr * nseg) * seg_len;
    const int xe = min(xs + seg_len, W);
    const int half = lane >> 5, pl = lane & 31;
    const int y = min(2 * pr + half, H - 1);  // an odd last row: both halves on it (same values, same place)
    const int d0 = d_begin;
    f4 *ring = ring_all[wave];
    f4 *myrow = ring + half * ROWE * Q;

    // staging share j of lane l: float4 n = j*64 + l of the batch's NST, with
    // n = ((r*2 + kind)*K + k)*Q + q: row r, kind 0 = right entry xb+1-d0+k, kind 1 =
    // left entry xb+1+k of the batch whose first step is xb (its entries are written at
    // the top of batch xb - K, the batch before the one that first reads them)
    using stg_t = f4;  // a staged share: 4 weights
    using elem_t = float;
    const elem_t *wre = wr, *wle = wl;
    const elem_t *wrrows[2] = {wre + (long long)min(2 * pr, H - 1) * W * TP, wre + (long long)min(2 * pr + 1, H - 1) * W * TP};
    const elem_t *wlrows[2] = {wle + (long long)min(2 * pr, H - 1) * W * TP, wle + (long long)min(2 * pr + 1, H - 1) * W * TP};
    auto weights = [](const stg_t &a) __attribute__((always_inline)) { return a; };
    // (the share's row is a global-address-space pointer: a generic one compiles to
    // flat loads, which also count against lgkmcnt, so every LDS wait of the step loop
    // would wait for the staging loads of the next batch as well; the clamp is the
    // same arithmetic for both kinds, st_sub = d0 or 0, so no branch either)
    using gelem_t = const __attribute__((address_space(1))) elem_t;
    gelem_t *st_row[SPL];
    int st_q4[SPL], st_k[SPL], st_kind[SPL], st_sub[SPL], st_slot[SPL], st_base[SPL];
#pragma unroll
    for (int j = 0; j < SPL; ++j) {
        const int n = min(j * 64 + lane, NST - 1);
        const int q = n % Q, k = (n / Q) % K, kind = (n / (Q * K)) % NK, r = n / (NK * Q * K);
        st_row[j] = (gelem_t *)(kind == 0 ? wrrows[r] : wlrows[r]);
        st_q4[j] = 4 * q;
        st_k[j] = k;
        st_kind[j] = kind;
        st_sub[j] = kind == 0 ? d0 : 0;
        // LDS float4 index of the entry for the first top (xb = xs: entries of batch xs + K)
        const int e = xs + K + 1 + k;
        st_slot[j] = kind == 0 ? (r * ROWE + (e - d0 + (1 << 20)) % RING) * Q + q
                               : (r * ROWE + RING + e % (DL ? 1 : LRING)) * Q + q;
        st_base[j] = kind == 0 ? r * ROWE * Q : (r * ROWE + RING) * Q;
    }
    auto st_load = [&](int j, int xb) __attribute__((always_inline)) {  // entry of the batch starting at xb
        const int c = clampi(xb + 1 + st_k[j] - st_sub[j], 0, W - 1);  // (left: xb + 1 + k >= 0)
        return *reinterpret_cast<const __attribute__((address_space(1))) stg_t *>(st_row[j] + c * TP + st_q4[j]);
    };

    // the rings before step xs: right entries [xs-d0-31, xs+K-d0], left [xs, xs+K]
    constexpr int NR0 = 32 + K, NL0 = DL ? 0 : K + 1;
    for (int t = lane; t < 2 * (NR0 + NL0) * Q; t += 64) {
        const int q = t % Q, ee = t / Q;
        const int r = ee / (NR0 + NL0), e = ee % (NR0 + NL0);
        f4 v;
        int slot;
        if (e < NR0) {
            const int xr = xs - d0 - 31 + e;
            v = weights(*reinterpret_cast<const stg_t *>(wrrows[r] + clampi(xr, 0, W - 1) * TP + 4 * q));
            slot = (xr + (1 << 20)) % RING;
        } else {
            const int x = xs + e - NR0;
            v = weights(*reinterpret_cast<const stg_t *>(wlrows[r] + min(x, W - 1) * TP + 4 * q));
            slot = RING + x % (DL ? 1 : LRING);
        }
        ring[(r * ROWE + slot) * Q + q] = v;
    }
    stg_t stg[SPL];
#pragma unroll
    for (int j = 0; j < SPL; ++j) stg[j] = st_load(j, xs + K);

    // buffer resources at the pair's first row (wave-uniform); half 1 reaches its row
    // through the lane offset (W * 128 B per row)
    const long long rowoff = (long long)(2 * pr) * W * kPlanes32;
    const rsrc_t rc = make_rsrc(cin + rowoff);
    const rsrc_t ro = make_rsrc(cout + rowoff);
    const rsrc_t rd = make_rsrc(den + rowoff);
    const int voff = pl * 4 + (y - 2 * pr) * W * kPlanes32 * 4;
    constexpr int xstride = kPlanes32 * 4;  // bytes per column
    // LDS float4 index of this lane's entries at step x.  The right slot (x - d0 - pl)
    // mod RING is per lane: computed once per U-step chunk (rs0, at its first step xb),
    // then slot(xb + s) = rs0 + s, less RING past the end (s <= U: at most two
    // subtractions), instead of a modulo per request
    static_assert(U < 2 * RING, "at most two wraps per chunk");
    auto wr_slot0 = [&](int xb) __attribute__((always_inline)) { return (xb - d0 - pl + (1 << 20)) % RING; };
    auto wr_at = [&](int rs0, int s) __attribute__((always_inline)) {
        int v = rs0 + s;
        v = v >= RING ? v - RING : v;
        if (s >= RING) v = v >= RING ? v - RING : v;  // (s is a compile-time step)
        return myrow + v * Q;
    };
    auto wl_at = [&](int x) __attribute__((always_inline)) { return myrow + (RING + x % (DL ? 1 : LRING)) * Q; };
    // DL: this lane's float4 of its row's left entry at a column (global-address pointer)
    using gf4 = const __attribute__((address_space(1))) f4;
    gelem_t *wlsrc = (gelem_t *)(wle + (long long)y * W * TP + 4 * min(lane & 15, Q - 1));
    auto wl_load = [&](int x) __attribute__((always_inline)) { return *(gf4 *)(wlsrc + min(x, W - 1) * TP); };
    constexpr int NLD = DL ? ring_div(U, PX ? 5 : P) : 1;  // left columns in flight (>= the window's P)
    f4 wld[NLD];
    if constexpr (DL) {
#pragma unroll
        for (int j = 0; j < NLD; ++j) wld[j] = wl_load(xs + j);
    }

    using PH = Phases<T, NPH>;
    float win[U];
    f4 wlp[DL ? 1 : NPH][PH::NG], wrp[NPH][PH::NG];
    float dring[KD];
#pragma unroll
    for (int j = 0; j < U - 1; ++j) win[j] = bload<CP>(rc, voff, clampi(xs - R + j, 0, W - 1) * xstride);
    if constexpr (DM == DM_READ) {
#pragma unroll
        for (int j = 0; j < KD; ++j) dring[j] = bload<CP>(rd, voff, min(xs + j, W - 1) * xstride);
    }
    // weights of phase k at step x = xb + s (rs0: the right slot at xb)
    auto request = [&](auto kc, int x, int rs0, int s) __attribute__((always_inline)) {
        constexpr int k = decltype(kc)::value;
        if constexpr (!DL) read_wr<T, PH::gb(k), PH::gb(k + 1)>(wlp[k], wl_at(x));
        read_wr<T, PH::gb(k), PH::gb(k + 1)>(wrp[k], wr_at(rs0, s));
    };
    request(std::integral_constant<int, 0>{}, xs, wr_slot0(xs), 0);

    auto body = [&](auto sc, auto chk, int xb, int rs0) __attribute__((always_inline)) {
        constexpr int s = decltype(sc)::value;
        constexpr bool CHK = decltype(chk)::value;
        const int x = xb + s;
        if constexpr (CHK) {
            if (x >= xe) return;
        }
        if constexpr (s % K == 0) {
            // top of a batch (steps [x, x+K)): write the entries the next batch reads
            // first (loaded a batch ago), then load the ones after them
            f4 wv[SPL];
#pragma unroll
            for (int j = 0; j < SPL; ++j) wv[j] = weights(stg[j]);
#pragma unroll
            for (int j = 0; j < SPL; ++j) {
                ring[st_slot[j]] = wv[j];
                // advance the slot by K entries inside its ring (RING or LRING entries)
                const int lim = st_kind[j] == 0 ? RING * Q : LRING * Q;
                int rel = st_slot[j] - st_base[j] + K * Q;
                rel = rel >= lim ? rel - lim : rel;
                st_slot[j] = st_base[j] + rel;
            }
#pragma unroll
            for (int j = 0; j < SPL; ++j) stg[j] = st_load(j, x + 2 * K);
        }
        float num = 1e-5f, dn = 1e-5f;
        static_for<0, NPH>([&](auto kc) __attribute__((always_inline)) {
            constexpr int k = decltype(kc)::value;
            wait_lgkm0();
            if constexpr (k == 0) asm volatile("" ::"v"(win[(s + T - 1) % U]));  // one vmcnt wait per step
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (k + 1 < NPH) request(std::integral_constant<int, k + 1>{}, x, rs0, s);
            else request(std::integral_constant<int, 0>{}, x + 1, rs0, s + 1);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (DL) taps32_dl<U, s, PH::tb(k), PH::tb(k + 1), DM != DM_READ>(num, dn, wld[s % NLD], wrp[k], win);
            else taps32<U, s, PH::tb(k), PH::tb(k + 1), DM != DM_READ>(num, dn, wlp[k], wrp[k], win);
            __builtin_amdgcn_sched_barrier(0);
        });
        if constexpr (DL) wld[s % NLD] = wl_load(x + NLD);  // column x+NLD's left entry
        const int xo = x * xstride;
        if constexpr (DM == DM_READ) {
            dn = dring[s % KD];
            dring[s % KD] = bload<CP>(rd, voff, min(x + KD, W - 1) * xstride);
        } else if constexpr (DM == DM_WRITE) {
            bstore<CP>(dn, rd, voff, xo);
        }
        bstore<CP>(div_pos(num, dn), ro, voff, xo);
        win[(s + U - 1) % U] = bload<CP>(rc, voff, min(x + R + P, W - 1) * xstride);
    };
    int xb = xs;
    for (; xb + U <= xe; xb += U) {
        const int rs0 = wr_slot0(xb);
        static_for<0, U>([&](auto sc) __attribute__((always_inline)) { body(sc, std::false_type{}, xb, rs0); });
    }
    if (xb < xe) {
        const int rs0 = wr_slot0(xb);
        static_for<0, U>([&](auto sc) __attribute__((always_inline)) { body(sc, std::true_type{}, xb, rs0); });
    }
}

// ---------------------------------------------------------------------------
// launchers (one (T, DM) per translation unit: build/p32_t<T>_d<DM>.hip)
// ---------------------------------------------------------------------------
template <int T, int NW, int DM, int CP, int NPH, bool C16 = false, bool HS = false>
void launch_v32(const asw_params *p, const float *wl, const float *wr, const float *cin, float *cout, float *den,
                hipStream_t st) {
    constexpr int U = pf9_period(T);
    const int W = p->width, H = p->height;
    const int nxb = (W + 2 * NW - 1) / (2 * NW);
    // row strips: about one block per CU slot (NW = 16: one block per CU, 256 slots) so
    // the grid is one full round, not a round and a tail; strips of whole U-row chunks,
    // >= 2T rows (the window prologue, U-1 row loads per strip).  Variant bits 16-19
    // (asw_tune_set) override the strip count.
    const int slots = 256 * 16 / NW;
    int nstrip = (slots + nxb / 2) / nxb;
    const int max_strip = H / (2 * T) > 1 ? H / (2 * T) : 1;
    if (nstrip > max_strip) nstrip = max_strip;
    if ((g_pass_variant >> 16) & 15) nstrip = (g_pass_variant >> 16) & 15;
    if (nstrip < 1) nstrip = 1;
    const int rows = ((H + nstrip - 1) / nstrip + U - 1) / U * U;
    nstrip = (H + rows - 1) / rows;
    const int per_xcd = (nxb + 7) / 8;
    hipLaunchKernelGGL((k_vpass32<T, NW, DM, CP, NPH, 2, 4, C16, HS>), dim3(8 * per_xcd * nstrip), dim3(NW * 64), 0, st, wl,
                       wr, cin, cout, den, W, H, p->d_begin, rows, nxb, nstrip, per_xcd);
    note_pass_kernel(ASW_DIR_V, DM, C16 ? "k_vpass32_c16" : "k_vpass32", T,
                     NW == 16 ? (NPH == 4 ? "NW=16,NPH=4" : "NW=16") : "NW=8,NPH=3", CP == kCPStream);
}

template <int T, int NWB, int DM, int CP, int NPH, bool RING16 = true, int WPE = 2, int KB = 0, bool DL = false,
          int PX = 0>
void launch_h32(const asw_params *p, const float *wl, const float *wr, const float *cin, float *cout, float *den,
                hipStream_t st, int seg_len) {
    const int W = p->width, H = p->height;
    const int nseg = (W + seg_len - 1) / seg_len;
    const int npairs = (H + 1) / 2 * nseg;  // work items: (row pair, segment)
    const int per_xcd = (npairs + 7) / 8;
    const int blocks_per_xcd = (per_xcd + NWB - 1) / NWB;
    hipLaunchKernelGGL((k_hpass32<T, NWB, DM, CP, NPH, RING16, WPE, KB, DL, PX>), dim3(8 * blocks_per_xcd), dim3(NWB * 64),
                       0, st, wl, wr, cin, cout, den, W, H, p->d_begin, nseg, seg_len, npairs, per_xcd);
    note_pass_kernel(ASW_DIR_H, DM, "k_hpass32", T,
                     DL ? (PX ? "NWB=1,NPH=4,DL,PX=8" : "NWB=1,NPH=4,DL") : NWB == 4 ? "NWB=4" : "NWB=2",
                     CP == kCPStream);
}

inline int finish32() {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_hip_error(e);
        return ASW_E_HIP;
    }
    return ASW_OK;
}

template <int T, int DM>
int launch_pass32_tm(const asw_params *p, int dir, const float *wl, const float *wr, const float *cin, float *cout,
                     float *den, hipStream_t st) {
    constexpr int U = pf9_period(T);
    // the nt cache policy for the cost / den / output streams from 256 MiB of volume (the
    // C4 8-way shard, 1920 x 1080 x 32 x 4 B = 253 MiB, stays below); variant bit 26 flips it
    bool stream = (long long)p->width * p->height * kPlanes32 * 4 >= (256LL << 20);
    if (g_pass_variant & (1 << 26)) stream = !stream;
    if (dir == ASW_DIR_V) {
        // 16 waves (1024 threads, 4 waves per SIMD: <= 128 VGPRs): the per-lane left
        // weights take as many registers as the right ones, so T >= 33 keeps two of
        // four phases' weights live (three phases: 179 VGPRs spilled at T = 35; four:
        // 118 VGPRs).  T > 35: 8 waves (16 columns), up to 256 VGPRs.
        constexpr int NW = T > 35 ? 8 : 16;
        constexpr int NPH = T > 35 ? 3 : T >= 33 ? 4 : 2;
        if (stream) launch_v32<T, NW, DM, kCPStream, NPH>(p, wl, wr, cin, cout, den, st);
        else launch_v32<T, NW, DM, 0, NPH>(p, wl, wr, cin, cout, den, st);
    } else {
        // T <= 35: the "lean" form, 4 weight phases in one-wave blocks (up to 11 waves per
        // CU against 8 for 4-wave blocks; C4 / 8 den-read 0.326 against 0.358 ms,
        // profiles/r04/pass32_h_r09e.log), the conflict-free 48-entry right ring (C4 8-way
        // shard frame 4.73 against 4.81-4.98 ms with the minimal 40-entry ring,
        // profiles/r04/shard_variants_r11g.log) and the left weights from DPP rows (DL: in
        // the C4 / 8 frame 0.325 against 0.355 ms per pass under rocprofv3, shard frame
        // 4.71-4.74 against 4.74-4.88 ms with the left ring in LDS, round 5,
        // profiles/r05/kernel_stats_r12q_shard8_hdl.csv, shard_hdl_r12q.log).  Segments per
        // row pair sized to the 11 wave slots per CU its LDS admits (C4: 5 segments of 384
        // columns); the window prologue (U-1 columns) is paid once per segment.  Variant
        // bits 20-23 (asw_tune_set) override the segment count.
        // T > 35: 2-wave blocks, 2 weight phases.
        const int pairs = (p->height + 1) / 2;
        const int slots = T <= 35 ? 256 * 11 : 2048;
        int nseg = (slots + pairs / 2) / (pairs > 0 ? pairs : 1);
        if ((g_pass_variant >> 20) & 15) nseg = (g_pass_variant >> 20) & 15;
        if (nseg < 1) nseg = 1;
        // (T = 35: the window period of the deeper-prefetch form below)
        constexpr int UH = T == 35 ? pf9_period(T) + 8 : U;
        int seg = ((p->width + nseg - 1) / nseg + UH - 1) / UH * UH;
        if (seg < 2 * UH) seg = 2 * UH;
        if constexpr (T <= 35) {
            // T = 35 (the C4 shard): the newest window element requested 13 instead of 5
            // steps ahead (the pass waits on vmcnt, not LDS: SQ_WAIT_INST_ANY 0.34 of its
            // wave cycles, WAIT_INST_LDS 0.006, profiles/r06/pmc_shard8_r15d.json), and
            // 48-column window periods tile the C4 segments of 384 columns exactly:
            // 0.286 against 0.295 ms per pass (profiles/r06/h32_px_r15f.log)
            constexpr int PXH = UH - U;
            if (stream) launch_h32<T, 1, DM, kCPStream, 4, true, 3, 0, true, PXH>(p, wl, wr, cin, cout, den, st, seg);
            else launch_h32<T, 1, DM, 0, 4, true, 3, 0, true, PXH>(p, wl, wr, cin, cout, den, st, seg);
        } else {
            if (stream) launch_h32<T, 2, DM, kCPStream, 2>(p, wl, wr, cin, cout, den, st, seg);
            else launch_h32<T, 2, DM, 0, 2>(p, wl, wr, cin, cout, den, st, seg);
        }
    }
    return finish32();
}

// the first V pass over the uint16 raw costs (asw_aggregate_pass_den16): den modes NONE
// (what a 32-plane shard's passes run) and WRITE
template <int T, int DM>
int launch_pass32_c16_tm(const asw_params *p, const float *wl, const float *wr, const uint16_t *cin16, float *cout,
                         float *den, hipStream_t st) {
    if constexpr (DM == DM_READ) {
        return ASW_E_INVALID;  // (never a first pass)
    } else {
        constexpr int NW = T > 35 ? 8 : 16;
        constexpr int NPH = T > 35 ? 3 : T >= 33 ? 4 : 2;
        bool stream = (long long)p->width * p->height * kPlanes32 * 4 >= (256LL << 20);
        if (g_pass_variant & (1 << 26)) stream = !stream;
        const float *c = reinterpret_cast<const float *>(cin16);
        if (stream) launch_v32<T, NW, DM, kCPStream, NPH, true>(p, wl, wr, c, cout, den, st);
        else launch_v32<T, NW, DM, 0, NPH, true>(p, wl, wr, c, cout, den, st);
        return finish32();
    }
}

}  // namespace agg
}  // namespace asw

#define ASW_INSTANTIATE_PASS32(TT, DM)                                                                            \
    template int asw::agg::launch_pass32_tm<TT, DM>(const asw_params *, int, const float *, const float *,       \
                                                    const float *, float *, float *, hipStream_t);               \
    template int asw::agg::launch_pass32_c16_tm<TT, DM>(const asw_params *, const float *, const float *,        \
                                                        const uint16_t *, float *, float *, hipStream_t);
