// asw_refine.hip — the lane-per-pixel WTA scan (asw_WTA and asw_WTA_REF) and the
// refinement loop of the reference (main.cpp:540-623): asw_ref_v, asw_ref_h,
// asw_WTA_REF, Constistency (asw_consistency), then the 3x3 Median.
//
// WTA scan (K/asw_wta.cl:25-67, K/asw_wta_ref.cl:21-57).  The reference scans d
// sequentially per pixel with strict '<'; here each LANE owns one pixel and runs
// that same sequential scan, so ties, the multiset second minimum and the
// 100000 sentinels are reproduced by construction (no cross-lane reduction).
// The volume is pixel-major [H][W][Dp]: a wave's 64 pixels are 64 rows of Dp
// floats, so a chunk of 32 planes is loaded coalesced (8 lanes per pixel, one
// float4 each) and transposed through a private LDS tile [64][33] (row pitch 33:
// the 32 lanes of a ds_read_b32 group hit 32 distinct banks, and so do the
// ds_write_b32 of the transpose).  The next chunk's loads are in flight while
// the current one is scanned.  The target scan (the bresenham diagonal
// C[b][y][max(0,x-i)], b = md + max(0,x-i) - x) is a per-lane gather of the
// row the wave just streamed (L2-resident).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "asw_common.h"

namespace asw {
namespace {

constexpr float kSentinel = 100000.0f;  // K/asw_wta.cl:25-26, K/asw_wta_ref.cl:20-21
constexpr int kChunk = 32;              // planes per transposed chunk
constexpr int kTilePitch = kChunk + 1;

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

using rsrc_t = __amdgpu_buffer_rsrc_t;
__device__ __forceinline__ rsrc_t make_rsrc_n(const void *p, int nbytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, nbytes, 0x00020000);
}
__device__ __forceinline__ float bload(rsrc_t r, int voff) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, 0, 0));
}

// one element of the sequential scan (K/asw_wta.cl:43-46 order)
__device__ __forceinline__ void scan_step(float t, int d, float &cur, float &last, int &md) {
    last = t < last ? t : last;
    md = t < cur ? d : md;
    last = t < cur ? cur : last;
    cur = t < cur ? t : cur;
}

// K/asw_wta_ref.cl:28: 0.085f * den * fabs(val - i) + cost, left to right, uncontracted
__device__ __forceinline__ float penalty(float a, float val, int i, float c) {
    const float b = fabsf(val - (float)i);
    return a * b + c;
}

// MODE 0: asw_WTA — scanned value = cost; outputs d_ref, conf_ref, d_tar, conf_tar, codes.
// MODE 1: asw_WTA_REF — scanned value = penalty + cost with the refinement
//   estimates ref_l / ref_r ([2][S]: value plane, den plane); outputs d_ref,
//   d_tar, codes, and conf_ref <- the TARGET confidence (the kernel's second,
//   overwriting store to `confidence`, K/asw_wta_ref.cl:64-66); conf_tar untouched.
// Own scan of the wave's 64 pixels over `nplanes` planes of a pixel-major volume
// (pitch Dp): the scanned index and the penalty's i are dbase + k.
template <bool PEN>
__device__ __forceinline__ void own_scan(float *tile, const float *__restrict__ cost, long long p0, long long S, int Dp,
                                         int nplanes, int dbase, int lane, float a, float val, float &cur, float &last,
                                         int &md) {
    using f4 = float __attribute__((ext_vector_type(4)));
    // chunk loader: instruction j (0..7) of lane l covers pixel j*8 + l/8, planes (l%8)*4..+3
    const int sub = lane & 7, prow = lane >> 3;
    const float *src[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const long long pp = min(p0 + j * 8 + prow, S - 1);
        src[j] = cost + pp * Dp + sub * 4;
    }
    f4 buf[8];
    const int nchunk = (nplanes + kChunk - 1) / kChunk;
#pragma unroll
    for (int j = 0; j < 8; ++j) buf[j] = *reinterpret_cast<const f4 *>(src[j]);
    for (int c = 0; c < nchunk; ++c) {
        // transpose the chunk into the wave's tile (row = pixel)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float *row = tile + (j * 8 + prow) * kTilePitch + sub * 4;
            row[0] = buf[j].x;
            row[1] = buf[j].y;
            row[2] = buf[j].z;
            row[3] = buf[j].w;
        }
        if (c + 1 < nchunk) {
#pragma unroll
            for (int j = 0; j < 8; ++j) buf[j] = *reinterpret_cast<const f4 *>(src[j] + (c + 1) * kChunk);
        }
        __builtin_amdgcn_wave_barrier();
        const float *mine = tile + lane * kTilePitch;
        const int d0 = c * kChunk;
        if (d0 + kChunk <= nplanes) {
#pragma unroll
            for (int k = 0; k < kChunk; ++k) {
                float t = mine[k];
                if constexpr (PEN) t = penalty(a, val, dbase + d0 + k, t);
                scan_step(t, dbase + d0 + k, cur, last, md);
            }
        } else {
            for (int k = 0; k < nplanes - d0; ++k) {
                float t = mine[k];
                if constexpr (PEN) t = penalty(a, val, dbase + d0 + k, t);
                scan_step(t, dbase + d0 + k, cur, last, md);
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

__device__ __forceinline__ int wave_min(int v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = min(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = max(v, __shfl_xor(v, o));
    return v;
}

// Target scan (K/asw_wta.cl:50-67, K/asw_wta_ref.cl:39-57) of pixel pc (x) with
// left disparity md: for i = 0..md-1, xq = max(0, x-i), b = md + xq - x, value
// C[b][y][xq].  Only b in [b_lo, b_lo + nloc) (this volume's planes; local plane
// b - b_lo) is visited: b = md - min(i, x) is non-increasing in i, so that is one
// interval [i_lo, i_hi) of i.
//   The lanes are skewed: at wave step j lane l is at i = j - (63 - l), so when
// the wave's 64 pixels are consecutive in one row every lane reads the SAME pixel
// xq = x0 + 63 - j, at planes md_l - i_l that a smooth disparity keeps within a
// few cache lines (an unskewed gather touches 64 distinct lines per load and is
// bound by the L1 tag rate).  Each lane still scans its own i in ascending order,
// so ties and the multiset second minimum are the sequential loop's.
//   Buffer addressing from the start of the wave's first row (wave-uniform base):
// the element of step i <= x is pixel x-i at plane md-i, one (Dp+1)-float stride
// per step, so its byte offset is A - (j+k)*stride with A per lane and
// (j+k)*stride uniform; past x it clamps to (0, md-x), the max() below.  A lane
// outside its interval reads a masked value (out-of-range offsets return 0
// through the buffer range check).  ibest = the first argmin's i, -1 if none.
template <bool PEN>
__device__ __forceinline__ void target_scan_skewed(const float *__restrict__ cost, long long p0, long long pc,
                                                   long long S, int W, int Dp, int md, int b_lo, int nloc, int lane,
                                                   float at, float valt, float &cur_t, float &last_t, int &ibest) {
    const int x = (int)(pc % W);
    const int b_hi = b_lo + nloc;
    int i_lo = max(0, md - b_hi + 1), i_hi = x <= md - b_lo ? md : min(md, md - b_lo + 1);
    if (x <= md - b_hi) i_hi = 0;  // every b(i) >= b_hi
    const int skew = 63 - lane;
    const bool any = i_lo < i_hi;
    const int jbeg = wave_min(any ? i_lo + skew : 0x7fffffff);
    const int jend = wave_max(any ? i_hi + skew : -1);
    const int ilen = any ? i_hi - i_lo : 0;
    const long long y0W = p0 / W * W;
    const long long vol_left = (S - y0W) * Dp * 4;
    const rsrc_t rsc = make_rsrc_n(cost + y0W * Dp, vol_left < 0x7fffffffLL ? (int)vol_left : 0x7fffffff);
    const int lanepix = (int)(pc - y0W);
    const int stride = (Dp + 1) * 4;
    const int A = (lanepix * Dp + md - b_lo) * 4 + skew * stride;
    const int flo = ((lanepix - x) * Dp + md - x - b_lo) * 4;
    cur_t = kSentinel;
    last_t = kSentinel;
    int mi = -1;  // the argmin's wave step j+k (i = mi - skew)
    // kGather steps' gathers are issued before any is consumed
    constexpr int kGather = 16;
    for (int j = jbeg; j < jend; j += kGather) {
        float tv[kGather];
#pragma unroll
        for (int k = 0; k < kGather; ++k) {
            // only lanes inside their interval issue the gather (exec-masked): the
            // address unit then serves fewer lanes, 0.634 -> 0.612 ms at C4
            // (profiles/r03/wta_probe_r08j.log); the others keep +inf
            const int i = j + k - skew;
            tv[k] = __builtin_inff();
            if ((unsigned)(i - i_lo) < (unsigned)ilen) tv[k] = bload(rsc, max(A - (j + k) * stride, flo));
        }
#pragma unroll
        for (int k = 0; k < kGather; ++k) {
            const int i = j + k - skew;
            float t = tv[k];
            if constexpr (PEN) t = penalty(at, valt, i, t);
            // a value >= the sentinel never changes the scan state: +inf masks
            t = (unsigned)(i - i_lo) < (unsigned)ilen ? t : __builtin_inff();
            scan_step(t, j + k, cur_t, last_t, mi);
        }
    }
    ibest = mi < 0 ? -1 : mi - skew;
}

template <int MODE>
__global__ __launch_bounds__(256) void k_wta_scan(const float *__restrict__ cost, int W, int H, int Dp, int D,
                                                  const float *__restrict__ ref_l, const float *__restrict__ ref_r,
                                                  int32_t *__restrict__ d_ref, float *__restrict__ conf_ref,
                                                  int32_t *__restrict__ d_tar, float *__restrict__ conf_tar,
                                                  uint8_t *__restrict__ code_ref, uint8_t *__restrict__ code_tar,
                                                  int nwaves, int per_xcd) {
    __shared__ float tile_all[4][64 * kTilePitch];
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    // XCD-aware: blocks b, b+8, b+16, ... run on one XCD; give each XCD a
    // contiguous range of per_xcd blocks (4 waves each) so its target gathers hit
    // rows its L2 just streamed
    const int wave_id = ((blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3)) * 4 + wv;
    if (wave_id >= nwaves) return;
    const long long S = (long long)W * H;
    const long long p0 = (long long)wave_id * 64;
    const long long p = p0 + lane;
    const bool live = p < S;
    const long long pc = live ? p : S - 1;

    float a = 0.0f, val = 0.0f;
    if constexpr (MODE == 1) {
        a = 0.085f * ref_l[S + pc];
        val = ref_l[pc];
    }
    float cur = kSentinel, last = kSentinel;
    int md = 0;
    own_scan<MODE == 1>(tile_all[wv], cost, p0, S, Dp, D, 0, lane, a, val, cur, last, md);

    float at = 0.0f, valt = 0.0f;
    if constexpr (MODE == 1) {
        at = 0.085f * ref_r[S + pc];
        valt = ref_r[pc];
    }
    float cur_t, last_t;
    int ib;
    target_scan_skewed<MODE == 1>(cost, p0, pc, S, W, Dp, live ? md : 0, 0, D, lane, at, valt, cur_t, last_t, ib);
    const int x = (int)(pc % W);
    const int mdr = ib < 0 ? md : md - min(ib, x);  // b = md + max(0, x-i) - x
    if (!live) return;
    d_ref[p] = md;
    d_tar[p] = mdr;
    if constexpr (MODE == 0) {
        conf_ref[p] = (last - cur) / last;
        conf_tar[p] = (last_t - cur_t) / last_t;
    } else {
        conf_ref[p] = (last_t - cur_t) / last_t;
    }
    if (code_ref) code_ref[p] = (uint8_t)code_u8(md, D);
    if (code_tar) code_tar[p] = (uint8_t)code_u8(mdr, D);
}

__device__ __forceinline__ long long scan_key(float v, int idx) {
    return (long long)(((unsigned long long)__float_as_uint(v) << 32) | (unsigned)idx);
}
constexpr long long kNoKeyScan = 0x7fffffffffffffffLL;

// d-sharded WTA, lane per pixel: the local halves of asw_wta_local /
// asw_wta_ref_local (own scan of planes [d_begin, d_begin + nloc): key =
// (m1 bits << 32 | first argmin), m1, m2) ...
template <bool PEN>
__global__ __launch_bounds__(256) void k_wta_local_scan(const float *__restrict__ cost, int W, int H, int Dp,
                                                        int d_begin, int nloc, const float *__restrict__ ref,
                                                        long long *__restrict__ key, float *__restrict__ m1,
                                                        float *__restrict__ m2, int nwaves, int per_xcd) {
    __shared__ float tile_all[4][64 * kTilePitch];
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int wave_id = ((blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3)) * 4 + wv;
    if (wave_id >= nwaves) return;
    const long long S = (long long)W * H;
    const long long p0 = (long long)wave_id * 64;
    const long long p = p0 + lane;
    const long long pc = p < S ? p : S - 1;
    float a = 0.0f, val = 0.0f;
    if constexpr (PEN) {
        a = 0.085f * ref[S + pc];
        val = ref[pc];
    }
    float cur = kSentinel, last = kSentinel;
    int md = -1;
    own_scan<PEN>(tile_all[wv], cost, p0, S, Dp, nloc, d_begin, lane, a, val, cur, last, md);
    if (p >= S) return;
    key[p] = md < 0 ? kNoKeyScan : scan_key(cur, md);
    m1[p] = cur;
    m2[p] = last;
}

// ... and of asw_wta_target_local / asw_wta_ref_target_local (the target scan
// restricted to the local planes, md from the global key; tkey = (t1 bits << 32 | i)).
template <bool PEN>
__global__ __launch_bounds__(256) void k_wta_target_local_scan(const float *__restrict__ cost, int W, int H, int Dp,
                                                               int d_begin, int nloc,
                                                               const long long *__restrict__ key_ref,
                                                               const float *__restrict__ ref,
                                                               long long *__restrict__ tkey, float *__restrict__ t1,
                                                               float *__restrict__ t2, int nwaves, int per_xcd) {
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int wave_id = ((blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3)) * 4 + wv;
    if (wave_id >= nwaves) return;
    const long long S = (long long)W * H;
    const long long p0 = (long long)wave_id * 64;
    const long long p = p0 + lane;
    const bool live = p < S;
    const long long pc = live ? p : S - 1;
    const long long kr = key_ref[pc];
    const int md = (!live || kr == kNoKeyScan) ? 0 : (int)(unsigned)(kr & 0xffffffffLL);
    float at = 0.0f, valt = 0.0f;
    if constexpr (PEN) {
        at = 0.085f * ref[S + pc];
        valt = ref[pc];
    }
    float cur_t, last_t;
    int ib;
    target_scan_skewed<PEN>(cost, p0, pc, S, W, Dp, md, d_begin, nloc, lane, at, valt, cur_t, last_t, ib);
    if (!live) return;
    tkey[p] = ib < 0 ? kNoKeyScan : scan_key(cur_t, ib);
    t1[p] = cur_t;
    t2[p] = last_t;
}

// asw_ref_v (K/asw_refinement_v.cl:13-51): per pixel, over the Tr vertical taps
// q = (x, clamp(y+i-Rr)): w = exp(-SAD/10.94 - |dy|/118.78) (LUT), D = (code/255)*(ndisp-1),
// F = conf[q]; t = w*F; num += t*D; den += t  (num = den = 1e-5 on entry).
// out = [num/den plane][den plane].  est is a u8 code image read with a stride
// (4: channel 0 of an RGBA8 image, as read_imagef(...).x does; 1: plain codes).
__global__ __launch_bounds__(256) void k_ref_v(const uchar4 *__restrict__ img, const uint8_t *__restrict__ est,
                                               int est_stride, const float *__restrict__ conf,
                                               const float *__restrict__ lut, int W, int H, int Tr, float scale,
                                               float *__restrict__ out) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (x >= W) return;
    const int Rr = Tr / 2;
    const long long S = (long long)W * H;
    const uchar4 pc = img[(long long)y * W + x];
    float num = 0.00001f, den = 0.00001f;
    // unrolled: the gathers of 8 taps are issued before their (in-order) sums
#pragma unroll 8
    for (int i = 0; i < Tr; ++i) {
        const int qy = clampi(y + i - Rr, 0, H - 1);
        const long long q = (long long)qy * W + x;
        const uchar4 qc = img[q];
        const int sad = abs((int)pc.x - qc.x) + abs((int)pc.y - qc.y) + abs((int)pc.z - qc.z);
        const int dist = y > qy ? y - qy : qy - y;
        const float w = lut[dist * kLutWidth + sad];
        const float Dv = ((float)est[q * est_stride] / 255.0f) * scale;
        const float t = w * conf[q];
        num = num + t * Dv;
        den = den + t;
    }
    out[(long long)y * W + x] = num / den;
    out[S + (long long)y * W + x] = den;
}

// asw_ref_h (K/asw_refinement_h.cl:16-53): over the Tr horizontal taps
// q = (clamp(x+i-Rr), y): t = w*F; num += (t*r)*n; den += t*n with r, n the value
// and den planes of asw_ref_v's output.
__global__ __launch_bounds__(256) void k_ref_h(const uchar4 *__restrict__ img, const float *__restrict__ conf,
                                               const float *__restrict__ in, const float *__restrict__ lut, int W,
                                               int H, int Tr, float *__restrict__ out) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (x >= W) return;
    const int Rr = Tr / 2;
    const long long S = (long long)W * H;
    const long long row = (long long)y * W;
    const uchar4 pc = img[row + x];
    float num = 0.00001f, den = 0.00001f;
#pragma unroll 8
    for (int i = 0; i < Tr; ++i) {
        const int qx = clampi(x + i - Rr, 0, W - 1);
        const long long q = row + qx;
        const uchar4 qc = img[q];
        const int sad = abs((int)pc.x - qc.x) + abs((int)pc.y - qc.y) + abs((int)pc.z - qc.z);
        const int dist = x > qx ? x - qx : qx - x;
        const float w = lut[dist * kLutWidth + sad];
        const float t = w * conf[q];
        const float tr = t * in[q];
        const float n = in[S + q];
        num = num + tr * n;
        den = den + t * n;
    }
    out[row + x] = num / den;
    out[S + row + x] = den;
}

// Median (K/median.cl:58-88): the min/max network there yields the exact median
// of the 9 clamped neighbours; here a 19-exchange sorting network on the codes.
__device__ __forceinline__ void cswap(int &a, int &b) {
    const int lo = min(a, b), hi = max(a, b);
    a = lo;
    b = hi;
}

__global__ __launch_bounds__(256) void k_median3(const uint8_t *__restrict__ in, int in_stride, int W, int H,
                                                 uchar4 *__restrict__ out) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (x >= W) return;
    int v[9];
    int n = 0;
#pragma unroll
    for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
        for (int dx = -1; dx <= 1; ++dx)
            v[n++] = in[((long long)clampi(y + dy, 0, H - 1) * W + clampi(x + dx, 0, W - 1)) * in_stride];
    // Paeth's median-of-9 exchange network
    cswap(v[1], v[2]); cswap(v[4], v[5]); cswap(v[7], v[8]);
    cswap(v[0], v[1]); cswap(v[3], v[4]); cswap(v[6], v[7]);
    cswap(v[1], v[2]); cswap(v[4], v[5]); cswap(v[7], v[8]);
    cswap(v[0], v[3]); cswap(v[5], v[8]); cswap(v[4], v[7]);
    cswap(v[3], v[6]); cswap(v[1], v[4]); cswap(v[2], v[5]);
    cswap(v[4], v[7]); cswap(v[4], v[2]); cswap(v[6], v[4]);
    cswap(v[4], v[2]);
    const unsigned char m = (unsigned char)v[4];
    out[(long long)y * W + x] = make_uchar4(m, m, m, 255);
}

inline int finish() {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_hip_error(e);
        return ASW_E_HIP;
    }
    return ASW_OK;
}

inline int d_end_of(const asw_params *p) { return p->d_end < 0 ? p->ndisp : p->d_end; }

}  // namespace

namespace {
inline void scan_grid(const asw_params *p, int &nwaves, int &per_xcd, unsigned &nblocks) {
    const long long S = (long long)p->width * p->height;
    nwaves = (int)((S + 63) / 64);
    per_xcd = ((nwaves + 3) / 4 + 7) / 8;  // blocks of 4 waves per XCD, the grid is exactly 8 x per_xcd
    nblocks = 8u * (unsigned)per_xcd;
}
}  // namespace

int launch_wta_local_scan(const asw_params *p, const float *cost, const float *ref, long long *key, float *m1,
                          float *m2, hipStream_t st) {
    int nwaves, per_xcd;
    unsigned nb;
    scan_grid(p, nwaves, per_xcd, nb);
    const int Dp = asw_disp_pitch(p), nloc = d_end_of(p) - p->d_begin;
    if (ref)
        hipLaunchKernelGGL(k_wta_local_scan<true>, dim3(nb), dim3(256), 0, st, cost, p->width, p->height, Dp,
                           p->d_begin, nloc, ref, key, m1, m2, nwaves, per_xcd);
    else
        hipLaunchKernelGGL(k_wta_local_scan<false>, dim3(nb), dim3(256), 0, st, cost, p->width, p->height, Dp,
                           p->d_begin, nloc, ref, key, m1, m2, nwaves, per_xcd);
    return finish();
}

int launch_wta_target_local_scan(const asw_params *p, const float *cost, const long long *key_ref, const float *ref,
                                 long long *tkey, float *t1, float *t2, hipStream_t st) {
    int nwaves, per_xcd;
    unsigned nb;
    scan_grid(p, nwaves, per_xcd, nb);
    const int Dp = asw_disp_pitch(p), nloc = d_end_of(p) - p->d_begin;
    if (ref)
        hipLaunchKernelGGL(k_wta_target_local_scan<true>, dim3(nb), dim3(256), 0, st, cost, p->width, p->height, Dp,
                           p->d_begin, nloc, key_ref, ref, tkey, t1, t2, nwaves, per_xcd);
    else
        hipLaunchKernelGGL(k_wta_target_local_scan<false>, dim3(nb), dim3(256), 0, st, cost, p->width, p->height, Dp,
                           p->d_begin, nloc, key_ref, ref, tkey, t1, t2, nwaves, per_xcd);
    return finish();
}

int launch_wta_scan(const asw_params *p, int mode, const float *cost, const float *ref_l, const float *ref_r,
                    int32_t *d_ref, float *conf_ref, int32_t *d_tar, float *conf_tar, uint8_t *code_ref,
                    uint8_t *code_tar, hipStream_t st) {
    const long long S = (long long)p->width * p->height;
    const int nwaves = (int)((S + 63) / 64);
    const int per_xcd = ((nwaves + 3) / 4 + 7) / 8;  // blocks of 4 waves per XCD, the grid is exactly 8 x per_xcd
    const unsigned nblocks = 8u * (unsigned)per_xcd;
    const int Dp = asw_disp_pitch(p);
    if (mode == 0)
        hipLaunchKernelGGL(k_wta_scan<0>, dim3(nblocks), dim3(256), 0, st, cost, p->width, p->height, Dp, p->ndisp,
                           ref_l, ref_r, d_ref, conf_ref, d_tar, conf_tar, code_ref, code_tar, nwaves, per_xcd);
    else
        hipLaunchKernelGGL(k_wta_scan<1>, dim3(nblocks), dim3(256), 0, st, cost, p->width, p->height, Dp, p->ndisp,
                           ref_l, ref_r, d_ref, conf_ref, d_tar, conf_tar, code_ref, code_tar, nwaves, per_xcd);
    return finish();
}

}  // namespace asw

using namespace asw;

extern "C" {

void asw_refine_params_default(asw_refine_params *rp) {
    if (!rp) return;
    rp->iters = 6;         // main.cpp:178 (k)
    rp->taps = 33;         // K/asw_refinement_v.cl:33 (i < 33, y + i - 16)
    rp->gamma_c = 10.94f;  // K/asw_refinement_v.cl:6
    rp->gamma_g = 118.78f; // K/asw_refinement_v.cl:7
    rp->alpha = 0.085f;    // K/asw_wta_ref.cl:28 (only the reference value is built)
}

int asw_refine_params_check(const asw_params *p, const asw_refine_params *rp) {
    const int s = asw_params_check(p);
    if (s != ASW_OK) return s;
    if (!rp || rp->iters < 0 || rp->taps < 1 || (rp->taps & 1) == 0) return ASW_E_INVALID;
    if (!(rp->gamma_c > 0.0f) || !(rp->gamma_g > 0.0f)) return ASW_E_INVALID;
    if (rp->alpha != 0.085f) return ASW_E_UNSUPPORTED;
    // the loop re-reads disparities through the reference's 8-bit codes
    if (p->ndisp > 256 || p->lr_mode != ASW_LR_U8) return ASW_E_UNSUPPORTED;
    if (p->d_begin != 0 || d_end_of(p) != p->ndisp) return ASW_E_UNSUPPORTED;  // whole volume on one device
    return ASW_OK;
}

size_t asw_refine_lut_bytes(const asw_refine_params *rp) {
    return rp ? (size_t)(rp->taps / 2 + 1) * kLutWidth * sizeof(float) : 0;
}

int asw_refine_lut(const asw_params *p, const asw_refine_params *rp, float *lut, void *stream) {
    const int s = asw_refine_params_check(p, rp);
    if (s != ASW_OK) return s;
    asw_params q = *p;  // same table kernel, refinement falloffs and window
    q.taps = rp->taps;
    q.gamma_c = rp->gamma_c;
    q.gamma_g = rp->gamma_g;
    return asw_support_lut(&q, lut, stream);
}

int asw_wta_ref(const asw_params *p, const float *cost, const float *ref_l, const float *ref_r, int32_t *d_ref,
                int32_t *d_tar, float *conf_ref, uint8_t *code_ref, uint8_t *code_tar, void *stream) {
    const int s = asw_params_check(p);
    if (s != ASW_OK) return s;
    if (p->d_begin != 0 || d_end_of(p) != p->ndisp) return ASW_E_INVALID;
    if (!cost || !ref_l || !ref_r || !d_ref || !d_tar || !conf_ref) return ASW_E_INVALID;
    return launch_wta_scan(p, 1, cost, ref_l, ref_r, d_ref, conf_ref, d_tar, nullptr, code_ref, code_tar,
                           (hipStream_t)stream);
}

int asw_ref_v(const asw_params *p, const asw_refine_params *rp, const uint8_t *img_rgba, const uint8_t *est,
              int est_stride, const float *conf, const float *lut, float *out, void *stream) {
    const int s = asw_refine_params_check(p, rp);
    if (s != ASW_OK) return s;
    if (!img_rgba || !est || !conf || !lut || !out || (est_stride != 1 && est_stride != 4)) return ASW_E_INVALID;
    const dim3 grid((unsigned)((p->width + 255) / 256), (unsigned)p->height);
    hipLaunchKernelGGL(k_ref_v, grid, dim3(256), 0, (hipStream_t)stream, reinterpret_cast<const uchar4 *>(img_rgba),
                       est, est_stride, conf, lut, p->width, p->height, rp->taps, (float)(p->ndisp - 1), out);
    return finish();
}

int asw_ref_h(const asw_params *p, const asw_refine_params *rp, const uint8_t *img_rgba, const float *conf,
              const float *in, const float *lut, float *out, void *stream) {
    const int s = asw_refine_params_check(p, rp);
    if (s != ASW_OK) return s;
    if (!img_rgba || !conf || !in || !lut || !out || in == out) return ASW_E_INVALID;
    const dim3 grid((unsigned)((p->width + 255) / 256), (unsigned)p->height);
    hipLaunchKernelGGL(k_ref_h, grid, dim3(256), 0, (hipStream_t)stream, reinterpret_cast<const uchar4 *>(img_rgba),
                       conf, in, lut, p->width, p->height, rp->taps, out);
    return finish();
}

int asw_median3(const asw_params *p, const uint8_t *codes, int stride, uint8_t *out_rgba, void *stream) {
    const int s = asw_params_check(p);
    if (s != ASW_OK) return s;
    if (!codes || !out_rgba || (stride != 1 && stride != 4)) return ASW_E_INVALID;
    const dim3 grid((unsigned)((p->width + 255) / 256), (unsigned)p->height);
    hipLaunchKernelGGL(k_median3, grid, dim3(256), 0, (hipStream_t)stream, codes, stride, p->width, p->height,
                       reinterpret_cast<uchar4 *>(out_rgba));
    return finish();
}

size_t asw_refine_workspace_bytes(const asw_params *p, const asw_refine_params *rp) {
    if (asw_refine_params_check(p, rp) != ASW_OK) return 0;
    const size_t S = (size_t)p->width * p->height;
    const size_t lut = (asw_refine_lut_bytes(rp) + 255) / 256 * 256;
    // lut, 4 x [2][S] f32 (V/H estimates of both views), 2 x S int32, 2 x S u8 codes
    return lut + 4 * 2 * S * 4 + 2 * S * 4 + 2 * S + 256;
}

int asw_refine(const asw_params *p, const asw_refine_params *rp, const uint8_t *left_rgba, const uint8_t *right_rgba,
               const float *cost, uint8_t *est_left_rgba, uint8_t *code_tar, float *conf_ref, float *conf_tar,
               void *workspace, uint8_t *post_red_rgba, uint8_t *final_rgba, int32_t *d_ref, int32_t *d_tar,
               void *stream) {
    int s = asw_refine_params_check(p, rp);
    if (s != ASW_OK) return s;
    if (!left_rgba || !right_rgba || !cost || !est_left_rgba || !code_tar || !conf_ref || !conf_tar || !workspace)
        return ASW_E_INVALID;
    const size_t S = (size_t)p->width * p->height;
    char *ws = static_cast<char *>(workspace);
    float *lut = reinterpret_cast<float *>(ws);
    ws += (asw_refine_lut_bytes(rp) + 255) / 256 * 256;
    float *vl = reinterpret_cast<float *>(ws), *vr = vl + 2 * S, *hl = vr + 2 * S, *hr = hl + 2 * S;
    int32_t *dr = reinterpret_cast<int32_t *>(hr + 2 * S), *dt = dr + S;
    uint8_t *kl = reinterpret_cast<uint8_t *>(dt + S);
    hipStream_t st = (hipStream_t)stream;
    if ((s = asw_refine_lut(p, rp, lut, st)) != ASW_OK) return s;
    // main.cpp:541-612: the left estimate is channel 0 of consistency_error (RGBA),
    // the right one the code image of the current target map
    for (int it = 0; it < rp->iters; ++it) {
        if ((s = asw_ref_v(p, rp, left_rgba, est_left_rgba, 4, conf_ref, lut, vl, st)) != ASW_OK) return s;
        if ((s = asw_ref_v(p, rp, right_rgba, code_tar, 1, conf_tar, lut, vr, st)) != ASW_OK) return s;
        if ((s = asw_ref_h(p, rp, left_rgba, conf_ref, vl, lut, hl, st)) != ASW_OK) return s;
        if ((s = asw_ref_h(p, rp, right_rgba, conf_tar, vr, lut, hr, st)) != ASW_OK) return s;
        if ((s = asw_wta_ref(p, cost, hl, hr, dr, dt, conf_ref, kl, code_tar, st)) != ASW_OK) return s;
        if ((s = asw_consistency(p, dr, dt, kl, code_tar, conf_ref, conf_tar, est_left_rgba, post_red_rgba, st)) !=
            ASW_OK)
            return s;
    }
    if (final_rgba && (s = asw_median3(p, est_left_rgba, 4, final_rgba, st)) != ASW_OK) return s;
    if (d_ref && rp->iters > 0 && hipMemcpyAsync(d_ref, dr, S * 4, hipMemcpyDeviceToDevice, st) != hipSuccess)
        return ASW_E_HIP;
    if (d_tar && rp->iters > 0 && hipMemcpyAsync(d_tar, dt, S * 4, hipMemcpyDeviceToDevice, st) != hipSuccess)
        return ASW_E_HIP;
    return ASW_OK;
}

}  // extern "C"
