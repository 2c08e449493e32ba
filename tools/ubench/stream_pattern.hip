// Achievable HBM rate of the aggregation passes' ACCESS PATTERNS, with the arithmetic
// taken out: every kernel reads a cost and a den volume and writes an output volume,
// [H][W][Dp] float32 at the C4 size (1920 x 1080 x 256 = 2.12 GB each), one 256-B
// wave access per (pixel, 64-plane block), nt cache policy, 8 rows / columns of
// loads in flight per wave.  The gap between these and the real passes is what the
// weights, the taps and their latency cost; the gap between the patterns is what the
// tiling costs.
//   flat      waves stream the volume linearly (the upper bound for 2 reads + 1 write)
//   v16_kbo   V: block = 16 columns x 1 plane block, plane block OUTER in dispatch (k_vpass10)
//   v16_kbi   V: the same, plane block INNER (the 4 blocks of a column group adjacent)
//   v4x4      V: block = 4 columns x all 4 plane blocks (1 KB contiguous per column)
//   v8x2      V: block = 8 columns x 2 plane blocks
//   h4        H: block = the 4 plane blocks of one pixel row segment (k_hpass11), 240 columns
// Access width: the patterns above move 4 B per lane per
// instruction, as the passes do.  flat_w8 / flat_w16 and h_w8 / h_w16 are the same
// streams with 8- and 16-byte loads and stores per lane (float2 / float4: a wave covers
// 128 / 256 consecutive planes), flat_*_pf16 with 16 accesses in flight per wave, and
// *_def the default cache policy instead of nt: whether the 4-B access width, not the
// machine, sets the ~5.2 TB/s of the 3-stream pattern.
// Build: hipcc --offload-arch=gfx950 -O3 -o stream_pattern stream_pattern.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

constexpr int W = 1920, H = 1080, Dp = 256, NKB = Dp / 64;
constexpr int PF = 8;

__device__ __forceinline__ float ld(const float *p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void st(float *p, float v) { __builtin_nontemporal_store(v, p); }

__global__ __launch_bounds__(1024) void k_flat(const float *a, const float *b, float *o, long long n) {
    const int lane = threadIdx.x & 63;
    const long long wave = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const long long nw = ((long long)gridDim.x * blockDim.x) >> 6;
    const long long chunks = n / 64;
    for (long long c = wave; c < chunks; c += nw * PF) {
        float x[PF], y[PF];
#pragma unroll
        for (int k = 0; k < PF; ++k) {
            const long long cc = c + k * nw;
            x[k] = cc < chunks ? ld(a + cc * 64 + lane) : 0.f;
            y[k] = cc < chunks ? ld(b + cc * 64 + lane) : 0.f;
        }
#pragma unroll
        for (int k = 0; k < PF; ++k) {
            const long long cc = c + k * nw;
            if (cc < chunks) st(o + cc * 64 + lane, x[k] * y[k]);
        }
    }
}

// flat streams with VW floats per lane and access (VW = 2: float2, 4: float4), PFW
// accesses of each input in flight per wave; NT = nontemporal loads / stores
template <int VW, int PFW, bool NT>
__global__ __launch_bounds__(1024) void k_flat_w(const float *a, const float *b, float *o, long long n) {
    using v_t = float __attribute__((ext_vector_type(VW)));
    const int lane = threadIdx.x & 63;
    const long long wave = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const long long nw = ((long long)gridDim.x * blockDim.x) >> 6;
    const long long chunks = n / (64 * VW);
    const v_t *av = reinterpret_cast<const v_t *>(a), *bv = reinterpret_cast<const v_t *>(b);
    v_t *ov = reinterpret_cast<v_t *>(o);
    for (long long c = wave; c < chunks; c += nw * PFW) {
        v_t x[PFW], y[PFW];
#pragma unroll
        for (int k = 0; k < PFW; ++k) {
            const long long cc = c + k * nw;
            if (cc < chunks) {
                if constexpr (NT) {
                    x[k] = __builtin_nontemporal_load(av + cc * 64 + lane);
                    y[k] = __builtin_nontemporal_load(bv + cc * 64 + lane);
                } else {
                    x[k] = av[cc * 64 + lane];
                    y[k] = bv[cc * 64 + lane];
                }
            }
        }
#pragma unroll
        for (int k = 0; k < PFW; ++k) {
            const long long cc = c + k * nw;
            if (cc < chunks) {
                if constexpr (NT) __builtin_nontemporal_store(x[k] * y[k], ov + cc * 64 + lane);
                else ov[cc * 64 + lane] = x[k] * y[k];
            }
        }
    }
}

// Controls: the guide's "float4 copy" (1 read + 1 write, 6.29 TB/s
// measured by the guide's authors) and a read-only stream, in the same harness, so the
// 2-read + 1-write rate above is read against the harness's own copy rate.
template <int VW, int PFW, bool NT>
__global__ __launch_bounds__(256) void k_copy_w(const float *a, float *o, long long n) {
    using v_t = float __attribute__((ext_vector_type(VW)));
    const int lane = threadIdx.x & 63;
    const long long wave = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const long long nw = ((long long)gridDim.x * blockDim.x) >> 6;
    const long long chunks = n / (64 * VW);
    const v_t *av = reinterpret_cast<const v_t *>(a);
    v_t *ov = reinterpret_cast<v_t *>(o);
    for (long long c = wave; c < chunks; c += nw * PFW) {
        v_t x[PFW];
#pragma unroll
        for (int k = 0; k < PFW; ++k) {
            const long long cc = c + k * nw;
            if (cc < chunks) x[k] = NT ? __builtin_nontemporal_load(av + cc * 64 + lane) : av[cc * 64 + lane];
        }
#pragma unroll
        for (int k = 0; k < PFW; ++k) {
            const long long cc = c + k * nw;
            if (cc < chunks) {
                if constexpr (NT) __builtin_nontemporal_store(x[k], ov + cc * 64 + lane);
                else ov[cc * 64 + lane] = x[k];
            }
        }
    }
}

template <int VW, int PFW>
__global__ __launch_bounds__(256) void k_read_w(const float *a, float *o, long long n) {
    using v_t = float __attribute__((ext_vector_type(VW)));
    const int lane = threadIdx.x & 63;
    const long long wave = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const long long nw = ((long long)gridDim.x * blockDim.x) >> 6;
    const long long chunks = n / (64 * VW);
    const v_t *av = reinterpret_cast<const v_t *>(a);
    float acc = 0.0f;
    for (long long c = wave; c < chunks; c += nw * PFW) {
        v_t x[PFW];
#pragma unroll
        for (int k = 0; k < PFW; ++k) {
            const long long cc = c + k * nw;
            x[k] = cc < chunks ? av[cc * 64 + lane] : v_t{};
        }
#pragma unroll
        for (int k = 0; k < PFW; ++k) acc += x[k][0];
    }
    if (acc == -1.0f) o[0] = acc;  // never (inputs are 0): keeps the loads
}

// H pattern with VW planes per lane: a wave covers 64*VW planes of one pixel, the
// block the Dp/(64 VW) waves of one row segment
template <int VW>
__global__ __launch_bounds__(256) void k_h_w(const float *a, const float *b, float *o, int nseg, int seg,
                                             int per_xcd) {
    using v_t = float __attribute__((ext_vector_type(VW)));
    const int xcd = blockIdx.x & 7, m = blockIdx.x >> 3;
    const int g = xcd * per_xcd + m;
    if (m >= per_xcd || g >= H * nseg) return;
    const int y = g / nseg, xs = (g % nseg) * seg, xe = min(W, xs + seg);
    const int lane = threadIdx.x & 63, kb = threadIdx.x >> 6;
    const long long base = ((long long)y * W * Dp + kb * 64 * VW) / VW + lane;  // in v_t units
    const v_t *av = reinterpret_cast<const v_t *>(a), *bv = reinterpret_cast<const v_t *>(b);
    v_t *ov = reinterpret_cast<v_t *>(o);
    constexpr int XS = Dp / VW;  // v_t per column
    for (int x = xs; x < xe; x += PF) {
        v_t u[PF], v[PF];
#pragma unroll
        for (int k = 0; k < PF; ++k) {
            const long long i = base + (long long)min(x + k, W - 1) * XS;
            u[k] = __builtin_nontemporal_load(av + i);
            v[k] = __builtin_nontemporal_load(bv + i);
        }
#pragma unroll
        for (int k = 0; k < PF; ++k)
            if (x + k < xe) __builtin_nontemporal_store(u[k] * v[k], ov + base + (long long)(x + k) * XS);
    }
}

// V patterns: a wave = (column x, plane block kb), sweeping rows [y0, y1).
// NC columns x NK plane blocks per block; KBI: plane-block groups innermost in dispatch.
template <int NC, int NK, bool KBI>
__global__ __launch_bounds__(NC *NK * 64) void k_v(const float *a, const float *b, float *o, int nstrip, int rows,
                                                 int per_xcd) {
    constexpr int NKG = NKB / NK;
    const int nxb = W / NC;
    const int xcd = blockIdx.x & 7, m = blockIdx.x >> 3;
    int xg, kg, strip;
    if (KBI) {
        kg = m % NKG;
        xg = xcd * per_xcd + (m / NKG) % per_xcd;
        strip = m / NKG / per_xcd;
    } else {
        xg = xcd * per_xcd + m % per_xcd;
        kg = (m / per_xcd) % NKG;
        strip = m / per_xcd / NKG;
    }
    if (xg >= nxb || strip >= nstrip) return;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int x = xg * NC + wv % NC, kb = kg * NK + wv / NC;
    const int y0 = strip * rows, y1 = min(H, y0 + rows);
    const long long col = (long long)x * Dp + kb * 64 + lane;
    const long long rs = (long long)W * Dp;
    for (int y = y0; y < y1; y += PF) {
        float u[PF], v[PF];
#pragma unroll
        for (int k = 0; k < PF; ++k) {
            const long long i = (long long)min(y + k, H - 1) * rs + col;
            u[k] = ld(a + i);
            v[k] = ld(b + i);
        }
#pragma unroll
        for (int k = 0; k < PF; ++k)
            if (y + k < y1) st(o + (long long)(y + k) * rs + col, u[k] * v[k]);
    }
}

// H pattern: a wave = (pixel row y, plane block kb), sweeping a 240-column segment.
__global__ __launch_bounds__(256) void k_h(const float *a, const float *b, float *o, int nseg, int seg,
                                           int per_xcd) {
    const int xcd = blockIdx.x & 7, m = blockIdx.x >> 3;
    const int g = xcd * per_xcd + m;
    if (m >= per_xcd || g >= H * nseg) return;
    const int y = g / nseg, xs = (g % nseg) * seg, xe = min(W, xs + seg);
    const int lane = threadIdx.x & 63, kb = threadIdx.x >> 6;
    const long long base = (long long)y * W * Dp + kb * 64 + lane;
    for (int x = xs; x < xe; x += PF) {
        float u[PF], v[PF];
#pragma unroll
        for (int k = 0; k < PF; ++k) {
            const long long i = base + (long long)min(x + k, W - 1) * Dp;
            u[k] = ld(a + i);
            v[k] = ld(b + i);
        }
#pragma unroll
        for (int k = 0; k < PF; ++k)
            if (x + k < xe) st(o + base + (long long)(x + k) * Dp, u[k] * v[k]);
    }
}

template <int NC, int NK, bool KBI>
void launch_v(const float *a, const float *b, float *o, int nstrip) {
    const int nxb = W / NC, per_xcd = (nxb + 7) / 8;
    const int rows = (H + nstrip - 1) / nstrip;
    const int nblocks = 8 * per_xcd * (NKB / NK) * nstrip;
    hipLaunchKernelGGL((k_v<NC, NK, KBI>), dim3(nblocks), dim3(NC * NK * 64), 0, 0, a, b, o, nstrip, rows, per_xcd);
}

int main() {
    const long long n = (long long)W * H * Dp;
    float *a, *b, *o;
    if (hipMalloc(&a, n * 4) || hipMalloc(&b, n * 4) || hipMalloc(&o, n * 4)) return 1;
    hipMemset(a, 0, n * 4);
    hipMemset(b, 0, n * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const double bytes = 3.0 * n * 4;
    auto time = [&](const char *name, auto fn) {
        std::vector<float> ts;
        for (int r = 0; r < 12; ++r) {
            hipEventRecord(e0);
            fn();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (r >= 2) ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        const float med = ts[ts.size() / 2];
        std::printf("{\"pattern\": \"%s\", \"ms\": %.4f, \"TBps\": %.3f}\n", name, med, bytes / med / 1e9);
    };
    time("flat", [&] { hipLaunchKernelGGL(k_flat, dim3(4096), dim3(1024), 0, 0, a, b, o, n); });
    for (int ns : {1, 5}) {
        char nm[64];
        std::snprintf(nm, sizeof nm, "v16_kbo_s%d", ns);
        time(nm, [&] { launch_v<16, 1, false>(a, b, o, ns); });
        std::snprintf(nm, sizeof nm, "v16_kbi_s%d", ns);
        time(nm, [&] { launch_v<16, 1, true>(a, b, o, ns); });
        std::snprintf(nm, sizeof nm, "v8x2_kbi_s%d", ns);
        time(nm, [&] { launch_v<8, 2, true>(a, b, o, ns); });
        std::snprintf(nm, sizeof nm, "v4x4_s%d", ns);
        time(nm, [&] { launch_v<4, 4, true>(a, b, o, ns); });
    }
    {
        const int seg = 240, nseg = (W + seg - 1) / seg, per_xcd = (H * nseg + 7) / 8;
        time("h4_seg240", [&] { hipLaunchKernelGGL(k_h, dim3(8 * per_xcd), dim3(256), 0, 0, a, b, o, nseg, seg, per_xcd); });
        time("h_w8_seg240", [&] {
            hipLaunchKernelGGL(k_h_w<2>, dim3(8 * per_xcd), dim3(128), 0, 0, a, b, o, nseg, seg, per_xcd);
        });
        time("h_w16_seg240", [&] {
            hipLaunchKernelGGL(k_h_w<4>, dim3(8 * per_xcd), dim3(64), 0, 0, a, b, o, nseg, seg, per_xcd);
        });
    }
    time("flat_w4_pf8_def", [&] { hipLaunchKernelGGL((k_flat_w<1, 8, false>), dim3(4096), dim3(1024), 0, 0, a, b, o, n); });
    time("flat_w4_pf16", [&] { hipLaunchKernelGGL((k_flat_w<1, 16, true>), dim3(4096), dim3(1024), 0, 0, a, b, o, n); });
    time("flat_w8", [&] { hipLaunchKernelGGL((k_flat_w<2, 8, true>), dim3(4096), dim3(1024), 0, 0, a, b, o, n); });
    time("flat_w8_def", [&] { hipLaunchKernelGGL((k_flat_w<2, 8, false>), dim3(4096), dim3(1024), 0, 0, a, b, o, n); });
    time("flat_w16", [&] { hipLaunchKernelGGL((k_flat_w<4, 4, true>), dim3(4096), dim3(1024), 0, 0, a, b, o, n); });
    time("flat_w16_pf8", [&] { hipLaunchKernelGGL((k_flat_w<4, 8, true>), dim3(4096), dim3(1024), 0, 0, a, b, o, n); });
    time("flat_w16_def", [&] { hipLaunchKernelGGL((k_flat_w<4, 4, false>), dim3(4096), dim3(1024), 0, 0, a, b, o, n); });
    time("flat_w16_g1024", [&] { hipLaunchKernelGGL((k_flat_w<4, 4, true>), dim3(1024), dim3(1024), 0, 0, a, b, o, n); });
    time("flat_w16_g16k", [&] { hipLaunchKernelGGL((k_flat_w<4, 2, true>), dim3(16384), dim3(256), 0, 0, a, b, o, n); });
    // controls: bytes = 2n*4 (copy) and n*4 (read); "TBps" printed on those bytes
    auto timeb = [&](const char *name, double nbytes, auto fn) {
        std::vector<float> ts;
        for (int r = 0; r < 12; ++r) {
            hipEventRecord(e0);
            fn();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (r >= 2) ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        const float med = ts[ts.size() / 2];
        std::printf("{\"pattern\": \"%s\", \"ms\": %.4f, \"TBps\": %.3f}\n", name, med, nbytes / med / 1e9);
    };
    const double cb = 2.0 * n * 4, rb = 1.0 * n * 4;
    timeb("copy_f4_g16k_pf2_def", cb, [&] { hipLaunchKernelGGL((k_copy_w<4, 2, false>), dim3(16384), dim3(256), 0, 0, a, o, n); });
    timeb("copy_f4_g16k_pf4_def", cb, [&] { hipLaunchKernelGGL((k_copy_w<4, 4, false>), dim3(16384), dim3(256), 0, 0, a, o, n); });
    timeb("copy_f4_g16k_pf2_nt", cb, [&] { hipLaunchKernelGGL((k_copy_w<4, 2, true>), dim3(16384), dim3(256), 0, 0, a, o, n); });
    timeb("copy_f4_g4k_pf4_def", cb, [&] { hipLaunchKernelGGL((k_copy_w<4, 4, false>), dim3(4096), dim3(256), 0, 0, a, o, n); });
    timeb("copy_f4_g64k_pf1_def", cb, [&] { hipLaunchKernelGGL((k_copy_w<4, 1, false>), dim3(65536), dim3(256), 0, 0, a, o, n); });
    timeb("copy_f1_g16k_pf8_def", cb, [&] { hipLaunchKernelGGL((k_copy_w<1, 8, false>), dim3(16384), dim3(256), 0, 0, a, o, n); });
    timeb("read_f4_g16k_pf4", rb, [&] { hipLaunchKernelGGL((k_read_w<4, 4>), dim3(16384), dim3(256), 0, 0, a, o, n); });
    timeb("read_f1_g16k_pf8", rb, [&] { hipLaunchKernelGGL((k_read_w<1, 8>), dim3(16384), dim3(256), 0, 0, a, o, n); });
    return 0;
}
