// asw_aggregate_any.hip — the aggregation pass for an odd tap count that has no
// compiled ring kernel (asw_aggregate_impl.h instantiates 3, 5, 7, 9, 15, 33, 35,
// 51).  The reference takes any window size (`win`, main.cpp:178 / the kernels'
// loop bound, K/asw_vcost_aggregation.cl:33-43, K/asw_hcost_aggregation.cl:34-41),
// so every other odd T runs here.  The FP sequence is the same as the ring
// kernels': ww = wl_i * wr_i(max(x-d,0)) rounded, num = fma(ww, c_i, num),
// den = den + ww, for i = 0..T-1 in order, out = num / den correctly rounded.
// Results are therefore bit-identical to the oracle; only the speed differs.
// One wave = one pixel, lanes = planes (coalesced cost loads and stores; the
// left weights are wave-uniform, the right ones a per-lane gather of
// neighbouring support entries).  DEN_READ recomputes den: den depends only on
// the supports, so it equals the cached value bit for bit.
#include <hip/hip_runtime.h>

#include "asw_common.h"

namespace asw {
namespace {

__device__ __forceinline__ int clampi_any(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

__global__ __launch_bounds__(256) void k_pass_any(const float *__restrict__ wl, const float *__restrict__ wr,
                                                  const float *__restrict__ cin, float *__restrict__ cout,
                                                  float *__restrict__ den, int W, int H, int Dp, int d_begin, int T,
                                                  int Tp, int dir, int write_den) {
    const long long pix = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (pix >= (long long)W * H) return;
    const int lane = threadIdx.x & 63;
    const int x = (int)(pix % W), y = (int)(pix / W);
    const int R = T / 2;
    const float *wlp = wl + pix * Tp;
    for (int k = lane; k < Dp; k += 64) {
        const int d = d_begin + k;
        const int xr = x - d < 0 ? 0 : x - d;
        const float *wrp = wr + ((long long)y * W + xr) * Tp;
        float num = 1e-5f, dn = 1e-5f;
        for (int i = 0; i < T; ++i) {
            const int qx = dir == ASW_DIR_V ? x : clampi_any(x + i - R, 0, W - 1);
            const int qy = dir == ASW_DIR_V ? clampi_any(y + i - R, 0, H - 1) : y;
            const float c = cin[((long long)qy * W + qx) * Dp + k];
            const float ww = wlp[i] * wrp[i];
            num = __builtin_fmaf(ww, c, num);
            dn = dn + ww;
        }
        cout[pix * Dp + k] = __fdiv_rn(num, dn);
        if (write_den) den[pix * Dp + k] = dn;
    }
}

}  // namespace

int launch_pass_any(const asw_params *p, int dir, const float *wl, const float *wr, const float *cin, float *cout,
                    float *den, int dm, hipStream_t st) {
    const long long S = (long long)p->width * p->height;
    const unsigned nb = (unsigned)((S + 3) / 4);
    hipLaunchKernelGGL(k_pass_any, dim3(nb), dim3(256), 0, st, wl, wr, cin, cout, den, p->width, p->height,
                       asw_disp_pitch(p), p->d_begin, p->taps, asw_tap_pitch(p), dir, dm == ASW_DEN_WRITE ? 1 : 0);
    note_pass_kernel(dir, dm, "k_pass_any", p->taps, "wave/pixel", false);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_hip_error(e);
        return ASW_E_HIP;
    }
    return ASW_OK;
}

}  // namespace asw
