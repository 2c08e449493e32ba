// Experimental pass kernels behind a tiny C interface, driven by tools/exp/exp_bench.py
// on the real C4 inputs (the production library computes raw cost and supports and the
// reference pass; this library only has the instantiations under test, so it builds in
// minutes).  Not part of the product.
#include <hip/hip_runtime.h>

#include "asw_aggregate_impl.h"
#include "asw_vpass11.h"

namespace asw {
namespace agg {
int g_pass_variant = 0;
}
void note_pass_kernel(int, int, const char *, int, const char *, bool) {}
}  // namespace asw

using namespace asw::agg;

namespace {
template <int T, int NKW, int DM>
int h11(const asw_params *p, const float *wl, const float *wr, const float *cin, float *cout, float *den, int kbg0,
        int nkbg, hipStream_t st) {
    constexpr int U = pf9_period(T);
    constexpr int RING = h11_ring(T, NKW);
    const int W = p->width, H = p->height, Dp = asw::round_up(asw::d_end_of_p(p) - p->d_begin, 64);
    const int seg = (240 + U / 2) / U * U;
    const int nseg = (W + seg - 1) / seg, ngroups = H * nseg, per_xcd = (ngroups + 7) / 8;
    const int ring_off = ((p->d_begin + Dp) / RING + 1) * RING;
    hipLaunchKernelGGL((k_hpass11<T, NKW, DM, kCPStream>), dim3(8 * per_xcd * nkbg), dim3(64 * NKW), 0, st, wl, wr,
                       cin, cout, den, W, H, Dp, p->d_begin, nseg, seg, per_xcd, ngroups, ring_off, kbg0, nkbg);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
}  // namespace

extern "C" int exp_h11(int nkw, int dm, const asw_params *p, const float *wl, const float *wr, const float *cin,
                       float *cout, float *den, int kbg0, int nkbg, void *stream) {
    hipStream_t st = (hipStream_t)stream;
    if (p->taps != 35) return -4;
#define C(N, M) \
    if (nkw == N && dm == M) return h11<35, N, M>(p, wl, wr, cin, cout, den, kbg0, nkbg, st);
    C(4, 0) C(4, 2) C(2, 0) C(2, 2) C(1, 0) C(1, 2)
#undef C
    return -4;
}

extern "C" int exp_v11(int dm, int nstrip, const asw_params *p, const float *wl, const float *wr, const float *cin,
                       float *cout, float *den, void *stream) {
    hipStream_t st = (hipStream_t)stream;
    if (p->taps != 35) return -4;
    if (dm == 2) launch_v11<35, 12, DM_READ, 2, kCPStream>(p, wl, wr, cin, cout, den, st, nstrip);
    else if (dm == 0) launch_v11<35, 12, DM_NONE, 2, kCPStream>(p, wl, wr, cin, cout, den, st, nstrip);
    else return -4;
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
