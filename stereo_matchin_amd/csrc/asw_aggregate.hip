// asw_aggregate.hip — dispatch of the aggregation passes over the compiled tap
// counts and den modes; the kernels are in asw_aggregate_impl.h, instantiated one
// (tap count, den mode) per translation unit (build/agg_t<T>_d<DM>.hip, generated
// by the Makefile) so they compile in parallel.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <mutex>

#include "asw_common.h"

namespace asw {
namespace agg {
int g_pass_variant = 0;
template <int T, int DM>
int launch_pass_tm(const asw_params *p, int dir, const float *wl, const float *wr, const float *cin, float *cout,
                   float *den, hipStream_t st, const RawSrc *raw);
template <int T, int DM>
int launch_pass32_tm(const asw_params *p, int dir, const float *wl, const float *wr, const float *cin, float *cout,
                     float *den, hipStream_t st);
template <int T, int DM>
int launch_pass32_c16_tm(const asw_params *p, const float *wl, const float *wr, const uint16_t *cin16, float *cout,
                         float *den, hipStream_t st);
// a shard of <= 32 planes (pitch 32): the half-wave passes of asw_pass32.h
template <int T>
int launch_pass32_t(const asw_params *p, int dir, const float *wl, const float *wr, const float *cin, float *cout,
                    float *den, int dm, hipStream_t st) {
    if (dm == 1) return launch_pass32_tm<T, 1>(p, dir, wl, wr, cin, cout, den, st);
    if (dm == 2) return launch_pass32_tm<T, 2>(p, dir, wl, wr, cin, cout, den, st);
    return launch_pass32_tm<T, 0>(p, dir, wl, wr, cin, cout, den, st);
}
template <int T>
int launch_pass_t(const asw_params *p, int dir, const float *wl, const float *wr, const float *cin, float *cout,
                  float *den, int dm, hipStream_t st, const RawSrc *raw) {
    if (asw_disp_pitch(p) == 32) {
        if (raw && dir == ASW_DIR_V) {  // the first V pass over the uint16 raw costs
            if (dm == 1) return launch_pass32_c16_tm<T, 1>(p, wl, wr, raw->cost16, cout, den, st);
            if (dm == 0) return launch_pass32_c16_tm<T, 0>(p, wl, wr, raw->cost16, cout, den, st);
            return ASW_E_INVALID;
        }
        return launch_pass32_t<T>(p, dir, wl, wr, cin, cout, den, dm, st);
    }
    if (dm == 1) return launch_pass_tm<T, 1>(p, dir, wl, wr, cin, cout, den, st, raw);
    if (dm == 2) return launch_pass_tm<T, 2>(p, dir, wl, wr, cin, cout, den, st, raw);
    return launch_pass_tm<T, 0>(p, dir, wl, wr, cin, cout, den, st, raw);
}
}  // namespace agg

// any other odd tap count (asw_aggregate_any.hip)
int launch_pass_any(const asw_params *p, int dir, const float *wl, const float *wr, const float *cin, float *cout,
                    float *den, int dm, hipStream_t st);

int set_pass_variant(int v) {
    const int old = agg::g_pass_variant;
    agg::g_pass_variant = v;
    return old;
}

namespace {
std::mutex g_note_mu;
char g_note[2][3][96];  // [dir][den mode]
}  // namespace

void note_pass_kernel(int dir, int dm, const char *kernel, int T, const char *shape, bool nt) {
    if (dir < 0 || dir > 1 || dm < 0 || dm > 2) return;
    std::lock_guard<std::mutex> lk(g_note_mu);
    std::snprintf(g_note[dir][dm], sizeof g_note[dir][dm], "%s<T=%d,%s,DM=%d%s>", kernel, T, shape, dm,
                  nt ? ",nt" : "");
}

int pass_shape_check(const asw_params *p) {
    const long long rowbytes = (long long)p->width * asw_disp_pitch(p) * 4;
    if (rowbytes * (2LL * p->taps + 16) >= (1LL << 31)) return ASW_E_UNSUPPORTED;
    if ((long long)asw_support_bytes(p) >= (1LL << 31)) return ASW_E_UNSUPPORTED;
    return ASW_OK;
}

bool ring_taps(int T) {
#ifdef ASW_DEV_TAPS
    return T == ASW_DEV_TAPS;
#else
    return T == 3 || T == 5 || T == 7 || T == 9 || T == 15 || T == 33 || T == 35 || T == 51;
#endif
}

int launch_pass(const asw_params *p, int dir, const float *wl, const float *wr, const float *cin, float *cout,
                float *den, int dm, hipStream_t st, const RawSrc *raw) {
    if (dm != 0 && !den) return ASW_E_INVALID;
    if (const int s = pass_shape_check(p)) return s;
    if (raw && (dir != ASW_DIR_V || dm == 2 || !ring_taps(p->taps))) return ASW_E_UNSUPPORTED;
#ifdef ASW_DEV_TAPS  // development build (make DEV=1): one ring-kernel tap count only
    if (p->taps == ASW_DEV_TAPS) return agg::launch_pass_t<ASW_DEV_TAPS>(p, dir, wl, wr, cin, cout, den, dm, st, raw);
    if (raw) return ASW_E_UNSUPPORTED;
    return launch_pass_any(p, dir, wl, wr, cin, cout, den, dm, st);
#endif
    switch (p->taps) {
#define ASW_CASE(TT) \
    case TT:         \
        return agg::launch_pass_t<TT>(p, dir, wl, wr, cin, cout, den, dm, st, raw);
        ASW_CASE(3)
        ASW_CASE(5)
        ASW_CASE(7)
        ASW_CASE(9)
        ASW_CASE(15)
        ASW_CASE(33)
        ASW_CASE(35)
        ASW_CASE(51)
#undef ASW_CASE
        default:  // no ring kernel for this T: the generic pass (the uint16 first pass: ring kernels only)
            if (raw) return ASW_E_UNSUPPORTED;
            return launch_pass_any(p, dir, wl, wr, cin, cout, den, dm, st);
    }
}

int h11_seg_len(int T, int variant) {
    int U9 = T + 3;  // pf9_period
    while (U9 % 4) ++U9;
    return ((variant >> 8) & 15 ? (variant >> 8) & 15 : (240 + U9 / 2) / U9) * U9;
}

bool h11_selected(const asw_params *p, int variant) {
    const int seg = h11_seg_len(p->taps, variant);
    const long long waves11 = (long long)p->height * ((p->width + seg - 1) / seg) * (asw_disp_pitch(p) / 64);
    return !(variant & 128) && (waves11 >= 8192 || (variant & 4096));  // bit 4096: k_hpass11 at any size
}

}  // namespace asw

extern "C" int asw_pass_kernel(int dir, int den_mode, char *buf, int len) {
    if (dir < 0 || dir > 1 || den_mode < 0 || den_mode > 2 || !buf || len < 1) return ASW_E_INVALID;
    std::lock_guard<std::mutex> lk(asw::g_note_mu);
    const char *n = asw::g_note[dir][den_mode];
    if (!n[0]) return ASW_E_INVALID;
    std::snprintf(buf, (size_t)len, "%s", n);
    return ASW_OK;
}
