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
                   float *den, hipStream_t st, const RawSrc *raw, const OtfSrc *otf);
template <int T, int DM>
int launch_pass32_tm(const asw_params *p, int dir, const float *wl, const float *wr, const float *cin, float *cout,
                     float *den, hipStream_t st);
template <int T, int DM>
int launch_pass32_c16_tm(const asw_params *p, const float *wl, const float *wr, const uint16_t *cin16, float *cout,
                         float *den, hipStream_t st);
template <int T>
int launch_pass32_otf_v_t(const asw_params *p, const uint8_t *left, const uint8_t *right, const float *lut,
                          const float *cin, float *cout, hipStream_t st);
template <int T>
int launch_pass32_idx_tm(const asw_params *p, int dir, const uint16_t *wl, const uint16_t *wr, const float *lut,
                         const float *cin, float *cout, float *den, int dm, hipStream_t st);
template <int T>
int launch_pass_wta_tm(const asw_params *p, const float *wl, const float *wr, const float *cin, float *cout,
                       const float *den, const WtaLocalOut &o, hipStream_t st);
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
                  float *den, int dm, hipStream_t st, const RawSrc *raw, const OtfSrc *otf) {
    if (asw_disp_pitch(p) == 32) {
        if (raw && raw->cost16 && dir == ASW_DIR_V) {  // the first V pass over the uint16 raw costs
            if (dm == 1) return launch_pass32_c16_tm<T, 1>(p, wl, wr, raw->cost16, cout, den, st);
            if (dm == 0) return launch_pass32_c16_tm<T, 0>(p, wl, wr, raw->cost16, cout, den, st);
            return ASW_E_INVALID;
        }
        if (raw || otf) return ASW_E_UNSUPPORTED;  // the fused raw cost and on-the-fly weights: 64-lane passes only
        return launch_pass32_t<T>(p, dir, wl, wr, cin, cout, den, dm, st);
    }
    if (dm == 1) return launch_pass_tm<T, 1>(p, dir, wl, wr, cin, cout, den, st, raw, otf);
    if (dm == 2) return launch_pass_tm<T, 2>(p, dir, wl, wr, cin, cout, den, st, raw, otf);
    return launch_pass_tm<T, 0>(p, dir, wl, wr, cin, cout, den, st, raw, otf);
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
                float *den, int dm, hipStream_t st, const RawSrc *raw, const OtfSrc *otf) {
    if (dm != 0 && !den) return ASW_E_INVALID;
    if (const int s = pass_shape_check(p)) return s;
    if (otf && (dir != ASW_DIR_H || raw || !ring_taps(p->taps))) return ASW_E_UNSUPPORTED;
    if (raw && (dir != ASW_DIR_V || (raw->cost16 && (dm == 2 || !ring_taps(p->taps))))) return ASW_E_UNSUPPORTED;
#ifdef ASW_DEV_TAPS  // development build (make DEV=1): one ring-kernel tap count only
    if (p->taps == ASW_DEV_TAPS) return agg::launch_pass_t<ASW_DEV_TAPS>(p, dir, wl, wr, cin, cout, den, dm, st, raw, otf);
    if (raw) return ASW_E_UNSUPPORTED;
    return launch_pass_any(p, dir, wl, wr, cin, cout, den, dm, st);
#endif
    switch (p->taps) {
#define ASW_CASE(TT) \
    case TT:         \
        return agg::launch_pass_t<TT>(p, dir, wl, wr, cin, cout, den, dm, st, raw, otf);
        ASW_CASE(3)
        ASW_CASE(5)
        ASW_CASE(7)
        ASW_CASE(9)
        ASW_CASE(15)
        ASW_CASE(33)
        ASW_CASE(35)
        ASW_CASE(51)
#undef ASW_CASE
        default:  // no ring kernel for this T: the generic pass (the fused raw cost is opt-in, ring kernels only)
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

// the den-read H pass with the local WTA scan fused (asw_aggregate_pass_wta_local):
// where that pass is k_hpass11 with one block over every plane (Dp = 256 or 128), at
// the ring tap counts <= 35 (4 waves per SIMD)
bool pass_wta_local_supported(const asw_params *p) {
    const int Dp = asw_disp_pitch(p);
    return ring_taps(p->taps) && p->taps <= 35 && (Dp == 256 || Dp == 128) &&
           h11_selected(p, agg::g_pass_variant);
}

int launch_pass_wta_local(const asw_params *p, const float *wl, const float *wr, const float *cin, float *cout,
                          const float *den, const WtaLocalOut &o, hipStream_t st) {
    if (const int s = pass_shape_check(p)) return s;
    if (!pass_wta_local_supported(p)) return ASW_E_UNSUPPORTED;
#ifdef ASW_DEV_TAPS
    if (p->taps == ASW_DEV_TAPS) return agg::launch_pass_wta_tm<ASW_DEV_TAPS>(p, wl, wr, cin, cout, den, o, st);
    return ASW_E_UNSUPPORTED;
#endif
    switch (p->taps) {
#define ASW_CASE(TT) \
    case TT:         \
        return agg::launch_pass_wta_tm<TT>(p, wl, wr, cin, cout, den, o, st);
        ASW_CASE(3)
        ASW_CASE(5)
        ASW_CASE(7)
        ASW_CASE(9)
        ASW_CASE(15)
        ASW_CASE(33)
        ASW_CASE(35)
#undef ASW_CASE
        default: return ASW_E_UNSUPPORTED;
    }
}

// the pass over index-form supports (asw_aggregate_pass_index): 32-plane shards, ring
// tap counts <= 35, V with den mode NONE (what the shard's frame runs), H in every mode
bool pass_index_supported(const asw_params *p, int dir, int dm) {
    const int T = p->taps;
    if (dir == ASW_DIR_V && dm != ASW_DEN_NONE) return false;
    return (dir == ASW_DIR_V || dir == ASW_DIR_H) && dm >= ASW_DEN_NONE && dm <= ASW_DEN_READ &&
           p->color_space == ASW_COLOR_RGB && asw_disp_pitch(p) == 32 && ring_taps(T) && T <= 35;
}

int launch_pass_index(const asw_params *p, int dir, const uint16_t *wl, const uint16_t *wr, const float *lut,
                      const float *cin, float *cout, float *den, int dm, hipStream_t st) {
    if (const int s = pass_shape_check(p)) return s;
    if (!pass_index_supported(p, dir, dm)) return ASW_E_UNSUPPORTED;
#ifdef ASW_DEV_TAPS
    if (p->taps == ASW_DEV_TAPS) return agg::launch_pass32_idx_tm<ASW_DEV_TAPS>(p, dir, wl, wr, lut, cin, cout, den, dm, st);
    return ASW_E_UNSUPPORTED;
#endif
    switch (p->taps) {
#define ASW_CASE(TT) \
    case TT:         \
        return agg::launch_pass32_idx_tm<TT>(p, dir, wl, wr, lut, cin, cout, den, dm, st);
        ASW_CASE(3)
        ASW_CASE(5)
        ASW_CASE(7)
        ASW_CASE(9)
        ASW_CASE(15)
        ASW_CASE(33)
        ASW_CASE(35)
#undef ASW_CASE
        default: return ASW_E_UNSUPPORTED;
    }
}

// the V pass of a 32-plane shard with both support weights on the fly
// (asw_aggregate_pass_otf_v): RGB, ring tap counts <= 35, den mode NONE
bool pass_otf_v_supported(const asw_params *p) {
    return p->color_space == ASW_COLOR_RGB && asw_disp_pitch(p) == 32 && ring_taps(p->taps) && p->taps <= 35;
}

int launch_pass_otf_v(const asw_params *p, const uint8_t *left, const uint8_t *right, const float *lut,
                      const float *cin, float *cout, hipStream_t st) {
    if (const int s = pass_shape_check(p)) return s;
    if (!pass_otf_v_supported(p)) return ASW_E_UNSUPPORTED;
#ifdef ASW_DEV_TAPS
    if (p->taps == ASW_DEV_TAPS) return agg::launch_pass32_otf_v_t<ASW_DEV_TAPS>(p, left, right, lut, cin, cout, st);
    return ASW_E_UNSUPPORTED;
#endif
    switch (p->taps) {
#define ASW_CASE(TT) \
    case TT:         \
        return agg::launch_pass32_otf_v_t<TT>(p, left, right, lut, cin, cout, st);
        ASW_CASE(3)
        ASW_CASE(5)
        ASW_CASE(7)
        ASW_CASE(9)
        ASW_CASE(15)
        ASW_CASE(33)
        ASW_CASE(35)
#undef ASW_CASE
        default: return ASW_E_UNSUPPORTED;
    }
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
