// asw_aggregate.hip — dispatch of the aggregation passes over the compiled tap
// counts and den modes; the kernels are in asw_aggregate_impl.h, instantiated one
// (tap count, den mode) per translation unit (build/agg_t<T>_d<DM>.hip, generated
// by the Makefile) so they compile in parallel.
#include <hip/hip_runtime.h>

#include "asw_common.h"

namespace asw {
namespace agg {
int g_pass_variant = 0;
template <int T, int DM>
int launch_pass_tm(const asw_params *p, int dir, const float *wl, const float *wr, const float *cin, float *cout,
                   float *den, hipStream_t st, const RawSrc *raw);
template <int T>
int launch_pass_t(const asw_params *p, int dir, const float *wl, const float *wr, const float *cin, float *cout,
                  float *den, int dm, hipStream_t st, const RawSrc *raw) {
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

int launch_pass(const asw_params *p, int dir, const float *wl, const float *wr, const float *cin, float *cout,
                float *den, int dm, hipStream_t st, const RawSrc *raw) {
    if (dm != 0 && !den) return ASW_E_INVALID;
    // the pass kernels address the cost volume with 32-bit buffer offsets of up to
    // ~2T+16 rows from a per-chunk base, and a support array from its base
    const long long rowbytes = (long long)p->width * asw_disp_pitch(p) * 4;
    if (rowbytes * (2LL * p->taps + 16) >= (1LL << 31)) return ASW_E_UNSUPPORTED;
    if ((long long)asw_support_bytes(p) >= (1LL << 31)) return ASW_E_UNSUPPORTED;
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
        default:  // no ring kernel for this T: the generic pass (the fused raw cost is opt-in, ring kernels only)
            if (raw) return ASW_E_UNSUPPORTED;
            return launch_pass_any(p, dir, wl, wr, cin, cout, den, dm, st);
    }
}

}  // namespace asw
