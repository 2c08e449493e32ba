// Shared host/device definitions of the ASW matcher (layout pitches, error state).
#pragma once
#include <hip/hip_runtime.h>

#include "asw.h"

namespace asw {

constexpr int kWave = 64;
constexpr int kSadMax = 765;        // 3 * 255: largest RGB SAD
constexpr int kLutWidth = kSadMax + 1;

// Tp: smallest multiple of 4 >= T whose quotient by 4 is odd.  A wave's lanes
// read the support slab at a stride of Tp floats; an odd number of 16-byte
// slots per row keeps ds_read_b128 conflict-free.
__host__ __device__ constexpr int tap_pitch(int T) {
    int k = (T + 3) / 4;
    if ((k & 1) == 0) ++k;
    return 4 * k;
}

__host__ __device__ constexpr int round_up(int v, int m) { return (v + m - 1) / m * m; }

// 8-bit code of disparity index d for D levels: round-half-down of 255*d/(D-1),
// the convention of the reference's write_imagef (K/asw_wta.cl:70-74).
__host__ __device__ inline int code_u8(int d, int D) {
    if (D <= 1) return 0;
    long long c = (510LL * d + (D - 2)) / (2LL * (D - 1));
    return c > 255 ? 255 : (c < 0 ? 0 : (int)c);
}

void set_hip_error(hipError_t e);

// last plane + 1 of the context's disparity shard (asw_params.d_end < 0: ndisp)
__host__ __device__ inline int d_end_of_p(const asw_params *p) { return p->d_end < 0 ? p->ndisp : p->d_end; }

// the first V pass over the raw costs as uint16 (asw_raw_cost16, asw_aggregate_pass_den16)
struct RawSrc {
    const uint16_t *cost16;
};

// one aggregation pass over every local plane (asw_aggregate.hip)
// den/dm: cached-denominator mode (ASW_DEN_*; den = NULL with ASW_DEN_NONE)
int launch_pass(const asw_params *p, int dir, const float *wl, const float *wr, const float *cin, float *cout,
                float *den, int dm, hipStream_t st, const RawSrc *raw = nullptr);
// the H pass's k_hpass11 segment length (variant bits 8..11: U-step chunks, else the
// multiple of U nearest 240) and its choice against k_hpass9 (launch_dm)
int h11_seg_len(int T, int variant);
bool h11_selected(const asw_params *p, int variant);
// the tap counts with ring kernels (the uint16 first pass needs one)
bool ring_taps(int T);
int set_pass_variant(int v);
// the asw_tune_set(ASW_TUNE_PASS_VARIANT) bits launch_dm reads: 128 = H by k_hpass9,
// 4096 = H by k_hpass11 at any size, 0xF00 = k_hpass11 segment length in U-step chunks
constexpr int kPassVariantBits = 128 | 4096 | 0xF00;
// records the instantiation a pass launch of (dir, dm) runs (asw_pass_kernel)
void note_pass_kernel(int dir, int dm, const char *kernel, int T, const char *shape, bool nt);
// ASW_OK when the pass kernels can address a (shard) context of this shape: they use
// 32-bit buffer offsets of up to ~2T+16 cost rows from a per-chunk base and a support
// array from its base; ASW_E_UNSUPPORTED otherwise (checked at asw_create, before
// any allocation, and by every pass launch)
int pass_shape_check(const asw_params *p);

// lane-per-pixel WTA scan (asw_refine.hip): mode 0 = asw_WTA, 1 = asw_WTA_REF
// lane-per-pixel d-sharded WTA halves (ref = NULL: asw_WTA; else asw_WTA_REF's penalty)
int launch_wta_local_scan(const asw_params *p, const float *cost, const float *ref, long long *key, float *m1,
                          float *m2, hipStream_t st);
int launch_wta_target_local_scan(const asw_params *p, const float *cost, const long long *key_ref, const float *ref,
                                 long long *tkey, float *t1, float *t2, hipStream_t st);
int launch_wta_scan(const asw_params *p, int mode, const float *cost, const float *ref_l, const float *ref_r,
                    int32_t *d_ref, float *conf_ref, int32_t *d_tar, float *conf_tar, uint8_t *code_ref,
                    uint8_t *code_tar, hipStream_t st);

}  // namespace asw
