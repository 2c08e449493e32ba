/*
 * asw.h — C-ABI of the MI355X-native adaptive-support-weight (ASW) stereo matcher.
 *
 * Drop-in boundary for the reference's OpenCL `kernels/` path
 * (manixq/stereo_matchin, stereo_matching/main.cpp:413-537).  Every entry point
 * is `extern "C"`, takes plain pointers and sizes, returns an int status
 * (ASW_OK or a negative ASW_E_* code; never throws), and names the reference
 * interface it replaces.
 *
 * Two levels:
 *   - STAGE API: device pointers, asynchronous on the caller's HIP stream
 *     (`void* stream` is a hipStream_t; NULL = default stream).  One call per
 *     reference kernel launch, with the same argument meaning.
 *   - FRAME API: host RGBA8 pointers in, host disparity maps out, synchronous
 *     (what main.cpp:183-186 -> :621-631 does for one image pair).
 *
 * Device data layout — NOT the reference's plane-major one:
 *   images   : row-major RGBA8, [H][W][4]                         (as lodepng decodes)
 *   cost     : PIXEL-major, [H][W][Dp] float32, Dp = asw_disp_pitch(p) (64k, or 32)
 *              element (y,x,k) holds disparity d = p->d_begin + k (k < d_end-d_begin)
 *   supports : [H][W][Tp] float32, Tp = asw_tap_pitch(p); element (y,x,i) = tap i
 *   LUT      : [(R+1)][766] float32 support-weight table, R = (taps-1)/2
 *   maps     : [H][W] int32 disparity indices, float32 confidences, u8 codes
 */
#ifndef ASW_H
#define ASW_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes (main.cpp:27-30 ErCheck prints cl_int and continues; we return) ---- */
#define ASW_OK 0
#define ASW_E_INVALID -1     /* bad parameter / shape                         */
#define ASW_E_HIP -2         /* a HIP runtime call failed (asw_last_hip_error) */
#define ASW_E_NOMEM -3       /* device or host allocation failed              */
#define ASW_E_UNSUPPORTED -4 /* parameter combination not built               */
#define ASW_E_COMM -5        /* a collective (RCCL) call failed               */

#define ASW_DIR_V 0 /* vertical pass / support   (asw_vSupport, asw_vCostAggregation) */
#define ASW_DIR_H 1 /* horizontal pass / support (asw_hSupport, asw_hCostAggregation) */

#define ASW_COLOR_RGB 0 /* reference: RGB sum of absolute differences (K/asw_vsupport.cl:22) */
#define ASW_COLOR_LAB 1 /* extension (north star): CIELab Euclidean distance (asw_lab)     */

#define ASW_LR_U8 0     /* parity: compare 8-bit codes like K/consist.cl:20-30 */
#define ASW_LR_NATIVE 1 /* |d_ref - d_tar| <= 1 on integer indices (D > 256)   */

/* Parameters.  asw_params_default() fills the reference values:
 * ndisp 61 (K/asw_aggr.cl:16), taps 33 (K/asw_vcost_aggregation.cl:33), iters 7
 * (main.cpp:177), gamma_c 30.91 / gamma_g 28.21 (K/asw_vsupport.cl:22,24),
 * untruncated AD (tad_tau >= 765), LR check on with 8-bit codes. */
typedef struct asw_params {
    int width, height;   /* image size W, H                                    */
    int ndisp;           /* D: disparity levels 0..D-1                          */
    int taps;            /* T = 2R+1 taps per 1-D pass (odd)                    */
    int iters;           /* r: (V,H) pass pairs                                 */
    float gamma_c;       /* colour falloff                                       */
    float gamma_g;       /* geometric falloff                                    */
    int color_space;     /* ASW_COLOR_*                                          */
    float tad_tau;       /* truncated-AD threshold; >= 765 is plain AD           */
    int lr_check;        /* run the left-right consistency stage                */
    int lr_mode;         /* ASW_LR_*                                             */
    int d_begin, d_end;  /* disparity shard owned by this context [begin, end)  */
    int flags;           /* ASW_FLAG_*: frame-API context options (0 = the default forms) */
} asw_params;

/* asw_params.flags: context options of the frame API (asw_create*).  Every option is
 * bit-identical to the default; asw_params_check rejects unknown bits.  (Round 6 removed
 * the opt-in forms that measured slower in every shape; their bits
 * 0x1, 0x2, 0x4, 0x8, 0x10, 0x80 and 0x100 are no longer accepted.)  The stage API
 * ignores flags. */
#define ASW_FLAG_COMM_LOCAL 0x20     /* asw_create_multi: the device-local exchange even for distinct ids */
#define ASW_FLAG_RAW_F32 0x40        /* keep the float raw-cost volume (asw_raw_cost) where the uint16 one
                                        (asw_raw_cost16 + asw_aggregate_pass_den16) is the default    */
#define ASW_FLAG_ALL 0x60

void asw_params_default(asw_params *p);
int asw_params_check(const asw_params *p);
const char *asw_strerror(int status);
int asw_last_hip_error(void); /* hipError_t of the last ASW_E_HIP */
/* ABI revision of this header.  The frame API's caller-allocated structs
 * (asw_outputs, asw_timings) grow between revisions: a host must check
 * asw_abi_version() == ASW_ABI_VERSION before calling asw_match / asw_match_batch,
 * or the library writes past a struct of an older layout.
 *   1: round 1;  2: asw_outputs.disp16 / lr16, asw_timings.exchange;
 *   3: asw_params.flags (the context options that were environment variables);
 *      asw_raw_cost16 / asw_aggregate_pass_den16 (the uint16 raw-cost volume);
 *   4: the measured-negative forms removed with their entry points and flags
 *      (on-the-fly, index-form and fused-raw passes, the fused WTA scan). */
#define ASW_ABI_VERSION 4
int asw_abi_version(void);

/* layout helpers */
/* Dp = round_up(d_end-d_begin, 64); a shard (d_begin > 0 or d_end < ndisp) of at most
 * 32 planes: Dp = 32 (its passes hold two pixels per wave, 32 planes each) */
int asw_disp_pitch(const asw_params *p);
int asw_tap_pitch(const asw_params *p);  /* Tp = smallest 4k >= taps with k odd        */
size_t asw_cost_bytes(const asw_params *p);    /* H*W*Dp*4   */
size_t asw_support_bytes(const asw_params *p); /* H*W*Tp*4   */
size_t asw_lut_bytes(const asw_params *p);     /* (R+1)*766*4 */
size_t asw_lab_bytes(const asw_params *p);     /* H*W*16 (float4 per pixel) */

/* ---------------- STAGE API (device pointers, async on `stream`) ---------------- */

/* replaces asw_Aggr (K/asw_aggr.cl:3-23), launched at main.cpp:463-466:
 * cost[y][x][k] = min(tad_tau, |dR|+|dG|+|dB|) between L(x,y) and R(max(x-d,0),y),
 * d = d_begin + k; padding lanes k >= d_end-d_begin are written 0. */
int asw_raw_cost(const asw_params *p, const uint8_t *left_rgba, const uint8_t *right_rgba, float *cost,
                 void *stream);
/* The same costs as uint16 [H][W][Dp] (half the bytes): |dR|+|dG|+|dB| is an integer
 * <= 765, so min(tad_tau, AD) is one too when tad_tau >= 765 or integral; other
 * tad_tau (or tad_tau < 0): ASW_E_UNSUPPORTED.  asw_aggregate_pass_den16 reads it as the
 * first V pass (main.cpp:494-500); the float values it converts are the ones
 * asw_raw_cost writes, so every output is bit-identical.  asw_raw16_supported: 1 when
 * both are built for p (that tad_tau, a ring tap count, iters >= 1), else 0. */
int asw_raw_cost16(const asw_params *p, const uint8_t *left_rgba, const uint8_t *right_rgba, uint16_t *cost,
                   void *stream);
int asw_aggregate_pass_den16(const asw_params *p, const float *wvl, const float *wvr, const uint16_t *cin16,
                             float *cout, float *den, int den_mode, void *stream); /* V; den_mode NONE or WRITE */
int asw_raw16_supported(const asw_params *p);

/* support-weight table (the exp of K/asw_vsupport.cl:22-25 for every (|delta|, SAD)) */
int asw_support_lut(const asw_params *p, float *lut, void *stream);

/* replaces asw_vSupport / asw_hSupport (K/asw_vsupport.cl:3-27, K/asw_hsupport.cl:3-28),
 * launched at main.cpp:469-484 (once per image and direction).  RGB contexts only
 * (ASW_E_INVALID for ASW_COLOR_LAB: use asw_lab + asw_support_lab). */
int asw_support(const asw_params *p, int dir, const uint8_t *img_rgba, const float *lut, float *w,
                void *stream);

/* the four support arrays of a frame in one launch (asw_vSupport and asw_hSupport of
 * both images, main.cpp:469-484): bit-identical to four asw_support calls. */
int asw_support_all(const asw_params *p, const uint8_t *left_rgba, const uint8_t *right_rgba, const float *lut,
                    float *wvl, float *whl, float *wvr, float *whr, void *stream);

/* CIELab extension (north star; the reference has no colour conversion, so this
 * is not reference-pinned: the oracle restates the same IEEE double sequence and
 * colorimetric known answers pin the conversion).  With p->color_space ==
 * ASW_COLOR_LAB the support weights use the Euclidean L*a*b* distance in place of
 * the RGB SAD of K/asw_vsupport.cl:19-25; the raw cost stays RGB AD/TAD.
 *   asw_lab:          lab[y][x] = (L*, a*, b*, 0) float4 of an RGBA8 image (sRGB, D65)
 *   asw_support_lab:  the asw_support of a LAB context, from a lab image. */
int asw_lab(const asw_params *p, const uint8_t *img_rgba, float *lab, void *stream);
int asw_support_lab(const asw_params *p, int dir, const float *lab, float *w, void *stream);

/* replaces asw_vCostAggregation / asw_hCostAggregation (K/asw_vcost_aggregation.cl:11-44,
 * K/asw_hcost_aggregation.cl:12-44), launched at main.cpp:494-509.  One pass over
 * every local plane: cout = sum_i wl_i*wr_i(xr)*cin_i / sum_i wl_i*wr_i(xr).
 * The reference's dead `denom` output is not produced.  cin != cout. */
int asw_aggregate_pass(const asw_params *p, int dir, const float *wl, const float *wr, const float *cin,
                       float *cout, void *stream);

/* Same pass with a cached denominator volume `den` ([H][W][Dp] float32, the cost
 * layout).  The reference recomputes den = 1e-5 + sum_i wl_i*wr_i(xr) in every pass
 * (K/asw_vcost_aggregation.cl:38, written to its dead asw_denom buffer); it does
 * not depend on the cost, so ASW_DEN_WRITE stores it during a pass and
 * ASW_DEN_READ reuses it in the later passes of the same direction (same
 * supports).  Results are bit-identical in every mode. */
#define ASW_DEN_NONE 0  /* compute den, do not touch `den` (may be NULL) */
#define ASW_DEN_WRITE 1 /* compute den and store it to `den`            */
#define ASW_DEN_READ 2  /* take den from `den` (written by a DEN_WRITE pass of this direction) */
int asw_aggregate_pass_den(const asw_params *p, int dir, const float *wl, const float *wr, const float *cin,
                           float *cout, float *den, int den_mode, void *stream);

/* r x (V,H) ping-pong of main.cpp:486-515 on two caller buffers; the result
 * ends in `c0` (c0 holds the raw cost on entry, c1 is scratch). */
int asw_aggregate(const asw_params *p, const float *wvl, const float *wvr, const float *whl, const float *whr,
                  float *c0, float *c1, void *stream);
/* asw_aggregate with cached denominators: den_v, den_h are two more [H][W][Dp]
 * volumes (asw_cost_bytes each); the first iteration writes them, the other r-1
 * read them.  den_v = den_h = NULL is asw_aggregate. */
int asw_aggregate_den(const asw_params *p, const float *wvl, const float *wvr, const float *whl, const float *whr,
                      float *c0, float *c1, float *den_v, float *den_h, void *stream);

/* replaces asw_WTA (K/asw_wta.cl:12-82), launched at main.cpp:517-526, for a context
 * that owns the whole disparity range: left first-argmin + confidence, the
 * bresenham target scan, and the 8-bit codes the reference writes to its images. */
int asw_wta(const asw_params *p, const float *cost, int32_t *d_ref, float *conf_ref, int32_t *d_tar,
            float *conf_tar, uint8_t *code_ref, uint8_t *code_tar, void *stream);

/* replaces Constistency (K/consist.cl:3-34), launched at main.cpp:529-537.
 * conf_ref / conf_tar are zeroed in place where inconsistent (RMW like the
 * reference).  out_rgba / out_red_rgba are [H][W][4]; either may be NULL. */
int asw_consistency(const asw_params *p, const int32_t *d_ref, const int32_t *d_tar, const uint8_t *code_ref,
                    const uint8_t *code_tar, float *conf_ref, float *conf_tar, uint8_t *out_rgba,
                    uint8_t *out_red_rgba, void *stream);

/* ---- d-sharded WTA (no reference counterpart: the reference runs one device) ----
 * key = (float_bits(m1) << 32) | index, reduced with an elementwise MIN across
 * shards (RCCL ncclMin on int64; keys are positive).  Sequence per frame:
 *   asw_wta_local      -> allreduce_min(key)   -> asw_wta_second(ref)  -> allreduce_min(m2)
 *   asw_wta_target_local(key) -> allreduce_min(tkey) -> asw_wta_second(tar) -> allreduce_min(t2)
 *   asw_wta_finalize.
 * Exact: the result equals asw_wta on the unsharded volume bit for bit. */
int asw_wta_local(const asw_params *p, const float *cost, int64_t *key, float *m1, float *m2, void *stream);
int asw_wta_target_local(const asw_params *p, const float *cost, const int64_t *key_ref, int64_t *tkey,
                         float *t1, float *t2, void *stream);
int asw_wta_second(const asw_params *p, const int64_t *key_global, const int64_t *key_local, const float *m1,
                   const float *m2, float *m2_contrib, void *stream);
int asw_wta_finalize(const asw_params *p, const int64_t *key, const float *m2, const int64_t *tkey,
                     const float *t2, int32_t *d_ref, float *conf_ref, int32_t *d_tar, float *conf_tar,
                     uint8_t *code_ref, uint8_t *code_tar, void *stream);

/* ---- d-sharded asw_WTA_REF (K/asw_wta_ref.cl:2-68): the refinement loop's volume
 * scan over a shard, the asw_wta_local protocol on the penalised values
 * 0.085*den*|val - i| + C (ref_l / ref_r = asw_ref_h's [2][S] output of each view):
 *   asw_wta_ref_local -> allreduce_min(key)
 *   asw_wta_ref_target_local(key) -> allreduce_min(tkey) -> asw_wta_second(tar) -> allreduce_min(t2)
 *   asw_wta_ref_finalize.
 * The left second minimum is not exchanged: the reference's `confidence` receives the
 * target confidence last (K/asw_wta_ref.cl:64-66).  Equals asw_wta_ref bit for bit. */
int asw_wta_ref_local(const asw_params *p, const float *cost, const float *ref_l, int64_t *key, float *m1, float *m2,
                      void *stream);
int asw_wta_ref_target_local(const asw_params *p, const float *cost, const float *ref_r, const int64_t *key_ref,
                             int64_t *tkey, float *t1, float *t2, void *stream);
int asw_wta_ref_finalize(const asw_params *p, const int64_t *key, const int64_t *tkey, const float *t2,
                         int32_t *d_ref, int32_t *d_tar, float *conf_ref, uint8_t *code_ref, uint8_t *code_tar,
                         void *stream);

/* ---- refinement loop (main.cpp:540-623): k x (asw_ref_v, asw_ref_h on both views,
 * asw_WTA_REF, Constistency), then the 3x3 Median -> asw_disparity.png ----
 * Whole-volume contexts only (d_begin = 0, d_end = ndisp), ndisp <= 256, ASW_LR_U8:
 * the loop feeds disparities back through the reference's 8-bit codes. */
typedef struct asw_refine_params {
    int iters;      /* k refinement iterations (main.cpp:178: 6)                      */
    int taps;       /* window of asw_ref_v / asw_ref_h (K/asw_refinement_v.cl:33: 33)  */
    float gamma_c;  /* 10.94 (K/asw_refinement_v.cl:6)                                 */
    float gamma_g;  /* 118.78 (K/asw_refinement_v.cl:7)                                */
    float alpha;    /* penalty slope 0.085 (K/asw_wta_ref.cl:28); only 0.085 is built  */
} asw_refine_params;

void asw_refine_params_default(asw_refine_params *rp);
int asw_refine_params_check(const asw_params *p, const asw_refine_params *rp);
size_t asw_refine_lut_bytes(const asw_refine_params *rp);
/* weight table of the refinement kernels (asw_support_lut with the refinement falloffs) */
int asw_refine_lut(const asw_params *p, const asw_refine_params *rp, float *lut, void *stream);

/* replaces asw_ref_v (K/asw_refinement_v.cl:13-51), main.cpp:547-558.  est: u8
 * disparity codes read at `est_stride` bytes per pixel (4 = channel 0 of an RGBA8
 * image such as consistency_error, 1 = a plain code map).  out: [2][H][W] f32,
 * plane 0 = the refined disparity estimate num/den, plane 1 = den. */
int asw_ref_v(const asw_params *p, const asw_refine_params *rp, const uint8_t *img_rgba, const uint8_t *est,
              int est_stride, const float *conf, const float *lut, float *out, void *stream);
/* replaces asw_ref_h (K/asw_refinement_h.cl:16-53), main.cpp:561-573; in/out [2][H][W]. */
int asw_ref_h(const asw_params *p, const asw_refine_params *rp, const uint8_t *img_rgba, const float *conf,
              const float *in, const float *lut, float *out, void *stream);
/* replaces asw_WTA_REF (K/asw_wta_ref.cl:2-68), main.cpp:576-586: first-argmin of
 * 0.085*den*|val - d| + C[d] (left) and the same along the target diagonal.
 * As the reference: conf_ref receives the TARGET confidence (its second store to
 * `confidence`), the target confidence array is not written. */
int asw_wta_ref(const asw_params *p, const float *cost, const float *ref_l, const float *ref_r, int32_t *d_ref,
                int32_t *d_tar, float *conf_ref, uint8_t *code_ref, uint8_t *code_tar, void *stream);
/* replaces Median (K/median.cl:58-88), main.cpp:615-617: 3x3 median of u8 codes
 * (stride 1 or 4 bytes per pixel), clamped borders; out = grey RGBA8. */
int asw_median3(const asw_params *p, const uint8_t *codes, int stride, uint8_t *out_rgba, void *stream);

/* The whole loop on device buffers.  In: the final aggregated volume `cost`, the
 * pre-refinement consistency image est_left_rgba (asw_consistency's out_rgba) and
 * target codes code_tar (asw_wta's), confidences after that consistency check.
 * All four are updated in place, as the reference's buffers are.  Out (any may be
 * NULL): post_red_rgba (asw_consistency_post-reff.png, written when iters > 0),
 * final_rgba (asw_disparity.png), d_ref / d_tar of the last asw_WTA_REF.
 * workspace: asw_refine_workspace_bytes() of device memory. */
size_t asw_refine_workspace_bytes(const asw_params *p, const asw_refine_params *rp);
int asw_refine(const asw_params *p, const asw_refine_params *rp, const uint8_t *left_rgba, const uint8_t *right_rgba,
               const float *cost, uint8_t *est_left_rgba, uint8_t *code_tar, float *conf_ref, float *conf_tar,
               void *workspace, uint8_t *post_red_rgba, uint8_t *final_rgba, int32_t *d_ref, int32_t *d_tar,
               void *stream);

/* tuning hook (benchmarks / kernel experiments): selects among compiled kernel
 * variants; returns the previous value, or ASW_E_INVALID for an unknown key.
 * Every variant computes bit-identical results. */
#define ASW_TUNE_PASS_VARIANT 1
#define ASW_TUNE_WTA_VARIANT 2 /* asw_wta: 0 lane-per-pixel scan (default), 2 row sweep (Dp 64/128/256; the
                                  scan elsewhere); 1 (round 1's wave per pixel) is no longer built */
int asw_tune_set(int key, int value);
/* the kernel instantiation the most recent aggregation-pass launch of (dir, den_mode)
 * in this process ran, e.g. "k_vpass10<T=35,NW=16,DM=2,nt>" (NUL-terminated, at most
 * len bytes): lets a test assert which compiled form a shape selects.  ASW_E_INVALID
 * when no such pass has been launched yet. */
int asw_pass_kernel(int dir, int den_mode, char *buf, int len);

/* ---------------- FRAME API (host pointers, synchronous) ---------------- */

typedef struct asw_ctx asw_ctx;

typedef struct asw_outputs { /* caller-owned host arrays; any may be NULL */
    int32_t *d_ref, *d_tar;  /* [H][W] disparity indices (left, right view)     */
    float *conf_ref, *conf_tar;
    uint8_t *disp_rgba;      /* [H][W][4] 8-bit disparity image (asw_left_wta)  */
    uint8_t *lr_rgba;        /* [H][W][4] consistency output ("consistency_error") */
    uint8_t *lr_red_rgba;    /* [H][W][4] asw_consistency_pre-reff.png image    */
    float *cost;             /* [H][W][Dp] final aggregated volume (optional)   */
    uint8_t *final_rgba;     /* [H][W][4] asw_disparity.png (refinement on)     */
    uint8_t *post_red_rgba;  /* [H][W][4] asw_consistency_post-reff.png (refinement on) */
    /* 16-bit disparity images: the 8-bit codes of K/asw_wta.cl:70-74
     * collide above D = 256 (C5: D = 512); these hold the disparity index itself. */
    uint16_t *disp16;        /* [H][W] d_ref                                              */
    uint16_t *lr16;          /* [H][W] d_ref where the LR check passes, else ASW_DISP16_INVALID
                                (the asw_consistency_pre-reff image; lr_check only)        */
} asw_outputs;
#define ASW_DISP16_INVALID 0xFFFF

typedef struct asw_timings { /* milliseconds from HIP events, columns of main.cpp:181 */
    double raw_cost, support, v_pass_mean, h_pass_mean, aggregation_total, wta, consistency, total;
    double h2d, d2h;
    double refine;           /* refinement loop + median (0 when off) */
    double exchange;         /* multi-GPU contexts: the WTA exchange (4 MIN all-reduces) */
} asw_timings;

/* marketing name of a HIP device (the reference names its TSV after the OpenCL
 * device, main.cpp:164-166); writes a NUL-terminated string of at most len bytes. */
int asw_device_name(int hip_device, char *buf, int len);

/* A context owns the device buffers of one image size, sized at create and reused
 * by every asw_match (the reference re-creates its cl_mem objects per run,
 * main.cpp:243-457).  p->d_begin / d_end must cover the whole range: contexts
 * shard the disparity axis themselves.  Shapes whose volume rows or support arrays
 * exceed the pass kernels' 32-bit offsets (e.g. 7680x4320 at D = 512) are rejected
 * here with ASW_E_UNSUPPORTED, before anything is allocated.
 *
 * asw_create: one GPU (HIP device ordinal), the whole disparity range. */
int asw_create(const asw_params *p, int hip_device, asw_ctx **out);
/* One process, n_devices GPUs: [0, ndisp) is split into n_devices
 * contiguous shards, shard i on hip_device_ids[i].  Raw cost, supports and the 2r
 * passes of a shard touch only its planes (no communication); the WTA is the one
 * exchange: 4 elementwise MIN all-reduces of S-element arrays (int64 keys
 * (float_bits(m1) << 32 | d) and float second minima, the asw_wta_local protocol).
 * They run over RCCL (ncclAllReduce / ncclMin in one ncclGroupStart/End, one
 * communicator per device from ncclCommInitAll) when the ids are distinct, and as
 * peer copies + a MIN kernel on hip_device_ids[0] when an id repeats (several
 * shards on one GPU).  The LR check and every output are on hip_device_ids[0];
 * results equal a one-GPU context bit for bit. */
int asw_create_multi(const asw_params *p, const int *hip_device_ids, int n_devices, asw_ctx **out);
/* Multi-process (one process per GPU): this process is shard `rank` of `nranks`,
 * the all-reduces run over an RCCL communicator made from `id` (ncclCommInitRank);
 * asw_comm_unique_id makes the id on one rank (ncclGetUniqueId) and the caller
 * shares it with the others (MPI, torch.distributed, a file).  Every rank returns
 * the whole frame's maps and images; the one exception is asw_outputs.cost, which
 * a rank fills only at its own planes [d_begin, d_end) (asw_ctx_shard) and leaves
 * untouched elsewhere (the volume is never gathered).
 * The cross-device RCCL path (distinct GPUs, nranks > 1, or asw_create_multi with
 * distinct ids) runs the same protocol as the tested one-rank and same-device
 * paths; it has not been executed on a multi-GPU box by this project's tests. */
#define ASW_COMM_ID_BYTES 128
int asw_comm_unique_id(uint8_t id[ASW_COMM_ID_BYTES]);
int asw_create_rank(const asw_params *p, int hip_device, int rank, int nranks, const uint8_t id[ASW_COMM_ID_BYTES],
                    asw_ctx **out);
/* shard layout of a context: number of shards it drives in this process and the
 * [d_begin, d_end) of shard i (ASW_E_INVALID for i out of range) */
int asw_ctx_shard(const asw_ctx *ctx, int i, int *n_shards, int *d_begin, int *d_end);
int asw_destroy(asw_ctx *ctx);
/* One stereo pair, host RGBA8 in, host outputs out (any output pointer may be NULL). */
int asw_match(asw_ctx *ctx, const uint8_t *left_rgba, const uint8_t *right_rgba, asw_outputs *out,
              asw_timings *t);
/* `batch` pairs (SURVEY §8(b) `asw_match(ctx, L, R, batch, ...)`): left_rgba /
 * right_rgba hold `batch` consecutive [H][W][4] images, out[b] and t[b] (t may be
 * NULL) receive pair b.  The pairs stream through the context's one set of
 * volumes (a 3840x2160 D512 pair needs ~75 GB with cached denominators; 8 of them
 * are never resident together). */
int asw_match_batch(asw_ctx *ctx, const uint8_t *left_rgba, const uint8_t *right_rgba, int batch,
                    asw_outputs *out, asw_timings *t);
/* turn the refinement loop on for later asw_match calls (rp = NULL or iters = 0:
 * off, the default).  Needs lr_check.  On a multi-shard context the loop's volume
 * scan (asw_WTA_REF) is d-sharded and exchanged like the WTA (asw_wta_ref_local
 * protocol); the per-pixel stages run on the first shard.  asw_match then
 * fills final_rgba / post_red_rgba; every other output (d_ref, d_tar, conf_*,
 * disp_rgba, lr_rgba, lr_red_rgba, disp16, lr16) stays the pre-refinement result
 * (they are copied out before the loop updates its buffers in place). */
int asw_set_refine(asw_ctx *ctx, const asw_refine_params *rp);
/* on != 0: from the next asw_match on, the frame's device work (raw cost to the
 * consistency images, and the refinement loop) is captured once into HIP graphs
 * (hipStreamBeginCapture) and replayed: one launch per graph instead of ~25 (+37 for
 * the loop) kernel launches, for small, launch-bound frames.  Same results.  Only
 * the coarse timings (h2d, total, refine, d2h) are measured.  One-shard contexts. */
int asw_set_graph(asw_ctx *ctx, int on);

#ifdef __cplusplus
}
#endif
#endif /* ASW_H */
