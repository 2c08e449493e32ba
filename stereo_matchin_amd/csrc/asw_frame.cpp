// asw_frame.cpp — FRAME half of the C-ABI (include/asw.h): a context owns one
// GPU's device buffers for one image size and disparity shard, and asw_match()
// runs the reference's ASW sequence for one stereo pair
// (main.cpp:243-244 upload, :463-537 kernels, :621-631 read-back) with HIP
// events in place of the reference's OpenCL profiling events (main.cpp:634-708).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>

#include "asw_common.h"

struct asw_ctx {
    asw_params p;
    int device = 0;
    hipStream_t stream = nullptr;
    uint8_t *left = nullptr, *right = nullptr;  // RGBA8 [H][W][4]
    float *lut = nullptr;
    float *lab_l = nullptr, *lab_r = nullptr;  // float4 [H][W] (ASW_COLOR_LAB only)
    float *wvl = nullptr, *wvr = nullptr, *whl = nullptr, *whr = nullptr;  // [H][W][Tp]
    float *c0 = nullptr, *c1 = nullptr;                                    // [H][W][Dp]
    float *den_v = nullptr, *den_h = nullptr;  // cached denominators [H][W][Dp] (iters >= 2)
    int32_t *d_ref = nullptr, *d_tar = nullptr;
    float *conf_ref = nullptr, *conf_tar = nullptr;
    uint8_t *code_ref = nullptr, *code_tar = nullptr;
    uint8_t *lr = nullptr, *lr_red = nullptr, *disp = nullptr;  // RGBA8
    // refinement loop (asw_set_refine): parameters, workspace, its estimate image
    // (a copy of lr, refined in place) and outputs
    asw_refine_params rp{};
    bool refine = false;
    void *rws = nullptr;
    uint8_t *est = nullptr, *post_red = nullptr, *final_rgba = nullptr;  // RGBA8
    hipEvent_t ev[32] = {};
};

namespace {

int hip_fail(hipError_t e) {
    asw::set_hip_error(e);
    return e == hipErrorOutOfMemory ? ASW_E_NOMEM : ASW_E_HIP;
}

#define HIPCHK(expr)                               \
    do {                                           \
        const hipError_t _e = (expr);              \
        if (_e != hipSuccess) return hip_fail(_e); \
    } while (0)

#define ASWCHK(expr)                \
    do {                            \
        const int _s = (expr);      \
        if (_s != ASW_OK) return _s; \
    } while (0)

template <class T>
int dev_alloc(T **ptr, size_t bytes) {
    void *v = nullptr;
    HIPCHK(hipMalloc(&v, bytes));
    *ptr = static_cast<T *>(v);
    return ASW_OK;
}

double ms_between(hipEvent_t a, hipEvent_t b) {
    float ms = 0.0f;
    if (hipEventElapsedTime(&ms, a, b) != hipSuccess) return -1.0;
    return (double)ms;
}

// grey RGBA image of the 8-bit codes (asw_left_wta written by K/asw_wta.cl:73)
__global__ void k_codes_to_rgba(long long n, const uint8_t *code, uchar4 *out) {
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p < n) {
        const uint8_t c = code[p];
        out[p] = make_uchar4(c, c, c, 255);
    }
}

}  // namespace

extern "C" {

int asw_destroy(asw_ctx *ctx) {
    if (!ctx) return ASW_OK;
    (void)hipSetDevice(ctx->device);
    void *bufs[] = {ctx->left, ctx->right, ctx->lut, ctx->lab_l, ctx->lab_r, ctx->wvl, ctx->wvr, ctx->whl, ctx->whr, ctx->c0, ctx->c1,
                    ctx->den_v, ctx->den_h,
                    ctx->d_ref, ctx->d_tar, ctx->conf_ref, ctx->conf_tar, ctx->code_ref, ctx->code_tar, ctx->lr,
                    ctx->lr_red, ctx->disp, ctx->rws, ctx->est, ctx->post_red, ctx->final_rgba};
    for (void *b : bufs)
        if (b) (void)hipFree(b);
    for (hipEvent_t &e : ctx->ev)
        if (e) (void)hipEventDestroy(e);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return ASW_OK;
}

int asw_create(const asw_params *p, int hip_device, asw_ctx **out) {
    if (!out) return ASW_E_INVALID;
    *out = nullptr;
    ASWCHK(asw_params_check(p));
    if (p->d_begin != 0 || (p->d_end >= 0 && p->d_end != p->ndisp))
        return ASW_E_INVALID;  // the frame API owns the whole range; shards use the stage API
    asw_ctx *c = new (std::nothrow) asw_ctx;
    if (!c) return ASW_E_NOMEM;
    c->p = *p;
    c->device = hip_device;
    const hipError_t e0 = hipSetDevice(hip_device);
    if (e0 != hipSuccess) {
        delete c;
        return hip_fail(e0);
    }
    const size_t S = (size_t)p->width * p->height;
    int s = ASW_OK;
    auto chain = [&](int r) {
        if (s == ASW_OK) s = r;
    };
    chain(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) == hipSuccess ? ASW_OK : ASW_E_HIP);
    chain(dev_alloc(&c->left, S * 4));
    chain(dev_alloc(&c->right, S * 4));
    chain(dev_alloc(&c->lut, asw_lut_bytes(p)));
    if (p->color_space == ASW_COLOR_LAB) {
        chain(dev_alloc(&c->lab_l, asw_lab_bytes(p)));
        chain(dev_alloc(&c->lab_r, asw_lab_bytes(p)));
    }
    chain(dev_alloc(&c->wvl, asw_support_bytes(p)));
    chain(dev_alloc(&c->wvr, asw_support_bytes(p)));
    chain(dev_alloc(&c->whl, asw_support_bytes(p)));
    chain(dev_alloc(&c->whr, asw_support_bytes(p)));
    chain(dev_alloc(&c->c0, asw_cost_bytes(p)));
    chain(dev_alloc(&c->c1, asw_cost_bytes(p)));
    if (p->iters >= 2) {  // the den of a direction is written by its first pass and read by the r-1 others
        chain(dev_alloc(&c->den_v, asw_cost_bytes(p)));
        chain(dev_alloc(&c->den_h, asw_cost_bytes(p)));
    }
    chain(dev_alloc(&c->d_ref, S * 4));
    chain(dev_alloc(&c->d_tar, S * 4));
    chain(dev_alloc(&c->conf_ref, S * 4));
    chain(dev_alloc(&c->conf_tar, S * 4));
    chain(dev_alloc(&c->code_ref, S));
    chain(dev_alloc(&c->code_tar, S));
    chain(dev_alloc(&c->lr, S * 4));
    chain(dev_alloc(&c->lr_red, S * 4));
    chain(dev_alloc(&c->disp, S * 4));
    for (hipEvent_t &e : c->ev) chain(hipEventCreate(&e) == hipSuccess ? ASW_OK : ASW_E_HIP);
    if (s != ASW_OK) {
        asw_destroy(c);
        return s;
    }
    *out = c;
    return ASW_OK;
}

int asw_device_name(int hip_device, char *buf, int len) {
    if (!buf || len < 1) return ASW_E_INVALID;
    buf[0] = '\0';
    hipDeviceProp_t prop;
    const hipError_t e = hipGetDeviceProperties(&prop, hip_device);
    if (e != hipSuccess) return hip_fail(e);
    std::snprintf(buf, (size_t)len, "%s", prop.name[0] ? prop.name : prop.gcnArchName);
    return ASW_OK;
}

int asw_set_refine(asw_ctx *c, const asw_refine_params *rp) {
    if (!c) return ASW_E_INVALID;
    if (!rp || rp->iters <= 0) {
        c->refine = false;
        return ASW_OK;
    }
    const int s = asw_refine_params_check(&c->p, rp);
    if (s != ASW_OK) return s;
    if (!c->p.lr_check) return ASW_E_INVALID;  // the loop starts from the consistency image
    HIPCHK(hipSetDevice(c->device));
    const size_t S = (size_t)c->p.width * c->p.height;
    const size_t ws = asw_refine_workspace_bytes(&c->p, rp);
    if (c->rws) (void)hipFree(c->rws);
    c->rws = nullptr;
    ASWCHK(dev_alloc(&c->rws, ws));
    if (!c->est) ASWCHK(dev_alloc(&c->est, S * 4));
    if (!c->post_red) ASWCHK(dev_alloc(&c->post_red, S * 4));
    if (!c->final_rgba) ASWCHK(dev_alloc(&c->final_rgba, S * 4));
    c->rp = *rp;
    c->refine = true;
    return ASW_OK;
}

int asw_match(asw_ctx *c, const uint8_t *left_rgba, const uint8_t *right_rgba, asw_outputs *o, asw_timings *t) {
    if (!c || !left_rgba || !right_rgba) return ASW_E_INVALID;
    HIPCHK(hipSetDevice(c->device));
    const asw_params *p = &c->p;
    const size_t S = (size_t)p->width * p->height;
    hipStream_t st = c->stream;
    hipEvent_t *ev = c->ev;
    const int r = p->iters;
    // event slots: 0 h2d start, 1 raw start, 2 raw end / support start, 3 support end,
    // 4.. per pass (2r+1 slots), then wta end, consistency end, d2h end.
    const int e_pass0 = 4;
    const int e_wta = e_pass0 + 2 * r + 1 > 28 ? -1 : e_pass0 + 2 * r + 1;  // slots up to e_wta + 3 = 31
    const bool timed = e_wta >= 0;

    HIPCHK(hipEventRecord(ev[0], st));
    HIPCHK(hipMemcpyAsync(c->left, left_rgba, S * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(c->right, right_rgba, S * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipEventRecord(ev[1], st));
    // asw_Aggr is fused into the first V pass (asw_aggregate_pass_raw): the raw
    // cost volume is never materialised and the "aggr" time slot stays empty,
    // unless there is no pass at all (r = 0)
    if (r == 0) ASWCHK(asw_raw_cost(p, c->left, c->right, c->c0, st));
    HIPCHK(hipEventRecord(ev[2], st));
    if (p->color_space == ASW_COLOR_LAB) {
        ASWCHK(asw_lab(p, c->left, c->lab_l, st));
        ASWCHK(asw_lab(p, c->right, c->lab_r, st));
        ASWCHK(asw_support_lab(p, ASW_DIR_V, c->lab_l, c->wvl, st));
        ASWCHK(asw_support_lab(p, ASW_DIR_H, c->lab_l, c->whl, st));
        ASWCHK(asw_support_lab(p, ASW_DIR_V, c->lab_r, c->wvr, st));
        ASWCHK(asw_support_lab(p, ASW_DIR_H, c->lab_r, c->whr, st));
    } else {
        ASWCHK(asw_support_lut(p, c->lut, st));
        ASWCHK(asw_support(p, ASW_DIR_V, c->left, c->lut, c->wvl, st));
        ASWCHK(asw_support(p, ASW_DIR_H, c->left, c->lut, c->whl, st));
        ASWCHK(asw_support(p, ASW_DIR_V, c->right, c->lut, c->wvr, st));
        ASWCHK(asw_support(p, ASW_DIR_H, c->right, c->lut, c->whr, st));
    }
    HIPCHK(hipEventRecord(ev[3], st));
    if (timed) HIPCHK(hipEventRecord(ev[e_pass0], st));
    for (int it = 0; it < r; ++it) {
        const int dm = !c->den_v ? ASW_DEN_NONE : (it == 0 ? ASW_DEN_WRITE : ASW_DEN_READ);
        if (it == 0)
            ASWCHK(asw_aggregate_pass_raw(p, c->wvl, c->wvr, c->left, c->right, c->c1, c->den_v, dm, st));
        else
            ASWCHK(asw_aggregate_pass_den(p, ASW_DIR_V, c->wvl, c->wvr, c->c0, c->c1, c->den_v, dm, st));
        if (timed) HIPCHK(hipEventRecord(ev[e_pass0 + 2 * it + 1], st));
        ASWCHK(asw_aggregate_pass_den(p, ASW_DIR_H, c->whl, c->whr, c->c1, c->c0, c->den_h, dm, st));
        if (timed) HIPCHK(hipEventRecord(ev[e_pass0 + 2 * it + 2], st));
    }
    ASWCHK(asw_wta(p, c->c0, c->d_ref, c->conf_ref, c->d_tar, c->conf_tar, c->code_ref, c->code_tar, st));
    if (timed) HIPCHK(hipEventRecord(ev[e_wta], st));
    hipLaunchKernelGGL(k_codes_to_rgba, dim3((unsigned)((S + 255) / 256)), dim3(256), 0, st, (long long)S,
                       c->code_ref, reinterpret_cast<uchar4 *>(c->disp));
    HIPCHK(hipGetLastError());
    if (p->lr_check)
        ASWCHK(asw_consistency(p, c->d_ref, c->d_tar, c->code_ref, c->code_tar, c->conf_ref, c->conf_tar, c->lr,
                               c->lr_red, st));
    if (timed) HIPCHK(hipEventRecord(ev[e_wta + 1], st));
    const bool refine = c->refine && p->lr_check;
    if (refine) {  // main.cpp:540-617 on a copy of consistency_error
        HIPCHK(hipMemcpyAsync(c->est, c->lr, S * 4, hipMemcpyDeviceToDevice, st));
        ASWCHK(asw_refine(p, &c->rp, c->left, c->right, c->c0, c->est, c->code_tar, c->conf_ref, c->conf_tar, c->rws,
                          c->post_red, c->final_rgba, nullptr, nullptr, st));
    }
    if (timed) HIPCHK(hipEventRecord(ev[e_wta + 2], st));
    if (o) {
        if (o->d_ref) HIPCHK(hipMemcpyAsync(o->d_ref, c->d_ref, S * 4, hipMemcpyDeviceToHost, st));
        if (o->d_tar) HIPCHK(hipMemcpyAsync(o->d_tar, c->d_tar, S * 4, hipMemcpyDeviceToHost, st));
        if (o->conf_ref) HIPCHK(hipMemcpyAsync(o->conf_ref, c->conf_ref, S * 4, hipMemcpyDeviceToHost, st));
        if (o->conf_tar) HIPCHK(hipMemcpyAsync(o->conf_tar, c->conf_tar, S * 4, hipMemcpyDeviceToHost, st));
        if (o->disp_rgba) HIPCHK(hipMemcpyAsync(o->disp_rgba, c->disp, S * 4, hipMemcpyDeviceToHost, st));
        if (o->lr_rgba && p->lr_check) HIPCHK(hipMemcpyAsync(o->lr_rgba, c->lr, S * 4, hipMemcpyDeviceToHost, st));
        if (o->lr_red_rgba && p->lr_check)
            HIPCHK(hipMemcpyAsync(o->lr_red_rgba, c->lr_red, S * 4, hipMemcpyDeviceToHost, st));
        if (o->cost) HIPCHK(hipMemcpyAsync(o->cost, c->c0, asw_cost_bytes(p), hipMemcpyDeviceToHost, st));
        if (o->final_rgba && refine)
            HIPCHK(hipMemcpyAsync(o->final_rgba, c->final_rgba, S * 4, hipMemcpyDeviceToHost, st));
        if (o->post_red_rgba && refine && c->rp.iters > 0)
            HIPCHK(hipMemcpyAsync(o->post_red_rgba, c->post_red, S * 4, hipMemcpyDeviceToHost, st));
    }
    if (timed) HIPCHK(hipEventRecord(ev[e_wta + 3], st));
    HIPCHK(hipStreamSynchronize(st));
    if (t && timed) {
        std::memset(t, 0, sizeof(*t));
        t->h2d = ms_between(ev[0], ev[1]);
        t->raw_cost = ms_between(ev[1], ev[2]);
        t->support = ms_between(ev[2], ev[3]);
        double v = 0.0, h = 0.0;
        for (int it = 0; it < r; ++it) {
            v += ms_between(ev[e_pass0 + 2 * it], ev[e_pass0 + 2 * it + 1]);
            h += ms_between(ev[e_pass0 + 2 * it + 1], ev[e_pass0 + 2 * it + 2]);
        }
        t->v_pass_mean = r ? v / r : 0.0;
        t->h_pass_mean = r ? h / r : 0.0;
        t->aggregation_total = ms_between(ev[e_pass0], ev[e_pass0 + 2 * r]);
        t->wta = ms_between(ev[e_pass0 + 2 * r], ev[e_wta]);
        t->consistency = ms_between(ev[e_wta], ev[e_wta + 1]);
        t->total = ms_between(ev[1], ev[e_wta + 1]);
        t->refine = refine ? ms_between(ev[e_wta + 1], ev[e_wta + 2]) : 0.0;
        t->d2h = ms_between(ev[e_wta + 2], ev[e_wta + 3]);
    }
    return ASW_OK;
}

}  // extern "C"
