// asw_frame.cpp — FRAME half of the C-ABI (include/asw.h): a context owns the
// device buffers of one image size and runs the reference's ASW sequence for a
// stereo pair (main.cpp:243-244 upload, :463-537 kernels, :540-623 refinement,
// :621-631 read-back), with HIP events in place of the reference's OpenCL
// profiling events (main.cpp:634-708).
//
// A context drives one or more SHARDS: contiguous disparity ranges, each with its
// own device, stream and volumes (the reference runs one device per pass of its
// device loop, main.cpp:158-172; it has no multi-device path).  Shards need no
// communication until the WTA, which is the exchange of the d-sharded protocol
// (asw_wta_local ... asw_wta_finalize): four elementwise MIN all-reduces, over
// RCCL when the shards' devices are distinct (one process: ncclCommInitAll; one
// process per GPU: ncclCommInitRank), else over peer copies and a MIN kernel on
// the first shard's device (several shards on one GPU).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "asw_common.h"

namespace {

constexpr int kMaxShards = 64;

enum CommMode { COMM_NONE = 0, COMM_RCCL = 1, COMM_LOCAL = 2 };

struct Shard {
    int device = 0;
    hipStream_t stream = nullptr;
    asw_params p{};                     // this shard's [d_begin, d_end)
    uint8_t *left = nullptr, *right = nullptr;  // RGBA8 [H][W][4]
    float *lut = nullptr;
    float *lab_l = nullptr, *lab_r = nullptr;  // float4 [H][W] (ASW_COLOR_LAB only)
    float *wvl = nullptr, *wvr = nullptr, *whl = nullptr, *whr = nullptr;  // [H][W][Tp]
    float *c0 = nullptr, *c1 = nullptr;                                    // [H][W][Dp]
    float *den_v = nullptr, *den_h = nullptr;  // cached denominators (iters >= 2)
    bool raw16 = false; // the raw costs as uint16 in c0 (asw_raw_cost16 + asw_aggregate_pass_den16)
    // d-sharded WTA (more than one shard in the frame)
    int64_t *key = nullptr, *key_g = nullptr, *tkey = nullptr, *tkey_g = nullptr;
    float *m1 = nullptr, *m2 = nullptr, *t1 = nullptr, *t2 = nullptr, *m2_g = nullptr, *t2_g = nullptr;
    ncclComm_t comm = nullptr;
    hipEvent_t ready = nullptr;  // COMM_LOCAL: this shard's operand is complete
    float *ref_l = nullptr, *ref_r = nullptr;  // sharded refinement, shards > 0: the per-view estimates
};

}  // namespace

struct asw_ctx {
    asw_params p{};          // the whole frame
    int n = 0;               // shards driven by this process
    int rank = 0, nranks = 1;  // multi-process: this process's shard of nranks (n = 1)
    CommMode comm = COMM_NONE;
    Shard sh[kMaxShards];
    void *red_tmp = nullptr;  // COMM_LOCAL: (n-1) x S int64 operands copied to shard 0's device
    hipEvent_t red_done = nullptr;
    // outputs, on shard 0's device
    int32_t *d_ref = nullptr, *d_tar = nullptr;
    float *conf_ref = nullptr, *conf_tar = nullptr;
    uint8_t *code_ref = nullptr, *code_tar = nullptr;
    uint8_t *lr = nullptr, *lr_red = nullptr, *disp = nullptr;  // RGBA8
    uint16_t *disp16 = nullptr, *lr16 = nullptr;
    // refinement loop (asw_set_refine): parameters, workspace, its estimate image
    // (a copy of lr, refined in place) and outputs
    asw_refine_params rp{};
    bool refine = false;
    void *rws = nullptr;
    uint8_t *est = nullptr, *post_red = nullptr, *final_rgba = nullptr;  // RGBA8
    std::vector<hipEvent_t> ev;  // timing events on shard 0's stream
    // asw_set_graph: the frame's device work captured once into HIP graphs, replayed
    bool graph = false;
    hipGraph_t g_main = nullptr, g_ref = nullptr;
    hipGraphExec_t gx_main = nullptr, gx_ref = nullptr;
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

#define ASWCHK(expr)                 \
    do {                             \
        const int _s = (expr);       \
        if (_s != ASW_OK) return _s; \
    } while (0)

#define NCCLCHK(expr)                                \
    do {                                             \
        const ncclResult_t _r = (expr);              \
        if (_r != ncclSuccess) return ASW_E_COMM;    \
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

// 16-bit disparity images: d_ref, and d_ref where the LR check of asw_consistency
// (same rule: 8-bit codes or native indices) passes, ASW_DISP16_INVALID elsewhere
__global__ void k_disp16(long long n, int D, int mode, int lr, const int32_t *d_ref, const int32_t *d_tar,
                         const uint8_t *code_ref, const uint8_t *code_tar, uint16_t *disp16, uint16_t *lr16) {
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const int dr = d_ref[p];
    if (disp16) disp16[p] = (uint16_t)dr;
    if (!lr16 || !lr) return;
    bool cons;
    if (mode == ASW_LR_U8) {
        const float scale = (float)(D - 1);
        const float qr = ((float)code_ref[p] / 255.0f) * scale;
        const float qt = ((float)code_tar[p] / 255.0f) * scale;
        cons = fabsf(qt - qr) < 1.001f;
    } else {
        const int dd = dr - d_tar[p];
        cons = dd <= 1 && dd >= -1;
    }
    lr16[p] = cons ? (uint16_t)dr : (uint16_t)ASW_DISP16_INVALID;
}

// elementwise MIN of n operands (COMM_LOCAL all-reduce), written to out
struct MinOperands {
    const void *p[kMaxShards];
    int n;
};
template <class T>
__global__ void k_min_n(long long count, MinOperands ops, T *out) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    T v = static_cast<const T *>(ops.p[0])[i];
    for (int k = 1; k < ops.n; ++k) {
        const T o = static_cast<const T *>(ops.p[k])[i];
        v = o < v ? o : v;
    }
    out[i] = v;
}

size_t frame_pixels(const asw_params *p) { return (size_t)p->width * p->height; }

// In-place elementwise MIN all-reduce of buf(shard) (count elements of T) over
// every shard of the frame.  Stream-ordered on each shard's stream.
template <class T>
int allreduce_min(asw_ctx *c, T *(*buf)(Shard &), ncclDataType_t type) {
    const size_t S = frame_pixels(&c->p);
    if (c->comm == COMM_RCCL) {
        NCCLCHK(ncclGroupStart());
        for (int i = 0; i < c->n; ++i) {
            Shard &s = c->sh[i];
            T *b = buf(s);
            const ncclResult_t r = ncclAllReduce(b, b, S, type, ncclMin, s.comm, s.stream);
            if (r != ncclSuccess) {
                (void)ncclGroupEnd();
                return ASW_E_COMM;
            }
        }
        NCCLCHK(ncclGroupEnd());
        return ASW_OK;
    }
    if (c->comm != COMM_LOCAL) return ASW_OK;  // one shard: nothing to reduce
    Shard &s0 = c->sh[0];
    MinOperands ops{};
    ops.n = c->n;
    for (int i = 0; i < c->n; ++i) {
        Shard &s = c->sh[i];
        HIPCHK(hipSetDevice(s.device));
        HIPCHK(hipEventRecord(s.ready, s.stream));
    }
    HIPCHK(hipSetDevice(s0.device));
    for (int i = 0; i < c->n; ++i) HIPCHK(hipStreamWaitEvent(s0.stream, c->sh[i].ready, 0));
    T *tmp = static_cast<T *>(c->red_tmp);
    for (int i = 0; i < c->n; ++i) {
        Shard &s = c->sh[i];
        if (s.device == s0.device) {
            ops.p[i] = buf(s);  // same device: read in place
        } else {
            T *dst = tmp + (size_t)(i - 1) * S;
            HIPCHK(hipMemcpyPeerAsync(dst, s0.device, buf(s), s.device, S * sizeof(T), s0.stream));
            ops.p[i] = dst;
        }
    }
    hipLaunchKernelGGL(k_min_n<T>, dim3((unsigned)((S + 255) / 256)), dim3(256), 0, s0.stream, (long long)S, ops,
                       buf(s0));
    HIPCHK(hipGetLastError());
    for (int i = 1; i < c->n; ++i) {
        Shard &s = c->sh[i];
        if (s.device == s0.device)
            HIPCHK(hipMemcpyAsync(buf(s), buf(s0), S * sizeof(T), hipMemcpyDeviceToDevice, s0.stream));
        else
            HIPCHK(hipMemcpyPeerAsync(buf(s), s.device, buf(s0), s0.device, S * sizeof(T), s0.stream));
    }
    HIPCHK(hipEventRecord(c->red_done, s0.stream));
    for (int i = 1; i < c->n; ++i) {
        HIPCHK(hipSetDevice(c->sh[i].device));
        HIPCHK(hipStreamWaitEvent(c->sh[i].stream, c->red_done, 0));
    }
    return ASW_OK;
}

int64_t *b_key_g(Shard &s) { return s.key_g; }
int64_t *b_tkey_g(Shard &s) { return s.tkey_g; }
float *b_m2_g(Shard &s) { return s.m2_g; }
float *b_t2_g(Shard &s) { return s.t2_g; }

void free_shard(Shard &s) {
    if (s.stream == nullptr && s.left == nullptr) return;
    (void)hipSetDevice(s.device);
    void *bufs[] = {s.left, s.right, s.lut, s.lab_l, s.lab_r, s.wvl, s.wvr, s.whl, s.whr, s.c0, s.c1, s.den_v,
                    s.den_h, s.key, s.key_g, s.tkey, s.tkey_g, s.m1, s.m2, s.t1, s.t2, s.m2_g, s.t2_g, s.ref_l,
                    s.ref_r};
    for (void *b : bufs)
        if (b) (void)hipFree(b);
    if (s.comm) (void)ncclCommDestroy(s.comm);
    if (s.ready) (void)hipEventDestroy(s.ready);
    if (s.stream) (void)hipStreamDestroy(s.stream);
    s = Shard{};
}

int alloc_shard(Shard &s, bool sharded) {
    const asw_params *p = &s.p;
    const size_t S = frame_pixels(p);
    HIPCHK(hipSetDevice(s.device));
    HIPCHK(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
    HIPCHK(hipEventCreateWithFlags(&s.ready, hipEventDisableTiming));
    ASWCHK(dev_alloc(&s.left, S * 4));
    ASWCHK(dev_alloc(&s.right, S * 4));
    ASWCHK(dev_alloc(&s.lut, asw_lut_bytes(p)));
    if (p->color_space == ASW_COLOR_LAB) {
        ASWCHK(dev_alloc(&s.lab_l, asw_lab_bytes(p)));
        ASWCHK(dev_alloc(&s.lab_r, asw_lab_bytes(p)));
    }
    // the raw-cost volume as uint16 (half the bytes written by asw_Aggr and read by the
    // first V pass; bit-identical) where built; ASW_FLAG_RAW_F32 keeps the float volume
    s.raw16 = !(p->flags & ASW_FLAG_RAW_F32) && asw_raw16_supported(p);
    ASWCHK(dev_alloc(&s.wvl, asw_support_bytes(p)));
    ASWCHK(dev_alloc(&s.wvr, asw_support_bytes(p)));
    ASWCHK(dev_alloc(&s.whl, asw_support_bytes(p)));
    ASWCHK(dev_alloc(&s.whr, asw_support_bytes(p)));
    ASWCHK(dev_alloc(&s.c0, asw_cost_bytes(p)));
    ASWCHK(dev_alloc(&s.c1, asw_cost_bytes(p)));
    if (p->iters >= 2 && asw_disp_pitch(p) != 32) {
        // the den of a direction is written by its first pass and read by the r-1 others
        // (a 32-plane shard's passes recompute it: at C4 / 8 k_vpass32 den-none 0.24 against
        // den-read 0.28 ms, k_hpass32 0.30-0.33 against 0.36, profiles/r04/h32_variants_r11d.log;
        // in the shard frame 4.99 against 5.04 ms, profiles/r04/shard_den_h_ab_r11e.log)
        ASWCHK(dev_alloc(&s.den_v, asw_cost_bytes(p)));
        ASWCHK(dev_alloc(&s.den_h, asw_cost_bytes(p)));
    }
    if (sharded) {
        ASWCHK(dev_alloc(&s.key, S * 8));
        ASWCHK(dev_alloc(&s.key_g, S * 8));
        ASWCHK(dev_alloc(&s.tkey, S * 8));
        ASWCHK(dev_alloc(&s.tkey_g, S * 8));
        ASWCHK(dev_alloc(&s.m1, S * 4));
        ASWCHK(dev_alloc(&s.m2, S * 4));
        ASWCHK(dev_alloc(&s.t1, S * 4));
        ASWCHK(dev_alloc(&s.t2, S * 4));
        ASWCHK(dev_alloc(&s.m2_g, S * 4));
        ASWCHK(dev_alloc(&s.t2_g, S * 4));
    }
    return ASW_OK;
}

// contiguous balanced split of [0, D) (stereo_matchin_amd/distributed.py shard_range)
void shard_range(int D, int i, int n, int *b, int *e) {
    const int base = D / n, rem = D % n;
    *b = i * base + (i < rem ? i : rem);
    *e = *b + base + (i < rem ? 1 : 0);
}

int destroy_ctx(asw_ctx *c) {
    if (!c) return ASW_OK;
    for (int i = 0; i < kMaxShards; ++i) free_shard(c->sh[i]);
    (void)hipSetDevice(c->sh[0].device);
    void *bufs[] = {c->red_tmp, c->d_ref, c->d_tar, c->conf_ref, c->conf_tar, c->code_ref, c->code_tar, c->lr,
                    c->lr_red, c->disp, c->disp16, c->lr16, c->rws, c->est, c->post_red, c->final_rgba};
    for (void *b : bufs)
        if (b) (void)hipFree(b);
    for (hipEvent_t e : c->ev)
        if (e) (void)hipEventDestroy(e);
    if (c->red_done) (void)hipEventDestroy(c->red_done);
    if (c->gx_main) (void)hipGraphExecDestroy(c->gx_main);
    if (c->gx_ref) (void)hipGraphExecDestroy(c->gx_ref);
    if (c->g_main) (void)hipGraphDestroy(c->g_main);
    if (c->g_ref) (void)hipGraphDestroy(c->g_ref);
    delete c;
    return ASW_OK;
}

// Shared constructor.  This process drives shards [shard0, shard0 + n) of `total`
// (devs[i] = the device of its i-th shard); comm selects the exchange.
int create_ctx(const asw_params *p, const int *devs, int n, int shard0, int total, CommMode comm,
               const ncclUniqueId *id, asw_ctx **out) {
    if (!out) return ASW_E_INVALID;
    *out = nullptr;
    ASWCHK(asw_params_check(p));
    if (p->d_begin != 0 || (p->d_end >= 0 && p->d_end != p->ndisp)) return ASW_E_INVALID;  // contexts shard themselves
    if (n < 1 || n > kMaxShards || total < n || total > p->ndisp) return ASW_E_INVALID;
    // a shape the pass kernels cannot address fails here, before any device call or
    // allocation (tens of GB for an 8K frame), not at the first pass
    for (int i = 0; i < n; ++i) {
        asw_params sp = *p;
        sp.d_end = p->ndisp;
        shard_range(p->ndisp, shard0 + i, total, &sp.d_begin, &sp.d_end);
        ASWCHK(asw::pass_shape_check(&sp));
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0;
    for (int i = 0; i < n; ++i)
        if (devs[i] < 0 || devs[i] >= ndev) return ASW_E_INVALID;
    asw_ctx *c = new (std::nothrow) asw_ctx;
    if (!c) return ASW_E_NOMEM;
    c->p = *p;
    c->p.d_end = p->ndisp;
    c->n = n;
    c->rank = shard0;
    c->nranks = total;
    c->comm = comm;
    const size_t S = frame_pixels(p);
    int s = ASW_OK;
    auto chain = [&](int r) {
        if (s == ASW_OK) s = r;
    };
    for (int i = 0; i < n && s == ASW_OK; ++i) {
        Shard &sh = c->sh[i];
        sh.device = devs[i];
        sh.p = c->p;
        shard_range(p->ndisp, shard0 + i, total, &sh.p.d_begin, &sh.p.d_end);
        chain(alloc_shard(sh, comm != COMM_NONE));
    }
    if (s == ASW_OK && comm == COMM_LOCAL) {
        chain(hipSetDevice(devs[0]) == hipSuccess ? ASW_OK : ASW_E_HIP);
        chain(hipEventCreateWithFlags(&c->red_done, hipEventDisableTiming) == hipSuccess ? ASW_OK : ASW_E_HIP);
        bool peers = false;
        for (int i = 1; i < n; ++i) peers = peers || devs[i] != devs[0];
        if (peers) chain(dev_alloc(&c->red_tmp, (size_t)(n - 1) * S * 8));
    }
    if (s == ASW_OK && comm == COMM_RCCL) {
        ncclComm_t comms[kMaxShards] = {};
        ncclResult_t r = ncclSuccess;
        if (id) {  // one process per GPU
            const hipError_t e = hipSetDevice(devs[0]);
            if (e != hipSuccess) s = hip_fail(e);  // a device-selection failure, not a communicator one
            else r = ncclCommInitRank(&comms[0], total, *id, shard0);
        } else {
            r = ncclCommInitAll(comms, n, devs);
        }
        if (s == ASW_OK && r != ncclSuccess) s = ASW_E_COMM;
        for (int i = 0; i < n; ++i) c->sh[i].comm = comms[i];
    }
    if (s == ASW_OK) {
        chain(hipSetDevice(devs[0]) == hipSuccess ? ASW_OK : ASW_E_HIP);
        chain(dev_alloc(&c->d_ref, S * 4));
        chain(dev_alloc(&c->d_tar, S * 4));
        chain(dev_alloc(&c->conf_ref, S * 4));
        chain(dev_alloc(&c->conf_tar, S * 4));
        chain(dev_alloc(&c->code_ref, S));
        chain(dev_alloc(&c->code_tar, S));
        chain(dev_alloc(&c->lr, S * 4));
        chain(dev_alloc(&c->lr_red, S * 4));
        chain(dev_alloc(&c->disp, S * 4));
        chain(dev_alloc(&c->disp16, S * 2));
        chain(dev_alloc(&c->lr16, S * 2));
        // h2d, raw, support, 2r+1 pass marks, exchange, wta, consistency, refine, d2h
        c->ev.assign(2 * (size_t)p->iters + 10, nullptr);
        for (hipEvent_t &e : c->ev)
            if (s == ASW_OK) chain(hipEventCreate(&e) == hipSuccess ? ASW_OK : ASW_E_HIP);
    }
    if (s != ASW_OK) {
        destroy_ctx(c);
        return s;
    }
    *out = c;
    return ASW_OK;
}

// raw cost + supports + 2r passes of one shard, asynchronous on its stream.
// Pass-boundary events (timing) are recorded only for shard 0.
int shard_aggregate(asw_ctx *c, int i, const uint8_t *left_rgba, const uint8_t *right_rgba, int e_raw, int e_pass0,
                    bool timing = true) {
    Shard &s = c->sh[i];
    const asw_params *p = &s.p;
    const size_t S = frame_pixels(p);
    hipStream_t st = s.stream;
    const bool timed = i == 0 && timing;
    HIPCHK(hipSetDevice(s.device));
    if (left_rgba) {  // NULL: the images are already on the device (graph replay)
        HIPCHK(hipMemcpyAsync(s.left, left_rgba, S * 4, hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(s.right, right_rgba, S * 4, hipMemcpyHostToDevice, st));
    }
    if (timed) HIPCHK(hipEventRecord(c->ev[e_raw], st));
    // the raw cost (uint16 where the first pass reads it so)
    if (s.raw16) ASWCHK(asw_raw_cost16(p, s.left, s.right, reinterpret_cast<uint16_t *>(s.c0), st));
    else ASWCHK(asw_raw_cost(p, s.left, s.right, s.c0, st));
    if (timed) HIPCHK(hipEventRecord(c->ev[e_raw + 1], st));
    if (p->color_space == ASW_COLOR_LAB) {
        ASWCHK(asw_lab(p, s.left, s.lab_l, st));
        ASWCHK(asw_lab(p, s.right, s.lab_r, st));
        ASWCHK(asw_support_lab(p, ASW_DIR_V, s.lab_l, s.wvl, st));
        ASWCHK(asw_support_lab(p, ASW_DIR_H, s.lab_l, s.whl, st));
        ASWCHK(asw_support_lab(p, ASW_DIR_V, s.lab_r, s.wvr, st));
        ASWCHK(asw_support_lab(p, ASW_DIR_H, s.lab_r, s.whr, st));
    } else {
        ASWCHK(asw_support_lut(p, s.lut, st));
        ASWCHK(asw_support_all(p, s.left, s.right, s.lut, s.wvl, s.whl, s.wvr, s.whr, st));
    }
    if (timed) HIPCHK(hipEventRecord(c->ev[e_pass0], st));
    for (int it = 0; it < p->iters; ++it) {
        const int dmv = !s.den_v ? ASW_DEN_NONE : (it == 0 ? ASW_DEN_WRITE : ASW_DEN_READ);
        const int dm = !s.den_h ? ASW_DEN_NONE : (it == 0 ? ASW_DEN_WRITE : ASW_DEN_READ);
        if (it == 0 && s.raw16)
            ASWCHK(asw_aggregate_pass_den16(p, s.wvl, s.wvr, reinterpret_cast<const uint16_t *>(s.c0), s.c1, s.den_v,
                                            dmv, st));
        else ASWCHK(asw_aggregate_pass_den(p, ASW_DIR_V, s.wvl, s.wvr, s.c0, s.c1, s.den_v, dmv, st));
        if (timed) HIPCHK(hipEventRecord(c->ev[e_pass0 + 2 * it + 1], st));
        ASWCHK(asw_aggregate_pass_den(p, ASW_DIR_H, s.whl, s.whr, s.c1, s.c0, s.den_h, dm, st));
        if (timed) HIPCHK(hipEventRecord(c->ev[e_pass0 + 2 * it + 2], st));
    }
    return ASW_OK;
}

// The WTA of a one-shard frame
int single_wta(asw_ctx *c) {
    Shard &s0 = c->sh[0];
    return asw_wta(&s0.p, s0.c0, c->d_ref, c->conf_ref, c->d_tar, c->conf_tar, c->code_ref, c->code_tar, s0.stream);
}

// The d-sharded WTA (asw_wta_local protocol, include/asw.h): maps on shard 0.
int sharded_wta(asw_ctx *c) {
    const size_t S = frame_pixels(&c->p);
    for (int i = 0; i < c->n; ++i) {
        Shard &s = c->sh[i];
        HIPCHK(hipSetDevice(s.device));
        ASWCHK(asw_wta_local(&s.p, s.c0, s.key, s.m1, s.m2, s.stream));
        HIPCHK(hipMemcpyAsync(s.key_g, s.key, S * 8, hipMemcpyDeviceToDevice, s.stream));
    }
    ASWCHK(allreduce_min<int64_t>(c, b_key_g, ncclInt64));
    for (int i = 0; i < c->n; ++i) {
        Shard &s = c->sh[i];
        HIPCHK(hipSetDevice(s.device));
        ASWCHK(asw_wta_second(&s.p, s.key_g, s.key, s.m1, s.m2, s.m2_g, s.stream));
    }
    ASWCHK(allreduce_min<float>(c, b_m2_g, ncclFloat32));
    for (int i = 0; i < c->n; ++i) {
        Shard &s = c->sh[i];
        HIPCHK(hipSetDevice(s.device));
        ASWCHK(asw_wta_target_local(&s.p, s.c0, s.key_g, s.tkey, s.t1, s.t2, s.stream));
        HIPCHK(hipMemcpyAsync(s.tkey_g, s.tkey, S * 8, hipMemcpyDeviceToDevice, s.stream));
    }
    ASWCHK(allreduce_min<int64_t>(c, b_tkey_g, ncclInt64));
    for (int i = 0; i < c->n; ++i) {
        Shard &s = c->sh[i];
        HIPCHK(hipSetDevice(s.device));
        ASWCHK(asw_wta_second(&s.p, s.tkey_g, s.tkey, s.t1, s.t2, s.t2_g, s.stream));
    }
    ASWCHK(allreduce_min<float>(c, b_t2_g, ncclFloat32));
    Shard &s0 = c->sh[0];
    HIPCHK(hipSetDevice(s0.device));
    return asw_wta_finalize(&s0.p, s0.key_g, s0.m2_g, s0.tkey_g, s0.t2_g, c->d_ref, c->conf_ref, c->d_tar,
                            c->conf_tar, c->code_ref, c->code_tar, s0.stream);
}

// The refinement loop (main.cpp:540-617) + median on a d-sharded frame.  The
// per-pixel stages (asw_ref_v / asw_ref_h, consistency, median) run on shard 0 (in
// one process per GPU: on every rank, identically); the volume scan (asw_WTA_REF)
// runs on every shard and is exchanged like the WTA: MIN all-reduces of the left
// key, the target key and the target second minimum (asw_wta_ref_local protocol).
int refine_sharded(asw_ctx *c) {
    const asw_params *p = &c->p;
    const asw_refine_params *rp = &c->rp;
    const size_t S = frame_pixels(p);
    Shard &s0 = c->sh[0];
    hipStream_t st = s0.stream;
    char *ws = static_cast<char *>(c->rws);
    float *lut = reinterpret_cast<float *>(ws);
    ws += (asw_refine_lut_bytes(rp) + 255) / 256 * 256;
    float *vl = reinterpret_cast<float *>(ws), *vr = vl + 2 * S, *hl = vr + 2 * S, *hr = hl + 2 * S;
    int32_t *dr = reinterpret_cast<int32_t *>(hr + 2 * S), *dt = dr + S;
    uint8_t *kl = reinterpret_cast<uint8_t *>(dt + S);
    HIPCHK(hipSetDevice(s0.device));
    ASWCHK(asw_refine_lut(p, rp, lut, st));
    for (int it = 0; it < rp->iters; ++it) {
        HIPCHK(hipSetDevice(s0.device));
        ASWCHK(asw_ref_v(p, rp, s0.left, c->est, 4, c->conf_ref, lut, vl, st));
        ASWCHK(asw_ref_v(p, rp, s0.right, c->code_tar, 1, c->conf_tar, lut, vr, st));
        ASWCHK(asw_ref_h(p, rp, s0.left, c->conf_ref, vl, lut, hl, st));
        ASWCHK(asw_ref_h(p, rp, s0.right, c->conf_tar, vr, lut, hr, st));
        for (int i = 1; i < c->n; ++i) {  // the estimates to the other shards' devices
            Shard &s = c->sh[i];
            HIPCHK(hipMemcpyPeerAsync(s.ref_l, s.device, hl, s0.device, 2 * S * 4, st));
            HIPCHK(hipMemcpyPeerAsync(s.ref_r, s.device, hr, s0.device, 2 * S * 4, st));
        }
        if (c->n > 1) {
            HIPCHK(hipEventRecord(c->red_done, st));
            for (int i = 1; i < c->n; ++i) {
                HIPCHK(hipSetDevice(c->sh[i].device));
                HIPCHK(hipStreamWaitEvent(c->sh[i].stream, c->red_done, 0));
            }
        }
        for (int i = 0; i < c->n; ++i) {
            Shard &s = c->sh[i];
            HIPCHK(hipSetDevice(s.device));
            ASWCHK(asw_wta_ref_local(&s.p, s.c0, i ? s.ref_l : hl, s.key, s.m1, s.m2, s.stream));
            HIPCHK(hipMemcpyAsync(s.key_g, s.key, S * 8, hipMemcpyDeviceToDevice, s.stream));
        }
        ASWCHK(allreduce_min<int64_t>(c, b_key_g, ncclInt64));
        for (int i = 0; i < c->n; ++i) {
            Shard &s = c->sh[i];
            HIPCHK(hipSetDevice(s.device));
            ASWCHK(asw_wta_ref_target_local(&s.p, s.c0, i ? s.ref_r : hr, s.key_g, s.tkey, s.t1, s.t2, s.stream));
            HIPCHK(hipMemcpyAsync(s.tkey_g, s.tkey, S * 8, hipMemcpyDeviceToDevice, s.stream));
        }
        ASWCHK(allreduce_min<int64_t>(c, b_tkey_g, ncclInt64));
        for (int i = 0; i < c->n; ++i) {
            Shard &s = c->sh[i];
            HIPCHK(hipSetDevice(s.device));
            ASWCHK(asw_wta_second(&s.p, s.tkey_g, s.tkey, s.t1, s.t2, s.t2_g, s.stream));
        }
        ASWCHK(allreduce_min<float>(c, b_t2_g, ncclFloat32));
        HIPCHK(hipSetDevice(s0.device));
        ASWCHK(asw_wta_ref_finalize(&s0.p, s0.key_g, s0.tkey_g, s0.t2_g, dr, dt, c->conf_ref, kl, c->code_tar, st));
        ASWCHK(asw_consistency(p, dr, dt, kl, c->code_tar, c->conf_ref, c->conf_tar, c->est, c->post_red, st));
    }
    HIPCHK(hipSetDevice(s0.device));
    return asw_median3(p, c->est, 4, c->final_rgba, st);
}

// The device work of a one-shard frame from uploaded images to the consistency
// images (no events): what asw_set_graph captures into one HIP graph.
int main_work_untimed(asw_ctx *c) {
    const asw_params *p = &c->p;
    const size_t S = frame_pixels(p);
    Shard &s0 = c->sh[0];
    hipStream_t st = s0.stream;
    ASWCHK(shard_aggregate(c, 0, nullptr, nullptr, 1, 3, false));
    ASWCHK(single_wta(c));
    hipLaunchKernelGGL(k_codes_to_rgba, dim3((unsigned)((S + 255) / 256)), dim3(256), 0, st, (long long)S,
                       c->code_ref, reinterpret_cast<uchar4 *>(c->disp));
    HIPCHK(hipGetLastError());
    if (p->lr_check)
        ASWCHK(asw_consistency(p, c->d_ref, c->d_tar, c->code_ref, c->code_tar, c->conf_ref, c->conf_tar, c->lr,
                               c->lr_red, st));
    hipLaunchKernelGGL(k_disp16, dim3((unsigned)((S + 255) / 256)), dim3(256), 0, st, (long long)S, p->ndisp,
                       p->lr_mode, p->lr_check, c->d_ref, c->d_tar, c->code_ref, c->code_tar, c->disp16, c->lr16);
    HIPCHK(hipGetLastError());
    return ASW_OK;
}

int refine_work(asw_ctx *c) {
    const size_t S = frame_pixels(&c->p);
    Shard &s0 = c->sh[0];
    hipStream_t st = s0.stream;
    HIPCHK(hipMemcpyAsync(c->est, c->lr, S * 4, hipMemcpyDeviceToDevice, st));
    if (c->comm == COMM_NONE)
        return asw_refine(&s0.p, &c->rp, s0.left, s0.right, s0.c0, c->est, c->code_tar, c->conf_ref, c->conf_tar,
                          c->rws, c->post_red, c->final_rgba, nullptr, nullptr, st);
    return refine_sharded(c);
}

// capture fn's work on stream st into *g / *gx (once), then launch it
template <class F>
int graph_run(hipStream_t st, hipGraph_t *g, hipGraphExec_t *gx, F &&fn) {
    if (!*gx) {
        HIPCHK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
        const int s = fn();
        hipGraph_t cap = nullptr;
        const hipError_t e = hipStreamEndCapture(st, &cap);
        if (s != ASW_OK || e != hipSuccess) {
            if (cap) (void)hipGraphDestroy(cap);
            return s != ASW_OK ? s : hip_fail(e);
        }
        const hipError_t ei = hipGraphInstantiate(gx, cap, nullptr, nullptr, 0);
        if (ei != hipSuccess) {  // nothing kept: the next call captures afresh
            (void)hipGraphDestroy(cap);
            *gx = nullptr;
            return hip_fail(ei);
        }
        *g = cap;
    }
    HIPCHK(hipGraphLaunch(*gx, st));
    return ASW_OK;
}

int match_one(asw_ctx *c, const uint8_t *left_rgba, const uint8_t *right_rgba, asw_outputs *o, asw_timings *t) {
    const asw_params *p = &c->p;
    const size_t S = frame_pixels(p);
    const int r = p->iters;
    Shard &s0 = c->sh[0];
    hipStream_t st = s0.stream;
    std::vector<hipEvent_t> &ev = c->ev;
    // event slots: 0 h2d start, 1 h2d end = raw start, 2 raw end, 3.. 3+2r pass marks,
    // then exchange end, wta end, consistency end, pre-refinement d2h end, refine end, d2h end
    const int e_pass0 = 3, e_x = e_pass0 + 2 * r + 1, e_wta = e_x + 1, e_cons = e_x + 2, e_pre = e_x + 3,
              e_ref = e_x + 4, e_d2h = e_x + 5;
    const bool graphed = c->graph && c->comm == COMM_NONE;
    HIPCHK(hipSetDevice(s0.device));
    HIPCHK(hipEventRecord(ev[0], st));
    if (graphed) {
        HIPCHK(hipMemcpyAsync(s0.left, left_rgba, S * 4, hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(s0.right, right_rgba, S * 4, hipMemcpyHostToDevice, st));
        HIPCHK(hipEventRecord(ev[1], st));
        ASWCHK(graph_run(st, &c->g_main, &c->gx_main, [&] { return main_work_untimed(c); }));
    } else {
        for (int i = 0; i < c->n; ++i) ASWCHK(shard_aggregate(c, i, left_rgba, right_rgba, 1, e_pass0));
        if (c->comm == COMM_NONE) {
            HIPCHK(hipSetDevice(s0.device));
            HIPCHK(hipEventRecord(ev[e_x], st));
            ASWCHK(single_wta(c));
        } else {
            ASWCHK(sharded_wta(c));
            HIPCHK(hipSetDevice(s0.device));
            HIPCHK(hipEventRecord(ev[e_x], st));
        }
        HIPCHK(hipEventRecord(ev[e_wta], st));
        hipLaunchKernelGGL(k_codes_to_rgba, dim3((unsigned)((S + 255) / 256)), dim3(256), 0, st, (long long)S,
                           c->code_ref, reinterpret_cast<uchar4 *>(c->disp));
        HIPCHK(hipGetLastError());
        if (p->lr_check)
            ASWCHK(asw_consistency(p, c->d_ref, c->d_tar, c->code_ref, c->code_tar, c->conf_ref, c->conf_tar, c->lr,
                                   c->lr_red, st));
        const bool want16 = o && (o->disp16 || o->lr16);
        if (want16) {
            hipLaunchKernelGGL(k_disp16, dim3((unsigned)((S + 255) / 256)), dim3(256), 0, st, (long long)S,
                               p->ndisp, p->lr_mode, p->lr_check, c->d_ref, c->d_tar, c->code_ref, c->code_tar,
                               c->disp16, c->lr16);
            HIPCHK(hipGetLastError());
        }
    }
    HIPCHK(hipEventRecord(ev[e_cons], st));
    // pre-refinement outputs leave before the loop updates its buffers in place
    if (o) {
        if (o->d_ref) HIPCHK(hipMemcpyAsync(o->d_ref, c->d_ref, S * 4, hipMemcpyDeviceToHost, st));
        if (o->d_tar) HIPCHK(hipMemcpyAsync(o->d_tar, c->d_tar, S * 4, hipMemcpyDeviceToHost, st));
        if (o->conf_ref) HIPCHK(hipMemcpyAsync(o->conf_ref, c->conf_ref, S * 4, hipMemcpyDeviceToHost, st));
        if (o->conf_tar) HIPCHK(hipMemcpyAsync(o->conf_tar, c->conf_tar, S * 4, hipMemcpyDeviceToHost, st));
        if (o->disp_rgba) HIPCHK(hipMemcpyAsync(o->disp_rgba, c->disp, S * 4, hipMemcpyDeviceToHost, st));
        if (o->lr_rgba && p->lr_check) HIPCHK(hipMemcpyAsync(o->lr_rgba, c->lr, S * 4, hipMemcpyDeviceToHost, st));
        if (o->lr_red_rgba && p->lr_check)
            HIPCHK(hipMemcpyAsync(o->lr_red_rgba, c->lr_red, S * 4, hipMemcpyDeviceToHost, st));
        if (o->disp16) HIPCHK(hipMemcpyAsync(o->disp16, c->disp16, S * 2, hipMemcpyDeviceToHost, st));
        if (o->lr16 && p->lr_check) HIPCHK(hipMemcpyAsync(o->lr16, c->lr16, S * 2, hipMemcpyDeviceToHost, st));
        if (o->cost) {
            // [H][W][Dp] of the whole range: shard i fills planes [d_begin_i, d_end_i)
            const size_t Dp = (size_t)asw_disp_pitch(p);
            for (int i = 0; i < c->n; ++i) {
                Shard &s = c->sh[i];
                const size_t dps = (size_t)asw_disp_pitch(&s.p), nloc = (size_t)(s.p.d_end - s.p.d_begin);
                HIPCHK(hipSetDevice(s.device));
                HIPCHK(hipMemcpy2DAsync(o->cost + s.p.d_begin, Dp * 4, s.c0, dps * 4, (c->nranks == 1 ? dps : nloc) * 4,
                                        S, hipMemcpyDeviceToHost, s.stream));
                HIPCHK(hipStreamSynchronize(s.stream));
            }
            HIPCHK(hipSetDevice(s0.device));
        }
    }
    HIPCHK(hipEventRecord(ev[e_pre], st));
    const bool refine = c->refine && p->lr_check;
    if (refine) {  // main.cpp:540-617 on a copy of consistency_error
        if (graphed) ASWCHK(graph_run(st, &c->g_ref, &c->gx_ref, [&] { return refine_work(c); }));
        else ASWCHK(refine_work(c));
    }
    HIPCHK(hipEventRecord(ev[e_ref], st));
    if (o && refine) {
        if (o->final_rgba) HIPCHK(hipMemcpyAsync(o->final_rgba, c->final_rgba, S * 4, hipMemcpyDeviceToHost, st));
        if (o->post_red_rgba && c->rp.iters > 0)
            HIPCHK(hipMemcpyAsync(o->post_red_rgba, c->post_red, S * 4, hipMemcpyDeviceToHost, st));
    }
    HIPCHK(hipEventRecord(ev[e_d2h], st));
    HIPCHK(hipStreamSynchronize(st));
    for (int i = 1; i < c->n; ++i) {
        HIPCHK(hipSetDevice(c->sh[i].device));
        HIPCHK(hipStreamSynchronize(c->sh[i].stream));
    }
    HIPCHK(hipSetDevice(s0.device));
    if (t && graphed) {  // one graph: only the coarse spans are measured
        std::memset(t, 0, sizeof(*t));
        t->h2d = ms_between(ev[0], ev[1]);
        t->total = ms_between(ev[1], ev[e_cons]);
        t->refine = refine ? ms_between(ev[e_pre], ev[e_ref]) : 0.0;
        t->d2h = ms_between(ev[e_cons], ev[e_pre]) + ms_between(ev[e_ref], ev[e_d2h]);
    } else if (t) {
        std::memset(t, 0, sizeof(*t));
        t->h2d = ms_between(ev[0], ev[1]);
        t->raw_cost = ms_between(ev[1], ev[2]);
        t->support = ms_between(ev[2], ev[e_pass0]);
        double v = 0.0, h = 0.0;
        for (int it = 0; it < r; ++it) {
            v += ms_between(ev[e_pass0 + 2 * it], ev[e_pass0 + 2 * it + 1]);
            h += ms_between(ev[e_pass0 + 2 * it + 1], ev[e_pass0 + 2 * it + 2]);
        }
        t->v_pass_mean = r ? v / r : 0.0;
        t->h_pass_mean = r ? h / r : 0.0;
        t->aggregation_total = ms_between(ev[e_pass0], ev[e_pass0 + 2 * r]);
        const bool sharded = c->comm != COMM_NONE;
        t->exchange = sharded ? ms_between(ev[e_pass0 + 2 * r], ev[e_x]) : 0.0;
        t->wta = sharded ? t->exchange : ms_between(ev[e_x], ev[e_wta]);
        t->consistency = ms_between(ev[e_wta], ev[e_cons]);
        t->total = ms_between(ev[1], ev[e_cons]);
        t->refine = refine ? ms_between(ev[e_pre], ev[e_ref]) : 0.0;
        t->d2h = ms_between(ev[e_cons], ev[e_pre]) + ms_between(ev[e_ref], ev[e_d2h]);
    }
    return ASW_OK;
}

}  // namespace

extern "C" {

int asw_destroy(asw_ctx *ctx) { return destroy_ctx(ctx); }

int asw_create(const asw_params *p, int hip_device, asw_ctx **out) {
    return create_ctx(p, &hip_device, 1, 0, 1, COMM_NONE, nullptr, out);
}

int asw_create_multi(const asw_params *p, const int *hip_device_ids, int n_devices, asw_ctx **out) {
    if (!out) return ASW_E_INVALID;
    *out = nullptr;
    if (!hip_device_ids || n_devices < 1 || n_devices > kMaxShards) return ASW_E_INVALID;
    CommMode comm = n_devices == 1 ? COMM_NONE : COMM_RCCL;
    for (int i = 0; i < n_devices; ++i)
        for (int j = 0; j < i; ++j)
            if (hip_device_ids[i] == hip_device_ids[j]) comm = COMM_LOCAL;  // RCCL needs one rank per device
    if (n_devices > 1 && p && (p->flags & ASW_FLAG_COMM_LOCAL)) comm = COMM_LOCAL;
    return create_ctx(p, hip_device_ids, n_devices, 0, n_devices, comm, nullptr, out);
}

int asw_comm_unique_id(uint8_t id[ASW_COMM_ID_BYTES]) {
    if (!id) return ASW_E_INVALID;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return ASW_E_COMM;
    static_assert(sizeof(u) == ASW_COMM_ID_BYTES, "ncclUniqueId size");
    std::memcpy(id, &u, sizeof u);
    return ASW_OK;
}

int asw_create_rank(const asw_params *p, int hip_device, int rank, int nranks, const uint8_t id[ASW_COMM_ID_BYTES],
                    asw_ctx **out) {
    if (!out) return ASW_E_INVALID;
    *out = nullptr;
    if (!id || nranks < 1 || rank < 0 || rank >= nranks) return ASW_E_INVALID;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    return create_ctx(p, &hip_device, 1, rank, nranks, COMM_RCCL, &u, out);
}

int asw_ctx_shard(const asw_ctx *ctx, int i, int *n_shards, int *d_begin, int *d_end) {
    if (!ctx) return ASW_E_INVALID;
    if (n_shards) *n_shards = ctx->n;
    if (i < 0 || i >= ctx->n) return ASW_E_INVALID;
    if (d_begin) *d_begin = ctx->sh[i].p.d_begin;
    if (d_end) *d_end = ctx->sh[i].p.d_end;
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
    const size_t S = frame_pixels(&c->p);
    for (int i = 1; i < c->n; ++i) {  // sharded refinement: the estimates of both views on every shard
        Shard &s = c->sh[i];
        HIPCHK(hipSetDevice(s.device));
        if (!s.ref_l) ASWCHK(dev_alloc(&s.ref_l, 2 * S * 4));
        if (!s.ref_r) ASWCHK(dev_alloc(&s.ref_r, 2 * S * 4));
    }
    if (c->n > 1 && !c->red_done) {
        HIPCHK(hipSetDevice(c->sh[0].device));
        HIPCHK(hipEventCreateWithFlags(&c->red_done, hipEventDisableTiming));
    }
    HIPCHK(hipSetDevice(c->sh[0].device));
    const size_t ws = asw_refine_workspace_bytes(&c->p, rp);
    if (c->rws) (void)hipFree(c->rws);
    c->rws = nullptr;
    ASWCHK(dev_alloc(&c->rws, ws));
    if (!c->est) ASWCHK(dev_alloc(&c->est, S * 4));
    if (!c->post_red) ASWCHK(dev_alloc(&c->post_red, S * 4));
    if (!c->final_rgba) ASWCHK(dev_alloc(&c->final_rgba, S * 4));
    c->rp = *rp;
    c->refine = true;
    if (c->gx_ref) {  // the captured loop used the previous workspace / parameters
        (void)hipGraphExecDestroy(c->gx_ref);
        (void)hipGraphDestroy(c->g_ref);
        c->gx_ref = nullptr;
        c->g_ref = nullptr;
    }
    return ASW_OK;
}

int asw_set_graph(asw_ctx *c, int on) {
    if (!c) return ASW_E_INVALID;
    if (on && c->comm != COMM_NONE) return ASW_E_UNSUPPORTED;  // one shard, one stream
    c->graph = on != 0;
    return ASW_OK;
}

int asw_match(asw_ctx *c, const uint8_t *left_rgba, const uint8_t *right_rgba, asw_outputs *o, asw_timings *t) {
    if (!c || !left_rgba || !right_rgba) return ASW_E_INVALID;
    return match_one(c, left_rgba, right_rgba, o, t);
}

int asw_match_batch(asw_ctx *c, const uint8_t *left_rgba, const uint8_t *right_rgba, int batch, asw_outputs *out,
                    asw_timings *t) {
    if (!c || !left_rgba || !right_rgba || batch < 0 || (batch > 0 && !out)) return ASW_E_INVALID;
    const size_t img = frame_pixels(&c->p) * 4;
    for (int b = 0; b < batch; ++b)
        ASWCHK(match_one(c, left_rgba + (size_t)b * img, right_rgba + (size_t)b * img, &out[b], t ? &t[b] : nullptr));
    return ASW_OK;
}

}  // extern "C"
