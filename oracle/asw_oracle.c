/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C CPU restatement of the reference's adaptive-support-weight (ASW)
 * hot path (manixq/stereo_matchin, OpenCL kernels under
 * stereo_matching/kernels/, driven by stereo_matching/main.cpp:413-537).
 * It exists to CHECK the HIP product path; it is never linked into, called
 * by, or shipped with the product library.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.
 *
 * Pinning: the reference's own OpenCL sources cannot be built here without
 * writing stand-ins for the OpenCL runtime builtins (read_imagef, get_global_id,
 * ...), which this project does not do.  Instead this restatement is pinned
 * against the reference's committed, device-produced outputs
 * (stereo_matching/<scene>/asw_consistency_pre-reff.png for the five Middlebury
 * scenes, captured as tests/golden/<scene>.npz by tests/golden/make_golden.py) —
 * see tests/test_oracle_golden.py and DESIGN.md §Oracle.
 *
 * Layout: every volume is PLANE-MAJOR like the reference: [plane][y][x], x fastest.
 * Images are row-major RGBA8 (what lodepng::decode hands main.cpp:183-186).
 *
 * Floating point: compiled with -ffp-contract=off; every fused multiply-add
 * is an explicit fmaf() so the operation sequence is fixed (DESIGN.md §FP policy).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "srgb_table.h"
#ifdef _OPENMP
#include <omp.h>
#endif

/* fp policy for the aggregation tap update (DESIGN.md §FP policy):
 *   0: num = num + ww*c ; den = den + ww           (no contraction)
 *   1: num = fma(ww,c,num); den = den + ww          (contract the num update)
 *   2: num = fma(ww,c,num); den = fma(wl,wr,den)    (aggressive contraction) */
#define ORACLE_FMA_NONE 0
#define ORACLE_FMA_NUM 1
#define ORACLE_FMA_ALL 2

static inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

int oracle_version(void) { return 4; }

int oracle_set_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
    return omp_get_max_threads();
#else
    (void)n;
    return 1;
#endif
}

/* K/asw_aggr.cl:12-21 — C0[d][y][x] = (|dR|+|dG|)+|dB| between L(x,y) and
 * R(clamp(x-d), y), read as float(c) (read_imagef(..)*255 == c exactly, and a
 * sum of integers <= 765 is exact in fp32). */
void oracle_raw_cost(const uint8_t *L, const uint8_t *R, int W, int H, int D, float *C) {
    const long S = (long)W * H;
#pragma omp parallel for schedule(static)
    for (int y = 0; y < H; ++y) {
        for (int d = 0; d < D; ++d) {
            float *row = C + (long)d * S + (long)y * W;
            for (int x = 0; x < W; ++x) {
                const uint8_t *lp = L + 4 * ((long)y * W + x);
                const uint8_t *rp = R + 4 * ((long)y * W + (x - d < 0 ? 0 : x - d));
                float r = fabsf((float)lp[0] - (float)rp[0]) + fabsf((float)lp[1] - (float)rp[1]);
                r = r + fabsf((float)lp[2] - (float)rp[2]);
                row[x] = r;
            }
        }
    }
}

/* K/asw_vsupport.cl:19-25 and K/asw_hsupport.cl:19-25:
 *   c_diff = ((-1)*(|dr|+|dg|+|db|)) / gamma_c ; g_dist = distance(p,q) / gamma_g ;
 *   w = exp(c_diff - g_dist)
 * distance() of two integer points on one axis is |delta| exactly.
 * exp is evaluated as (float)exp((double)arg) — correctly rounded in practice;
 * the reference's vendor exp (<= 3 ulp by the OpenCL spec) is unpinned. */
float oracle_support_weight(int sad, int dist, float gamma_c, float gamma_g) {
    float c_diff = (float)(-sad) / gamma_c;
    float g_dist = (float)dist / gamma_g;
    float arg = c_diff - g_dist;
    return (float)exp((double)arg);
}

/* dir 0 = vertical (asw_vSupport), 1 = horizontal (asw_hSupport).
 * out is [T][H][W]; tap i pairs p=(x,y) with q = (x, clamp(y+i-R)) (V) or
 * (clamp(x+i-R), y) (H). */
void oracle_support(const uint8_t *img, int W, int H, int T, int dir, float gamma_c, float gamma_g,
                    float *out) {
    const int Rr = T / 2;
    const long S = (long)W * H;
#pragma omp parallel for schedule(static)
    for (int y = 0; y < H; ++y) {
        for (int i = 0; i < T; ++i) {
            for (int x = 0; x < W; ++x) {
                int qx = x, qy = y;
                if (dir == 0) qy = clampi(y + i - Rr, 0, H - 1);
                else qx = clampi(x + i - Rr, 0, W - 1);
                const uint8_t *p = img + 4 * ((long)y * W + x);
                const uint8_t *q = img + 4 * ((long)qy * W + qx);
                int sad = abs((int)p[0] - q[0]) + abs((int)p[1] - q[1]) + abs((int)p[2] - q[2]);
                int dist = dir == 0 ? abs(y - qy) : abs(x - qx);
                out[(long)i * S + (long)y * W + x] = oracle_support_weight(sad, dist, gamma_c, gamma_g);
            }
        }
    }
}

/* K/asw_vcost_aggregation.cl:23-42 (dir 0) and K/asw_hcost_aggregation.cl:24-43 (dir 1):
 *   xr = max(x-d,0); num = den = 1e-5f;
 *   for i in 0..T-1 (in order): ww = sL[i][y][x]*sR[i][y][xr];
 *       num += ww * Cin[d][q]  (q = (x, clamp(y+i-R)) or (clamp(x+i-R), y)); den += ww;
 *   Cout = num/den.
 * The dead `denom` output of the reference is not produced.
 * Voxels of planes [d0, d1) are computed; Cin/Cout are indexed by absolute plane
 * relative to plane_base (Cin/Cout hold planes [plane_base, plane_base+nplanes)). */
void oracle_pass(const float *sL, const float *sR, const float *Cin, float *Cout, int W, int H, int T,
                 int dir, int d0, int d1, int plane_base, int fma_mode) {
    const int Rr = T / 2;
    const long S = (long)W * H;
    const int nd = d1 - d0;
#pragma omp parallel
    {
        float *num = (float *)malloc(sizeof(float) * W);
        float *den = (float *)malloc(sizeof(float) * W);
#pragma omp for schedule(static) collapse(2)
        for (int dd = 0; dd < nd; ++dd) {
            for (int y = 0; y < H; ++y) {
                const int d = d0 + dd;
                const float *cin = Cin + (long)(d - plane_base) * S;
                float *cout = Cout + (long)(d - plane_base) * S + (long)y * W;
                for (int x = 0; x < W; ++x) { num[x] = 1e-5f; den[x] = 1e-5f; }
                for (int i = 0; i < T; ++i) {
                    const float *wl = sL + (long)i * S + (long)y * W;
                    const float *wr = sR + (long)i * S + (long)y * W;
                    const float *crow;
                    if (dir == 0) crow = cin + (long)clampi(y + i - Rr, 0, H - 1) * W;
                    else crow = cin + (long)y * W;
                    for (int x = 0; x < W; ++x) {
                        const int xr = x - d < 0 ? 0 : x - d;
                        const float a = wl[x];
                        const float b = wr[xr];
                        const float c = dir == 0 ? crow[x] : crow[clampi(x + i - Rr, 0, W - 1)];
                        const float ww = a * b;
                        if (fma_mode == ORACLE_FMA_NONE) {
                            float t = ww * c;
                            num[x] = num[x] + t;
                            den[x] = den[x] + ww;
                        } else if (fma_mode == ORACLE_FMA_NUM) {
                            num[x] = fmaf(ww, c, num[x]);
                            den[x] = den[x] + ww;
                        } else {
                            num[x] = fmaf(ww, c, num[x]);
                            den[x] = fmaf(a, b, den[x]);
                        }
                    }
                }
                for (int x = 0; x < W; ++x) cout[x] = num[x] / den[x];
            }
        }
        free(num);
        free(den);
    }
}

/* One sequential strict-'<' top-2 update (K/asw_wta.cl:43-46):
 *   m2 = t<m2 ? t : m2 ; idx = t<m1 ? d : idx ; m2 = t<m1 ? m1 : m2 ; m1 = t<m1 ? t : m1
 * m1 ends as the first minimum, m2 as the second smallest of the multiset. */
#define TOP2_UPDATE(t, d, m1, m2, idx)           \
    do {                                         \
        float _t = (t);                          \
        (m2) = _t < (m2) ? _t : (m2);            \
        if (_t < (m1)) (idx) = (d);              \
        (m2) = _t < (m1) ? (m1) : (m2);          \
        (m1) = _t < (m1) ? _t : (m1);            \
    } while (0)

/* K/asw_wta.cl:22-80 (asw_WTA + bresenham, :3-9).
 * Left ("reference") map: scan d = 0..D-1.  Right ("target") map: for i in
 * 0..min_d-1, xq = max(0, x-i) and b = bresenham((0,x-min_d),(min_d,x),xq) which
 * is always min_d + xq - x (slope (0-min_d)/((x-min_d)-x) == 1 in integer
 * arithmetic); scan C[b][y][xq] with the same update; min_d_r starts at min_d.
 * conf = (m2 - m1) / m2 (confidence_reference / confidence_target). */
void oracle_wta(const float *C, int W, int H, int D, int32_t *d_ref, float *conf_ref, int32_t *d_tar,
                float *conf_tar) {
    const long S = (long)W * H;
#pragma omp parallel for schedule(static)
    for (int y = 0; y < H; ++y) {
        for (int x = 0; x < W; ++x) {
            const long p = (long)y * W + x;
            float m1 = 100000.0f, m2 = 100000.0f;
            int idx = 0;
            for (int d = 0; d < D; ++d) TOP2_UPDATE(C[(long)d * S + p], d, m1, m2, idx);
            const int md = idx;
            float t1 = 100000.0f, t2 = 100000.0f;
            int mdr = md;
            for (int i = 0; i < md; ++i) {
                const int xq = x - i < 0 ? 0 : x - i;
                const int b = md + xq - x;
                TOP2_UPDATE(C[(long)b * S + (long)y * W + xq], b, t1, t2, mdr);
            }
            d_ref[p] = md;
            conf_ref[p] = (m2 - m1) / m2;
            d_tar[p] = mdr;
            conf_tar[p] = (t2 - t1) / t2;
        }
    }
}

/* UNORM8 code of a disparity index, K/asw_wta.cl:70-74: write_imagef of d/(D-1).
 * Device convention (pinned by the committed PNGs): round half DOWN
 * of 255*d/(D-1), computed exactly in integers: floor((510 d + D - 2) / (2 (D-1))).
 * For D = 61 this is (17 d + 1) >> 2. */
int oracle_code_u8(int d, int D) {
    if (D <= 1) return 0;
    long num = 510L * d + (D - 2);
    long den = 2L * (D - 1);
    long c = num / den;
    return (int)(c > 255 ? 255 : (c < 0 ? 0 : c));
}

/* K/consist.cl:14-33 (Constistency): q = (code/255)*(D-1) per map, consistent iff
 * |qR - qL| < 1.001f.  output_red = consistent ? ref : (255,0,0,255);
 * output = consistent ? ref : tar; confidences zeroed where inconsistent (in place).
 * (c/255)*(D-1)/(D-1) written back as UNORM8 returns c, so outputs are codes. */
void oracle_consistency(const uint8_t *code_ref, const uint8_t *code_tar, float *conf_ref, float *conf_tar,
                        int W, int H, int D, uint8_t *out_rgba, uint8_t *out_red_rgba) {
    const long S = (long)W * H;
    const float scale = (float)(D - 1);
#pragma omp parallel for schedule(static)
    for (long p = 0; p < S; ++p) {
        const float qr = ((float)code_ref[p] / 255.0f) * scale;
        const float qt = ((float)code_tar[p] / 255.0f) * scale;
        const int cons = fabsf(qt - qr) < 1.001f;
        uint8_t *o = out_rgba + 4 * p, *r = out_red_rgba + 4 * p;
        const uint8_t cr = code_ref[p], ct = code_tar[p];
        if (cons) {
            o[0] = o[1] = o[2] = cr;
            r[0] = r[1] = r[2] = cr;
        } else {
            o[0] = o[1] = o[2] = ct;
            r[0] = 255; r[1] = 0; r[2] = 0;
            conf_ref[p] = 0.0f;
            conf_tar[p] = 0.0f;
        }
        o[3] = 255;
        r[3] = 255;
    }
}

/* Truncated AD (north-star extension): min(tau, AD) with the AD of
 * oracle_raw_cost; tau >= 765 is the reference's plain AD. */
void oracle_raw_cost_tad(const uint8_t *L, const uint8_t *R, int W, int H, int D, float tau, float *C) {
    const long S = (long)W * H;
    oracle_raw_cost(L, R, W, H, D, C);
    if (tau >= 765.0f) return;
#pragma omp parallel for schedule(static)
    for (long i = 0; i < S * D; ++i) C[i] = fminf(C[i], tau);
}

/* ---- CIELab extension (north star, no reference counterpart) ----
 * sRGB (D65) 8-bit -> CIE L*a*b*.  Linear light from the shared generated table
 * (srgb_table.h), XYZ by the IEC 61966-2-1 matrix, white (0.95047, 1, 1.08883),
 * f(t) = cbrt(t) above (6/29)^3 else (kappa t + 16)/116, kappa = 24389/27.
 * A fixed sequence of IEEE double operations (no libm): the cube root is 12
 * Newton steps from 1.0, so the HIP kernel reproduces it bit for bit.  Results
 * are rounded to float. */
static double cbrt_newton(double t) {
    double y = 1.0;
    for (int k = 0; k < 12; ++k) y = (2.0 * y + t / (y * y)) / 3.0;
    return y;
}

static double lab_f(double t) {
    const double eps = 216.0 / 24389.0, kappa = 24389.0 / 27.0;
    return t > eps ? cbrt_newton(t) : (kappa * t + 16.0) / 116.0;
}

void oracle_lab(const uint8_t *img, int W, int H, float *lab) {
    const long S = (long)W * H;
#pragma omp parallel for schedule(static)
    for (long p = 0; p < S; ++p) {
        const double r = SRGB_LINEAR[img[4 * p]], g = SRGB_LINEAR[img[4 * p + 1]], b = SRGB_LINEAR[img[4 * p + 2]];
        const double X = (0.4124564 * r + 0.3575761 * g) + 0.1804375 * b;
        const double Y = (0.2126729 * r + 0.7151522 * g) + 0.0721750 * b;
        const double Z = (0.0193339 * r + 0.1191920 * g) + 0.9503041 * b;
        const double fx = lab_f(X / 0.95047), fy = lab_f(Y / 1.0), fz = lab_f(Z / 1.08883);
        lab[4 * p] = (float)(116.0 * fy - 16.0);
        lab[4 * p + 1] = (float)(500.0 * (fx - fy));
        lab[4 * p + 2] = (float)(200.0 * (fy - fz));
        lab[4 * p + 3] = 0.0f;
    }
}

/* Support weights with the colour term on CIELab: the reference formula of
 * K/asw_vsupport.cl:19-25 with the RGB SAD replaced by the Euclidean Lab
 * distance dc = sqrt((dL^2 + da^2) + db^2) (float sums, double sqrt rounded to
 * float = the correctly rounded float sqrt). */
float oracle_support_weight_lab(const float *lp, const float *lq, int dist, float gamma_c, float gamma_g) {
    const float dL = lp[0] - lq[0], da = lp[1] - lq[1], db = lp[2] - lq[2];
    float s = dL * dL + da * da;
    s = s + db * db;
    const float dc = (float)sqrt((double)s);
    const float c_diff = (-dc) / gamma_c;
    const float g_dist = (float)dist / gamma_g;
    return (float)exp((double)(c_diff - g_dist));
}

void oracle_support_lab(const float *lab, int W, int H, int T, int dir, float gamma_c, float gamma_g, float *out) {
    const int Rr = T / 2;
    const long S = (long)W * H;
#pragma omp parallel for schedule(static)
    for (int y = 0; y < H; ++y) {
        for (int i = 0; i < T; ++i) {
            for (int x = 0; x < W; ++x) {
                int qx = x, qy = y;
                if (dir == 0) qy = clampi(y + i - Rr, 0, H - 1);
                else qx = clampi(x + i - Rr, 0, W - 1);
                const int dist = dir == 0 ? abs(y - qy) : abs(x - qx);
                out[(long)i * S + (long)y * W + x] = oracle_support_weight_lab(
                    lab + 4 * ((long)y * W + x), lab + 4 * ((long)qy * W + qx), dist, gamma_c, gamma_g);
            }
        }
    }
}

/* main.cpp:463-537 — raw cost, 4 support launches, r x (V,H), WTA, consistency.
 * Scratch is allocated here.  Outputs may be NULL when not wanted.
 * cost_out (if not NULL) receives the final aggregated volume [D][H][W]. */
int oracle_match_ex(const uint8_t *L, const uint8_t *R, int W, int H, int D, int T, int iters, float gamma_c,
                    float gamma_g, int fma_mode, int color_space, float tad_tau, int32_t *d_ref, float *conf_ref,
                    int32_t *d_tar, float *conf_tar, uint8_t *out_rgba, uint8_t *out_red_rgba, float *cost_out) {
    const long S = (long)W * H;
    float *c0 = (float *)malloc(sizeof(float) * S * D);
    float *c1 = (float *)malloc(sizeof(float) * S * D);
    float *vl = (float *)malloc(sizeof(float) * S * T);
    float *vr = (float *)malloc(sizeof(float) * S * T);
    float *hl = (float *)malloc(sizeof(float) * S * T);
    float *hr = (float *)malloc(sizeof(float) * S * T);
    int32_t *dr = (int32_t *)malloc(sizeof(int32_t) * S);
    int32_t *dt = (int32_t *)malloc(sizeof(int32_t) * S);
    float *cr = (float *)malloc(sizeof(float) * S);
    float *ct = (float *)malloc(sizeof(float) * S);
    uint8_t *kr = (uint8_t *)malloc(S), *kt = (uint8_t *)malloc(S);
    uint8_t *o1 = (uint8_t *)malloc(4 * S), *o2 = (uint8_t *)malloc(4 * S);
    if (!c0 || !c1 || !vl || !vr || !hl || !hr || !dr || !dt || !cr || !ct || !kr || !kt || !o1 || !o2) return -1;
    oracle_raw_cost_tad(L, R, W, H, D, tad_tau, c0);
    if (color_space == 1) {
        float *labL = (float *)malloc(sizeof(float) * 4 * S), *labR = (float *)malloc(sizeof(float) * 4 * S);
        if (!labL || !labR) return -1;
        oracle_lab(L, W, H, labL);
        oracle_lab(R, W, H, labR);
        oracle_support_lab(labL, W, H, T, 0, gamma_c, gamma_g, vl);
        oracle_support_lab(labL, W, H, T, 1, gamma_c, gamma_g, hl);
        oracle_support_lab(labR, W, H, T, 0, gamma_c, gamma_g, vr);
        oracle_support_lab(labR, W, H, T, 1, gamma_c, gamma_g, hr);
        free(labL);
        free(labR);
    } else {
        oracle_support(L, W, H, T, 0, gamma_c, gamma_g, vl);
        oracle_support(L, W, H, T, 1, gamma_c, gamma_g, hl);
        oracle_support(R, W, H, T, 0, gamma_c, gamma_g, vr);
        oracle_support(R, W, H, T, 1, gamma_c, gamma_g, hr);
    }
    for (int it = 0; it < iters; ++it) {
        oracle_pass(vl, vr, c0, c1, W, H, T, 0, 0, D, 0, fma_mode); /* V: c0 -> c1 */
        oracle_pass(hl, hr, c1, c0, W, H, T, 1, 0, D, 0, fma_mode); /* H: c1 -> c0 */
    }
    oracle_wta(c0, W, H, D, dr, cr, dt, ct);
    for (long p = 0; p < S; ++p) {
        kr[p] = (uint8_t)oracle_code_u8(dr[p], D);
        kt[p] = (uint8_t)oracle_code_u8(dt[p], D);
    }
    oracle_consistency(kr, kt, cr, ct, W, H, D, o1, o2);
    if (d_ref) memcpy(d_ref, dr, sizeof(int32_t) * S);
    if (d_tar) memcpy(d_tar, dt, sizeof(int32_t) * S);
    if (conf_ref) memcpy(conf_ref, cr, sizeof(float) * S);
    if (conf_tar) memcpy(conf_tar, ct, sizeof(float) * S);
    if (out_rgba) memcpy(out_rgba, o1, 4 * S);
    if (out_red_rgba) memcpy(out_red_rgba, o2, 4 * S);
    if (cost_out) memcpy(cost_out, c0, sizeof(float) * S * D);
    free(c0); free(c1); free(vl); free(vr); free(hl); free(hr);
    free(dr); free(dt); free(cr); free(ct); free(kr); free(kt); free(o1); free(o2);
    return 0;
}

/* the reference configuration: RGB colour term, plain AD */
int oracle_match(const uint8_t *L, const uint8_t *R, int W, int H, int D, int T, int iters, float gamma_c,
                 float gamma_g, int fma_mode, int32_t *d_ref, float *conf_ref, int32_t *d_tar, float *conf_tar,
                 uint8_t *out_rgba, uint8_t *out_red_rgba, float *cost_out) {
    return oracle_match_ex(L, R, W, H, D, T, iters, gamma_c, gamma_g, fma_mode, 0, 765.0f, d_ref, conf_ref, d_tar,
                           conf_tar, out_rgba, out_red_rgba, cost_out);
}

/* ===================== refinement loop =====================
 * main.cpp:540-623 — k iterations of
 *   asw_ref_v (K/asw_refinement_v.cl:13-51) on (L, est_left, conf_ref) and (R, est_right, conf_tar),
 *   asw_ref_h (K/asw_refinement_h.cl:16-53) on their outputs,
 *   asw_WTA_REF (K/asw_wta_ref.cl:2-68) over the final aggregated volume,
 *   Constistency (K/consist.cl) on the new codes,
 * then the 3x3 Median (K/median.cl:58-88) of the last consistency image.
 * Refinement weight: exp((-SAD)/10.94 - dist/118.78) (K/asw_refinement_v.cl:1-9).
 * est images are read back as D = (code/255)*60 (general D: *(D-1)).
 * Reproduced as written, including asw_WTA_REF storing the TARGET confidence into
 * confidence_reference (its second write, K/asw_wta_ref.cl:64-66) and never
 * writing confidence_target (only Constistency zeroes it), and the target
 * penalty using |ref_target - i| with i the scan index (K/asw_wta_ref.cl:45).
 *
 * Contraction policy `pol` (the vendor compiler's choice is not in the source;
 * tests/test_oracle_golden.py picks the one the device PNGs agree with):
 *   bit 0: V num = fma(w*F, D, num)        else num + (w*F)*D
 *   bit 1: V den = fma(w, F, den)          else den + w*F
 *   bit 2: H num = fma((w*F)*r, n, num)    else num + ((w*F)*r)*n
 *   bit 3: H den = fma(w*F, n, den)        else den + (w*F)*n
 *   bit 4: penalty = fma(0.085*n, |r-i|, c) else (0.085*n)*|r-i| + c          */
#define REF_GC 10.94f
#define REF_GG 118.78f

static float ref_weight(const uint8_t *p, const uint8_t *q, int dist) {
    const int sad = abs((int)p[0] - q[0]) + abs((int)p[1] - q[1]) + abs((int)p[2] - q[2]);
    return oracle_support_weight(sad, dist, REF_GC, REF_GG);
}

/* out[0..S) = num/den, out[S..2S) = den */
static void ref_v(const uint8_t *img, const uint8_t *est, const float *conf, int W, int H, int D, int Tr, int pol,
                  float *out) {
    const long S = (long)W * H;
    const int Rr = Tr / 2;
    const float scale = (float)(D - 1);
#pragma omp parallel for schedule(static)
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const uint8_t *p = img + 4 * ((long)y * W + x);
            float num = 0.00001f, den = 0.00001f;
            for (int i = 0; i < Tr; ++i) {
                const int qy = clampi(y + i - Rr, 0, H - 1);
                const long q = (long)qy * W + x;
                const float w = ref_weight(p, img + 4 * q, abs(y - qy));
                const float Dv = ((float)est[q] / 255.0f) * scale;
                const float F = conf[q];
                const float t = w * F;
                num = (pol & 1) ? fmaf(t, Dv, num) : num + t * Dv;
                den = (pol & 2) ? fmaf(w, F, den) : den + t;
            }
            out[(long)y * W + x] = num / den;
            out[S + (long)y * W + x] = den;
        }
}

static void ref_h(const uint8_t *img, const float *conf, const float *in, int W, int H, int Tr, int pol, float *out) {
    const long S = (long)W * H;
    const int Rr = Tr / 2;
#pragma omp parallel for schedule(static)
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const uint8_t *p = img + 4 * ((long)y * W + x);
            float num = 0.00001f, den = 0.00001f;
            for (int i = 0; i < Tr; ++i) {
                const int qx = clampi(x + i - Rr, 0, W - 1);
                const long q = (long)y * W + qx;
                const float w = ref_weight(p, img + 4 * q, abs(x - qx));
                const float F = conf[q];
                const float r = in[q], n = in[S + q];
                const float t = w * F;
                const float tr = t * r;
                num = (pol & 4) ? fmaf(tr, n, num) : num + tr * n;
                den = (pol & 8) ? fmaf(t, n, den) : den + t * n;
            }
            out[(long)y * W + x] = num / den;
            out[S + (long)y * W + x] = den;
        }
}

static inline float penalty(float n, float r, int i, float c, int pol) {
    const float a = 0.085f * n;
    const float b = fabsf(r - (float)i);
    return (pol & 16) ? fmaf(a, b, c) : a * b + c;
}

/* asw_WTA_REF: codes of min_d / min_d_r; conf_ref <- the target confidence */
static void wta_ref(const float *C, const float *ref, const float *ref_t, int W, int H, int D, int pol,
                    int32_t *d_ref, int32_t *d_tar, float *conf_ref) {
    const long S = (long)W * H;
#pragma omp parallel for schedule(static)
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const long p = (long)y * W + x;
            float cur = 100000.0f, last = 100000.0f;
            int md = 0;
            for (int i = 0; i < D; ++i) {
                const float pen = penalty(ref[S + p], ref[p], i, C[(long)i * S + p], pol);
                last = pen < last ? pen : last;
                md = pen < cur ? i : md;
                last = pen < cur ? cur : last;
                cur = pen < cur ? pen : cur;
            }
            int mdr = md;
            float cur_t = 100000.0f, last_t = 100000.0f;
            for (int i = 0; i < md; ++i) {
                const int xq = x - i < 0 ? 0 : x - i;
                const int b = md + xq - x;
                const float pen = penalty(ref_t[S + p], ref_t[p], i, C[(long)b * S + (long)y * W + xq], pol);
                last_t = pen < last_t ? pen : last_t;
                mdr = pen < cur_t ? b : mdr;
                last_t = pen < cur_t ? cur_t : last_t;
                cur_t = pen < cur_t ? pen : cur_t;
            }
            d_ref[p] = md;
            d_tar[p] = mdr;
            conf_ref[p] = (last_t - cur_t) / last_t;  /* the second (overwriting) write of K/asw_wta_ref.cl */
        }
}

/* 3x3 median of a u8 code image with clamped borders (K/median.cl: the
 * min/max network yields the exact median of the 9 samples per channel). */
static void median3(const uint8_t *in, int W, int H, uint8_t *out) {
#pragma omp parallel for schedule(static)
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            int hist[9], n = 0;
            for (int dy = -1; dy <= 1; ++dy)
                for (int dx = -1; dx <= 1; ++dx) hist[n++] = in[(long)clampi(y + dy, 0, H - 1) * W + clampi(x + dx, 0, W - 1)];
            for (int i = 1; i < 9; ++i)
                for (int j = i; j > 0 && hist[j - 1] > hist[j]; --j) {
                    const int t = hist[j];
                    hist[j] = hist[j - 1];
                    hist[j - 1] = t;
                }
            out[(long)y * W + x] = (uint8_t)hist[4];
        }
}

/* The whole loop.  Inputs: final aggregated volume C [D][H][W], the codes of the
 * pre-refinement consistency image (est_left = cons ? code_ref : code_tar) and of
 * the initial target map (est_right = code_tar), conf_ref / conf_tar after that
 * consistency check (modified in place).  Outputs (any may be NULL):
 * post_red_rgba (asw_consistency_post-reff.png), final_rgba (asw_disparity.png),
 * d_ref / d_tar of the last WTA_REF. */
int oracle_refine(const uint8_t *L, const uint8_t *R, int W, int H, int D, int k, int Tr, int pol, const float *C,
                  const uint8_t *est_left_in, const uint8_t *est_right_in, float *conf_ref, float *conf_tar,
                  uint8_t *post_red_rgba, uint8_t *final_rgba, int32_t *d_ref_out, int32_t *d_tar_out) {
    const long S = (long)W * H;
    float *vl = (float *)malloc(sizeof(float) * 2 * S), *vr = (float *)malloc(sizeof(float) * 2 * S);
    float *hl = (float *)malloc(sizeof(float) * 2 * S), *hr = (float *)malloc(sizeof(float) * 2 * S);
    uint8_t *el = (uint8_t *)malloc(S), *er = (uint8_t *)malloc(S), *kl = (uint8_t *)malloc(S);
    uint8_t *o1 = (uint8_t *)malloc(4 * S), *o2 = (uint8_t *)malloc(4 * S), *fin = (uint8_t *)malloc(S);
    int32_t *dr = (int32_t *)malloc(sizeof(int32_t) * S), *dt = (int32_t *)malloc(sizeof(int32_t) * S);
    if (!vl || !vr || !hl || !hr || !el || !er || !kl || !o1 || !o2 || !fin || !dr || !dt) return -1;
    memcpy(el, est_left_in, S);
    memcpy(er, est_right_in, S);
    memset(o2, 0, 4 * S);
    for (int it = 0; it < k; ++it) {
        ref_v(L, el, conf_ref, W, H, D, Tr, pol, vl);
        ref_v(R, er, conf_tar, W, H, D, Tr, pol, vr);
        ref_h(L, conf_ref, vl, W, H, Tr, pol, hl);
        ref_h(R, conf_tar, vr, W, H, Tr, pol, hr);
        wta_ref(C, hl, hr, W, H, D, pol, dr, dt, conf_ref);
        for (long p = 0; p < S; ++p) {
            kl[p] = (uint8_t)oracle_code_u8(dr[p], D);
            er[p] = (uint8_t)oracle_code_u8(dt[p], D);
        }
        oracle_consistency(kl, er, conf_ref, conf_tar, W, H, D, o1, o2);
        for (long p = 0; p < S; ++p) el[p] = o1[4 * p];
    }
    median3(el, W, H, fin);
    if (post_red_rgba) memcpy(post_red_rgba, o2, 4 * S);
    if (final_rgba)
        for (long p = 0; p < S; ++p) {
            final_rgba[4 * p] = final_rgba[4 * p + 1] = final_rgba[4 * p + 2] = fin[p];
            final_rgba[4 * p + 3] = 255;
        }
    if (d_ref_out) memcpy(d_ref_out, dr, sizeof(int32_t) * S);
    if (d_tar_out) memcpy(d_tar_out, dt, sizeof(int32_t) * S);
    free(vl); free(vr); free(hl); free(hr); free(el); free(er); free(kl); free(o1); free(o2); free(fin);
    free(dr); free(dt);
    return 0;
}
