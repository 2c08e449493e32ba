/* asan_check.c — TEST INFRASTRUCTURE ONLY (never part of the product path): runs every
 * oracle entry point on small, ragged shapes so the AddressSanitizer + UBSan build
 * (make -C oracle ASAN=1 -> _ref/asan_check) checks the restatement's indexing:
 * the full match (RGB and CIELab supports, plain and truncated AD, T = 1..9, D up
 * to W), the refinement loop and median, and sharded passes (d0 > 0).  Prints one
 * checksum line per case; a sanitizer report aborts with a non-zero status. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

int oracle_match_ex(const uint8_t *L, const uint8_t *R, int W, int H, int D, int T, int iters, float gamma_c,
                    float gamma_g, int fma_mode, int color_space, float tad_tau, int32_t *d_ref, float *conf_ref,
                    int32_t *d_tar, float *conf_tar, uint8_t *out_rgba, uint8_t *out_red_rgba, float *cost_out);
int oracle_refine(const uint8_t *L, const uint8_t *R, int W, int H, int D, int k, int Tr, int pol, const float *C,
                  const uint8_t *est_left_in, const uint8_t *est_right_in, float *conf_ref, float *conf_tar,
                  uint8_t *post_red_rgba, uint8_t *final_rgba, int32_t *d_ref_out, int32_t *d_tar_out);
void oracle_support(const uint8_t *img, int W, int H, int T, int dir, float gamma_c, float gamma_g, float *out);
void oracle_pass(const float *sL, const float *sR, const float *Cin, float *Cout, int W, int H, int T, int dir,
                 int d0, int d1, int plane_base, int fma_mode);
int oracle_code_u8(int d, int D);
int oracle_set_threads(int n);

static uint64_t st = 0x5EED;
static uint8_t rnd8(void) {
    st = st * 6364136223846793005ULL + 1442695040888963407ULL;
    return (uint8_t)(st >> 56);
}

static int run(int W, int H, int D, int T, int iters, int lab, float tau, int k) {
    const long S = (long)W * H;
    uint8_t *L = malloc(4 * S), *R = malloc(4 * S), *o1 = malloc(4 * S), *o2 = malloc(4 * S);
    uint8_t *post = malloc(4 * S), *fin = malloc(4 * S), *kt = malloc(S);
    int32_t *dr = malloc(4 * S), *dt = malloc(4 * S);
    float *cr = malloc(4 * S), *ct = malloc(4 * S), *C = malloc(sizeof(float) * S * D);
    if (!L || !R || !o1 || !o2 || !post || !fin || !kt || !dr || !dt || !cr || !ct || !C) return 1;
    for (long i = 0; i < 4 * S; ++i) {
        L[i] = rnd8();
        R[i] = rnd8();
    }
    if (oracle_match_ex(L, R, W, H, D, T, iters, 30.91f, 28.21f, 1, lab, tau, dr, cr, dt, ct, o1, o2, C)) return 1;
    unsigned long sum = 0;
    for (long p = 0; p < S; ++p) sum = sum * 31 + (unsigned)dr[p] * 7 + (unsigned)dt[p] + o2[4 * p];
    if (k > 0 && D <= 256) {
        for (long p = 0; p < S; ++p) kt[p] = (uint8_t)oracle_code_u8(dt[p], D);
        uint8_t *est = malloc(S);
        if (!est) return 1;
        for (long p = 0; p < S; ++p) est[p] = o1[4 * p];
        if (oracle_refine(L, R, W, H, D, k, 5, 0, C, est, kt, cr, ct, post, fin, dr, dt)) return 1;
        for (long p = 0; p < S; ++p) sum = sum * 31 + fin[4 * p] + post[4 * p + 1];
        free(est);
    }
    printf("W=%d H=%d D=%d T=%d r=%d lab=%d tau=%g k=%d sum=%lu\n", W, H, D, T, iters, lab, tau, k, sum);
    free(L); free(R); free(o1); free(o2); free(post); free(fin); free(kt);
    free(dr); free(dt); free(cr); free(ct); free(C);
    return 0;
}

/* a d-shard pass [d0, d1) of a V and an H pass (the sharded tests' oracle calls) */
static int shard(int W, int H, int D, int T, int d0, int d1) {
    const long S = (long)W * H;
    uint8_t *img = malloc(4 * S), *img2 = malloc(4 * S);
    float *sl = malloc(sizeof(float) * S * T), *sr = malloc(sizeof(float) * S * T);
    float *cin = malloc(sizeof(float) * S * D), *cout = malloc(sizeof(float) * S * D);
    if (!img || !img2 || !sl || !sr || !cin || !cout) return 1;
    for (long i = 0; i < 4 * S; ++i) {
        img[i] = rnd8();
        img2[i] = rnd8();
    }
    for (long i = 0; i < S * D; ++i) cin[i] = (float)rnd8();
    for (int dir = 0; dir < 2; ++dir) {
        oracle_support(img, W, H, T, dir, 30.91f, 28.21f, sl);
        oracle_support(img2, W, H, T, dir, 30.91f, 28.21f, sr);
        oracle_pass(sl, sr, cin, cout, W, H, T, dir, d0, d1, 0, 1);
    }
    printf("shard W=%d H=%d D=%d [%d,%d) ok\n", W, H, D, d0, d1);
    free(img); free(img2); free(sl); free(sr); free(cin); free(cout);
    return 0;
}

int main(void) {
    oracle_set_threads(2);
    int bad = 0;
    bad |= run(37, 23, 16, 5, 2, 0, 765.0f, 2);
    bad |= run(31, 17, 31, 9, 1, 1, 765.0f, 0);
    bad |= run(19, 29, 7, 1, 3, 0, 40.0f, 1);
    bad |= run(8, 5, 8, 7, 2, 0, 765.0f, 1);
    bad |= run(1, 1, 1, 3, 1, 0, 765.0f, 1);
    bad |= shard(33, 21, 24, 7, 5, 19);
    return bad;
}
