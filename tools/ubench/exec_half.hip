// Microbenchmark: does a wave64 VALU / LDS instruction whose EXEC covers only one
// 32-lane half cost less than a full one on gfx950 (SIMD-32: a wave64 VALU op issues
// over two passes of 32 lanes)?  The 32-plane shard passes (asw_pass32.h) hold two
// pixels per wave, one per half, so their left weight differs per half; with EXEC
// masks the multiply wl*wr could take each half's weight from an SGPR:
//   [exec = lo] v_mul ww, sA, wr ; [exec = hi] v_mul ww, sB, wr
// instead of reading it per lane from LDS.  That pays only if a half-EXEC op takes
// half the cycles.
//   mode 0: 48 independent v_mul_f32, full EXEC
//   mode 1: the same 48 with EXEC = lanes 0-31
//   mode 2: 24 of them with EXEC = lo then 24 with EXEC = hi (each lane does 24)
//   mode 3: tap form, 8 taps: 8 v_mul (lo, sA), 8 v_mul (hi, sB), 8 v_fmac, 8 v_add
//   mode 4: tap form, 8 taps, the shipped 64-lane shape: v_mul (sgpr), v_fmac, v_add
//   mode 5: 16 ds_read_b128, full EXEC (then lgkmcnt(0))
//   mode 6: 16 ds_read_b128 with EXEC = lanes 0-31
//   mode 7: tap form with an LDS-read VGPR left weight (the shipped 32-plane shape):
//           v_mul ww, vwl, wr ; v_fmac ; v_add  (8 taps; the reads are left out)
// Prints wave-instructions (mode 0-2, 5-6: as issued; 3, 4, 7: taps) per ns per SIMD.
#include <hip/hip_runtime.h>

#include <cstdio>

#define MUL8 "v_mul_f32 v10, s0, v2\n v_mul_f32 v11, s0, v3\n v_mul_f32 v12, s0, v4\n v_mul_f32 v13, s0, v5\n" \
             "v_mul_f32 v14, s0, v6\n v_mul_f32 v15, s0, v7\n v_mul_f32 v16, s0, v8\n v_mul_f32 v17, s0, v9\n"
#define MUL8B "v_mul_f32 v10, s1, v2\n v_mul_f32 v11, s1, v3\n v_mul_f32 v12, s1, v4\n v_mul_f32 v13, s1, v5\n" \
              "v_mul_f32 v14, s1, v6\n v_mul_f32 v15, s1, v7\n v_mul_f32 v16, s1, v8\n v_mul_f32 v17, s1, v9\n"
#define FMA8 "v_fmac_f32 v20, v10, v2\n v_fmac_f32 v20, v11, v3\n v_fmac_f32 v20, v12, v4\n v_fmac_f32 v20, v13, v5\n" \
             "v_fmac_f32 v20, v14, v6\n v_fmac_f32 v20, v15, v7\n v_fmac_f32 v20, v16, v8\n v_fmac_f32 v20, v17, v9\n"
#define ADD8 "v_add_f32 v21, v21, v10\n v_add_f32 v21, v21, v11\n v_add_f32 v21, v21, v12\n v_add_f32 v21, v21, v13\n" \
             "v_add_f32 v21, v21, v14\n v_add_f32 v21, v21, v15\n v_add_f32 v21, v21, v16\n v_add_f32 v21, v21, v17\n"
#define VMUL8 "v_mul_f32 v10, v30, v2\n v_mul_f32 v11, v31, v3\n v_mul_f32 v12, v32, v4\n v_mul_f32 v13, v33, v5\n" \
              "v_mul_f32 v14, v34, v6\n v_mul_f32 v15, v35, v7\n v_mul_f32 v16, v36, v8\n v_mul_f32 v17, v37, v9\n"
#define LO "s_mov_b32 exec_hi, 0\n"
#define HI "s_mov_b32 exec_hi, -1\n s_mov_b32 exec_lo, 0\n"
#define ALL "s_mov_b64 exec, -1\n"
#define RD16 "ds_read_b128 v[40:43], v1\n ds_read_b128 v[44:47], v1 offset:16\n ds_read_b128 v[48:51], v1 offset:32\n" \
             "ds_read_b128 v[52:55], v1 offset:48\n ds_read_b128 v[56:59], v1 offset:64\n ds_read_b128 v[60:63], v1 offset:80\n" \
             "ds_read_b128 v[40:43], v1 offset:96\n ds_read_b128 v[44:47], v1 offset:112\n ds_read_b128 v[48:51], v1 offset:128\n" \
             "ds_read_b128 v[52:55], v1 offset:144\n ds_read_b128 v[56:59], v1 offset:160\n ds_read_b128 v[60:63], v1 offset:176\n" \
             "ds_read_b128 v[40:43], v1 offset:192\n ds_read_b128 v[44:47], v1 offset:208\n ds_read_b128 v[48:51], v1 offset:224\n" \
             "ds_read_b128 v[52:55], v1 offset:240\n s_waitcnt lgkmcnt(0)\n"

#define CLOB "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v20", "v21", "s0", "s1"

template <int MODE>
__global__ __launch_bounds__(256) void k(float *out, int iters) {
    __shared__ float lds[64 * 4 * 17];
    lds[threadIdx.x] = 1.0f;
    __syncthreads();
    const unsigned addr = (threadIdx.x & 63) * 16 * 17 % (64 * 4 * 16);  // conflict-free b128 (odd 16-B stride)
    for (int it = 0; it < iters; ++it) {
        if constexpr (MODE == 0) {
            asm volatile("s_mov_b32 s0, 0x3f800000\n" MUL8 MUL8 MUL8 MUL8 MUL8 MUL8 ::: CLOB);
        } else if constexpr (MODE == 1) {
            asm volatile("s_mov_b32 s0, 0x3f800000\n" LO MUL8 MUL8 MUL8 MUL8 MUL8 MUL8 ALL ::: CLOB);
        } else if constexpr (MODE == 2) {
            asm volatile("s_mov_b32 s0, 0x3f800000\n" LO MUL8 MUL8 MUL8 HI MUL8 MUL8 MUL8 ALL ::: CLOB);
        } else if constexpr (MODE == 3) {
            asm volatile("s_mov_b32 s0, 0x3f800000\n s_mov_b32 s1, 0x3f800000\n" LO MUL8 HI MUL8B ALL FMA8 ADD8 ::: CLOB);
        } else if constexpr (MODE == 4) {
            asm volatile("s_mov_b32 s0, 0x3f800000\n" MUL8 FMA8 ADD8 ::: CLOB);
        } else if constexpr (MODE == 5) {
            asm volatile(RD16 ::"v"(addr) : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50",
                         "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63");
        } else if constexpr (MODE == 6) {
            asm volatile(LO RD16 ALL ::"v"(addr) : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49",
                         "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62",
                         "v63");
        } else {
            asm volatile(VMUL8 FMA8 ADD8 ::: CLOB);
        }
    }
    if (threadIdx.x == 999999) out[0] = lds[3];
}

template <int MODE>
double run(int waves_per_simd, int iters, double ops_per_iter) {
    int dev;
    hipGetDevice(&dev);
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, dev);
    const int cus = prop.multiProcessorCount;
    float *out;
    hipMalloc(&out, 4);
    const dim3 block(256), grid(cus * waves_per_simd);
    hipLaunchKernelGGL(k<MODE>, grid, block, 0, 0, out, 10);
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL(k<MODE>, grid, block, 0, 0, out, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    hipFree(out);
    return ops_per_iter * iters * grid.x * 4.0 / (cus * 4.0) / (ms * 1e6);
}

int main() {
    const int it = 20000;
    for (int w : {1, 2, 4}) {
        std::printf("waves/SIMD %d\n", w);
        std::printf("  0 v_mul full EXEC          %.3f inst/ns/SIMD\n", run<0>(w, it, 48));
        std::printf("  1 v_mul EXEC lo            %.3f inst/ns/SIMD\n", run<1>(w, it, 48));
        std::printf("  2 v_mul 24 lo + 24 hi      %.3f inst/ns/SIMD\n", run<2>(w, it, 48));
        std::printf("  3 tap, wl by EXEC halves   %.3f taps/ns/SIMD\n", run<3>(w, it, 8));
        std::printf("  4 tap, wl sgpr (64 lanes)  %.3f taps/ns/SIMD\n", run<4>(w, it, 8));
        std::printf("  7 tap, wl vgpr (32 planes) %.3f taps/ns/SIMD\n", run<7>(w, it, 8));
        std::printf("  5 ds_read_b128 full EXEC   %.3f inst/ns/SIMD\n", run<5>(w, it / 4, 16));
        std::printf("  6 ds_read_b128 EXEC lo     %.3f inst/ns/SIMD\n", run<6>(w, it / 4, 16));
    }
    return 0;
}
