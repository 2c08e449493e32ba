// Microbenchmark: VALU issue rate of the aggregation tap instruction mix on gfx950.
// Each variant runs ITER x (16 taps) per wave; waves/SIMD set by the launch.
//   mode 0: 3 independent plain VALU ops per tap (v_mul, v_fma, v_add, no deps)
//   mode 1: the tap triple: v_mul_f32_dpp row_newbcast ; v_fmac (num chain) ; v_add (den chain)
//   mode 2: same triple with a plain v_mul (no DPP)
//   mode 3: tap triple, two outputs interleaved (4 chains)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define TAP_DPP(L) \
  "v_mul_f32_dpp v10, v1, v2 row_newbcast:" #L " row_mask:0xf bank_mask:0xf bound_ctrl:1\n" \
  "v_fmac_f32 v20, v10, v3\n" \
  "v_add_f32 v21, v21, v10\n"
#define TAP_PLAIN \
  "v_mul_f32 v10, v1, v2\n" \
  "v_fmac_f32 v20, v10, v3\n" \
  "v_add_f32 v21, v21, v10\n"
#define TAP_INDEP \
  "v_mul_f32 v10, v1, v2\n" \
  "v_fma_f32 v11, v4, v3, v5\n" \
  "v_add_f32 v12, v6, v7\n"
#define TAP_PK \
  "v_pk_mul_f32 v[10:11], s[0:1], v[2:3] op_sel_hi:[0,1]\n" \
  "v_pk_fma_f32 v[20:21], v[10:11], v[4:5], v[20:21]\n" \
  "v_pk_add_f32 v[22:23], v[22:23], v[10:11]\n"
#define TAP_PKV \
  "v_pk_mul_f32 v[10:11], v[6:7], v[2:3]\n" \
  "v_pk_fma_f32 v[20:21], v[10:11], v[4:5], v[20:21]\n" \
  "v_pk_add_f32 v[22:23], v[22:23], v[10:11]\n"
// skewed: ww of tap i+1 is computed before tap i's fmac/add (alternating v10/v11)
#define SKEW_PAIR \
  "v_mul_f32 v11, s1, v2\n" \
  "v_fmac_f32 v20, v10, v3\n" \
  "v_add_f32 v21, v21, v10\n" \
  "v_mul_f32 v10, s0, v2\n" \
  "v_fmac_f32 v20, v11, v3\n" \
  "v_add_f32 v21, v21, v11\n"
// plain tap triple with an SGPR left weight (the kernel's form)
#define TAP_S \
  "v_mul_f32 v10, s0, v2\n" \
  "v_fmac_f32 v20, v10, v3\n" \
  "v_add_f32 v21, v21, v10\n"
#define TAP2(L) \
  "v_mul_f32_dpp v10, v1, v2 row_newbcast:" #L " row_mask:0xf bank_mask:0xf bound_ctrl:1\n" \
  "v_mul_f32_dpp v11, v4, v5 row_newbcast:" #L " row_mask:0xf bank_mask:0xf bound_ctrl:1\n" \
  "v_fmac_f32 v20, v10, v3\n" \
  "v_fmac_f32 v22, v11, v6\n" \
  "v_add_f32 v21, v21, v10\n" \
  "v_add_f32 v23, v23, v11\n"

template <int MODE>
__global__ void k(float* out, int iters) {
  float r = 0.f;
  for (int it = 0; it < iters; ++it) {
    if (MODE == 0) {
      asm volatile(TAP_INDEP TAP_INDEP TAP_INDEP TAP_INDEP TAP_INDEP TAP_INDEP TAP_INDEP TAP_INDEP
                   TAP_INDEP TAP_INDEP TAP_INDEP TAP_INDEP TAP_INDEP TAP_INDEP TAP_INDEP TAP_INDEP
                   ::: "v10","v11","v12","v20","v21");
    } else if (MODE == 1) {
      asm volatile(TAP_DPP(0) TAP_DPP(1) TAP_DPP(2) TAP_DPP(3) TAP_DPP(4) TAP_DPP(5) TAP_DPP(6) TAP_DPP(7)
                   TAP_DPP(8) TAP_DPP(9) TAP_DPP(10) TAP_DPP(11) TAP_DPP(12) TAP_DPP(13) TAP_DPP(14) TAP_DPP(15)
                   ::: "v10","v20","v21");
    } else if (MODE == 2) {
      asm volatile(TAP_PLAIN TAP_PLAIN TAP_PLAIN TAP_PLAIN TAP_PLAIN TAP_PLAIN TAP_PLAIN TAP_PLAIN
                   TAP_PLAIN TAP_PLAIN TAP_PLAIN TAP_PLAIN TAP_PLAIN TAP_PLAIN TAP_PLAIN TAP_PLAIN
                   ::: "v10","v20","v21");
    } else if (MODE == 4) {
      asm volatile("s_mov_b32 s0, 0x3f800000\n s_mov_b32 s1, 0x3f800000\n"
                   TAP_PK TAP_PK TAP_PK TAP_PK TAP_PK TAP_PK TAP_PK TAP_PK
                   TAP_PK TAP_PK TAP_PK TAP_PK TAP_PK TAP_PK TAP_PK TAP_PK
                   ::: "v10","v11","v20","v21","v22","v23","s0","s1");
    } else if (MODE == 5) {
      asm volatile(TAP_PKV TAP_PKV TAP_PKV TAP_PKV TAP_PKV TAP_PKV TAP_PKV TAP_PKV
                   TAP_PKV TAP_PKV TAP_PKV TAP_PKV TAP_PKV TAP_PKV TAP_PKV TAP_PKV
                   ::: "v10","v11","v20","v21","v22","v23");
    } else if (MODE == 6) {
      asm volatile("s_mov_b32 s0, 0x3f800000\n s_mov_b32 s1, 0x3f800000\n v_mul_f32 v10, s0, v2\n"
                   SKEW_PAIR SKEW_PAIR SKEW_PAIR SKEW_PAIR SKEW_PAIR SKEW_PAIR SKEW_PAIR SKEW_PAIR
                   ::: "v10","v11","v20","v21","s0","s1");
    } else if (MODE == 7) {
      asm volatile("s_mov_b32 s0, 0x3f800000\n"
                   TAP_S TAP_S TAP_S TAP_S TAP_S TAP_S TAP_S TAP_S
                   TAP_S TAP_S TAP_S TAP_S TAP_S TAP_S TAP_S TAP_S
                   ::: "v10","v20","v21","s0");
    } else {
      asm volatile(TAP2(0) TAP2(1) TAP2(2) TAP2(3) TAP2(4) TAP2(5) TAP2(6) TAP2(7)
                   ::: "v10","v11","v20","v21","v22","v23");
    }
  }
  if (threadIdx.x == 999999) out[0] = r;
}

template <int MODE>
double run(int waves_per_simd, int iters) {
  int dev; hipGetDevice(&dev);
  hipDeviceProp_t prop; hipGetDeviceProperties(&prop, dev);
  int cus = prop.multiProcessorCount;
  float* out; hipMalloc(&out, 4);
  dim3 block(256);  // 4 waves = one per SIMD
  dim3 grid(cus * waves_per_simd);
  hipLaunchKernelGGL(k<MODE>, grid, block, 0, 0, out, 10);
  hipDeviceSynchronize();
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipEventRecord(a);
  hipLaunchKernelGGL(k<MODE>, grid, block, 0, 0, out, iters);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  double ninst_per_wave = (double)iters * 48.0;
  double waves = (double)grid.x * 4;
  double simds = cus * 4.0;
  double inst_per_simd_per_ns = ninst_per_wave * waves / simds / (ms * 1e6);
  hipFree(out);
  return inst_per_simd_per_ns;  // wave-instructions per ns per SIMD
}

int main() {
  const int iters = 20000;
  const char* names[] = {"indep plain", "tap triple DPP", "tap triple plain", "2 taps DPP interleaved",
                         "packed tap triple (sgpr wl)", "packed tap triple (vgpr wl)",
                         "skewed tap triple (sgpr wl)", "tap triple (sgpr wl)"};
  for (int w : {1, 2, 3, 4, 5, 8}) {
    double r0 = run<0>(w, iters), r1 = run<1>(w, iters), r2 = run<2>(w, iters), r3 = run<3>(w, iters);
    double r4 = run<4>(w, iters), r5 = run<5>(w, iters), r6 = run<6>(w, iters), r7 = run<7>(w, iters);
    double rs[] = {r0, r1, r2, r3, r4, r5, r6, r7};
    for (int m = 0; m < 8; ++m)
      printf("{\"waves_per_simd\": %d, \"mode\": \"%s\", \"wave_inst_per_ns_per_simd\": %.4f, \"cycles_per_inst_at_2.1GHz\": %.3f}\n",
             w, names[m], rs[m], 2.1 / rs[m]);
  }
  return 0;
}
