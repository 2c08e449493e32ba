// Microbenchmark: cost of the aggregation step's weight loads in a VALU-dense loop.
// One "step" = 35 taps x (v_mul v,s,v ; v_fmac ; v_add) + 8 VALU, and optionally
//   9 ds_read_b128 (per-lane conflict-free addresses) and/or 4 s_load (x16,x16,x2,x1)
// issued at the start of the step, with s_waitcnt lgkmcnt(0) at the end (one step of
// latency cover) or right after the loads (latency exposed).
#include <hip/hip_runtime.h>
#include <cstdio>

#define TAP(s, v) "v_mul_f32 v10, " s ", " v "\n v_fmac_f32 v20, v10, v3\n v_add_f32 v21, v21, v10\n"
#define T4(s0, s1, s2, s3, va, vb, vc, vd) TAP(s0, va) TAP(s1, vb) TAP(s2, vc) TAP(s3, vd)
#define TAPS                                                    \
  T4("s20", "s21", "s22", "s23", "v64", "v65", "v66", "v67")    \
  T4("s24", "s25", "s26", "s27", "v68", "v69", "v70", "v71")    \
  T4("s28", "s29", "s30", "s31", "v72", "v73", "v74", "v75")    \
  T4("s32", "s33", "s34", "s35", "v76", "v77", "v78", "v79")    \
  T4("s36", "s37", "s38", "s39", "v80", "v81", "v82", "v83")    \
  T4("s40", "s41", "s42", "s43", "v84", "v85", "v86", "v87")    \
  T4("s44", "s45", "s46", "s47", "v88", "v89", "v90", "v91")    \
  T4("s48", "s49", "s50", "s51", "v92", "v93", "v94", "v95")    \
  TAP("s52", "v96") TAP("s53", "v97") TAP("s54", "v98")         \
  "v_add_f32 v22, v20, v21\n v_add_f32 v23, v20, v21\n v_add_f32 v24, v20, v21\n v_add_f32 v25, v20, v21\n" \
  "v_add_f32 v26, v20, v21\n v_add_f32 v27, v20, v21\n v_add_f32 v28, v20, v21\n v_add_f32 v29, v20, v21\n"
// two voxel chains (A: v20/v21, B: v24/v25) interleaved tap by tap, sharing the right weight
#define TAPI(sa, sb, v) "v_mul_f32 v10, " sa ", " v "\n v_mul_f32 v11, " sb ", " v "\n" \
  " v_fmac_f32 v20, v10, v3\n v_fmac_f32 v24, v11, v4\n v_add_f32 v21, v21, v10\n v_add_f32 v25, v25, v11\n"
#define TAPS2 \
  TAPI("s20", "s21", "v64") TAPI("s22", "s23", "v65") TAPI("s24", "s25", "v66") TAPI("s26", "s27", "v67") \
  TAPI("s28", "s29", "v68") TAPI("s30", "s31", "v69") TAPI("s32", "s33", "v70") TAPI("s34", "s35", "v71") \
  TAPI("s36", "s37", "v72") TAPI("s38", "s39", "v73") TAPI("s40", "s41", "v74") TAPI("s42", "s43", "v75") \
  TAPI("s44", "s45", "v76") TAPI("s46", "s47", "v77") TAPI("s48", "s49", "v78") TAPI("s50", "s51", "v79") \
  TAPI("s52", "s53", "v80") TAPI("s20", "s21", "v81") TAPI("s22", "s23", "v82") TAPI("s24", "s25", "v83") \
  TAPI("s26", "s27", "v84") TAPI("s28", "s29", "v85") TAPI("s30", "s31", "v86") TAPI("s32", "s33", "v87") \
  TAPI("s34", "s35", "v88") TAPI("s36", "s37", "v89") TAPI("s38", "s39", "v90") TAPI("s40", "s41", "v91") \
  TAPI("s42", "s43", "v92") TAPI("s44", "s45", "v93") TAPI("s46", "s47", "v94") TAPI("s48", "s49", "v95") \
  TAPI("s50", "s51", "v96") TAPI("s52", "s53", "v97") TAPI("s54", "s20", "v98") \
  "v_add_f32 v22, v20, v21\n v_add_f32 v23, v20, v21\n v_add_f32 v26, v20, v21\n v_add_f32 v27, v20, v21\n" \
  "v_add_f32 v28, v20, v21\n v_add_f32 v29, v20, v21\n v_add_f32 v22, v24, v25\n v_add_f32 v23, v24, v25\n" \
  "v_add_f32 v26, v24, v25\n v_add_f32 v27, v24, v25\n v_add_f32 v28, v24, v25\n v_add_f32 v29, v24, v25\n" \
  "v_add_f32 v22, v24, v25\n v_add_f32 v23, v24, v25\n v_add_f32 v26, v24, v25\n v_add_f32 v27, v24, v25\n"
// kernel-like register pattern: ww in v40 (bank 0), acc v43 (bank 3) / v35 (bank 3),
// window operand stepping through v96, v98, ... (banks 0, 2): fmac reads v40 & v96 -> same bank
#define TAPK(s, w, c) "v_mul_f32 v40, " s ", " w "\n v_fmac_f32 v43, v40, " c "\n v_add_f32 v35, v40, v35\n"
#define TAPSK \
  TAPK("s20", "v64", "v96") TAPK("s21", "v65", "v98") TAPK("s22", "v66", "v100") TAPK("s23", "v67", "v102") \
  TAPK("s24", "v68", "v104") TAPK("s25", "v69", "v106") TAPK("s26", "v70", "v108") TAPK("s27", "v71", "v110") \
  TAPK("s28", "v72", "v112") TAPK("s29", "v73", "v114") TAPK("s30", "v74", "v116") TAPK("s31", "v75", "v118") \
  TAPK("s32", "v76", "v120") TAPK("s33", "v77", "v122") TAPK("s34", "v78", "v124") TAPK("s35", "v79", "v126") \
  TAPK("s36", "v80", "v128") TAPK("s37", "v81", "v130") TAPK("s38", "v82", "v132") TAPK("s39", "v83", "v134") \
  TAPK("s40", "v84", "v136") TAPK("s41", "v85", "v138") TAPK("s42", "v86", "v140") TAPK("s43", "v87", "v142") \
  TAPK("s44", "v88", "v96") TAPK("s45", "v89", "v98") TAPK("s46", "v90", "v100") TAPK("s47", "v91", "v102") \
  TAPK("s48", "v92", "v104") TAPK("s49", "v93", "v106") TAPK("s50", "v94", "v108") TAPK("s51", "v95", "v110") \
  TAPK("s52", "v96", "v112") TAPK("s53", "v97", "v114") TAPK("s54", "v98", "v116") \
  "v_add_f32 v22, v20, v21\n v_add_f32 v23, v20, v21\n v_add_f32 v24, v20, v21\n v_add_f32 v25, v20, v21\n" \
  "v_add_f32 v26, v20, v21\n v_add_f32 v27, v20, v21\n v_add_f32 v28, v20, v21\n v_add_f32 v29, v20, v21\n"
// conflict-free variant of the same: ww in v41 (bank 1), window v96+2k (banks 0/2), acc v43 (3), den v39 (3)
#define TAPF(s, w, c) "v_mul_f32 v41, " s ", " w "\n v_fmac_f32 v43, v41, " c "\n v_add_f32 v39, v41, v39\n"
#define TAPSF \
  TAPF("s20", "v64", "v96") TAPF("s21", "v65", "v98") TAPF("s22", "v66", "v100") TAPF("s23", "v67", "v102") \
  TAPF("s24", "v68", "v104") TAPF("s25", "v69", "v106") TAPF("s26", "v70", "v108") TAPF("s27", "v71", "v110") \
  TAPF("s28", "v72", "v112") TAPF("s29", "v73", "v114") TAPF("s30", "v74", "v116") TAPF("s31", "v75", "v118") \
  TAPF("s32", "v76", "v120") TAPF("s33", "v77", "v122") TAPF("s34", "v78", "v124") TAPF("s35", "v79", "v126") \
  TAPF("s36", "v80", "v128") TAPF("s37", "v81", "v130") TAPF("s38", "v82", "v132") TAPF("s39", "v83", "v134") \
  TAPF("s40", "v84", "v136") TAPF("s41", "v85", "v138") TAPF("s42", "v86", "v140") TAPF("s43", "v87", "v142") \
  TAPF("s44", "v88", "v96") TAPF("s45", "v89", "v98") TAPF("s46", "v90", "v100") TAPF("s47", "v91", "v102") \
  TAPF("s48", "v92", "v104") TAPF("s49", "v93", "v106") TAPF("s50", "v94", "v108") TAPF("s51", "v95", "v110") \
  TAPF("s52", "v96", "v112") TAPF("s53", "v97", "v114") TAPF("s54", "v98", "v116") \
  "v_add_f32 v22, v20, v21\n v_add_f32 v23, v20, v21\n v_add_f32 v24, v20, v21\n v_add_f32 v25, v20, v21\n" \
  "v_add_f32 v26, v20, v21\n v_add_f32 v27, v20, v21\n v_add_f32 v28, v20, v21\n v_add_f32 v29, v20, v21\n"
#define LDS9                                                                                       \
  "ds_read_b128 v[64:67], %0\n ds_read_b128 v[68:71], %0 offset:16\n ds_read_b128 v[72:75], %0 offset:32\n" \
  "ds_read_b128 v[76:79], %0 offset:48\n ds_read_b128 v[80:83], %0 offset:64\n ds_read_b128 v[84:87], %0 offset:80\n" \
  "ds_read_b128 v[88:91], %0 offset:96\n ds_read_b128 v[92:95], %0 offset:112\n ds_read_b96 v[96:98], %0 offset:128\n"
#define SMEM4                                                                                      \
  "s_load_dwordx16 s[20:35], %1, 0x0\n s_load_dwordx16 s[36:51], %1, 0x40\n"                       \
  "s_load_dwordx2 s[52:53], %1, 0x80\n s_load_dword s54, %1, 0x88\n"
#define WAIT "s_waitcnt lgkmcnt(0)\n"
#define CLOB "v10", "v11", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v24", "v25", \
  "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", \
  "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", \
  "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v35", "v39", "v40", "v41", "v43", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127", "v128", "v129", "v130", "v131", "v132", "v133", "v134", "v135", "v136", "v137", "v138", "v139", "v140", "v141", "v142", \
  "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27", "s28", "s29", "s30", "s31", "s32", "s33", \
  "s34", "s35", "s36", "s37", "s38", "s39", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", \
  "s48", "s49", "s50", "s51", "s52", "s53", "s54"

template <int MODE>
__global__ __launch_bounds__(256) void k(const float *g, float *out, int iters) {
  __shared__ float lds[4096];
  for (int i = threadIdx.x; i < 4096; i += blockDim.x) lds[i] = 1.0f;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const unsigned a = (unsigned)(((63 - lane) + 10 * (threadIdx.x >> 6)) * 36 * 4);  // stride 36 floats
  const float *p = g + 36 * (blockIdx.x & 63);
  for (int it = 0; it < iters; ++it) {
    if (MODE == 0) asm volatile(TAPS :: "v"(a), "s"(p) : CLOB);
    if (MODE == 1) asm volatile(LDS9 TAPS WAIT :: "v"(a), "s"(p) : CLOB);
    if (MODE == 2) asm volatile(SMEM4 TAPS WAIT :: "v"(a), "s"(p) : CLOB);
    if (MODE == 3) asm volatile(LDS9 SMEM4 TAPS WAIT :: "v"(a), "s"(p) : CLOB);
    if (MODE == 4) asm volatile(LDS9 SMEM4 WAIT TAPS :: "v"(a), "s"(p) : CLOB);
    if (MODE == 5) asm volatile(LDS9 TAPS WAIT SMEM4 TAPS WAIT :: "v"(a), "s"(p) : CLOB);  // 2 steps: alternate
    if (MODE == 6) asm volatile(TAPS2 :: "v"(a), "s"(p) : CLOB);                            // 2 chains, = 2 steps
    if (MODE == 7) asm volatile(LDS9 SMEM4 TAPS2 WAIT :: "v"(a), "s"(p) : CLOB);
    if (MODE == 8) asm volatile(TAPSK :: "v"(a), "s"(p) : CLOB);
    if (MODE == 9) asm volatile(TAPSF :: "v"(a), "s"(p) : CLOB);
  }
  if (threadIdx.x == 999999) out[0] = 0;
}

template <int MODE>
double run(const float *g, int waves_per_simd, int iters) {
  int dev; (void)hipGetDevice(&dev);
  hipDeviceProp_t prop; (void)hipGetDeviceProperties(&prop, dev);
  const int cus = prop.multiProcessorCount;
  float *out; (void)hipMalloc(&out, 4);
  hipLaunchKernelGGL(k<MODE>, dim3(cus * waves_per_simd), dim3(256), 0, 0, g, out, 10);
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(k<MODE>, dim3(cus * waves_per_simd), dim3(256), 0, 0, g, out, iters);
  (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipFree(out);
  const double steps = (double)iters * (MODE >= 5 && MODE <= 7 ? 2 : 1);
  const double valu = steps * 113.0 * waves_per_simd;  // per SIMD
  return valu / (ms * 1e6);                           // VALU wave-instructions per ns per SIMD
}

int main() {
  float *g; (void)hipMalloc(&g, 1 << 20);
  (void)hipMemset(g, 0, 1 << 20);
  const char *names[] = {"VALU only", "+9 ds_read_b128, wait at end", "+4 s_load, wait at end",
                         "+both, wait at end", "+both, wait right after loads", "alternating LDS / SMEM steps",
                         "2 chains interleaved, VALU only", "2 chains interleaved + both loads per 2 voxels",
                         "kernel register pattern (bank conflicts)", "same, conflict-free registers"};
  for (int w : {1, 2, 4}) {
    double r[10] = {run<0>(g, w, 4000), run<1>(g, w, 4000), run<2>(g, w, 4000), run<3>(g, w, 4000),
                    run<4>(g, w, 4000), run<5>(g, w, 2000), run<6>(g, w, 2000), run<7>(g, w, 2000),
                    run<8>(g, w, 4000), run<9>(g, w, 4000)};
    for (int m = 0; m < 10; ++m)
      printf("{\"waves_per_simd\": %d, \"mode\": \"%s\", \"valu_inst_per_ns_per_simd\": %.4f}\n", w, names[m], r[m]);
  }
  return 0;
}
