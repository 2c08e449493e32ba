// Microbenchmark: the aggregation inner-loop mixes, per 4 taps:
//   mode 0 "sgpr wl": 1 ds_read_b128 (per-lane wr, conflict-free stride) + 4 x (v_mul v,s,v ; v_fmac ; v_add)
//   mode 1 "lds bcast wl": mode 0 + 1 ds_read_b128 from a wave-uniform address (wl) and v_mul v,v,v
//   mode 2 "lds only b128 per-lane": 1 ds_read_b128 per-lane, no VALU  (LDS rate)
//   mode 3 "lds only b128 uniform": 1 ds_read_b128 uniform, no VALU
// 9 groups of 4 taps (36 taps) per iteration.  Reports taps per ns per CU.
#include <hip/hip_runtime.h>
#include <cstdio>

#define WAIT "s_waitcnt lgkmcnt(0)\n"
#define G0 "ds_read_b128 v[40:43], v30 offset:0\n" WAIT \
  "v_mul_f32 v10, s4, v40\n v_fmac_f32 v20, v10, v3\n v_add_f32 v21, v21, v10\n" \
  "v_mul_f32 v10, s5, v41\n v_fmac_f32 v20, v10, v4\n v_add_f32 v21, v21, v10\n" \
  "v_mul_f32 v10, s6, v42\n v_fmac_f32 v20, v10, v5\n v_add_f32 v21, v21, v10\n" \
  "v_mul_f32 v10, s7, v43\n v_fmac_f32 v20, v10, v6\n v_add_f32 v21, v21, v10\n"
#define G1 "ds_read_b128 v[40:43], v30 offset:0\n ds_read_b128 v[44:47], v31 offset:0\n" WAIT \
  "v_mul_f32 v10, v44, v40\n v_fmac_f32 v20, v10, v3\n v_add_f32 v21, v21, v10\n" \
  "v_mul_f32 v10, v45, v41\n v_fmac_f32 v20, v10, v4\n v_add_f32 v21, v21, v10\n" \
  "v_mul_f32 v10, v46, v42\n v_fmac_f32 v20, v10, v5\n v_add_f32 v21, v21, v10\n" \
  "v_mul_f32 v10, v47, v43\n v_fmac_f32 v20, v10, v6\n v_add_f32 v21, v21, v10\n"
#define G2 "ds_read_b128 v[40:43], v30 offset:0\n"
#define G3 "ds_read_b128 v[40:43], v31 offset:0\n"
#define X9(g) g g g g g g g g g

template <int MODE>
__global__ void k(float* out, int iters) {
  __shared__ float4 lds[4096];
  int t = threadIdx.x;
  for (int i = t; i < 4096; i += blockDim.x) lds[i] = make_float4(1, 1, 1, 1);
  __syncthreads();
  int lane = t & 63;
  unsigned a_lane = ((63 - lane) * 9) * 16;      // per-lane entry, stride 36 floats
  unsigned a_unif = (2000 + (t >> 6) * 9) * 16;  // wave-uniform entry
  for (int it = 0; it < iters; ++it) {
    if (MODE == 0) asm volatile(X9(G0) :: "v"(a_lane), "v"(a_unif) : "v10","v20","v21","v40","v41","v42","v43");
    else if (MODE == 1) asm volatile(X9(G1) :: "v"(a_lane), "v"(a_unif) : "v10","v20","v21","v40","v41","v42","v43","v44","v45","v46","v47");
    else if (MODE == 2) asm volatile(X9(G2) WAIT :: "v"(a_lane), "v"(a_unif) : "v40","v41","v42","v43");
    else asm volatile(X9(G3) WAIT :: "v"(a_lane), "v"(a_unif) : "v40","v41","v42","v43");
  }
  if (t == 999999) out[0] = 0;
}

template <int MODE>
double run(int waves_per_cu, int iters) {
  int dev; (void)hipGetDevice(&dev);
  hipDeviceProp_t prop; (void)hipGetDeviceProperties(&prop, dev);
  int cus = prop.multiProcessorCount;
  float* out; (void)hipMalloc(&out, 4);
  dim3 block(64 * waves_per_cu);
  dim3 grid(cus);
  hipLaunchKernelGGL(k<MODE>, grid, block, 0, 0, out, 10);
  (void)hipDeviceSynchronize();
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  (void)hipEventRecord(a);
  hipLaunchKernelGGL(k<MODE>, grid, block, 0, 0, out, iters);
  (void)hipEventRecord(b); (void)hipEventSynchronize(b);
  float ms; (void)hipEventElapsedTime(&ms, a, b);
  double taps = (double)iters * 36 * 64 * waves_per_cu;  // lane-taps per CU
  (void)hipFree(out);
  return taps / (ms * 1e6);  // lane-taps per ns per CU
}

int main() {
  const int iters = 4000;
  const char* names[] = {"sgpr wl + lds wr", "lds bcast wl + lds wr", "lds b128 per-lane only", "lds b128 uniform only"};
  for (int w : {4, 8, 16}) {
    double r[4] = {run<0>(w, iters), run<1>(w, iters), run<2>(w, iters), run<3>(w, iters)};
    for (int m = 0; m < 4; ++m)
      printf("{\"waves_per_cu\": %d, \"mode\": \"%s\", \"lane_taps_per_ns_per_cu\": %.2f}\n", w, names[m], r[m]);
  }
  return 0;
}
