// V-pass experiments at the C4 size (1920 x 1080, D = 256, T = 35), den-read mode:
// instantiates k_vpass10 (stereo_matchin_amd/csrc/asw_aggregate_impl.h) with
// different den-ring depths, staging rings, barrier periods, dispatch orders and strip
// counts, checks each against a one-thread-per-voxel reference pass (the FP sequence
// of DESIGN.md §FP policy) bit for bit, and prints the median time of 10 launches.
// Synthetic inputs: cost = integers 0..765, weights = exp(-u) with the centre tap 1.
// Build (from the repo root):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -mllvm -pragma-unroll-threshold=1000000 \
//     -fno-slp-vectorize -Iinclude -Istereo_matchin_amd/csrc -o tools/ubench/vexp tools/ubench/vexp.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "asw_aggregate_impl.h"

namespace asw {
namespace agg {
int g_pass_variant = 0;
}
void note_pass_kernel(int, int, const char *, int, const char *, bool) {}
}  // namespace asw

using namespace asw::agg;

constexpr int W = 1920, H = 1080, D = 256, Dp = 256, T = 35, R = T / 2, TP = asw::tap_pitch(T);

// reference: one thread per voxel, taps in order, num fma-contracted, den added
__global__ void k_ref(const float *wl, const float *wr, const float *cin, float *out, float *den) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long long)W * H * Dp) return;
    const int d = (int)(i % Dp);
    const long long px = i / Dp;
    const int x = (int)(px % W), y = (int)(px / W);
    const int xr = max(x - d, 0);
    float num = 1e-5f, dn = 1e-5f;
    for (int t = 0; t < T; ++t) {
        const int yy = min(max(y + t - R, 0), H - 1);
        const float ww = wl[px * TP + t] * wr[((long long)y * W + xr) * TP + t];
        num = __builtin_fmaf(ww, cin[((long long)yy * W + x) * Dp + d], num);
        dn = dn + ww;
    }
    out[i] = num / dn;
    den[i] = dn;
}

template <class K>
void launch(K kern, int nstrip, const float *wl, const float *wr, const float *cin, float *cout, float *den) {
    constexpr int NW = 16, U = pf9_period(T);
    const int nkb = Dp / 64, nxb = (W + NW - 1) / NW;
    const int rows = ((H + nstrip - 1) / nstrip + U - 1) / U * U;
    nstrip = (H + rows - 1) / rows;
    const int per_xcd = (nxb + 7) / 8;
    const int nblocks = 8 * per_xcd * nkb * nstrip;
    hipLaunchKernelGGL(kern, dim3(nblocks), dim3(NW * 64), 0, 0, wl, wr, cin, cout, den, W, H, Dp, 0, rows, nxb,
                       nstrip, per_xcd);
}

int main() {
    const size_t nv = (size_t)W * H * Dp, ns = (size_t)W * H * TP;
    std::vector<float> hw(ns), hc(nv);
    uint64_t st = 12345;
    auto rnd = [&] {
        st = st * 6364136223846793005ULL + 1442695040888963407ULL;
        return (uint32_t)(st >> 33);
    };
    for (size_t i = 0; i < ns; ++i) hw[i] = (i % TP == R) ? 1.0f : ((i % TP) < T ? std::exp(-(float)(rnd() % 4000) / 500.0f) : 0.0f);
    for (size_t i = 0; i < nv; ++i) hc[i] = (float)(rnd() % 766);
    float *wl, *wr, *cin, *cout, *den, *ref, *refden;
    if (hipMalloc(&wl, ns * 4) || hipMalloc(&wr, ns * 4) || hipMalloc(&cin, nv * 4) || hipMalloc(&cout, nv * 4) ||
        hipMalloc(&den, nv * 4) || hipMalloc(&ref, nv * 4) || hipMalloc(&refden, nv * 4))
        return 1;
    (void)hipMemcpy(wl, hw.data(), ns * 4, hipMemcpyHostToDevice);
    std::rotate(hw.begin(), hw.begin() + TP * 7, hw.end());  // a different right image
    (void)hipMemcpy(wr, hw.data(), ns * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(cin, hc.data(), nv * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_ref, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, 0, wl, wr, cin, ref, refden);
    (void)hipMemcpy(den, refden, nv * 4, hipMemcpyDeviceToDevice);
    (void)hipDeviceSynchronize();
    std::vector<float> a(nv), b(nv);
    (void)hipMemcpy(a.data(), ref, nv * 4, hipMemcpyDeviceToHost);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto run = [&](const char *name, auto kern, int nstrip) {
        (void)hipMemset(cout, 0, nv * 4);
        launch(kern, nstrip, wl, wr, cin, cout, den);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(b.data(), cout, nv * 4, hipMemcpyDeviceToHost);
        const bool ok = std::memcmp(a.data(), b.data(), nv * 4) == 0;
        std::vector<float> ts;
        for (int r = 0; r < 12; ++r) {
            (void)hipEventRecord(e0);
            launch(kern, nstrip, wl, wr, cin, cout, den);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (r >= 2) ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        std::printf("{\"exp\": \"%s\", \"nstrip\": %d, \"ms\": %.4f, \"min\": %.4f, \"exact\": %s}\n", name, nstrip,
                    ts[ts.size() / 2], ts[0], ok ? "true" : "false");
        std::fflush(stdout);
    };
    constexpr int NT = kCPStream;
    for (int ns : {5, 1, 2, 3, 10}) run("base", k_vpass10<T, 16, DM_READ, 2, NT, NT, 2, 4, false>, ns);
    run("kd4", k_vpass10<T, 16, DM_READ, 2, NT, NT, 4, 4, false>, 5);
    run("kbi", k_vpass10<T, 16, DM_READ, 2, NT, NT, 2, 4, true>, 5);
    run("rb4", k_vpass10<T, 16, DM_READ, 4, NT, NT, 2, 5, false>, 5);
    run("rb4_kd4_kbi", k_vpass10<T, 16, DM_READ, 4, NT, NT, 4, 5, true>, 5);
    return 0;
}
