// Calibration of the rocprofv3 HBM byte counters (FETCH_SIZE / WRITE_SIZE) for the
// access shapes the ASW kernels use, on a known byte count (MI355X_MICROARCH.md
// §HBM: "other access widths are uncalibrated: calibrate on a known byte count").
//
// Each kernel streams a 2 GiB buffer (8x the Infinity Cache) exactly once:
//   k_read_b32    buffer_load_dword, 4 B/lane, 256 B per wave-instruction (the
//                 cost-volume loads of k_vpass9 / k_hpass9 / k_wta_scan)
//   k_read_b128   global_load_dwordx4, 16 B/lane (the guide's calibrated case)
//   k_write_b32   buffer_store_dword, 4 B/lane (the pass output stores)
//   k_write_b128  global_store_dwordx4, 16 B/lane
// Run:  rocprofv3 --pmc FETCH_SIZE -- ./fetch_calib ; rocprofv3 --pmc WRITE_SIZE -- ./fetch_calib
// counter_KB * 1024 / 2 GiB = the factor the counter reads for that shape.
#include <hip/hip_runtime.h>

#include <cstdio>

using rsrc_t = __amdgpu_buffer_rsrc_t;

__global__ void k_read_b32(const float *p, long long n, float *sink) {
    // one wave = 256 contiguous bytes per iteration, grid-stride over 64-float rows
    const rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(p), 0, 0x7fffffff, 0x00020000);
    float acc = 0.0f;
    const long long rows = n / 64;
    const int lane = threadIdx.x & 63;
    const long long wave = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const long long nw = ((long long)gridDim.x * blockDim.x) >> 6;
    // rebase the resource every 2^29 bytes (32-bit offsets)
    for (long long row = wave; row < rows; row += nw) {
        const long long byte = row * 256;
        const rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(reinterpret_cast<const char *>(p)) +
                                                                 (byte & ~((1LL << 29) - 1)),
                                                             0, 0x7fffffff, 0x00020000);
        acc += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rr, lane * 4, (int)(byte & ((1LL << 29) - 1)), 0));
    }
    (void)r;
    if (acc == -1.0f) sink[threadIdx.x] = acc;  // never true (buffer is zero): keeps the loads
}

__global__ void k_read_b128(const float4 *p, long long n4, float *sink) {
    float acc = 0.0f;
    const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long nt = (long long)gridDim.x * blockDim.x;
    for (long long i = tid; i < n4; i += nt) {
        const float4 v = p[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == -1.0f) sink[threadIdx.x] = acc;
}

__global__ void k_write_b32(float *p, long long n) {
    const int lane = threadIdx.x & 63;
    const long long wave = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const long long nw = ((long long)gridDim.x * blockDim.x) >> 6;
    const long long rows = n / 64;
    for (long long row = wave; row < rows; row += nw) {
        const long long byte = row * 256;
        const rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<char *>(p) + (byte & ~((1LL << 29) - 1)), 0,
                                                            0x7fffffff, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b32(0u, rr, lane * 4, (int)(byte & ((1LL << 29) - 1)), 0);
    }
}

__global__ void k_write_b128(float4 *p, long long n4) {
    const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long nt = (long long)gridDim.x * blockDim.x;
    for (long long i = tid; i < n4; i += nt) p[i] = make_float4(0.f, 0.f, 0.f, 0.f);
}

#define CHK(x)                                                                             \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) {                                                             \
            std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e));             \
            return 1;                                                                      \
        }                                                                                  \
    } while (0)

int main() {
    const long long bytes = 2LL << 30;
    const long long n = bytes / 4;
    float *a = nullptr, *b = nullptr, *sink = nullptr;
    CHK(hipMalloc(&a, bytes));
    CHK(hipMalloc(&b, bytes));
    CHK(hipMalloc(&sink, 4096));
    CHK(hipMemset(a, 0, bytes));
    CHK(hipMemset(b, 0, bytes));
    const dim3 grid(256 * 16), block(256);
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    auto report = [&](const char *name) {
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        std::printf("{\"kernel\": \"%s\", \"bytes\": %lld, \"ms\": %.4f, \"GBps\": %.1f}\n", name, bytes, ms,
                    bytes / (ms * 1e6));
    };
    // each kernel runs after the other buffer was streamed, so `a` is not cache-resident
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_write_b128, grid, block, 0, 0, reinterpret_cast<float4 *>(b), n / 4);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    report("k_write_b128");
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_read_b32, grid, block, 0, 0, a, n, sink);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    report("k_read_b32");
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_write_b32, grid, block, 0, 0, b, n);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    report("k_write_b32");
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_read_b128, grid, block, 0, 0, reinterpret_cast<const float4 *>(a), n / 4, sink);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    report("k_read_b128");
    CHK(hipGetLastError());
    CHK(hipFree(a));
    CHK(hipFree(b));
    CHK(hipFree(sink));
    return 0;
}
