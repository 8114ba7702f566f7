// microbench.hip -- MI355X primitive costs that decide the round-kernel design
// (experiment tool; results recorded in DESIGN.md §5).
//   1. Philox4x32-10 throughput (the per-node draw)
//   2. streaming copy, 16 B / lane (the state stream)
//   3. random 16-B gathers from a 16 GB array (pull: receiver reads sender)
//   4. random 16-B scatters into a 16 GB array (push: sender writes mailbox)
//   5. random 8-B gathers from a 125 MB bitmap-sized array (MALL-resident table)
// Build: hipcc --offload-arch=gfx950 -O3 -o build/microbench tools/microbench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "../gossipprotocol_amd/csrc/gp_device.hpp"

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e = (x);                                                         \
        if (e != hipSuccess) {                                                      \
            std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);   \
            std::exit(1);                                                           \
        }                                                                           \
    } while (0)

__global__ void k_philox(uint32_t n, uint32_t reps, uint32_t* out) {
    uint32_t acc = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        for (uint32_t r = 0; r < reps; ++r) acc += gp::uniform(1u, 2u, 3u, i, r, 7u);
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_copy(const double2* __restrict__ a, double2* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}

// index of the k-th random access: a cheap hash (not Philox) so the index math is negligible
__device__ __forceinline__ uint32_t hidx(uint32_t k, uint32_t n) {
    uint32_t x = k * 0x9E3779B1u;
    x ^= x >> 15;
    x *= 0x85EBCA77u;
    x ^= x >> 13;
    return (uint32_t)(((uint64_t)x * n) >> 32);
}

__global__ void k_gather(const double2* __restrict__ a, double2* __restrict__ out, uint32_t n, uint32_t m) {
    double s = 0, w = 0;
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < m; k += gridDim.x * blockDim.x) {
        const double2 v = a[hidx(k, n)];
        s += v.x;
        w += v.y;
    }
    if (s == 1.2345) out[0] = make_double2(s, w);
}

__global__ void k_scatter(double2* __restrict__ a, uint32_t n, uint32_t m) {
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < m; k += gridDim.x * blockDim.x)
        a[hidx(k, n)] = make_double2((double)k, 1.0);
}

__global__ void k_gather8(const uint64_t* __restrict__ a, uint64_t* out, uint32_t n, uint32_t m) {
    uint64_t acc = 0;
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < m; k += gridDim.x * blockDim.x) acc ^= a[hidx(k, n)];
    if (acc == 0x1234) out[0] = acc;
}

template <typename F>
float timeit(F f, int reps = 5) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) f();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

int main() {
    const uint32_t P = 1000000000u;
    const int grid = 16384, tpb = 256;
    uint32_t* dummy;
    CK(hipMalloc(&dummy, 64));
    {
        const uint32_t reps = 4;
        float ms = timeit([&] { hipLaunchKernelGGL(k_philox, dim3(grid), dim3(tpb), 0, 0, P, reps, dummy); });
        std::printf("philox4x32-10 + U(m): %.3f ms for %.2e draws -> %.3e draws/s\n", ms, (double)P * reps,
                    (double)P * reps / (ms * 1e-3));
    }
    double2 *a, *b;
    CK(hipMalloc(&a, sizeof(double2) * (size_t)P));
    CK(hipMalloc(&b, sizeof(double2) * (size_t)P));
    CK(hipMemset(a, 0, sizeof(double2) * (size_t)P));
    {
        float ms = timeit([&] { hipLaunchKernelGGL(k_copy, dim3(grid), dim3(tpb), 0, 0, a, b, (size_t)P); });
        std::printf("stream copy 16 B/lane: %.3f ms for 2 x 16 GB -> %.0f GB/s\n", ms, 32e9 / (ms * 1e-3) / 1e9 * 1.0);
    }
    const uint32_t m = P / 7;
    {
        float ms = timeit([&] { hipLaunchKernelGGL(k_gather, dim3(grid), dim3(tpb), 0, 0, a, b, P, m); });
        std::printf("random 16-B gather (1e9 x 16 B table): %.3f ms for %u -> %.3e /s (%.0f GB/s payload)\n", ms, m,
                    m / (ms * 1e-3), m * 16.0 / (ms * 1e-3) / 1e9);
    }
    {
        float ms = timeit([&] { hipLaunchKernelGGL(k_scatter, dim3(grid), dim3(tpb), 0, 0, b, P, m); });
        std::printf("random 16-B scatter (1e9 x 16 B table): %.3f ms for %u -> %.3e /s (%.0f GB/s payload)\n", ms, m,
                    m / (ms * 1e-3), m * 16.0 / (ms * 1e-3) / 1e9);
    }
    {
        const uint32_t words = P / 64;
        float ms = timeit([&] {
            hipLaunchKernelGGL(k_gather8, dim3(grid), dim3(tpb), 0, 0, reinterpret_cast<const uint64_t*>(a),
                               reinterpret_cast<uint64_t*>(b), words, P);
        });
        std::printf("random 8-B gather (125 MB table): %.3f ms for %u -> %.3e /s\n", ms, P, P / (ms * 1e-3));
    }
    return 0;
}
