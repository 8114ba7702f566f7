// scatter_bench.hip -- rate of the exchange unpack's access shape (experiment tool).
//
// k_unpack (gossipprotocol_amd/csrc/gp_xchg.hip) writes each received random-edge
// message, 16 bytes, to rmsg[slot]: M ~ 15.6 M messages per slab and round at
// C5 / W = 8 into an array of ~109 M remote in-edge slots, the slots uniform.
// This measures, on arrays far larger than the Infinity Cache:
//   s16        16-B writes at random 16-B slots (the current unpack)
//   s32        the same messages in 32-B slots, each write a whole aligned
//              32-B sector (16 B of payload + 16 B of padding, two lanes)
//   s32one     the same 32-B slots, but only the 16 payload bytes written
//   s16sorted  16-B writes, slots ascending in runs of 4096
//   s16grpG    16-B writes, messages grouped by slot range (G groups of the
//              array, random order inside a group; a pack that bins messages
//              by destination range), groups in order
//   s16full    16-B writes, all slots ascending
//   r16 / r32  reading the used slots back by gather (the round kernel's
//              remote in-edge reads), 16-B vs 32-B slot stride
// Build: hipcc --offload-arch=gfx950 -O3 -o build/scatter_bench tools/scatter_bench.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e = (x);                                                       \
        if (e != hipSuccess) {                                                    \
            std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
            std::exit(1);                                                         \
        }                                                                         \
    } while (0)

constexpr int TPB = 256;

__global__ __launch_bounds__(TPB) void k_s16(double2* __restrict__ a, const uint32_t* __restrict__ slot, uint32_t m) {
    for (uint32_t k = blockIdx.x * TPB + threadIdx.x; k < m; k += gridDim.x * TPB)
        a[slot[k]] = make_double2((double)k, 1.0);
}

// two lanes per message: lane pair (2q, 2q+1) writes the two halves of the 32-B sector
__global__ __launch_bounds__(TPB) void k_s32(double2* __restrict__ a, const uint32_t* __restrict__ slot, uint32_t m) {
    for (uint32_t t = blockIdx.x * TPB + threadIdx.x; t < 2 * m; t += gridDim.x * TPB) {
        const uint32_t k = t >> 1;
        const uint32_t s = slot[k];
        a[(size_t)s * 2 + (t & 1)] = (t & 1) ? make_double2(0.0, 0.0) : make_double2((double)k, 1.0);
    }
}

__global__ __launch_bounds__(TPB) void k_s32one(double2* __restrict__ a, const uint32_t* __restrict__ slot,
                                                uint32_t m) {
    for (uint32_t k = blockIdx.x * TPB + threadIdx.x; k < m; k += gridDim.x * TPB)
        a[(size_t)slot[k] * 2] = make_double2((double)k, 1.0);
}

template <int STRIDE>
__global__ __launch_bounds__(TPB) void k_r(const double2* __restrict__ a, const uint32_t* __restrict__ slot, uint32_t m,
                                           double* out) {
    double s = 0;
    for (uint32_t k = blockIdx.x * TPB + threadIdx.x; k < m; k += gridDim.x * TPB) {
        const double2 v = a[(size_t)slot[k] * STRIDE];
        s += v.x + v.y;
    }
    if (s == 1.25) out[0] = s;
}

__global__ void k_flush(double2* __restrict__ a, size_t n) {
    for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB)
        a[i] = make_double2(1.0, (double)i);
}

template <typename F>
float timeit(F f) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    f();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms;
}

int main(int argc, char** argv) {
    const uint32_t NS = argc > 1 ? (uint32_t)std::atol(argv[1]) : 109000000u;  // slots
    const uint32_t M = argc > 2 ? (uint32_t)std::atol(argv[2]) : 15600000u;    // messages
    const int grid = 8192;
    double2 *a, *fl;
    double* dout;
    uint32_t *slot, *sorted, *grp64, *grp512, *full;
    CK(hipMalloc(&a, (size_t)NS * 32));
    const size_t NF = (size_t)1 << 26;  // 1 GiB flush buffer
    CK(hipMalloc(&fl, NF * 16));
    CK(hipMalloc(&dout, 256));
    CK(hipMalloc(&slot, (size_t)M * 4));
    CK(hipMalloc(&sorted, (size_t)M * 4));
    CK(hipMalloc(&grp64, (size_t)M * 4));
    CK(hipMalloc(&grp512, (size_t)M * 4));
    CK(hipMalloc(&full, (size_t)M * 4));
    CK(hipMemset(a, 0, (size_t)NS * 32));
    // M distinct uniform slots (a random subset), in random order; and the same sorted in runs of 4096
    std::vector<uint32_t> h(M);
    {
        uint64_t x = 88172645463325252ull;
        std::vector<uint8_t> used(NS, 0);
        for (uint32_t k = 0; k < M;) {
            x ^= x << 13;
            x ^= x >> 7;
            x ^= x << 17;
            const uint32_t s = (uint32_t)(x % NS);
            if (used[s]) continue;
            used[s] = 1;
            h[k++] = s;
        }
    }
    CK(hipMemcpy(slot, h.data(), (size_t)M * 4, hipMemcpyHostToDevice));
    {  // grouped by slot range, random order inside a group (stable partition of the random order)
        for (int G : {64, 512}) {
            std::vector<uint32_t> g2(h);
            const uint64_t span = ((uint64_t)NS + G - 1) / G;
            std::stable_sort(g2.begin(), g2.end(), [&](uint32_t x, uint32_t y) { return x / span < y / span; });
            CK(hipMemcpy(G == 64 ? grp64 : grp512, g2.data(), (size_t)M * 4, hipMemcpyHostToDevice));
        }
        std::vector<uint32_t> f(h);
        std::sort(f.begin(), f.end());
        CK(hipMemcpy(full, f.data(), (size_t)M * 4, hipMemcpyHostToDevice));
    }
    for (uint32_t k = 0; k < M; k += 4096) std::sort(h.begin() + k, h.begin() + std::min<uint32_t>(M, k + 4096));
    CK(hipMemcpy(sorted, h.data(), (size_t)M * 4, hipMemcpyHostToDevice));
    CK(hipDeviceSynchronize());
    auto flush = [&] { hipLaunchKernelGGL(k_flush, dim3(grid), dim3(TPB), 0, 0, fl, NF); };
    std::printf("slots %u messages %u\n", NS, M);
    for (int rep = 0; rep < 3; ++rep) {
        float t;
        flush();
        t = timeit([&] { hipLaunchKernelGGL(k_s16, dim3(grid), dim3(TPB), 0, 0, a, slot, M); });
        std::printf("s16        %.3f ms  %.1f M/ms\n", t, M / t / 1e6);
        flush();
        t = timeit([&] { hipLaunchKernelGGL(k_s32, dim3(grid), dim3(TPB), 0, 0, a, slot, M); });
        std::printf("s32        %.3f ms  %.1f M/ms\n", t, M / t / 1e6);
        flush();
        t = timeit([&] { hipLaunchKernelGGL(k_s32one, dim3(grid), dim3(TPB), 0, 0, a, slot, M); });
        std::printf("s32one     %.3f ms  %.1f M/ms\n", t, M / t / 1e6);
        flush();
        t = timeit([&] { hipLaunchKernelGGL(k_s16, dim3(grid), dim3(TPB), 0, 0, a, sorted, M); });
        std::printf("s16sorted  %.3f ms  %.1f M/ms\n", t, M / t / 1e6);
        flush();
        t = timeit([&] { hipLaunchKernelGGL(k_s16, dim3(grid), dim3(TPB), 0, 0, a, grp64, M); });
        std::printf("s16grp64   %.3f ms  %.1f M/ms\n", t, M / t / 1e6);
        flush();
        t = timeit([&] { hipLaunchKernelGGL(k_s16, dim3(grid), dim3(TPB), 0, 0, a, grp512, M); });
        std::printf("s16grp512  %.3f ms  %.1f M/ms\n", t, M / t / 1e6);
        flush();
        t = timeit([&] { hipLaunchKernelGGL(k_s16, dim3(grid), dim3(TPB), 0, 0, a, full, M); });
        std::printf("s16full    %.3f ms  %.1f M/ms\n", t, M / t / 1e6);
        flush();
        t = timeit([&] { hipLaunchKernelGGL(k_s32, dim3(grid), dim3(TPB), 0, 0, a, sorted, M); });
        std::printf("s32sorted  %.3f ms  %.1f M/ms\n", t, M / t / 1e6);
        flush();
        t = timeit([&] { hipLaunchKernelGGL((k_r<1>), dim3(grid), dim3(TPB), 0, 0, a, sorted, M, dout); });
        std::printf("r16        %.3f ms  %.1f M/ms\n", t, M / t / 1e6);
        flush();
        t = timeit([&] { hipLaunchKernelGGL((k_r<2>), dim3(grid), dim3(TPB), 0, 0, a, sorted, M, dout); });
        std::printf("r32        %.3f ms  %.1f M/ms\n", t, M / t / 1e6);
    }
    CK(hipDeviceSynchronize());
    return 0;
}
