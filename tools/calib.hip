// calib.hip -- FETCH_SIZE / WRITE_SIZE calibration for the access shapes of the
// push-sum tile kernel (experiment tool; the factors land in
// profiles/r02/calib/ and bench.py uses them to turn the round kernel's raw
// counters into HBM bytes).
//
// Each kernel moves a known number of bytes with ONE access shape, over
// buffers far larger than the 256 MiB Infinity Cache, so every byte comes from
// HBM once.  Run it under separate rocprofv3 passes:
//   rocprofv3 --pmc FETCH_SIZE -- build/calib     (and --pmc WRITE_SIZE)
// and divide the per-dispatch counter by the bytes printed here
// (tools/calib_summary.py).
//
// Shapes (as the tile kernel issues them, gp_round.hip):
//   rd16       16 B per lane, lane-contiguous global_load_dwordx4 (own (s, w))
//   rd16_nt    the same, non-temporal
//   rd4_nt     4 B per lane, non-temporal global_load_dword (in-list senders)
//   dma16      LDS-DMA global_load_lds_dwordx4, 1 KiB per wave-instruction
//              (node bytes, x-plane segments)
//   dma16_nt   the same, non-temporal (in-list offsets)
//   gat16_line random 16-B gathers into registers, one per distinct 128-B line
//              (lattice neighbours that miss L2)
//   gatdma_nt_line  random 16-B gathers by LDS-DMA, non-temporal, one per
//              distinct line (random-edge messages)
//   gat16, gatdma_nt  the same with the random-edge statistics: 1/7 of the
//              rows of a 16 GB table, uniformly (some lines twice)
//   st16_nt    16 B per lane non-temporal stores (next-round (s, w))
//   st4_nt     4 B per lane non-temporal stores (node bytes as words)
// Build: hipcc --offload-arch=gfx950 -O3 -o build/calib tools/calib.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e = (x);                                                       \
        if (e != hipSuccess) {                                                    \
            std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
            std::exit(1);                                                         \
        }                                                                         \
    } while (0)

typedef __attribute__((address_space(1))) void gvoid_t;
typedef __attribute__((address_space(3))) void lvoid_t;

constexpr int TPB = 256;

__global__ __launch_bounds__(TPB) void k_rd16(const double2* __restrict__ a, size_t n, double* out) {
    double s = 0;
    for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB) {
        const double2 v = a[i];
        s += v.x + v.y;
    }
    if (s == 1.25) out[0] = s;
}

__global__ __launch_bounds__(TPB) void k_rd16_nt(const double2* __restrict__ a, size_t n, double* out) {
    double s = 0;
    for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB)
        s += __builtin_nontemporal_load(&a[i].x) + __builtin_nontemporal_load(&a[i].y);
    if (s == 1.25) out[0] = s;
}

__global__ __launch_bounds__(TPB) void k_rd4_nt(const uint32_t* __restrict__ a, size_t n, uint32_t* out) {
    uint32_t s = 0;
    for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB)
        s ^= __builtin_nontemporal_load(a + i);
    if (s == 0x12345u) out[0] = s;
}

// LDS-DMA of consecutive 4 KiB pieces (one per block per step, 1 KiB per wave)
template <int AUX>
__global__ __launch_bounds__(TPB) void k_dma16(const char* __restrict__ a, size_t nbytes, uint32_t* out) {
    __shared__ uint32_t lds[1024];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    for (size_t c = (size_t)blockIdx.x * 4096; c < nbytes; c += (size_t)gridDim.x * 4096) {
        const size_t o = c + wv * 1024 + lane * 16;
        if (o < nbytes)
            __builtin_amdgcn_global_load_lds((gvoid_t*)(a + o), (lvoid_t*)(lds + wv * 256), 16, 0, AUX);
        __syncthreads();
    }
    if (lds[threadIdx.x] == 0x12345u) out[0] = 1;
}

__device__ __forceinline__ uint32_t hidx(uint32_t k, uint32_t n) {
    uint32_t x = k * 0x9E3779B1u;
    x ^= x >> 15;
    x *= 0x85EBCA77u;
    x ^= x >> 13;
    return (uint32_t)(((uint64_t)x * n) >> 32);
}

// LINES: the k-th gather reads row 8 * ((k * odd) mod 2^27), one per distinct
// 128-B line (a bijection), so the bytes fetched are known exactly; otherwise
// rows hidx(k, n), the random-edge statistics (some lines hit more than once)
template <bool LINES>
__device__ __forceinline__ uint32_t gidx(uint32_t k, uint32_t n) {
    return LINES ? ((k * 0x9E3779B1u) & ((1u << 27) - 1u)) * 8u : hidx(k, n);
}

template <bool LINES>
__global__ __launch_bounds__(TPB) void k_gat16(const double2* __restrict__ a, uint32_t n, uint32_t m, double* out) {
    double s = 0;
    for (uint32_t k = blockIdx.x * TPB + threadIdx.x; k < m; k += gridDim.x * TPB) {
        const double2 v = a[gidx<LINES>(k, n)];
        s += v.x + v.y;
    }
    if (s == 1.25) out[0] = s;
}

template <bool LINES>
__global__ __launch_bounds__(TPB) void k_gatdma_nt(const double2* __restrict__ a, uint32_t n, uint32_t m, uint32_t* out) {
    __shared__ double2 lds[TPB];
    const uint32_t wv = threadIdx.x >> 6;
    for (uint32_t k0 = blockIdx.x * TPB; k0 < m; k0 += gridDim.x * TPB) {
        const uint32_t k = k0 + threadIdx.x;
        if (k < m) __builtin_amdgcn_global_load_lds((gvoid_t*)(a + gidx<LINES>(k, n)), (lvoid_t*)(lds + wv * 64), 16, 0, 2);
        __syncthreads();
    }
    if (lds[threadIdx.x].x == 1.25) out[0] = 1;
}

// random 16-B gathers by LDS-DMA, one per distinct line, with cache-policy bits
// AUX (bit 0 sc0, bit 1 nt, bit 4 sc1): which policy fetches less than a line
template <int AUX>
__global__ __launch_bounds__(TPB) void k_gatdma_aux(const double2* __restrict__ a, uint32_t m, uint32_t* out) {
    __shared__ double2 lds[TPB];
    const uint32_t wv = threadIdx.x >> 6;
    for (uint32_t k0 = blockIdx.x * TPB; k0 < m; k0 += gridDim.x * TPB) {
        const uint32_t k = k0 + threadIdx.x;
        if (k < m) __builtin_amdgcn_global_load_lds((gvoid_t*)(a + gidx<true>(k, 0)), (lvoid_t*)(lds + wv * 64), 16, 0, AUX);
        __syncthreads();
    }
    if (lds[threadIdx.x].x == 1.25) out[0] = 1;
}

// uncached memory (hipDeviceMallocUncached): random 16-B reads into registers
// and sparse 16-B stores (one row in every 8th line, i.e. partial lines)
// (m must be a power of two: row 8 * ((k * odd) mod m) of a buffer of 8 m rows)
__global__ __launch_bounds__(TPB) void k_gat16_uc(const double2* __restrict__ a, uint32_t m, double* out) {
    double s = 0;
    for (uint32_t k = blockIdx.x * TPB + threadIdx.x; k < m; k += gridDim.x * TPB) {
        const double2 v = a[(size_t)((k * 0x9E3779B1u) & (m - 1u)) * 8u];
        s += v.x + v.y;
    }
    if (s == 1.25) out[0] = s;
}

__global__ __launch_bounds__(TPB) void k_sc16_uc(double2* __restrict__ a, uint32_t m) {
    for (uint32_t k = blockIdx.x * TPB + threadIdx.x; k < m; k += gridDim.x * TPB)
        a[(size_t)k * 8] = make_double2((double)k, 1.0);
}

// the same sparse 16-B stores into ordinary (cached) memory
__global__ __launch_bounds__(TPB) void k_sc16(double2* __restrict__ a, uint32_t m) {
    for (uint32_t k = blockIdx.x * TPB + threadIdx.x; k < m; k += gridDim.x * TPB)
        a[(size_t)k * 8] = make_double2((double)k, 1.0);
}

__global__ __launch_bounds__(TPB) void k_st16_nt(double2* __restrict__ a, size_t n) {
    for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB) {
        __builtin_nontemporal_store((double)i, &a[i].x);
        __builtin_nontemporal_store(1.0, &a[i].y);
    }
}

__global__ __launch_bounds__(TPB) void k_st4_nt(uint32_t* __restrict__ a, size_t n) {
    for (size_t i = blockIdx.x * (size_t)TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB)
        __builtin_nontemporal_store((uint32_t)i, a + i);
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

int main() {
    const size_t N16 = 1ull << 30;  // 16 GiB of 16-B rows
    const int grid = 16384;
    double2* a;
    double2* b;
    double* dout;
    CK(hipMalloc(&a, N16 * 16));
    CK(hipMalloc(&b, N16 * 16));
    CK(hipMalloc(&dout, 256));
    CK(hipMemset(a, 0, N16 * 16));
    CK(hipMemset(b, 0, N16 * 16));
    CK(hipDeviceSynchronize());
    const uint32_t M = (uint32_t)(N16 / 7);  // gathers: 1/7 of the rows, as the random-edge messages
    // one line per shape: name, algorithmic bytes read, bytes written, ms
    auto line = [](const char* name, double rd, double wr, float ms) {
        std::printf("%-10s read_bytes %.0f write_bytes %.0f ms %.3f GBps %.0f\n", name, rd, wr, ms,
                    (rd + wr) / (ms * 1e-3) / 1e9);
    };
    // touch b between shapes so no shape finds the previous one's lines in the Infinity Cache
    auto flush = [&] { hipLaunchKernelGGL(k_st16_nt, dim3(grid), dim3(TPB), 0, 0, b, (size_t)(1u << 26)); };
    flush();
    line("rd16", N16 * 16.0, 0,
         timeit([&] { hipLaunchKernelGGL(k_rd16, dim3(grid), dim3(TPB), 0, 0, a, N16, dout); }));
    flush();
    line("rd16_nt", N16 * 16.0, 0,
         timeit([&] { hipLaunchKernelGGL(k_rd16_nt, dim3(grid), dim3(TPB), 0, 0, a, N16, dout); }));
    flush();
    line("rd4_nt", N16 * 16.0, 0, timeit([&] {
             hipLaunchKernelGGL(k_rd4_nt, dim3(grid), dim3(TPB), 0, 0, reinterpret_cast<const uint32_t*>(a), N16 * 4,
                                reinterpret_cast<uint32_t*>(dout));
         }));
    flush();
    line("dma16", N16 * 16.0, 0, timeit([&] {
             hipLaunchKernelGGL((k_dma16<0>), dim3(grid), dim3(TPB), 0, 0, reinterpret_cast<const char*>(a), N16 * 16,
                                reinterpret_cast<uint32_t*>(dout));
         }));
    flush();
    line("dma16_nt", N16 * 16.0, 0, timeit([&] {
             hipLaunchKernelGGL((k_dma16<2>), dim3(grid), dim3(TPB), 0, 0, reinterpret_cast<const char*>(a), N16 * 16,
                                reinterpret_cast<uint32_t*>(dout));
         }));
    const uint32_t ML = 1u << 24;  // distinct-line gathers: one row in each of 2^24 of the 2^27 lines
    flush();
    line("gat16_line", ML * 16.0, 0, timeit([&] {
             hipLaunchKernelGGL((k_gat16<true>), dim3(grid), dim3(TPB), 0, 0, a, (uint32_t)N16, ML, dout);
         }));
    flush();
    line("gatdma_nt_line", ML * 16.0, 0, timeit([&] {
             hipLaunchKernelGGL((k_gatdma_nt<true>), dim3(grid), dim3(TPB), 0, 0, a, (uint32_t)N16, ML,
                                reinterpret_cast<uint32_t*>(dout));
         }));
    flush();
    line("gat16", M * 16.0, 0, timeit([&] {
             hipLaunchKernelGGL((k_gat16<false>), dim3(grid), dim3(TPB), 0, 0, a, (uint32_t)N16, M, dout);
         }));
    flush();
    line("gatdma_nt", M * 16.0, 0, timeit([&] {
             hipLaunchKernelGGL((k_gatdma_nt<false>), dim3(grid), dim3(TPB), 0, 0, a, (uint32_t)N16, M,
                                reinterpret_cast<uint32_t*>(dout));
         }));
#define AUXCASE(X)                                                                                       \
    flush();                                                                                             \
    line("gatdma_aux" #X, ML * 16.0, 0, timeit([&] {                                                     \
             hipLaunchKernelGGL((k_gatdma_aux<X>), dim3(grid), dim3(TPB), 0, 0, a, ML,                   \
                                reinterpret_cast<uint32_t*>(dout));                                      \
         }));
    AUXCASE(0)
    AUXCASE(1)
    AUXCASE(3)
    AUXCASE(16)
    AUXCASE(17)
    AUXCASE(19)
    {
        double2* uc;
        CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&uc), (size_t)ML * 8 * 16, hipDeviceMallocUncached));
        CK(hipMemset(uc, 0, (size_t)ML * 8 * 16));
        flush();
        line("gat16_uc", ML * 16.0, 0, timeit([&] {
                 hipLaunchKernelGGL(k_gat16_uc, dim3(grid), dim3(TPB), 0, 0, uc, ML, dout);
             }));
        flush();
        line("sc16_uc", 0, ML * 16.0, timeit([&] { hipLaunchKernelGGL(k_sc16_uc, dim3(grid), dim3(TPB), 0, 0, uc, ML); }));
        flush();
        line("sc16", 0, ML * 16.0, timeit([&] { hipLaunchKernelGGL(k_sc16, dim3(grid), dim3(TPB), 0, 0, b, ML); }));
        CK(hipFree(uc));
    }
    flush();
    line("st16_nt", 0, N16 * 16.0,
         timeit([&] { hipLaunchKernelGGL(k_st16_nt, dim3(grid), dim3(TPB), 0, 0, a, N16); }));
    flush();
    line("st4_nt", 0, N16 * 16.0, timeit([&] {
             hipLaunchKernelGGL(k_st4_nt, dim3(grid), dim3(TPB), 0, 0, reinterpret_cast<uint32_t*>(a), N16 * 4);
         }));
    CK(hipDeviceSynchronize());
    return 0;
}
