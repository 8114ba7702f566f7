// gp_wavecommon.hpp -- helpers of the column-march round kernels (gp_col.hip).
// Included by that translation unit only.
#pragma once

#include "gp_internal.hpp"

namespace gp {
namespace wk {

constexpr int WPB = BULK_THREADS / 64;  // waves per 256-thread block

template <typename T>
__device__ __forceinline__ T ld_agent(const T* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Block-wide sum of two per-thread counters, one atomic each (if non-zero).
__device__ __forceinline__ void block_add2(uint32_t x, uint32_t y, unsigned long long* px, unsigned long long* py) {
    __shared__ uint32_t red[2][WPB];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        x += __shfl_xor(x, o, 64);
        y += __shfl_xor(y, o, 64);
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) {
        red[0][wid] = x;
        red[1][wid] = y;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        x = 0;
        y = 0;
#pragma unroll
        for (int w = 0; w < WPB; ++w) {
            x += red[0][w];
            y += red[1][w];
        }
        if (x && px) atomicAdd(px, (unsigned long long)x);
        if (y && py) atomicAdd(py, (unsigned long long)y);
    }
}

}  // namespace wk
}  // namespace gp
