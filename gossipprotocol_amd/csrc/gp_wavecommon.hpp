// gp_wavecommon.hpp -- helpers shared by the column-march round kernels
// (gp_col.hip, gp_pscol.hip).  Included by those translation units only.
#pragma once

#include "gp_internal.hpp"

namespace gp {
namespace wk {

constexpr int WPB = BULK_THREADS / 64;  // waves per 256-thread block

template <typename T>
__device__ __forceinline__ T ld_agent(const T* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint32_t lane_prefix(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// LDS written by lanes of this wave and read back by other lanes of it: keep the
// compiler from moving DS operations across this point (the hardware executes
// one wave's DS operations in order).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
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
