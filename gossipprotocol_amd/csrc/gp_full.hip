// gp_full.hip -- gossip on the full topology on several ranks (gfx950).
//
// Every node can message every other node (Program.fs:211-216), so with W
// ranks (W-1)/W of the deliveries cross ranks each round.  Deliveries are
// integer increments (order-independent): remote ones are appended per
// destination rank with wave-aggregated atomics into the fixed-capacity
// exchange buffers (gp_xchg.hpp layout), exchanged over RCCL, and added by the
// owner.  Push-sum on several ranks bins its messages through the same buffers
// (gp_fullbin.hip k_fbm_send / k_fbm_coarse); the single-rank full topology has
// its own kernels (gp_kernels.hip, gp_fullbin.hip).
#include "gp_full.hpp"

namespace gp {
namespace {

__device__ __forceinline__ uint32_t lane_prefix64(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

template <typename T>
__device__ __forceinline__ T ld_agent(const T* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void block_add(uint32_t x, uint32_t y, unsigned long long* px, unsigned long long* py) {
    __shared__ uint32_t red[2][4];
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
        x = red[0][0] + red[0][1] + red[0][2] + red[0][3];
        y = red[1][0] + red[1][1] + red[1][2] + red[1][3];
        if (x && px) atomicAdd(px, (unsigned long long)x);
        if (y && py) atomicAdd(py, (unsigned long long)y);
    }
}

}  // namespace

__global__ __launch_bounds__(256) void k_fullm_gossip_send(FullArgs a, uint32_t r) {
    if (ld_agent(&a.ctl->done)) return;
    const int lane = threadIdx.x & 63;
    for (uint32_t b0 = blockIdx.x * 256; b0 < a.nloc; b0 += gridDim.x * 256) {
        const uint32_t li = b0 + threadIdx.x;
        const bool valid = li < a.nloc;
        const uint32_t i = a.lo + li;
        uint32_t t = 0, own = a.me;
        bool send = false;
        if (valid) {
            const int32_t ci = a.c[li];
            if (((i == a.seed_node) || ci >= 1) && ci <= 10) {
                t = full_target(i, uniform(a.k0, a.k1, S_GOSSIP, i, r, a.P - 1));
                own = 0;
                for (int w = 1; w < a.W; ++w) own += t >= a.bounds[w] ? 1u : 0u;
                send = true;
                if (own == (uint32_t)a.me) atomicAdd(&a.inc[t - a.lo], 1);  // integer: order-independent
            }
        }
        for (int p = 0; p < a.W; ++p) {
            if (p == a.me) continue;
            const bool mine = send && own == (uint32_t)p;
            const unsigned long long m = __ballot(mine);
            if (!m) continue;
            const int leader = __ffsll((long long)m) - 1;
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(a.peer[p].cnt, (uint32_t)__popcll(m));
            base = __shfl(base, leader, 64);
            if (mine) {
                const uint32_t idx = base + lane_prefix64(m);
                if (idx < a.peer[p].cap) a.peer[p].slots[idx] = t - a.bounds[p];
                else atomicOr(a.overflow, 1u);
            }
        }
    }
}

// blockIdx.y = source rank: add the received deliveries.
__global__ __launch_bounds__(256) void k_fullm_gossip_unpack(FullArgs a) {
    const int p = blockIdx.y;
    if (p == a.me || !a.rpeer[p].cnt) return;
    const uint32_t sent = *a.rpeer[p].cnt;
    if (sent > a.rpeer[p].cap && blockIdx.x == 0 && threadIdx.x == 0) atomicOr(a.overflow, 1u);
    const uint32_t n = min(sent, a.rpeer[p].cap);
    for (uint32_t k = blockIdx.x * 256 + threadIdx.x; k < n; k += gridDim.x * 256) {
        const uint32_t t = a.rpeer[p].slots[k];
        if (t < a.nloc) atomicAdd(&a.inc[t], 1);
    }
}

__global__ __launch_bounds__(256) void k_fullm_gossip_recv(FullArgs a) {
    if (ld_agent(&a.ctl->done)) return;
    uint32_t alerts = 0;
    for (uint32_t lj = blockIdx.x * 256 + threadIdx.x; lj < a.nloc; lj += gridDim.x * 256) {
        const int32_t d = a.inc[lj];
        if (!d) continue;
        a.inc[lj] = 0;
        const int32_t c0 = a.c[lj];
        if (c0 < (int32_t)GOSSIP_DONE) {  // dropped at converged receivers (Program.fs:87)
            a.c[lj] = c0 + d;
            alerts += c0 + d > 10;
        }
    }
    block_add(alerts, 0u, &a.ctl->round_alerts, nullptr);
}

// ---------------------------------------------------------------- launchers
hipError_t launch_fullm_gossip_send(const FullArgs& a, uint32_t r, int grid, hipStream_t st) {
    hipLaunchKernelGGL(k_fullm_gossip_send, dim3(grid), dim3(256), 0, st, a, r);
    return hipGetLastError();
}
hipError_t launch_fullm_gossip_unpack(const FullArgs& a, int grid, hipStream_t st) {
    hipLaunchKernelGGL(k_fullm_gossip_unpack, dim3(grid, a.W), dim3(256), 0, st, a);
    return hipGetLastError();
}
hipError_t launch_fullm_gossip_recv(const FullArgs& a, int grid, hipStream_t st) {
    hipLaunchKernelGGL(k_fullm_gossip_recv, dim3(grid), dim3(256), 0, st, a);
    return hipGetLastError();
}

}  // namespace gp
