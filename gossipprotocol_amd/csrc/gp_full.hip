// gp_full.hip -- full topology on several ranks (gfx950).
//
// Every node can message every other node (Program.fs:211-216), so with W
// ranks (W-1)/W of the messages cross ranks each round.  Per round on rank A:
//
//   push-sum: every active local sender draws its target t = full_target(i,
//     U(P-1)) (Program.fs:103,128) and stages (t, sender); a stable radix sort
//     by t groups the messages by destination rank and, inside a rank, by
//     target with senders ascending.  Each destination's segment is packed
//     as {target - lo_B, s, w} into that rank's fixed-capacity exchange buffer
//     (gp_xchg.hpp layout) and exchanged over RCCL.  The receiver concatenates
//     the segments in ascending source rank -- its own segment in its rank's
//     place -- and a second stable sort by target yields, for every receiver,
//     its senders in ascending global id: the canonical fold order of SRS v1.
//   gossip: deliveries are integer increments (order-independent), so remote
//     ones are appended with wave-aggregated atomics and added at the owner.
//
// The single-rank full topology keeps its own kernels (gp_kernels.hip).
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

// ---------------------------------------------------------------- push-sum
__global__ __launch_bounds__(256) void k_fullm_ps_send(FullArgs a, uint32_t r) {
    if (ld_agent(&a.ctl->done)) return;
    for (uint32_t li = blockIdx.x * 256 + threadIdx.x; li < a.nloc; li += gridDim.x * 256) {
        const uint32_t i = a.lo + li;
        const bool act = (a.nb[li] & B_ACTIVE) != 0;
        a.key0[li] = act ? full_target(i, uniform(a.k0, a.k1, S_PUSHSUM, i, r, a.P - 1)) : 0xFFFFFFFFu;
        a.val0[li] = li;
    }
}

// seg[b] = first sorted position whose target lies at or beyond rank b's first id.
__global__ void k_fullm_split(FullArgs a) {
    const int b = threadIdx.x;
    if (b > a.W) return;
    const uint32_t lim = b == a.W ? 0xFFFFFFFFu : a.bounds[b];
    uint32_t lo = 0, hi = a.nloc;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a.key1[mid] < lim) lo = mid + 1;
        else hi = mid;
    }
    a.seg[b] = lo;  // seg[W] = number of messages (inactive senders sort last)
}

// Remote segments -> exchange buffers {target - lo_B, s, w}.
__global__ __launch_bounds__(256) void k_fullm_ps_pack(FullArgs a) {
    const int b = blockIdx.y;
    if (b == a.me || !a.peer[b].cnt) return;
    const uint32_t s0 = a.seg[b], s1 = a.seg[b + 1];
    const uint32_t n = s1 - s0;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        *a.peer[b].cnt = min(n, a.peer[b].cap);
        if (n > a.peer[b].cap) atomicOr(a.overflow, 1u);
    }
    for (uint32_t k = blockIdx.x * 256 + threadIdx.x; k < n && k < a.peer[b].cap; k += gridDim.x * 256) {
        const uint32_t p = s0 + k;
        a.peer[b].slots[k] = a.key1[p] - a.bounds[b];
        a.peer[b].vals[k] = a.swc[a.val1[p]];
    }
}

// Concatenate the segments in ascending source rank into ckey / cval (padded to
// the capacity with key ~0 so the second sort runs on a host-known size).
__global__ __launch_bounds__(256) void k_fullm_ps_combine(FullArgs a) {
    __shared__ uint32_t off[XMAXW + 1];
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (int p = 0; p < a.W; ++p) {
            off[p] = run;
            if (p == a.me) run += a.seg[a.me + 1] - a.seg[a.me];
            else if (a.rpeer[p].cnt) run += min(*a.rpeer[p].cnt, a.rpeer[p].cap);
        }
        off[a.W] = run;
    }
    __syncthreads();
    const uint32_t total = off[a.W];
    for (uint32_t q = blockIdx.x * 256 + threadIdx.x; q < a.ccap; q += gridDim.x * 256) {
        if (q >= total) {
            a.ckey[q] = 0xFFFFFFFFu;
            a.cidx[q] = q;
            continue;
        }
        int p = 0;
        while (p + 1 < a.W && q >= off[p + 1]) ++p;
        const uint32_t k = q - off[p];
        if (p == a.me) {
            const uint32_t pp = a.seg[a.me] + k;
            a.ckey[q] = a.key1[pp] - a.lo;
            a.cval[q] = a.swc[a.val1[pp]];
        } else {
            a.ckey[q] = a.rpeer[p].slots[k];
            a.cval[q] = a.rpeer[p].vals[k];
        }
        a.cidx[q] = q;
    }
}

__global__ __launch_bounds__(256) void k_fullm_ps_mark(FullArgs a) {
    if (ld_agent(&a.ctl->done)) return;
    for (uint32_t p = blockIdx.x * 256 + threadIdx.x; p < a.ccap; p += gridDim.x * 256) {
        const uint32_t k = a.ckey2[p];
        if (k < a.nloc && (p == 0 || a.ckey2[p - 1] != k)) a.head[k] = p;
    }
}

__global__ __launch_bounds__(256) void k_fullm_ps_recv(FullArgs a) {
    if (ld_agent(&a.ctl->done)) return;
    uint32_t alerts = 0, newly = 0;
    for (uint32_t lj = blockIdx.x * 256 + threadIdx.x; lj < a.nloc; lj += gridDim.x * 256) {
        const uint8_t b = a.nb[lj];
        const double2 sv = a.swc[lj];
        const bool active = (b & B_ACTIVE) != 0;
        double acc_s = active ? sv.x * 0.5 : sv.x;
        double acc_w = active ? sv.y * 0.5 : sv.y;
        uint32_t p = a.head[lj];
        bool recv = false;
        if (p != 0xFFFFFFFFu) {
            for (; p < a.ccap && a.ckey2[p] == lj; ++p) {
                const double2 m = a.cval[a.cidx2[p]];
                acc_s = acc_s + m.x * 0.5;
                acc_w = acc_w + m.y * 0.5;
                recv = true;
            }
        }
        uint32_t flags = b;
        if (recv) {
            if (!(b & B_CONV)) {
                const double r_old = sv.x / sv.y;
                const double r_new = acc_s / acc_w;
                uint32_t cnt = (b >> CNT_SHIFT) & 3u;
                cnt = fabs(r_new - r_old) > 1e-10 ? 0u : cnt + 1u;
                flags = (flags & ~(3u << CNT_SHIFT)) | (cnt << CNT_SHIFT);
                if (cnt == 3) {
                    flags |= B_CONV;
                    ++alerts;
                }
            }
            if (!active) {
                ++newly;
                flags |= B_ACTIVE;
            }
            a.nb[lj] = (uint8_t)flags;
        }
        a.swn[lj] = make_double2(acc_s, acc_w);
    }
    block_add(alerts, newly, &a.ctl->round_alerts, &a.ctl->round_active);
}

// ---------------------------------------------------------------- gossip
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
hipError_t launch_fullm_ps_send(const FullArgs& a, uint32_t r, int grid, hipStream_t st) {
    hipLaunchKernelGGL(k_fullm_ps_send, dim3(grid), dim3(256), 0, st, a, r);
    return hipGetLastError();
}
hipError_t launch_fullm_split(const FullArgs& a, hipStream_t st) {
    hipLaunchKernelGGL(k_fullm_split, dim3(1), dim3(64), 0, st, a);
    return hipGetLastError();
}
hipError_t launch_fullm_ps_pack(const FullArgs& a, int grid, hipStream_t st) {
    hipLaunchKernelGGL(k_fullm_ps_pack, dim3(grid, a.W), dim3(256), 0, st, a);
    return hipGetLastError();
}
hipError_t launch_fullm_ps_combine(const FullArgs& a, int grid, hipStream_t st) {
    hipLaunchKernelGGL(k_fullm_ps_combine, dim3(grid), dim3(256), 0, st, a);
    return hipGetLastError();
}
hipError_t launch_fullm_ps_mark(const FullArgs& a, int grid, hipStream_t st) {
    hipLaunchKernelGGL(k_fullm_ps_mark, dim3(grid), dim3(256), 0, st, a);
    return hipGetLastError();
}
hipError_t launch_fullm_ps_recv(const FullArgs& a, int grid, hipStream_t st) {
    hipLaunchKernelGGL(k_fullm_ps_recv, dim3(grid), dim3(256), 0, st, a);
    return hipGetLastError();
}
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
