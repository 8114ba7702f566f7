// gp_xchg.hip -- multi-rank support kernels (gfx950): the random-edge message
// exchange of Imp3D slabs, the rank-sum of the round bookkeeping for in-process
// ranks, and the setup kernels that cut the global topology into slabs.
//
// Random edges cross slabs (7/8 of them at 8 ranks).  After round r every rank
// packs, per destination rank, the messages of its senders that chose their
// random edge for round r+1 (dir byte == DIR_RANDOM, written by the round
// kernel): {slot, (s, w)} where `slot` is the message's in-edge position in the
// destination's receiver-sorted CSR (static, precomputed).  Buffers have a
// fixed capacity per rank pair (expected count + 12 sigma), so
// RCCL moves fixed sizes on the stream with no host synchronisation; the
// in-band count says how many entries are real, and an overflow is recorded
// and fails the run loudly.  The receiver scatters each message to
// rmsg[slot] / rtag[slot] = r+1; its round kernel reads the tag instead of the
// sender's Philox draw.  Entry order inside a buffer does not matter: every
// message carries its slot, so results are independent of the atomics' order.
#include "gp_xchg.hpp"

namespace gp {
namespace {

__device__ __forceinline__ uint32_t owner_of(uint32_t t, const uint32_t* bounds, int W) {
    int o = 0;
    for (int w = 1; w < W; ++w) o += t >= bounds[w] ? 1 : 0;
    return (uint32_t)o;
}

__device__ __forceinline__ uint32_t lane_prefix64(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

}  // namespace

__global__ __launch_bounds__(256) void k_pack(PackArgs a) {
    const int lane = threadIdx.x & 63;
    for (uint32_t b0 = blockIdx.x * 256; b0 < a.nloc; b0 += gridDim.x * 256) {
        const uint32_t li = b0 + threadIdx.x;
        const bool valid = li < a.nloc;
        const uint32_t i = a.lo + li;
        bool rnd_send = false;
        uint32_t own = a.me;
        if (valid && (a.nbn[i - a.base] & DIR_MASK) == DIR_RANDOM) {
            own = owner_of(a.rnd[li], a.bounds, a.W);
            rnd_send = own != (uint32_t)a.me;
        }
        for (int p = 0; p < a.W; ++p) {
            if (p == a.me) continue;
            const bool mine = rnd_send && own == (uint32_t)p;
            const unsigned long long m = __ballot(mine);
            if (!m) continue;
            const int leader = __ffsll((long long)m) - 1;
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(a.peer[p].cnt, (uint32_t)__popcll(m));
            base = __shfl(base, leader, 64);
            if (mine) {
                const uint32_t idx = base + lane_prefix64(m);
                if (idx < a.peer[p].cap) {
                    a.peer[p].slots[idx] = a.pos[li];
                    if (a.push) a.peer[p].vals[idx] = a.swn[i - a.base];
                } else {
                    atomicOr(a.overflow, 1u);
                }
            }
        }
    }
}

// blockIdx.y = source rank.
__global__ __launch_bounds__(256) void k_unpack(UnpackArgs a, uint32_t round) {
    const int p = blockIdx.y;
    if (p == a.me || !a.peer[p].cnt) return;
    const uint32_t sent = *a.peer[p].cnt;
    if (sent > a.peer[p].cap && blockIdx.x == 0 && threadIdx.x == 0) atomicOr(a.overflow, 1u);
    const uint32_t n = min(sent, a.peer[p].cap);
    for (uint32_t k = blockIdx.x * 256 + threadIdx.x; k < n; k += gridDim.x * 256) {
        const uint32_t slot = a.peer[p].slots[k];
        if (slot >= a.nedges) continue;  // never: slots are in-edge positions of this rank
        a.rtag[slot] = round;
        if (a.push) a.rmsg[slot] = a.peer[p].vals[k];
    }
}

__global__ void k_zero_counts(ZeroArgs z) {
    const int p = threadIdx.x;
    if (p < z.n && z.cnt[p]) *z.cnt[p] = 0u;
}

// In-process ranks: sum xchg over the ranks' control blocks, write it back to all.
__global__ void k_sum_xchg(SumArgs s) {
    const int q = threadIdx.x;
    if (q >= 4) return;
    unsigned long long t = 0;
    for (int w = 0; w < s.W; ++w) t += s.ctl[w]->xchg[q];
    for (int w = 0; w < s.W; ++w) s.ctl[w]->xchg[q] = t;
}

// ---------------------------------------------------------------- setup
// rnd[i - first] = U_TOPO(i, P - 1) for i in [first, first + n) (Program.fs:259).
__global__ __launch_bounds__(256) void k_topo_rnd_range(uint32_t k0, uint32_t k1, uint32_t P, uint32_t first,
                                                        uint32_t n, uint32_t* out) {
    for (uint32_t q = blockIdx.x * 256 + threadIdx.x; q < n; q += gridDim.x * 256)
        out[q] = uniform(k0, k1, S_TOPO, first + q, 0, P - 1);
}

__global__ __launch_bounds__(256) void k_inverse(const uint32_t* perm, uint32_t n, uint32_t* inv) {
    for (uint32_t q = blockIdx.x * 256 + threadIdx.x; q < n; q += gridDim.x * 256) inv[perm[q]] = q;
}

__global__ __launch_bounds__(256) void k_sub(uint32_t* v, uint32_t n, uint32_t d) {
    for (uint32_t q = blockIdx.x * 256 + threadIdx.x; q < n; q += gridDim.x * 256) v[q] -= d;
}

// pos[li] = position of sender lo+li in its target owner's local in-edge array
// (global sorted position minus the owner's first edge); ~0 for local targets.
__global__ __launch_bounds__(256) void k_make_pos(PosArgs a) {
    for (uint32_t li = blockIdx.x * 256 + threadIdx.x; li < a.nloc; li += gridDim.x * 256) {
        const uint32_t own = owner_of(a.rnd[li], a.bounds, a.W);
        a.pos[li] = own == (uint32_t)a.me ? 0xFFFFFFFFu : a.inv[a.lo + li] - a.edge0[own];
    }
}

// Per destination rank: number of local senders whose random edge lands there
// and the expected number of them that use it in a round, sum 1/deg_i.
__global__ __launch_bounds__(256) void k_expect(ExpectArgs a) {
    __shared__ double ssum[XMAXW];
    __shared__ unsigned long long scnt[XMAXW];
    if (threadIdx.x < XMAXW) {
        ssum[threadIdx.x] = 0.0;
        scnt[threadIdx.x] = 0ull;
    }
    __syncthreads();
    for (uint32_t li = blockIdx.x * 256 + threadIdx.x; li < a.nloc; li += gridDim.x * 256) {
        const uint32_t own = owner_of(a.rnd[li], a.bounds, a.W);
        if (own == (uint32_t)a.me) continue;
        const uint32_t deg = popc6(present_mask<IMP3D>(a.lo + li, a.G)) + 1u;
        atomicAdd(&ssum[own], 1.0 / (double)deg);
        atomicAdd(&scnt[own], 1ull);
    }
    __syncthreads();
    if (threadIdx.x < (unsigned)a.W) {
        atomicAdd(&a.mu[threadIdx.x], ssum[threadIdx.x]);
        atomicAdd(&a.n[threadIdx.x], scnt[threadIdx.x]);
    }
}

// ---------------------------------------------------------------- launchers
hipError_t launch_pack(const PackArgs& a, int grid, hipStream_t st) {
    hipLaunchKernelGGL(k_pack, dim3(grid), dim3(256), 0, st, a);
    return hipGetLastError();
}
hipError_t launch_unpack(const UnpackArgs& a, uint32_t round, int grid, hipStream_t st) {
    hipLaunchKernelGGL(k_unpack, dim3(grid, a.W), dim3(256), 0, st, a, round);
    return hipGetLastError();
}
hipError_t launch_zero_counts(const ZeroArgs& z, hipStream_t st) {
    hipLaunchKernelGGL(k_zero_counts, dim3(1), dim3(XMAXW), 0, st, z);
    return hipGetLastError();
}
hipError_t launch_sum_xchg(const SumArgs& s, hipStream_t st) {
    hipLaunchKernelGGL(k_sum_xchg, dim3(1), dim3(64), 0, st, s);
    return hipGetLastError();
}
hipError_t launch_topo_rnd_range(uint32_t k0, uint32_t k1, uint32_t P, uint32_t first, uint32_t n, uint32_t* out,
                                 int grid, hipStream_t st) {
    hipLaunchKernelGGL(k_topo_rnd_range, dim3(grid), dim3(256), 0, st, k0, k1, P, first, n, out);
    return hipGetLastError();
}
hipError_t launch_inverse(const uint32_t* perm, uint32_t n, uint32_t* inv, int grid, hipStream_t st) {
    hipLaunchKernelGGL(k_inverse, dim3(grid), dim3(256), 0, st, perm, n, inv);
    return hipGetLastError();
}
hipError_t launch_sub(uint32_t* v, uint32_t n, uint32_t d, int grid, hipStream_t st) {
    hipLaunchKernelGGL(k_sub, dim3(grid), dim3(256), 0, st, v, n, d);
    return hipGetLastError();
}
hipError_t launch_make_pos(const PosArgs& a, int grid, hipStream_t st) {
    hipLaunchKernelGGL(k_make_pos, dim3(grid), dim3(256), 0, st, a);
    return hipGetLastError();
}
hipError_t launch_expect(const ExpectArgs& a, int grid, hipStream_t st) {
    hipLaunchKernelGGL(k_expect, dim3(grid), dim3(256), 0, st, a);
    return hipGetLastError();
}

}  // namespace gp
