// gp_xchg.hip -- multi-rank support kernels (gfx950): the random-edge message
// exchange of Imp3D slabs, the rank-sum of the round bookkeeping for in-process
// ranks, and the setup kernels that cut the global topology into slabs.
//
// Random edges cross slabs (7/8 of them at 8 ranks).  After round r every rank
// packs, per destination rank, the messages of its senders that chose their
// random edge for round r+1 (dir byte == DIR_RANDOM, written by the round
// kernel): {slot, (s, w)} where `slot` is the message's in-edge position in the
// destination's receiver-sorted CSR (static, precomputed) -- or, for gossip on the
// column kernel, {target's local id}: a rumour count the receiver adds to its
// next-round delivery counter (integer, so order-free).  Buffers have a
// fixed capacity per rank pair (expected count + 12 sigma), so
// RCCL moves fixed sizes on the stream with no host synchronisation; the
// in-band count says how many entries are real, and an overflow is recorded
// and fails the run loudly.  The receiver scatters each message to
// rmsg[slot] and, for gossip and during push-sum activation, rtag[slot] = r+1;
// its round kernel reads the tag instead of the sender's Philox draw (once every
// node is active a push-sum sender's draw alone decides, remote or not).  Entry
// order inside a buffer does not matter: every
// message carries its slot, so results are independent of the atomics' order.
#include <algorithm>

#include "gp_xchg.hpp"

namespace gp {
namespace {

__device__ __forceinline__ uint32_t owner_of(uint32_t t, const uint32_t* bounds, int W) {
    int o = 0;
    for (int w = 1; w < W; ++w) o += t >= bounds[w] ? 1 : 0;
    return (uint32_t)o;
}

}  // namespace

// Range binning: a block owns PACK_RANGE consecutive senders.  Sweep 1 finds
// every sender's destination rank (its next direction is the random edge and
// the edge's target lives elsewhere: xdst, a byte per sender precomputed at
// create, instead of the 4-byte edge), kept as a nibble per sender in registers,
// and counts them per rank in LDS; one global reservation per (block, rank)
// on the buffer's in-band counter; sweep 2 writes each message at the block's
// run offset (an LDS counter per rank).  (The previous form reserved per wave
// and rank: ~7 returning atomics per 64 senders on 7 words -- 15.4 ms per slab
// and round at world 8, against 2.2 ms for the round kernel.)
//
// Sweep 2 takes 8 senders per thread at a time: their run slots (LDS atomics),
// then every slot / payload load of the 8 at once, then the stores.  The loads
// are buffer loads over the block's senders; a sender without a message loads
// from past the end of the buffer, which returns 0 and touches no memory -- so
// no load sits under a branch (the compiler would wait for each in turn) and
// only senders with a message cost bytes.  The destination buffers' addresses
// sit in LDS (indexing the kernel arguments by a per-lane rank was a global
// load per message).
#ifndef GP_XCHG_PRIO
// wave priority raised (s_setprio 1) while k_pack / k_unpack issue their loads.  C5 at W = 8
// virtual ranks, same box, alternated: pack 4.97-4.99 -> 4.83 ms and unpack 5.59-5.73 ->
// 5.36-5.71 ms over the 8 slabs (profiles/r04/setprio_xchg.txt)
#define GP_XCHG_PRIO 1
#endif
template <int P>
__device__ __forceinline__ void xchg_prio() {
    if (GP_XCHG_PRIO) __builtin_amdgcn_s_setprio(P);
}

constexpr int PACK_PER = 32;                     // senders per thread
constexpr uint32_t PACK_RANGE = 256u * PACK_PER;  // senders per block
static_assert(XMAXW <= 16, "k_pack keeps a destination rank in 4 bits");
constexpr int BUF_WORD3 = 0x00020000;             // gfx9 raw buffer: 32-bit data format, no swizzle
constexpr uint32_t BUF_NONE = 0x80000000u;        // an offset past every buffer's end

__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, BUF_WORD3);
}

__global__ __launch_bounds__(256) void k_pack(PackArgs a) {
    __shared__ uint32_t cnt[XMAXW], off[XMAXW], cap[XMAXW];
    __shared__ uint32_t* oslots[XMAXW];
    __shared__ double2* ovals[XMAXW];
    __shared__ uint32_t bnd[XMAXW + 1];
    const uint32_t r0 = a.s_lo + blockIdx.x * PACK_RANGE;
    if (r0 >= a.s_hi) return;
    if (threadIdx.x < XMAXW) {
        cnt[threadIdx.x] = 0u;
        if (threadIdx.x < (uint32_t)a.W) {
            oslots[threadIdx.x] = a.peer[threadIdx.x].slots;
            ovals[threadIdx.x] = a.peer[threadIdx.x].vals;
            cap[threadIdx.x] = a.peer[threadIdx.x].cap;
        }
    }
    if (threadIdx.x <= (uint32_t)a.W) bnd[threadIdx.x] = a.bounds[threadIdx.x];
    __syncthreads();
    const uint32_t me = (uint32_t)a.me;
    const uint32_t last = a.s_hi - 1;
    // destination rank per sender, a nibble each; `me` means "no message" (a sender never
    // packs for its own rank, so the value is free for every world size up to XMAXW = 16)
    const uint32_t none = (uint32_t)a.me;
    uint32_t dst[PACK_PER / 8];
#pragma unroll
    for (int g = 0; g < PACK_PER / 8; ++g) {
        uint8_t b[8], t[8];
        xchg_prio<1>();
#pragma unroll
        for (int h = 0; h < 8; ++h) {  // unconditional loads (clamped), all in flight
            const uint32_t li = min(r0 + (g * 8 + h) * 256u + threadIdx.x, last);
            b[h] = a.nbn[a.lo + li - a.base];
            t[h] = a.xdst[li];
        }
        xchg_prio<0>();
        uint32_t w = 0;
#pragma unroll
        for (int h = 0; h < 8; ++h) {
            const uint32_t li = r0 + (g * 8 + h) * 256u + threadIdx.x;
            uint32_t d = none;
            if (li < a.s_hi && (b[h] & DIR_MASK) == DIR_RANDOM && t[h] != me) {
                d = t[h];
                atomicAdd(&cnt[d], 1u);
            }
            w |= d << (4 * h);
        }
        dst[g] = w;
    }
    __syncthreads();
    if (threadIdx.x < (uint32_t)a.W) {
        const uint32_t n = cnt[threadIdx.x];
        off[threadIdx.x] = n ? atomicAdd(a.peer[threadIdx.x].cnt, n) : 0u;
    }
    __syncthreads();
    // (uniform values kept in scalar registers: a resource in vector registers costs a
    // readfirstlane loop around every buffer load)
    const uint32_t nr = __builtin_amdgcn_readfirstlane(min(PACK_RANGE, a.s_hi - r0));
    const uint32_t sw0 = __builtin_amdgcn_readfirstlane(a.lo + r0 - a.base);
    // the entry: the in-edge slot at the destination, or (counts mode) the random edge's target
    const __amdgpu_buffer_rsrc_t rs_ent = buf_rsrc((a.counts ? a.rnd : a.pos) + r0, nr * 4u);
    const __amdgpu_buffer_rsrc_t rs_sw = buf_rsrc(a.swn + sw0, a.push ? nr * 16u : 0u);
#pragma unroll
    for (int g = 0; g < PACK_PER / 8; ++g) {
        uint32_t d[8], idx[8], ent[8];
        double2 v[8];
#pragma unroll
        for (int h = 0; h < 8; ++h) {
            d[h] = (dst[g] >> (4 * h)) & 15u;
            idx[h] = d[h] != none ? atomicAdd(&off[d[h]], 1u) : 0u;
        }
        xchg_prio<1>();
#pragma unroll
        for (int h = 0; h < 8; ++h) {
            const uint32_t q = (g * 8 + h) * 256u + threadIdx.x;  // sender r0 + q
            const bool m = d[h] != none;
            ent[h] = __builtin_amdgcn_raw_buffer_load_b32(rs_ent, m ? q * 4u : BUF_NONE, 0, 0);
            const auto x = __builtin_amdgcn_raw_buffer_load_b128(rs_sw, m ? q * 16u : BUF_NONE, 0, 0);
            v[h] = __builtin_bit_cast(double2, x);
        }
        xchg_prio<0>();
#pragma unroll
        for (int h = 0; h < 8; ++h) {
            if (d[h] == none) continue;
            const uint32_t k = d[h];
            if (idx[h] < cap[k]) {
                oslots[k][idx[h]] = a.counts ? ent[h] - bnd[k] : ent[h];
                if (a.push) ovals[k][idx[h]] = v[h];
            } else {
                atomicOr(a.overflow, 1u);
            }
        }
    }
}

// blockIdx.y = source rank.  A thread owns UNP entries UNP_STRIDE apart: their
// slots and payloads are loaded together (all in flight), then the scatters.  The
// grid covers the largest buffer's capacity (launch_unpack), so no thread loops.
constexpr int UNP = 4;
constexpr uint32_t UNP_BLOCK = 256u * UNP;
__global__ __launch_bounds__(256) void k_unpack(UnpackArgs a, uint32_t round) {
    const int p = blockIdx.y;
    if (p == a.me || !a.peer[p].cnt) return;
    const uint32_t sent = *a.peer[p].cnt;
    if (sent > a.peer[p].cap && blockIdx.x == 0 && threadIdx.x == 0) atomicOr(a.overflow, 1u);
    const uint32_t n = min(sent, a.peer[p].cap);
    const uint32_t k0 = blockIdx.x * UNP_BLOCK + threadIdx.x;
    if (k0 >= n) return;
    // push-sum with every node active: the round kernels decide remote senders by their
    // Philox draw and read no tag (all_active only ever goes 0 -> 1, and a round kernel
    // reads it after this unpack); gossip and the activation phase need the tags
    const bool tags = !a.push || __hip_atomic_load(a.all_active, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u;
    uint32_t slot[UNP];
    double2 v[UNP];
    xchg_prio<1>();
#pragma unroll
    for (int u = 0; u < UNP; ++u) {  // clamped: every load unconditional
        const uint32_t k = min(k0 + u * 256u, n - 1u);
        slot[u] = a.peer[p].slots[k];
        if (a.push) v[u] = a.peer[p].vals[k];
    }
    xchg_prio<0>();
#pragma unroll
    for (int u = 0; u < UNP; ++u) {
        if (k0 + u * 256u >= n) break;
        const uint32_t e = slot[u];
        if (e >= a.nedges) continue;  // never: slots are in-edge positions (or nodes) of this rank
        if (a.rq) {  // gossip column kernel: a rumour for local node `e` next round (integer count)
            rq_add(a.rq, a.rq8, e);
            continue;
        }
        if (tags) a.rtag[e] = round;
        if (a.push) a.rmsg[e] = v[u];
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

// xdst[li] = owner rank of sender lo+li's random-edge target; pos[li] = position
// of the sender in that owner's local in-edge array (global sorted position minus
// the owner's first edge), ~0 for local targets.
__global__ __launch_bounds__(256) void k_make_pos(PosArgs a) {
    for (uint32_t li = blockIdx.x * 256 + threadIdx.x; li < a.nloc; li += gridDim.x * 256) {
        const uint32_t own = owner_of(a.rnd[li], a.bounds, a.W);
        a.xdst[li] = (uint8_t)own;
        if (a.pos) a.pos[li] = own == (uint32_t)a.me ? 0xFFFFFFFFu : a.inv[a.lo + li] - a.edge0[own];
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
    for (uint32_t li = a.s_lo + blockIdx.x * 256 + threadIdx.x; li < a.s_hi; li += gridDim.x * 256) {
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
    (void)grid;
    const uint32_t blocks = a.s_hi > a.s_lo ? (a.s_hi - a.s_lo + PACK_RANGE - 1) / PACK_RANGE : 0u;
    if (blocks) hipLaunchKernelGGL(k_pack, dim3(blocks), dim3(256), 0, st, a);
    return hipGetLastError();
}
hipError_t launch_unpack(const UnpackArgs& a, uint32_t round, int grid, hipStream_t st) {
    (void)grid;
    uint32_t cap = 0;
    for (int p = 0; p < a.W; ++p)
        if (p != a.me) cap = std::max(cap, a.peer[p].cap);
    const uint32_t blocks = (cap + UNP_BLOCK - 1) / UNP_BLOCK;
    if (blocks) hipLaunchKernelGGL(k_unpack, dim3(blocks, a.W), dim3(256), 0, st, a, round);
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
