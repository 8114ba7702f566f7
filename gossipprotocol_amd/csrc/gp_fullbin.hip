// gp_fullbin.hip -- push-sum on the full topology, one rank (gfx950): the
// scattered receives of a round are staged and binned through LDS, then folded
// per receiver tile in the canonical order.
//
// Reference: every node's neighbour list is all j != i (Program.fs:209-216);
// an active node halves (sum, weight) and sends the halves to one uniform
// neighbour (Program.fs:104-106,125-128); a receiver folds its messages (SRS v1
// B.4: own half, then messages by ascending sender id) and runs the ratio test
// (Program.fs:114-123).
//
// Per round, three kernels:
//   A  k_fb_send   senders in chunks of FBO_CHUNK: target t = U(P-1) mapped past i
//                  (Philox), LDS counting by coarse bin (t >> s1), one global
//                  reservation per (chunk, bin), each message {i | s/2, w/2}
//                  written into its coarse bin's run;
//   B  k_fb_split  each coarse bin's messages in chunks: the target recomputed
//                  from the sender's Philox draw, LDS counting by fine tile
//                  (t >> FB_TB, FB_TILE receivers), reservation, copy;
//   C  k_fb_fold   one fine tile per block: LDS counting sort of the tile's
//                  messages by receiver (target recomputed once more), each
//                  receiver's (few) messages put in ascending sender order,
//                  folded, ratio test, next state.
// Order inside a bin is whatever the LDS atomics produce; the fold restores the
// canonical order by sender id, so results do not depend on it.  Every message
// is moved as 20 bytes (sender id 4 + payload 16; recomputing the target costs
// a Philox draw per pass instead of 4 bytes per move), each pass coalesced -- no
// random 16-byte gather of a sender's (s, w) anywhere.  Bin capacities are the
// expected load + 12 sigma + slack; an overflow is flagged (Ctl::overflow) and
// fails the batch in gp_step.
#include <algorithm>
#include <cmath>

#include "gp_fullbin.hpp"

namespace gp {
namespace {

// Passes A and B: 1024-thread blocks over chunks of FBO_CHUNK senders / messages
// (8 per thread), so a chunk writes runs of ~43 (A) and ~16 (B) consecutive
// messages per bin and reserves each run with one global atomic.
constexpr int FB_THREADS = 256;                    // C
constexpr int FBX_THREADS = 1024;                  // A, B
constexpr int FB_MAXBINS = 4096;                   // LDS counters of A and B
constexpr uint32_t FB_NONE = 0xFFFFu;
#ifndef GP_FB_BATCH
#define GP_FB_BATCH 8
#endif
constexpr int FB_BATCH = GP_FB_BATCH;              // loads issued together before their stores


template <typename T>
__device__ __forceinline__ T ld_agent(const T* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}


// Exclusive scan of cnt[0..n) in LDS (n <= FB_MAXBINS), one block of NT threads;
// returns the total.
template <int NT>
__device__ uint32_t lds_excl_scan(uint32_t* cnt, uint32_t n, uint32_t* tmp) {
    constexpr int PER = (FB_MAXBINS + NT - 1) / NT;
    uint32_t v[PER], s = 0;
    const uint32_t b = threadIdx.x * PER;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        v[k] = b + k < n ? cnt[b + k] : 0u;
        s += v[k];
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t incl = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
    }
    if (lane == 63) tmp[wid] = incl;
    __syncthreads();
    uint32_t wbase = 0, total = 0;
    for (int w = 0; w < NT / 64; ++w) {
        if (w < wid) wbase += tmp[w];
        total += tmp[w];
    }
    uint32_t run = wbase + incl - s;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        if (b + k < n) cnt[b + k] = run;
        run += v[k];
    }
    __syncthreads();
    return total;
}

}  // namespace

// ---------------------------------------------------------------- A, B: binning passes
// A chunk's messages are put in bin order in LDS (perm) first, so consecutive
// threads write consecutive slots of one bin's run (whole lines) instead of 64
// different runs per store instruction (measured: send 2.06 -> 1.37 ms, split
// 2.31 -> 2.00 ms at P = 1e8); the payload loads become gathers inside the
// chunk's input instead.
constexpr int FBO_PER = 8;
constexpr int FBO_CHUNK = FBX_THREADS * FBO_PER;  // 8192

__global__ __launch_bounds__(FBX_THREADS) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_fb_send(FullBinArgs a,
                                                                                                      uint32_t r) {
    __shared__ uint32_t loff[FB_MAXBINS];      // per bin: count, then the bin's first position in perm
    __shared__ uint32_t gb[FB_MAXBINS];        // per bin: the chunk's reserved base in the global bin
    __shared__ uint16_t bin[FBO_CHUNK];
    __shared__ uint16_t rank[FBO_CHUNK];
    __shared__ uint16_t perm[FBO_CHUNK];       // chunk positions in bin order
    uint32_t* tmp = reinterpret_cast<uint32_t*>(perm);  // scan scratch, used before perm is written
    if (ld_agent(&a.ctl->done)) return;
    const uint32_t P = a.P;
    for (uint64_t c0 = (uint64_t)blockIdx.x * FBO_CHUNK; c0 < P; c0 += (uint64_t)gridDim.x * FBO_CHUNK) {
        for (uint32_t b = threadIdx.x; b < a.nb1; b += FBX_THREADS) loff[b] = 0u;
        __syncthreads();
        {
            uint32_t node[FBO_PER], x[FBO_PER], y[FBO_PER];
#pragma unroll
            for (int k = 0; k < FBO_PER; ++k) node[k] = (uint32_t)(c0 + k * FBX_THREADS + threadIdx.x);
            philox2_batch<FBO_PER>(node, r, S_PUSHSUM, a.k0, a.k1, x, y);
#pragma unroll
            for (int k = 0; k < FBO_PER; ++k) {
                const uint32_t i = node[k], q = k * FBX_THREADS + threadIdx.x;
                uint32_t bb = FB_NONE;
                if (i < P && (a.nb[i] & B_ACTIVE) && P > 1) {
                    bb = full_target(i, uniform_from(x[k], y[k], P - 1)) >> a.s1;  // Program.fs:213-215
                    rank[q] = (uint16_t)atomicAdd(&loff[bb], 1u);
                }
                bin[q] = (uint16_t)bb;
            }
        }
        __syncthreads();
        for (uint32_t b = threadIdx.x; b < a.nb1; b += FBX_THREADS) {
            const uint32_t n = loff[b];
            gb[b] = n ? atomicAdd(&a.cnt1[b], n) : 0u;
        }
        const uint32_t total = lds_excl_scan<FBX_THREADS>(loff, a.nb1, tmp);
#pragma unroll
        for (int k = 0; k < FBO_PER; ++k) {
            const uint32_t q = k * FBX_THREADS + threadIdx.x, b = bin[q];
            if (b != FB_NONE) perm[loff[b] + rank[q]] = (uint16_t)q;
        }
        __syncthreads();
        for (uint32_t p0 = 0; p0 < total; p0 += FBX_THREADS * FB_BATCH) {
            uint32_t qq[FB_BATCH];
            double2 sv[FB_BATCH];
#pragma unroll
            for (int k = 0; k < FB_BATCH; ++k) {
                const uint32_t p = p0 + k * FBX_THREADS + threadIdx.x;
                qq[k] = p < total ? perm[p] : 0xFFFFu;
                sv[k] = qq[k] != 0xFFFFu ? a.swc[(uint32_t)(c0 + qq[k])] : make_double2(0.0, 0.0);
            }
#pragma unroll
            for (int k = 0; k < FB_BATCH; ++k) {
                const uint32_t p = p0 + k * FBX_THREADS + threadIdx.x;
                if (p >= total) continue;
                const uint32_t b = bin[qq[k]], pos = gb[b] + (p - loff[b]);
                if (pos >= a.cap1) {
                    atomicOr(a.overflow, 1u);
                    continue;
                }
                const size_t o = (size_t)b * a.cap1 + pos;
                a.hdr1[o] = (uint32_t)(c0 + qq[k]);
                a.pay1[o] = make_double2(sv[k].x * 0.5, sv[k].y * 0.5);
            }
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(FBX_THREADS) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_fb_split(FullBinArgs a,
                                                                                                       uint32_t r) {
    __shared__ uint32_t loff[FB_MAXBINS];
    __shared__ uint32_t gb[FB_MAXBINS];
    __shared__ uint16_t fine[FBO_CHUNK];
    __shared__ uint16_t rank[FBO_CHUNK];
    __shared__ uint16_t perm[FBO_CHUNK];
    uint32_t* tmp = reinterpret_cast<uint32_t*>(perm);  // scan scratch, used before perm is written
    if (ld_agent(&a.ctl->done)) return;
    const uint32_t per_bin = (a.cap1 + FBO_CHUNK - 1) / FBO_CHUNK;
    const uint32_t nfine = 1u << (a.s1 - FB_TB);
    for (uint32_t w = blockIdx.x; w < a.nb1 * per_bin; w += gridDim.x) {
        const uint32_t b = w / per_bin, c = w % per_bin;
        const uint32_t n_bin = min(ld_agent(&a.cnt1[b]), a.cap1);
        const uint32_t q0 = c * FBO_CHUNK;
        if (q0 >= n_bin) continue;  // block-uniform
        const uint32_t n = min((uint32_t)FBO_CHUNK, n_bin - q0);
        for (uint32_t f = threadIdx.x; f < nfine; f += FBX_THREADS) loff[f] = 0u;
        __syncthreads();
        const size_t base = (size_t)b * a.cap1 + q0;
        constexpr int PB = 4;
#pragma unroll 1
        for (int k0 = 0; k0 < FBO_PER; k0 += PB) {
            uint32_t node[PB], x[PB], y[PB];
#pragma unroll
            for (int k = 0; k < PB; ++k) {
                const uint32_t q = (k0 + k) * FBX_THREADS + threadIdx.x;
                node[k] = q < n ? a.hdr1[base + q] : 0u;
            }
            philox2_batch<PB>(node, r, S_PUSHSUM, a.k0, a.k1, x, y);
#pragma unroll
            for (int k = 0; k < PB; ++k) {
                const uint32_t q = (k0 + k) * FBX_THREADS + threadIdx.x;
                if (q < n) {
                    const uint32_t t = full_target(node[k], uniform_from(x[k], y[k], a.P - 1));
                    const uint32_t f = (t >> FB_TB) & (nfine - 1u);
                    fine[q] = (uint16_t)f;
                    rank[q] = (uint16_t)atomicAdd(&loff[f], 1u);
                }
            }
        }
        __syncthreads();
        const uint32_t f0 = b << (a.s1 - FB_TB);
        for (uint32_t f = threadIdx.x; f < nfine; f += FBX_THREADS) {
            const uint32_t m = loff[f];
            gb[f] = m && f0 + f < a.nb2 ? atomicAdd(&a.cnt2[f0 + f], m) : 0u;
        }
        lds_excl_scan<FBX_THREADS>(loff, nfine, tmp);
        for (uint32_t q = threadIdx.x; q < n; q += FBX_THREADS) perm[loff[fine[q]] + rank[q]] = (uint16_t)q;
        __syncthreads();
#pragma unroll 1
        for (uint32_t p0 = 0; p0 < n; p0 += FBX_THREADS * FB_BATCH) {
            uint32_t qq[FB_BATCH], h[FB_BATCH];
            double2 pv[FB_BATCH];
#pragma unroll
            for (int k = 0; k < FB_BATCH; ++k) {
                const uint32_t p = p0 + k * FBX_THREADS + threadIdx.x;
                qq[k] = p < n ? perm[p] : 0xFFFFu;
                h[k] = 0u;
                pv[k] = make_double2(0.0, 0.0);
                if (qq[k] != 0xFFFFu) {
                    h[k] = a.hdr1[base + qq[k]];
                    pv[k] = a.pay1[base + qq[k]];
                }
            }
#pragma unroll
            for (int k = 0; k < FB_BATCH; ++k) {
                const uint32_t p = p0 + k * FBX_THREADS + threadIdx.x;
                if (p >= n) continue;
                const uint32_t f = fine[qq[k]], pos = gb[f] + (p - loff[f]);
                if (f0 + f >= a.nb2 || pos >= a.cap2) {
                    atomicOr(a.overflow, 1u);
                    continue;
                }
                const size_t o = (size_t)(f0 + f) * a.cap2 + pos;
                a.hdr2[o] = h[k];
                a.pay2[o] = pv[k];
            }
        }
        __syncthreads();
    }
}
// ---------------------------------------------------------------- C: fold per fine tile
__global__ __launch_bounds__(FB_THREADS) void k_fb_fold(FullBinArgs a, uint32_t r) {
    constexpr int TILE = 1 << FB_TB;
    constexpr int NPT = TILE / FB_THREADS;
    __shared__ uint32_t cnt[TILE + 1];            // per receiver: count, then start
    __shared__ uint32_t src[FB_CAP2];             // message sender ids in receiver order
    __shared__ uint16_t idx[FB_CAP2];             // message index in the fine bin, receiver order
    __shared__ uint16_t rnk[FB_CAP2];
    __shared__ uint16_t loc[FB_CAP2];             // message's receiver within the tile
    __shared__ uint32_t tmp[FB_THREADS / 64];
    __shared__ uint32_t red[2][FB_THREADS / 64];
    Ctl* ctl = a.ctl;
    if (ld_agent(&ctl->done)) return;
    const uint32_t P = a.P;
    const double2* __restrict__ swc = a.swc;
    const double2* __restrict__ pay2 = a.pay2;
    double2* __restrict__ swn = a.swn;
    uint8_t* __restrict__ nbp = a.nb;
    uint32_t alerts = 0, newly = 0;
    for (uint32_t f = blockIdx.x; f < a.nb2; f += gridDim.x) {
        const uint32_t n = min(ld_agent(&a.cnt2[f]), (uint32_t)a.cap2);
        const size_t base = (size_t)f * a.cap2;
        for (uint32_t v = threadIdx.x; v < TILE; v += FB_THREADS) cnt[v] = 0u;
        __syncthreads();
        {
            // the tile's messages, FQ per thread: senders loaded together, targets
            // recomputed as one Philox batch
            constexpr int FQ = (FB_CAP2 + FB_THREADS - 1) / FB_THREADS;
            uint32_t snd[FQ], x[FQ], y[FQ];
#pragma unroll
            for (int k = 0; k < FQ; ++k) {
                const uint32_t q = k * FB_THREADS + threadIdx.x;
                snd[k] = q < n ? a.hdr2[base + q] : 0u;
            }
            philox2_batch<FQ>(snd, r, S_PUSHSUM, a.k0, a.k1, x, y);
#pragma unroll
            for (int k = 0; k < FQ; ++k) {
                const uint32_t q = k * FB_THREADS + threadIdx.x;
                if (q < n) {
                    const uint32_t v = full_target(snd[k], uniform_from(x[k], y[k], P - 1)) & (TILE - 1);
                    loc[q] = (uint16_t)v;
                    rnk[q] = (uint16_t)atomicAdd(&cnt[v], 1u);
                }
            }
        }
        __syncthreads();
        lds_excl_scan<FB_THREADS>(cnt, TILE, tmp);
        if (threadIdx.x == 0) cnt[TILE] = n;
        for (uint32_t q = threadIdx.x; q < n; q += FB_THREADS) {
            const uint32_t p = cnt[loc[q]] + rnk[q];
            src[p] = a.hdr2[base + q];
            idx[p] = (uint16_t)q;
        }
        __syncthreads();
        // every node's byte and (s, w) in flight before any store of the tile
        uint8_t bk[NPT];
        double2 svk[NPT];
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
            const uint32_t j = f * TILE + k * FB_THREADS + threadIdx.x;
            bk[k] = 0;
            svk[k] = make_double2(0.0, 1.0);
            if (j < P) {
                bk[k] = nbp[j];
                svk[k] = swc[j];
            }
        }
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
            const uint32_t v = k * FB_THREADS + threadIdx.x;
            const uint32_t j = f * TILE + v;
            if (j >= P) continue;
            const uint32_t p0 = cnt[v], p1 = cnt[v + 1];
            // this receiver's messages in ascending sender id (canonical order):
            // insertion sort of its (few) entries in place
            for (uint32_t p = p0 + 1; p < p1; ++p) {
                const uint32_t s = src[p];
                const uint16_t x = idx[p];
                uint32_t q = p;
                while (q > p0 && src[q - 1] > s) {
                    src[q] = src[q - 1];
                    idx[q] = idx[q - 1];
                    --q;
                }
                src[q] = s;
                idx[q] = x;
            }
            const uint8_t b = bk[k];
            const double2 sv = svk[k];
            const bool active = (b & B_ACTIVE) != 0;
            double acc_s = active && P > 1 ? sv.x * 0.5 : sv.x;
            double acc_w = active && P > 1 ? sv.y * 0.5 : sv.y;
            for (uint32_t p = p0; p < p1; ++p) {
                const double2 m = pay2[base + idx[p]];  // already halved by the sender
                acc_s = acc_s + m.x;
                acc_w = acc_w + m.y;
            }
            if (p1 > p0) {
                uint32_t flags = b;
                if (!(b & B_CONV)) {
                    const double r_old = sv.x / sv.y;
                    const double r_new = acc_s / acc_w;
                    uint32_t c = (b >> CNT_SHIFT) & 3u;
                    c = fabs(r_new - r_old) > 1e-10 ? 0u : c + 1u;
                    flags = (flags & ~(3u << CNT_SHIFT)) | (c << CNT_SHIFT);
                    if (c == 3) {
                        flags |= B_CONV;
                        ++alerts;
                    }
                }
                if (!active) {
                    ++newly;
                    flags |= B_ACTIVE;
                }
                nbp[j] = (uint8_t)flags;
            }
            swn[j] = make_double2(acc_s, acc_w);
        }
        __syncthreads();
    }
    uint32_t x = alerts, y = newly;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        x += __shfl_xor(x, o, 64);
        y += __shfl_xor(y, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = x;
        red[1][threadIdx.x >> 6] = y;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        x = y = 0;
        for (int w = 0; w < FB_THREADS / 64; ++w) {
            x += red[0][w];
            y += red[1][w];
        }
        if (x) atomicAdd(&ctl->round_alerts, (unsigned long long)x);
        if (y) atomicAdd(&ctl->round_active, (unsigned long long)y);
    }
}

// ---------------------------------------------------------------- host side
FullBinPlan full_bin_plan(uint32_t P) {
    FullBinPlan p{};
    uint32_t bits = 1;
    while (bits < 32 && ((uint64_t)1 << bits) < P) ++bits;
    // coarse bins ~ sqrt(P / TILE) so both passes write runs of ~10-20 messages;
    // at most FB_MAXBINS coarse bins and FB_MAXBINS fine tiles per coarse bin
    uint32_t s1 = (bits + FB_TB + 1) / 2;
    if (s1 < FB_TB) s1 = FB_TB;
    while (((uint64_t)P >> s1) >= FB_MAXBINS) ++s1;
    while (s1 - FB_TB > 12) --s1;
    p.s1 = s1;
    p.nb1 = (uint32_t)(((uint64_t)P + (1ull << s1) - 1) >> s1);
    p.nb2 = (uint32_t)(((uint64_t)P + (1u << FB_TB) - 1) >> FB_TB);
    const double m1 = (double)(1ull << s1) * ((double)P / (double)(P > 1 ? P - 1 : 1));
    p.cap1 = (uint32_t)(m1 + 12.0 * std::sqrt(m1) + 1024.0);
    p.cap2 = FB_CAP2;
    return p;
}

hipError_t launch_full_bin_round(const FullBinArgs& a, uint32_t round, int grid, hipStream_t st) {
    hipError_t e;
    if ((e = hipMemsetAsync(a.cnt1, 0, sizeof(uint32_t) * a.nb1, st)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(a.cnt2, 0, sizeof(uint32_t) * a.nb2, st)) != hipSuccess) return e;
    const uint32_t gx = (uint32_t)std::max(1, grid / 4);  // 1024-thread blocks
    const uint32_t chunks = (a.P + FBO_CHUNK - 1) / FBO_CHUNK;
    hipLaunchKernelGGL(k_fb_send, dim3(std::min<uint32_t>(chunks, gx)), dim3(FBX_THREADS), 0, st, a, round);
    const uint32_t items = a.nb1 * ((a.cap1 + FBO_CHUNK - 1) / FBO_CHUNK);
    hipLaunchKernelGGL(k_fb_split, dim3(std::min<uint32_t>(items, gx)), dim3(FBX_THREADS), 0, st, a, round);
    hipLaunchKernelGGL(k_fb_fold, dim3(std::min<uint32_t>(a.nb2, (uint32_t)grid)), dim3(FB_THREADS), 0, st, a,
                       round);
    return hipGetLastError();
}

}  // namespace gp
