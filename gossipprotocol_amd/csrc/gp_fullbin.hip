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
//   A  k_fb_send   ranges of senders (FB_RANGE chunks of FBR_CHUNK, one
//                  1024-thread block each): target t = U(P-1) mapped past i
//                  (Philox); sweep 1 counts the range's messages per coarse bin
//                  (t >> s1) in LDS and reserves one run per (range, bin); sweep
//                  2 puts each chunk in bin order in LDS and writes {i | s/2,
//                  w/2} into the runs, coalesced, the next chunk's loads in
//                  flight meanwhile;
//   B  k_fb_split  ranges of each coarse bin's messages, the same two sweeps by
//                  fine tile (t >> FB_TB), the target recomputed from the
//                  sender's Philox draw;
//   C  k_fb_fold   one fine tile per block: the tile's messages loaded in bin
//                  order (coalesced), LDS counting sort by receiver (target
//                  recomputed once more) with the payloads, each receiver's (few)
//                  messages put in ascending sender order, folded from LDS, ratio
//                  test, next state.
// Order inside a bin is whatever the LDS atomics produce; the fold restores the
// canonical order by sender id, so results do not depend on it.  Every message
// is moved as 20 bytes (sender id 4 + payload 16; recomputing the target costs
// a Philox draw per pass instead of 4 bytes per move), every global access is
// coalesced -- no random 16-byte gather anywhere.  Bin capacities are the
// expected load + 12 sigma + slack; an overflow is flagged (Ctl::overflow) and
// fails the batch in gp_step.
#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "gp_fullbin.hpp"

namespace gp {
namespace {

constexpr int FB_MAXBINS = 4096;                   // LDS counters of A and B
// (No wave priority here: raised while the fold / split issue their loads and stores it measured
// 3.17-3.18 against 3.03-3.17 ms/round, C4 same box, profiles/r04/setprio_c3c4.txt.)
constexpr uint32_t FB_NONE = 0xFFFFu;


template <typename T>
__device__ __forceinline__ T ld_agent(const T* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}


// Workgroup barrier for LDS traffic only: waits for this wave's LDS operations,
// not for its global loads (__syncthreads waits vmcnt(0) too), so loads issued
// ahead -- the next chunk's input -- stay in flight across it.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <bool LDS_ONLY>
__device__ __forceinline__ void block_barrier() {
    if (LDS_ONLY)
        lds_barrier();
    else
        __syncthreads();
}

// Exclusive scan of cnt[0..n) in LDS (n <= FB_MAXBINS), one block of NT threads;
// returns the total.
template <int NT, bool LDS_ONLY = false>
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
    block_barrier<LDS_ONLY>();
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
    block_barrier<LDS_ONLY>();
    return total;
}

}  // namespace

// ---------------------------------------------------------------- A, B: binning passes
// Range binning (default).  A work item is a range of FBR_RANGE chunks of
// FBR_CHUNK messages (A: senders; B: one coarse bin's messages), one 1024-thread
// block per item:
//   sweep 1  keys of every message of the range (Philox), LDS counts per bin;
//            one global reservation per (range, bin) -- the range's messages of
//            a bin then occupy one contiguous run of that bin;
//   sweep 2  per chunk: loads in input order (coalesced), keys again, LDS rank
//            per bin, the chunk put in bin order in LDS (payload, header, slot),
//            written out in that order: consecutive threads write consecutive
//            slots of one bin, and consecutive chunks continue the same runs.
// No gather anywhere (the previous version gathered payloads in bin order from
// an input window larger than the XCD's L2), and reservations drop from one per
// (chunk, bin) to one per (range, bin).
// One 1024-thread block per CU (two per CU with spills: 4.40-4.52 against 3.70 ms/round; 512-
// thread blocks 4.45), ranges of 4 chunks (best of 2 / 4 / 8 / 16; profiles/r02/c4_v2/).
constexpr int FBR_THREADS = 1024;
constexpr int FBR_PER = 4;
constexpr int FBR_CHUNK = FBR_THREADS * FBR_PER;
constexpr int FB_RANGE = 4;
constexpr uint32_t FBR_ITEM = (uint32_t)FB_RANGE * FBR_CHUNK;  // messages per work item
static_assert(FB_RANGE % 2 == 0, "sweep 1 takes two chunks at a time");

struct FbRangeLds {
    double2 pay[FBR_CHUNK];     // the chunk's payloads in bin order
    uint32_t hdr[FBR_CHUNK];    // sender ids in bin order
    uint32_t pos[FBR_CHUNK];    // slot in the bin
    uint16_t key[FBR_CHUNK];    // bin
    uint32_t tmp[FBR_THREADS / 64];
};
// Dynamic LDS, 2 x nbins words (launch_full_bin_round): cnt = the chunk's count
// per bin, then its first LDS position; base = the range's count per bin, then
// the bin's next slot.
extern __shared__ uint32_t fbr_dyn[];

// Sweep 2's tail for one chunk whose keys / ranks are in registers: LDS bin
// order, running slots, coalesced write-out through store(bin, slot, header,
// payload).  LDS-only barriers, so the next chunk's loads (issued before this
// call) stay in flight.
template <class Store>
__device__ __forceinline__ void fbr_emit_to(FbRangeLds& L, uint32_t* cnt, uint32_t* base, uint32_t nbins,
                                            const uint32_t (&key)[FBR_PER], const uint32_t (&rank)[FBR_PER],
                                            const uint32_t (&hdr)[FBR_PER], const double2 (&pay)[FBR_PER],
                                            const Store& store) {
    const uint32_t total = lds_excl_scan<FBR_THREADS, true>(cnt, nbins, L.tmp);
#pragma unroll
    for (int k = 0; k < FBR_PER; ++k) {
        if (key[k] == FB_NONE) continue;
        const uint32_t p = cnt[key[k]] + rank[k];
        L.pay[p] = pay[k];
        L.hdr[p] = hdr[k];
        L.key[p] = (uint16_t)key[k];
        L.pos[p] = base[key[k]] + rank[k];
    }
    lds_barrier();
    for (uint32_t b = threadIdx.x; b < nbins; b += FBR_THREADS)
        base[b] += (b + 1 < nbins ? cnt[b + 1] : total) - cnt[b];
    // fixed trip count: a loop of unknown length would make the compiler wait for
    // every outstanding load (the next chunk's) before entering it
#pragma unroll
    for (int k = 0; k < FBR_PER; ++k) {
        const uint32_t p = k * FBR_THREADS + threadIdx.x;
        if (p >= total) break;
        store(L.key[p], L.pos[p], L.hdr[p], L.pay[p]);
    }
    lds_barrier();
}

// the bins as [nbins_out * cap] arrays from bin obin0 on (coarse bins, fine tiles)
__device__ __forceinline__ void fbr_emit(FbRangeLds& L, uint32_t* cnt, uint32_t* base, uint32_t nbins,
                                         const uint32_t (&key)[FBR_PER], const uint32_t (&rank)[FBR_PER],
                                         const uint32_t (&hdr)[FBR_PER], const double2 (&pay)[FBR_PER],
                                         uint32_t* __restrict__ ohdr, double2* __restrict__ opay, uint32_t cap,
                                         uint32_t obin0, uint32_t nbins_out, unsigned int* overflow) {
    fbr_emit_to(L, cnt, base, nbins, key, rank, hdr, pay, [&](uint32_t k, uint32_t pos, uint32_t h, double2 v) {
        const uint32_t b = obin0 + k;
        if (pos >= cap || b >= nbins_out) {
            atomicOr(overflow, 1u);
            return;
        }
        const size_t o = (size_t)b * cap + pos;
        ohdr[o] = h;
        opay[o] = v;
    });
}

// one global reservation per bin with messages in this range (base: count -> first slot)
__device__ __forceinline__ void fbr_reserve(uint32_t* base, uint32_t nbins, uint32_t* gcnt, uint32_t gbin0,
                                            uint32_t nbins_out) {
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nbins; b += FBR_THREADS) {
        const uint32_t n = base[b];
        base[b] = n && gbin0 + b < nbins_out ? atomicAdd(&gcnt[gbin0 + b], n) : 0u;
    }
}

// A's input of one chunk: node bytes and (s, w) of its senders.  Loads are
// unconditional (indices clamped into the range, validity tested at use), so
// no branch or phi makes the compiler wait for them -- or for the previous
// chunk's stores, which vmcnt also counts -- before they are consumed.
struct SendIn {
    uint8_t nbv[FBR_PER];
    double2 sv[FBR_PER];
    __device__ __forceinline__ void load(const FullBinArgs& a, uint64_t c0, uint64_t i1) {
#pragma unroll
        for (int k = 0; k < FBR_PER; ++k) {
            const uint64_t g = std::min<uint64_t>(c0 + k * FBR_THREADS + threadIdx.x, i1 - 1);
            nbv[k] = a.nb[g];
            sv[k] = a.swc[g];
        }
    }
};

__global__ __launch_bounds__(FBR_THREADS, 1) void k_fb_send(FullBinArgs a, uint32_t r) {
    __shared__ FbRangeLds L;
    if (ld_agent(&a.ctl->done)) return;
    const uint32_t P = a.P;
    const uint64_t i0 = (uint64_t)blockIdx.x * FBR_ITEM;
    if (i0 >= P || P < 2) return;
    const uint64_t i1 = std::min<uint64_t>(P, i0 + FBR_ITEM);
    uint32_t* const cnt = fbr_dyn;
    uint32_t* const base = fbr_dyn + a.nb1;
    for (uint32_t b = threadIdx.x; b < a.nb1; b += FBR_THREADS) base[b] = 0u;
    // sweep 2's first chunk is loaded now, in flight through sweep 1 and the reservations
    SendIn cur;
    cur.load(a, i0, i1);
    __syncthreads();
    // sweep 1: coarse bin (target >> s1) of every active sender, counted; two
    // chunks per iteration (one Philox batch of 2 FBR_PER).  The bins stay in
    // registers for sweep 2 (16-bit, two per word), so each message's Philox draw
    // is computed once per pass
    constexpr int P2 = 2 * FBR_PER;
    constexpr int NCH = FB_RANGE;  // chunks per work item
    uint32_t keys[NCH * FBR_PER / 2];
#pragma unroll
    for (int it = 0; it < NCH / 2; ++it) {
        const uint64_t c0 = i0 + (uint64_t)it * 2 * FBR_CHUNK;
        uint32_t node[P2], x[P2], y[P2];
        uint8_t nbv[P2];
#pragma unroll
        for (int k = 0; k < P2; ++k) {
            const uint64_t g = c0 + k * FBR_THREADS + threadIdx.x;
            node[k] = (uint32_t)g;
            nbv[k] = a.nb[std::min<uint64_t>(g, i1 - 1)];
        }
        philox2_batch<P2>(node, r, S_PUSHSUM, a.k0, a.k1, x, y);
#pragma unroll
        for (int k = 0; k < P2; k += 2) {
            uint32_t kk[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                kk[h] = FB_NONE;
                if ((nbv[k + h] & B_ACTIVE) && c0 + (k + h) * FBR_THREADS + threadIdx.x < i1) {  // Program.fs:213-215
                    kk[h] = full_target(node[k + h], uniform_from(x[k + h], y[k + h], P - 1)) >> a.s1;
                    atomicAdd(&base[kk[h]], 1u);
                }
            }
            keys[(it * P2 + k) / 2] = kk[0] | (kk[1] << 16);
        }
    }
    fbr_reserve(base, a.nb1, a.cnt1, 0, a.nb1);
    // sweep 2: {sender id | s/2, w/2} into the runs; the next chunk's input is
    // loaded while this one is put in order and written
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
        const uint64_t c0 = i0 + (uint64_t)ch * FBR_CHUNK;
        if (c0 >= i1) break;
        for (uint32_t b = threadIdx.x; b < a.nb1; b += FBR_THREADS) cnt[b] = 0u;
        uint32_t node[FBR_PER], key[FBR_PER], rank[FBR_PER];
        double2 pay[FBR_PER];
#pragma unroll
        for (int k = 0; k < FBR_PER; ++k) node[k] = (uint32_t)(c0 + k * FBR_THREADS + threadIdx.x);
        lds_barrier();  // counters zeroed
#pragma unroll
        for (int k = 0; k < FBR_PER; ++k) {
            const int m = ch * FBR_PER + k;
            key[k] = (keys[m / 2] >> (16 * (m & 1))) & 0xFFFFu;
            rank[k] = key[k] != FB_NONE ? atomicAdd(&cnt[key[k]], 1u) : 0u;
            pay[k] = make_double2(cur.sv[k].x * 0.5, cur.sv[k].y * 0.5);
        }
        cur.load(a, c0 + FBR_CHUNK < i1 ? c0 + FBR_CHUNK : c0, i1);  // (the last chunk reloads itself)
        lds_barrier();  // ranks counted
        fbr_emit(L, cnt, base, a.nb1, key, rank, node, pay, a.hdr1, a.pay1, a.cap1, 0, a.nb1, a.overflow);
    }
}

// B's input of one chunk: sender ids and payloads of a coarse bin's messages
// (unconditional loads, as SendIn)
struct SplitIn {
    uint32_t node[FBR_PER];
    double2 pv[FBR_PER];
    __device__ __forceinline__ void load(const uint32_t* hdr, const double2* pay, size_t base, uint32_t c0, uint32_t q1) {
#pragma unroll
        for (int k = 0; k < FBR_PER; ++k) {
            const uint32_t q = min(c0 + k * FBR_THREADS + threadIdx.x, q1 - 1);
            node[k] = hdr[base + q];
            pv[k] = pay[base + q];
        }
    }
};

// One rank: work items are ranges of each coarse bin of hdr1 / pay1.  MULTI (several ranks, one
// launch per exchange region): ranges of every source rank's bins in the region's received
// buffers (in[p], items from in_item0[p]) -- a coarse bin's messages arrive from every source
// and region, each range reserves its own runs in the fine tiles.
template <bool MULTI>
__global__ __launch_bounds__(FBR_THREADS, 1) void k_fb_split(FullBinArgs a, uint32_t r) {
    __shared__ FbRangeLds L;
    if (ld_agent(&a.ctl->done)) return;
    uint32_t b, c, n_bin;
    const uint32_t* bin_hdr;  // the coarse bins' sender ids and payloads; this bin's from ibase on
    const double2* bin_pay;
    size_t ibase;
    if constexpr (MULTI) {
        int p = 0;
        while (p + 1 < a.W && blockIdx.x >= a.in_item0[p + 1]) ++p;  // block-uniform
        p = __builtin_amdgcn_readfirstlane(p);
        const uint32_t cap = a.in[p].cap;
        if (!cap) return;
        const uint32_t per_bin = (cap + FBR_ITEM - 1) / FBR_ITEM, item = blockIdx.x - a.in_item0[p];
        b = item / per_bin;
        c = item % per_bin;
        if (b >= a.in[p].nb) return;
        n_bin = min(ld_agent(&a.in[p].cnt[b]), cap);
        bin_hdr = a.in[p].hdr;
        bin_pay = a.in[p].pay;
        ibase = (size_t)b * cap;
    } else {
        const uint32_t per_bin = (a.cap1 + FBR_ITEM - 1) / FBR_ITEM;
        b = blockIdx.x / per_bin;
        c = blockIdx.x % per_bin;
        n_bin = min(ld_agent(&a.cnt1[b]), a.cap1);
        bin_hdr = a.hdr1;
        bin_pay = a.pay1;
        ibase = (size_t)b * a.cap1;
    }
    // (ranges of whole items: dealing a bin's messages evenly over its items measured slower,
    // C4 at W = 8 0.087 -> 0.095 ms per region's split -- more partly filled chunks)
    const uint32_t q0 = c * FBR_ITEM;
    if (q0 >= n_bin) return;
    const uint32_t q1 = min(n_bin, q0 + FBR_ITEM);
    const uint32_t nfine = 1u << (a.s1 - FB_TB), f0 = b << (a.s1 - FB_TB);
    uint32_t* const cnt = fbr_dyn;
    uint32_t* const base = fbr_dyn + nfine;
    for (uint32_t f = threadIdx.x; f < nfine; f += FBR_THREADS) base[f] = 0u;
    SplitIn cur;  // sweep 2's first chunk, in flight through sweep 1 and the reservations
    cur.load(bin_hdr, bin_pay, ibase, q0, q1);
    __syncthreads();
    // sweep 1: fine tile of every message (target recomputed from the sender's
    // draw), two chunks per iteration; the tiles stay in registers for sweep 2
    constexpr int P2 = 2 * FBR_PER;
    constexpr int NCH = FB_RANGE;
    uint32_t keys[NCH * FBR_PER / 2];
#pragma unroll
    for (int it = 0; it < NCH / 2; ++it) {
        const uint32_t c0 = q0 + it * 2 * FBR_CHUNK;
        uint32_t node[P2], x[P2], y[P2];
#pragma unroll
        for (int k = 0; k < P2; ++k) node[k] = bin_hdr[ibase + min(c0 + k * FBR_THREADS + threadIdx.x, q1 - 1)];
        philox2_batch<P2>(node, r, S_PUSHSUM, a.k0, a.k1, x, y);
#pragma unroll
        for (int k = 0; k < P2; k += 2) {
            uint32_t kk[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                kk[h] = FB_NONE;
                if (c0 + (k + h) * FBR_THREADS + threadIdx.x < q1) {
                    kk[h] = ((full_target(node[k + h], uniform_from(x[k + h], y[k + h], a.P - 1)) - a.lo) >> FB_TB) &
                            (nfine - 1u);
                    atomicAdd(&base[kk[h]], 1u);
                }
            }
            keys[(it * P2 + k) / 2] = kk[0] | (kk[1] << 16);
        }
    }
    fbr_reserve(base, nfine, a.cnt2, f0, a.nb2);
    // sweep 2: into the fine tiles' runs, the next chunk loaded meanwhile
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
        const uint32_t c0 = q0 + ch * FBR_CHUNK;
        if (c0 >= q1) break;
        for (uint32_t f = threadIdx.x; f < nfine; f += FBR_THREADS) cnt[f] = 0u;
        uint32_t node[FBR_PER], key[FBR_PER], rank[FBR_PER];
        double2 pay[FBR_PER];
#pragma unroll
        for (int k = 0; k < FBR_PER; ++k) {
            node[k] = cur.node[k];
            pay[k] = cur.pv[k];
        }
        lds_barrier();  // counters zeroed
#pragma unroll
        for (int k = 0; k < FBR_PER; ++k) {
            const int m = ch * FBR_PER + k;
            key[k] = (keys[m / 2] >> (16 * (m & 1))) & 0xFFFFu;
            rank[k] = key[k] != FB_NONE ? atomicAdd(&cnt[key[k]], 1u) : 0u;
        }
        cur.load(bin_hdr, bin_pay, ibase, c0 + FBR_CHUNK < q1 ? c0 + FBR_CHUNK : c0, q1);
        lds_barrier();  // ranks counted
        fbr_emit(L, cnt, base, nfine, key, rank, node, pay, a.hdr2, a.pay2, a.cap2, f0, a.nb2, a.overflow);
    }
}

// ---------------------------------------------------------------- several ranks
// Contiguous id slabs (gp_api.hip make_bounds); W <= XMAXW.  Every rank's coarse bins
// have the size 2^s1 (full_bin_multi_s1), so a message to target t has the LDS key
// kb(b) + ((t - bounds[b]) >> s1), b = owner of t, kb(b) = the bins of the ranks below b:
// key order = destination rank, then the destination's coarse bin.
__device__ __forceinline__ uint32_t multi_key(const FullBinArgs& a, uint32_t t) {
    uint32_t base = 0, kb = 0;
    for (int w = 1; w < a.W; ++w)
        if (t >= a.bounds[w]) {
            base = a.bounds[w];
            kb += a.out[w - 1].nb;
        }
    return kb + ((t - base) >> a.s1);
}

constexpr uint32_t FBF_MAXB1 = 1024;  // keys (coarse bins) the fold's send phase can bin into (LDS reservation slots)

// A block's destination bins, in LDS: indexing the kernel arguments by a per-lane rank
// would be a global load per message.
struct MultiOutLds {
    uint32_t* cnt[XMAXW];
    uint32_t* hdr[XMAXW];
    double2* pay[XMAXW];
    uint32_t cap[XMAXW];
    uint32_t kb[XMAXW + 1];   // first key of rank b; kb[W] = keys
    uint8_t keyb[FBF_MAXB1];  // the rank of every key
    __device__ void init(const FullBinArgs& a) {
        if (threadIdx.x == 0) {
            uint32_t k = 0;
            for (int b = 0; b < a.W; ++b) {
                cnt[b] = a.out[b].cnt;
                hdr[b] = a.out[b].hdr;
                pay[b] = a.out[b].pay;
                cap[b] = a.out[b].cap;
                kb[b] = k;
                k += a.out[b].nb;
            }
            kb[a.W] = k;
        }
        __syncthreads();
        for (uint32_t q = threadIdx.x; q < kb[a.W] && q < FBF_MAXB1; q += blockDim.x) {
            uint32_t b = 0;
            for (int w = 1; w < a.W; ++w) b += q >= kb[w] ? 1u : 0u;
            keyb[q] = (uint8_t)b;
        }
        __syncthreads();
    }
    // message `pos` of key q's run: false (and the overflow flag) beyond the bin's capacity
    __device__ __forceinline__ void store(uint32_t q, uint32_t pos, uint32_t h, double2 v, unsigned int* overflow) {
        const uint32_t b = keyb[q], c = q - kb[b];
        if (pos >= cap[b]) {
            atomicOr(overflow, 1u);
            return;
        }
        const size_t o = (size_t)c * cap[b] + pos;
        *gptr(hdr[b] + o) = h;
        st_global(pay[b] + o, v);
    }
};

// A on several ranks, round 0 (later rounds' messages are binned by the fold): the senders
// lo + [s_lo, s_hi) (one exchange region) binned by key straight into the region's exchange
// buffers -- {sender id | s/2, w/2}, one reservation per (range, key) on the bin's in-band
// counter; rank me's share goes to its own receive region.  Receivers recompute targets from
// the sender's Philox draw.
__global__ __launch_bounds__(FBR_THREADS, 1) void k_fbm_send(FullBinArgs a, uint32_t r) {
    __shared__ FbRangeLds L;
    __shared__ MultiOutLds O;
    if (ld_agent(&a.ctl->done)) return;
    const uint32_t P = a.P;
    const uint64_t i0 = (uint64_t)a.s_lo + (uint64_t)blockIdx.x * FBR_ITEM;
    if (i0 >= a.s_hi || P < 2) return;
    const uint64_t i1 = std::min<uint64_t>(a.s_hi, i0 + FBR_ITEM);
    O.init(a);
    const uint32_t nk = O.kb[a.W];
    uint32_t* const cnt = fbr_dyn;
    uint32_t* const base = fbr_dyn + nk;
    for (uint32_t q = threadIdx.x; q < nk; q += FBR_THREADS) base[q] = 0u;
    SendIn cur;
    cur.load(a, i0, i1);
    __syncthreads();
    // sweep 1: key of every active sender, counted
    for (uint64_t c0 = i0; c0 < i1; c0 += FBR_CHUNK) {
        uint32_t node[FBR_PER], x[FBR_PER], y[FBR_PER];
        uint8_t nbv[FBR_PER];
#pragma unroll
        for (int k = 0; k < FBR_PER; ++k) {
            const uint64_t g = c0 + k * FBR_THREADS + threadIdx.x;
            node[k] = a.lo + (uint32_t)g;
            nbv[k] = a.nb[std::min<uint64_t>(g, i1 - 1)];
        }
        philox2_batch<FBR_PER>(node, r, S_PUSHSUM, a.k0, a.k1, x, y);
#pragma unroll
        for (int k = 0; k < FBR_PER; ++k)
            if ((nbv[k] & B_ACTIVE) && c0 + k * FBR_THREADS + threadIdx.x < i1)  // Program.fs:213-215
                atomicAdd(&base[multi_key(a, full_target(node[k], uniform_from(x[k], y[k], P - 1)))], 1u);
    }
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < nk; q += FBR_THREADS) {
        const uint32_t n = base[q], b = O.keyb[q];
        base[q] = n ? __hip_atomic_fetch_add(gptr(O.cnt[b] + (q - O.kb[b])), n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    }
    // sweep 2: into the bins' runs
    for (uint64_t c0 = i0; c0 < i1; c0 += FBR_CHUNK) {
        for (uint32_t q = threadIdx.x; q < nk; q += FBR_THREADS) cnt[q] = 0u;
        uint32_t node[FBR_PER], x[FBR_PER], y[FBR_PER], key[FBR_PER], rank[FBR_PER];
        double2 pay[FBR_PER];
#pragma unroll
        for (int k = 0; k < FBR_PER; ++k) node[k] = a.lo + (uint32_t)(c0 + k * FBR_THREADS + threadIdx.x);
        philox2_batch<FBR_PER>(node, r, S_PUSHSUM, a.k0, a.k1, x, y);
        lds_barrier();  // counters zeroed
#pragma unroll
        for (int k = 0; k < FBR_PER; ++k) {
            key[k] = FB_NONE;
            rank[k] = 0;
            if ((cur.nbv[k] & B_ACTIVE) && c0 + k * FBR_THREADS + threadIdx.x < i1) {
                key[k] = multi_key(a, full_target(node[k], uniform_from(x[k], y[k], P - 1)));
                rank[k] = atomicAdd(&cnt[key[k]], 1u);
            }
            pay[k] = make_double2(cur.sv[k].x * 0.5, cur.sv[k].y * 0.5);
        }
        cur.load(a, c0 + FBR_CHUNK < i1 ? c0 + FBR_CHUNK : c0, i1);
        lds_barrier();  // ranks counted
        fbr_emit_to(L, cnt, base, nk, key, rank, node, pay,
                    [&](uint32_t q, uint32_t pos, uint32_t h, double2 v) { O.store(q, pos, h, v, a.overflow); });
    }
}

// Several ranks: the counters a round fills, cleared in one launch (ZeroList: block k clears
// list entry k).
__global__ __launch_bounds__(256) void k_zero_list(ZeroList z) {
    uint32_t* p = z.p[blockIdx.x];
    const uint32_t n = z.n[blockIdx.x];
    for (uint32_t c = threadIdx.x; c < n; c += 256) p[c] = 0u;
}

// ---------------------------------------------------------------- C: fold per fine tile
// One fine tile per block.  The tile's messages (sender id + payload) are loaded
// in bin order, coalesced, together with the receivers' own bytes and (s, w);
// targets recomputed as one Philox batch; LDS counting sort by receiver puts
// sender ids and payloads in receiver order; each receiver's (few) messages are
// put in ascending sender order (insertion sort of (sender, LDS position)) and
// folded from LDS -- no gather of the bin's payloads from global memory.
constexpr int FBF_THREADS = 1024;  // (256-thread fold blocks: 3.76 against 3.70 ms/round, profiles/r02/c4_v2/)

//
// Send phase (FOLD_SEND, one rank, FullBinArgs::fused): after a tile is folded, its
// nodes' sends of round r+1 are binned straight from the registers that hold the new
// state -- the active flag and (s, w) the fold just wrote (Program.fs:104-106,125-128
// one round on) -- into the coarse bins of A, as k_fb_send would bin them: target
// from the node's Philox draw for round r+1, {id | s/2, w/2}, LDS bin order (reusing
// the fold's arrays), one reservation per (tile, bin), coalesced runs.  The next round
// then starts at B: no send pass re-reads the state (18 B/node).
// FOLD_SEND_RANKS (several ranks, round 6): the same send phase with the destination
// rank as the first level of the key (multi_key), into the exchange region's buffers
// (out[b]) -- the fold of a region's tiles produces that region's exchange, so no send
// pass re-reads the state and no coarse pass re-bins the received messages.
enum FoldMode { FOLD = 0, FOLD_SEND = 1, FOLD_SEND_RANKS = 2 };

template <int MODE>
__global__ __launch_bounds__(FBF_THREADS) void k_fb_fold(FullBinArgs a, uint32_t r) {
    constexpr bool SEND = MODE != FOLD;
    constexpr bool RANKS = MODE == FOLD_SEND_RANKS;
    constexpr int TILE = 1 << FB_TB;
    constexpr int NPT = TILE / FBF_THREADS;
    constexpr int FQ = (FB_CAP2 + FBF_THREADS - 1) / FBF_THREADS;
    static_assert(TILE <= FB_CAP2 && FBF_MAXB1 <= TILE, "the fused send reuses msg / src / idx / cnt");
    static_assert(!SEND || NPT % 2 == 0, "the fused send packs two coarse bins per word");
    __shared__ uint32_t cnt[TILE + 1];            // per receiver: count, then start
    __shared__ double2 msg[FB_CAP2];              // payloads in receiver order
    __shared__ uint32_t src[FB_CAP2];             // sender ids in receiver order, sorted per receiver
    __shared__ uint16_t idx[FB_CAP2];             // the message's slot in msg, permuted with src
    __shared__ uint32_t tmp[FBF_THREADS / 64];
    __shared__ uint32_t red[2][FBF_THREADS / 64];
    __shared__ uint32_t sbase[SEND ? FBF_MAXB1 : 1];  // send phase: the tile's run start per key
    __shared__ MultiOutLds O[1];  // (FOLD_SEND_RANKS only; unreferenced otherwise)
    Ctl* ctl = a.ctl;
    if (ld_agent(&ctl->done)) return;
    const uint32_t P = a.P;
    const double2* __restrict__ swc = a.swc;
    double2* __restrict__ swn = a.swn;
    uint8_t* __restrict__ nbp = a.nb;
    uint32_t alerts = 0, newly = 0;
    uint32_t nkeys = a.nb1;  // send phase: keys of the LDS bins
    if constexpr (RANKS) {
        O[0].init(a);
        nkeys = O[0].kb[a.W];
    }
    for (uint32_t v = threadIdx.x; v < TILE; v += FBF_THREADS) cnt[v] = 0u;
    __syncthreads();
    // the tile's messages (sender ids, payloads) -- send phase: the next tile's are loaded
    // while this tile's messages of round r+1 are scattered and written out (round 5: C4
    // 3.158 / 3.165 -> 3.083 / 3.079 ms/round, same box, profiles/r05/c4/)
    uint32_t snd[FQ];
    double ps[FQ], pw[FQ];  // (two scalar arrays: a double2 array here went to scratch)
    auto load_msgs = [&](uint32_t f, uint32_t n) {
        const size_t base = (size_t)f * a.cap2;
#pragma unroll
        for (int k = 0; k < FQ; ++k) {
            const uint32_t q = min((uint32_t)(k * FBF_THREADS + threadIdx.x), n > 0 ? n - 1 : 0u);
            snd[k] = a.hdr2[base + q];
            const double2 m = a.pay2[base + q];
            ps[k] = m.x;
            pw[k] = m.y;
        }
    };
    const uint32_t t_hi = a.t_hi;
    uint32_t n_pf = 0;
    if (SEND && a.t_lo + blockIdx.x < t_hi) {
        n_pf = min(ld_agent(&a.cnt2[a.t_lo + blockIdx.x]), (uint32_t)a.cap2);
        load_msgs(a.t_lo + blockIdx.x, n_pf);
    }
    for (uint32_t f = a.t_lo + blockIdx.x; f < t_hi; f += gridDim.x) {
        constexpr bool pf = SEND;
        const uint32_t n = pf ? n_pf : min(ld_agent(&a.cnt2[f]), (uint32_t)a.cap2);
        // the next tile's message count, early (a scalar load; its messages are loaded later)
        const uint32_t fn = f + gridDim.x;
        // (a scalar load: an agent-scope vector load here was waited for at once, and with it
        // every store of the last tile's write-out)
        if (pf) n_pf = fn < t_hi ? min(ld_const(a.cnt2 + fn), (uint32_t)a.cap2) : 0u;
        // every load of the tile in flight at once (indices clamped, validity at use)
        uint32_t x[FQ], y[FQ], vr[FQ], rk[FQ];
        uint8_t bk[NPT];
        double2 svk[NPT];
        uint32_t nfl[NPT];  // send phase: active in round r+1, and the half it sends
        double2 nsw[NPT];
        if (!pf) load_msgs(f, n);
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
            const uint32_t j = min(f * TILE + k * FBF_THREADS + threadIdx.x, a.nloc - 1);
            bk[k] = nbp[j];
            svk[k] = swc[j];
        }
        // send phase: the key of each of this thread's nodes' round-r+1 targets, drawn while
        // the tile's loads are in flight (whether the node sends is known after the fold)
        uint32_t nkey[SEND ? NPT / 2 : 1];
        if (SEND) {
            uint32_t node[NPT], xs[NPT], ys[NPT];
#pragma unroll
            for (int k = 0; k < NPT; ++k) node[k] = a.lo + f * TILE + k * FBF_THREADS + threadIdx.x;
            philox2_batch<NPT>(node, r + 1, S_PUSHSUM, a.k0, a.k1, xs, ys);
            auto key_of = [&](int k) -> uint32_t {
                if (P < 2) return 0u;
                const uint32_t t = full_target(node[k], uniform_from(xs[k], ys[k], P - 1));
                if constexpr (RANKS) return multi_key(a, t);
                return t >> a.s1;
            };
#pragma unroll
            for (int k = 0; k < NPT; k += 2) nkey[k / 2] = key_of(k) | (key_of(k + 1) << 16);
        }
        philox2_batch<FQ>(snd, r, S_PUSHSUM, a.k0, a.k1, x, y);
#pragma unroll
        for (int k = 0; k < FQ; ++k) {
            const uint32_t q = k * FBF_THREADS + threadIdx.x;
            vr[k] = (full_target(snd[k], uniform_from(x[k], y[k], P - 1)) - a.lo) & (TILE - 1);
            rk[k] = q < n ? atomicAdd(&cnt[vr[k]], 1u) : 0u;
        }
        lds_barrier();
        lds_excl_scan<FBF_THREADS, true>(cnt, TILE, tmp);
        if (threadIdx.x == 0) cnt[TILE] = n;
#pragma unroll
        for (int k = 0; k < FQ; ++k) {
            if (k * FBF_THREADS + threadIdx.x < n) {
                const uint32_t p = cnt[vr[k]] + rk[k];
                src[p] = snd[k];
                msg[p] = make_double2(ps[k], pw[k]);
            }
        }
        lds_barrier();
        // per receiver after its fold: ratio test, flags, state out (and the send phase's inputs)
        auto close_receiver = [&](int k, uint32_t p0, uint32_t p1, double acc_s, double acc_w) {
            const uint32_t j = f * TILE + k * FBF_THREADS + threadIdx.x;
            const uint8_t b = bk[k];
            const double2 sv = svk[k];
            const bool active = (b & B_ACTIVE) != 0;
            if (p1 > p0) {
                uint32_t flags = b;
                if (!(b & B_CONV)) {
                    uint32_t c = (b >> CNT_SHIFT) & 3u;
                    c = ratio_moved(sv.x, sv.y, acc_s, acc_w) ? 0u : c + 1u;
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
            if (j < a.nloc) swn[j] = make_double2(acc_s, acc_w);
            if (SEND) {
                nfl[k] = j < a.nloc && P > 1 && (b & B_ACTIVE || p1 > p0) ? 1u : 0u;  // active next round
                nsw[k] = make_double2(acc_s * 0.5, acc_w * 0.5);
            }
        };
        // this receiver's messages in ascending sender id (canonical order): insertion sort
        auto sort_receiver = [&](uint32_t p0, uint32_t p1) {
            for (uint32_t p = p0 + 1; p < p1; ++p) {
                const uint32_t s = src[p];
                const double2 mv = msg[p];
                uint32_t q = p;
                while (q > p0 && src[q - 1] > s) {
                    src[q] = src[q - 1];
                    msg[q] = msg[q - 1];
                    --q;
                }
                src[q] = s;
                msg[q] = mv;
            }
        };
        // FG receivers folded in lock step (one LDS chain each in flight, each receiver's own
        // order kept): C4 3.177 -> 3.165 ms/round against one after the other, same box
        // (profiles/r05/c4/ilp.txt); their insertion sorts in lock step too +10 %
        // (profiles/r05/rejected/c4_sort_ilp.txt)
        constexpr int FG = 2;
        static_assert(FG >= 1 && NPT % FG == 0, "fold groups");
#pragma unroll
        for (int g0 = 0; g0 < NPT; g0 += FG) {
            uint32_t fp0[FG], fp1[FG];
            double fs[FG], fw[FG];
            uint32_t most = 0;
#pragma unroll
            for (int i = 0; i < FG; ++i) {
                const int k = g0 + i;
                const uint32_t v = k * FBF_THREADS + threadIdx.x;
                const uint32_t j = f * TILE + v;
                fp0[i] = cnt[v];
                fp1[i] = j < a.nloc ? cnt[v + 1] : fp0[i];
                sort_receiver(fp0[i], fp1[i]);
                most = max(most, fp1[i] - fp0[i]);
                const bool active = (bk[k] & B_ACTIVE) != 0;
                fs[i] = active && P > 1 ? svk[k].x * 0.5 : svk[k].x;
                fw[i] = active && P > 1 ? svk[k].y * 0.5 : svk[k].y;
            }
            for (uint32_t t = 0; t < most; ++t) {
                double2 m[FG];
#pragma unroll
                for (int i = 0; i < FG; ++i) m[i] = msg[min(fp0[i] + t, (uint32_t)FB_CAP2 - 1u)];
#pragma unroll
                for (int i = 0; i < FG; ++i) {
                    const bool ok = fp0[i] + t < fp1[i];
                    fs[i] = fs[i] + (ok ? m[i].x : 0.0);  // already halved by the sender
                    fw[i] = fw[i] + (ok ? m[i].y : 0.0);
                }
            }
#pragma unroll
            for (int i = 0; i < FG; ++i) close_receiver(g0 + i, fp0[i], fp1[i], fs[i], fw[i]);
        }
        lds_barrier();
        for (uint32_t v = threadIdx.x; v < TILE; v += FBF_THREADS) cnt[v] = 0u;
        lds_barrier();
        if (SEND) {
            // round r+1: the key of every active node's target (drawn above), LDS rank per key
            uint32_t node[NPT], key[NPT], rank[NPT];
#pragma unroll
            for (int k = 0; k < NPT; ++k) {
                node[k] = a.lo + f * TILE + k * FBF_THREADS + threadIdx.x;
                key[k] = FB_NONE;
                rank[k] = 0u;
                if (nfl[k]) {
                    key[k] = (nkey[k / 2] >> (16 * (k & 1))) & 0xFFFFu;
                    rank[k] = atomicAdd(&cnt[key[k]], 1u);
                }
            }
            lds_barrier();
            const uint32_t total = lds_excl_scan<FBF_THREADS, true>(cnt, nkeys, tmp);  // count -> first LDS position
            // one reservation per (tile, key), thread q for key q (keys <= FBF_MAXB1 <= threads);
            // the returned offset is stored after the LDS scatter, so the atomic's round
            // trip overlaps it
            static_assert(FBF_MAXB1 <= FBF_THREADS, "one key per thread");
            uint32_t res = 0u;
            uint32_t q0 = threadIdx.x;
            asm volatile("" : "+v"(q0));  // (the reservation address is not hoisted out of the tile loop and spilled)
            if (q0 < nkeys) {
                const uint32_t n = (q0 + 1 < nkeys ? cnt[q0 + 1] : total) - cnt[q0];
                if (n) {
                    if constexpr (RANKS) {
                        const uint32_t b = O[0].keyb[q0];
                        res = __hip_atomic_fetch_add(gptr(O[0].cnt[b] + (q0 - O[0].kb[b])), n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    } else {
                        res = atomicAdd(&a.cnt1[q0], n);
                    }
                }
            }
            // the next tile's messages, issued after the reservation (so that waiting for its
            // result does not wait for them) and in flight through the scatter and write-out.
            // Unconditional (the last tile reloads its own): with the loads on one path only,
            // the compiler's wait for the reservation became vmcnt(0), i.e. for them too
            load_msgs(fn < t_hi ? fn : f, n_pf);
#pragma unroll
            for (int k = 0; k < NPT; ++k) {
                if (key[k] == FB_NONE) continue;
                const uint32_t p = cnt[key[k]] + rank[k];
                src[p] = node[k];
                msg[p] = nsw[k];
                idx[p] = (uint16_t)key[k];
            }
            if (q0 < nkeys) sbase[q0] = res;
            // the reservation retired on every path -- only the 2 FQ message loads above may still
            // be in flight -- so no later register reuse makes the compiler wait for those loads
            // or for the write-out's stores below
            __builtin_amdgcn_s_waitcnt(vmcnt_enc(2 * FQ));
            lds_barrier();
            // write-out in key order: consecutive threads, consecutive slots of one run.  One
            // rank: two stores per slot k on every lane (a lane without a message writes the junk
            // slots past the last bin), so the wait for the next tile's messages, loaded before
            // these stores, is an exact count and does not wait for the stores to be acknowledged
            bool ovf = false;
#pragma unroll
            for (int k = 0; k < NPT; ++k) {
                const uint32_t p = k * FBF_THREADS + threadIdx.x;
                if constexpr (RANKS) {
                    if (p >= total) break;
                    const uint32_t q = idx[p];
                    O[0].store(q, sbase[q] + (p - cnt[q]), src[p], msg[p], a.overflow);
                } else {
                    const bool has = p < total;
                    const uint32_t q = has ? idx[p] : 0u;
                    const uint32_t slot = sbase[q] + (p - cnt[q]);
                    ovf |= has && slot >= a.cap1;
                    const size_t o = has && slot < a.cap1 ? (size_t)q * a.cap1 + slot
                                                          : (size_t)a.nb1 * a.cap1 + (threadIdx.x & (FB_JUNK - 1));
                    a.hdr1[o] = src[p];
                    a.pay1[o] = msg[p];
                }
            }
            if (ovf) atomicOr(a.overflow, 1u);
            lds_barrier();
            for (uint32_t v = threadIdx.x; v < nkeys; v += FBF_THREADS) cnt[v] = 0u;
            lds_barrier();
        }
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
        for (int w = 0; w < FBF_THREADS / 64; ++w) {
            x += red[0][w];
            y += red[1][w];
        }
        if (x) atomicAdd(&ctl->round_alerts, (unsigned long long)x);
        if (y) atomicAdd(&ctl->round_active, (unsigned long long)y);
    }
}

// ---------------------------------------------------------------- host side
// Bins for the nrecv receivers of a rank (one rank: nrecv = P).
FullBinPlan full_bin_plan(uint32_t P, bool fused) {
    FullBinPlan p{};
    uint32_t bits = 1;
    while (bits < 32 && ((uint64_t)1 << bits) < P) ++bits;
    // coarse bins ~ sqrt(P / TILE) so both passes write runs of ~10-20 messages;
    // at most FB_MAXBINS coarse bins and FB_MAXBINS fine tiles per coarse bin.  The
    // fused fold (one rank) takes coarse bins half that size: the split's runs get
    // longer and the fold's shorter; P = 1e8, same box: rule 3.37, -1 3.26, -2 3.25,
    // -3 3.38-3.40 ms/round (profiles/r04/c4_fused/s1_sweep.txt)
    uint32_t s1 = (bits + FB_TB + 1) / 2 - (fused ? 1u : 0u);
    if (s1 < FB_TB) s1 = FB_TB;
    while (((uint64_t)P >> s1) >= FB_MAXBINS) ++s1;
    while (fused && (((uint64_t)P + (1ull << s1) - 1) >> s1) > FBF_MAXB1) ++s1;
    while (s1 - FB_TB > 12) --s1;
    p.s1 = s1;
    p.nb1 = (uint32_t)(((uint64_t)P + (1ull << s1) - 1) >> s1);
    p.nb2 = (uint32_t)(((uint64_t)P + (1u << FB_TB) - 1) >> FB_TB);
    const double m1 = (double)(1ull << s1) * ((double)P / (double)(P > 1 ? P - 1 : 1));
    p.cap1 = (uint32_t)(m1 + 12.0 * std::sqrt(m1) + 1024.0);
    p.cap2 = FB_CAP2;
    return p;
}

// Several ranks: the smallest coarse-bin size (>= a fine tile) that keeps the keys of all ranks'
// bins together at most FBM_KEYS -- about the one-rank fused fold's 191 bins at C4, whose runs
// (~21 messages per (tile, key)) measured best there; larger bins also carry less 12-sigma
// padding through the exchange (C4 at W = 8: 2^19 receivers, 24 bins per rank, +6.8 %).
constexpr uint32_t FBM_KEYS = 192;
uint32_t full_bin_multi_s1(const uint32_t* bounds, int W) {
    uint32_t s1 = FB_TB;
    for (;; ++s1) {
        uint64_t keys = 0;
        for (int b = 0; b < W; ++b) keys += ((uint64_t)(bounds[b + 1] - bounds[b]) + (1ull << s1) - 1) >> s1;
        if (keys <= FBM_KEYS || s1 - FB_TB >= 12) break;
    }
    return s1;
}

uint32_t full_bin_multi_cap(uint32_t n, uint32_t s1, uint32_t P) {
    const double m = (double)n * (double)(1ull << s1) / (double)(P > 1 ? P - 1 : 1);
    return (uint32_t)std::min<double>(std::ceil(m + 12.0 * std::sqrt(m) + 64.0), (double)n);
}

size_t fb_bins_bytes(uint32_t nb, uint32_t cap) {
    if (!nb || !cap) return 0;
    const size_t c = ((size_t)nb * 4 + 15) & ~(size_t)15, h = ((size_t)nb * cap * 4 + 15) & ~(size_t)15;
    return c + h + (size_t)nb * cap * 16;
}

FbBins fb_bins_at(uint8_t* base, uint32_t nb, uint32_t cap) {
    FbBins f{};
    if (!nb || !cap) return f;
    const size_t c = ((size_t)nb * 4 + 15) & ~(size_t)15, h = ((size_t)nb * cap * 4 + 15) & ~(size_t)15;
    f.cnt = reinterpret_cast<uint32_t*>(base);
    f.hdr = reinterpret_cast<uint32_t*>(base + c);
    f.pay = reinterpret_cast<double2*>(base + c + h);
    f.cap = cap;
    f.nb = nb;
    return f;
}

uint32_t full_bin_item_messages() {
    return FBR_ITEM;
}

hipError_t launch_full_bin_send_multi(const FullBinArgs& a, uint32_t round, hipStream_t st) {
    const uint32_t items = (uint32_t)(((uint64_t)(a.s_hi - a.s_lo) + FBR_ITEM - 1) / FBR_ITEM);
    if (items) hipLaunchKernelGGL(k_fbm_send, dim3(items), dim3(FBR_THREADS), 2 * sizeof(uint32_t) * FBF_MAXB1, st, a, round);
    return hipGetLastError();
}

hipError_t launch_zero_list(const ZeroList& z, hipStream_t st) {
    if (z.k > 0) hipLaunchKernelGGL(k_zero_list, dim3(z.k), dim3(256), 0, st, z);
    return hipGetLastError();
}

hipError_t launch_full_bin_split_multi(const FullBinArgs& a, uint32_t round, hipStream_t st) {
    if (a.in_item0[a.W])
        hipLaunchKernelGGL(k_fb_split<true>, dim3(a.in_item0[a.W]), dim3(FBR_THREADS),
                           2 * sizeof(uint32_t) * (1u << (a.s1 - FB_TB)), st, a, round);
    return hipGetLastError();
}

// C's grid, one rank: two blocks per CU's worth (the bulk grid is 64 blocks of 256 threads per
// CU), each walking ~P / 2^FB_TB / 512 tiles.  P = 1e8, same box: 4096 / 2048 / 1024 / 512 / 256 blocks
// 3.16-3.18 / 3.145-3.147 / 3.137-3.145 / 3.130-3.138 / 3.143-3.147 ms/round once the GPU is
// warm, one tile per block 3.28 (profiles/r04/c4_fused/fold_grid.txt)
static uint32_t fold_blocks(uint32_t tiles, int grid) {
    return std::max<uint32_t>(1, std::min<uint32_t>(tiles, (uint32_t)grid * 256 / FBF_THREADS / 8));
}

// Several ranks: the fold of one exchange region's tiles [t_lo, t_hi), binning their next-round
// messages into the region's exchange buffers; one block per CU (the block holds the CU's LDS),
// each walking its ~tiles / CUs tiles with the next one's messages prefetched -- a region has
// only ~1500 tiles at C4 / W = 8, so a second wave of blocks would pay every block's start-up
// and unprefetched first tile twice.
hipError_t launch_full_bin_fold_multi(const FullBinArgs& a, uint32_t round, int cus, hipStream_t st) {
    if (a.t_hi > a.t_lo)
        hipLaunchKernelGGL(k_fb_fold<FOLD_SEND_RANKS>, dim3(std::max<uint32_t>(1, std::min<uint32_t>(a.t_hi - a.t_lo, (uint32_t)cus))),
                           dim3(FBF_THREADS), 0, st, a, round);
    return hipGetLastError();
}

// B's grid: every coarse bin's ranges
static uint32_t split_items(const FullBinArgs& a) { return a.nb1 * ((a.cap1 + FBR_ITEM - 1) / FBR_ITEM); }

uint32_t full_bin_fused_max_bins() {
    return FBF_MAXB1;
}

// One rank.  Three passes (A send, B split, C fold); fused (a.fused): round 0
// runs A, every fold bins the next round's messages, so a round is B + C.  The
// coarse-bin counters are cleared once B has read them, before C refills them.
hipError_t launch_full_bin_round(const FullBinArgs& a, uint32_t round, int grid, hipStream_t st) {
    hipError_t e;
    if (!a.fused || round == 0) {
        if ((e = hipMemsetAsync(a.cnt1, 0, sizeof(uint32_t) * a.nb1, st)) != hipSuccess) return e;
        const uint32_t items_a = (uint32_t)(((uint64_t)a.P + FBR_ITEM - 1) / FBR_ITEM);
        hipLaunchKernelGGL(k_fb_send, dim3(items_a), dim3(FBR_THREADS), 2 * sizeof(uint32_t) * a.nb1, st, a, round);
    }
    if ((e = hipMemsetAsync(a.cnt2, 0, sizeof(uint32_t) * a.nb2, st)) != hipSuccess) return e;
    const uint32_t items_b = split_items(a);
    hipLaunchKernelGGL(k_fb_split<false>, dim3(items_b), dim3(FBR_THREADS), 2 * sizeof(uint32_t) * (1u << (a.s1 - FB_TB)),
                       st, a, round);
    const dim3 gc(fold_blocks(a.nb2, grid));
    if (a.fused) {
        if ((e = hipMemsetAsync(a.cnt1, 0, sizeof(uint32_t) * a.nb1, st)) != hipSuccess) return e;
        hipLaunchKernelGGL(k_fb_fold<FOLD_SEND>, gc, dim3(FBF_THREADS), 0, st, a, round);
    } else {
        hipLaunchKernelGGL(k_fb_fold<FOLD>, gc, dim3(FBF_THREADS), 0, st, a, round);
    }
    return hipGetLastError();
}

}  // namespace gp
