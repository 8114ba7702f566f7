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

struct SlabTable {
    uint32_t v[XMAXW + 1];
    int W;
};

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
// Wave priority raised (s_setprio 1) while k_pack / k_unpack issue their loads.  C5 at W = 8
// virtual ranks, same box, alternated: pack 4.97-4.99 -> 4.83 ms and unpack 5.59-5.73 ->
// 5.36-5.71 ms over the 8 slabs (profiles/r04/setprio_xchg.txt)
template <int P>
__device__ __forceinline__ void xchg_prio() {
    __builtin_amdgcn_s_setprio(P);
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
                *gptr(oslots[k] + idx[h]) = a.counts ? ent[h] - bnd[k] : ent[h];
                if (a.push) st_global(ovals[k] + idx[h], v[h]);
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

// ---------------------------------------------------------------- sender-ordered lists
// (Imp3D push-sum across ranks, round 5; gp_xchg.hpp).  A tile is XTILE = 1024 ids on
// a global multiple of XTILE, node slot k of thread t = id T + 256 k + t (the layout of
// the push-sum tile kernel).
namespace {

__device__ __forceinline__ uint32_t lane_below(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

struct RankLds {
    uint32_t c[4][4][XMAXW];  // [slot][wave][destination]: counts, then exclusive offsets
    uint32_t tot[XMAXW];      // the tile's list entries per destination
};

// rho[k]: rank of node slot k among the tile's list entries with the same destination,
// in id order; dst[k] < W, or XNONE for no entry.  256 threads; two barriers.
__device__ __forceinline__ void tile_list_rank(const uint32_t (&dst)[4], uint32_t (&rho)[4], RankLds& R, int W) {
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        rho[k] = 0u;
        for (int d = 0; d < W; ++d) {  // W is uniform
            const unsigned long long m = __ballot(dst[k] == (uint32_t)d);
            if (dst[k] == (uint32_t)d) rho[k] = lane_below(m);
            if (lane == 0) R.c[k][wv][d] = (uint32_t)__popcll(m);
        }
    }
    __syncthreads();
    if (threadIdx.x < (uint32_t)W) {
        const uint32_t d = threadIdx.x;
        uint32_t o = 0;
        for (int k = 0; k < 4; ++k)
            for (int w = 0; w < 4; ++w) {
                const uint32_t c = R.c[k][w][d];
                R.c[k][w][d] = o;
                o += c;
            }
        R.tot[d] = o;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (dst[k] != XNONE) rho[k] += R.c[k][wv][dst[k]];
}

struct TileSpan {
    uint32_t T, j0, j1;
};
__device__ __forceinline__ TileSpan tile_span(uint32_t lo, uint32_t nloc, uint32_t t) {
    TileSpan s;
    s.T = (lo / XTILE + t) * XTILE;
    s.j0 = max(lo, s.T);
    s.j1 = min(lo + nloc, s.T + XTILE);
    return s;
}

}  // namespace

// Setup, slab a: list entries per (tile, destination).  One block per tile.
__global__ __launch_bounds__(256) void k_list_count(ListCountArgs a) {
    __shared__ uint32_t c[XMAXW];
    if (threadIdx.x < XMAXW) c[threadIdx.x] = 0u;
    __syncthreads();
    const TileSpan sp = tile_span(a.lo, a.nloc, blockIdx.x);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t j = sp.T + k * 256u + threadIdx.x;
        if (j >= sp.j0 && j < sp.j1) {
            const uint32_t d = owner_of(a.rnd[j], a.bounds, a.W);
            if (d != (uint32_t)a.a) atomicAdd(&c[d], 1u);
        }
    }
    __syncthreads();
    if (threadIdx.x < (uint32_t)a.W) a.cnt[(size_t)blockIdx.x * a.W + threadIdx.x] = c[threadIdx.x];
}

// Setup, slab a: key[i] = 64 * (header word of i's list entry in its destination's header
// region) + its bit, for every sender i of the slab whose random edge leaves the slab.
__global__ __launch_bounds__(256) void k_list_key(ListKeyArgs a) {
    __shared__ RankLds R;
    const uint32_t t = blockIdx.x;
    const TileSpan sp = tile_span(a.lo, a.nloc, t);
    uint32_t dst[4], rho[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t j = sp.T + k * 256u + threadIdx.x;
        dst[k] = XNONE;
        if (j >= sp.j0 && j < sp.j1) {
            const uint32_t d = owner_of(a.rnd[j], a.bounds, a.W);
            if (d != (uint32_t)a.a) dst[k] = d;
        }
    }
    tile_list_rank(dst, rho, R, a.W);
    int h = 0;
    while (h + 1 < a.NH && t >= a.tb[h + 1]) ++h;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t j = sp.T + k * 256u + threadIdx.x;
        if (dst[k] != XNONE) a.key[j] = (a.hw[h][dst[k]] + a.gw[(size_t)t * a.W + dst[k]]) * 64u + rho[k];
        if (a.xdr && j >= sp.j0 && j < sp.j1)
            a.xdr[j - a.lo] = dst[k] != XNONE ? (uint16_t)((dst[k] << 10) | rho[k]) : XDR_NONE;
    }
}

// One round, one region: the header words and the compacted messages of every
// destination.  A block of LP_TILES waves takes LP_TILES consecutive tiles (8192
// senders), one per wave, walked as 16 slots of 64 consecutive ids.  A sender's
// destination and rank in its tile's list are static (xdr, k_list_key at create) and so
// is the tile's LDS word layout (lwt): a used entry's bit is one LDS atomic, no ranking
// per round (ballots per slot and destination made the pack VALU-bound: 0.69 -> 0.52-0.60 ms per
// C5 slab at W = 8).  The wave scans its words' counts; then, for all the block's tiles
// at once, ONE reservation per destination (a reservation per tile queued ~60 k
// returning atomics on each of a C5 slab's 14 counters per round: 0.73 ms per region),
// the header words and the messages in list order.  Two barriers per block.
constexpr int LIST_LW = XTILE / 64 + XMAXW;  // LDS words of one tile's segments (<= 16 full + 1 partial each)
// tiles per block, one per wave (16: 0.52 -> 0.59 ms per C5 slab at W = 8, profiles/r05/rejected/pack_shapes.txt)
constexpr int LP_TILES = 8;
constexpr int LP_WT = 1;                     // tiles per wave
constexpr int LP_THREADS = 64 * LP_TILES / LP_WT;
constexpr int LP_SLOTS = XTILE / 64;         // 64-id slots per tile
__global__ __launch_bounds__(LP_THREADS) void k_list_pack(ListPackArgs a) {
    __shared__ uint32_t mk[LP_TILES][2 * LIST_LW];  // the segments' bitmaps, 64 bits per word
    __shared__ uint32_t wb[LP_TILES][LIST_LW];      // used entries before the word in its tile's run
    __shared__ uint32_t lw[LP_TILES][XMAXW + 1];    // first LDS word of each destination's segment
    __shared__ uint32_t tn[LP_TILES][XMAXW];        // used entries per (tile, destination), then run offsets
    __shared__ uint32_t off[XMAXW];                 // the block's reserved run in each destination's chunk
    __shared__ double2* ovals[XMAXW];
    __shared__ uint32_t ocap[XMAXW];
    const uint32_t tb = a.t0 + blockIdx.x * LP_TILES;
    if (tb >= a.t1) return;
    const int ntl = (int)min((uint32_t)LP_TILES, a.t1 - tb);
    const uint32_t lane = threadIdx.x & 63u;
    // the wave's index, known uniform: its tiles' buffer resources are then scalar (a per-lane
    // resource made every buffer load a waterfall loop)
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t me = (uint32_t)a.me;
    const int W = a.W;
    for (uint32_t q = threadIdx.x; q < LP_TILES * 2 * LIST_LW; q += LP_THREADS) (&mk[0][0])[q] = 0u;
    if (threadIdx.x < (uint32_t)W) {
        ovals[threadIdx.x] = a.peer[threadIdx.x].vals;
        ocap[threadIdx.x] = a.peer[threadIdx.x].cap;
    }
    if (threadIdx.x < (uint32_t)(LP_TILES * (W + 1))) {  // the tiles' static LDS word layouts
        const uint32_t tt = threadIdx.x / (W + 1), d = threadIdx.x - tt * (W + 1);
        if ((int)tt < ntl) lw[tt][d] = a.lwt[(size_t)(tb + tt) * (W + 1) + d];
    }
    __syncthreads();
    // per tile of this wave and slot: used ? 1 << 31 | d << 11 | rho : 0 (rho < 1024)
    uint32_t st[LP_WT][LP_SLOTS];
#pragma unroll
    for (int u = 0; u < LP_WT; ++u) {
#pragma unroll
        for (int q = 0; q < LP_SLOTS; ++q) st[u][q] = 0u;
        const int tt = (int)wv * LP_WT + u;
        if (tt >= ntl) break;  // (wave-uniform)
        const TileSpan sp = tile_span(a.lo, a.nloc, tb + tt);
        uint8_t b[LP_SLOTS];
        uint16_t x[LP_SLOTS];
        xchg_prio<1>();
#pragma unroll
        for (int q = 0; q < LP_SLOTS; ++q) {  // unconditional (clamped) loads, all in flight
            const uint32_t j = min(max(sp.T + q * 64u + lane, sp.j0), sp.j1 - 1u);
            b[q] = a.nbn[j - a.base];
            x[q] = a.xdr[j - a.lo];
        }
        xchg_prio<0>();
#pragma unroll
        for (int q = 0; q < LP_SLOTS; ++q) {
            const uint32_t j = sp.T + q * 64u + lane;
            const bool used = j >= sp.j0 && j < sp.j1 && (b[q] & DIR_MASK) == DIR_RANDOM && x[q] != XDR_NONE;
            if (used) {
                const uint32_t d = x[q] >> 10, rho = x[q] & 1023u;
                st[u][q] = 0x80000000u | (d << 11) | rho;
                const uint32_t w = lw[tt][d] + (rho >> 6);
                atomicOr(&mk[tt][2 * w + ((rho >> 5) & 1u)], 1u << (rho & 31u));
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        // word prefixes within each destination's segment, and the tile's used entries per destination
        const uint32_t nw = lw[tt][W];  // <= LIST_LW <= 64: one wave-wide scan
        const uint32_t l = lane;
        uint32_t seg = 0;
        for (int d = 1; d < W; ++d) seg += l >= lw[tt][d] ? 1u : 0u;
        const unsigned long long m = l < nw ? ((unsigned long long)mk[tt][2 * l + 1] << 32) | mk[tt][2 * l] : 0ull;
        const uint32_t p = (uint32_t)__popcll(m);
        uint32_t incl = p;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t v = __shfl_up(incl, o, 64);
            if (l >= (uint32_t)o) incl += v;
        }
        const uint32_t s0 = lw[tt][seg];
        const uint32_t before = __shfl(incl, (int)(s0 > 0 ? s0 - 1 : 0), 64);
        if (l < nw) wb[tt][l] = incl - p - (s0 > 0 ? before : 0u);
        const uint32_t dl = min(l, (uint32_t)W - 1u);
        const uint32_t e0 = lw[tt][dl], e1 = lw[tt][dl + 1];
        const uint32_t a1 = __shfl(incl, (int)(e1 > 0 ? e1 - 1 : 0), 64);
        const uint32_t a0 = __shfl(incl, (int)(e0 > 0 ? e0 - 1 : 0), 64);
        if (l < (uint32_t)W) tn[tt][l] = e1 > e0 ? a1 - (e0 > 0 ? a0 : 0u) : 0u;
    }
    __syncthreads();
    if (threadIdx.x < (uint32_t)W) {  // the block's run per destination: one reservation
        const uint32_t d = threadIdx.x;
        uint32_t r = 0;
        for (int tt = 0; tt < ntl; ++tt) {
            const uint32_t c = tn[tt][d];
            tn[tt][d] = r;
            r += c;
        }
        off[d] = d != me && r ? atomicAdd(a.peer[d].cnt, r) : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < LP_WT; ++u) {
        const int tt = (int)wv * LP_WT + u;
        if (tt >= ntl) break;
        const TileSpan sp = tile_span(a.lo, a.nloc, tb + tt);
        {  // header words (lane = word)
            const uint32_t l = lane;
            if (l < lw[tt][W]) {
                uint32_t seg = 0;
                for (int d = 1; d < W; ++d) seg += l >= lw[tt][d] ? 1u : 0u;
                XHdr h;
                h.mask = ((unsigned long long)mk[tt][2 * l + 1] << 32) | mk[tt][2 * l];
                h.base = a.peer[seg].vbase + off[seg] + tn[tt][seg] + wb[tt][l];
                h.pad = 0u;
                a.peer[seg].hdr[a.gw[(size_t)(tb + tt) * W + seg] + (l - lw[tt][seg])] = h;
            }
        }
        // the used entries' (s, w): buffer loads over the tile's ids, past the end for the
        // others (no memory touched, no load under a branch), four slots in flight.  (A compacted
        // outbox of the random-edge senders' (s, w), written by the round kernel, cut the pack's
        // reads but cost the round kernel more than it saved, with non-temporal or plain stores
        // of the state: profiles/r05/rejected/outbox.txt)
        const __amdgpu_buffer_rsrc_t rs = buf_rsrc(a.swn + (sp.j0 - a.base), (sp.j1 - sp.j0) * 16u);
#pragma unroll
        for (int q0 = 0; q0 < LP_SLOTS; q0 += 4) {
            double2 v[4];
            xchg_prio<1>();
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                const int q = q0 + h;
                const uint32_t j = sp.T + q * 64u + lane;
                const uint32_t e = st[u][q];
                const auto w4 =
                    __builtin_amdgcn_raw_buffer_load_b128(rs, (e & 0x80000000u) ? (j - sp.j0) * 16u : BUF_NONE, 0, 0);
                v[h] = __builtin_bit_cast(double2, w4);
            }
            xchg_prio<0>();
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                const int q = q0 + h;
                const uint32_t e = st[u][q];
                if (!(e & 0x80000000u)) continue;
                const uint32_t d = (e >> 11) & 15u, rho = e & 0x7FFu;
                const uint32_t w = lw[tt][d] + (rho >> 6), bit = rho & 63u;
                const unsigned long long m = ((unsigned long long)mk[tt][2 * w + 1] << 32) | mk[tt][2 * w];
                const uint32_t idx = off[d] + tn[tt][d] + wb[tt][w] + (uint32_t)__popcll(m & ((1ull << bit) - 1ull));
                if (idx < ocap[d]) st_global(ovals[d] + idx, v[h]);
                else atomicOr(a.overflow, 1u);
            }
        }
    }
}

// A halo plane's senders toward the neighbour: their (s, w) compacted per 1024-node chunk, in
// id order (PACK), or put back at their ids in the receiver's halo plane (!PACK) -- both sides
// rank the same direction bytes the same way, so no counts travel.
template <bool PACK>
__global__ __launch_bounds__(256) void k_halo(HaloArgs a) {
    __shared__ uint32_t wc[HALO_CHUNK / 64];  // senders per 64-node group, in id order
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t c0 = blockIdx.x * HALO_CHUNK;
    bool m[HALO_CHUNK / 256];
    uint32_t below[HALO_CHUNK / 256];
#pragma unroll
    for (int k = 0; k < (int)(HALO_CHUNK / 256); ++k) {
        const uint32_t i = c0 + k * 256u + threadIdx.x;
        m[k] = i < a.n && (a.nb[i] & DIR_MASK) == a.dir;
        const unsigned long long bal = __ballot(m[k]);
        below[k] = lane_below(bal);
        if (lane == 0) wc[k * 4 + wv] = (uint32_t)__popcll(bal);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < (int)(HALO_CHUNK / 256); ++k) {
        if (!m[k]) continue;
        uint32_t rank = below[k];
        for (uint32_t q = 0; q < (uint32_t)k * 4u + wv; ++q) rank += wc[q];
        const uint32_t i = c0 + k * 256u + threadIdx.x;
        double2* slot = a.buf + (size_t)blockIdx.x * a.cap + rank;
        if (rank >= a.cap) {
            if (PACK) atomicOr(a.overflow, 1u);
        } else if (PACK) {
            st_global(slot, ld_global(a.sw + i));
        } else {
            st_global(a.sw + i, ld_global(slot));
        }
    }
}

__global__ __launch_bounds__(256) void k_gather_keys(const uint32_t* __restrict__ key, const uint32_t* __restrict__ src,
                                                     uint32_t n, uint32_t* __restrict__ out) {
    for (uint32_t e = blockIdx.x * 256 + threadIdx.x; e < n; e += gridDim.x * 256) out[e] = key[src[e]];
}

// ---------------------------------------------------------------- gossip bitmaps (setup + apply)
__global__ __launch_bounds__(256) void k_src_flag(const uint32_t* __restrict__ src, uint32_t n, SlabTable b, int a,
                                                  uint32_t* __restrict__ flag) {
    for (uint32_t q = blockIdx.x * 256 + threadIdx.x; q <= n; q += gridDim.x * 256)
        flag[q] = q < n && owner_of(src[q], b.v, b.W) == (uint32_t)a ? 1u : 0u;
}

// pos[q] for the edges q whose sender is on slab a: their rank among the edges of the
// same receiver slab with a sender on a, in receiver order.
__global__ __launch_bounds__(256) void k_bits_pos(BitsSetupArgs a) {
    for (uint32_t q = blockIdx.x * 256 + threadIdx.x; q < a.n; q += gridDim.x * 256) {
        if (owner_of(a.src[q], a.bounds, a.W) != (uint32_t)a.a) continue;
        const uint32_t b = owner_of(a.recv[q], a.bounds, a.W);
        a.pos[q] = a.scan[q] - a.scan[a.edge0[b]];
    }
}

__global__ __launch_bounds__(256) void k_bits_ends(BitsEndsArgs a) {
    for (uint32_t li = blockIdx.x * 256 + threadIdx.x; li < a.nloc; li += gridDim.x * 256) {
        const uint32_t t = a.rnd[li];
        const uint32_t d = owner_of(t, a.bounds, a.W);
        a.rtg[li] = d == (uint32_t)a.me ? t - a.lo : 0x80000000u | (a.bo[d] + a.pos[a.inv[a.lo + li]]);
    }
    for (uint32_t q = a.e0 + blockIdx.x * 256 + threadIdx.x; q < a.e1; q += gridDim.x * 256) {
        const uint32_t s = owner_of(a.src[q], a.bounds, a.W);
        if (s != (uint32_t)a.me) a.tgt[a.ro[s] + a.pos[q]] = a.recv[q] - a.lo;
    }
}

// One rumour for next round per set bit of the received bitmaps (Program.fs:84-89: the
// sender's Tell to its random neighbour), at the bit's target.
__global__ __launch_bounds__(256) void k_apply_bits(const uint32_t* __restrict__ bits, uint32_t nwords,
                                                    const uint32_t* __restrict__ tgt, uint32_t* rq, uint32_t rq8) {
    for (uint32_t w = blockIdx.x * 256 + threadIdx.x; w < nwords; w += gridDim.x * 256) {
        uint32_t m = bits[w];
        while (m) {
            const uint32_t b = (uint32_t)__builtin_ctz(m);
            m &= m - 1u;
            rq_add(rq, rq8, tgt[w * 32u + b]);
        }
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
hipError_t launch_src_flag(const uint32_t* src, uint32_t n, const uint32_t* bounds, int W, int a, uint32_t* flag,
                           int grid, hipStream_t st) {
    SlabTable b{};
    for (int w = 0; w <= W; ++w) b.v[w] = bounds[w];
    b.W = W;
    hipLaunchKernelGGL(k_src_flag, dim3(grid), dim3(256), 0, st, src, n, b, a, flag);
    return hipGetLastError();
}
hipError_t launch_bits_pos(const BitsSetupArgs& a, int grid, hipStream_t st) {
    hipLaunchKernelGGL(k_bits_pos, dim3(grid), dim3(256), 0, st, a);
    return hipGetLastError();
}
hipError_t launch_bits_ends(const BitsEndsArgs& a, int grid, hipStream_t st) {
    hipLaunchKernelGGL(k_bits_ends, dim3(grid), dim3(256), 0, st, a);
    return hipGetLastError();
}
hipError_t launch_apply_bits(const uint32_t* bits, uint32_t nwords, const uint32_t* tgt, uint32_t* rq, uint32_t rq8,
                             hipStream_t st) {
    const uint32_t blocks = std::min<uint32_t>((nwords + 255) / 256, 4096u);
    if (blocks) hipLaunchKernelGGL(k_apply_bits, dim3(blocks), dim3(256), 0, st, bits, nwords, tgt, rq, rq8);
    return hipGetLastError();
}
hipError_t launch_list_count(const ListCountArgs& a, hipStream_t st) {
    const uint32_t nt = (uint32_t)(((uint64_t)a.lo + a.nloc + XTILE - 1) / XTILE - a.lo / XTILE);
    if (nt) hipLaunchKernelGGL(k_list_count, dim3(nt), dim3(256), 0, st, a);
    return hipGetLastError();
}
hipError_t launch_list_key(const ListKeyArgs& a, hipStream_t st) {
    const uint32_t nt = (uint32_t)(((uint64_t)a.lo + a.nloc + XTILE - 1) / XTILE - a.lo / XTILE);
    if (nt) hipLaunchKernelGGL(k_list_key, dim3(nt), dim3(256), 0, st, a);
    return hipGetLastError();
}
hipError_t launch_list_pack(const ListPackArgs& a, hipStream_t st) {
    if (a.t1 > a.t0)
        hipLaunchKernelGGL(k_list_pack, dim3((a.t1 - a.t0 + LP_TILES - 1) / LP_TILES), dim3(LP_THREADS), 0, st, a);
    return hipGetLastError();
}
hipError_t launch_halo_pack(const HaloArgs& a, hipStream_t st) {
    if (a.n) hipLaunchKernelGGL(k_halo<true>, dim3((a.n + HALO_CHUNK - 1) / HALO_CHUNK), dim3(256), 0, st, a);
    return hipGetLastError();
}
hipError_t launch_halo_expand(const HaloArgs& a, hipStream_t st) {
    if (a.n) hipLaunchKernelGGL(k_halo<false>, dim3((a.n + HALO_CHUNK - 1) / HALO_CHUNK), dim3(256), 0, st, a);
    return hipGetLastError();
}

// Slots per 1024-node chunk of a slab-boundary plane (HaloArgs): the senders toward one x
// neighbour in a chunk are a sum of Bernoulli(1 / deg) over its nodes (Program.fs:246-260: a
// boundary plane's nodes have both x neighbours, y / z ones unless on the lattice's edge, and
// Imp3D's random edge); the largest mean + 12 sigma over the plane's chunks, rounded up to 8.
// g = 1000: 3D 360 (the chunk of row y = 0), Imp3D 320.
uint32_t halo_chunk_cap(uint32_t g, bool imp3d) {
    const uint64_t n = (uint64_t)g * g;
    double best = 0.0, mu = 0.0, var = 0.0;
    for (uint64_t i = 0; i <= n; ++i) {
        if (i == n || (i % HALO_CHUNK == 0 && i > 0)) {
            best = std::max(best, mu + 12.0 * std::sqrt(var));
            mu = var = 0.0;
            if (i == n) break;
        }
        const uint32_t y = (uint32_t)(i / g), z = (uint32_t)(i % g);
        const uint32_t deg = 2u + (y > 0) + (y + 1 < g) + (z > 0) + (z + 1 < g) + (imp3d ? 1u : 0u);
        const double p = 1.0 / deg;
        mu += p;
        var += p * (1.0 - p);
    }
    const uint32_t c = (uint32_t)std::ceil(best);
    return std::min<uint32_t>(HALO_CHUNK, std::max<uint32_t>(8u, (c + 7u) & ~7u));
}
hipError_t launch_gather_keys(const uint32_t* key, const uint32_t* src, uint32_t n, uint32_t* out, int grid,
                              hipStream_t st) {
    if (n) hipLaunchKernelGGL(k_gather_keys, dim3(grid), dim3(256), 0, st, key, src, n, out);
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

