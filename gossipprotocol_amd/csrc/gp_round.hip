// gp_round.hip -- the per-round bulk kernels for line / 3D / Imp3D (gfx950).
//
// One synchronous round of SRS v1 in PULL form: every node
// reads who sent to it and folds the messages in canonical order, then draws
// its own direction for the next round.  Layout per workgroup (256 threads,
// TILE = 1024 consecutive nodes, 4 per thread, lane-contiguous):
//
//   1. stage in LDS with wide coalesced loads: the direction bytes of the tile
//      and its +-g rows (y/z neighbours, or +-1 for line), the x-1 and x+1
//      plane segments (3D), the tile's in-list offsets and senders (Imp3D);
//   2. per node: lattice senders are read from LDS and only the (s, w) of the
//      neighbours that actually sent here are gathered (independent loads, no
//      dependent byte loads); Imp3D in-edges decide "sent on its random edge"
//      from the sender's Philox draw (every node active) or from a ballot-packed
//      bitmap (activation phase), then gather;
//   3. fold in canonical order (own half, lattice slots, random edges by
//      ascending sender), ratio test, next-round Philox draw; node bytes leave
//      through LDS as 32-bit words, random-edge bits as one 64-bit ballot per
//      wave.
// Tiles are walked XCD-contiguously (blocks b and b+8 share an XCD on
// MI355X), so the +-g rows a tile gathers from were just read by its XCD.
// Built with -ffp-contract=off: the fold must round exactly like the oracle.
#include <algorithm>
#include <type_traits>
#include <vector>

#include "gp_internal.hpp"

namespace gp {
#ifdef GP_ROUND_WIDE
// gp_round_wide.hip: this file again with 1024-thread tiles of one node per
// thread (the small-population size class), its host entry points in gp::wide
namespace wide {
#endif

// Size class: gp_round_wide.hip defines these before including this file.
#ifndef GP_ROUND_WIDE
#define GP_TPB 256
#define GP_NPT 4
// __launch_bounds__ minimum waves per SIMD (= resident 256-thread blocks per CU): the LDS
// tile allows 5, so keep VGPRs <= 96 to not lose the fifth
#define GP_MINB 5
#endif

// Measured choices of the push-sum tile kernel (the rejected alternatives and their
// records are in DESIGN.md §5.1 and profiles/; git history has their code):
//  * wave priority: raised (s_setprio PRIO) while a wave issues its memory operations --
//    the in-edge pass's gathers, the staging copies, each node slot's loads -- and dropped
//    for the fold and the direction draws, so waves about to issue loads win the SIMD over
//    waves with ALU work and more loads are in flight (P = 1e9, same box, alternated:
//    13.19-13.68 -> 12.93-13.15 ms/round, profiles/r04/setprio_ab.txt);
//  * walk 3 work stealing: a block whose XCD's queue is empty takes items from the other
//    XCDs' queues (12.85-12.87 -> 12.75-12.81 ms/round; W = 8 slab 1.714 -> 1.699 ms,
//    profiles/r04/walk_steal.txt);
//  * the j +- 1 messages from the neighbour lanes' registers by DPP, one node slot's loads
//    in flight at a time (two spilled), non-temporal staging loads and state stores.
constexpr int PRIO = 1;  // the raised wave priority

namespace {

constexpr int TPB = GP_TPB;                // 256 (wide size class: 1024)
constexpr int NPT = GP_NPT;                // nodes per thread per tile
constexpr int TILE = TPB * NPT;            // 1024
constexpr int HMAX = 1625;                 // largest lattice edge with g^3 < 2^32
constexpr int W_ROWS = (TILE + 2 * HMAX) / 4 + 4;
constexpr int W_PLANE = TILE / 4 + 4;
constexpr int SRC_CAP = TILE * 3 / 2;       // gossip: staged in-list entries per tile (mean TILE)

// Staged ranges are moved by 16-byte LDS-DMA (global_load_lds_dwordx4) from a
// 16-byte aligned start: every array has 8 words of slack for the alignment.
constexpr int DMA_SLACK = 8;

struct TileLds {
    uint32_t rows[W_ROWS + DMA_SLACK];   // direction bytes of [j0 - H, j1 + H)
    uint32_t xm[W_PLANE + DMA_SLACK];    // direction bytes of [j0 - g^2, j1 - g^2)
    uint32_t xp[W_PLANE + DMA_SLACK];    // direction bytes of [j0 + g^2, j1 + g^2)
    uint32_t off[TILE + 1 + DMA_SLACK];  // in_off[j0 .. j1]
    uint32_t sent[SRC_CAP / 4];          // byte per staged in-edge: its sender used the random edge
    uint32_t out[TILE / 4];              // next-round node bytes, stored as words
    uint32_t red[2][TPB / 64];
};

// k_ps_tile: the tile decides its in-edges itself.  The used in-edges' (s, w) are gathered by LDS-DMA straight into per-edge
// slots (edge q's message at slot q -- lane-linear, so one global_load_lds per
// edge batch, no registers, no compaction).  A tile with more than SLOTS
// in-edges takes the unstaged path, so the node fold reads LDS only (no global
// fallback inside its loop, whose join would cost a vmcnt(0) wait per message).
//
// One rank (SNDPF): the next tile's in-edge senders are LDS-DMA'd during this tile's node phase,
// so a tile's in-edge pass starts from LDS (C5, same box, alternated: 12.92-13.07 -> 12.78-12.86
// ms on one box, 12.78-12.82 -> 12.74-12.77 on another, profiles/r05/sndpf/).  Their buffer takes
// LDS from the slots: 1152 slots (a tile's in-degree is ~Poisson(1024); 4 sigma, ~4e-5 of tiles
// -- about 40 per C5 round -- take the unstaged path).  The REMOTE kernel (several ranks) has no
// such buffer (measured within noise there, profiles/r05/sndpf/w8.txt) and keeps 1216 slots (6
// sigma, ~2.5e-9 of tiles): both fill the LDS of 5 blocks per CU.
template <bool REMOTE>
struct PsSlots {
    static constexpr bool SNDPF = !REMOTE;
    static constexpr int SLOTS = SNDPF ? TILE + TILE / 8 : TILE + TILE / 8 + TILE / 16;
    static constexpr int FU = (SLOTS + TPB - 1) / TPB;  // in-edges per thread in the in-edge pass
};

template <bool REMOTE>
struct TileLdsP {
    static constexpr int SLOTS = PsSlots<REMOTE>::SLOTS, SLOT_FU = PsSlots<REMOTE>::FU;
    uint32_t rows[W_ROWS + DMA_SLACK];
    uint32_t xm[W_PLANE + DMA_SLACK];
    uint32_t xp[W_PLANE + DMA_SLACK];
    uint32_t ind[TILE / 8 + DMA_SLACK];  // in-degrees of the tile's nodes, a nibble each (DevState::ind4)
    unsigned long long bits[SLOT_FU * (TPB / 64) + 1];  // bit q: in-edge q (tile order) was used by its sender; then 0
    double2 msg[SLOTS];               // edge q's message at slot q
    uint32_t out[TILE / 4];
    uint32_t red[2][TPB / 64];
    uint32_t qn[2];                   // walk 3: the block's next item, by iteration parity
    double2 zb[TPB / 64][NPT][2];     // (s, w) across each wave's ends, slot k: [0] node - 1, [1] node + 64
};

// set bits of m below this lane
__device__ __forceinline__ uint32_t mbcnt64(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ uint32_t lds_byte(const uint32_t* w, uint32_t idx) {
    return reinterpret_cast<const uint8_t*>(w)[idx];
}

typedef __attribute__((address_space(1))) void gvoid_t;
typedef __attribute__((address_space(3))) void lvoid_t;

// Copy nbytes (rounded up to 16) from a 16-byte aligned global address into LDS
// with LDS-DMA: no VGPR round trip and no wait inside the loop, so every
// staging copy of a tile is in flight at once (retired by the next
// __syncthreads, which waits vmcnt(0)).  One wave-instruction moves 1 KiB.
template <int AUX = 0>
__device__ __forceinline__ void dma_copy(void* lds, const char* g16, uint32_t nbytes) {
    const uint32_t lane = threadIdx.x & 63u;
    for (uint32_t c = (threadIdx.x >> 6) * 1024u; c < nbytes; c += TPB * 16u) {
        const uint32_t o = c + lane * 16u;
        if (o < nbytes)
            __builtin_amdgcn_global_load_lds((gvoid_t*)(g16 + o), (lvoid_t*)(reinterpret_cast<char*>(lds) + c), 16, 0,
                                             AUX);
    }
}
// cache-policy bits of a single-use (streamed once per round) staging copy: nt
constexpr int DMA_ONCE = 2;

// Node bytes nb[lo, hi) clamped to [ext_lo,
// ext_hi); returns the node id of LDS byte 0 (up to 15 bytes below lo).  Reads
// at most 15 bytes past hi (node arrays are padded).
__device__ __forceinline__ uint32_t dma_stage_bytes(uint32_t* lds, const uint8_t* nb, int64_t lo, int64_t hi,
                                                    uint32_t ext_lo, uint32_t ext_hi) {
    if (lo < (int64_t)ext_lo) lo = ext_lo;
    if (hi > (int64_t)ext_hi) hi = ext_hi;
    const char* p = reinterpret_cast<const char*>(nb + lo);
    const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 15u);
    if (hi > lo) dma_copy(lds, p - mis, (uint32_t)(hi - lo) + mis);
    return (uint32_t)lo - mis;
}

// LDS-DMA of the words w[lo, hi); returns how many words below lo were staged
// (w[lo + i] lands in lds[i + returned]).  Reads at most 3 words past hi
// (the in-list arrays are padded).
__device__ __forceinline__ uint32_t dma_stage_words(uint32_t* lds, const uint32_t* w, uint32_t lo, uint32_t hi) {
    const char* p = reinterpret_cast<const char*>(w + lo);
    const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 15u);
    if (hi > lo) dma_copy<DMA_ONCE>(lds, p - mis, (hi - lo) * 4u + mis);
    return mis >> 2;
}

template <typename T>
__device__ __forceinline__ T ld_agent(const T* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Tile walks (speed only -- any placement is correct; every tile of the slab
// is visited exactly once).  Blocks with equal blockIdx % 8 share an XCD.
//   walk 0: XCD-contiguous eighths of the tile range;
//   walk 1: one global sweep (tile t -> block t % grid);
//   walk 2 (3D / Imp3D): x-window walk.  Each XCD owns an eighth of the slab's
//     x-planes, cut into windows of ~wx planes; inside a window the walk is
//     x-fastest: item u -> plane x = x_w + u % nx_w, k-th tile starting in that
//     plane.  The blocks resident on an XCD at one time then work on the same
//     in-plane position of ~wx consecutive planes (x+-1 neighbours) and of a few
//     consecutive k (y+-1 rows), so lattice gathers and the x+-1 byte planes hit
//     the XCD's L2 instead of HBM.
//   walk 3 (k_ps_tile): walk 2's items without the empty ones, listed per XCD
//     at create time (DevState::wtiles, build_walk_list in gp_api.hip) and
//     claimed in order from a per-XCD counter (one returning atomic per tile,
//     issued a tile ahead) on a grid of exactly the resident blocks.  The tiles
//     an XCD has in flight are then always ~160 consecutive items (20 in-plane
//     positions of 8 planes), and the tiles just finished are their y-1 / x+-1
//     neighbours; walk 2's static stride keeps items 2048 apart in flight, and
//     its item -> tile arithmetic (64-bit divisions) costs ~100 scalar
//     instructions per tile and wave.
struct TileWalk {
    uint32_t t, end, step;
    // walk 2
    uint32_t mode, tb, tend, g2, x0, xa, nxa, kp, nwin;
    // walk 3: this XCD's item counter and tile list
    uint32_t* qc;
    const uint32_t* wl;
    __device__ TileWalk(const RoundArgs& a) {
        const uint32_t G = gridDim.x;
        mode = a.walk;
        qc = nullptr;
        wl = nullptr;
        if (mode == 3 && (a.wt == nullptr || G < 8 || (G & 7) != 0)) mode = 1;
        if (mode == 3) {
            const uint32_t c = blockIdx.x & 7;
            qc = a.tq + c * TQ_STRIDE;
            wl = a.wt + a.wo[c];
            t = 0;
            end = a.wo[c + 1] - a.wo[c];
            step = 1;
        } else if (mode == 2 && a.G.g2 && G >= 8 && (G & 7) == 0) {
            const uint32_t c = blockIdx.x & 7;
            g2 = a.G.g2;
            tb = a.lo / TILE;
            tend = (uint32_t)(((uint64_t)a.lo + a.nloc + TILE - 1) / TILE);
            x0 = a.lo / g2;
            const uint32_t X0 = x0, nx = a.nloc / g2;
            xa = X0 + (uint32_t)((uint64_t)nx * c / 8);
            nxa = X0 + (uint32_t)((uint64_t)nx * (c + 1) / 8) - xa;
            kp = (g2 + TILE - 1) / TILE + 1;
            nwin = a.wx ? (nxa + a.wx - 1) / a.wx : 1u;
            if (nwin == 0) nwin = 1;
            t = blockIdx.x >> 3;
            end = nxa * kp;
            step = G >> 3;
        } else if (mode == 0 && G >= 8 && (G & 7) == 0) {
            mode = 0;
            const uint32_t x = blockIdx.x & 7, k = blockIdx.x >> 3;
            const uint32_t lo = (uint32_t)((uint64_t)a.ntiles * x / 8);
            end = (uint32_t)((uint64_t)a.ntiles * (x + 1) / 8);
            t = lo + k;
            step = G >> 3;
        } else {
            mode = 1;
            t = blockIdx.x;
            end = a.ntiles;
            step = G;
        }
    }
    // first global tile index of plane x (the slab's first tile may start below lo)
    __device__ __forceinline__ uint32_t first(uint32_t x) const {
        return x <= x0 ? tb : min((uint32_t)(((uint64_t)x * g2 + TILE - 1) / TILE), tend);
    }
    // tile (relative to lo / TILE) of walk item t; false: empty item (block-uniform)
    __device__ __forceinline__ bool tile(uint32_t& rel) const {
        if (mode == 3) {
            rel = ld_const(wl + t);
            return true;
        }
        if (mode != 2) {
            rel = t;
            return true;
        }
        const uint32_t pl = t / kp;  // planes of this XCD before the item's window start (approx.)
        uint32_t v = (uint32_t)((uint64_t)pl * nwin / nxa);
        if (v >= nwin) v = nwin - 1;
        uint32_t xs = (uint32_t)((uint64_t)nxa * v / nwin);
        while (v > 0 && xs * kp > t) {
            --v;
            xs = (uint32_t)((uint64_t)nxa * v / nwin);
        }
        for (;;) {
            const uint32_t xe = (uint32_t)((uint64_t)nxa * (v + 1) / nwin);
            if (v + 1 >= nwin || xe * kp > t) break;
            ++v;
            xs = xe;
        }
        const uint32_t xe = (uint32_t)((uint64_t)nxa * (v + 1) / nwin);
        const uint32_t u = t - xs * kp, nxv = xe - xs;
        const uint32_t x = xa + xs + u % nxv, k = u / nxv;
        const uint32_t ti = first(x) + k;
        if (ti >= first(x + 1)) return false;
        rel = ti - tb;
        return true;
    }
};

__device__ __forceinline__ double2 ld_sw(const double2* p) { return *p; }

// v of another lane of the wave by DPP (CTRL 0x130 wave_shl:1 = lane + 1's,
// 0x138 wave_shr:1 = lane - 1's; the lane at the wave's end gets 0 -- bound_ctrl,
// so no zeroed destination register is needed)
template <int CTRL>
__device__ __forceinline__ double2 dpp_double2(double2 v) {
    auto mv = [](double d) {
        const uint64_t u = __builtin_bit_cast(uint64_t, d);
        const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)u, CTRL, 0xF, 0xF, true);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), CTRL, 0xF, 0xF, true);
        return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
    };
    return make_double2(mv(v.x), mv(v.y));
}

// Next-round state is written once and not read again this round: non-temporal
// stores keep it from displacing the current round's (s, w) in the XCD's L2,
// where the neighbouring tiles' lattice gathers look for it.
__device__ __forceinline__ void st_stream(double2* p, double2 v) {
    __builtin_nontemporal_store(v.x, &p->x);
    __builtin_nontemporal_store(v.y, &p->y);
}
__device__ __forceinline__ void st_stream(uint32_t* p, uint32_t v) { __builtin_nontemporal_store(v, p); }

}  // namespace

// ---------------------------------------------------------------- push-sum
// One synchronous push-sum round (SRS v1 B.4; Program.fs:101-131) over a
// lattice slab, in pull form.  REMOTE: some in-edge senders live on other
// ranks (multi-GPU slabs); the single-GPU build has no exchange-tag paths.
//
// Per tile:
//   1. in-edge pass (Imp3D): did each in-edge's sender use its random edge
//      this round?  Every node active: the sender's own Philox draw, redrawn --
//      the senders are streamed in at the tile's start, and the FU redraws of a
//      thread run as one straight-line batch so the chains interleave; during
//      activation: the ballot-packed bitmap.  Used edges' (s, w) are gathered by
//      LDS-DMA into slot q (edge order);
//   2. staging by LDS-DMA: node bytes of the tile, its +-g rows and +-g^2 plane
//      segments, the tile's in-list offsets; own (s, w) to registers;
//   3. per node: lattice senders from the staged bytes, one gather per
//      direction (no sender: the zero sentinel), the canonical fold (own half,
//      lattice slots in slot order, random edges by ascending sender), the ratio
//      test (Program.fs:114-123);
//   4. next-round directions of the thread's NPT nodes as one Philox batch;
//      node bytes out as words, random-edge bits as one ballot per wave.
template <int TOPO, bool REMOTE>
__device__ __forceinline__ void ps_tiles(const RoundArgs& a, uint32_t r, TileLdsP<REMOTE>& L, uint32_t* snd,
                                         bool all_active, uint32_t& alerts, uint32_t& newly, bool& tiny) {
    const double2* __restrict__ swc = a.swc;
    double2* __restrict__ swn = a.swn;
    const uint64_t* __restrict__ rbc = a.rbc;
    const uint32_t* __restrict__ in_src = a.in_src;
    const bool packed = a.in_srcd != nullptr;  // staged senders carry deg - 4 in bits 30-31
    const uint32_t* __restrict__ srcp = packed ? a.in_srcd : in_src;
    const Geom G = a.G;
    const uint32_t H = TOPO == LINE ? 1u : G.g;
    constexpr int FU = PsSlots<REMOTE>::FU;
    const uint32_t cap = min((uint32_t)PsSlots<REMOTE>::SLOTS, a.stage_cap);
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;

    // loaded one tile ahead: the next tile's in-edge range (two uniform loads); the
    // staged tile's senders, FU words per thread (loaded at the tile's start)
    uint32_t pf_tile = 0xFFFFFFFFu, pf_lo = 0, pf_hi = 0;
    uint32_t snd_tile = 0xFFFFFFFFu, snd_off = 0;  // SNDPF: snd holds tile snd_tile's senders from word snd_off
    constexpr bool SNDPF = PsSlots<REMOTE>::SNDPF;
    uint32_t raw[FU];
#pragma unroll
    for (int m = 0; m < FU; ++m) raw[m] = 0u;
    TileWalk tw(a);
    const bool dyn = tw.mode == 3;  // block-uniform
    uint32_t it = 0;                // iteration: parity selects the LDS slot of the next claim
    if (dyn) {
        if (blockIdx.x == 0 && threadIdx.x < 8) a.tq_next[threadIdx.x * TQ_STRIDE] = 0u;  // next round's counters
        if (threadIdx.x == 0) L.qn[0] = atomicAdd(tw.qc, 1u);
        __syncthreads();
        tw.t = __builtin_amdgcn_readfirstlane(L.qn[0]);
        ++it;
    }
    // walk 3: once this XCD's list is exhausted, the block takes items from the other
    // XCDs' queues in turn (their tiles' lattice lines are in another L2, but only
    // the round's tail runs this way), so no XCD idles while another has work
    for (uint32_t victim = 0;;) {
    while (tw.t < tw.end) {
        uint32_t ti;
        // walk 3: thread 0 claims the next item now; it is published in LDS at the
        // staging barrier (which waits for the atomic anyway)
        uint32_t claim = 0;
        if (dyn && threadIdx.x == 0) claim = atomicAdd(tw.qc, 1u);
        if (!tw.tile(ti)) {  // an empty item (a plane has fewer tiles than kp)
            if (dyn) {
                if (threadIdx.x == 0) L.qn[it & 1] = claim;
                __syncthreads();
                tw.t = __builtin_amdgcn_readfirstlane(L.qn[it & 1]);
                ++it;
            } else {
                tw.t += tw.step;
            }
            continue;
        }
        // tiles sit on global multiples of TILE (4-aligned word I/O, 64-aligned
        // ballot words); the slab's first and last tile may be partial
        const uint32_t T = (a.lo / TILE + ti) * TILE;
        const uint32_t j0 = max(a.lo, T);
        const uint32_t j1 = min(a.lo + a.nloc, T + TILE);
        const bool have_pf = pf_tile == ti;  // block-uniform
        uint32_t e_lo = 0, e_hi = 0;
        if (TOPO == IMP3D) {
            if (have_pf) {
                e_lo = pf_lo;
                e_hi = pf_hi;
            } else {
                e_lo = ld_const(a.in_off + j0);
                e_hi = ld_const(a.in_off + j1);
            }
        }
        const uint32_t cnt = e_hi - e_lo;
        const bool staged = cnt <= cap;
        if (TOPO == IMP3D && !dyn) {
            TileWalk nw = tw;
            nw.t += nw.step;
            uint32_t nti;
            pf_tile = 0xFFFFFFFFu;
            if (nw.t < nw.end && nw.tile(nti)) {
                const uint32_t nT = (a.lo / TILE + nti) * TILE;
                pf_lo = ld_const(a.in_off + max(a.lo, nT));
                pf_hi = ld_const(a.in_off + min(a.lo + a.nloc, nT + TILE));
                pf_tile = nti;
            }
        }
        if constexpr (TOPO == IMP3D) {
            if (staged) {
                // in-edge q = m * TPB + wave * 64 + lane is bit `lane` of bitmap word
                // m * 4 + wave; its message (if used) lands in slot q
                if (SNDPF && snd_tile == ti) {  // (block-uniform) prefetched during the last tile
#pragma unroll
                    for (int m = 0; m < FU; ++m) {
                        const uint32_t q = threadIdx.x + m * TPB;
                        raw[m] = q < cnt ? snd[snd_off + q] : 0u;
                    }
                } else {
#pragma unroll
                    for (int m = 0; m < FU; ++m) {
                        const uint32_t q = threadIdx.x + m * TPB;
                        raw[m] = q < cnt ? __builtin_nontemporal_load(srcp + e_lo + q) : 0u;
                    }
                }
                // REMOTE: the list keys of the tile's in-edges (meaningful for remote senders),
                // issued with the senders so their latency hides behind the draws (round 5 loaded
                // them after the draws: live across the Philox batch they spilled then; at 96 VGPRs
                // now without spills, C5 W = 8 REMOTE kernel -1.5 %, profiles/r06/remote/)
                uint32_t rkv[REMOTE ? FU : 1];
                if constexpr (REMOTE) {
#pragma unroll
                    for (int m = 0; m < FU; ++m) {
                        const uint32_t q = threadIdx.x + m * TPB;
                        rkv[m] = q < cnt ? __builtin_nontemporal_load(a.rk + e_lo + q) : 0u;
                    }
                }
                uint32_t isrc[FU];
                bool sent[FU], pick[FU];
#pragma unroll
                for (int m = 0; m < FU; ++m) isrc[m] = packed ? raw[m] & 0x3FFFFFFFu : raw[m];
                if (all_active) {
                    // the first NPT edges per thread cover a tile's mean in-degree (TILE);
                    // the slots above are drawn only by waves that hold an edge there
                    // (a wave-uniform test: most tiles have fewer than TILE + 64 in-edges)
                    constexpr int F0 = FU < NPT ? FU : NPT;
                    uint32_t x[FU], y[FU];
                    {
                        uint32_t n0[F0], x0[F0], y0[F0];
#pragma unroll
                        for (int m = 0; m < F0; ++m) n0[m] = isrc[m];
                        philox2_batch<F0>(n0, r, S_PUSHSUM, a.k0, a.k1, x0, y0);
#pragma unroll
                        for (int m = 0; m < F0; ++m) {
                            x[m] = x0[m];
                            y[m] = y0[m];
                        }
                    }
#pragma unroll
                    for (int m = F0; m < FU; ++m) {
                        x[m] = y[m] = 0u;
                        if (cnt > (uint32_t)(m * TPB) + (__builtin_amdgcn_readfirstlane(threadIdx.x) & ~63u)) {
                            uint32_t n1[1] = {isrc[m]}, x1[1], y1[1];
                            philox2_batch<1>(n1, r, S_PUSHSUM, a.k0, a.k1, x1, y1);
                            x[m] = x1[0];
                            y[m] = y1[0];
                        }
                    }
#pragma unroll
                    for (int m = 0; m < FU; ++m) {
                        const uint32_t q = threadIdx.x + m * TPB;
                        const uint32_t di = packed ? (raw[m] >> 30) + 4u : popc6(present_mask<IMP3D>(isrc[m], G)) + 1u;
                        sent[m] = pick[m] = q < cnt && uniform_from(x[m], y[m], di) == di - 1u;
                    }
                } else {
                    // activation: the sender sends on its random edge iff its draw picks
                    // that slot AND it is active -- redraw first, then read the ballot
                    // bitmap (bit = dir == random, i.e. both) only for the ~1/7 of edges
                    // the draw selects, instead of a random bitmap read per edge
                    uint32_t x[FU], y[FU];
                    philox2_batch<FU>(isrc, r, S_PUSHSUM, a.k0, a.k1, x, y);
                    // picks first, then every pick's bitmap word in flight together: loads
                    // unconditional (non-picks read the slab's first word, one shared line),
                    // since under a branch each load was waited on at once
                    bool lpick[FU];
#pragma unroll
                    for (int m = 0; m < FU; ++m) {
                        const uint32_t q = threadIdx.x + m * TPB;
                        const uint32_t i = isrc[m];
                        const uint32_t di = packed ? (raw[m] >> 30) + 4u : popc6(present_mask<IMP3D>(i, G)) + 1u;
                        pick[m] = q < cnt && uniform_from(x[m], y[m], di) == di - 1u;
                        lpick[m] = pick[m] && (!REMOTE || i - a.lo < a.nloc);
                    }
                    unsigned long long wbits[FU];
#pragma unroll
                    for (int m = 0; m < FU; ++m) wbits[m] = rbc[lpick[m] ? (isrc[m] >> 6) - (a.lo >> 6) : 0u];
                    // (the asm consumes every loaded word, so no load can be sunk into a
                    // branch on pick; its memory clobber keeps all loads ahead of the first)
#pragma unroll
                    for (int m = 0; m < FU; ++m) asm volatile("" : "+v"(wbits[m])::"memory");
#pragma unroll
                    for (int m = 0; m < FU; ++m) wbits[m] = lpick[m] ? wbits[m] : 0ull;
#pragma unroll
                    for (int m = 0; m < FU; ++m) sent[m] = (wbits[m] >> (isrc[m] & 63)) & 1ull;
                }
                // sender on another rank: its rank's list for this one says whether it used the
                // edge (the header word's bit) and where its message is (the word's base +
                // the used entries below it).  Only the drawn / picked edges (~1/7) read a
                // header word; the others load word 0 (one shared line), unconditionally,
                // so no load waits under a branch.
                uint32_t ridx[REMOTE ? FU : 1];
                if constexpr (REMOTE) {
                    uint2 hm[FU];
                    uint32_t hb[FU];
#pragma unroll
                    for (int m = 0; m < FU; ++m) {
                        const bool cand = pick[m] && isrc[m] - a.lo >= a.nloc;
                        const XHdr* hp = a.xhdr + (cand ? rkv[m] >> 6 : 0u);
                        hm[m] = *reinterpret_cast<const uint2*>(&hp->mask);
                        hb[m] = hp->base;
                    }
#pragma unroll
                    for (int m = 0; m < FU; ++m) asm volatile("" : "+v"(hm[m].x), "+v"(hm[m].y), "+v"(hb[m])::"memory");
#pragma unroll
                    for (int m = 0; m < FU; ++m) {
                        ridx[m] = 0u;
                        if (pick[m] && isrc[m] - a.lo >= a.nloc) {
                            const unsigned long long mk = ((unsigned long long)hm[m].y << 32) | hm[m].x;
                            const uint32_t bit = rkv[m] & 63u;
                            sent[m] = (mk >> bit) & 1ull;
                            ridx[m] = min(hb[m] + (uint32_t)__popcll(mk & ((1ull << bit) - 1ull)), a.xnv - 1u);
                        }
                    }
                }
                __builtin_amdgcn_s_setprio(PRIO);
#pragma unroll
                for (int m = 0; m < FU; ++m) {
                    const unsigned long long bal = __ballot(sent[m]);
                    if (lane == 0) L.bits[m * (TPB / 64) + wv] = bal;
                    if (sent[m]) {
                        const double2* src;
                        if constexpr (REMOTE) {
                            // (the index opaque: hoisted out of the tile loop, per-lane addresses
                            // were spilled, and each reload waited vmcnt(0))
                            uint32_t xi = ridx[m];
                            asm volatile("" : "+v"(xi));
                            src = isrc[m] - a.lo >= a.nloc ? a.xvals + xi : swc + isrc[m];
                        } else {
                            src = swc + isrc[m];
                        }
                        __builtin_amdgcn_global_load_lds((gvoid_t*)src, (lvoid_t*)(L.msg + (m * TPB + wv * 64)), 16,
                                                         0, DMA_ONCE);
                    }
                }
                if (threadIdx.x == 0) L.bits[FU * (TPB / 64)] = 0ull;
            }
        }
        // own (s, w): loaded with the node's lattice gathers (ahead of the staging
        // copies it kept 12 more VGPRs live and measured slower)
        double2 own[NPT];
        // every staging copy of the tile in flight at once (LDS-DMA)
        const uint32_t b_rows = dma_stage_bytes(L.rows, a.nbc, (int64_t)j0 - H, (int64_t)j1 + H, a.ext_lo, a.ext_hi);
        uint32_t b_xm = 0, b_xp = 0;
        if (TOPO != LINE) {
            b_xm = dma_stage_bytes(L.xm, a.nbc, (int64_t)j0 - G.g2, (int64_t)j1 - G.g2, a.ext_lo, a.ext_hi);
            b_xp = dma_stage_bytes(L.xp, a.nbc, (int64_t)j0 + G.g2, (int64_t)j1 + G.g2, a.ext_lo, a.ext_hi);
        }
        // (s, w) across every wave's ends, slot k: node T + k*TPB + 64 wave - 1 and + 64
        // (clamped into the node arrays; used only where that neighbour sent)
        if (lane < 2u * NPT) {
            int64_t jn = (int64_t)T + (int64_t)((lane >> 1) * TPB + wv * 64u) + ((lane & 1u) ? 64 : -1);
            if (jn < (int64_t)a.ext_lo) jn = a.ext_lo;
            if (jn > (int64_t)a.ext_hi) jn = a.ext_hi;
            __builtin_amdgcn_global_load_lds((gvoid_t*)(swc + jn), (lvoid_t*)&L.zb[wv][0][0], 16, 0, 0);
        }
        // the tile's in-degrees, a nibble per node (512 bytes; the slab's arrays
        // cover whole tiles, ids outside the slab are 0)
        if (TOPO == IMP3D) dma_copy<DMA_ONCE>(L.ind, reinterpret_cast<const char*>(a.ind4 + T / 2), TILE / 2);
        if (dyn && threadIdx.x == 0) L.qn[it & 1] = claim;
        __builtin_amdgcn_s_setprio(0);
        __syncthreads();  // staging copies, in-edge bitmap and gathered messages retired
        // Imp3D: node jl's in-edges are [e_lo + pre(jl), + d(jl)), pre = exclusive
        // prefix of the nibble in-degrees.  Every wave sums all 16 64-node chunks
        // (lane L: nodes 16L..16L+15) and keeps the prefixes of its own chunks
        // 4k + wave (scalars); the lane part comes from ballots in the node loop.
        // A tile holding a node of in-degree >= 15 (nibble 15, ~1e-12 of nodes)
        // reads in_off from HBM instead.
        uint32_t cinc = 0;
        bool wide = false;
        if (TOPO == IMP3D) {
            const uint2 w2 = reinterpret_cast<const uint2*>(L.ind)[lane];
            auto nsum = [](uint32_t w) { return (((w & 0x0F0F0F0Fu) + ((w >> 4) & 0x0F0F0F0Fu)) * 0x01010101u) >> 24; };
            auto has15 = [](uint32_t w) { return (w & (w >> 1) & (w >> 2) & (w >> 3) & 0x11111111u) != 0u; };
            uint32_t incl = nsum(w2.x) + nsum(w2.y);
            wide = __ballot(has15(w2.x) || has15(w2.y)) != 0ull;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t t = __shfl_up(incl, o, 64);
                if (lane >= (uint32_t)o) incl += t;
            }
            // exclusive chunk prefix at lane 4c (read per slot in the node loop)
            const uint32_t ex = __shfl_up(incl, 1, 64);
            cinc = lane == 0 ? 0u : ex;
        }
        uint32_t t_next = tw.t + tw.step;
        if (dyn) {
            // (block-uniform, and known to be: the next tile's in-list range is then two scalar
            // loads, not vector loads whose wait at the next tile's start also waited for this
            // tile's state stores)
            t_next = __builtin_amdgcn_readfirstlane(L.qn[it & 1]);
            ++it;
            // the next tile's in-edge range (two uniform loads, consumed next tile)
            if (TOPO == IMP3D) {
                TileWalk nw = tw;
                nw.t = t_next;
                uint32_t nti;
                pf_tile = 0xFFFFFFFFu;
                if (nw.t < nw.end && nw.tile(nti)) {
                    const uint32_t nT = (a.lo / TILE + nti) * TILE;
                    pf_lo = ld_const(a.in_off + max(a.lo, nT));
                    pf_hi = ld_const(a.in_off + min(a.lo + a.nloc, nT + TILE));
                    pf_tile = nti;
                }
            }
        }

        // per node, 16 bits (two nodes per word): bits 0-5 lattice mask, bit 6 draw a
        // next-round direction, bits 7-10 the node byte's flag bits 3-6
        uint32_t pend[(NPT + 1) / 2];
#pragma unroll
        for (int k = 0; k < (NPT + 1) / 2; ++k) pend[k] = 0u;
        {
            // Lattice coordinates of the WAVE's first node of slot k (wave-uniform, so
            // scalar), advanced by TPB per slot.  A wave whose 64 nodes are all
            // interior (no lattice boundary; ~93 % of waves at g = 1000) takes mask =
            // 63 without per-lane coordinates; the others compute each node's mask.
            const uint32_t wbase = __builtin_amdgcn_readfirstlane(threadIdx.x & ~63u);
            uint32_t wcx = 0, wcy = 0, wcz = 0;
            if (TOPO != LINE) {
                const uint32_t jw = T + wbase;
                wcx = fastdiv(jw, G.div_g2);
                const uint32_t rem = jw - wcx * G.g2;
                wcy = fastdiv(rem, G.div_g);
                wcz = rem - wcy * G.g;
            }
            // lattice directions gathered from HBM / L2; the j +- 1 ones (z +- 1, or both
            // line neighbours) are the neighbour lanes' own (s, w)
            constexpr uint32_t NDG = TOPO == LINE ? 0u : 4u;
            constexpr int NG = 1;  // node slots per group in flight (2 at 5 waves/SIMD spilled 49 VGPRs)
#pragma unroll
            for (int k0 = 0; k0 < NPT; k0 += NG) {
                __builtin_amdgcn_s_setprio(PRIO);
                // phase A: node byte, present mask, lattice senders (from the staged
                // direction bytes), one gather per direction -- a direction without a
                // sender reads the zero sentinel swc[ext_hi] (adding +0.0 is exact)
                // in-edge ranges of the group's nodes (all lanes take part in the ballots)
                uint32_t epre[NG], edeg[NG];
#pragma unroll
                for (int h = 0; h < NG; ++h) {
                    epre[h] = edeg[h] = 0u;
                    if (TOPO == IMP3D) {
                        const int k = k0 + h;
                        const uint32_t jl = k * TPB + threadIdx.x;
                        const uint32_t d = (lds_byte(L.ind, jl >> 1) >> ((jl & 1u) * 4u)) & 15u;
                        uint32_t ex = mbcnt64(__ballot(d & 1u)) + 2u * mbcnt64(__ballot(d & 2u));
                        if (__ballot(d >= 4u)) ex += 4u * mbcnt64(__ballot(d & 4u)) + 8u * mbcnt64(__ballot(d & 8u));
                        const int wvu = __builtin_amdgcn_readfirstlane((int)wv);
                        epre[h] = (uint32_t)__builtin_amdgcn_readlane((int)cinc, 16 * k + 4 * wvu) + ex;
                        edeg[h] = d;
                    }
                }
                // per node: byte | mask << 8 | from << 14 | in-degree << 20 (one register)
                uint32_t gst[NG];
                double2 m[NG][NDG > 0 ? NDG : 1];
#pragma unroll
                for (int h = 0; h < NG; ++h) {
                    const int k = k0 + h;
                    const uint32_t j = T + k * TPB + threadIdx.x;
                    if (TOPO != LINE && k > 0) {
                        wcz += TPB;
                        if (wcz >= G.g) {
                            const uint32_t q = fastdiv(wcz, G.div_g);
                            wcz -= q * G.g;
                            wcy += q;
                            if (wcy >= G.g) {
                                const uint32_t q2 = fastdiv(wcy, G.div_g);
                                wcy -= q2 * G.g;
                                wcx += q2;
                            }
                        }
                    }
                    const uint32_t jr = j - b_rows;
                    const uint32_t gbv = lds_byte(L.rows, jr);
                    uint32_t mask;
                    if (TOPO == LINE) {
                        mask = present_mask<TOPO>(j, G);
                    } else {
                        const uint32_t gm = G.g - 1u;
                        const bool interior = wcz >= 1u && wcz + 64u < gm && wcy >= 1u && wcy < gm && wcx >= 1u && wcx < gm;
                        mask = interior ? 63u : present_mask<TOPO>(j, G);
                    }
                    uint32_t from = 0;
                    if (TOPO == LINE) {
                        from |= ((mask & 1u) && (lds_byte(L.rows, (mask & 1u) ? jr - 1 : jr) & DIR_MASK) == 1u) ? 1u : 0u;
                        from |= ((mask & 2u) && (lds_byte(L.rows, (mask & 2u) ? jr + 1 : jr) & DIR_MASK) == 0u) ? 2u : 0u;
                    } else {
                        // absent neighbours read a harmless in-range byte and are masked out
                        const uint32_t bxm = lds_byte(L.xm, (mask & 1u) ? j - G.g2 - b_xm : 0u);
                        const uint32_t bxp = lds_byte(L.xp, (mask & 2u) ? j + G.g2 - b_xp : 0u);
                        const uint32_t byp = lds_byte(L.rows, (mask & 4u) ? jr + G.g : jr);
                        const uint32_t bym = lds_byte(L.rows, (mask & 8u) ? jr - G.g : jr);
                        const uint32_t bzp = lds_byte(L.rows, (mask & 16u) ? jr + 1 : jr);
                        const uint32_t bzm = lds_byte(L.rows, (mask & 32u) ? jr - 1 : jr);
                        from = ((bxm & DIR_MASK) == 1u ? 1u : 0u) | ((bxp & DIR_MASK) == 0u ? 2u : 0u) |
                               ((byp & DIR_MASK) == 3u ? 4u : 0u) | ((bym & DIR_MASK) == 2u ? 8u : 0u) |
                               ((bzp & DIR_MASK) == 5u ? 16u : 0u) | ((bzm & DIR_MASK) == 4u ? 32u : 0u);
                        from &= mask;
                    }
                    if (!(j >= j0 && j < j1)) from = 0u;
                    gst[h] = gbv | (mask << 8) | (from << 14) | (edeg[h] << 20);
                    // unconditional (index clamped into the tile's valid range; invalid lanes'
                    // values are never used): a load under a branch made the compiler wait
                    // for it before issuing the lattice gathers
                    own[k] = swc[min(max(j, j0), j1 - 1u)];
#pragma unroll
                    for (uint32_t d = 0; d < NDG; ++d)
                        m[h][d] = ld_sw(swc + ((from >> d) & 1u ? nbr<TOPO>(j, d, G) : a.ext_hi));
                }
                __builtin_amdgcn_s_setprio(0);
                // phase B: canonical fold (own half, lattice slots in slot order, random
                // edges by ascending sender; every message contributes the sender's half),
                // ratio test, next-round state
#pragma unroll
                for (int h = 0; h < NG; ++h) {
                    const int k = k0 + h;
                    const uint32_t jl = k * TPB + threadIdx.x;
                    const uint32_t j = T + jl;
                    const bool valid = j >= j0 && j < j1;
                    // Imp3D, staged tile: the node's window of the used-in-edge bitmap and its first
                    // used in-edge's message, read from LDS while the slot's loads are in flight (the
                    // fold needed both after the loads, one LDS round trip after the other).  A node's
                    // in-edges fit one 32-bit window (in-degree <= 14 outside `wide` tiles).
                    uint32_t pwin = 0u, pqb = 0u;
                    if (TOPO == IMP3D && staged && !wide) {
                        const uint32_t* bw = reinterpret_cast<const uint32_t*>(L.bits);
                        pqb = epre[h];
                        const uint32_t nd = gst[h] >> 20;
                        pwin = __builtin_amdgcn_alignbit(bw[(pqb >> 5) + 1], bw[pqb >> 5], pqb & 31u) & ((1u << nd) - 1u);
                    }
                    // j + 1 / j - 1: the neighbour lane's own (s, w) by DPP (all lanes active
                    // here), across the wave's ends from the values staged in L.zb; a load
                    // only where that lane's node is outside the tile's valid range
                    // (partial tiles at slab ends)
                    double2 zP = make_double2(0.0, 0.0), zM = zP;
                    {
                        constexpr uint32_t dP = TOPO == LINE ? 1u : 4u, dM = TOPO == LINE ? 0u : 5u;
                        const uint32_t from = (gst[h] >> 14) & 63u;
                        zP = dpp_double2<0x130>(own[k]);  // wave_shl:1 -- lane + 1's (s, w)
                        zM = dpp_double2<0x138>(own[k]);  // wave_shr:1 -- lane - 1's (s, w)
                        if (lane == 63u) zP = L.zb[wv][k][1];
                        if (lane == 0u) zM = L.zb[wv][k][0];
                        if (!((from >> dP) & 1u)) zP = make_double2(0.0, 0.0);
                        else if (lane != 63u && j + 1u >= j1) zP = ld_sw(swc + j + 1);
                        if (!((from >> dM) & 1u)) zM = make_double2(0.0, 0.0);
                        else if (lane != 0u && j <= j0) zM = ld_sw(swc + j - 1);
                    }
                    // every load of the slot retired here, on all paths: the slot's state store is then the
                    // only memory operation the next slot's loads could wait for, and they do not
                    // (without it the compiler waited vmcnt(0) before every slot's gathers -- a lane
                    // range with no valid node skips the fold that consumes the loads)
                    __builtin_amdgcn_s_waitcnt(vmcnt_enc(0));
                    if (valid) {
                        const uint32_t b = gst[h] & 0xFFu, mask = (gst[h] >> 8) & 63u, from = (gst[h] >> 14) & 63u;
                        const uint32_t deg = popc6(mask) + (TOPO == IMP3D ? 1u : 0u);
                        bool active = (b & B_ACTIVE) != 0;
                        const double2 sv = own[k];

                        const bool halve = active && deg > 0;
                        const double hf = halve ? 0.5 : 1.0;  // exact either way
                        double acc_s = sv.x * hf;
                        double acc_w = sv.y * hf;
                        // fused: fma(m, 0.5, acc) rounds once, exactly like the specification's
                        // acc + m * 0.5 whenever m * 0.5 is exact, i.e. |m| >= 2^-1021; every
                        // node checks its own round-start (s, w) -- the values its messages
                        // carry this round -- against 2^-1020 (Ctl::tiny, gp_step fails)
                        auto fold = [&](const double2 mi) {
                            acc_s = __builtin_fma(mi.x, 0.5, acc_s);
                            acc_w = __builtin_fma(mi.y, 0.5, acc_w);
                        };
                        tiny |= (sv.y < 0x1p-1020) | (sv.x != 0.0 && sv.x < 0x1p-1020);
                        bool recv = from != 0;
                        // lattice slots in slot order: line j-1, j+1; 3D x-1, x+1, y+1, y-1, z+1, z-1
                        if (TOPO == LINE) {
                            fold(zM);
                            fold(zP);
                        } else {
#pragma unroll
                            for (uint32_t d = 0; d < NDG; ++d) fold(m[h][d]);
                            fold(zP);
                            fold(zM);
                        }
                        if (TOPO == IMP3D) {
                            uint32_t e_b = e_lo + epre[h], e_e = e_b + (gst[h] >> 20);
                            if (wide) {
                                e_b = a.in_off[j];
                                e_e = a.in_off[j + 1];
                            }
                            if (staged && !wide) {
                                // the window and first message read above; the rest set bit by set
                                // bit (ascending sender = canonical order), edge q's message at slot q
                                uint32_t win = pwin;
                                while (win) {
                                    const uint32_t q = pqb + (uint32_t)__builtin_ctz(win);
                                    win &= win - 1u;
                                    fold(L.msg[q]);
                                    recv = true;
                                }
                            } else if (staged) {
                                // the node's used in-edges: its window of the tile bitmap, 32 bits
                                // at a time (funnel shift of two LDS words), walked set bit by set
                                // bit (ascending sender = canonical order); edge q's message is at
                                // slot q
                                const uint32_t* bw = reinterpret_cast<const uint32_t*>(L.bits);
                                const uint32_t qe = e_e - e_lo;
                                for (uint32_t q0 = e_b - e_lo; q0 < qe; q0 += 32u) {
                                    uint32_t win = __builtin_amdgcn_alignbit(bw[(q0 >> 5) + 1], bw[q0 >> 5], q0 & 31u);
                                    if (qe - q0 < 32u) win &= (1u << (qe - q0)) - 1u;
                                    while (win) {
                                        const uint32_t q = q0 + (uint32_t)__builtin_ctz(win);
                                        win &= win - 1u;
                                        fold(L.msg[q]);
                                        recv = true;
                                    }
                                }
                            } else {  // rare: tile in-degree above SLOTS
                                for (uint32_t e = e_b; e < e_e; ++e) {
                                    const uint32_t i = in_src[e];
                                    bool sent;
                                    double2 mi = make_double2(0.0, 0.0);
                                    const bool rem = REMOTE && i - a.lo >= a.nloc;
                                    uint32_t xi = 0;
                                    if (rem) {  // the sender's list entry (see the in-edge pass)
                                        const uint32_t k = a.rk[e];
                                        const XHdr h = a.xhdr[k >> 6];
                                        sent = (h.mask >> (k & 63u)) & 1ull;
                                        xi = min(h.base + (uint32_t)__popcll(h.mask & ((1ull << (k & 63u)) - 1ull)),
                                                 a.xnv - 1u);
                                    } else if (all_active) {
                                        const uint32_t di = popc6(present_mask<IMP3D>(i, G)) + 1u;
                                        sent = uniform(a.k0, a.k1, S_PUSHSUM, i, r, di) == di - 1u;
                                    } else {
                                        sent = (rbc[(i >> 6) - (a.lo >> 6)] >> (i & 63)) & 1ull;
                                    }
                                    if (sent) mi = rem ? a.xvals[xi] : ld_sw(swc + i);
                                    if (sent) {
                                        fold(mi);
                                        recv = true;
                                    }
                                }
                            }
                        }
                        uint32_t flags = b & (B_ACTIVE | B_CONV | (3u << CNT_SHIFT));
                        if (recv) {
                            if (!(b & B_CONV)) {
                                uint32_t cnt3 = (b >> CNT_SHIFT) & 3u;
                                cnt3 = ratio_moved(sv.x, sv.y, acc_s, acc_w) ? 0u : cnt3 + 1u;
                                flags = (flags & ~(3u << CNT_SHIFT)) | (cnt3 << CNT_SHIFT);
                                if (cnt3 == 3) {
                                    flags |= B_CONV;
                                    ++alerts;
                                }
                            }
                            if (!active) {
                                ++newly;
                                flags |= B_ACTIVE;
                                active = true;
                            }
                        }
                        // next-round direction drawn below, one Philox batch for the thread's nodes
                        pend[k >> 1] |= (mask | (active && deg > 0 ? 64u : 0u) | ((flags >> 3) << 7)) << (16 * (k & 1));
                        st_stream(swn + j, make_double2(acc_s, acc_w));
                    }
                }
                // SNDPF: after the first node slot (the next tile's in-edge range has arrived by
                // then), its senders by LDS-DMA; this tile's were read in its in-edge pass, and the
                // tile's closing barrier retires the copy before the next tile reads it
                if (SNDPF && TOPO == IMP3D && k0 == 0) {
                    snd_tile = 0xFFFFFFFFu;
                    if (pf_tile != 0xFFFFFFFFu && pf_hi - pf_lo <= cap) {
                        snd_off = dma_stage_words(snd, srcp, pf_lo, pf_hi);
                        snd_tile = pf_tile;
                    }
                }
            }
        }
        // next-round directions of this thread's nodes: one Philox batch
        {
            uint32_t node[NPT], x[NPT], y[NPT];
#pragma unroll
            for (int k = 0; k < NPT; ++k) node[k] = T + k * TPB + threadIdx.x;
            philox2_batch<NPT>(node, r + 1, S_PUSHSUM, a.k0, a.k1, x, y);
#pragma unroll
            for (int k = 0; k < NPT; ++k) {
                const uint32_t jl = k * TPB + threadIdx.x;
                const bool valid = node[k] >= j0 && node[k] < j1;
                const uint32_t pk = pend[k >> 1] >> (16 * (k & 1));
                const uint32_t mask = pk & 63u;
                uint32_t dir = DIR_NONE;
                if (pk & 64u) dir = slot_to_dir_fast(mask, uniform_from(x[k], y[k], popc6(mask) + (TOPO == IMP3D ? 1u : 0u)));
                if (valid) reinterpret_cast<uint8_t*>(L.out)[jl] = (uint8_t)((((pk >> 7) & 15u) << 3) | dir);
                if (TOPO == IMP3D) {
                    const unsigned long long bits = __ballot(valid && dir == DIR_RANDOM);
                    if (lane == 0) {  // the slab's first tile may start below lo: no word there
                        const int64_t wi = (int64_t)((T + k * TPB + (threadIdx.x & ~63u)) >> 6) - (int64_t)(a.lo >> 6);
                        if (wi >= 0) a.rbn[wi] = bits;
                    }
                }
            }
        }
        __syncthreads();
        // node bytes out as words (allocations are padded past P)
        for (uint32_t w = threadIdx.x; w < (uint32_t)(TILE / 4); w += TPB) {
            const uint32_t jw = T + w * 4;
            if (jw >= j0 && jw + 4 <= j1) {
                st_stream(reinterpret_cast<uint32_t*>(a.nbn + T) + w, L.out[w]);
            } else {
                for (uint32_t b = 0; b < 4; ++b)
                    if (jw + b >= j0 && jw + b < j1) a.nbn[jw + b] = reinterpret_cast<const uint8_t*>(L.out)[w * 4 + b];
            }
        }
        // no barrier here: the next tile's in-edge pass and staging copies write
        // bits / msg / rows / xm / xp / off, none of which this byte output reads,
        // and its node phase writes L.out only after its staging barrier
        tw.t = t_next;
    }
        if (!dyn || ++victim >= 8u) break;
        const uint32_t c = (blockIdx.x + victim) & 7u;
        tw.qc = a.tq + c * TQ_STRIDE;
        tw.wl = a.wt + a.wo[c];
        tw.end = a.wo[c + 1] - a.wo[c];
        if (threadIdx.x == 0) L.qn[it & 1] = atomicAdd(tw.qc, 1u);
        __syncthreads();
        tw.t = __builtin_amdgcn_readfirstlane(L.qn[it & 1]);
        ++it;
    }
}

// Block sums of this block's alerts / newly active nodes (valid in thread 0).
// Uses L.red; the barrier also orders the block's last byte output before any
// later LDS reuse.
__device__ __forceinline__ void block_counts(uint32_t (*red)[TPB / 64], uint32_t& x, uint32_t& y) {
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        x += __shfl_xor(x, o, 64);
        y += __shfl_xor(y, o, 64);
    }
    if (lane == 0) {
        red[0][wv] = x;
        red[1][wv] = y;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        x = 0;
        y = 0;
        for (int w = 0; w < TPB / 64; ++w) {
            x += red[0][w];
            y += red[1][w];
        }
    }
}

// Thread 0: add the block's counts to the round accumulators with returning
// atomics and wait for them, so they are performed before the block arrives
// at the round close.
__device__ __forceinline__ void add_round_counts(Ctl* ctl, uint32_t x, uint32_t y) {
    unsigned long long d = 0;
    if (x) d += __hip_atomic_fetch_add(&ctl->round_alerts, (unsigned long long)x, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
    if (y) d += __hip_atomic_fetch_add(&ctl->round_active, (unsigned long long)y, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("" ::"v"(d));
    __builtin_amdgcn_s_waitcnt(0);
}

template <int TOPO, bool REMOTE>
__global__ __launch_bounds__(TPB, GP_MINB) void k_ps_tile(RoundArgs a, uint32_t r) {
    __shared__ TileLdsP<REMOTE> L;
    // one rank: the next tile's in-edge senders, LDS-DMA'd during this tile's node phase.  An LDS
    // object of its own, so the compiler can tell that the node phase's LDS reads do not read it
    // and does not wait for the copy before each of them
    __shared__ uint32_t snd[PsSlots<REMOTE>::SNDPF ? PsSlots<REMOTE>::SLOTS + DMA_SLACK : 1];
    Ctl* ctl = a.ctl;
    if (ld_agent(&ctl->done)) return;
    const bool all_active = ld_agent(&ctl->all_active) != 0;
    uint32_t alerts = 0, newly = 0;
    bool tiny = false;
    ps_tiles<TOPO, REMOTE>(a, r, L, snd, all_active, alerts, newly, tiny);
    if (__ballot(tiny) && (threadIdx.x & 63u) == 0) atomicOr(&ctl->tiny, 1u);
    block_counts(L.red, alerts, newly);
    if (threadIdx.x == 0) {
        if (a.fuse == 2) {
            block_done_close_sharded(ctl, a.G.P, a.G.T, r, alerts, newly);
        } else if (a.fuse) {
            add_round_counts(ctl, alerts, newly);
            block_done_close(ctl, a.G.P, a.G.T, r);
        } else {
            if (alerts) atomicAdd(&ctl->round_alerts, (unsigned long long)alerts);
            if (newly) atomicAdd(&ctl->round_active, (unsigned long long)newly);
        }
    }
}

// ---------------------------------------------------------------- gossip
// Deliveries to j = lattice senders pointing here + Imp3D random-edge senders
// (bitmap) + the injector; all dropped if j was converged at round start.
template <int TOPO, bool REMOTE>
__global__ __launch_bounds__(TPB, GP_MINB) void k_gossip_tile(RoundArgs a, uint32_t r) {
    __shared__ TileLds L;
    Ctl* ctl = a.ctl;
    if (ld_agent(&ctl->done)) return;
    const long long inj = ld_agent(&ctl->inj_target);
    const Geom G = a.G;
    const uint32_t H = TOPO == LINE ? 1u : G.g;
    uint32_t alerts = 0;
    const int lane = threadIdx.x & 63;

    for (TileWalk tw(a); tw.t < tw.end; tw.t += tw.step) {
        uint32_t ti;
        if (!tw.tile(ti)) continue;
        // tiles sit on global multiples of TILE (4-aligned word I/O, 64-aligned
        // ballot words); the slab's first and last tile may be partial
        const uint32_t T = (a.lo / TILE + ti) * TILE;
        const uint32_t j0 = max(a.lo, T);
        const uint32_t j1 = min(a.lo + a.nloc, T + TILE);
        uint32_t e_lo = 0, e_hi = 0;
        if (TOPO == IMP3D) {
            e_lo = ld_const(a.in_off + j0);
            e_hi = ld_const(a.in_off + j1);
        }
        int32_t c0[NPT];
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
            const uint32_t j = T + k * TPB + threadIdx.x;
            c0[k] = (j >= j0 && j < j1) ? a.c[j] : (int32_t)GOSSIP_DONE;
        }
        const uint32_t b_rows = dma_stage_bytes(L.rows, a.nbc, (int64_t)j0 - H, (int64_t)j1 + H, a.ext_lo, a.ext_hi);
        uint32_t b_xm = 0, b_xp = 0;
        if (TOPO != LINE) {
            b_xm = dma_stage_bytes(L.xm, a.nbc, (int64_t)j0 - G.g2, (int64_t)j1 - G.g2, a.ext_lo, a.ext_hi);
            b_xp = dma_stage_bytes(L.xp, a.nbc, (int64_t)j0 + G.g2, (int64_t)j1 + G.g2, a.ext_lo, a.ext_hi);
        }
        const uint32_t cnt = e_hi - e_lo;
        const bool staged = cnt <= (uint32_t)SRC_CAP;
        int o_off = 0;  // L.off[jl + o_off] = in_off[T + jl]
        if (TOPO == IMP3D) {
            o_off = (int)dma_stage_words(L.off, a.in_off, j0, j1 + 1) - (int)(j0 - T);
            if (staged) {
                // all sender loads, then all bitmap loads, in flight together
                constexpr int FU = SRC_CAP / TPB;
                uint32_t isrc[FU];
#pragma unroll
                for (int m = 0; m < FU; ++m) {
                    const uint32_t q = threadIdx.x + m * TPB;
                    isrc[m] = q < cnt ? a.in_src[e_lo + q] : 0u;
                }
                // the senders' direction draws of round r as one Philox batch; the
                // bitmap (bit = active and the draw picks the random slot) is read
                // only where the draw picks it, ~1/7 of the in-edges, instead of a
                // random 128-byte line per in-edge
                uint32_t X[FU], Y[FU];
                philox2_batch<FU>(isrc, r, S_GOSSIP, a.k0, a.k1, X, Y);
                unsigned long long wv[FU];
#pragma unroll
                for (int m = 0; m < FU; ++m) {
                    const uint32_t q = threadIdx.x + m * TPB;
                    const uint32_t li = isrc[m] - a.lo;
                    const uint32_t di = popc6(present_mask<IMP3D>(isrc[m], G)) + 1u;
                    const bool pick = uniform_from(X[m], Y[m], di) == di - 1u;
                    wv[m] = q >= cnt ? 0ull
                            : (!REMOTE || li < a.nloc) ? (pick ? a.rbc[(isrc[m] >> 6) - (a.lo >> 6)] : 0ull)
                                          : (a.rtag[e_lo + q] == r ? ~0ull : 0ull);
                }
#pragma unroll
                for (int m = 0; m < FU; ++m) {
                    const uint32_t q = threadIdx.x + m * TPB;
                    if (q < cnt)
                        reinterpret_cast<uint8_t*>(L.sent)[q] = (uint8_t)((wv[m] >> (isrc[m] & 63)) & 1ull);
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
            const uint32_t jl = k * TPB + threadIdx.x;
            const uint32_t j = T + jl;
            const bool valid = j >= j0 && j < j1;
            uint32_t dir = DIR_NONE;
            if (valid) {
                const uint32_t mask = present_mask<TOPO>(j, G);
                int32_t c1 = c0[k];
                if (c1 < (int32_t)GOSSIP_DONE) {
                    uint32_t inc = (long long)j == inj ? 1u : 0u;
                    if (TOPO == LINE) {
                        inc += (mask & 1u) && (lds_byte(L.rows, j - 1 - b_rows) & DIR_MASK) == 1u;
                        inc += (mask & 2u) && (lds_byte(L.rows, j + 1 - b_rows) & DIR_MASK) == 0u;
                    } else {
                        inc += (mask & 1u) && (lds_byte(L.xm, j - G.g2 - b_xm) & DIR_MASK) == 1u;
                        inc += (mask & 2u) && (lds_byte(L.xp, j + G.g2 - b_xp) & DIR_MASK) == 0u;
                        inc += (mask & 4u) && (lds_byte(L.rows, j + G.g - b_rows) & DIR_MASK) == 3u;
                        inc += (mask & 8u) && (lds_byte(L.rows, j - G.g - b_rows) & DIR_MASK) == 2u;
                        inc += (mask & 16u) && (lds_byte(L.rows, j + 1 - b_rows) & DIR_MASK) == 5u;
                        inc += (mask & 32u) && (lds_byte(L.rows, j - 1 - b_rows) & DIR_MASK) == 4u;
                    }
                    if (TOPO == IMP3D) {
                        const uint32_t e_b = L.off[jl + o_off], e_e = L.off[jl + 1 + o_off];
                        if (staged) {
                            for (uint32_t e = e_b; e < e_e; ++e) inc += lds_byte(L.sent, e - e_lo);
                        } else {
                            for (uint32_t e = e_b; e < e_e; ++e) {
                                const uint32_t i = a.in_src[e];
                                const uint32_t li = i - a.lo;
                                inc += (!REMOTE || li < a.nloc) ? (uint32_t)((a.rbc[(i >> 6) - (a.lo >> 6)] >> (i & 63)) & 1ull)
                                                   : (a.rtag[e] == r ? 1u : 0u);
                            }
                        }
                    }
                    if (inc) {
                        c1 += (int32_t)inc;
                        a.c[j] = c1;
                        alerts += c1 > 10;  // the receipt that finds rumours == 10 (Program.fs:92-94)
                    }
                }
                const bool active = ((j == a.seed_node) || c1 >= 1) && c1 <= 10;
                if (active) {
                    const uint32_t deg = popc6(mask) + (TOPO == IMP3D ? 1u : 0u);
                    if (deg > 0) dir = slot_to_dir(mask, uniform(a.k0, a.k1, S_GOSSIP, j, r + 1, deg));
                }
                reinterpret_cast<uint8_t*>(L.out)[jl] = (uint8_t)dir;
            }
            if (TOPO == IMP3D) {
                const unsigned long long bits = __ballot(valid && dir == DIR_RANDOM);
                if (lane == 0) {  // the slab's first tile may start below lo: no word there
                    const int64_t wi = (int64_t)((T + k * TPB + (threadIdx.x & ~63u)) >> 6) - (int64_t)(a.lo >> 6);
                    if (wi >= 0) a.rbn[wi] = bits;
                }
            }
        }
        __syncthreads();
        for (uint32_t w = threadIdx.x; w < (uint32_t)(TILE / 4); w += TPB) {
            const uint32_t jw = T + w * 4;
            if (jw >= j0 && jw + 4 <= j1) {
                reinterpret_cast<uint32_t*>(a.nbn + T)[w] = L.out[w];
            } else {
                for (uint32_t b = 0; b < 4; ++b)
                    if (jw + b >= j0 && jw + b < j1) a.nbn[jw + b] = reinterpret_cast<const uint8_t*>(L.out)[w * 4 + b];
            }
        }
        __syncthreads();
    }
    uint32_t x = alerts;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    if (lane == 0) L.red[0][threadIdx.x >> 6] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        x = 0;
        for (int w = 0; w < TPB / 64; ++w) x += L.red[0][w];
        if (x) atomicAdd(&ctl->round_alerts, (unsigned long long)x);
    }
}

// Random-edge bits of round 0 (only the seed can be sending).
// nb indexed by global id; bit (j - lo) of rb for the slab's nodes.
// Word w holds ids [64 (w + lo/64), +64) (global 64-alignment, as the round kernels).
__global__ __launch_bounds__(TPB) void k_rbits_init(const uint8_t* nb, uint64_t* rb, uint32_t lo, uint32_t nloc,
                                                    uint32_t nwords) {
    const uint32_t j00 = lo & ~63u;
    for (uint32_t jb = blockIdx.x * TPB; jb < nwords * 64u; jb += gridDim.x * TPB) {
        const uint32_t j = j00 + jb + threadIdx.x;
        const bool bit = j >= lo && j - lo < nloc && (nb[j] & DIR_MASK) == DIR_RANDOM;
        const unsigned long long bits = __ballot(bit);
        if ((threadIdx.x & 63) == 0) rb[(j >> 6) - (lo >> 6)] = bits;
    }
}

// Tiles covering the ids [lo, lo + nloc) (tiles sit on global multiples of TILE).
static uint32_t tiles_for(uint32_t lo, uint32_t nloc) {
    return (uint32_t)(((uint64_t)lo + nloc + TILE - 1) / TILE - lo / TILE);
}
// 64-bit words the ballot stores of one round touch (whole tiles) plus slack.
uint32_t rbits_words_for(uint32_t lo, uint32_t nloc) { return tiles_for(lo, nloc) * (TILE / 64) + 16u; }

RoundArgs make_round_args(const DevState& S, uint32_t round) {
    const int cur = round & 1;
    RoundArgs a;
    // node arrays indexed by global id: pointers offset by the slab's first id
    a.swc = S.sw[cur] ? S.sw[cur] - S.base : nullptr;
    a.swn = S.sw[cur ^ 1] ? S.sw[cur ^ 1] - S.base : nullptr;
    a.nbc = S.nb[cur] ? S.nb[cur] - S.base : nullptr;
    a.nbn = S.nb[cur ^ 1] ? S.nb[cur ^ 1] - S.base : nullptr;
    a.rbc = S.rbits[cur];
    a.rbn = S.rbits[cur ^ 1];
    a.in_off = S.in_off ? S.in_off - S.lo : nullptr;
    a.in_src = S.in_src;
    a.in_srcd = S.in_srcd;
    a.ind4 = S.ind4 ? S.ind4 - (S.lo / TILE) * (TILE / 2) : nullptr;
    a.rtag = S.rtag;
    a.rmsg = S.rmsg;
    a.rk = S.rk;
    a.xhdr = S.xhdr[round & 1];
    a.xvals = S.xvals[round & 1];
    a.xnv = S.xnv;
    a.c = S.c ? S.c - S.lo : nullptr;
    a.lo = S.lo;
    a.nloc = S.nloc;
    a.ext_lo = S.ext_lo;
    a.ext_hi = S.ext_hi;
    a.ctl = S.ctl;
    a.G = S.G;
    a.k0 = S.k0;
    a.k1 = S.k1;
    a.seed_node = S.seed_node;
    a.ntiles = tiles_for(S.lo, S.nloc);
    a.walk = S.tile_walk;
    a.stage_cap = S.tile_stage_cap;
    a.wx = S.tile_wx;
    a.fuse = S.fuse_finalize;
    a.wt = S.wtiles;
    for (int c = 0; c <= 8; ++c) a.wo[c] = S.woff[0][c];
    a.tq = S.tq + (round & 1) * 8 * TQ_STRIDE;
    a.tq_next = S.tq + ((round + 1) & 1) * 8 * TQ_STRIDE;
    return a;
}

// First plane (relative to the slab's) of region h of NR equal regions over nx planes.  (A last
// region half the size of the others measured within noise, profiles/r05/rejected/rlast.txt.)
uint32_t region_plane(uint32_t nx, int NR, int h) {
    if (h >= NR) return nx;
    return (uint32_t)((uint64_t)nx * h / NR);
}

// Region h of NR of a plane-aligned slab: planes [x0 + region_plane(h), x0 + region_plane(h + 1)),
// whose tiles (relative to lo / TILE) are [rb[h], rb[h + 1]) -- a tile belongs to the plane it
// starts in (the slab's first tile to the first plane).  False if the slab is not plane-aligned.
bool region_tiles(uint32_t lo, uint32_t nloc, uint64_t g2, int NR, uint32_t* rb) {
    if (!g2 || nloc % g2 || lo % g2 || NR < 1) return false;
    const uint32_t tb = lo / TILE;
    const uint32_t tend = (uint32_t)(((uint64_t)lo + nloc + TILE - 1) / TILE);
    const uint32_t x0 = (uint32_t)(lo / g2), nx = (uint32_t)(nloc / g2);
    for (int h = 0; h <= NR; ++h) {
        const uint64_t x = x0 + region_plane(nx, NR, h);
        rb[h] = (x <= x0 ? tb : (uint32_t)std::min<uint64_t>((x * g2 + TILE - 1) / TILE, tend)) - tb;
    }
    return true;
}

// Walk 3's visiting order (host, at create): walk 2's items (TileWalk) for each
// of the 8 XCDs, empty items dropped -- every tile of the slab exactly once.
// list: tiles relative to lo / TILE; woff[0][c]..woff[0][c + 1]: XCD c's items.
// NR > 1 (launch_round_regions): the planes of region h (region_tiles) dealt to the
// 8 XCDs in the same way, XCD c's items at woff[h][c]..woff[h][c + 1].
bool build_walk_list(const DevState& S, int NR, std::vector<uint32_t>& list, uint32_t woff[][9]) {
    const uint64_t g2 = S.G.g2;
    if (!g2 || S.nloc % g2 || S.lo % g2 || NR < 1 || NR > RREG_MAX) return false;
    const uint32_t tb = S.lo / TILE;
    const uint32_t tend = (uint32_t)(((uint64_t)S.lo + S.nloc + TILE - 1) / TILE);
    const uint32_t x0 = (uint32_t)(S.lo / g2), nx = (uint32_t)(S.nloc / g2);
    const uint32_t kp = (uint32_t)((g2 + TILE - 1) / TILE + 1);
    auto first = [&](uint32_t x) -> uint32_t {
        return x <= x0 ? tb : (uint32_t)std::min<uint64_t>((x * g2 + TILE - 1) / TILE, tend);
    };
    list.clear();
    for (int h = 0; h < NR; ++h) {
        const uint32_t r0 = x0 + region_plane(nx, NR, h);
        const uint32_t nr = x0 + region_plane(nx, NR, h + 1) - r0;
        for (uint32_t c = 0; c < 8; ++c) {
            woff[h][c] = (uint32_t)list.size();
            const uint32_t xa = r0 + (uint32_t)((uint64_t)nr * c / 8);
            const uint32_t nxa = r0 + (uint32_t)((uint64_t)nr * (c + 1) / 8) - xa;
            uint32_t nwin = S.tile_wx ? (nxa + S.tile_wx - 1) / S.tile_wx : 1u;
            if (nwin == 0) nwin = 1;
            for (uint32_t v = 0; v < nwin && nxa; ++v) {
                const uint32_t xs = (uint32_t)((uint64_t)nxa * v / nwin), xe = (uint32_t)((uint64_t)nxa * (v + 1) / nwin);
                for (uint32_t k = 0; k < kp; ++k)
                    for (uint32_t x = xa + xs; x < xa + xe; ++x) {
                        const uint32_t ti = first(x) + k;
                        if (ti < first(x + 1)) list.push_back(ti - tb);
                    }
            }
        }
        woff[h][8] = (uint32_t)list.size();
    }
    return list.size() == (size_t)(tend - tb);
}

// Resident 256-thread blocks of the push-sum tile kernel on this device (walk 3
// runs exactly that grid); 0 if unknown.
int ps_tile_resident_blocks(int topo, bool remote, int device) {
    const void* f = topo == LINE     ? reinterpret_cast<const void*>(&k_ps_tile<LINE, false>)
                    : topo == GRID3D ? reinterpret_cast<const void*>(&k_ps_tile<GRID3D, false>)
                    : remote         ? reinterpret_cast<const void*>(&k_ps_tile<IMP3D, true>)
                                     : reinterpret_cast<const void*>(&k_ps_tile<IMP3D, false>);
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, TPB, 0) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) return 0;
    return per_cu * cus;
}

// Launch h of round `round` when the round kernel runs region by region (DevState::rregions;
// Imp3D push-sum across ranks): region h's tiles, its own pair of queue counters by launch parity.
hipError_t launch_round_tile_region(const DevState& S, uint32_t round, uint32_t h, int grid, hipStream_t st) {
    if (S.alg != PUSHSUM || S.topo != IMP3D || !S.rk || !S.ind4 || !S.wtiles || S.tile_walk != 3 ||
        h >= S.rregions || (grid & 7))
        return hipErrorInvalidValue;
    RoundArgs a = make_round_args(S, round);
    for (int c = 0; c <= 8; ++c) a.wo[c] = S.woff[h][c];
    const uint64_t L = (uint64_t)round * S.rregions + h;
    a.tq = S.tq + (L & 1) * 8 * TQ_STRIDE;
    a.tq_next = S.tq + ((L + 1) & 1) * 8 * TQ_STRIDE;
    hipLaunchKernelGGL((k_ps_tile<IMP3D, true>), dim3(grid), dim3(TPB), 0, st, a, round);
    return hipGetLastError();
}

hipError_t launch_round_tile(const DevState& S, uint32_t round, int grid, hipStream_t st) {
    if (S.rregions > 1) return hipErrorInvalidValue;  // launch_round_tile_region per region
    const RoundArgs a = make_round_args(S, round);
    const dim3 g(grid), b(TPB);
    // Imp3D slabs of a multi-rank run (push-sum: received lists; gossip: tagged slots)
    const bool remote = S.alg == PUSHSUM ? S.rk != nullptr : S.rtag != nullptr;
    if (S.alg == PUSHSUM && S.topo == IMP3D && !S.ind4) return hipErrorInvalidValue;
    if (S.alg == PUSHSUM) {
        switch (S.topo) {
            case LINE: hipLaunchKernelGGL((k_ps_tile<LINE, false>), g, b, 0, st, a, round); break;
            case GRID3D: hipLaunchKernelGGL((k_ps_tile<GRID3D, false>), g, b, 0, st, a, round); break;
            default:
                if (remote) hipLaunchKernelGGL((k_ps_tile<IMP3D, true>), g, b, 0, st, a, round);
                else hipLaunchKernelGGL((k_ps_tile<IMP3D, false>), g, b, 0, st, a, round);
                break;
        }
    } else {
        switch (S.topo) {
            case LINE: hipLaunchKernelGGL((k_gossip_tile<LINE, false>), g, b, 0, st, a, round); break;
            case GRID3D: hipLaunchKernelGGL((k_gossip_tile<GRID3D, false>), g, b, 0, st, a, round); break;
            default:
                if (remote) hipLaunchKernelGGL((k_gossip_tile<IMP3D, true>), g, b, 0, st, a, round);
                else hipLaunchKernelGGL((k_gossip_tile<IMP3D, false>), g, b, 0, st, a, round);
                break;
        }
    }
    return hipGetLastError();
}

// Imp3D push-sum senders with their degree packed in the top two bits
// (deg - 4 in [0, 3]; every node has 3..6 lattice slots + the random one when
// g >= 2), so the tile kernel's in-edge pass needs no division to find it.
// Valid when every id fits 30 bits (P <= 2^30).
__global__ __launch_bounds__(TPB) void k_pack_src_deg(const uint32_t* src, uint32_t* out, uint32_t n, Geom G) {
    for (uint32_t e = blockIdx.x * TPB + threadIdx.x; e < n; e += gridDim.x * TPB) {
        const uint32_t i = src[e];
        const uint32_t deg = popc6(present_mask<IMP3D>(i, G)) + 1u;
        out[e] = i | ((deg - 4u) << 30);
    }
}

hipError_t launch_pack_src_deg(const uint32_t* src, uint32_t* out, uint32_t n, const Geom& G, int grid,
                               hipStream_t st) {
    hipLaunchKernelGGL(k_pack_src_deg, dim3(grid), dim3(TPB), 0, st, src, out, n, G);
    return hipGetLastError();
}

// Nibble in-degrees of the slab's tiles (DevState::ind4) from in_off.
// wide_at: in-degrees from this value on are stored as 15, the "read in_off"
// mark (15 in the product; tests lower it to exercise that path).
__global__ __launch_bounds__(TPB) void k_pack_ind4(const uint32_t* __restrict__ in_off, uint32_t lo, uint32_t nloc,
                                                   uint32_t j00, uint8_t* __restrict__ out, uint32_t nbytes,
                                                   uint32_t wide_at) {
    for (uint32_t b = blockIdx.x * TPB + threadIdx.x; b < nbytes; b += gridDim.x * TPB) {
        uint32_t v = 0;
#pragma unroll
        for (uint32_t h = 0; h < 2; ++h) {
            const uint32_t j = j00 + 2 * b + h;
            if (j - lo < nloc) {
                const uint32_t d = in_off[j + 1] - in_off[j];
                v |= (d >= wide_at ? 15u : d) << (4 * h);
            }
        }
        out[b] = (uint8_t)v;
    }
}

uint32_t ind4_bytes_for(uint32_t lo, uint32_t nloc) { return tiles_for(lo, nloc) * (TILE / 2) + 16u; }

hipError_t launch_pack_ind4(const DevState& S, uint32_t wide_at, int grid, hipStream_t st) {
    const uint32_t nbytes = tiles_for(S.lo, S.nloc) * (TILE / 2);
    hipLaunchKernelGGL(k_pack_ind4, dim3(grid), dim3(TPB), 0, st, S.in_off - S.lo, S.lo, S.nloc, (S.lo / TILE) * TILE,
                       S.ind4, nbytes, std::min(wide_at, 15u));
    return hipGetLastError();
}

hipError_t launch_rbits_init(const DevState& S, int grid, hipStream_t st) {
    hipLaunchKernelGGL(k_rbits_init, dim3(grid), dim3(TPB), 0, st, S.nb[0] - S.base, S.rbits[0], S.lo, S.nloc,
                       S.rbits_words);
    return hipGetLastError();
}

#ifdef GP_ROUND_WIDE
}  // namespace wide
#endif
}  // namespace gp
