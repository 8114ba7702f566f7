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
#include <type_traits>

#include "gp_internal.hpp"

namespace gp {

// Experiment knobs (tools/ablate.py); the product build uses the defaults.
#ifndef GP_PREFETCH
#define GP_PREFETCH 0
#endif
#ifndef GP_TPB
#define GP_TPB 256
#endif
#ifndef GP_NPT
#define GP_NPT 4
#endif
#ifndef GP_NT_LOADS
#define GP_NT_LOADS 1
#endif
#ifndef GP_NT_STORES
#define GP_NT_STORES 1
#endif
#ifndef GP_ABLATE
#define GP_ABLATE 0
#endif
#ifndef GP_MINB
#define GP_MINB 5  // __launch_bounds__ minimum waves per SIMD (= resident 256-thread blocks per CU):
                   // the LDS tile allows 5, so keep VGPRs <= 96 to not lose the fifth
#endif
#ifndef GP_MINB2
#define GP_MINB2 4  // k_ps_tile2: its message burst needs the registers of 4 waves/SIMD
#endif
#define ABL_NO_RGATHER 1   // in-list: decide but do not gather the sender's (s, w)
#define ABL_NO_LGATHER 2   // lattice: decide but do not gather
#define ABL_NO_INLIST 4    // skip the Imp3D in-list
#define ABL_NO_NEXTDIR 8   // skip the next-round Philox draw
#define ABL_NO_EPHILOX 16  // in-list: no Philox (sender never random)
#define ABL_BITMAP_ONLY 32 // in-list: always read the random-edge bitmap, never recompute Philox
#define ABL_NO_RATIO 64    // skip the ratio test
#define ABL_CHEAP_DECIDE 128  // in-list: a one-multiply hash instead of the sender's Philox draw
#define ABL_NO_XGATHER 256    // lattice: no gather from the x-1 / x+1 planes
#define ABL_NO_YGATHER 512    // lattice: no gather from the y-1 / y+1 rows
#define ABL_NO_ZGATHER 1024   // lattice: no gather from z-1 / z+1 (k_ps_tile2 only)
#define ABL_NO_RFOLD 2048     // in-list: decide and gather, but the nodes do not walk their bitmap window
#define ABL_FAKE_SRC 4096     // in-list: senders hashed from the edge index instead of loaded

namespace {

constexpr int TPB = GP_TPB;                // 256 (experiments: 128)
constexpr int NPT = GP_NPT;                // nodes per thread per tile
constexpr int TILE = TPB * NPT;            // 1024
constexpr int HMAX = 1625;                 // largest lattice edge with g^3 < 2^32
constexpr int W_ROWS = (TILE + 2 * HMAX) / 4 + 4;
constexpr int W_PLANE = TILE / 4 + 4;
constexpr int SRC_CAP = TILE * 3 / 2;       // staged in-list entries per tile (mean TILE)
constexpr int MSG_CAP = TILE * 3 / 8;       // random-edge messages parked per tile (mean ~TILE / 7)
constexpr uint16_t POS_NONE = 0xFFFF, POS_GLOBAL = 0xFFFE;

// Staged ranges are moved by 16-byte LDS-DMA (global_load_lds_dwordx4) from a
// 16-byte aligned start: every array has 8 words of slack for the alignment.
constexpr int DMA_SLACK = 8;

struct TileLds {
    uint32_t rows[W_ROWS + DMA_SLACK];   // direction bytes of [j0 - H, j1 + H)
    uint32_t xm[W_PLANE + DMA_SLACK];    // direction bytes of [j0 - g^2, j1 - g^2)
    uint32_t xp[W_PLANE + DMA_SLACK];    // direction bytes of [j0 + g^2, j1 + g^2)
    uint32_t off[TILE + 1 + DMA_SLACK];  // in_off[j0 .. j1]
    uint32_t src[SRC_CAP + DMA_SLACK];   // in_src[in_off[j0] .. in_off[j1])
    uint32_t sent[SRC_CAP / 4];  // gossip: byte per staged in-edge, sender used its random edge
    uint16_t pos[SRC_CAP];     // push-sum: slot of the edge's parked message (POS_NONE: not sent)
    double2 msg[MSG_CAP];      // push-sum: random-edge messages gathered by the flattened pass
    uint32_t out[TILE / 4];    // next-round node bytes, stored as words
    uint32_t red[2][TPB / 64];
};

// k_ps_tile<IMP3D, *, EDGES = true>: the in-edge decisions and random-edge
// gathers were done by k_ps_edges; the tile stages its in-edge bitmap and its
// compact messages instead of the senders.
constexpr int EW = SRC_CAP / 64;  // in-edge bitmap words per tile (k_ps_edges)

struct TileLdsE {
    uint32_t rows[W_ROWS + DMA_SLACK];
    uint32_t xm[W_PLANE + DMA_SLACK];
    uint32_t xp[W_PLANE + DMA_SLACK];
    uint32_t off[TILE + 1 + DMA_SLACK];
    unsigned long long bits[EW + 1];  // bit q: staged in-edge q (tile order) was used by its sender; bits[EW] = 0
    uint32_t bpre[EW + 1];            // sent edges before word w; bpre[EW] = all of them
    double2 msg[MSG_CAP];          // the tile's messages, in edge order
    uint32_t out[TILE / 4];
    uint32_t red[2][TPB / 64];
};

static_assert(TILE != 1024 || (EW == (int)EDGE_WORDS && MSG_CAP == (int)EDGE_MSGS), "gp_internal.hpp sizes");

// k_ps_tile<*, *, EDGES = false>: the tile decides its in-edges itself and
// parks the used ones' messages compactly in edge order (same layout as
// k_ps_edges' output).
// The used in-edges' (s, w) are gathered by LDS-DMA straight into per-edge
// slots (edge q's message at slot q -- lane-linear, so one global_load_lds per
// edge batch, no registers, no compaction).  A tile with more than SLOTS
// in-edges (6 sigma above the mean TILE: ~1e-9 of tiles) takes the unstaged path,
// so the node fold reads LDS only (no global fallback inside its loop, whose
// join would cost a vmcnt(0) wait per message).
constexpr int SLOTS = TILE + TILE / 8 + TILE / 16;  // 1216 at TILE = 1024: the LDS of 5 blocks per CU
constexpr int SLOT_FU = (SLOTS + TPB - 1) / TPB;  // in-edges per thread in the in-edge pass
constexpr int SLOT_W = (SLOTS + 63) / 64;         // bitmap words

struct TileLdsP {
    uint32_t rows[W_ROWS + DMA_SLACK];
    uint32_t xm[W_PLANE + DMA_SLACK];
    uint32_t xp[W_PLANE + DMA_SLACK];
    uint32_t off[TILE + 1 + DMA_SLACK];
    uint32_t src[1];                  // unused: the senders go straight to registers
    unsigned long long bits[SLOT_FU * (TPB / 64) + 1];  // bit q: in-edge q (tile order) was used by its sender; then 0
    uint32_t bpre[1];                                    // unused (EDGES layout)
    double2 msg[SLOTS];               // edge q's message at slot q
    uint32_t out[TILE / 4];
    uint32_t red[2][TPB / 64];
};

template <bool EDGES> struct TileLdsSel { using type = TileLdsP; };
template <> struct TileLdsSel<true> { using type = TileLdsE; };

__device__ __forceinline__ uint32_t lds_byte(const uint32_t* w, uint32_t idx) {
    return reinterpret_cast<const uint8_t*>(w)[idx];
}

// Copy the bytes of nb[lo, hi) (clamped to the ids [ext_lo, ext_hi) the slab's
// arrays hold, halos included) into LDS words; returns the node id of LDS byte
// 0.  `nb` is indexed by global id; reads at most 3 bytes either side of the
// range (allocations are padded and start 4-aligned).
__device__ __forceinline__ uint32_t stage_bytes(uint32_t* lds, const uint8_t* nb, int64_t lo, int64_t hi,
                                                uint32_t ext_lo, uint32_t ext_hi) {
    if (lo < (int64_t)ext_lo) lo = ext_lo;
    if (hi > (int64_t)ext_hi) hi = ext_hi;
    const uint32_t ws = (uint32_t)lo & ~3u;
    const int nw = hi > lo ? (int)(((uint32_t)hi + 3u - ws) >> 2) : 0;
    const uint32_t* src = reinterpret_cast<const uint32_t*>(nb + ws);
    for (int w = threadIdx.x; w < nw; w += TPB) lds[w] = src[w];
    return ws;
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
constexpr int DMA_ONCE = GP_NT_LOADS ? 2 : 0;

// LDS-DMA version of stage_bytes: node bytes nb[lo, hi) clamped to [ext_lo,
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
struct TileWalk {
    uint32_t t, end, step;
    // walk 2 only
    uint32_t mode, tb, tend, g2, x0, xa, nxa, kp, nwin;
    __device__ TileWalk(const RoundArgs& a) {
        const uint32_t G = gridDim.x;
        mode = a.walk;
        if (mode == 2 && a.G.g2 && G >= 8 && (G & 7) == 0) {
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

// Random-edge gathers touch one line per message and are never re-read this
// round: load them non-temporally so they do not evict the lattice
// neighbourhood the tiles share through the XCD's L2.
typedef double gp_d2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double2 ld_sw_once(const double2* p) {
#if GP_NT_LOADS
    const gp_d2v v = __builtin_nontemporal_load(reinterpret_cast<const gp_d2v*>(p));
    return make_double2(v.x, v.y);
#else
    return *p;
#endif
}

// Next-round state is written once and not read again this round: non-temporal
// stores keep it from displacing the current round's (s, w) in the XCD's L2,
// where the neighbouring tiles' lattice gathers look for it.
__device__ __forceinline__ void st_stream(double2* p, double2 v) {
#if GP_NT_STORES
    __builtin_nontemporal_store(v.x, &p->x);
    __builtin_nontemporal_store(v.y, &p->y);
#else
    *p = v;
#endif
}
__device__ __forceinline__ void st_stream(uint32_t* p, uint32_t v) {
#if GP_NT_STORES
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}

// ---- compacted-gather tile (k_ps_tile2)
constexpr int MCAP2 = 1280;                 // lattice + random messages gathered per tile (mean ~1030)
constexpr int MI2 = MCAP2 / TPB;            // gathers per thread
constexpr uint32_t REMOTE_TAG = 0xFFFFF000u;  // list entry >= this: remote message of staged edge ~entry

struct Tile2Lds {
    union {
        struct {
            uint32_t rows[W_ROWS];  // direction bytes of [j0 - H, j1 + H)
            uint32_t xm[W_PLANE];   // direction bytes of [j0 - g^2, j1 - g^2)
            uint32_t xp[W_PLANE];   // direction bytes of [j0 + g^2, j1 + g^2)
            uint32_t src[SRC_CAP];  // in_src[in_off[j0] .. in_off[j1])
        } s;
        double2 msg[MCAP2];         // after the decisions: the tile's messages (slot m's first
                                    // dword holds its source id until the gather lands)
    } u;
    uint32_t off[TILE + 1];         // in_off[T .. T + TILE]
    uint16_t pos[SRC_CAP];          // staged in-edge -> message slot (POS_NONE / POS_GLOBAL)
    uint32_t out[TILE / 4];
    uint32_t scan[TPB / 64 + 1];
    uint32_t red[2][TPB / 64];
};

// Exclusive scan of one value per thread over the block; `total` = block sum.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* lds, uint32_t& total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
    }
    if (lane == 63) lds[wid] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (int w = 0; w < TPB / 64; ++w) {
            const uint32_t t = lds[w];
            lds[w] = run;
            run += t;
        }
        lds[TPB / 64] = run;
    }
    __syncthreads();
    total = lds[TPB / 64];
    return incl - v + lds[wid];
}

}  // namespace

// ---------------------------------------------------------------- push-sum
// REMOTE: some in-edge senders live on other ranks (multi-GPU slabs); the
// single-GPU build of the kernel has no exchange-tag paths at all.
// LTAG: one-rank opt-in (GP_LTAG=1) -- the in-edge pass reads edge tags the senders
// wrote last round instead of redrawing their Philox (DevState::ltag).
template <int TOPO, bool REMOTE, bool EDGES, bool LTAG = false>
__global__ __launch_bounds__(TPB, GP_MINB) void k_ps_tile(RoundArgs a, uint32_t r) {
    static_assert(!EDGES || TOPO == IMP3D, "edge pass is Imp3D only");
    static_assert(!LTAG || (TOPO == IMP3D && !REMOTE && !EDGES), "edge tags: one-rank Imp3D only");
    __shared__ typename TileLdsSel<EDGES>::type L;
    Ctl* ctl = a.ctl;
    if (ld_agent(&ctl->done)) return;
    const bool all_active = ld_agent(&ctl->all_active) != 0;
    const double2* __restrict__ swc = a.swc;
    double2* __restrict__ swn = a.swn;
    const uint64_t* __restrict__ rbc = a.rbc;
    const uint32_t* __restrict__ in_src = a.in_src;
    const bool packed = a.in_srcd != nullptr;  // staged senders carry deg - 4 in bits 30-31
    const Geom G = a.G;
    const uint32_t H = TOPO == LINE ? 1u : G.g;
    uint32_t alerts = 0, newly = 0;
    const int lane = threadIdx.x & 63;

    // the next tile's in-edge range is loaded one tile ahead (two uniform loads),
    // so the senders can be staged in the same phase as everything else
    uint32_t pf_tile = 0xFFFFFFFFu, pf_lo = 0, pf_hi = 0, pf_tot = 0, pf_j0 = 0, pf_j1 = 0;
    for (TileWalk tw(a); tw.t < tw.end; tw.t += tw.step) {
        uint32_t ti;
        if (!tw.tile(ti)) continue;
        // tiles sit on global multiples of TILE (4-aligned word I/O, 64-aligned
        // ballot words); the slab's first and last tile may be partial
        const uint32_t T = (a.lo / TILE + ti) * TILE;
        const uint32_t j0 = max(a.lo, T);
        const uint32_t j1 = min(a.lo + a.nloc, T + TILE);
        uint32_t e_lo = 0, e_hi = 0, e_tot = 0;
        if (TOPO == IMP3D) {
            if (pf_tile == ti) {
                e_lo = pf_lo;
                e_hi = pf_hi;
                e_tot = pf_tot;
            } else {
                e_lo = a.in_off[j0];
                e_hi = a.in_off[j1];
                if (EDGES) e_tot = a.etot[ti];
            }
        }
        const uint32_t cnt = e_hi - e_lo;
        const bool staged = cnt <= min((uint32_t)(EDGES ? SRC_CAP : SLOTS), a.stage_cap);
        constexpr int FU = SLOT_FU;
        if (TOPO == IMP3D) {  // prefetch the next tile's in-edge range
            TileWalk nw = tw;
            nw.t += nw.step;
            uint32_t nti;
            if (nw.t < nw.end && nw.tile(nti)) {
                const uint32_t nT = (a.lo / TILE + nti) * TILE;
                pf_lo = a.in_off[max(a.lo, nT)];
                pf_hi = a.in_off[min(a.lo + a.nloc, nT + TILE)];
                if (EDGES) pf_tot = a.etot[nti];
                pf_tile = nti;
                pf_j0 = max(a.lo, nT);
                pf_j1 = min(a.lo + a.nloc, nT + TILE);
            }
        }
        if constexpr (TOPO == IMP3D && !EDGES) {
            if (staged) {
                // In-edge pass, ahead of the staging copies (its Philox chains wait for
                // the senders only, and its gathers retire at the staging barrier):
                // flattened, lane-balanced over the tile's in-edges, decide whether each
                // sender used its random edge (all FU Philox chains of a thread
                // independent), record the answers as a bitmap (edge
                // q = m * TPB + wave * 64 + lane is bit lane of word m * 4 + wave), and
                // gather the used edges' (s, w) by LDS-DMA into slot q (non-temporal:
                // one line per message, never re-read).  The previous tile's node phase
                // ended at a barrier and its byte output reads L.out only.
                const uint32_t wv = threadIdx.x >> 6;
                const uint32_t* srcp = packed ? a.in_srcd : in_src;
                // one rank, every node active, round > 0: the senders tagged this round's
                // random-edge sends in edge order last round (coalesced read, no Philox
                // redraw); round 0's directions come from k_init, which writes no tags
                const bool tagged = LTAG && all_active && r > 0;
                uint32_t isrc[FU], ideg[FU], itag[FU];
#pragma unroll
                for (int m = 0; m < FU; ++m) {
                    const uint32_t q = threadIdx.x + m * TPB;
                    const uint32_t raw = q < cnt ? ((GP_ABLATE & ABL_FAKE_SRC) ? ((e_lo + q) * 2654435761u) % a.G.P | 0xC0000000u
                                                                               : srcp[e_lo + q])
                                                 : 0u;
                    if (LTAG) itag[m] = (tagged && q < cnt) ? a.ltc[e_lo + q] : ~0u;
                    isrc[m] = packed ? raw & 0x3FFFFFFFu : raw;
                    ideg[m] = (raw >> 30) + 4u;
                }
#pragma unroll
                for (int m = 0; m < FU; ++m) {
                    const uint32_t q = threadIdx.x + m * TPB;
                    const uint32_t i = isrc[m];
                    bool sent = false;
                    if (q < cnt) {
                        if (REMOTE && i - a.lo >= a.nloc) {  // sender on another rank: the exchange tagged its message
                            sent = a.rtag[e_lo + q] == r;
                        } else if (GP_ABLATE & ABL_NO_EPHILOX) {
                            sent = false;
                        } else if (LTAG && tagged) {
                            sent = itag[m] == r;
                        } else if ((GP_ABLATE & ABL_CHEAP_DECIDE) && all_active) {
                            sent = ((i * 2654435761u + r * 40503u) >> 29) == 0u;
                        } else if (all_active && !(GP_ABLATE & ABL_BITMAP_ONLY)) {
                            const uint32_t di = packed ? ideg[m] : popc6(present_mask<IMP3D>(i, G)) + 1u;
                            sent = uniform(a.k0, a.k1, S_PUSHSUM, i, r, di) == di - 1u;
                        } else {
                            sent = (rbc[(i >> 6) - (a.lo >> 6)] >> (i & 63)) & 1ull;
                        }
                    }
                    const unsigned long long bal = __ballot(sent);
                    if (lane == 0) L.bits[m * (TPB / 64) + wv] = bal;
                    if (sent && !(GP_ABLATE & ABL_NO_RGATHER)) {
                        const double2* src = (REMOTE && i - a.lo >= a.nloc) ? a.rmsg + e_lo + q : swc + i;
                        __builtin_amdgcn_global_load_lds((gvoid_t*)src,
                                                         (lvoid_t*)(L.msg + (m * TPB + wv * 64)), 16, 0, DMA_ONCE);
                    }
                }
                if (threadIdx.x == 0) L.bits[FU * (TPB / 64)] = 0ull;
            }
        }
        // own (s, w): consumed after staging
        double2 own[NPT];
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
            const uint32_t j = T + k * TPB + threadIdx.x;
            own[k] = (j >= j0 && j < j1) ? swc[j] : make_double2(0.0, 1.0);
        }
        // every staging copy of the tile in flight at once (LDS-DMA)
        const uint32_t b_rows = dma_stage_bytes(L.rows, a.nbc, (int64_t)j0 - H, (int64_t)j1 + H, a.ext_lo, a.ext_hi);
        uint32_t b_xm = 0, b_xp = 0;
        if (TOPO != LINE) {
            b_xm = dma_stage_bytes(L.xm, a.nbc, (int64_t)j0 - G.g2, (int64_t)j1 - G.g2, a.ext_lo, a.ext_hi);
            b_xp = dma_stage_bytes(L.xp, a.nbc, (int64_t)j0 + G.g2, (int64_t)j1 + G.g2, a.ext_lo, a.ext_hi);
        }
        int o_off = 0;  // L.off[jl + o_off] = in_off[T + jl]
        if (TOPO == IMP3D) {
            o_off = (int)dma_stage_words(L.off, a.in_off, j0, j1 + 1) - (int)(j0 - T);
            if constexpr (EDGES) {
                if (staged) {
                    dma_copy(L.bits, reinterpret_cast<const char*>(a.ebits + (size_t)ti * EW), EW * 8u);
                    dma_copy(L.msg, reinterpret_cast<const char*>(a.emsg + (size_t)ti * MSG_CAP),
                             min(e_tot, (uint32_t)MSG_CAP) * 16u);
                }
            }
        }
        __syncthreads();  // staging copies, in-edge bitmap and gathered messages retired
        if constexpr (EDGES) {
            if (staged && threadIdx.x < 64) {  // sent edges before each bitmap word
                const uint32_t c = threadIdx.x < (uint32_t)EW ? (uint32_t)__popcll(L.bits[threadIdx.x]) : 0u;
                uint32_t incl = c;
#pragma unroll
                for (int o = 1; o < 32; o <<= 1) {
                    const uint32_t t = __shfl_up(incl, o, 64);
                    if (lane >= o) incl += t;
                }
                if (threadIdx.x <= (uint32_t)EW) L.bpre[threadIdx.x] = incl - c;
                if (threadIdx.x == (uint32_t)EW) L.bits[EW] = 0ull;
            }
            __syncthreads();
        }

        if constexpr (!EDGES) {
            // warm the XCD's L2 with the next tile's (s, w) while this tile folds: LDS-DMA
            // into a dead staging area (the senders are not read again this tile)
            if (GP_PREFETCH && TOPO == IMP3D && pf_tile != 0xFFFFFFFFu && pf_j1 > pf_j0) {
                const char* g = reinterpret_cast<const char*>(swc + pf_j0);
                const uint32_t nbytes = (pf_j1 - pf_j0) * 16u;
                char* sink = reinterpret_cast<char*>(L.src) + (threadIdx.x >> 6) * 1024u;
                for (uint32_t c = (threadIdx.x >> 6) * 1024u; c < nbytes; c += TPB * 16u) {
                    const uint32_t o = c + lane * 16u;
                    if (o < nbytes) __builtin_amdgcn_global_load_lds((gvoid_t*)(g + o), (lvoid_t*)sink, 16, 0, 0);
                }
            }
        }
        {
            // lattice coordinates of this thread's first node, advanced by TPB per node
            uint32_t cx = 0, cy = 0, cz = 0;
            if (TOPO != LINE) {
                const uint32_t j = T + threadIdx.x;
                cx = fastdiv(j, G.div_g2);
                const uint32_t rem = j - cx * G.g2;
                cy = fastdiv(rem, G.div_g);
                cz = rem - cy * G.g;
            }
#pragma unroll
            for (int k = 0; k < NPT; ++k) {
                const uint32_t jl = k * TPB + threadIdx.x;
                const uint32_t j = T + jl;
                const bool valid = j >= j0 && j < j1;
                uint32_t dir = DIR_NONE;
                if (TOPO != LINE && k > 0) {
                    cz += TPB;
                    if (cz >= G.g) {
                        const uint32_t q = fastdiv(cz, G.div_g);
                        cz -= q * G.g;
                        cy += q;
                        if (cy >= G.g) {
                            const uint32_t q2 = fastdiv(cy, G.div_g);
                            cy -= q2 * G.g;
                            cx += q2;
                        }
                    }
                }
                if (valid) {
                    const uint32_t jr = j - b_rows;
                    const uint32_t b = lds_byte(L.rows, jr);
                    const uint32_t mask = TOPO == LINE ? present_mask<TOPO>(j, G) : mask_xyz(cx, cy, cz, G.g - 1u);
                    const uint32_t deg = popc6(mask) + (TOPO == IMP3D ? 1u : 0u);
                    bool active = (b & B_ACTIVE) != 0;
                    const double2 sv = own[k];
                    const bool halve = active && deg > 0;
                    // canonical fold: own half, lattice slots in slot order, random edges by
                    // ascending sender; every message contributes the sender's half
                    double acc_s = halve ? sv.x * 0.5 : sv.x;
                    double acc_w = halve ? sv.y * 0.5 : sv.y;
                    auto fold = [&](const double2 mi) {
                        acc_s = acc_s + mi.x * 0.5;
                        acc_w = acc_w + mi.y * 0.5;
                    };
                    // lattice senders from the staged direction bytes (absent neighbours read
                    // a harmless in-range byte and are masked out)
                    uint32_t from = 0;
                    if (TOPO == LINE) {
                        from |= ((mask & 1u) && (lds_byte(L.rows, (mask & 1u) ? jr - 1 : jr) & DIR_MASK) == 1u) ? 1u : 0u;
                        from |= ((mask & 2u) && (lds_byte(L.rows, (mask & 2u) ? jr + 1 : jr) & DIR_MASK) == 0u) ? 2u : 0u;
                    } else {
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
                    if (GP_ABLATE & ABL_NO_LGATHER) from = 0;
                    // one gather per direction, all in flight together; a direction without a
                    // sender reads the zero sentinel swc[ext_hi] (adding +0.0 is exact)
                    constexpr uint32_t ND = TOPO == LINE ? 2 : 6;
                    double2 m[ND];
#pragma unroll
                    for (uint32_t d = 0; d < ND; ++d) m[d] = ld_sw(swc + ((from >> d) & 1u ? nbr<TOPO>(j, d, G) : a.ext_hi));
                    bool recv = from != 0;
#pragma unroll
                    for (uint32_t d = 0; d < ND; ++d) fold(m[d]);
                    if (TOPO == IMP3D && !(GP_ABLATE & ABL_NO_INLIST)) {
                        const uint32_t e_b = L.off[jl + o_off], e_e = L.off[jl + 1 + o_off];
                        if (GP_ABLATE & ABL_NO_RFOLD) {
                            recv = recv || L.bits[(e_b - e_lo) >> 6] != 0ull;
                        } else if (staged && !EDGES) {
                            // the node's used in-edges: its window of the tile bitmap, 32 bits at a
                            // time (funnel shift of two LDS words), walked set bit by set bit
                            // (ascending sender = canonical order); edge q's message is at slot q
                            const uint32_t* bw = reinterpret_cast<const uint32_t*>(L.bits);
                            const uint32_t qe = e_e - e_lo;
                            for (uint32_t q0 = e_b - e_lo; q0 < qe; q0 += 32u) {
                                uint32_t win = __builtin_amdgcn_alignbit(bw[(q0 >> 5) + 1], bw[q0 >> 5], q0 & 31u);
                                if (qe - q0 < 32u) win &= (1u << (qe - q0)) - 1u;
                                while (win) {
                                    const uint32_t q = q0 + (uint32_t)__builtin_ctz(win);
                                    win &= win - 1u;
                                    fold((GP_ABLATE & ABL_NO_RGATHER) ? make_double2(1.0, 1.0) : L.msg[q]);
                                    recv = true;
                                }
                            }
                        } else if (staged) {
                            // k_ps_edges stored the used in-edges' messages compactly in edge
                            // order, so this node's messages are the slots [prefix(e_b),
                            // prefix(e_e)), already in canonical (ascending sender) order
                            auto prefix = [&](uint32_t q) {
                                const uint32_t w = q >> 6;
                                return L.bpre[w] + (uint32_t)__popcll(L.bits[w] & ((1ull << (q & 63u)) - 1ull));
                            };
                            const uint32_t s0 = prefix(e_b - e_lo), s1 = prefix(e_e - e_lo);
                            for (uint32_t sl = s0; sl < s1; ++sl) {
                                double2 mi;
                                if (sl < (uint32_t)MSG_CAP) {
                                    mi = L.msg[sl];
                                } else {  // rare: more messages than the tile's slots -- find the edge
                                    uint32_t q = e_b - e_lo, k2 = sl - s0;
                                    for (;; ++q) {
                                        if ((L.bits[q >> 6] >> (q & 63u)) & 1ull) {
                                            if (k2 == 0) break;
                                            --k2;
                                        }
                                    }
                                    const uint32_t i = in_src[e_lo + q];
                                    mi = (REMOTE && i - a.lo >= a.nloc) ? a.rmsg[e_lo + q] : ld_sw(swc + i);
                                }
                                fold(mi);
                            }
                            recv = recv || s1 > s0;
                        } else {  // rare: tile in-degree above SLOTS (SRC_CAP for k_ps_edges, which skipped it)
                            for (uint32_t e = e_b; e < e_e; ++e) {
                                const uint32_t i = in_src[e];
                                bool sent;
                                double2 mi = make_double2(0.0, 0.0);
                                if (REMOTE && i - a.lo >= a.nloc) {
                                    sent = a.rtag[e] == r;
                                    if (sent) mi = a.rmsg[e];
                                } else {
                                    if (all_active) {
                                        const uint32_t di = popc6(present_mask<IMP3D>(i, G)) + 1u;
                                        sent = uniform(a.k0, a.k1, S_PUSHSUM, i, r, di) == di - 1u;
                                    } else {
                                        sent = (rbc[(i >> 6) - (a.lo >> 6)] >> (i & 63)) & 1ull;
                                    }
                                    if (sent) mi = ld_sw(swc + i);
                                }
                                if (sent) {
                                    fold(mi);
                                    recv = true;
                                }
                            }
                        }
                    }
                    uint32_t flags = b & (B_ACTIVE | B_CONV | (3u << CNT_SHIFT));
                    if (recv) {
                        if (!(GP_ABLATE & ABL_NO_RATIO) && !(b & B_CONV)) {
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
                            active = true;
                        }
                    }
                    if (active && deg > 0)
                        dir = (GP_ABLATE & ABL_NO_NEXTDIR)
                                  ? (j % 7u) % (deg)
                                  : slot_to_dir_fast(mask, uniform(a.k0, a.k1, S_PUSHSUM, j, r + 1, deg));
                    if (LTAG && dir == DIR_RANDOM)
                        a.ltn[a.lpos[j]] = r + 1;  // tag the edge for its receiver's next in-edge pass
                    reinterpret_cast<uint8_t*>(L.out)[jl] = (uint8_t)(flags | dir);
                    st_stream(swn + j, make_double2(acc_s, acc_w));
                }
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
    }
    // block reduction of alerts / newly active
    uint32_t x = alerts, y = newly;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        x += __shfl_xor(x, o, 64);
        y += __shfl_xor(y, o, 64);
    }
    if (lane == 0) {
        L.red[0][threadIdx.x >> 6] = x;
        L.red[1][threadIdx.x >> 6] = y;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        x = 0;
        y = 0;
        for (int w = 0; w < TPB / 64; ++w) {
            x += L.red[0][w];
            y += L.red[1][w];
        }
        if (x) atomicAdd(&ctl->round_alerts, (unsigned long long)x);
        if (y) atomicAdd(&ctl->round_active, (unsigned long long)y);
    }
}

// ---------------------------------------------------------------- push-sum, in-edge pass (Imp3D)
// Runs before k_ps_tile<IMP3D, *, true> in the same round.  For every tile
// (same tiles as the round kernel) and every in-edge of it, in receiver order:
// did the sender use its random edge this round (its Philox draw; the ballot
// bitmap during activation; the exchange tag for senders on other ranks)?  The
// answers go to ebits (one bit per edge, EW words per tile), the senders' (s, w)
// are gathered and stored compactly in edge order (emsg, MSG_CAP slots per
// tile, count in etot).  No block-wide phase waits on another tile's data, so
// the Philox chains and the random gathers of many tiles overlap freely.
template <bool REMOTE>
__global__ __launch_bounds__(TPB) void k_ps_edges(RoundArgs a, uint32_t r) {
    __shared__ uint32_t wcnt[EW];
    Ctl* ctl = a.ctl;
    if (ld_agent(&ctl->done)) return;
    const bool all_active = ld_agent(&ctl->all_active) != 0;
    const double2* __restrict__ swc = a.swc;
    const uint64_t* __restrict__ rbc = a.rbc;
    const Geom G = a.G;
    constexpr int FU = SRC_CAP / TPB;
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    for (uint32_t ti = blockIdx.x; ti < a.ntiles; ti += gridDim.x) {
        const uint32_t T = (a.lo / TILE + ti) * TILE;
        const uint32_t j0 = max(a.lo, T);
        const uint32_t j1 = min(a.lo + a.nloc, T + TILE);
        const uint32_t e_lo = a.in_off[j0], e_hi = a.in_off[j1];
        const uint32_t cnt = e_hi - e_lo;
        if (cnt > (uint32_t)SRC_CAP) continue;  // the round kernel handles such a tile by itself
        uint32_t isrc[FU];
#pragma unroll
        for (int m = 0; m < FU; ++m) {
            const uint32_t q = threadIdx.x + m * TPB;
            isrc[m] = q < cnt ? a.in_src[e_lo + q] : 0u;
        }
        bool snt[FU];
#pragma unroll
        for (int m = 0; m < FU; ++m) {
            const uint32_t q = threadIdx.x + m * TPB;
            const uint32_t i = isrc[m];
            bool sent = false;
            if (q < cnt) {
                if (REMOTE && i - a.lo >= a.nloc) {
                    sent = a.rtag[e_lo + q] == r;
                } else if (all_active) {
                    const uint32_t di = popc6(present_mask<IMP3D>(i, G)) + 1u;
                    sent = uniform(a.k0, a.k1, S_PUSHSUM, i, r, di) == di - 1u;
                } else {
                    sent = (rbc[(i >> 6) - (a.lo >> 6)] >> (i & 63)) & 1ull;
                }
            }
            snt[m] = sent;
        }
        double2 v[FU];
#pragma unroll
        for (int m = 0; m < FU; ++m) {
            v[m] = make_double2(0.0, 0.0);
            if (snt[m]) {
                const uint32_t q = threadIdx.x + m * TPB;
                v[m] = (REMOTE && isrc[m] - a.lo >= a.nloc) ? a.rmsg[e_lo + q] : ld_sw(swc + isrc[m]);
            }
        }
        // edge q = m * TPB + wv * 64 + lane sits in bitmap word m * 4 + wv
        unsigned long long bal[FU];
#pragma unroll
        for (int m = 0; m < FU; ++m) {
            bal[m] = __ballot(snt[m]);
            if (lane == 0) {
                a.ebits[(size_t)ti * EW + m * (TPB / 64) + wv] = bal[m];
                wcnt[m * (TPB / 64) + wv] = (uint32_t)__popcll(bal[m]);
            }
        }
        __syncthreads();
        const uint32_t c = lane < (uint32_t)EW ? wcnt[lane] : 0u;
        uint32_t incl = c;
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) {
            const uint32_t t = __shfl_up(incl, o, 64);
            if (lane >= (uint32_t)o) incl += t;
        }
        const uint32_t excl = incl - c;
        const uint32_t total = __shfl(incl, EW - 1, 64);
#pragma unroll
        for (int m = 0; m < FU; ++m) {
            const uint32_t slot = __shfl(excl, m * (TPB / 64) + wv, 64) +
                                  __builtin_amdgcn_mbcnt_hi((uint32_t)(bal[m] >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)bal[m], 0u));
            if (snt[m] && slot < (uint32_t)MSG_CAP) a.emsg[(size_t)ti * MSG_CAP + slot] = v[m];
        }
        if (threadIdx.x == 0) a.etot[ti] = total;
        __syncthreads();
    }
}

// ---------------------------------------------------------------- push-sum, compacted gathers
// Same round as k_ps_tile, different schedule: after staging, every thread
// decides its nodes' lattice senders (from the staged bytes) and its share of
// the tile's in-edges (Philox / bitmap / tag); a block scan assigns every
// message of the tile -- lattice and random alike -- a slot, the source ids go
// into those slots (the staging area is dead by then), and the whole tile's
// messages are gathered as one dense burst (MI2 loads per thread instead of 6
// mostly-masked loads per node), overlapped with the next-round Philox draws.
// The fold then reads every message from LDS, in canonical order.
template <int TOPO, bool REMOTE>
__global__ __launch_bounds__(TPB, GP_MINB2) void k_ps_tile2(RoundArgs a, uint32_t r) {
    __shared__ Tile2Lds L;
    Ctl* ctl = a.ctl;
    if (ld_agent(&ctl->done)) return;
    const bool all_active = ld_agent(&ctl->all_active) != 0;
    const double2* __restrict__ swc = a.swc;
    double2* __restrict__ swn = a.swn;
    const uint64_t* __restrict__ rbc = a.rbc;
    const uint32_t* __restrict__ in_src = a.in_src;
    const Geom G = a.G;
    const uint32_t H = TOPO == LINE ? 1u : G.g;
    constexpr uint32_t ND = TOPO == LINE ? 2 : 6;
    constexpr int FU = SRC_CAP / TPB;
    uint32_t alerts = 0, newly = 0;
    const int lane = threadIdx.x & 63;
    uint32_t* const list = reinterpret_cast<uint32_t*>(L.u.msg);

    for (TileWalk tw(a); tw.t < tw.end; tw.t += tw.step) {
        uint32_t ti;
        if (!tw.tile(ti)) continue;
        const uint32_t T = (a.lo / TILE + ti) * TILE;
        const uint32_t j0 = max(a.lo, T);
        const uint32_t j1 = min(a.lo + a.nloc, T + TILE);
        uint32_t e_lo = 0, e_hi = 0;
        if (TOPO == IMP3D) {
            e_lo = a.in_off[j0];
            e_hi = a.in_off[j1];
        }
        const uint32_t b_rows = stage_bytes(L.u.s.rows, a.nbc, (int64_t)j0 - H, (int64_t)j1 + H, a.ext_lo, a.ext_hi);
        uint32_t b_xm = 0, b_xp = 0;
        if (TOPO != LINE) {
            b_xm = stage_bytes(L.u.s.xm, a.nbc, (int64_t)j0 - G.g2, (int64_t)j1 - G.g2, a.ext_lo, a.ext_hi);
            b_xp = stage_bytes(L.u.s.xp, a.nbc, (int64_t)j0 + G.g2, (int64_t)j1 + G.g2, a.ext_lo, a.ext_hi);
        }
        const uint32_t cnt = e_hi - e_lo;
        const bool staged = TOPO == IMP3D && cnt <= (uint32_t)SRC_CAP;
        if (TOPO == IMP3D) {
            for (uint32_t q = j0 - T + threadIdx.x; q <= j1 - T; q += TPB) L.off[q] = a.in_off[T + q];
            if (staged)
                for (uint32_t q = threadIdx.x; q < cnt; q += TPB) L.u.s.src[q] = in_src[e_lo + q];
        }
        __syncthreads();
        // ---- 1a. decisions: lattice senders per node, random-edge senders per staged edge
        uint32_t frp = 0, bown = 0, msk = 0;  // per node k, byte k: from-bits, own byte, present mask
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
            const uint32_t jl = k * TPB + threadIdx.x;
            const uint32_t j = T + jl;
            const bool valid = j >= j0 && j < j1;
            uint32_t from = 0, mask = 0, b = 0;
            if (valid) {
                b = lds_byte(L.u.s.rows, j - b_rows);
                mask = present_mask<TOPO>(j, G);
                if (TOPO == LINE) {
                    if ((mask & 1u) && (lds_byte(L.u.s.rows, j - 1 - b_rows) & DIR_MASK) == 1u) from |= 1u;
                    if ((mask & 2u) && (lds_byte(L.u.s.rows, j + 1 - b_rows) & DIR_MASK) == 0u) from |= 2u;
                } else {
                    if ((mask & 1u) && (lds_byte(L.u.s.xm, j - G.g2 - b_xm) & DIR_MASK) == 1u) from |= 1u;
                    if ((mask & 2u) && (lds_byte(L.u.s.xp, j + G.g2 - b_xp) & DIR_MASK) == 0u) from |= 2u;
                    if ((mask & 4u) && (lds_byte(L.u.s.rows, j + G.g - b_rows) & DIR_MASK) == 3u) from |= 4u;
                    if ((mask & 8u) && (lds_byte(L.u.s.rows, j - G.g - b_rows) & DIR_MASK) == 2u) from |= 8u;
                    if ((mask & 16u) && (lds_byte(L.u.s.rows, j + 1 - b_rows) & DIR_MASK) == 5u) from |= 16u;
                    if ((mask & 32u) && (lds_byte(L.u.s.rows, j - 1 - b_rows) & DIR_MASK) == 4u) from |= 32u;
                }
            }
            frp |= from << (8 * k);
            bown |= b << (8 * k);
            msk |= mask << (8 * k);
        }
        uint32_t isrc[FU];
        uint32_t sbits = 0;  // bit m: staged edge tid + m * TPB was used by its sender
        if (staged) {
#pragma unroll
            for (int m = 0; m < FU; ++m) {
                const uint32_t q = threadIdx.x + m * TPB;
                isrc[m] = q < cnt ? L.u.s.src[q] : a.lo;
            }
#pragma unroll
            for (int m = 0; m < FU; ++m) {
                const uint32_t q = threadIdx.x + m * TPB;
                const uint32_t i = isrc[m];
                bool sent = false;
                if (q < cnt) {
                    if (REMOTE && i - a.lo >= a.nloc) {
                        sent = a.rtag[e_lo + q] == r;
                    } else if (all_active) {
                        const uint32_t di = popc6(present_mask<IMP3D>(i, G)) + 1u;
                        sent = uniform(a.k0, a.k1, S_PUSHSUM, i, r, di) == di - 1u;
                    } else {
                        sent = (rbc[(i >> 6) - (a.lo >> 6)] >> (i & 63)) & 1ull;
                    }
                }
                sbits |= sent ? (1u << m) : 0u;
            }
        }
        uint32_t mine = (uint32_t)__popc(sbits);
#pragma unroll
        for (int k = 0; k < NPT; ++k) mine += popc6((frp >> (8 * k)) & 0xFFu);
        uint32_t total;
        const uint32_t tbase = block_excl_scan(mine, L.scan, total);  // barriers: the staging area is dead now
        // ---- 1b. slots: this thread's messages get [tbase, tbase + mine); sources into the slots
        uint32_t slot = tbase;
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
            const uint32_t j = T + k * TPB + threadIdx.x;
            const uint32_t f = (frp >> (8 * k)) & 0xFFu;
#pragma unroll
            for (uint32_t d = 0; d < ND; ++d) {
                if ((f >> d) & 1u) {
                    if (slot < (uint32_t)MCAP2) list[4 * slot] = nbr<TOPO>(j, d, G);
                    ++slot;
                }
            }
        }
        if (staged) {
#pragma unroll
            for (int m = 0; m < FU; ++m) {
                const uint32_t q = threadIdx.x + m * TPB;
                if (q < cnt) {
                    uint16_t p = POS_NONE;
                    if ((sbits >> m) & 1u) {
                        if (slot < (uint32_t)MCAP2) {
                            list[4 * slot] = (REMOTE && isrc[m] - a.lo >= a.nloc) ? 0xFFFFFFFFu - q : isrc[m];
                            p = (uint16_t)slot;
                        } else {
                            p = POS_GLOBAL;
                        }
                        ++slot;
                    }
                    L.pos[q] = p;
                }
            }
        }
        __syncthreads();
        // ---- 2. one dense gather burst for the tile's messages, overlapped with
        //         the next-round direction draws of this thread's nodes
        const uint32_t M = min(total, (uint32_t)MCAP2);
        double2 own[NPT];  // own (s, w): loaded with the burst, used by the fold
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
            const uint32_t j = T + k * TPB + threadIdx.x;
            own[k] = (j >= j0 && j < j1) ? swc[j] : make_double2(0.0, 1.0);
        }
        double2 v[MI2];
#pragma unroll
        for (int it = 0; it < MI2; ++it) {
            const uint32_t m = it * TPB + threadIdx.x;
            v[it] = make_double2(0.0, 0.0);
            if (m < M) {
                const uint32_t src = list[4 * m];
                v[it] = (REMOTE && src >= REMOTE_TAG) ? a.rmsg[e_lo + (0xFFFFFFFFu - src)] : ld_sw(swc + src);
            }
        }
        uint32_t dirs = 0;
        if (!(TOPO == IMP3D && !staged)) {
#pragma unroll
            for (int k = 0; k < NPT; ++k) {
                const uint32_t jl = k * TPB + threadIdx.x;
                const uint32_t j = T + jl;
                const bool valid = j >= j0 && j < j1;
                bool recv = ((frp >> (8 * k)) & 0xFFu) != 0;
                if (TOPO == IMP3D && valid) {
                    const uint32_t e_b = L.off[jl], e_e = L.off[jl + 1];
                    for (uint32_t e = e_b; e < e_e && !recv; ++e) recv = L.pos[e - e_lo] != POS_NONE;
                }
                const uint32_t b = (bown >> (8 * k)) & 0xFFu;
                const uint32_t mask = (msk >> (8 * k)) & 0xFFu;
                const uint32_t deg = popc6(mask) + (TOPO == IMP3D ? 1u : 0u);
                const bool active = valid && ((b & B_ACTIVE) || recv);
                uint32_t dir = DIR_NONE;
                if (active && deg > 0) dir = slot_to_dir(mask, uniform(a.k0, a.k1, S_PUSHSUM, j, r + 1, deg));
                dirs |= dir << (8 * k);

            }
        }
#pragma unroll
        for (int it = 0; it < MI2; ++it) {
            const uint32_t m = it * TPB + threadIdx.x;
            if (m < M) L.u.msg[m] = v[it];
        }
        __syncthreads();
        // ---- 3. fold in canonical order from LDS, ratio test, outputs
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
            const uint32_t jl = k * TPB + threadIdx.x;
            const uint32_t j = T + jl;
            const bool valid = j >= j0 && j < j1;
            uint32_t dir = DIR_NONE;
            if (valid) {
                const uint32_t b = (bown >> (8 * k)) & 0xFFu;
                const uint32_t mask = (msk >> (8 * k)) & 0xFFu;
                const uint32_t deg = popc6(mask) + (TOPO == IMP3D ? 1u : 0u);
                bool active = (b & B_ACTIVE) != 0;
                const double2 sv = own[k];
                const bool halve = active && deg > 0;
                double acc_s = halve ? sv.x * 0.5 : sv.x;
                double acc_w = halve ? sv.y * 0.5 : sv.y;
                const uint32_t f = (frp >> (8 * k)) & 0xFFu;
                uint32_t mm = tbase;  // this node's lattice slots follow those of the thread's earlier nodes
#pragma unroll
                for (int k2 = 0; k2 < k; ++k2) mm += popc6((frp >> (8 * k2)) & 0xFFu);
#pragma unroll
                for (uint32_t d = 0; d < ND; ++d) {
                    if ((f >> d) & 1u) {
                        const double2 mv = mm < (uint32_t)MCAP2 ? L.u.msg[mm] : ld_sw(swc + nbr<TOPO>(j, d, G));
                        acc_s = acc_s + mv.x * 0.5;
                        acc_w = acc_w + mv.y * 0.5;
                        ++mm;
                    }
                }
                bool recv = f != 0;
                if (TOPO == IMP3D) {
                    const uint32_t e_b = L.off[jl], e_e = L.off[jl + 1];
                    for (uint32_t e = e_b; e < e_e; ++e) {
                        bool sent = false;
                        double2 mi = make_double2(0.0, 0.0);
                        if (staged) {
                            const uint16_t p = L.pos[e - e_lo];
                            sent = p != POS_NONE;
                            if (p < (uint16_t)MCAP2) {
                                mi = L.u.msg[p];
                            } else if (p == POS_GLOBAL) {
                                const uint32_t i = in_src[e];
                                mi = (REMOTE && i - a.lo >= a.nloc) ? a.rmsg[e] : ld_sw(swc + i);
                            }
                        } else {  // rare: tile in-degree above SRC_CAP
                            const uint32_t i = in_src[e];
                            if (REMOTE && i - a.lo >= a.nloc) {
                                sent = a.rtag[e] == r;
                                if (sent) mi = a.rmsg[e];
                            } else {
                                if (all_active) {
                                    const uint32_t di = popc6(present_mask<IMP3D>(i, G)) + 1u;
                                    sent = uniform(a.k0, a.k1, S_PUSHSUM, i, r, di) == di - 1u;
                                } else {
                                    sent = (rbc[(i >> 6) - (a.lo >> 6)] >> (i & 63)) & 1ull;
                                }
                                if (sent) mi = ld_sw(swc + i);
                            }
                        }
                        if (sent) {
                            acc_s = acc_s + mi.x * 0.5;
                            acc_w = acc_w + mi.y * 0.5;
                            recv = true;
                        }
                    }
                }
                uint32_t flags = b & (B_ACTIVE | B_CONV | (3u << CNT_SHIFT));
                if (recv) {
                    if (!(b & B_CONV)) {
                        const double r_old = sv.x / sv.y;
                        const double r_new = acc_s / acc_w;
                        uint32_t cn = (b >> CNT_SHIFT) & 3u;
                        cn = fabs(r_new - r_old) > 1e-10 ? 0u : cn + 1u;
                        flags = (flags & ~(3u << CNT_SHIFT)) | (cn << CNT_SHIFT);
                        if (cn == 3) {
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
                if (TOPO == IMP3D && !staged) {
                    if (active && deg > 0) dir = slot_to_dir(mask, uniform(a.k0, a.k1, S_PUSHSUM, j, r + 1, deg));
                } else {
                    dir = (dirs >> (8 * k)) & 0xFFu;
                }
                reinterpret_cast<uint8_t*>(L.out)[jl] = (uint8_t)(flags | dir);
                swn[j] = make_double2(acc_s, acc_w);
            }
            if (TOPO == IMP3D && !all_active) {
                const unsigned long long bits = __ballot(valid && dir == DIR_RANDOM);
                if (lane == 0) {
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
    uint32_t x = alerts, y = newly;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        x += __shfl_xor(x, o, 64);
        y += __shfl_xor(y, o, 64);
    }
    if (lane == 0) {
        L.red[0][threadIdx.x >> 6] = x;
        L.red[1][threadIdx.x >> 6] = y;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        x = 0;
        y = 0;
        for (int w = 0; w < TPB / 64; ++w) {
            x += L.red[0][w];
            y += L.red[1][w];
        }
        if (x) atomicAdd(&ctl->round_alerts, (unsigned long long)x);
        if (y) atomicAdd(&ctl->round_active, (unsigned long long)y);
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
            e_lo = a.in_off[j0];
            e_hi = a.in_off[j1];
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
                unsigned long long wv[FU];
#pragma unroll
                for (int m = 0; m < FU; ++m) {
                    const uint32_t q = threadIdx.x + m * TPB;
                    const uint32_t li = isrc[m] - a.lo;
                    wv[m] = q >= cnt ? 0ull
                            : (!REMOTE || li < a.nloc) ? a.rbc[(isrc[m] >> 6) - (a.lo >> 6)]
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

uint32_t round_tiles(uint32_t P) { return (P + TILE - 1) / TILE; }
// 64-bit words the ballot stores of one round touch (whole tiles) plus slack.
uint32_t rbits_words_for(uint32_t lo, uint32_t nloc) {
    return ((lo + nloc + TILE - 1) / TILE - lo / TILE) * (TILE / 64) + 16u;
}

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
    a.rtag = S.rtag;
    a.rmsg = S.rmsg;
    a.ltc = S.ltag[cur];
    a.ltn = S.ltag[cur ^ 1];
    a.lpos = S.lpos;
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
    a.ntiles = (S.lo + S.nloc + TILE - 1) / TILE - S.lo / TILE;
    a.walk = S.tile_walk;
    a.stage_cap = S.tile_stage_cap;
    a.ebits = S.ebits;
    a.etot = S.etot;
    a.emsg = S.emsg;
    a.wx = S.tile_wx;
    a.xs_len = 0;
    if (S.G.g2) {
        const uint32_t planes = S.nloc / S.G.g2, xs = S.col_xsegs ? S.col_xsegs : 1u;
        a.xs_len = (planes + xs - 1) / xs;
    }
    return a;
}

hipError_t launch_round_tile(const DevState& S, uint32_t round, int grid, hipStream_t st) {
    const RoundArgs a = make_round_args(S, round);
    const dim3 g(grid), b(TPB);
    const bool remote = S.rtag != nullptr;  // Imp3D slabs of a multi-rank run
    if (S.alg == PUSHSUM && S.kernel == KERNEL_XTILE && S.topo != LINE)
        return launch_round_xtile(a, S.topo, remote, round, grid, st);
    if (S.alg == PUSHSUM && S.kernel == KERNEL_TILE2) {
        switch (S.topo) {
            case LINE: hipLaunchKernelGGL((k_ps_tile2<LINE, false>), g, b, 0, st, a, round); break;
            case GRID3D: hipLaunchKernelGGL((k_ps_tile2<GRID3D, false>), g, b, 0, st, a, round); break;
            default:
                if (remote) hipLaunchKernelGGL((k_ps_tile2<IMP3D, true>), g, b, 0, st, a, round);
                else hipLaunchKernelGGL((k_ps_tile2<IMP3D, false>), g, b, 0, st, a, round);
                break;
        }
    } else if (S.alg == PUSHSUM) {
        switch (S.topo) {
            case LINE: hipLaunchKernelGGL((k_ps_tile<LINE, false, false>), g, b, 0, st, a, round); break;
            case GRID3D: hipLaunchKernelGGL((k_ps_tile<GRID3D, false, false>), g, b, 0, st, a, round); break;
            default:
                if (S.emsg) {  // in-edge pass first (same stream)
                    if (remote) {
                        hipLaunchKernelGGL((k_ps_edges<true>), g, b, 0, st, a, round);
                        hipLaunchKernelGGL((k_ps_tile<IMP3D, true, true>), g, b, 0, st, a, round);
                    } else {
                        hipLaunchKernelGGL((k_ps_edges<false>), g, b, 0, st, a, round);
                        hipLaunchKernelGGL((k_ps_tile<IMP3D, false, true>), g, b, 0, st, a, round);
                    }
                } else if (remote) {
                    hipLaunchKernelGGL((k_ps_tile<IMP3D, true, false>), g, b, 0, st, a, round);
                } else if (S.ltag[0]) {
                    hipLaunchKernelGGL((k_ps_tile<IMP3D, false, false, true>), g, b, 0, st, a, round);
                } else {
                    hipLaunchKernelGGL((k_ps_tile<IMP3D, false, false>), g, b, 0, st, a, round);
                }
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

hipError_t launch_rbits_init(const DevState& S, int grid, hipStream_t st) {
    hipLaunchKernelGGL(k_rbits_init, dim3(grid), dim3(TPB), 0, st, S.nb[0] - S.base, S.rbits[0], S.lo, S.nloc,
                       S.rbits_words);
    return hipGetLastError();
}

}  // namespace gp
