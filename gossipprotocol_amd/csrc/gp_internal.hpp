// gp_internal.hpp -- device-memory layout and kernel launch wrappers shared by
// the translation units of libgossip_hip.so.  Not part of the C-ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "gp_device.hpp"

namespace gp {

constexpr int HIST = 4096;            // per-round alert ring (host syncs at least every HIST rounds)
constexpr uint32_t INJ_CHUNK = 65536; // injector live-list chunk (ids); 2048 bitmap words
constexpr int BULK_THREADS = 256;

// The immediate of `s_waitcnt vmcnt(n)` with the other counters left alone (gfx9 encoding:
// vmcnt bits 3:0 and 15:14, expcnt 6:4 = 7, lgkmcnt 11:8 = 15), for __builtin_amdgcn_s_waitcnt.
// vmcnt retires in issue order, so an explicit count can wait for an older operation without
// waiting for the n newest; the compiler takes such a wait into its own accounting.
constexpr int vmcnt_enc(int n) { return 0x0F70 | (n & 15) | ((n >> 4) << 14); }

// A load of data the running kernel does not write (in-lists, the walk's tile list, counts an
// earlier kernel produced) through the constant address space: at a wave-uniform address it
// becomes a scalar load, counted by lgkmcnt, so waiting for it does not also wait for the
// wave's earlier vector stores (vmcnt retires in issue order).  The scalar cache is invalidated
// at every kernel start.
template <typename T>
__device__ __forceinline__ T ld_const(const T* p) {
    return *(const __attribute__((address_space(4))) T*)(p);
}

// A pointer known to address global memory.  Pointers a kernel reads from LDS or from a
// per-lane-indexed table are generic to the compiler, which then emits flat instructions:
// those count in lgkmcnt as well as vmcnt, so every later LDS wait also waited for them.
template <typename T>
__device__ __forceinline__ __attribute__((address_space(1))) T* gptr(T* p) {
    return (__attribute__((address_space(1))) T*)(p);
}
typedef double gp_d2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void st_global(double2* p, double2 v) {
    *gptr(reinterpret_cast<gp_d2v*>(p)) = gp_d2v{v.x, v.y};
}
__device__ __forceinline__ double2 ld_global(const double2* p) {
    const gp_d2v t = *gptr(reinterpret_cast<gp_d2v*>(const_cast<double2*>(p)));
    return make_double2(t.x, t.y);
}
constexpr int FIN_THREADS = 1024;
constexpr int RREG_MAX = 8;           // round kernel launches per round, at most (DevState::rregions)

// Device-resident control block.  Written by the single-block finalize kernel
// between bulk rounds; bulk kernels only read it (plus atomics on the
// round_* accumulators, which nobody reads inside the same kernel).
struct Ctl {
    unsigned long long alerts_total;  // cumulative alerts through the last finalized round
    unsigned long long round_alerts;  // accumulated by the bulk kernel of the current round
    unsigned long long active_total;  // push-sum: nodes ever activated (monotone)
    unsigned long long round_active;  // accumulated newly-active count of the current round
    unsigned long long live;          // injector |L| (Program.fs:142-158)
    long long inj_target;             // node the injector delivers to this round, -1 none
    unsigned int done;                // cumulative alerts reached T (Program.fs:53)
    unsigned int all_active;          // every node active at round start (push-sum)
    unsigned long long xchg[4];       // multi-rank: {alerts, newly active, injector pick converged, 0}, summed over ranks
    long long inj_pick;               // multi-rank: the injector's pick for the next round (-1 none)
    unsigned int overflow;            // multi-rank: a random-edge exchange buffer overflowed (run is invalid)
    unsigned int blocks_done;         // fused finalize: blocks of the current round kernel that have finished
    unsigned int tiny;                // push-sum: some (s, w) fell below 2^-1020 (the FMA fold's exactness bound)
    unsigned int pad_;
    // fused round close, sharded: blocks b with b % 8 == k count into shard k
    // (one 256-byte line each, so the shards' atomics do not queue on one line)
    struct alignas(256) Shard {
        unsigned long long alerts, active;
        unsigned int done, pad_[3];
    } shard[8];
    unsigned long long hist[HIST];    // alerts of round r at hist[r % HIST]
};

// Scheduler bookkeeping of round `round_done` from its global counts a (alerts)
// and na (newly active) (Program.fs:51-56); returns 1 when the run is over.
// One thread (the finalize kernel's, or the last block of a round kernel that
// closes its own round).
__device__ inline int close_round_ctl(Ctl* ctl, uint32_t P, uint32_t T, uint32_t round_done, unsigned long long a,
                                      unsigned long long na) {
    const unsigned long long tot =
        __hip_atomic_load(&ctl->alerts_total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + a;
    __hip_atomic_store(&ctl->alerts_total, tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ctl->hist[round_done % HIST] = a;
    const unsigned long long act =
        __hip_atomic_load(&ctl->active_total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + na;
    __hip_atomic_store(&ctl->active_total, act, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (act >= P) __hip_atomic_store(&ctl->all_active, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tot >= T) {
        __hip_atomic_store(&ctl->done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 1;
    }
    return 0;
}

// Round kernels that close their own round (single rank, no injector): every
// block counts itself out after its alert atomics; the last one moves the
// round's counts into the bookkeeping (replaces a k_finalize launch).  Thread 0
// of each block, after the block's round_alerts / round_active atomics.
__device__ inline void block_done_close(Ctl* ctl, uint32_t P, uint32_t T, uint32_t round) {
    // No fences (a release fence at agent scope writes back the XCD's L2): the
    // block's round_* updates are atomics performed at the device coherence point,
    // and the caller waits for their results before arriving here (see k_ps_tile),
    // so they are complete before this arrival; the last block reads them with
    // atomics too.  Everything else it writes reaches the next round's kernel
    // through the kernel boundary.
    const unsigned int prev = __hip_atomic_fetch_add(&ctl->blocks_done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev != gridDim.x - 1) return;
    __hip_atomic_store(&ctl->blocks_done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long a = __hip_atomic_exchange(&ctl->round_alerts, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long na = __hip_atomic_exchange(&ctl->round_active, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    close_round_ctl(ctl, P, T, round, a, na);
}

// block_done_close with the arrivals spread over 8 shards (block b counts into
// shard b % 8 -- on MI355X the blocks of one XCD): one word takes ~88 returning
// atomics per microsecond, so a grid of 16384 blocks queued on a single word
// holds its blocks' CU slots for a large part of a round.  The last block of a
// shard forwards the shard's sums and arrives at the global counter; the last
// of those closes the round.  Thread 0, with the block's counts x (alerts) and
// y (newly active).
__device__ inline void block_done_close_sharded(Ctl* ctl, uint32_t P, uint32_t T, uint32_t round, uint32_t x,
                                                uint32_t y) {
    const uint32_t G = gridDim.x, k = blockIdx.x & 7u;
    Ctl::Shard* sh = &ctl->shard[k];
    unsigned long long d = 0;
    if (x) d += __hip_atomic_fetch_add(&sh->alerts, (unsigned long long)x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (y) d += __hip_atomic_fetch_add(&sh->active, (unsigned long long)y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("" ::"v"(d));
    __builtin_amdgcn_s_waitcnt(0);
    const uint32_t members = (G - k + 7u) / 8u;  // blocks with b % 8 == k
    const unsigned int prev = __hip_atomic_fetch_add(&sh->done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev != members - 1) return;
    __hip_atomic_store(&sh->done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long a = __hip_atomic_exchange(&sh->alerts, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long na = __hip_atomic_exchange(&sh->active, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    d = 0;
    if (a) d += __hip_atomic_fetch_add(&ctl->round_alerts, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (na) d += __hip_atomic_fetch_add(&ctl->round_active, na, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("" ::"v"(d));
    __builtin_amdgcn_s_waitcnt(0);
    const uint32_t shards = G < 8u ? G : 8u;
    const unsigned int p2 = __hip_atomic_fetch_add(&ctl->blocks_done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (p2 != shards - 1) return;
    __hip_atomic_store(&ctl->blocks_done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long ga = __hip_atomic_exchange(&ctl->round_alerts, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long gna = __hip_atomic_exchange(&ctl->round_active, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    close_round_ctl(ctl, P, T, round, ga, gna);
}

// One more random-edge rumour for local node t next round (gossip column kernel):
// rq holds a word per node, or (rq8) a byte per node packed four to a word -- a
// node's count in one round is at most its random in-degree (Poisson(1): never
// near 256).
__device__ inline void rq_add(uint32_t* rq, uint32_t rq8, uint32_t t) {
    if (rq8) atomicAdd(&rq[t >> 2], 1u << (8u * (t & 3u)));
    else atomicAdd(&rq[t], 1u);
}

// Imp3D push-sum across ranks (gp_xchg.hpp, sender-ordered lists): one header word
// of a received list, 64 entries.
struct XHdr {
    unsigned long long mask;   // bit: the entry's sender used its random edge this round
    uint32_t base;             // vals index of the word's first used entry (this rank's vals region)
    uint32_t pad;
};
static_assert(sizeof(XHdr) == 16, "header words move as 16-byte loads");

// KERNEL_BLOCK (gp_block.hip): the lattice cut into nbx * nby * nbz boxes, one per workgroup.
struct BlockPlan {
    uint32_t nbx, nby, nbz;  // boxes per axis
    uint32_t vmax, fmax;     // largest box (nodes) and largest face
    uint32_t lds;            // dynamic LDS bytes per workgroup
};

// Node state in HBM (structure of arrays, single GPU / one slab).
struct DevState {
    Geom G;
    int topo, alg;
    uint32_t k0, k1;    // Philox key = seed
    uint32_t seed_node;
    Ctl* ctl;
    // push-sum: (s, w) interleaved, double buffered; node byte double buffered
    double2* sw[2];
    uint8_t* nb[2];
    // gossip: rumour counters (in place), direction byte double buffered (nb)
    int32_t* c;
    // gossip, Imp3D, column kernel: random-edge rumours each local node receives, by
    // round parity, indexed from lo -- counted a round ahead by the senders (atomics
    // from local senders in k_gossip_col, the exchange's counts from remote ones in
    // k_unpack) and read (then zeroed) by the receiver
    uint32_t* rq[2];
    uint32_t rq8;         // rq holds one byte per node (four per word) instead of one word
    // gossip column kernel across ranks (gp_xchg.hpp, bitmaps): per local sender its
    // random edge's local target (t - lo) or 0x80000000 | its bit in sbits, the send
    // bitmap of the round being prepared
    uint32_t* rtg;
    uint32_t* sbits;
    // Imp3D: bit i of rbits[b] = node i sends on its random edge in the round
    // of buffer b (ballot-packed by the round kernel)
    uint64_t* rbits[2];
    uint32_t rbits_words;
    // Imp3D: random edge and receiver-sorted in-lists (CSR)
    uint32_t* rnd;
    uint32_t* in_off;  // P+1
    uint32_t* in_src;  // P
    uint32_t* in_srcd; // push-sum tile kernel: in_src with deg - 4 in bits 30-31 (P <= 2^30), else null
    uint8_t* ind4;     // push-sum tile kernel: in-degree of every node of the slab's tiles, a nibble each
                       // (min(deg, 15); 0 outside the slab), byte (j - lo / TILE * TILE) / 2, low nibble first
    // gossip injector
    uint32_t* live_bits;   // ceil(T / INJ_CHUNK) * 2048 words, bit = id still listed
    uint32_t* chunk_live;  // live ids per chunk
    uint32_t nchunks;
    // full topology scratch
    int32_t* inc;          // gossip deliveries per node
    // push-sum, one rank: two-level LDS binning of the round's messages (gp_fullbin.hip)
    uint32_t fb_s1, fb_nb1, fb_nb2, fb_cap1, fb_cap2;
    uint32_t fb_fused;  // one rank: the fold bins the next round's messages (no send pass after round 0)
    uint32_t *fb_cnt1, *fb_cnt2;
    uint32_t *fb_hdr1, *fb_hdr2;  // sender ids
    double2 *fb_pay1, *fb_pay2;
    // slab of this rank (single GPU: lo = 0, nloc = P, base = 0): node ids
    // [lo, lo + nloc) are owned; per-node arrays (sw, nb) start at id `base`
    // (= lo - halo); c, in_off and rbits are indexed from lo
    uint32_t lo, nloc, base;
    uint32_t ext_lo, ext_hi;  // ids the node arrays hold: [lo - halo, lo + nloc + halo) within [0, P)
    // Imp3D random edges from senders on other ranks, per local in-edge:
    // round tag (the round the message was delivered for) and the message
    uint32_t* rtag;
    double2* rmsg;
    // Imp3D push-sum across ranks (sender-ordered lists, gp_xchg.hpp): per local in-edge
    // whose sender lives on another rank, its list key (64 * header word + bit) in this
    // rank's received header region; the received headers and messages of the round
    // ([b]: the buffer the exchange for a round of parity b fills; one buffer for both unless
    // the round kernel runs region by region, when the next round's lists arrive during this one)
    uint32_t* rk;
    const XHdr* xhdr[2];
    const double2* xvals[2];
    uint32_t xnv;  // message slots in the vals region
    int kernel;  // KERNEL_* below
    // column kernels: x segments per patch (set at create from the resident grid)
    uint32_t col_xsegs;
    uint32_t tile_walk;  // RoundArgs::walk
    uint32_t tile_wx;    // RoundArgs::wx
    uint32_t tile_stage_cap;  // RoundArgs::stage_cap (experiments build only; default: no limit)
    uint32_t fuse_finalize;   // the round kernel closes its own round (single rank push-sum)
    BlockPlan bplan;          // KERNEL_BLOCK (gp_block.hip): boxes, face buffer, barrier scratch
    void* bface;
    void* bscratch;
    uint32_t tile_wide;       // KERNEL_TILE: the 1024-thread size class (gp_round_wide.hip)
    // Imp3D: the rank's in-edge count
    uint32_t nedges;
    // walk 3 (dynamic tile queue): per round parity, 8 per-XCD item counters,
    // TQ_STRIDE words apart (one 256-byte line each)
    uint32_t* tq;
    // walk 3: the slab's tiles (relative to lo / TILE) in visiting order, XCD c's
    // items at [woff[0][c], woff[0][c + 1]); with rregions > 1 launches per round
    // (launch_round_regions, gp_api.hip) launch h visits region h's tiles, XCD c's
    // at [woff[h][c], woff[h][c + 1])
    uint32_t* wtiles;
    uint32_t rregions;
    uint32_t woff[RREG_MAX][9];
};
constexpr int TQ_STRIDE = 64;
hipError_t launch_round_tile_region(const DevState& S, uint32_t round, uint32_t h, int grid, hipStream_t st);

// Arguments of the tiled round kernels (gp_round.hip): only what they read.
struct RoundArgs {
    const double2* swc;
    double2* swn;
    const uint8_t* nbc;
    uint8_t* nbn;
    const uint64_t* rbc;
    uint64_t* rbn;
    const uint32_t* in_off;  // indexed by global id
    const uint32_t* in_src;
    const uint32_t* in_srcd; // in_src with the sender's deg - 4 in bits 30-31, or null
    const uint8_t* ind4;     // nibble in-degrees (DevState::ind4), offset so that ind4 + j / 2 is node j's byte
    const uint32_t* rtag;    // per local in-edge: round of the delivered remote message (gossip)
    const double2* rmsg;
    const uint32_t* rk;      // push-sum: per local in-edge, the remote sender's list key (DevState::rk)
    const XHdr* xhdr;        // push-sum: the received header words / messages of the round
    const double2* xvals;
    uint32_t xnv;
    int32_t* c;              // indexed by global id
    Ctl* ctl;
    Geom G;
    uint32_t k0, k1, seed_node, ntiles;
    uint32_t lo, nloc, ext_lo, ext_hi;  // owned ids [lo, lo + nloc); arrays hold [ext_lo, ext_hi)
    uint32_t walk;  // 0: XCD-contiguous eighths, 1: one global sweep (tile t -> block t % grid), 2: x-windows,
                    // 3: x-windows claimed from per-XCD counters (k_ps_tile)
    uint32_t wx;    // walk 2: planes per x-window
    uint32_t stage_cap;  // k_ps_tile: tiles with more in-edges take the unstaged path (tests force it)
    uint32_t fuse;       // k_ps_tile: the last block closes the round (no k_finalize launch)
    const uint32_t* wt;  // walk 3: tile list (DevState::wtiles), XCD c's items at [wo[c], wo[c + 1])
    uint32_t wo[9];
    uint32_t* tq;        // walk 3: this round's 8 per-XCD tile-item counters (TQ_STRIDE apart)
    uint32_t* tq_next;   // walk 3: the next round's counters, zeroed by block 0 this round
};

enum KernelVariant : int { KERNEL_TILE = 1, KERNEL_COL = 2, KERNEL_BLOCK = 3 };

// ---- LDS-resident push-sum on a small 3D lattice (gp_block.hip): one cooperative launch
// per batch of rounds (BlockPlan above DevState)
bool block_plan(uint32_t g, int cus, BlockPlan& p);
size_t block_face_bytes(const BlockPlan& p);
hipError_t block_kernel_setup(const BlockPlan& p);
bool block_plan_resident(const BlockPlan& p, int cus);
// rounds [r0, r0 + nrounds) (fewer once the cumulative alerts reach T); scratch:
// BLOCK_SCRATCH_BYTES, word 1 is set if a grid barrier timed out
constexpr int BLOCK_EPOCH = 64;       // rounds between the kernel's grid barriers
constexpr size_t BLOCK_SCRATCH_BYTES = 4 * (144 + 12 * BLOCK_EPOCH);
hipError_t launch_round_block(const struct DevState& S, const BlockPlan& p, uint32_t r0, uint32_t nrounds, void* face,
                              void* scratch, hipStream_t st);

// Arguments of the column-march gossip kernels (gp_col.hip).
struct WaveArgs {
    const double2* swc;
    double2* swn;
    const uint8_t* nbc;
    uint8_t* nbn;
    const uint64_t* rbc;
    uint64_t* rbn;
    const uint32_t* in_off;
    const uint32_t* in_src;
    const uint32_t* rtag;
    const double2* rmsg;
    int32_t* c;
    uint32_t* rq_cur;        // Imp3D gossip: this round's random-edge deliveries per local node (read, then zeroed)
    uint32_t* rq_next;       // next round's, counted by local senders with atomics (remote ones: k_unpack)
    uint32_t rq8;            // byte counters (DevState::rq8)
    const uint32_t* rnd;     // random edge of each local sender (id - lo)
    const uint32_t* rtg;     // several ranks: local target or send-bitmap bit of it (DevState::rtg)
    uint32_t* sbits;
    Ctl* ctl;
    Geom G;
    uint32_t k0, k1, seed_node;
    uint32_t lo, nloc, base;
    // column kernels (gp_col.hip): planes [x_lo, x_hi) of this rank, patches of
    // 64 z x 4 y rows, x split into segments of xs_len planes
    uint32_t x_lo, x_hi, zsegs, yblocks, xs_len, nitems;
};

// ---- column-march round kernels (gp_col.hip): 3D / Imp3D
WaveArgs make_wave_args(const DevState& S, uint32_t round);

hipError_t launch_round_col(const WaveArgs& a, int topo, int alg, uint32_t round, int grid, hipStream_t st);
int col_blocks_per_cu(int topo, int alg);
// Imp3D gossip: count the seed's round-0 random-edge send at its target (rq)
hipError_t launch_col_seed_init(const DevState& S, hipStream_t st);

// ---- tiled round kernels (gp_round.hip)
uint32_t rbits_words_for(uint32_t lo, uint32_t nloc);
hipError_t launch_round_tile(const DevState& S, uint32_t round, int grid, hipStream_t st);
int ps_tile_resident_blocks(int topo, bool remote, int device);
bool build_walk_list(const DevState& S, int NR, std::vector<uint32_t>& list, uint32_t woff[][9]);
bool region_tiles(uint32_t lo, uint32_t nloc, uint64_t g2, int NR, uint32_t* rb);
hipError_t launch_rbits_init(const DevState& S, int grid, hipStream_t st);
uint32_t ind4_bytes_for(uint32_t lo, uint32_t nloc);
hipError_t launch_pack_ind4(const DevState& S, uint32_t wide_at, int grid, hipStream_t st);
hipError_t launch_pack_src_deg(const uint32_t* src, uint32_t* out, uint32_t n, const Geom& G, int grid,
                               hipStream_t st);

// ---- the same tiled kernels as the small-population size class (gp_round_wide.hip)
namespace wide {
hipError_t launch_round_tile(const DevState& S, uint32_t round, int grid, hipStream_t st);
int ps_tile_resident_blocks(int topo, bool remote, int device);
}  // namespace wide

// ---- kernels (gp_kernels.hip)
hipError_t launch_init(const DevState& S, int grid, hipStream_t st);
hipError_t launch_injector_init(const DevState& S, int grid, hipStream_t st);
hipError_t launch_bulk(const DevState& S, uint32_t round, int grid, hipStream_t st);
hipError_t launch_finalize(const DevState& S, uint32_t round_done, uint32_t round_next, hipStream_t st);
hipError_t launch_finalize_pre(const DevState& S, uint32_t round_next, hipStream_t st);
hipError_t launch_count_alerted(const uint8_t* nb, const int32_t* c, uint32_t n, unsigned long long* out, int grid,
                                hipStream_t st);
hipError_t launch_finalize_post(const DevState& S, uint32_t round_done, uint32_t round_next, hipStream_t st);
hipError_t launch_full_pushsum_round(const DevState& S, uint32_t round, int grid, hipStream_t st);
hipError_t launch_iota(uint32_t* v, uint32_t n, int grid, hipStream_t st);
hipError_t launch_histogram(const uint32_t* keys, uint32_t n, uint32_t* counts, int grid, hipStream_t st);
const char* bulk_kernel_name(const DevState& S);

// ---- sorting (gp_sort.hip, rocPRIM)
// Stable sort of (key, value) pairs on the low `bits` bits of the key.
hipError_t sort_pairs(void* tmp, size_t& tmp_bytes, const uint32_t* kin, uint32_t* kout,
                      const uint32_t* vin, uint32_t* vout, uint32_t n, uint32_t bits, hipStream_t st);
// out[0] = 0, out[i] = sum(in[0..i-1]) for i <= n-1 (n entries).
hipError_t exclusive_scan_u32(void* tmp, size_t& tmp_bytes, const uint32_t* in, uint32_t* out, uint32_t n,
                              hipStream_t st);

}  // namespace gp
