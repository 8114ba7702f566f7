// gp_xchg.hpp -- argument blocks of the multi-rank kernels (gp_xchg.hip).
// Not part of the C-ABI.
#pragma once

#include "gp_internal.hpp"

namespace gp {

constexpr int XMAXW = 16;  // ranks supported by the exchange (one node: 8 GPUs)

// One rank pair's exchange buffer: [count u32 | pad][slots: cap u32][vals: cap (s, w)].
struct XPeer {
    uint32_t* cnt;
    uint32_t* slots;
    double2* vals;
    uint32_t cap;
};

struct PackArgs {
    const uint8_t* nbn;   // node bytes of the round being prepared (local array, id - base)
    const double2* swn;   // (s, w) of that round (local array, id - base)
    const uint32_t* rnd;  // random edge of each local sender (id - lo)
    const uint8_t* xdst;  // owner rank of that edge's target (id - lo)
    const uint32_t* pos;  // its slot in the destination's in-edge array (id - lo; null in counts mode)
    uint32_t lo, nloc, base;
    uint32_t s_lo, s_hi;  // the senders packed by this launch (local ids, one exchange region)
    int W, me, push;
    int counts;           // gossip column kernel: the entry is the target's local id at its owner
                          // (a delivery count, k_unpack adds it to rq), not an in-edge slot
    uint32_t bounds[XMAXW + 1];
    XPeer peer[XMAXW];    // send side
    unsigned int* overflow;
};

struct UnpackArgs {
    uint32_t* rtag;
    double2* rmsg;
    uint32_t* rq;         // counts mode (gossip column kernel): next round's deliveries per local node
    uint32_t rq8;         // (byte counters, DevState::rq8)
    uint32_t nedges;      // entries must be below this bound (in-edges; counts mode: local nodes)
    int W, me, push;
    XPeer peer[XMAXW];    // receive side
    unsigned int* overflow;  // set when a sender packed more messages than the buffer holds
    const unsigned int* all_active;  // Ctl::all_active of this rank (push-sum: no tags once set)
};

struct ZeroArgs {
    uint32_t* cnt[XMAXW];
    int n;
};

struct SumArgs {
    Ctl* ctl[XMAXW];
    int W;
};

struct PosArgs {
    const uint32_t* rnd;  // local senders' random edges
    const uint32_t* inv;  // global sorted position of every sender
    uint32_t* pos;        // may be null (counts mode)
    uint8_t* xdst;
    uint32_t lo, nloc;
    int W, me;
    uint32_t bounds[XMAXW + 1];
    uint32_t edge0[XMAXW];  // first global sorted position owned by each rank
};

struct ExpectArgs {
    const uint32_t* rnd;
    uint32_t lo, nloc;
    uint32_t s_lo, s_hi;  // senders counted (local ids)
    int W, me;
    uint32_t bounds[XMAXW + 1];
    Geom G;
    double* mu;               // [W] expected messages per round to each rank
    unsigned long long* n;    // [W] random edges to each rank
};

// ---- Imp3D push-sum: sender-ordered lists (round 5).  For each rank pair a -> b
// the static list L_ab = a's senders whose random edge lands on b, in id order,
// cut into the slab's 1024-id tiles (XTILE, the push-sum tile kernel's TILE) and
// NH <= XMAXH regions of consecutive tiles (tb[h] <= tile < tb[h + 1]); every (tile, b) segment starts
// on a 64-entry boundary of the region's list (gw: its first header word).  Per
// round the sender writes, per region and destination, one header word per 64
// list entries -- the bitmap of the entries whose sender used its random edge and
// the index of the first such message in the destination's vals region -- and the
// used entries' (s, w) compacted in list order.  The receiver finds a used remote
// in-edge's message at base + popcount(mask below its bit): no scatter, no slots.
constexpr uint32_t XTILE = 1024;
constexpr int XMAXH = 8;           // exchange regions of a slab (push-sum), at most
constexpr uint32_t XNONE = 0xFFu;  // "no list entry" (local target or no sender)

struct ListPeer {              // send side: region h, destination d
    XHdr* hdr;                 // NW header words
    double2* vals;             // cap message slots
    uint32_t* cnt;             // reservation counter (zeroed before the region's pack)
    uint32_t cap;
    uint32_t vbase;            // index of this chunk's first slot in d's vals region
};

struct ListPackArgs {
    const uint8_t* nbn;        // node bytes of the round being prepared (local array, id - base)
    const double2* swn;        // (s, w) of that round (local array, id - base)
    const uint16_t* xdr;       // [id - lo]: d << 10 | the sender's rank in its tile's list for d (static), or XDR_NONE
    const uint8_t* lwt;        // [tile * (W + 1) + d]: first LDS word of d's segment in the tile (static)
    const uint32_t* gw;        // [tile * W + d]: first header word of the tile's segment in chunk (region, d)
    uint32_t lo, nloc, base;
    uint32_t t0, t1;           // the region's tiles (relative to lo / XTILE)
    int W, me;
    ListPeer peer[XMAXW];
    unsigned int* overflow;
};

struct ListCountArgs {         // setup, slab a: list entries per (tile, destination)
    const uint32_t* rnd;       // global random edges (rnd[i] for every id)
    uint32_t lo, nloc;
    int W, a;
    uint32_t bounds[XMAXW + 1];
    uint32_t* cnt;             // [tile * W + d]
};

struct ListKeyArgs {           // setup, slab a: every sender's list key at its destination
    const uint32_t* rnd;       // global random edges
    const uint32_t* gw;        // slab a's [tile * W + d]
    uint32_t lo, nloc;
    uint32_t tb[XMAXH + 1];    // region h: tiles [tb[h], tb[h + 1]) of the slab (relative to lo / XTILE)
    int NH, W, a;
    uint32_t bounds[XMAXW + 1];
    uint32_t hw[XMAXH][XMAXW]; // [h][b]: first header word of chunk (h, a) in b's header region
    uint32_t* key;             // [global id]: 64 * header word + bit at the destination (local targets untouched)
    uint16_t* xdr;             // optional, [id - lo]: d << 10 | rank in the tile's list for d, or XDR_NONE
};
constexpr uint16_t XDR_NONE = 0xFFFFu;

// ---- Imp3D gossip on the column kernel across ranks: random-edge sends as bitmaps
// (round 5).  For each rank pair a -> b the static list of edges from a's senders to
// b's nodes, in b's receiver order (target, then sender), one bit per edge.  A sender
// whose next direction is its random edge sets its edge's bit (k_gossip_col, an
// atomicOr; rtg names the bit), the bitmaps travel (1 bit per remote edge instead of a
// 4-byte entry per send, no pack pass), and the receiver adds one rumour per set bit
// to its target's next-round count (k_apply_bits; tgt names the target of every bit).
// Counts are integers, so the order of the additions is free.
struct BitsSetupArgs {
    const uint32_t* src;      // global senders in receiver order (the in-list sort)
    const uint32_t* recv;     // their receivers (sorted random edges)
    const uint32_t* scan;     // exclusive scan of [slab(src[q]) == a] (k_src_flag)
    uint32_t* pos;            // out: for edges with a sender on slab a, the bit in its (a -> b) list
    uint32_t n;               // edges (= P)
    int W, a;
    uint32_t bounds[XMAXW + 1];
    uint32_t edge0[XMAXW + 1];  // first edge (global sorted position) of each receiver slab
};

struct BitsEndsArgs {         // this rank's encodings
    const uint32_t* rnd;      // local senders' random edges (id - lo)
    const uint32_t* inv;      // global sorted position of every sender's edge
    const uint32_t* src;      // global senders in receiver order
    const uint32_t* recv;     // their receivers
    const uint32_t* pos;      // k_bits_pos's output for every edge
    uint32_t* rtg;            // out [nloc]: local target (t - lo), or 0x80000000 | bit of the send bitmap
    uint32_t* tgt;            // out: local receiver of every bit of the receive bitmap
    uint32_t lo, nloc, e0, e1;  // this rank's ids and in-edges [e0, e1)
    int W, me;
    uint32_t bounds[XMAXW + 1];
    uint32_t bo[XMAXW];       // bit offset of destination d's chunk in the send bitmap
    uint32_t ro[XMAXW];       // bit offset of source a's chunk in the receive bitmap
};

// Push-sum halo planes over several ranks (3D / Imp3D): a neighbour's round kernel reads the
// (s, w) of a halo node only when that node sends to it (its direction byte, which travels in
// full), so only those (s, w) travel, compacted per 1024-node chunk into `cap` slots (a fuller
// chunk sets the overflow flag).  k_halo_pack on the sender, k_halo_expand into the receiver's
// halo plane.  The capacity is sized for the lattice's worst chunk (halo_chunk_cap): a node of
// degree d sends toward the neighbour with probability 1/d, so a chunk made of a plane's
// boundary row y = 0 (3D: degree 5; Imp3D: 6) expects 205 / 171 senders where an interior
// chunk expects 146 (Imp3D) -- 12 sigma over the worst, as the other exchange buffers.
constexpr uint32_t HALO_CHUNK = 1024;
struct HaloArgs {
    const uint8_t* nb;      // direction bytes of the plane's nodes
    double2* sw;            // the plane's (s, w): read by the pack, written by the expand
    double2* buf;           // [chunk * cap + rank]: the senders' (s, w), in id order per chunk
    uint32_t n;             // nodes in the plane
    uint32_t cap;           // slots per chunk
    uint32_t dir;           // the direction whose senders' (s, w) travel
    unsigned int* overflow;
};
inline size_t halo_buf_slots(uint32_t n, uint32_t cap) { return (size_t)((n + HALO_CHUNK - 1) / HALO_CHUNK) * cap; }
uint32_t halo_chunk_cap(uint32_t g, bool imp3d);
hipError_t launch_halo_pack(const HaloArgs& a, hipStream_t st);
hipError_t launch_halo_expand(const HaloArgs& a, hipStream_t st);

hipError_t launch_src_flag(const uint32_t* src, uint32_t n, const uint32_t* bounds, int W, int a, uint32_t* flag,
                           int grid, hipStream_t st);
hipError_t launch_bits_pos(const BitsSetupArgs& a, int grid, hipStream_t st);
hipError_t launch_bits_ends(const BitsEndsArgs& a, int grid, hipStream_t st);
hipError_t launch_apply_bits(const uint32_t* bits, uint32_t nwords, const uint32_t* tgt, uint32_t* rq, uint32_t rq8,
                             hipStream_t st);

hipError_t launch_list_count(const ListCountArgs& a, hipStream_t st);
hipError_t launch_list_key(const ListKeyArgs& a, hipStream_t st);
hipError_t launch_list_pack(const ListPackArgs& a, hipStream_t st);
hipError_t launch_gather_keys(const uint32_t* key, const uint32_t* src, uint32_t n, uint32_t* out, int grid,
                              hipStream_t st);

hipError_t launch_pack(const PackArgs& a, int grid, hipStream_t st);
hipError_t launch_unpack(const UnpackArgs& a, uint32_t round, int grid, hipStream_t st);
hipError_t launch_zero_counts(const ZeroArgs& z, hipStream_t st);
hipError_t launch_sum_xchg(const SumArgs& s, hipStream_t st);
hipError_t launch_topo_rnd_range(uint32_t k0, uint32_t k1, uint32_t P, uint32_t first, uint32_t n, uint32_t* out,
                                 int grid, hipStream_t st);
hipError_t launch_inverse(const uint32_t* perm, uint32_t n, uint32_t* inv, int grid, hipStream_t st);
hipError_t launch_sub(uint32_t* v, uint32_t n, uint32_t d, int grid, hipStream_t st);
hipError_t launch_make_pos(const PosArgs& a, int grid, hipStream_t st);
hipError_t launch_expect(const ExpectArgs& a, int grid, hipStream_t st);

}  // namespace gp
