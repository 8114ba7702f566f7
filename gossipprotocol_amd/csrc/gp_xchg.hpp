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
