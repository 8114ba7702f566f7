// gp_full.hpp -- argument block of the multi-rank full-topology gossip kernels
// (gp_full.hip).  Not part of the C-ABI.
#pragma once

#include "gp_xchg.hpp"

namespace gp {

struct FullArgs {
    // node state of this rank, indexed by local id (id - lo)
    uint8_t* nb;            // push-sum node byte (single buffer, updated by recv)
    const double2* swc;     // (s, w) at round start
    double2* swn;           // (s, w) after the round
    int32_t* c;             // gossip rumour counters
    int32_t* inc;           // gossip deliveries of the round
    Ctl* ctl;
    unsigned int* overflow;
    uint32_t P, lo, nloc, k0, k1, seed_node;
    int W, me;
    uint32_t bounds[XMAXW + 1];
    XPeer peer[XMAXW];      // send buffers
    XPeer rpeer[XMAXW];     // receive buffers
};

hipError_t launch_fullm_gossip_send(const FullArgs& a, uint32_t r, int grid, hipStream_t st);
hipError_t launch_fullm_gossip_unpack(const FullArgs& a, int grid, hipStream_t st);
hipError_t launch_fullm_gossip_recv(const FullArgs& a, int grid, hipStream_t st);

}  // namespace gp
