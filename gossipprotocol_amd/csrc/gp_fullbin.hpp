// gp_fullbin.hpp -- single-rank full-topology push-sum round by two-level LDS
// binning (gp_fullbin.hip).  Not part of the C-ABI.
#pragma once

#include "gp_xchg.hpp"

namespace gp {

// fine tile = 2^FB_TB receivers (one fold block); 4096 (measured: 10 / 11 / 12 -> 3.65 / 3.63 /
// 3.60 ms at P = 1e8)
constexpr int FB_TB = 12;
// messages per fine tile: expected 2^FB_TB + 12 sigma + 128 (4992 at 4096 receivers)
constexpr int FB_CAP2 = ((1 << FB_TB) + 12 * (1 << (FB_TB / 2)) * (FB_TB % 2 ? 1414 : 1000) / 1000 + 128 + 63) / 64 * 64;

struct FullBinPlan {
    uint32_t s1;    // coarse bin = target >> s1
    uint32_t nb1;   // coarse bins
    uint32_t nb2;   // fine tiles
    uint32_t cap1;  // message capacity per coarse bin
    uint32_t cap2;  // message capacity per fine tile
};

struct FullBinArgs {
    const double2* swc;  // (s, w) at round start
    double2* swn;        // (s, w) after the round
    uint8_t* nb;         // node byte (active / converged / count), single buffer
    Ctl* ctl;
    unsigned int* overflow;
    uint32_t P, k0, k1;
    uint32_t s1, nb1, nb2, cap1, cap2;
    uint32_t* cnt1;      // [nb1] messages per coarse bin (zeroed every round)
    uint32_t* cnt2;      // [nb2] messages per fine tile
    uint32_t* hdr1;      // [nb1 * cap1] sender id (the target is recomputed from its Philox draw)
    double2* pay1;       // [nb1 * cap1] {s / 2, w / 2}
    uint32_t* hdr2;      // [nb2 * cap2] sender id
    double2* pay2;
    // receivers of this rank: global ids [lo, lo + nloc) (one rank: 0, P); node
    // arrays (swc, swn, nb) are indexed by id - lo, coarse bins and fine tiles count
    // from lo
    uint32_t lo, nloc;
    uint32_t s_lo, s_hi;  // several ranks: k_fbm_send bins the senders lo + [s_lo, s_hi) (a half of the slab)
    uint32_t fused;       // one rank: k_fb_fold<true> also bins the next round's messages into hdr1 / pay1
    // several ranks (k_fbm_send / k_fbm_coarse): senders' messages binned by
    // destination rank into the exchange buffers, then the received ones by coarse bin
    int W, me;
    uint32_t bounds[XMAXW + 1];
    XPeer out[XMAXW];       // this rank's messages to rank b (b == me: its own receive buffer)
    XPeer in[XMAXW];        // messages from rank b (after the exchange)
    uint32_t in_item0[XMAXW + 1];  // first k_fbm_coarse work item of each source rank
};

FullBinPlan full_bin_plan(uint32_t nrecv, bool fused);  // fused: one rank, k_fb_fold<true>
hipError_t launch_full_bin_round(const FullBinArgs& a, uint32_t round, int grid, hipStream_t st);
// several ranks: messages of the senders [s_lo, s_hi) into the exchange buffers (before the
// exchange) ...
hipError_t launch_full_bin_send_multi(const FullBinArgs& a, uint32_t round, hipStream_t st);
// ... then, per round, the bin counters reset, the received messages of each exchange region
// binned by coarse bin, and the split and fold
hipError_t launch_full_bin_recv_reset(const FullBinArgs& a, hipStream_t st);
hipError_t launch_full_bin_coarse(const FullBinArgs& a, uint32_t round, hipStream_t st);
hipError_t launch_full_bin_split_fold(const FullBinArgs& a, uint32_t round, int grid, hipStream_t st);
uint32_t full_bin_item_messages();
uint32_t full_bin_fused_max_bins();  // coarse bins the fused fold can bin into

}  // namespace gp
