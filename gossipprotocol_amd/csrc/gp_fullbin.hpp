// gp_fullbin.hpp -- full-topology push-sum rounds by two-level LDS binning
// (gp_fullbin.hip).  Not part of the C-ABI.
#pragma once

#include "gp_xchg.hpp"

namespace gp {

// fine tile = 2^FB_TB receivers (one fold block); 4096 (measured: 10 / 11 / 12 -> 3.65 / 3.63 /
// 3.60 ms at P = 1e8)
constexpr int FB_TB = 12;
// messages per fine tile: expected 2^FB_TB + 12 sigma + 128 (4992 at 4096 receivers)
constexpr int FB_CAP2 = ((1 << FB_TB) + 12 * (1 << (FB_TB / 2)) * (FB_TB % 2 ? 1414 : 1000) / 1000 + 128 + 63) / 64 * 64;

// one rank: slots past the last coarse bin (hdr1 / pay1) that the fused fold's write-out sends
// its lanes without a message to, so that every thread issues the same stores (k_fb_fold)
constexpr size_t FB_JUNK = 64;

struct FullBinPlan {
    uint32_t s1;    // coarse bin = target >> s1
    uint32_t nb1;   // coarse bins
    uint32_t nb2;   // fine tiles
    uint32_t cap1;  // message capacity per coarse bin
    uint32_t cap2;  // message capacity per fine tile
};

// A set of `nb` coarse bins of `cap` messages each -- one rank's own coarse bins (cnt1 / hdr1 /
// pay1), or, across ranks, the coarse bins of one destination rank's receivers that one exchange
// region carries: [counts: nb u32 | pad to 16 B][sender ids: nb * cap u32 | pad][payloads:
// nb * cap (s / 2, w / 2)], one contiguous buffer (fb_bins_bytes / fb_bins_at), so it travels
// as one RCCL send with its counts in band.
struct FbBins {
    uint32_t* cnt;
    uint32_t* hdr;
    double2* pay;
    uint32_t cap;
    uint32_t nb;
};
size_t fb_bins_bytes(uint32_t nb, uint32_t cap);
FbBins fb_bins_at(uint8_t* base, uint32_t nb, uint32_t cap);

struct FullBinArgs {
    const double2* swc;  // (s, w) at round start
    double2* swn;        // (s, w) after the round
    uint8_t* nb;         // node byte (active / converged / count), single buffer
    Ctl* ctl;
    unsigned int* overflow;
    uint32_t P, k0, k1;
    uint32_t s1, nb1, nb2, cap1, cap2;
    uint32_t* cnt1;      // [nb1] messages per coarse bin (one rank; zeroed every round)
    uint32_t* cnt2;      // [nb2] messages per fine tile
    uint32_t* hdr1;      // [nb1 * cap1] sender id (the target is recomputed from its Philox draw)
    double2* pay1;       // [nb1 * cap1] {s / 2, w / 2}
    uint32_t* hdr2;      // [nb2 * cap2] sender id
    double2* pay2;
    // receivers of this rank: global ids [lo, lo + nloc) (one rank: 0, P); node
    // arrays (swc, swn, nb) are indexed by id - lo, coarse bins and fine tiles count
    // from lo
    uint32_t lo, nloc;
    uint32_t s_lo, s_hi;  // send pass: the senders lo + [s_lo, s_hi) (several ranks: one exchange region)
    uint32_t t_lo, t_hi;  // fold: the fine tiles [t_lo, t_hi) (several ranks: one exchange region's)
    uint32_t fused;       // one rank: the fold bins the next round's messages into hdr1 / pay1
    // several ranks: every rank's coarse bins have the size 2^s1, so a message to target t
    // has the key kb(b) + ((t - bounds[b]) >> s1), b = owner of t, kb(b) = the bins of the
    // ranks below b -- the LDS bins of the send pass and of the fold's send phase
    int W, me;
    uint32_t bounds[XMAXW + 1];
    FbBins out[XMAXW];   // this region's bins for rank b's receivers (b == me: its own receive region)
    FbBins in[XMAXW];    // the region's bins from rank p for this rank's receivers (after the exchange)
    uint32_t in_item0[XMAXW + 1];  // first split work item of each source rank
};

FullBinPlan full_bin_plan(uint32_t nrecv, bool fused);  // fused: one rank, the fold bins the next round
// several ranks: the coarse-bin shift every rank uses (all slabs' bins together within the
// fold's LDS reservation slots)
uint32_t full_bin_multi_s1(const uint32_t* bounds, int W);
// several ranks: the per-bin capacity of the messages a region of n senders sends to one
// rank's coarse bin (Binomial(n, 2^s1 / (P - 1)) + 12 sigma + 64)
uint32_t full_bin_multi_cap(uint32_t n_senders, uint32_t s1, uint32_t P);
hipError_t launch_full_bin_round(const FullBinArgs& a, uint32_t round, int grid, hipStream_t st);
// several ranks: round 0's messages (senders [s_lo, s_hi)) into the exchange buffers ...
hipError_t launch_full_bin_send_multi(const FullBinArgs& a, uint32_t round, hipStream_t st);
// ... per round: the counters the round fills cleared in one launch (the fine tiles', every
// region's send bins', this rank's own next-round bins': ZeroList), each region's received bins
// split into this rank's fine tiles, and the fold of each region's tiles, which bins their
// next-round messages into the region's exchange buffers
constexpr int FB_REGIONS = 2;  // exchange regions of a slab (full push-sum)
struct ZeroList {
    static constexpr int MAX = 1 + FB_REGIONS * (XMAXW - 1) + 2 * FB_REGIONS;
    uint32_t* p[MAX];
    uint32_t n[MAX];
    int k;
};
hipError_t launch_zero_list(const ZeroList& z, hipStream_t st);
hipError_t launch_full_bin_split_multi(const FullBinArgs& a, uint32_t round, hipStream_t st);
hipError_t launch_full_bin_fold_multi(const FullBinArgs& a, uint32_t round, int cus, hipStream_t st);
uint32_t full_bin_item_messages();
uint32_t full_bin_fused_max_bins();  // coarse bins the fused fold can bin into

}  // namespace gp
