// gp_api.hip -- C-ABI of libgossip_hip.so (include/gossip_hip.h) and the host
// orchestrator of the synchronous round loop, on one GPU or sharded over ranks.
//
// Replaces, in /root/reference/Project2/Program.fs:
//   * actor population + topology build (Program.fs:169-176,180-191,209-216,238-261)
//     -> gp_create / gp_create_rank: SoA device state per slab, implicit
//     neighbours, Imp3D receiver-sorted in-lists;
//   * message loop + scheduler (Program.fs:41-61,84-131,141-163) -> gp_step / gp_run:
//     per round the bulk round kernel, the inter-rank exchange and the
//     finalize kernel(s), queued in batches with one host synchronisation per
//     batch (never per round).
//
// Sharding: contiguous node-id slabs, plane-aligned for 3D /
// Imp3D.  Each slab's node arrays carry one halo plane (line: one node) per
// neighbouring slab.  After every round the halos are refreshed from the
// neighbours and the Imp3D random-edge messages are exchanged (gp_xchg.hip);
// the round's alert / activation / injector counts are summed over ranks.
// Two transports: RCCL between processes (one process per GPU, gp_create_rank),
// and in-process "virtual ranks" on one device (gp_config.flags
// GP_FLAG_VIRTUAL_RANKS), which run the same kernels and exchange plan with
// device copies -- the single-GPU test bed of the multi-GPU path.
#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cerrno>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <rccl/rccl.h>

#include "../../include/gossip_hip.h"
#include "gp_internal.hpp"
#include "gp_full.hpp"
#include "gp_fullbin.hpp"

namespace {
// The experiments build (-DGP_EXPERIMENTS, libgossip_hip_exp.so) reads the GP_* environment
// overrides the kernel-variant tests use; the product library reads none (nullptr: every
// override below folds away, its name included -- tests/test_abi.py checks the strings).
inline const char* exp_env(const char* name) {
#ifdef GP_EXPERIMENTS
    return std::getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}
}  // namespace
#include "gp_xchg.hpp"

using namespace gp;

namespace {

thread_local std::string g_err;

void set_err(const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
}

#define HIP_TRY(expr)                                                                   \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess) {                                                         \
            set_err("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
            return GP_EHIP;                                                             \
        }                                                                               \
    } while (0)

#define NCCL_TRY(expr)                                                                  \
    do {                                                                                \
        ncclResult_t r_ = (expr);                                                       \
        if (r_ != ncclSuccess) {                                                        \
            set_err("%s failed: %s (%s:%d)", #expr, ncclGetErrorString(r_), __FILE__, __LINE__); \
            return GP_ENCCL;                                                            \
        }                                                                               \
    } while (0)

constexpr int64_t BATCH = 1024;  // rounds queued per host synchronisation (<= HIST)
static_assert(BATCH <= HIST, "alert ring must cover a batch");

enum Mode { MODE_SINGLE = 0, MODE_VIRTUAL = 1, MODE_RCCL = 2 };

// One rank's share of the network.
struct Slab {
    DevState S{};
    int rank = 0;
    uint32_t hi = 0;  // one past the last owned id
    // Imp3D random-edge exchange (W > 1)
    uint32_t* pos = nullptr;
    uint8_t* xdst = nullptr;  // owner rank of each local sender's random-edge target (k_pack)
    uint8_t* xsend = nullptr;
    uint8_t* xrecv = nullptr;
    uint32_t nedges = 0;
    std::vector<uint32_t> cap_out, cap_in;           // [h * W + b]: region h of the buffer to / from rank b
    std::vector<size_t> soff, sbytes, roff, rbytes;
    unsigned int* overflow = nullptr;  // device flag
    // Imp3D push-sum over several ranks: sender-ordered lists (gp_xchg.hpp)
    bool lists = false;
    uint32_t nt = 0;                   // the slab's tiles
    uint32_t tb[XMAXH + 1] = {};       // region h: tiles [tb[h], tb[h + 1])
    uint32_t* gw = nullptr;            // [tile * W + d]: first header word of the tile's segment
    uint16_t* xdr = nullptr;           // [id - lo]: d << 10 | rank in the tile's list for d (static)
    uint8_t* lwt = nullptr;            // [tile * (W + 1) + d]: the tile's LDS word layout in k_list_pack
    uint32_t* xcnt = nullptr;          // [h * W + d]: reservation counters of the send chunks
    std::vector<size_t> lhdr, lval;    // send buffer: byte offsets of chunk (h, d)'s header words / slots
    std::vector<size_t> rhdr, rval;    // receive buffer: byte offsets of chunk (h, p)'s header words / slots
    size_t xr_stride = 0;              // the receive buffer of odd rounds at xrecv + xr_stride (region-by-region
                                       // rounds: the next round's lists arrive during this one), else 0
    std::vector<uint32_t> vbase;       // [h * W + d]: index of my chunk's first slot in d's vals region
    // full push-sum over several ranks: this rank's own share of region h's bins, by round parity:
    // parity 0 in xrecv (its receive region from itself), parity 1 in xown -- the fold of round r
    // fills parity r + 1 while the split of round r has read parity r, and a round's counters are
    // all cleared at its start (launch_round_full_multi)
    uint8_t* xown = nullptr;
    size_t ooff[FB_REGIONS] = {};
    // Imp3D gossip (column kernel) over several ranks: random-edge sends as bitmaps (gp_xchg.hpp)
    bool bits = false;
    uint32_t* rbits_in = nullptr;      // receive bitmap: source a's chunk at bit ro[a]
    uint32_t* tgt = nullptr;           // local target of every receive-bitmap bit
    uint32_t nbits_out = 0, nbits_in = 0;  // bitmap sizes (multiples of BITS_ALIGN)
    std::vector<uint32_t> bo, bn, ro, rn;  // [peer]: chunk bit offset / bits, send and receive side
    // push-sum halo planes (3D / Imp3D, W > 1): the senders' (s, w) toward each neighbour, compacted
    // ([0]: lower neighbour, [1]: upper; k_halo_pack / k_halo_expand, gp_xchg.hpp)
    double2* hsend[2] = {nullptr, nullptr};
    double2* hrecv[2] = {nullptr, nullptr};
};

constexpr uint32_t BITS_ALIGN = 1024;  // bitmap chunks start on 128-byte boundaries

size_t xbuf_bytes(uint32_t cap, bool push) {
    if (!cap) return 0;
    const size_t slots = ((size_t)cap * 4 + 15) & ~(size_t)15;
    return 16 + slots + (push ? (size_t)cap * 16 : 0);
}

XPeer xpeer(uint8_t* buf, size_t off, uint32_t cap) {
    XPeer p{};
    if (!cap) return p;
    uint8_t* b = buf + off;
    p.cnt = reinterpret_cast<uint32_t*>(b);
    p.slots = reinterpret_cast<uint32_t*>(b + 16);
    p.vals = reinterpret_cast<double2*>(b + 16 + (((size_t)cap * 4 + 15) & ~(size_t)15));
    p.cap = cap;
    return p;
}

}  // namespace

struct gp_sim {
    gp_config cfg{};
    int device = 0;
    hipStream_t stream = nullptr;
    int grid = 1;
    int cus = 1;  // compute units of the device
    int64_t P = 0, T = 0, g = 0;
    int mode = MODE_SINGLE;
    int world = 1, rank = 0;  // ranks sharing the population; this process's rank (RCCL)
    std::vector<uint32_t> bounds;  // world + 1 slab boundaries (global ids)
    uint32_t halo = 0;             // ids per halo side
    std::vector<Slab> slab;        // MODE_VIRTUAL: all ranks; otherwise this rank's
    ncclComm_t comm = nullptr;
    int64_t rounds_done = 0;
    int64_t alerts_total = 0;
    bool done = false;
    Ctl* host_ctl = nullptr;  // pinned mirror of slab 0's control block (global bookkeeping)
    std::vector<void*> allocs;
    // kernel timing
    bool timing = false;
    std::vector<hipEvent_t> ev;
    double kernel_ms = 0.0;
    int64_t launches = 0;
    // exchange buffers per rank pair: xhalves regions (2: full-topology push-sum, whose exchange runs
    // in two halves of each rank's senders on xstream, overlapped with the send / coarse passes)
    int xhalves = 1;
    size_t halo_slots = 0;  // push-sum halo planes travel compacted (setup_halo): slots per buffer, else 0
    uint32_t halo_cap = 0;  // ... slots per 1024-node chunk (halo_chunk_cap)
    // Imp3D push-sum lists: header words of chunk (h, a -> b) at [(a * xhalves + h) * world + b],
    // every slab's (each rank computes the whole table from the global random edges)
    std::vector<uint32_t> list_nw;
    hipStream_t xstream = nullptr;
    hipEvent_t ev_send[XMAXH] = {}, ev_xfer[XMAXH] = {};
    // region rounds (launch_round_regions): the packs' stream -- region h's pack runs beside the
    // round kernel's launch h + 1 -- and the events that release it
    BlockPlan bplan{};  // KERNEL_BLOCK
};

namespace {

int dev_alloc(gp_sim* s, void** p, size_t bytes) {
    if (bytes == 0) bytes = 16;
    hipError_t e = hipMalloc(p, bytes);
    if (e != hipSuccess) {
        set_err("hipMalloc(%zu bytes) failed: %s", bytes, hipGetErrorString(e));
        return GP_ENOMEM;
    }
    s->allocs.push_back(*p);
    return GP_OK;
}

template <typename T>
int dev_alloc_t(gp_sim* s, T** p, size_t count) {
    void* v = nullptr;
    int rc = dev_alloc(s, &v, count * sizeof(T));
    *p = static_cast<T*>(v);
    return rc;
}

// Setup temporaries: freed when the scope ends, on success and on every error return.
struct Scratch {
    std::vector<void*> ptrs;
    template <typename T>
    hipError_t alloc(T** p, size_t count) {
        void* v = nullptr;
        const hipError_t e = hipMalloc(&v, count * sizeof(T));
        if (e == hipSuccess) ptrs.push_back(v);
        *p = static_cast<T*>(v);
        return e;
    }
    ~Scratch() {
        for (void* v : ptrs) (void)hipFree(v);
    }
};

void free_all(gp_sim* s) {
    for (void* p : s->allocs) (void)hipFree(p);
    s->allocs.clear();
}

uint32_t bits_for(uint64_t maxval) {
    uint32_t b = 1;
    while (b < 32 && (maxval >> b) != 0) ++b;
    return b;
}

int check_device(int device) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
        set_err("no HIP device visible (libgossip_hip needs an MI355X / gfx950)");
        return GP_ENODEV;
    }
    if (device < 0 || device >= n) {
        set_err("device %d out of range (%d visible)", device, n);
        return GP_EINVAL;
    }
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        set_err("device %d is %s; libgossip_hip is built for gfx950 (MI355X) only", device, prop.gcnArchName);
        return GP_ENODEV;
    }
    return GP_OK;
}

// Slab boundaries: 3D / Imp3D whole x-planes (Program.fs:246-257 id = x g^2 + y g + z),
// line contiguous ids; full topology is single-rank.
int make_bounds(gp_sim* s) {
    const int W = s->world;
    s->bounds.assign(W + 1, 0);
    const int topo = s->cfg.topology;
    if (W == 1) {
        s->bounds[1] = (uint32_t)s->P;
        s->halo = 0;
        return GP_OK;
    }
    if (W > XMAXW) {
        set_err("at most %d ranks are supported (got %d)", XMAXW, W);
        return GP_EINVAL;
    }
    if (topo == GP_FULL) {  // contiguous ids, no halo: every message goes through the exchange
        if (s->P < W) {
            set_err("full topology with %lld nodes cannot be split over %d ranks", (long long)s->P, W);
            return GP_EINVAL;
        }
        for (int w = 0; w <= W; ++w) s->bounds[w] = (uint32_t)(s->P * w / W);
        s->halo = 0;
    } else if (topo == GP_LINE) {
        if (s->P < W) {
            set_err("line with %lld nodes cannot be split over %d ranks", (long long)s->P, W);
            return GP_EINVAL;
        }
        for (int w = 0; w <= W; ++w) s->bounds[w] = (uint32_t)(s->P * w / W);
        s->halo = 1;
    } else {
        if (s->g < W) {
            set_err("a %lld^3 lattice has fewer planes than ranks (%d)", (long long)s->g, W);
            return GP_EINVAL;
        }
        for (int w = 0; w <= W; ++w) s->bounds[w] = (uint32_t)((s->g * w / W) * s->g * s->g);
        s->halo = (uint32_t)(s->g * s->g);
    }
    return GP_OK;
}

// Imp3D gossip on the column kernel: random-edge deliveries are counted by their
// senders (rq) and cross ranks as counts; no bitmap, in-edge tags or slots.
bool col_gossip_counts(const DevState& S) { return S.topo == IMP3D && S.alg == GOSSIP && S.kernel == KERNEL_COL; }

// Device state of slab `r` (rank r): ids [bounds[r], bounds[r+1]) plus halos.
int alloc_slab(gp_sim* s, Slab& sl, int r) {
    DevState& S = sl.S;
    const int W = s->world;
    sl.rank = r;
    const uint32_t lo = s->bounds[r], hi = s->bounds[r + 1];
    sl.hi = hi;
    S.topo = s->cfg.topology;
    S.alg = s->cfg.algorithm;
    S.G.P = (uint32_t)s->P;
    S.G.T = (uint32_t)s->T;
    S.G.g = (uint32_t)s->g;
    S.G.g2 = (uint32_t)(s->g * s->g);
    S.G.div_g = make_fastdiv(S.G.g ? S.G.g : 1);
    S.G.div_g2 = make_fastdiv(S.G.g2 ? S.G.g2 : 1);
    S.k0 = (uint32_t)s->cfg.seed;
    S.k1 = (uint32_t)(s->cfg.seed >> 32);
    // choice = Random().Next(0, nodes) (Program.fs:193,221,263)
    S.seed_node = uniform(S.k0, S.k1, S_START, 0, 0, (uint32_t)s->T);
    S.lo = lo;
    S.nloc = hi - lo;
    S.ext_lo = r > 0 ? lo - s->halo : lo;
    S.ext_hi = r < W - 1 ? hi + s->halo : hi;
    S.base = S.ext_lo & ~3u;  // 4-aligned: the tile kernels move node bytes as words
    S.rtag = nullptr;
    S.rmsg = nullptr;
    S.rk = nullptr;
    S.rtg = nullptr;
    S.sbits = nullptr;
    S.xhdr[0] = S.xhdr[1] = nullptr;
    S.xvals[0] = S.xvals[1] = nullptr;
    S.xnv = 0;
    int rc;
    const size_t next = (size_t)(S.ext_hi - S.base) + 1024;  // node arrays (+ word-I/O padding)
    const size_t nl = S.nloc;
    if ((rc = dev_alloc_t(s, &S.ctl, 1))) return rc;
    if ((rc = dev_alloc_t(s, &S.tq, 2 * 8 * TQ_STRIDE))) return rc;
    HIP_TRY(hipMemsetAsync(S.tq, 0, sizeof(uint32_t) * 2 * 8 * TQ_STRIDE, s->stream));
    if (S.alg == PUSHSUM) {
        if ((rc = dev_alloc_t(s, &S.sw[0], next)) || (rc = dev_alloc_t(s, &S.sw[1], next)) ||
            (rc = dev_alloc_t(s, &S.nb[0], next)))
            return rc;
        if (S.topo != FULL && (rc = dev_alloc_t(s, &S.nb[1], next))) return rc;
        // zero sentinel just past the ids the slab holds: the tile kernels gather it for
        // lattice directions without a sender (never written by any round)
        for (int bb = 0; bb < 2; ++bb)
            HIP_TRY(hipMemsetAsync(S.sw[bb] + (S.ext_hi - S.base), 0, sizeof(double2), s->stream));
    } else {
        if ((rc = dev_alloc_t(s, &S.c, nl))) return rc;
        if (S.topo == FULL) {
            if ((rc = dev_alloc_t(s, &S.inc, nl))) return rc;
        } else {
            if ((rc = dev_alloc_t(s, &S.nb[0], next)) || (rc = dev_alloc_t(s, &S.nb[1], next))) return rc;
            S.nchunks = (uint32_t)((s->T + INJ_CHUNK - 1) / INJ_CHUNK);
            if ((rc = dev_alloc_t(s, &S.live_bits, (size_t)S.nchunks * (INJ_CHUNK / 32))) ||
                (rc = dev_alloc_t(s, &S.chunk_live, S.nchunks)))
                return rc;
        }
    }
    if (S.topo == FULL && S.alg == PUSHSUM) {  // LDS-binned message staging of this rank's receivers (gp_fullbin.hip)
        const FullBinPlan fp = full_bin_plan(S.nloc, W == 1);
        S.fb_nb2 = fp.nb2;
        S.fb_cap2 = fp.cap2;
        const size_t m2 = (size_t)fp.nb2 * fp.cap2;
        if ((rc = dev_alloc_t(s, &S.fb_cnt2, fp.nb2)) || (rc = dev_alloc_t(s, &S.fb_hdr2, m2)) ||
            (rc = dev_alloc_t(s, &S.fb_pay2, m2)))
            return rc;
        if (W == 1) {
            // one rank: coarse bins hdr1 / pay1; the fold of round r bins round r+1's messages
            // into them (k_fb_fold<FOLD_SEND>; GP_FB_FUSED=0, experiments: three passes)
            bool fused = true;
            if (const char* e = exp_env("GP_FB_FUSED")) fused = e[0] == '1';
            const FullBinPlan f1 = full_bin_plan(S.nloc, fused);
            S.fb_s1 = f1.s1;
            S.fb_nb1 = f1.nb1;
            S.fb_cap1 = f1.cap1;
            S.fb_fused = fused && f1.nb1 <= full_bin_fused_max_bins() ? 1u : 0u;
            const size_t m1 = (size_t)f1.nb1 * f1.cap1;
            // (+ FB_JUNK: the fold's write-out sends lanes without a message to the slots past the
            // last bin, so every thread issues the same number of stores)
            if ((rc = dev_alloc_t(s, &S.fb_cnt1, f1.nb1)) || (rc = dev_alloc_t(s, &S.fb_hdr1, m1 + FB_JUNK)) ||
                (rc = dev_alloc_t(s, &S.fb_pay1, m1 + FB_JUNK)))
                return rc;
        } else {
            // several ranks (round 6): the coarse bins are the exchange buffers (setup_exchange) --
            // the fold bins the next round's messages by destination rank and coarse bin into them,
            // and each rank's split reads them where they arrive (k_fb_fold<FOLD_SEND_RANKS>)
            S.fb_s1 = full_bin_multi_s1(s->bounds.data(), W);
            S.fb_nb1 = (uint32_t)(((uint64_t)S.nloc + (1ull << S.fb_s1) - 1) >> S.fb_s1);
            S.fb_cap1 = 0;
            S.fb_fused = 1;
            S.fb_cnt1 = S.fb_hdr1 = nullptr;
            S.fb_pay1 = nullptr;
        }
    }
    if (col_gossip_counts(S)) {  // senders count their random-edge deliveries at the target (k_gossip_col)
        // byte counters, four per word (C3: 0.632 -> 0.600 ms per round, reads 16.5 -> 11.7 and
        // writes 11.2 -> 9.8 B/node; profiles/r04/c3_byte_counters.txt)
        S.rq8 = 1;
        if (const char* e = exp_env("GP_RQ8")) S.rq8 = e[0] == '1' ? 1u : 0u;
        for (int q = 0; q < 2; ++q) {
            if ((rc = dev_alloc_t(s, &S.rq[q], (size_t)S.nloc + 64))) return rc;
            HIP_TRY(hipMemsetAsync(S.rq[q], 0, sizeof(uint32_t) * ((size_t)S.nloc + 64), s->stream));
        }
    }
    // random-edge bitmaps of the tile kernels (the column kernel counts deliveries instead)
    if (S.topo == IMP3D && !col_gossip_counts(S)) {
        S.rbits_words = rbits_words_for(S.lo, S.nloc);
        if ((rc = dev_alloc_t(s, &S.rbits[0], S.rbits_words)) || (rc = dev_alloc_t(s, &S.rbits[1], S.rbits_words)))
            return rc;
    }
    return GP_OK;
}

// Push-sum on a 3D / Imp3D lattice over several ranks: the halo planes' (s, w) travel compacted
// (only the senders toward the neighbour, HaloArgs in gp_xchg.hpp): C5 at W = 8, 16 MB -> 3.9 MB
// per direction and round.
int setup_halo(gp_sim* s) {
    s->halo_slots = 0;
    const bool lattice = s->cfg.topology == GP_3D || s->cfg.topology == GP_IMP3D;
    if (!lattice || s->cfg.algorithm != GP_PUSHSUM || s->world < 2 || s->halo < HALO_CHUNK) return GP_OK;
    s->halo_cap = halo_chunk_cap((uint32_t)s->g, s->cfg.topology == GP_IMP3D);
    s->halo_slots = halo_buf_slots(s->halo, s->halo_cap);
    int rc;
    for (Slab& sl : s->slab) {
        for (int k = 0; k < 2; ++k) {
            const bool has = k == 0 ? sl.rank > 0 : sl.rank < s->world - 1;
            if (!has) continue;
            if ((rc = dev_alloc_t(s, &sl.hsend[k], s->halo_slots)) || (rc = dev_alloc_t(s, &sl.hrecv[k], s->halo_slots)))
                return rc;
        }
    }
    return GP_OK;
}

// The halo planes' compacted (s, w) of buffers b: pack (the slab's first / last plane, before the
// transfer) or expand (into the halo planes, after it).  Lower side: the first plane's senders
// toward x - 1 (direction 0) go down; the lower halo takes the neighbour's senders toward x + 1
// (direction 1).  The upper side the other way round.
int halo_pack_expand(gp_sim* s, int b, bool pack, hipStream_t st) {
    const uint32_t H = s->halo;
    for (Slab& sl : s->slab) {
        DevState& S = sl.S;
        for (int k = 0; k < 2; ++k) {
            if (!sl.hsend[k]) continue;
            // plane start: pack -- lo (k = 0) / hi - H; expand -- lo - H (k = 0) / hi
            const uint32_t at = pack ? (k == 0 ? S.lo : sl.hi - H) : (k == 0 ? S.lo - H : sl.hi);
            HaloArgs h{};
            h.nb = S.nb[b] + (at - S.base);
            h.sw = S.sw[b] + (at - S.base);
            h.buf = pack ? sl.hsend[k] : sl.hrecv[k];
            h.n = H;
            h.cap = s->halo_cap;
            h.dir = pack ? (k == 0 ? 0u : 1u) : (k == 0 ? 1u : 0u);
            h.overflow = sl.overflow ? sl.overflow : &S.ctl->overflow;
            HIP_TRY(pack ? launch_halo_pack(h, st) : launch_halo_expand(h, st));
        }
    }
    return GP_OK;
}

constexpr int XREGIONS = 4;  // Imp3D push-sum exchange regions (see exchange_regions)
constexpr uint32_t RREG_MIN_NODES = 1u << 24;  // region rounds from this slab size on (round_regions)

// Exchange regions of a slab's senders: push-sum runs two (one's transfer overlaps the
// other's packing), gossip one.  Imp3D push-sum cuts them at a tile boundary (the lists'
// tiles); the full topology at a fine-tile boundary (full_region).
int exchange_regions(const gp_sim* s) {
    const bool push = s->cfg.algorithm == GP_PUSHSUM;
    // Imp3D push-sum lists: XREGIONS regions of the slab's tiles (the last one's transfer is what
    // the round cannot hide); the full topology's two halves.  Two ranks with large slabs: eight
    // regions, where one link carries half of every rank's messages -- C5, region rounds, same box
    // (profiles/r05/rregions/reg8.txt): W = 2 10.72 -> 10.21 ms at 128 GB/s, 12.53 -> 11.50 at
    // 64; at W = 4 and 8 eight were slower (5.50 -> 5.69, 2.82 -> 3.00 ms at 128 GB/s)
    int NH = push ? (s->cfg.topology == GP_IMP3D ? XREGIONS : FB_REGIONS) : 1;
    if (push && s->cfg.topology == GP_IMP3D && s->world == 2 && s->bounds.size() == 3 &&
        std::min(s->bounds[1] - s->bounds[0], s->bounds[2] - s->bounds[1]) >= RREG_MIN_NODES)
        NH = 8;
    static_assert(XMAXH >= 8 && RREG_MAX >= 8, "eight regions for two ranks");
    return NH;
}

// Round kernel launches per round (DevState::rregions).  Imp3D push-sum across ranks runs the
// round kernel region by region (launch_round_regions): region h's lists are packed and travel
// while the later regions compute.  C5 modelled from virtual ranks, same box, against one launch
// per round with the lists packed and sent after it (profiles/r05/rregions/): W = 2 12.92 ->
// 10.50 ms at 128 GB/s per link and direction, 17.97 -> 12.48 at 64; W = 4 5.46 -> 5.48 and
// 6.76 -> 5.81; W = 8 2.75 -> 2.74 and 2.96 -> 2.83 (the round kernel itself +2-5 %: four launch
// tails).  Small slabs (< RREG_MIN_NODES) move little and keep one launch per round: their rounds
// are launch-bound, and rank processes sharing one GPU (the tests) run them several times slower
// with four persistent launches per round.  The experiments build's GP_RREGIONS=0/1 overrides.
uint32_t round_regions(const gp_sim* s, int kernel, uint32_t walk) {
    if (s->world < 2 || s->cfg.topology != GP_IMP3D || s->cfg.algorithm != GP_PUSHSUM || kernel != KERNEL_TILE ||
        walk != 3)
        return 1;
    int on = 1;
    for (int w = 0; w < s->world; ++w)
        if (s->bounds[w + 1] - s->bounds[w] < RREG_MIN_NODES) on = 0;
    if (const char* e = exp_env("GP_RREGIONS")) on = std::atoi(e);
    const int NH = exchange_regions(s);
    if (!on || NH < 2 || NH > RREG_MAX) return 1;
    uint32_t rb[RREG_MAX + 1];
    for (int w = 0; w < s->world; ++w)
        if (!region_tiles(s->bounds[w], s->bounds[w + 1] - s->bounds[w], (uint64_t)s->g * s->g, NH, rb)) return 1;
    return (uint32_t)NH;
}

// Full-topology push-sum over several ranks: region h of NH of a slab is its fine tiles
// [t0, t1) (2^FB_TB local ids each, counted from lo) -- the fold of those tiles bins their
// next-round messages into region h's exchange buffers -- whose senders are the local ids
// [s0, s1).
void full_region(uint32_t nloc, int NH, int h, uint32_t& t0, uint32_t& t1, uint32_t& s0, uint32_t& s1) {
    const uint32_t nt = (uint32_t)(((uint64_t)nloc + (1u << FB_TB) - 1) >> FB_TB);
    t0 = (uint32_t)((uint64_t)nt * h / NH);
    t1 = (uint32_t)((uint64_t)nt * (h + 1) / NH);
    s0 = (uint32_t)std::min<uint64_t>(nloc, (uint64_t)t0 << FB_TB);
    s1 = (uint32_t)std::min<uint64_t>(nloc, (uint64_t)t1 << FB_TB);
}

uint32_t slab_tiles(uint32_t lo, uint32_t nloc) {
    return (uint32_t)(((uint64_t)lo + nloc + XTILE - 1) / XTILE - lo / XTILE);
}

// Local sender ids [s_lo, s_hi) of region h.
void xregion(const Slab& sl, int NH, int h, uint32_t& s_lo, uint32_t& s_hi) {
    const DevState& S = sl.S;
    uint32_t split = S.nloc / 2;
    if (sl.lists) {  // tiles [tb[h], tb[h + 1])
        auto at = [&](uint32_t t) {
            const int64_t b = (int64_t)(S.lo / XTILE + t) * XTILE - S.lo;
            return (uint32_t)std::min<int64_t>(S.nloc, std::max<int64_t>(0, b));
        };
        s_lo = at(sl.tb[h]);
        s_hi = h + 1 == NH ? S.nloc : at(sl.tb[h + 1]);
        return;
    }
    s_lo = NH == 1 || h == 0 ? 0u : split;
    s_hi = NH == 1 || h == 1 ? S.nloc : split;
}

// Header-word offset of chunk (h, a) in rank b's header region, and slot offset of chunk
// (h, a) in b's vals region: chunks in (h, a) order, a != b (every rank lays out its
// receive buffer this way, and every sender addresses it this way).
uint32_t list_hw(const gp_sim* s, int b, int h, int a) {
    const int W = s->world, NH = s->xhalves;
    uint64_t o = 0;
    for (int hh = 0; hh < NH; ++hh)
        for (int aa = 0; aa < W; ++aa) {
            if (aa == b) continue;
            if (hh == h && aa == a) return (uint32_t)o;
            o += s->list_nw[((size_t)aa * NH + hh) * W + b];
        }
    return (uint32_t)o;
}

// Imp3D push-sum over several ranks: the static list plan (gp_xchg.hpp) of every slab
// from the global random edges, the header-word counts of every chunk, and for this
// rank's slabs the tile table gw and every remote in-edge's list key (rk).  kk: a
// P-word scratch array; src: senders in receiver order (global); edge0: first global
// in-edge of every rank.
int build_lists(gp_sim* s, const uint32_t* rnd_all, uint32_t* kk, const uint32_t* src,
                const std::vector<uint32_t>& edge0) {
    const int W = s->world;
    const int NH = s->xhalves = exchange_regions(s);
    s->list_nw.assign((size_t)W * NH * W, 0);
    std::vector<std::vector<uint32_t>> gw_all(W);
    std::vector<std::vector<uint8_t>> lwt_all(W);
    std::vector<std::array<uint32_t, XMAXH + 1>> tb(W);  // per slab: region tile boundaries
    Scratch tmp_mem;
    for (int a = 0; a < W; ++a) {
        const uint32_t lo = s->bounds[a], nloc = s->bounds[a + 1] - lo;
        const uint32_t nt = slab_tiles(lo, nloc);
        // regions of whole planes (region_tiles: the round kernel's regions when it runs region by
        // region), else of equal tile counts
        if (!region_tiles(lo, nloc, (uint64_t)s->g * s->g, NH, tb[a].data()))
            for (int h = 0; h <= NH; ++h) tb[a][h] = (uint32_t)((uint64_t)nt * h / NH);
        for (int h = NH + 1; h <= XMAXH; ++h) tb[a][h] = nt;
        uint32_t* cnt = nullptr;
        HIP_TRY(tmp_mem.alloc(&cnt, (size_t)nt * W + 1));
        ListCountArgs ca{};
        ca.rnd = rnd_all;
        ca.lo = lo;
        ca.nloc = nloc;
        ca.W = W;
        ca.a = a;
        for (int w = 0; w <= W; ++w) ca.bounds[w] = s->bounds[w];
        ca.cnt = cnt;
        HIP_TRY(launch_list_count(ca, s->stream));
        std::vector<uint32_t> hc((size_t)nt * W);
        HIP_TRY(hipMemcpyAsync(hc.data(), cnt, sizeof(uint32_t) * hc.size(), hipMemcpyDeviceToHost, s->stream));
        HIP_TRY(hipStreamSynchronize(s->stream));
        std::vector<uint32_t>& gw = gw_all[a];
        gw.assign((size_t)nt * W, 0);
        std::vector<uint8_t>& lwt = lwt_all[a];  // per tile: prefix over d of its segments' words
        lwt.assign((size_t)nt * (W + 1), 0);
        for (uint32_t t = 0; t < nt; ++t) {
            uint32_t w = 0;
            for (int d = 0; d < W; ++d) {
                lwt[(size_t)t * (W + 1) + d] = (uint8_t)w;
                w += (hc[(size_t)t * W + d] + 63u) / 64u;
            }
            lwt[(size_t)t * (W + 1) + W] = (uint8_t)w;  // <= 16 + W words
        }
        for (int d = 0; d < W; ++d) {
            uint64_t run[XMAXH] = {};
            for (uint32_t t = 0, h = 0; t < nt; ++t) {
                while ((int)h + 1 < NH && t >= tb[a][h + 1]) ++h;
                gw[(size_t)t * W + d] = (uint32_t)run[h];
                run[h] += (hc[(size_t)t * W + d] + 63u) / 64u;
            }
            for (int h = 0; h < NH; ++h) {
                if (run[h] >= (1ull << 26)) {
                    set_err("internal: random-edge list %d -> %d has %llu header words (limit 2^26)", a, d,
                            (unsigned long long)run[h]);
                    return GP_EINVAL;
                }
                s->list_nw[((size_t)a * NH + h) * W + d] = (uint32_t)run[h];
            }
        }
    }
    // every sender's key at its destination, then this rank's in-edges' keys
    for (int a = 0; a < W; ++a) {
        const uint32_t lo = s->bounds[a], nloc = s->bounds[a + 1] - lo;
        uint32_t* gw = nullptr;
        HIP_TRY(tmp_mem.alloc(&gw, gw_all[a].size() + 1));
        HIP_TRY(hipMemcpyAsync(gw, gw_all[a].data(), sizeof(uint32_t) * gw_all[a].size(), hipMemcpyHostToDevice,
                               s->stream));
        ListKeyArgs ka{};
        ka.rnd = rnd_all;
        ka.gw = gw;
        ka.lo = lo;
        ka.nloc = nloc;
        for (int h = 0; h <= XMAXH; ++h) ka.tb[h] = tb[a][h];
        ka.NH = NH;
        ka.W = W;
        ka.a = a;
        for (int w = 0; w <= W; ++w) ka.bounds[w] = s->bounds[w];
        for (int h = 0; h < NH; ++h)
            for (int b = 0; b < W; ++b) ka.hw[h][b] = b == a ? 0u : list_hw(s, b, h, a);
        ka.key = kk;
        ka.xdr = nullptr;
        for (Slab& sl : s->slab) {
            if (sl.rank != a) continue;
            int rc;
            if ((rc = dev_alloc_t(s, &sl.xdr, (size_t)nloc + 64))) return rc;
            ka.xdr = sl.xdr;
        }
        HIP_TRY(launch_list_key(ka, s->stream));
        HIP_TRY(hipStreamSynchronize(s->stream));  // (gw is freed at scope end; keep it simple)
    }
    int rc;
    for (Slab& sl : s->slab) {
        DevState& S = sl.S;
        const int r = sl.rank;
        sl.lists = true;
        sl.nt = slab_tiles(S.lo, S.nloc);
        for (int h = 0; h <= XMAXH; ++h) sl.tb[h] = tb[r][h];
        if ((rc = dev_alloc_t(s, &sl.gw, gw_all[r].size() + 1)) || (rc = dev_alloc_t(s, &sl.lwt, lwt_all[r].size() + 16)))
            return rc;
        HIP_TRY(hipMemcpyAsync(sl.gw, gw_all[r].data(), sizeof(uint32_t) * gw_all[r].size(), hipMemcpyHostToDevice,
                               s->stream));
        HIP_TRY(hipMemcpyAsync(sl.lwt, lwt_all[r].data(), lwt_all[r].size(), hipMemcpyHostToDevice, s->stream));
        const uint32_t ne = edge0[r + 1] - edge0[r];
        if ((rc = dev_alloc_t(s, &S.rk, (size_t)ne + 4))) return rc;
        HIP_TRY(launch_gather_keys(kk, src + edge0[r], ne, S.rk, s->grid, s->stream));

    }
    HIP_TRY(hipStreamSynchronize(s->stream));
    return GP_OK;
}

// Imp3D gossip on the column kernel over several ranks: the bitmap plan (gp_xchg.hpp).
// For every source slab a, the edges with a sender on a get their rank among the
// same receiver slab's edges from a (exclusive scan of a flag over the global
// receiver order); this rank's senders learn their bit (rtg) and its receivers
// the target of every received bit (tgt).  flag / scan / pos: P + 1 words of scratch.
int build_bits(gp_sim* s, const uint32_t* src, const uint32_t* recv, const uint32_t* inv,
               const std::vector<uint32_t>& edge0, uint32_t* flag, uint32_t* scan, uint32_t* pos) {
    const int W = s->world;
    const uint32_t P = (uint32_t)s->P;
    Scratch tmp_mem;
    size_t scan_bytes = 0;
    HIP_TRY(exclusive_scan_u32(nullptr, scan_bytes, flag, scan, P + 1, s->stream));
    uint8_t* scan_tmp = nullptr;
    HIP_TRY(tmp_mem.alloc(&scan_tmp, scan_bytes ? scan_bytes : 4));
    std::vector<std::vector<uint32_t>> n(W, std::vector<uint32_t>(W, 0));  // edges a -> b
    for (int a = 0; a < W; ++a) {
        HIP_TRY(launch_src_flag(src, P, s->bounds.data(), W, a, flag, s->grid, s->stream));
        HIP_TRY(exclusive_scan_u32(scan_tmp, scan_bytes, flag, scan, P + 1, s->stream));
        BitsSetupArgs ba{};
        ba.src = src;
        ba.recv = recv;
        ba.scan = scan;
        ba.pos = pos;
        ba.n = P;
        ba.W = W;
        ba.a = a;
        for (int w = 0; w <= W; ++w) {
            ba.bounds[w] = s->bounds[w];
            ba.edge0[w] = edge0[w];
        }
        HIP_TRY(launch_bits_pos(ba, s->grid, s->stream));
        std::vector<uint32_t> at(W + 1);
        for (int b = 0; b <= W; ++b)
            HIP_TRY(hipMemcpyAsync(&at[b], scan + edge0[b], sizeof(uint32_t), hipMemcpyDeviceToHost, s->stream));
        HIP_TRY(hipStreamSynchronize(s->stream));
        for (int b = 0; b < W; ++b) n[a][b] = a == b ? 0u : at[b + 1] - at[b];
    }
    auto pad = [](uint64_t x) { return (x + BITS_ALIGN - 1) / BITS_ALIGN * BITS_ALIGN; };
    int rc;
    for (Slab& sl : s->slab) {
        DevState& S = sl.S;
        const int me = sl.rank;
        sl.bits = true;
        sl.bo.assign(W, 0);
        sl.bn.assign(W, 0);
        sl.ro.assign(W, 0);
        sl.rn.assign(W, 0);
        uint64_t so = 0, ri = 0;
        for (int d = 0; d < W; ++d) {
            if (d == me) continue;
            sl.bo[d] = (uint32_t)so;
            sl.bn[d] = n[me][d];
            so += pad(n[me][d]);
            sl.ro[d] = (uint32_t)ri;
            sl.rn[d] = n[d][me];
            ri += pad(n[d][me]);
        }
        if (so >= (1ull << 31) || ri >= (1ull << 31)) {
            set_err("internal: random-edge bitmaps beyond 2^31 bits");
            return GP_EINVAL;
        }
        sl.nbits_out = (uint32_t)so;
        sl.nbits_in = (uint32_t)ri;
        if ((rc = dev_alloc_t(s, &S.rtg, (size_t)S.nloc + 64)) || (rc = dev_alloc_t(s, &S.sbits, so / 32 + 1)) ||
            (rc = dev_alloc_t(s, &sl.rbits_in, ri / 32 + 1)) || (rc = dev_alloc_t(s, &sl.tgt, ri + 1)))
            return rc;
        HIP_TRY(hipMemsetAsync(S.sbits, 0, (so / 32 + 1) * 4, s->stream));
        HIP_TRY(hipMemsetAsync(sl.rbits_in, 0, (ri / 32 + 1) * 4, s->stream));
        BitsEndsArgs ea{};
        ea.rnd = S.rnd;
        ea.inv = inv;
        ea.src = src;
        ea.recv = recv;
        ea.pos = pos;
        ea.rtg = S.rtg;
        ea.tgt = sl.tgt;
        ea.lo = S.lo;
        ea.nloc = S.nloc;
        ea.e0 = edge0[me];
        ea.e1 = edge0[me + 1];
        ea.W = W;
        ea.me = me;
        for (int w = 0; w <= W; ++w) ea.bounds[w] = s->bounds[w];
        for (int w = 0; w < W; ++w) {
            ea.bo[w] = sl.bo[w];
            ea.ro[w] = sl.ro[w];
        }
        HIP_TRY(launch_bits_ends(ea, s->grid, s->stream));
    }
    HIP_TRY(hipStreamSynchronize(s->stream));
    return GP_OK;
}

// Imp3D: draw rnd[] for every node (Program.fs:258-260), then a stable sort of
// (key(rnd[i]), i) by key gives every receiver's senders in ascending id order,
// and the exclusive scan of the per-receiver in-degrees the CSR offsets (in_off,
// in_src in id order).  Every rank builds the global order (it is
// deterministic; ranks own consecutive id ranges) and keeps its
// receivers' slice; with several ranks, each local sender also learns the
// position of its message in the destination's in-edge array (pos).

int build_imp3d(gp_sim* s) {
    const uint32_t P = (uint32_t)s->P;
    const int W = s->world;
    DevState& S0 = s->slab[0].S;
    Scratch tmp_mem;  // setup temporaries, freed on every exit path
    uint32_t *rnd_all = nullptr, *iota = nullptr, *keys_sorted = nullptr, *src_sorted = nullptr, *counts = nullptr,
             *off_all = nullptr, *inv = nullptr;
    const uint64_t nkeys = P;
    HIP_TRY(tmp_mem.alloc(&rnd_all, P));
    HIP_TRY(tmp_mem.alloc(&iota, P));
    HIP_TRY(tmp_mem.alloc(&keys_sorted, P));
    HIP_TRY(tmp_mem.alloc(&src_sorted, P));
    HIP_TRY(tmp_mem.alloc(&counts, (size_t)nkeys + 1));
    HIP_TRY(tmp_mem.alloc(&off_all, (size_t)nkeys + 1));
    HIP_TRY(launch_topo_rnd_range(S0.k0, S0.k1, P, 0, P, rnd_all, s->grid, s->stream));
    HIP_TRY(launch_iota(iota, P, s->grid, s->stream));
    const uint32_t bits = bits_for(nkeys > 1 ? nkeys - 1 : 0);
    size_t tmp_bytes = 0;
    HIP_TRY(sort_pairs(nullptr, tmp_bytes, rnd_all, keys_sorted, iota, src_sorted, P, bits, s->stream));
    uint8_t* tmp = nullptr;
    HIP_TRY(tmp_mem.alloc(&tmp, tmp_bytes ? tmp_bytes : 4));
    HIP_TRY(sort_pairs(tmp, tmp_bytes, rnd_all, keys_sorted, iota, src_sorted, P, bits, s->stream));
    HIP_TRY(hipMemsetAsync(counts, 0, sizeof(uint32_t) * ((size_t)nkeys + 1), s->stream));
    HIP_TRY(launch_histogram(rnd_all, P, counts, s->grid, s->stream));
    size_t scan_bytes = 0;
    HIP_TRY(exclusive_scan_u32(nullptr, scan_bytes, counts, off_all, (uint32_t)nkeys + 1, s->stream));
    uint8_t* scan_tmp = nullptr;
    HIP_TRY(tmp_mem.alloc(&scan_tmp, scan_bytes ? scan_bytes : 4));
    HIP_TRY(exclusive_scan_u32(scan_tmp, scan_bytes, counts, off_all, (uint32_t)nkeys + 1, s->stream));
    if (W > 1) {
        HIP_TRY(tmp_mem.alloc(&inv, P));
        HIP_TRY(launch_inverse(src_sorted, P, inv, s->grid, s->stream));
    }
    // first global edge of every rank
    std::vector<uint32_t> edge0(W + 1);
    for (int w = 0; w <= W; ++w)
        HIP_TRY(hipMemcpyAsync(&edge0[w], off_all + s->bounds[w], sizeof(uint32_t), hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    int rc;
    for (Slab& sl : s->slab) {
        DevState& S = sl.S;
        const int r = sl.rank;
        const uint32_t ne = edge0[r + 1] - edge0[r];
        sl.nedges = ne;
        S.nedges = ne;
        if ((rc = dev_alloc_t(s, &S.rnd, S.nloc))) return rc;
        HIP_TRY(hipMemcpyAsync(S.rnd, rnd_all + S.lo, sizeof(uint32_t) * S.nloc, hipMemcpyDeviceToDevice, s->stream));
        // in-lists padded by 4 words: the tile kernels stage them with 16-byte LDS-DMA
        if ((rc = dev_alloc_t(s, &S.in_off, (size_t)S.nloc + 1 + 4)) ||
            (rc = dev_alloc_t(s, &S.in_src, (size_t)ne + 4)))
            return rc;
        HIP_TRY(hipMemcpyAsync(S.in_off, off_all + S.lo, sizeof(uint32_t) * ((size_t)S.nloc + 1),
                               hipMemcpyDeviceToDevice, s->stream));
        HIP_TRY(launch_sub(S.in_off, S.nloc + 1, edge0[r], s->grid, s->stream));
        if (ne)
            HIP_TRY(hipMemcpyAsync(S.in_src, src_sorted + edge0[r], sizeof(uint32_t) * ne,
                                   hipMemcpyDeviceToDevice, s->stream));
        S.in_srcd = nullptr;
        bool pack = true;
        if (const char* np = exp_env("GP_NO_PACK")) pack = np[0] != '1';  // force the unpacked (P > 2^30) path
        if (S.alg == PUSHSUM && S.kernel == KERNEL_TILE && s->P <= (1ll << 30) && s->g >= 2 && pack) {
            if ((rc = dev_alloc_t(s, &S.in_srcd, (size_t)ne + 4))) return rc;
            if (ne) HIP_TRY(launch_pack_src_deg(S.in_src, S.in_srcd, ne, S.G, s->grid, s->stream));
        }
        S.ind4 = nullptr;
        if (S.alg == PUSHSUM && S.kernel == KERNEL_TILE) {
            if ((rc = dev_alloc_t(s, &S.ind4, ind4_bytes_for(S.lo, S.nloc)))) return rc;
            uint32_t wide_at = 15;  // in-degree >= 15: the tile reads in_off (gp_round.hip)
            if (const char* e = exp_env("GP_IND4_WIDE")) wide_at = (uint32_t)std::max(1, std::atoi(e));
            HIP_TRY(launch_pack_ind4(S, wide_at, s->grid, s->stream));
        }
        if (W > 1 && !col_gossip_counts(S)) {  // (the gossip column kernel's bitmaps: build_bits)
            // push-sum: sender-ordered lists (build_lists), no slots or tags; gossip tile kernel:
            // {slot} entries and round tags (k_pack / k_unpack)
            const bool slots = S.alg != PUSHSUM;
            if ((rc = dev_alloc_t(s, &sl.xdst, (size_t)S.nloc + 64))) return rc;
            if (slots && ((rc = dev_alloc_t(s, &sl.pos, S.nloc)) || (rc = dev_alloc_t(s, &S.rtag, ne))))
                return rc;
            if (slots) HIP_TRY(hipMemsetAsync(S.rtag, 0xFF, sizeof(uint32_t) * (ne ? ne : 1), s->stream));
            PosArgs pa{};
            pa.rnd = S.rnd;
            pa.inv = inv;
            pa.pos = slots ? sl.pos : nullptr;
            pa.xdst = sl.xdst;
            pa.lo = S.lo;
            pa.nloc = S.nloc;
            pa.W = W;
            pa.me = r;
            for (int w = 0; w <= W; ++w) pa.bounds[w] = s->bounds[w];
            for (int w = 0; w < W; ++w) pa.edge0[w] = edge0[w];
            HIP_TRY(launch_make_pos(pa, s->grid, s->stream));
        }
    }
    // (iota, the sort's value input, is free again: the lists' key scratch)
    if (W > 1 && s->cfg.algorithm == GP_PUSHSUM && (rc = build_lists(s, rnd_all, iota, src_sorted, edge0))) return rc;
    // (counts, off_all -- copied into the slabs' in_off -- and iota are free again: the bitmaps'
    // scratch, in stream order after those copies)
    if (W > 1 && col_gossip_counts(S0) && (rc = build_bits(s, src_sorted, keys_sorted, inv, edge0, counts, off_all, iota)))
        return rc;
    HIP_TRY(hipStreamSynchronize(s->stream));
    return GP_OK;
}

int finalize(gp_sim* s, uint32_t round_done, uint32_t round_next);

// Fixed-capacity exchange buffers per rank pair: capacity = expected messages
// per round + 12 sigma + 64 (never more than the pair's random edges).  Push-sum
// exchanges have two regions per pair, one per half of the sender's senders
// (s->xhalves), moved separately on the exchange stream so that one half's
// transfer overlaps the other half's packing / unpacking (full topology:
// launch_round_full_multi; Imp3D: exchange).
int setup_exchange(gp_sim* s) {
    const int W = s->world;
    const bool push = s->cfg.algorithm == GP_PUSHSUM;
    const bool full = s->cfg.topology == GP_FULL;
    if (!s->slab.empty() && s->slab[0].bits) {  // gossip column kernel: fixed-size bitmaps (build_bits)
        s->xhalves = 1;
        for (Slab& sl : s->slab) sl.overflow = &sl.S.ctl->overflow;
        return GP_OK;
    }
    const int NH = exchange_regions(s);
    s->xhalves = NH;
    std::vector<uint32_t> caps((size_t)NH * W * W, 0);  // caps[(h * W + a) * W + b]: a -> b, region h
    Scratch tmp_mem;
    double* mu = nullptr;
    unsigned long long* n = nullptr;
    HIP_TRY(tmp_mem.alloc(&mu, XMAXW));
    HIP_TRY(tmp_mem.alloc(&n, XMAXW));
    // full push-sum: the coarse bins of every destination travel as the exchange buffers
    // (FbBins, gp_fullbin.hpp); the coarse-bin size every rank uses, and a rank's bin count
    const uint32_t fs1 = full && push ? full_bin_multi_s1(s->bounds.data(), W) : 0;
    auto fnb = [&](int b) { return (uint32_t)(((uint64_t)s->bounds[b + 1] - s->bounds[b] + (1ull << fs1) - 1) >> fs1); };
    if (full) {
        // every active sender picks a uniform target among P-1: a function of the slab bounds
        // only, so every rank computes the whole table
        for (int a = 0; a < W; ++a) {
            const uint32_t na = s->bounds[a + 1] - s->bounds[a];
            for (int h = 0; h < NH; ++h) {
                uint32_t t0, t1, s0, s1;
                full_region(na, NH, h, t0, t1, s0, s1);
                const double nah = (double)(s1 - s0);
                for (int b = 0; b < W; ++b) {
                    if (push) {
                        // push-sum: messages from a's region h to one coarse bin of b (2^fs1
                        // receivers; a rank's messages to itself included, they pass through its
                        // own receive buffer) are at most Binomial(na_h, 2^fs1 / (P-1))
                        caps[((size_t)h * W + a) * W + b] = full_bin_multi_cap(s1 - s0, fs1, (uint32_t)s->P);
                        continue;
                    }
                    // gossip: messages a -> b at most Binomial(na, nb / (P-1))
                    if (b == a) continue;
                    const double nb = (double)(s->bounds[b + 1] - s->bounds[b]);
                    const double m = nah * nb / (double)(s->P - 1);
                    const double c = std::ceil(m + 12.0 * std::sqrt(m) + 64.0);
                    caps[((size_t)h * W + a) * W + b] = (uint32_t)std::min(c, nah);
                }
            }
        }
    }
    for (Slab& sl : s->slab) {
        if (full) break;
        DevState& S = sl.S;
        for (int h = 0; h < NH; ++h) {  // region h: senders [s_lo, s_hi) of the slab (xhalf_range)
            HIP_TRY(hipMemsetAsync(mu, 0, sizeof(double) * XMAXW, s->stream));
            HIP_TRY(hipMemsetAsync(n, 0, sizeof(unsigned long long) * XMAXW, s->stream));
            ExpectArgs ea{};
            ea.rnd = S.rnd;
            ea.lo = S.lo;
            ea.nloc = S.nloc;
            xregion(sl, NH, h, ea.s_lo, ea.s_hi);
            ea.W = W;
            ea.me = sl.rank;
            for (int w = 0; w <= W; ++w) ea.bounds[w] = s->bounds[w];
            ea.G = S.G;
            ea.mu = mu;
            ea.n = n;
            HIP_TRY(launch_expect(ea, s->grid, s->stream));
            double hmu[XMAXW];
            unsigned long long hn[XMAXW];
            HIP_TRY(hipMemcpyAsync(hmu, mu, sizeof hmu, hipMemcpyDeviceToHost, s->stream));
            HIP_TRY(hipMemcpyAsync(hn, n, sizeof hn, hipMemcpyDeviceToHost, s->stream));
            HIP_TRY(hipStreamSynchronize(s->stream));
            for (int b = 0; b < W; ++b) {
                if (b == sl.rank || hn[b] == 0) continue;
                const double c = std::ceil(hmu[b] + 12.0 * std::sqrt(hmu[b]) + 64.0);
                caps[((size_t)h * W + sl.rank) * W + b] = (uint32_t)std::min<double>(c, (double)hn[b]);
            }
        }
    }
    if (const char* e = exp_env("GP_XCAP")) {  // tests: force tiny buffers (overflow handling)
        const uint32_t cap = (uint32_t)std::max(1, std::atoi(e));
        for (auto& c : caps) c = std::min(c, cap);
    }
    if (s->mode == MODE_RCCL && !full) {
        // every rank learns the capacities of the buffers it will receive (per region)
        uint32_t* d = nullptr;
        HIP_TRY(tmp_mem.alloc(&d, (size_t)W * W));
        for (int h = 0; h < NH; ++h) {
            uint32_t* row = caps.data() + (size_t)h * W * W;
            HIP_TRY(hipMemcpyAsync(d + (size_t)s->rank * W, row + (size_t)s->rank * W, sizeof(uint32_t) * W,
                                   hipMemcpyHostToDevice, s->stream));
            NCCL_TRY(ncclAllGather(d + (size_t)s->rank * W, d, W, ncclUint32, s->comm, s->stream));
            HIP_TRY(hipMemcpyAsync(row, d, sizeof(uint32_t) * W * W, hipMemcpyDeviceToHost, s->stream));
            HIP_TRY(hipStreamSynchronize(s->stream));
        }
    }
    int rc;
    if (!s->slab.empty() && s->slab[0].lists) {  // Imp3D push-sum: sender-ordered lists (gp_xchg.hpp)
        auto cap = [&](int h, int a, int b) { return caps[((size_t)h * W + a) * W + b]; };
        auto nw = [&](int h, int a, int b) { return s->list_nw[((size_t)a * NH + h) * W + b]; };
        // slot offset of chunk (h, a) in rank b's vals region (the order of list_hw)
        auto vo = [&](int b, int h, int a) {
            uint64_t o = 0;
            for (int hh = 0; hh < NH; ++hh)
                for (int aa = 0; aa < W; ++aa) {
                    if (aa == b) continue;
                    if (hh == h && aa == a) return o;
                    o += cap(hh, aa, b);
                }
            return o;
        };
        for (Slab& sl : s->slab) {
            const int a = sl.rank;
            const size_t R = (size_t)NH * W;
            sl.cap_out.assign(R, 0);
            sl.cap_in.assign(R, 0);
            sl.lhdr.assign(R, 0);
            sl.lval.assign(R, 0);
            sl.rhdr.assign(R, 0);
            sl.rval.assign(R, 0);
            sl.vbase.assign(R, 0);
            size_t so = 0, hdr_in = 0;
            uint64_t nv_in = 0;
            for (int h = 0; h < NH; ++h)
                for (int b = 0; b < W; ++b) {
                    if (b == a) continue;
                    const size_t i = (size_t)h * W + b;
                    sl.cap_out[i] = cap(h, a, b);
                    sl.cap_in[i] = cap(h, b, a);
                    sl.lhdr[i] = so;
                    so += (size_t)nw(h, a, b) * 16;
                    sl.lval[i] = so;
                    so += (size_t)sl.cap_out[i] * 16;
                    sl.rhdr[i] = (size_t)list_hw(s, a, h, b) * 16;
                    hdr_in += (size_t)nw(h, b, a) * 16;
                    nv_in += sl.cap_in[i];
                    const uint64_t vb = vo(b, h, a);
                    if (vb >= (1ull << 32) || nv_in >= (1ull << 32)) {
                        set_err("internal: exchange vals region beyond 2^32 slots");
                        return GP_EINVAL;
                    }
                    sl.vbase[i] = (uint32_t)vb;
                }
            for (int h = 0; h < NH; ++h)
                for (int b = 0; b < W; ++b)
                    if (b != a) sl.rval[(size_t)h * W + b] = hdr_in + (size_t)vo(a, h, b) * 16;
            const size_t ro = hdr_in + (size_t)nv_in * 16;
            sl.xr_stride = sl.S.rregions > 1 ? (ro + 255) & ~(size_t)255 : 0;  // one buffer per round parity
            const size_t rt = sl.xr_stride ? 2 * sl.xr_stride : ro;
            if ((rc = dev_alloc_t(s, &sl.xsend, so)) || (rc = dev_alloc_t(s, &sl.xrecv, rt)) ||
                (rc = dev_alloc_t(s, &sl.xcnt, R)))
                return rc;
            HIP_TRY(hipMemsetAsync(sl.xsend, 0, so ? so : 16, s->stream));
            HIP_TRY(hipMemsetAsync(sl.xrecv, 0, rt ? rt : 16, s->stream));
            for (int k = 0; k < 2; ++k) {
                sl.S.xhdr[k] = reinterpret_cast<const XHdr*>(sl.xrecv + k * sl.xr_stride);
                sl.S.xvals[k] = reinterpret_cast<const double2*>(sl.xrecv + k * sl.xr_stride + hdr_in);
            }
            sl.S.xnv = (uint32_t)std::max<uint64_t>(1, nv_in);
            sl.overflow = &sl.S.ctl->overflow;
        }
    }
    for (Slab& sl : s->slab) {
        if (sl.lists) break;
        const int a = sl.rank;
        const size_t R = (size_t)NH * W;
        sl.cap_out.assign(R, 0);
        sl.cap_in.assign(R, 0);
        sl.soff.assign(R, 0);
        sl.sbytes.assign(R, 0);
        sl.roff.assign(R, 0);
        sl.rbytes.assign(R, 0);
        size_t so = 0, ro = 0;
        for (int h = 0; h < NH; ++h)
            for (int b = 0; b < W; ++b) {
                const size_t i = (size_t)h * W + b;
                sl.cap_out[i] = caps[((size_t)h * W + a) * W + b];
                sl.cap_in[i] = caps[((size_t)h * W + b) * W + a];
                sl.soff[i] = so;
                // (own messages: straight to xrecv; full push-sum: b's coarse bins, FbBins)
                sl.sbytes[i] = b == a ? 0 : full && push ? fb_bins_bytes(fnb(b), sl.cap_out[i]) : xbuf_bytes(sl.cap_out[i], push);
                so += sl.sbytes[i];
                sl.roff[i] = ro;
                sl.rbytes[i] = full && push ? fb_bins_bytes(fnb(a), sl.cap_in[i]) : xbuf_bytes(sl.cap_in[i], push);
                ro += sl.rbytes[i];
            }
        if ((rc = dev_alloc_t(s, &sl.xsend, so)) || (rc = dev_alloc_t(s, &sl.xrecv, ro))) return rc;
        HIP_TRY(hipMemsetAsync(sl.xsend, 0, so ? so : 16, s->stream));
        HIP_TRY(hipMemsetAsync(sl.xrecv, 0, ro ? ro : 16, s->stream));
        if (full && push) {  // the own share's second parity (Slab::xown)
            size_t oo = 0;
            for (int h = 0; h < NH && h < FB_REGIONS; ++h) {
                sl.ooff[h] = oo;
                oo += sl.rbytes[(size_t)h * W + a];
            }
            if ((rc = dev_alloc_t(s, &sl.xown, oo))) return rc;
            HIP_TRY(hipMemsetAsync(sl.xown, 0, oo ? oo : 16, s->stream));
        }
        sl.overflow = &sl.S.ctl->overflow;
    }
    if (NH > 1) {  // the second stream and the events that order it with the compute stream
        HIP_TRY(hipStreamCreateWithFlags(&s->xstream, hipStreamNonBlocking));
        for (int h = 0; h < NH; ++h) {
            HIP_TRY(hipEventCreateWithFlags(&s->ev_send[h], hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&s->ev_xfer[h], hipEventDisableTiming));
        }
    }
    return GP_OK;
}

// Move region h of every rank's exchange buffers to their destinations on
// stream st (device copies for in-process ranks, one RCCL group otherwise).
int transfer_xbufs(gp_sim* s, int h, hipStream_t st) {
    const int W = s->world;
    if (s->mode == MODE_VIRTUAL) {
        for (Slab& a : s->slab)
            for (Slab& d : s->slab) {
                const size_t i = (size_t)h * W + d.rank, j = (size_t)h * W + a.rank;
                if (&a != &d && a.sbytes[i])
                    HIP_TRY(hipMemcpyAsync(d.xrecv + d.roff[j], a.xsend + a.soff[i], a.sbytes[i],
                                           hipMemcpyDeviceToDevice, st));
            }
        return GP_OK;
    }
    Slab& sl = s->slab[0];
    NCCL_TRY(ncclGroupStart());
    for (int p = 0; p < W; ++p) {
        if (p == sl.rank) continue;
        const size_t i = (size_t)h * W + p;
        if (sl.sbytes[i]) NCCL_TRY(ncclSend(sl.xsend + sl.soff[i], sl.sbytes[i], ncclUint8, p, s->comm, st));
        if (sl.rbytes[i]) NCCL_TRY(ncclRecv(sl.xrecv + sl.roff[i], sl.rbytes[i], ncclUint8, p, s->comm, st));
    }
    NCCL_TRY(ncclGroupEnd());
    return GP_OK;
}

FullArgs make_full_args(gp_sim* s, Slab& sl, uint32_t round) {
    DevState& S = sl.S;
    const int cur = round & 1;
    const bool push = S.alg == PUSHSUM;
    const uint32_t d = S.lo - S.base;  // node arrays start at `base`; index these by id - lo
    FullArgs a{};
    a.nb = push ? S.nb[0] + d : nullptr;
    a.swc = push ? S.sw[cur] + d : nullptr;
    a.swn = push ? S.sw[cur ^ 1] + d : nullptr;
    a.c = S.c;
    a.inc = S.inc;
    a.ctl = S.ctl;
    a.overflow = sl.overflow;
    a.P = S.G.P;
    a.lo = S.lo;
    a.nloc = S.nloc;
    a.k0 = S.k0;
    a.k1 = S.k1;
    a.seed_node = S.seed_node;
    a.W = s->world;
    a.me = sl.rank;
    for (int w = 0; w <= s->world; ++w) a.bounds[w] = s->bounds[w];
    for (int p = 0; p < s->world; ++p) {
        a.peer[p] = xpeer(sl.xsend, sl.soff[p], sl.cap_out[p]);
        a.rpeer[p] = xpeer(sl.xrecv, sl.roff[p], sl.cap_in[p]);
    }
    return a;
}

// Push-sum on the full topology, one rank of several (gp_fullbin.hip): this
// rank's receivers [lo, lo + nloc), node arrays indexed by id - lo; exchange region h:
// the fold's tiles and senders (full_region), the bins it sends to every rank (out;
// its own share into its own receive region) and the bins received from every rank (in).
// This rank's own share of region h's bins, round parity `par` (Slab::xown).
FbBins own_bins(gp_sim* s, Slab& sl, int h, uint32_t par) {
    const size_t i = (size_t)h * s->world + sl.rank;
    uint8_t* base = par & 1u ? sl.xown + sl.ooff[h] : sl.xrecv + sl.roff[i];
    return fb_bins_at(base, sl.S.fb_nb1, sl.cap_in[i]);
}

// send_pass: round 0's send pass fills this round's own bins (the fold fills the next round's).
FullBinArgs make_fullbin_args(gp_sim* s, Slab& sl, uint32_t round, int h, bool send_pass = false) {
    DevState& S = sl.S;
    const int cur = round & 1;
    const uint32_t d = S.lo - S.base;
    const int W = s->world;
    FullBinArgs a{};
    a.swc = S.sw[cur] + d;
    a.swn = S.sw[cur ^ 1] + d;
    a.nb = S.nb[0] + d;
    a.ctl = S.ctl;
    a.overflow = sl.overflow;
    a.P = S.G.P;
    a.k0 = S.k0;
    a.k1 = S.k1;
    a.s1 = S.fb_s1;
    a.nb1 = S.fb_nb1;
    a.nb2 = S.fb_nb2;
    a.cap2 = S.fb_cap2;
    a.cnt2 = S.fb_cnt2;
    a.hdr2 = S.fb_hdr2;
    a.pay2 = S.fb_pay2;
    a.lo = S.lo;
    a.nloc = S.nloc;
    full_region(S.nloc, s->xhalves, h, a.t_lo, a.t_hi, a.s_lo, a.s_hi);
    a.fused = 1;
    a.W = W;
    a.me = sl.rank;
    for (int w = 0; w <= W; ++w) a.bounds[w] = s->bounds[w];
    const uint32_t item = full_bin_item_messages();
    a.in_item0[0] = 0;
    for (int p = 0; p < W; ++p) {
        const size_t i = (size_t)h * W + p;
        const uint32_t nbp = (uint32_t)(((uint64_t)s->bounds[p + 1] - s->bounds[p] + (1ull << S.fb_s1) - 1) >> S.fb_s1);
        a.in[p] = p == sl.rank ? own_bins(s, sl, h, round) : fb_bins_at(sl.xrecv + sl.roff[i], S.fb_nb1, sl.cap_in[i]);
        a.out[p] = p == sl.rank ? own_bins(s, sl, h, send_pass ? round : round + 1)
                                : fb_bins_at(sl.xsend + sl.soff[i], nbp, sl.cap_out[i]);
        a.in_item0[p + 1] = a.in_item0[p] + (sl.cap_in[i] ? S.fb_nb1 * ((sl.cap_in[i] + item - 1) / item) : 0u);
    }
    return a;
}

// Full topology on several ranks: one round (push-sum gp_fullbin.hip, gossip gp_full.hip).
// Push-sum (round 6): the messages of round r reach this rank as the coarse bins of its
// receivers in the exchange buffers of every region and source, where the split reads them;
// the fold then runs region by region, and region h's fold bins its tiles' round-(r+1)
// messages by destination rank and coarse bin straight into region h's buffers, which travel
// (exchange stream, one RCCL group) while the next region's fold runs.  Round 0's messages
// come from the send pass (only the seed sends).  Events order the streams; every RCCL
// operation is issued in one order on every rank (group region 0, 1, then the finalize
// all-reduce, which waits for the last group).
int launch_round_full_multi(gp_sim* s, uint32_t r, hipEvent_t e0, hipEvent_t e1) {
    const bool push = s->cfg.algorithm == GP_PUSHSUM;
    int rc;
    if (e0) HIP_TRY(hipEventRecord(e0, s->stream));
    if (push) {
        const int NH = s->xhalves;
        hipStream_t xs = s->xstream ? s->xstream : s->stream;
        auto send_region = [&](int h) -> int {  // region h's buffers to the exchange stream
            if (xs != s->stream) {
                HIP_TRY(hipEventRecord(s->ev_send[h], s->stream));
                HIP_TRY(hipStreamWaitEvent(xs, s->ev_send[h], 0));
            }
            int rc2;
            if ((rc2 = transfer_xbufs(s, h, xs))) return rc2;
            if (xs != s->stream) HIP_TRY(hipEventRecord(s->ev_xfer[h], xs));
            return GP_OK;
        };
        // the counters this round fills, in one launch: the fine tiles', every region's send bins'
        // (their last transfer is done: finalize waited for it), the own next-round bins' (the
        // split of round r - 1 read them); round 0 also this round's own bins, for the send pass
        // (zero_send: the send bins alone -- round 0's send pass has used them once already)
        auto zero_counts = [&](bool zero_send) -> int {
            for (Slab& sl : s->slab) {
                ZeroList z{};
                auto add = [&](uint32_t* p, uint32_t n) {
                    if (p && n && z.k < ZeroList::MAX) {
                        z.p[z.k] = p;
                        z.n[z.k++] = n;
                    }
                };
                if (!zero_send) add(sl.S.fb_cnt2, sl.S.fb_nb2);
                for (int h = 0; h < NH; ++h) {
                    const FullBinArgs a = make_fullbin_args(s, sl, r, h);
                    for (int p = 0; p < s->world; ++p)
                        if (p != sl.rank || !zero_send) add(a.out[p].cnt, a.out[p].nb);  // (own: next parity)
                    if (r == 0 && !zero_send) add(a.in[sl.rank].cnt, a.in[sl.rank].nb);
                }
                HIP_TRY(launch_zero_list(z, s->stream));
            }
            return GP_OK;
        };
        if ((rc = zero_counts(false))) return rc;
        if (r == 0) {  // round 0's messages: the send pass
            for (int h = 0; h < NH; ++h) {
                for (Slab& sl : s->slab) HIP_TRY(launch_full_bin_send_multi(make_fullbin_args(s, sl, r, h, true), r, s->stream));
                if ((rc = send_region(h))) return rc;
            }
        }
        for (int h = 0; h < NH; ++h) {  // region h's bins into the fine tiles once they are here
            if (xs != s->stream) HIP_TRY(hipStreamWaitEvent(s->stream, s->ev_xfer[h], 0));
            for (Slab& sl : s->slab) HIP_TRY(launch_full_bin_split_multi(make_fullbin_args(s, sl, r, h), r, s->stream));
        }
        if (r == 0 && (rc = zero_counts(true))) return rc;  // (the send pass's transfers are done)
        for (int h = 0; h < NH; ++h) {  // the fold, region by region; round r+1's messages travel behind it
            for (Slab& sl : s->slab)
                HIP_TRY(launch_full_bin_fold_multi(make_fullbin_args(s, sl, r, h), r, s->cus, s->stream));
            if ((rc = send_region(h))) return rc;
        }
        if (e1) HIP_TRY(hipEventRecord(e1, s->stream));
        if (xs != s->stream) HIP_TRY(hipStreamWaitEvent(s->stream, s->ev_xfer[NH - 1], 0));
        return finalize(s, r, r + 1);
    }
    for (Slab& sl : s->slab) {
        FullArgs a = make_full_args(s, sl, r);
        ZeroArgs z{};
        for (int p = 0; p < s->world; ++p) z.cnt[p] = a.peer[p].cnt;
        z.n = s->world;
        HIP_TRY(launch_zero_counts(z, s->stream));
        HIP_TRY(launch_fullm_gossip_send(a, r, s->grid, s->stream));
    }
    if ((rc = transfer_xbufs(s, 0, s->stream))) return rc;
    for (Slab& sl : s->slab) {
        FullArgs a = make_full_args(s, sl, r);
        HIP_TRY(launch_fullm_gossip_unpack(a, std::max(1, s->grid / 8), s->stream));
        HIP_TRY(launch_fullm_gossip_recv(a, s->grid, s->stream));
    }
    if (e1) HIP_TRY(hipEventRecord(e1, s->stream));
    return finalize(s, r, r + 1);
}

// Halo refresh + Imp3D random-edge exchange for round `rn`, whose state the
// previous round kernel has just written to buffers rn & 1.  Push-sum moves the
// random-edge messages as sender-ordered lists (k_list_pack: header words + compacted
// messages, read in place by the next round kernel -- no unpack) in two regions
// (s->xhalves): region 0 is packed and handed to the exchange stream, whose transfer
// (with the halo planes) overlaps region 1's packing.  Gossip packs {slot} or {count}
// entries and unpacks them (k_pack / k_unpack).  Events order the streams, so every
// rank issues its RCCL groups in one order (region 0, region 1), before the finalize
// all-reduce on the compute stream.  exchange() = exchange_open, exchange_region for every
// region (halo planes in region 0's group), exchange_close; launch_round_regions runs the same
// pieces region by region behind the round kernel's launches (halo planes in the last group).
struct XchgCtx {
    int W, b, NH;
    bool push, imp, lists, bits;
    hipStream_t xs;
    size_t H, HS;
    XchgCtx(const gp_sim* s, uint32_t rn) {
        W = s->world;
        b = rn & 1;
        push = s->cfg.algorithm == GP_PUSHSUM;
        imp = s->cfg.topology == GP_IMP3D;
        NH = imp ? s->xhalves : 1;
        xs = NH > 1 && s->xstream ? s->xstream : s->stream;
        H = s->halo;
        HS = s->halo_slots;  // push-sum: the halo planes' (s, w) compacted (setup_halo)
        lists = imp && push && s->slab[0].lists;
        bits = imp && s->slab[0].bits;
    }
};

// The halo planes of round rn: compacted (s, w) packed; in-process ranks copy them here.
// cs: the stream of the packs.
int exchange_open(gp_sim* s, uint32_t rn, hipStream_t cs) {
    const XchgCtx x(s, rn);
    const int W = x.W, b = x.b;
    const size_t H = x.H, HS = x.HS;
    int rc;
    if (x.push && HS && (rc = halo_pack_expand(s, b, true, cs))) return rc;
    if (s->mode == MODE_VIRTUAL) {  // halo planes by device copies (round kernel -> next round kernel)
        for (int r = 0; r + 1 < W; ++r) {
            DevState& A = s->slab[r].S;  // lower slab
            DevState& B = s->slab[r + 1].S;
            const uint32_t edge = B.lo;  // A's hi
            // A's last H ids -> B's lower halo; B's first H ids -> A's upper halo
            HIP_TRY(hipMemcpyAsync(B.nb[b] + (edge - H - B.base), A.nb[b] + (edge - H - A.base), H,
                                   hipMemcpyDeviceToDevice, cs));
            HIP_TRY(hipMemcpyAsync(A.nb[b] + (edge - A.base), B.nb[b] + (edge - B.base), H, hipMemcpyDeviceToDevice,
                                   cs));
            if (x.push && HS) {
                HIP_TRY(hipMemcpyAsync(s->slab[r + 1].hrecv[0], s->slab[r].hsend[1], HS * 16, hipMemcpyDeviceToDevice,
                                       cs));
                HIP_TRY(hipMemcpyAsync(s->slab[r].hrecv[1], s->slab[r + 1].hsend[0], HS * 16, hipMemcpyDeviceToDevice,
                                       cs));
            } else if (x.push) {
                HIP_TRY(hipMemcpyAsync(B.sw[b] + (edge - H - B.base), A.sw[b] + (edge - H - A.base), H * 16,
                                       hipMemcpyDeviceToDevice, cs));
                HIP_TRY(hipMemcpyAsync(A.sw[b] + (edge - A.base), B.sw[b] + (edge - B.base), H * 16,
                                       hipMemcpyDeviceToDevice, cs));
            }
        }
    }
    return GP_OK;
}

// Region h of round rn's random-edge exchange: packed on the compute stream, then handed to the
// exchange stream (one RCCL group per region; the halo planes travel in region hg's group).
int exchange_region(gp_sim* s, uint32_t rn, int h, int hg, hipStream_t cs) {
    const XchgCtx x(s, rn);
    const int W = x.W, b = x.b, NH = x.NH;
    const bool push = x.push, imp = x.imp, lists = x.lists, bits = x.bits;
    const hipStream_t xs = x.xs;
    const size_t H = x.H, HS = x.HS;
    int rc;
    if (imp && !bits) {  // (bitmaps: set by the round kernel itself)
        for (Slab& sl : s->slab) {
            DevState& S = sl.S;
            if (lists) {  // header words + compacted messages of region h (k_list_pack)
                HIP_TRY(hipMemsetAsync(sl.xcnt + (size_t)h * W, 0, sizeof(uint32_t) * W, cs));
                ListPackArgs la{};
                la.nbn = S.nb[b];
                la.swn = S.sw[b];
                la.xdr = sl.xdr;
                la.lwt = sl.lwt;
                la.gw = sl.gw;
                la.lo = S.lo;
                la.nloc = S.nloc;
                la.base = S.base;
                la.t0 = sl.tb[h];
                la.t1 = h + 1 == NH ? sl.nt : sl.tb[h + 1];
                la.W = W;
                la.me = sl.rank;
                for (int d = 0; d < W; ++d) {
                    if (d == sl.rank) continue;
                    const size_t i = (size_t)h * W + d;
                    la.peer[d].hdr = reinterpret_cast<XHdr*>(sl.xsend + sl.lhdr[i]);
                    la.peer[d].vals = reinterpret_cast<double2*>(sl.xsend + sl.lval[i]);
                    la.peer[d].cnt = sl.xcnt + i;
                    la.peer[d].cap = sl.cap_out[i];
                    la.peer[d].vbase = sl.vbase[i];
                }
                la.overflow = sl.overflow;
                HIP_TRY(launch_list_pack(la, cs));
                continue;
            }
            ZeroArgs z{};
            PackArgs pa{};
            pa.nbn = S.nb[b];
            pa.swn = push ? S.sw[b] : nullptr;
            pa.rnd = S.rnd;
            pa.pos = sl.pos;
            pa.xdst = sl.xdst;
            pa.lo = S.lo;
            pa.nloc = S.nloc;
            pa.s_lo = NH == 1 || h == 0 ? 0u : S.nloc / 2;
            pa.s_hi = NH == 1 || h == 1 ? S.nloc : S.nloc / 2;
            pa.base = S.base;
            pa.W = W;
            pa.me = sl.rank;
            pa.push = push ? 1 : 0;
            pa.counts = col_gossip_counts(S) ? 1 : 0;
            for (int w = 0; w <= W; ++w) pa.bounds[w] = s->bounds[w];
            for (int p = 0; p < W; ++p) {
                const size_t i = (size_t)h * W + p;
                pa.peer[p] = xpeer(sl.xsend, sl.soff[i], sl.cap_out[i]);
                z.cnt[p] = pa.peer[p].cnt;
            }
            z.n = W;
            pa.overflow = sl.overflow;
            HIP_TRY(launch_zero_counts(z, cs));
            HIP_TRY(launch_pack(pa, s->grid, cs));
        }
    }
    if (xs != s->stream) {
        HIP_TRY(hipEventRecord(s->ev_send[h], cs));
        HIP_TRY(hipStreamWaitEvent(xs, s->ev_send[h], 0));
    }
    if (s->mode == MODE_VIRTUAL) {
        if (bits) {
            for (Slab& a : s->slab)
                for (Slab& d : s->slab)
                    if (&a != &d && a.bn[d.rank])
                        HIP_TRY(hipMemcpyAsync(d.rbits_in + d.ro[a.rank] / 32, a.S.sbits + a.bo[d.rank] / 32,
                                               (size_t)(a.bn[d.rank] + 31) / 32 * 4, hipMemcpyDeviceToDevice, xs));
        } else if (lists) {
            for (Slab& a : s->slab)
                for (Slab& d : s->slab) {
                    if (&a == &d) continue;
                    const size_t i = (size_t)h * W + d.rank, j = (size_t)h * W + a.rank;
                    const size_t hb = (size_t)s->list_nw[((size_t)a.rank * NH + h) * W + d.rank] * 16;
                    if (hb)
                        HIP_TRY(hipMemcpyAsync(d.xrecv + (size_t)b * d.xr_stride + d.rhdr[j], a.xsend + a.lhdr[i], hb,
                                               hipMemcpyDeviceToDevice, xs));
                    if (a.cap_out[i])
                        HIP_TRY(hipMemcpyAsync(d.xrecv + (size_t)b * d.xr_stride + d.rval[j], a.xsend + a.lval[i],
                                               (size_t)a.cap_out[i] * 16,
                                               hipMemcpyDeviceToDevice, xs));
                }
        } else if (imp) {
            rc = transfer_xbufs(s, h, xs);
            if (rc) return rc;
        }
    } else {
        Slab& sl = s->slab[0];
        DevState& S = sl.S;
        const int r = sl.rank;
        uint8_t* xr = sl.xrecv + (size_t)b * sl.xr_stride;  // lists: this round parity's receive buffer
        NCCL_TRY(ncclGroupStart());
        if (h == hg && r > 0) {  // my first H ids <-> lower neighbour's last H ids
            NCCL_TRY(ncclSend(S.nb[b] + (S.lo - S.base), H, ncclUint8, r - 1, s->comm, xs));
            NCCL_TRY(ncclRecv(S.nb[b] + (S.lo - H - S.base), H, ncclUint8, r - 1, s->comm, xs));
            if (push && HS) {
                NCCL_TRY(ncclSend(sl.hsend[0], HS * 16, ncclUint8, r - 1, s->comm, xs));
                NCCL_TRY(ncclRecv(sl.hrecv[0], HS * 16, ncclUint8, r - 1, s->comm, xs));
            } else if (push) {
                NCCL_TRY(ncclSend(S.sw[b] + (S.lo - S.base), H * 16, ncclUint8, r - 1, s->comm, xs));
                NCCL_TRY(ncclRecv(S.sw[b] + (S.lo - H - S.base), H * 16, ncclUint8, r - 1, s->comm, xs));
            }
        }
        if (h == hg && r < W - 1) {  // my last H ids <-> upper neighbour's first H ids
            NCCL_TRY(ncclSend(S.nb[b] + (sl.hi - H - S.base), H, ncclUint8, r + 1, s->comm, xs));
            NCCL_TRY(ncclRecv(S.nb[b] + (sl.hi - S.base), H, ncclUint8, r + 1, s->comm, xs));
            if (push && HS) {
                NCCL_TRY(ncclSend(sl.hsend[1], HS * 16, ncclUint8, r + 1, s->comm, xs));
                NCCL_TRY(ncclRecv(sl.hrecv[1], HS * 16, ncclUint8, r + 1, s->comm, xs));
            } else if (push) {
                NCCL_TRY(ncclSend(S.sw[b] + (sl.hi - H - S.base), H * 16, ncclUint8, r + 1, s->comm, xs));
                NCCL_TRY(ncclRecv(S.sw[b] + (sl.hi - S.base), H * 16, ncclUint8, r + 1, s->comm, xs));
            }
        }
        if (bits)
            for (int p = 0; p < W; ++p) {  // the bitmap chunks, each way
                if (p == r) continue;
                const size_t ob = (size_t)(sl.bn[p] + 31) / 32 * 4, ib = (size_t)(sl.rn[p] + 31) / 32 * 4;
                if (ob) NCCL_TRY(ncclSend(S.sbits + sl.bo[p] / 32, ob, ncclUint8, p, s->comm, xs));
                if (ib) NCCL_TRY(ncclRecv(sl.rbits_in + sl.ro[p] / 32, ib, ncclUint8, p, s->comm, xs));
            }
        else if (lists)
            for (int p = 0; p < W; ++p) {  // header words, then messages, each way
                if (p == r) continue;
                const size_t i = (size_t)h * W + p;
                const size_t ho = (size_t)s->list_nw[((size_t)r * NH + h) * W + p] * 16;
                const size_t hi = (size_t)s->list_nw[((size_t)p * NH + h) * W + r] * 16;
                if (ho) NCCL_TRY(ncclSend(sl.xsend + sl.lhdr[i], ho, ncclUint8, p, s->comm, xs));
                if (sl.cap_out[i])
                    NCCL_TRY(ncclSend(sl.xsend + sl.lval[i], (size_t)sl.cap_out[i] * 16, ncclUint8, p, s->comm, xs));
                if (hi) NCCL_TRY(ncclRecv(xr + sl.rhdr[i], hi, ncclUint8, p, s->comm, xs));
                if (sl.cap_in[i])
                    NCCL_TRY(ncclRecv(xr + sl.rval[i], (size_t)sl.cap_in[i] * 16, ncclUint8, p, s->comm, xs));
            }
        else if (imp)
            for (int p = 0; p < W; ++p) {
                if (p == r) continue;
                const size_t i = (size_t)h * W + p;
                if (sl.sbytes[i]) NCCL_TRY(ncclSend(sl.xsend + sl.soff[i], sl.sbytes[i], ncclUint8, p, s->comm, xs));
                if (sl.rbytes[i]) NCCL_TRY(ncclRecv(sl.xrecv + sl.roff[i], sl.rbytes[i], ncclUint8, p, s->comm, xs));
            }
        NCCL_TRY(ncclGroupEnd());
    }
    if (xs != s->stream) HIP_TRY(hipEventRecord(s->ev_xfer[h], xs));
    return GP_OK;
}

// After the last region: received bitmaps applied / entries unpacked, halo planes expanded.
int exchange_close(gp_sim* s, uint32_t rn) {
    const XchgCtx x(s, rn);
    const int W = x.W, b = x.b, NH = x.NH;
    const bool push = x.push, imp = x.imp, lists = x.lists, bits = x.bits;
    const hipStream_t xs = x.xs;
    const size_t HS = x.HS;
    int rc;
    if (bits) {
        if (xs != s->stream) HIP_TRY(hipStreamWaitEvent(s->stream, s->ev_xfer[NH - 1], 0));
        for (Slab& sl : s->slab) {
            // one rumour per received bit at its target, counted for round rn; then the send
            // bitmap is cleared for the next round kernel
            HIP_TRY(launch_apply_bits(sl.rbits_in, sl.nbits_in / 32, sl.tgt, sl.S.rq[rn & 1], sl.S.rq8, s->stream));
            if (sl.nbits_out) HIP_TRY(hipMemsetAsync(sl.S.sbits, 0, (size_t)sl.nbits_out / 8, s->stream));
        }
    } else if (imp && !lists) {
        for (int h = 0; h < NH; ++h) {
            if (xs != s->stream) HIP_TRY(hipStreamWaitEvent(s->stream, s->ev_xfer[h], 0));
            for (Slab& sl : s->slab) {
                UnpackArgs ua{};
                ua.rtag = sl.S.rtag;
                ua.rmsg = sl.S.rmsg;
                ua.rq = col_gossip_counts(sl.S) ? sl.S.rq[rn & 1] : nullptr;  // next round's deliveries
                ua.rq8 = sl.S.rq8;
                ua.nedges = ua.rq ? sl.S.nloc : sl.nedges;
                ua.W = W;
                ua.me = sl.rank;
                ua.push = push ? 1 : 0;
                for (int p = 0; p < W; ++p) {
                    const size_t i = (size_t)h * W + p;
                    ua.peer[p] = xpeer(sl.xrecv, sl.roff[i], sl.cap_in[i]);
                }
                ua.overflow = sl.overflow;
                ua.all_active = &sl.S.ctl->all_active;
                HIP_TRY(launch_unpack(ua, rn, std::max(1, s->grid / 8), s->stream));
            }
        }
    } else if (xs != s->stream) {
        HIP_TRY(hipStreamWaitEvent(s->stream, s->ev_xfer[NH - 1], 0));
    }
    if (push && HS && (rc = halo_pack_expand(s, b, false, s->stream))) return rc;
    return GP_OK;
}

int exchange(gp_sim* s, uint32_t rn) {
    if (s->world == 1 || s->cfg.topology == GP_FULL) return GP_OK;  // full: the exchange is inside the round
    const XchgCtx x(s, rn);
    int rc;
    if ((rc = exchange_open(s, rn, s->stream))) return rc;
    for (int h = 0; h < x.NH; ++h)
        if ((rc = exchange_region(s, rn, h, 0, s->stream))) return rc;
    return exchange_close(s, rn);
}

// Close round `round_done` (if round_next > 0) and prepare round `round_next`.
int finalize(gp_sim* s, uint32_t round_done, uint32_t round_next) {
    if (s->mode == MODE_SINGLE) {
        HIP_TRY(launch_finalize(s->slab[0].S, round_done, round_next, s->stream));
        return GP_OK;
    }
    for (Slab& sl : s->slab) HIP_TRY(launch_finalize_pre(sl.S, round_next, s->stream));
    if (s->mode == MODE_VIRTUAL) {
        SumArgs sa{};
        sa.W = (int)s->slab.size();
        for (int w = 0; w < sa.W; ++w) sa.ctl[w] = s->slab[w].S.ctl;
        HIP_TRY(launch_sum_xchg(sa, s->stream));
    } else {
        Ctl* c = s->slab[0].S.ctl;
        NCCL_TRY(ncclAllReduce(c->xchg, c->xchg, 4, ncclUint64, ncclSum, s->comm, s->stream));
    }
    for (Slab& sl : s->slab) HIP_TRY(launch_finalize_post(sl.S, round_done, round_next, s->stream));
    return GP_OK;
}

// One round of Imp3D push-sum across ranks, region by region (DevState::rregions): the round
// kernel over region h's tiles, then region h's lists packed and handed to the exchange stream,
// whose transfer overlaps the next regions' round kernel launches; the halo planes (first and
// last region) travel in the last group.  The lists arrive in the other parity's receive buffer
// (Slab::xr_stride): this round's kernels still read theirs.  ev (kernel timing, else null):
// 2 NR events, ev[2h] / ev[2h + 1] around launch h (the round kernel time excludes the packs).
int launch_round_regions(gp_sim* s, uint32_t r, hipEvent_t* ev) {
    const uint32_t NR = s->slab[0].S.rregions;
    const uint32_t rn = r + 1;
    int rc;
    for (uint32_t h = 0; h < NR; ++h) {
        if (ev) HIP_TRY(hipEventRecord(ev[2 * h], s->stream));
        for (Slab& sl : s->slab) HIP_TRY(launch_round_tile_region(sl.S, r, h, s->grid, s->stream));
        if (ev) HIP_TRY(hipEventRecord(ev[2 * h + 1], s->stream));
        // (region h's pack on a stream of its own, beside launch h + 1: 2-5 % slower,
        // profiles/r05/rejected/pack_stream.txt)
        const hipStream_t cs = s->stream;
        if (h + 1 == NR && (rc = exchange_open(s, rn, cs))) return rc;
        if ((rc = exchange_region(s, rn, (int)h, (int)NR - 1, cs))) return rc;
    }
    if ((rc = exchange_close(s, rn))) return rc;
    return finalize(s, r, rn);
}

// Round kernel launches per round the kernel timing brackets (DevState::rregions, else 1).
uint32_t round_launches(const gp_sim* s) { return std::max<uint32_t>(1u, s->slab[0].S.rregions); }

// One synchronous round r: round kernel(s), exchange, finalize.
// ev (kernel timing, else null): 2 * round_launches(s) events.
int launch_round(gp_sim* s, uint32_t r, hipEvent_t* ev) {
    if (s->slab[0].S.rregions > 1) return launch_round_regions(s, r, ev);
    const hipEvent_t e0 = ev ? ev[0] : nullptr, e1 = ev ? ev[1] : nullptr;
    if (s->cfg.topology == GP_FULL && s->world > 1) return launch_round_full_multi(s, r, e0, e1);
    for (size_t q = 0; q < s->slab.size(); ++q) {
        DevState& S = s->slab[q].S;
        if (q == 0 && e0) HIP_TRY(hipEventRecord(e0, s->stream));
        HIP_TRY(launch_bulk(S, r, s->grid, s->stream));
        if (q == 0 && e1) HIP_TRY(hipEventRecord(e1, s->stream));
    }
    int rc;
    if ((rc = exchange(s, r + 1))) return rc;
    if (s->slab[0].S.fuse_finalize) return GP_OK;  // the round kernel closed its own round
    return finalize(s, r, r + 1);
}

double alg_bytes(const gp_sim* s) {
    const DevState& S = s->slab[0].S;
    if (S.alg == PUSHSUM) {
        // sw r+w 32, node byte r+w 2 (+ Imp3D: in-degree nibble 0.5 + sender 4 of the
        // in-list, and the random-edge message payload, 16 B for the ~1/7 of senders
        // that use the random edge -- a random gather, moved as a 128-B line)
        if (S.topo == IMP3D) return 38.5 + 16.0 / 7.0;
        if (S.kernel == KERNEL_BLOCK) {
            // LDS-resident: per round only the boxes' boundary layers move (17 B per face node,
            // written once, read once by the neighbour), through L2 / Infinity Cache
            const BlockPlan& p = S.bplan;
            const double g = S.G.g;
            const double faces = g * g * ((p.nbx - 1) + (p.nby - 1) + (p.nbz - 1)) * 2.0;
            return 2.0 * 17.0 * faces / (double)S.G.P;
        }
        if (S.topo != FULL) return 34.0;
        // send: byte 1 (sweep 1) + byte 1 + own (s, w) 16 + message write 20; split: sender
        // id 4 (sweep 1) + message r+w 40; fold: message 20 + own (s, w) r+w 32 + byte r+w 2
        // (gp_fullbin.hip, range binning).  One rank: the fold writes the next round's
        // messages from the state it just computed, so the send's reads (18) go.
        if (S.fb_fused) return 20.0 + 4.0 + 40.0 + 20.0 + 32.0 + 2.0;
        return 1.0 + 1.0 + 16.0 + 20.0 + 4.0 + 40.0 + 20.0 + 32.0 + 2.0;
    }
    // gossip: counter r+w 8, direction byte r+w 2; Imp3D:
    //   column kernel (counts random-edge sends at their targets a round ahead): rnd 4 +
    //   delivery count read (a byte since round 4; was 4 B), its zeroing where non-zero
    //   and the senders' atomic increments (~1/7 of nodes each, a 4-B word atomic) ->
    //   15 + 5/7 (4-B counts: 18 + 8/7; several ranks: the remote 7/8 of the increments
    //   arrive through k_unpack instead);
    //   tile kernel: in-list 8
    if (S.topo == IMP3D) return S.rq[0] ? (S.rq8 ? 15.0 + 5.0 / 7.0 : 18.0 + 8.0 / 7.0) : 18.0;
    if (S.topo != FULL) return 10.0;
    return 4.0 + 8.0 + 8.0 + 8.0;  // send: c + atomic RMW; recv: inc r+w, c r+w
}

// Kernel variant and grid for this run (measured defaults; GP_KERNEL / GP_XSEGS / GP_WALK /
// GP_WX / GP_WIDE override them in the experiments build).
void choose_kernel(gp_sim* s, int64_t nloc_max, int& kernel, uint32_t& col_xsegs, uint32_t& walk, uint32_t& wx,
                   uint32_t& wide) {
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, s->device);
    s->cus = std::max(1, prop.multiProcessorCount);
    const gp_config* cfg = &s->cfg;
    const int64_t g = s->g;
    int64_t blocks = (nloc_max + BULK_THREADS - 1) / BULK_THREADS;
    // 64 workgroups per CU: measured best for the tiled round kernels (tools/ablate.py:
    // 2048 -> 27.5, 8192 -> 22.1, 16384 -> 21.2 ms/round at P = 1e9)
    int64_t cap = (int64_t)prop.multiProcessorCount * 64;
    // (measured: gossip on a large lattice -> column march, profiles/r01; push-sum and
    // small lattices and line -> tiled; the push-sum column march was measured slower,
    // profiles/r03 and DESIGN.md §5.1)
    kernel = KERNEL_TILE;
    const bool lattice = cfg->topology == GP_3D || cfg->topology == GP_IMP3D;
    const bool push = cfg->algorithm == GP_PUSHSUM;
    if (lattice && g >= 200 && !push) kernel = KERNEL_COL;
    // 3D push-sum on one rank whose lattice fits the chip's LDS (C2: g = 100): one cooperative
    // launch per batch, the state resident in LDS (gp_block.hip)
    BlockPlan bp{};
    const bool block_ok = cfg->topology == GP_3D && push && s->world == 1 && g >= 2 &&
                          block_plan((uint32_t)g, prop.multiProcessorCount, bp) &&
                          block_plan_resident(bp, prop.multiProcessorCount);
    if (block_ok) kernel = KERNEL_BLOCK;
    if (const char* e = exp_env("GP_KERNEL")) {
        if (!std::strcmp(e, "tile")) kernel = KERNEL_TILE;
        else if (!std::strcmp(e, "col") && lattice && !push) kernel = KERNEL_COL;
        else if (!std::strcmp(e, "block") && block_ok) kernel = KERNEL_BLOCK;
    }
    s->bplan = bp;
    col_xsegs = 1;
    if (cfg->topology != GP_FULL && kernel == KERNEL_COL) {
        // gossip: exactly the resident grid (a persistent sweep), a multiple of the 8 XCDs
        cap = (int64_t)prop.multiProcessorCount * col_blocks_per_cu(cfg->topology, cfg->algorithm);
        // x segments per patch: enough work items for every resident wave, >= 16 planes each
        const int64_t patches = ((g + 63) / 64) * ((g + 3) / 4);
        const int64_t slots = cap * (BULK_THREADS / 64);
        const int64_t planes = std::max<int64_t>(1, g / s->world);
        int64_t xs = std::max<int64_t>(1, slots / std::max<int64_t>(1, patches));
        xs = std::min<int64_t>(xs, std::max<int64_t>(1, planes / 16));
        col_xsegs = (uint32_t)xs;
    }
    if (kernel == KERNEL_TILE)  // 1024-node tiles (+1: a slab may start mid-tile), a multiple of the 8 XCDs
        blocks = ((nloc_max + 1023) / 1024 + 1 + 7) / 8 * 8;
    if (const char* e = exp_env("GP_XSEGS")) col_xsegs = (uint32_t)std::max(1, std::atoi(e));
    s->grid = (int)std::max<int64_t>(1, std::min(kernel == KERNEL_COL ? cap : blocks, cap));
    // tile walk: x-windows of 8 planes once every XCD gets a few windows (measured,
    // profiles/r01: 18.2 -> 17.2 ms/round at P = 1e9), else XCD-contiguous eighths
    walk = (lattice && g / s->world >= 64) ? 2u : 0u;
    // push-sum: the same x-windows claimed from per-XCD counters on exactly the
    // resident grid (walk 3; measured, profiles/r02/walk3.txt)
    if (walk == 2 && kernel == KERNEL_TILE && cfg->algorithm == GP_PUSHSUM) walk = 3;
    // x-window of 8 planes (walk 2); 16 for walk 3 since round 4, where the wave priority
    // of the tile kernel moved the optimum: P = 1e9, same box, 8 / 12 / 16 / 24 / 32 planes
    // 13.34-13.36 / 13.17-13.28 / 13.17-13.22 / 13.22-13.25 / 13.15-13.17 ms/round
    // (profiles/r04/walk_window_nt.txt)
    wx = walk == 3 ? 16 : 8;
    if (const char* e = exp_env("GP_WALK")) walk = (uint32_t)std::atoi(e);
    if (const char* e = exp_env("GP_WX")) wx = (uint32_t)std::max(1, std::atoi(e));
    // size class of the tiled kernels: line / 3D push-sum on a slab with at most two tiles per
    // resident block of the 4-nodes-per-thread kernel (~2500 tiles, P <~ 2.6e6 per slab) runs the
    // 1024-thread, one-node-per-thread build (gp_round_wide.hip): its node phase is one memory
    // round trip per tile instead of four, which is what bounds a round with few tiles per block
    // (C2, 3D push-sum P = 1e6: 26.5 -> 20.7 us per round; line push-sum n = 1000: 10.2 -> 8.8).
    // Imp3D push-sum (its in-edge pass spills at 8 waves) and the gossip tile kernel measured
    // slower in that build at every size (profiles/r04/tile_size_class.txt)
    wide = 0;
    if (kernel == KERNEL_TILE && push && cfg->topology != GP_IMP3D) {
        const int topo = cfg->topology == GP_LINE ? LINE : cfg->topology == GP_3D ? GRID3D : IMP3D;
        const int64_t tiles = (nloc_max + 1023) / 1024 + 1;
        const int64_t res4 = ps_tile_resident_blocks(topo, s->world > 1 && topo == IMP3D, s->device);
        wide = res4 > 0 && tiles <= 2 * res4 ? 1u : 0u;
        if (const char* e = exp_env("GP_WIDE")) wide = e[0] == '1' ? 1u : 0u;
    }
    if (walk == 3) {
        const int topo = cfg->topology == GP_LINE ? LINE : cfg->topology == GP_3D ? GRID3D : IMP3D;
        const bool rem = s->world > 1 && topo == IMP3D;
        const int64_t res = (wide ? wide::ps_tile_resident_blocks(topo, rem, s->device)
                                  : ps_tile_resident_blocks(topo, rem, s->device)) / 8 * 8;
        if (res >= 8) s->grid = (int)std::min<int64_t>(s->grid, res);
        else walk = 2;
    }
}

// Everything after the handle exists: slabs, topology, initial state, round 0.
int build_sim(gp_sim* s) {
    int rc;
    if ((rc = make_bounds(s))) return rc;
    int64_t nloc_max = 0;
    for (int w = 0; w < s->world; ++w) nloc_max = std::max<int64_t>(nloc_max, s->bounds[w + 1] - s->bounds[w]);
    int kernel;
    uint32_t col_xsegs, walk, wx, wide;
    choose_kernel(s, nloc_max, kernel, col_xsegs, walk, wx, wide);
    const uint32_t rreg = round_regions(s, kernel, walk);
    if (s->mode == MODE_VIRTUAL) {
        s->slab.resize(s->world);
        for (int w = 0; w < s->world; ++w) s->slab[w].rank = w;
    } else {
        s->slab.resize(1);
        s->slab[0].rank = s->rank;
    }
    for (Slab& sl : s->slab) {
        sl.S.kernel = kernel;
        sl.S.tile_wide = wide;
        sl.S.col_xsegs = col_xsegs;
        sl.S.tile_walk = walk;
        sl.S.tile_wx = wx;
        sl.S.tile_stage_cap = 0xFFFFFFFFu;
        // single-rank lattice push-sum: the round kernel's last block closes the
        // round (no injector, nothing to exchange), saving a k_finalize launch per round
        // (2: arrivals sharded over 8 counters; a single counter -- 1, experiments
        // only -- serialises ~16k returning atomics per round: measured 1.93 vs
        // 0.40 ms/round at P = 2.7e7, profiles/r02/round_close.txt)
        sl.S.fuse_finalize = (s->mode == MODE_SINGLE && s->cfg.algorithm == GP_PUSHSUM &&
                              s->cfg.topology != GP_FULL) ? 2u : 0u;
        sl.S.bplan = s->bplan;
        sl.S.bface = sl.S.bscratch = nullptr;
        if (kernel == KERNEL_BLOCK) {  // face exchange buffers + barrier / accumulator scratch
            if ((rc = dev_alloc(s, &sl.S.bface, block_face_bytes(s->bplan))) || (rc = dev_alloc(s, &sl.S.bscratch, BLOCK_SCRATCH_BYTES)))
                return rc;
            HIP_TRY(block_kernel_setup(s->bplan));
        }
        if (const char* e = exp_env("GP_FUSE")) sl.S.fuse_finalize = sl.S.fuse_finalize ? (uint32_t)(e[0] - '0') : 0u;
        if (const char* e = exp_env("GP_STAGE_CAP")) sl.S.tile_stage_cap = (uint32_t)std::max(0, std::atoi(e));
        if ((rc = alloc_slab(s, sl, sl.rank))) return rc;
        sl.S.rregions = rreg;
        if (sl.S.tile_walk == 3) {  // the tile list of the per-XCD queues
            std::vector<uint32_t> list;
            if (!build_walk_list(sl.S, (int)sl.S.rregions, list, sl.S.woff)) {
                set_err("internal: walk-3 tile list does not cover the slab");
                return GP_EINVAL;
            }
            if ((rc = dev_alloc_t(s, &sl.S.wtiles, list.size() + 1))) return rc;
            HIP_TRY(hipMemcpy(sl.S.wtiles, list.data(), sizeof(uint32_t) * list.size(), hipMemcpyHostToDevice));
        }
    }
    if (s->cfg.topology == GP_IMP3D && (rc = build_imp3d(s))) return rc;
    if ((s->cfg.topology == GP_IMP3D || s->cfg.topology == GP_FULL) && s->world > 1 && (rc = setup_exchange(s)))
        return rc;
    if ((rc = setup_halo(s))) return rc;
    if (hipHostMalloc((void**)&s->host_ctl, sizeof(Ctl), hipHostMallocDefault) != hipSuccess) {
        set_err("hipHostMalloc failed");
        return GP_ENOMEM;
    }
    Ctl& init = *s->host_ctl;
    std::memset(&init, 0, sizeof init);
    init.active_total = 1;  // the seed
    init.all_active = s->P <= 1 ? 1u : 0u;
    init.inj_target = -1;
    init.inj_pick = -1;
    for (Slab& sl : s->slab) {
        DevState& S = sl.S;
        HIP_TRY(hipMemcpyAsync(S.ctl, &init, sizeof(Ctl), hipMemcpyHostToDevice, s->stream));
        HIP_TRY(launch_init(S, s->grid, s->stream));
        if (S.topo == IMP3D)
            HIP_TRY(col_gossip_counts(S) ? launch_col_seed_init(S, s->stream) : launch_rbits_init(S, s->grid, s->stream));
        if (S.alg == GOSSIP && S.topo != FULL) HIP_TRY(launch_injector_init(S, s->grid, s->stream));
    }
    if ((rc = exchange(s, 0))) return rc;     // halos and random edges of round 0
    if ((rc = finalize(s, 0, 0))) return rc;  // prepare round 0
    hipError_t e = hipStreamSynchronize(s->stream);
    if (e != hipSuccess) {
        set_err("initialisation failed: %s", hipGetErrorString(e));
        return GP_EHIP;
    }
    if (s->timing) {
        s->ev.resize((size_t)2 * BATCH * round_launches(s));
        for (auto& x : s->ev) HIP_TRY(hipEventCreate(&x));
    }
    return GP_OK;
}

int create_common(const gp_config* cfg, int mode, int world, int rank, const uint8_t* uid, gp_sim** out) {
    if (!cfg || !out) {
        set_err("gp_create: null argument");
        return GP_EINVAL;
    }
    *out = nullptr;
    if (cfg->algorithm != GP_GOSSIP && cfg->algorithm != GP_PUSHSUM) {
        set_err("option invalid: algorithm id %d", cfg->algorithm);
        return GP_EINVAL;
    }
    int64_t P, T, g;
    int rc = gp_resolve(cfg->num_nodes, cfg->topology, &P, &T, &g);
    if (rc) return rc;
    if ((rc = check_device(cfg->device))) return rc;
    gp_sim* s = new gp_sim();
    s->cfg = *cfg;
    s->device = cfg->device;
    s->P = P;
    s->T = T;
    s->g = g;
    s->mode = mode;
    s->world = world;
    s->rank = rank;
    s->timing = (cfg->flags & GP_FLAG_KERNEL_TIMING) != 0;
    if (hipSetDevice(s->device) != hipSuccess || hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess) {
        set_err("hipSetDevice/hipStreamCreate failed on device %d", s->device);
        gp_destroy(s);
        return GP_EHIP;
    }
    if (mode == MODE_RCCL) {
        ncclUniqueId id;
        std::memcpy(id.internal, uid, NCCL_UNIQUE_ID_BYTES);
        ncclResult_t r = ncclCommInitRank(&s->comm, world, id, rank);
        if (r != ncclSuccess) {
            set_err("ncclCommInitRank(rank %d of %d) failed: %s", rank, world, ncclGetErrorString(r));
            s->comm = nullptr;
            gp_destroy(s);
            return GP_ENCCL;
        }
    }
    rc = build_sim(s);
    if (rc) {
        const std::string msg = g_err;
        gp_destroy(s);
        g_err = msg;
        return rc;
    }
    *out = s;
    return GP_OK;
}

}  // namespace

extern "C" {

int gp_version(void) { return GP_VERSION; }

const char* gp_last_error(void) { return g_err.c_str(); }

int gp_parse_topology(const char* t) {
    if (!t) return GP_EINVAL;
    if (!std::strcmp(t, "line")) return GP_LINE;
    if (!std::strcmp(t, "full")) return GP_FULL;
    if (!std::strcmp(t, "3D")) return GP_3D;
    if (!std::strcmp(t, "Imp3D") || !std::strcmp(t, "imp3D")) return GP_IMP3D;
    set_err("unknown topology '%s' (line | full | 3D | Imp3D)", t);
    return GP_EINVAL;
}

int gp_parse_algorithm(const char* a) {
    if (!a) return GP_EINVAL;
    if (!std::strcmp(a, "gossip")) return GP_GOSSIP;
    if (!std::strcmp(a, "push-sum")) return GP_PUSHSUM;
    set_err("option invalid: algorithm '%s' (gossip | push-sum)", a);
    return GP_EINVAL;
}

int gp_resolve(int64_t n, int32_t topology, int64_t* P, int64_t* T, int64_t* g) {
    if (!P || !T || !g) {
        set_err("gp_resolve: null output");
        return GP_EINVAL;
    }
    if (n < 1) {
        set_err("num_nodes must be >= 1 (got %lld)", (long long)n);
        return GP_EINVAL;
    }
    if (topology == GP_LINE || topology == GP_FULL) {
        *P = n + 1;
        *T = n;
        *g = 0;
    } else if (topology == GP_3D || topology == GP_IMP3D) {
        int64_t gg = (int64_t)std::cbrt((double)n);  // exact integer ceil(cbrt(n)) (Q3)
        while (gg > 0 && gg * gg * gg >= n) --gg;
        while (gg * gg * gg < n) ++gg;
        *g = gg;
        *P = gg * gg * gg;
        *T = *P;
    } else {
        set_err("unknown topology id %d", topology);
        return GP_EINVAL;
    }
    if (*P > (int64_t)GP_MAX_POPULATION) {
        set_err("population %lld exceeds the 32-bit node-id range", (long long)*P);
        return GP_EINVAL;
    }
    return GP_OK;
}

int gp_create(const gp_config* cfg, gp_sim** out) {
    if (!cfg || !out) {
        set_err("gp_create: null argument");
        return GP_EINVAL;
    }
    if (cfg->num_gpus > 1) {
        if (cfg->flags & GP_FLAG_VIRTUAL_RANKS) return create_common(cfg, MODE_VIRTUAL, cfg->num_gpus, 0, nullptr, out);
        set_err("num_gpus > 1: one process per GPU -- launch `gossip <n> <topology> <algorithm> --gpus %d` "
                "(or GOSSIP_GPUS=%d), which joins every rank through gp_rendezvous_id + gp_create_rank; "
                "GP_FLAG_VIRTUAL_RANKS runs the slabs in this process on one GPU", cfg->num_gpus, cfg->num_gpus);
        return GP_EINVAL;
    }
    return create_common(cfg, MODE_SINGLE, 1, 0, nullptr, out);
}

int gp_get_unique_id(uint8_t unique_id[128]) {
    if (!unique_id) {
        set_err("gp_get_unique_id: null buffer");
        return GP_EINVAL;
    }
    static_assert(NCCL_UNIQUE_ID_BYTES == 128, "RCCL unique id size");
    ncclUniqueId id;
    NCCL_TRY(ncclGetUniqueId(&id));
    std::memcpy(unique_id, id.internal, NCCL_UNIQUE_ID_BYTES);
    return GP_OK;
}

int gp_rendezvous_id(int32_t rank, const char* path, int32_t timeout_ms, uint8_t unique_id[128]) {
    if (!path || !*path || !unique_id || rank < 0) {
        set_err("gp_rendezvous_id: bad argument");
        return GP_EINVAL;
    }
    const size_t N = 128;
    // GOSSIP_RDV_NONCE (set by the launchers, one value per launch): rank 0 writes it after
    // the id and readers accept only a file that carries theirs, so a file a crashed run
    // left at a caller-chosen path is never read as this run's id
    const char* nv = std::getenv("GOSSIP_RDV_NONCE");
    const std::string nonce = nv ? std::string(nv).substr(0, 64) : std::string();
    if (rank == 0) {  // publish: write a private name, then rename (readers never see a partial id)
        struct stat st;
        if (::stat(path, &st) == 0) {
            set_err("gp_rendezvous_id: '%s' already exists (left by an earlier run?); the path must be fresh", path);
            return GP_ESTATE;
        }
        int rc = gp_get_unique_id(unique_id);
        if (rc) return rc;
        const std::string tmp = std::string(path) + ".tmp." + std::to_string((long long)getpid());
        const int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0600);
        if (fd < 0) {
            set_err("gp_rendezvous_id: cannot create '%s': %s", tmp.c_str(), std::strerror(errno));
            return GP_EINVAL;
        }
        std::string blob(reinterpret_cast<const char*>(unique_id), N);
        blob += nonce;
        const bool ok = ::write(fd, blob.data(), blob.size()) == (ssize_t)blob.size() && ::fsync(fd) == 0;
        ::close(fd);
        if (!ok || ::rename(tmp.c_str(), path) != 0) {
            set_err("gp_rendezvous_id: cannot publish '%s': %s", path, std::strerror(errno));
            ::unlink(tmp.c_str());
            return GP_EINVAL;
        }
        return GP_OK;
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {  // wait for rank 0's file (with this launch's nonce)
        const int fd = ::open(path, O_RDONLY | O_CLOEXEC);
        if (fd >= 0) {
            char buf[128 + 65];
            const ssize_t got = ::read(fd, buf, sizeof buf);
            ::close(fd);
            if (got < (ssize_t)N) {
                set_err("gp_rendezvous_id: '%s' holds %zd bytes, expected %zu", path, got, N);
                return GP_EINVAL;
            }
            if (std::string(buf + N, (size_t)got - N) == nonce) {
                std::memcpy(unique_id, buf, N);
                return GP_OK;
            }
            // another launch's file: keep waiting for ours (rank 0 refuses to overwrite it,
            // so this ends at the timeout with the error below)
        }
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (timeout_ms >= 0 && ms >= timeout_ms) {
            set_err("gp_rendezvous_id: rank %d waited %d ms for rank 0's id at '%s'%s", rank, timeout_ms, path,
                    fd >= 0 ? " (the file there carries another launch's nonce)" : "");
            return GP_ESTATE;
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(5));
    }
}

int gp_create_rank(const gp_config* cfg, int32_t rank, int32_t world, const uint8_t unique_id[128], gp_sim** out) {
    if (!cfg || !out || world < 1 || rank < 0 || rank >= world) {
        set_err("gp_create_rank: bad argument (rank %d, world %d)", rank, world);
        return GP_EINVAL;
    }
    bool force = false;
    // GP_FORCE_RCCL=1 (experiments): a one-rank RCCL communicator (test of the RCCL transport
    // on a single GPU: init, bookkeeping all-reduce, teardown)
    if (const char* e = exp_env("GP_FORCE_RCCL")) force = e[0] == '1';
    if (world == 1 && !force) return create_common(cfg, MODE_SINGLE, 1, 0, nullptr, out);
    if (!unique_id) {
        set_err("gp_create_rank: null unique id");
        return GP_EINVAL;
    }
    return create_common(cfg, MODE_RCCL, world, rank, unique_id, out);
}

int64_t gp_step(gp_sim* s, int64_t nrounds, int64_t* alerts_out) {
    if (!s) {
        set_err("gp_step: null handle");
        return GP_EINVAL;
    }
    if (nrounds < 0) {
        set_err("gp_step: negative round count");
        return GP_EINVAL;
    }
    if (hipSetDevice(s->device) != hipSuccess) {
        set_err("hipSetDevice failed");
        return GP_EHIP;
    }
    int64_t executed = 0;
    while (executed < nrounds && !s->done) {
        int64_t batch = std::min<int64_t>(nrounds - executed, BATCH);
        if (s->cfg.max_rounds > 0) batch = std::min<int64_t>(batch, s->cfg.max_rounds - s->rounds_done);
        if (batch <= 0) break;
        const bool block = s->slab[0].S.kernel == KERNEL_BLOCK;
        if (block) {  // the whole batch in one cooperative launch (gp_block.hip)
            const DevState& S = s->slab[0].S;
            if (s->timing) HIP_TRY(hipEventRecord(s->ev[0], s->stream));
            const hipError_t le = launch_round_block(S, S.bplan, (uint32_t)s->rounds_done, (uint32_t)batch, S.bface,
                                                     S.bscratch, s->stream);
            if (le != hipSuccess) {
                set_err("the LDS-resident round kernel's cooperative launch failed: %s (its %u workgroups must be "
                        "resident on the device at once)",
                        hipGetErrorString(le), S.bplan.nbx * S.bplan.nby * S.bplan.nbz);
                return GP_EHIP;
            }
            if (s->timing) HIP_TRY(hipEventRecord(s->ev[1], s->stream));
            unsigned int flags[2] = {0, 0};
            HIP_TRY(hipMemcpyAsync(flags, S.bscratch, sizeof flags, hipMemcpyDeviceToHost, s->stream));
            HIP_TRY(hipStreamSynchronize(s->stream));
            if (flags[1]) {
                set_err("the LDS-resident round kernel's grid barrier timed out (a workgroup never arrived); "
                        "the rounds of this batch are invalid");
                return GP_ESTATE;
            }
        } else {
            const size_t nl = round_launches(s);
            for (int64_t k = 0; k < batch; ++k) {
                const uint32_t r = (uint32_t)(s->rounds_done + k);
                int rc = launch_round(s, r, s->timing ? &s->ev[2 * nl * k] : nullptr);
                if (rc) return rc;
            }
        }
        HIP_TRY(hipMemcpyAsync(s->host_ctl, s->slab[0].S.ctl, sizeof(Ctl), hipMemcpyDeviceToHost, s->stream));
        HIP_TRY(hipStreamSynchronize(s->stream));
        const Ctl& hc = *s->host_ctl;
        if (hc.tiny) {
            set_err("a push-sum (s, w) value fell below 2^-1020, where the tile kernel's fused fold "
                    "(v_fma_f64(m, 0.5, acc)) is no longer guaranteed to round like the specification's "
                    "acc + m * 0.5; the rounds of this batch are invalid");
            return GP_ESTATE;
        }
        if (hc.overflow) {
            set_err("message buffer overflow (an exchange buffer or a message bin exceeded its capacity = "
                    "expected + 12 sigma); the rounds of this batch are invalid");
            return GP_ESTATE;
        }
        int64_t cum = s->alerts_total, ex = 0;
        for (int64_t k = 0; k < batch; ++k) {
            const int64_t r = s->rounds_done + k;
            const int64_t a = (int64_t)hc.hist[r % HIST];
            cum += a;
            if (alerts_out) alerts_out[executed + ex] = a;
            ++ex;
            if (cum >= s->T) break;
        }
        if (hc.done ? (cum != (int64_t)hc.alerts_total || cum < s->T)
                    : (ex != batch || cum != (int64_t)hc.alerts_total)) {
            set_err("round bookkeeping mismatch (device %llu alerts, host %lld)", hc.alerts_total, (long long)cum);
            return GP_ESTATE;
        }
        if (s->timing && block) {  // one launch for the batch: its time over the rounds it ran
            float ms = 0.f;
            HIP_TRY(hipEventElapsedTime(&ms, s->ev[0], s->ev[1]));
            s->kernel_ms += ms;
            s->launches += ex;
        } else if (s->timing) {  // per round: the sum over its round kernel launches
            const size_t nl = round_launches(s);
            for (int64_t k = 0; k < ex; ++k) {
                for (size_t h = 0; h < nl; ++h) {
                    float ms = 0.f;
                    HIP_TRY(hipEventElapsedTime(&ms, s->ev[2 * (nl * k + h)], s->ev[2 * (nl * k + h) + 1]));
                    s->kernel_ms += ms;
                }
                ++s->launches;
            }
        }
        s->rounds_done += ex;
        s->alerts_total = cum;
        s->done = hc.done != 0;
        executed += ex;
        if (s->mode != MODE_RCCL && exp_env("GP_CHECK_CLOSE")) {  // tests: recount the alerts from the state
            Scratch tmp;
            unsigned long long* d = nullptr;
            HIP_TRY(tmp.alloc(&d, 1));
            HIP_TRY(hipMemsetAsync(d, 0, sizeof(unsigned long long), s->stream));
            for (Slab& sl : s->slab) {
                const DevState& S = sl.S;
                const uint8_t* nb = nullptr;
                if (S.alg == PUSHSUM) nb = (S.topo == FULL ? S.nb[0] : S.nb[s->rounds_done & 1]) + (S.lo - S.base);
                HIP_TRY(launch_count_alerted(nb, S.alg == PUSHSUM ? nullptr : S.c, S.nloc, d, s->grid, s->stream));
            }
            unsigned long long h = 0;
            HIP_TRY(hipMemcpyAsync(&h, d, sizeof h, hipMemcpyDeviceToHost, s->stream));
            HIP_TRY(hipStreamSynchronize(s->stream));
            if ((int64_t)h != cum) {
                set_err("round close check: %llu alerted nodes in the state, %lld counted by the round closes", h,
                        (long long)cum);
                return GP_ESTATE;
            }
        }
    }
    return executed;
}

int gp_run(gp_sim* s, gp_result* out) {
    if (!s || !out) {
        set_err("gp_run: null argument");
        return GP_EINVAL;
    }
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipStreamSynchronize(s->stream));
    const int64_t r0 = s->rounds_done;
    const auto t0 = std::chrono::steady_clock::now();
    while (!s->done) {
        if (s->cfg.max_rounds > 0 && s->rounds_done >= s->cfg.max_rounds) break;
        int64_t n = gp_step(s, BATCH, nullptr);
        if (n < 0) return (int)n;
        if (n == 0) break;
    }
    const auto t1 = std::chrono::steady_clock::now();
    const double ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
    const int64_t rounds = s->rounds_done - r0;
    out->rounds = s->rounds_done;
    out->converged = s->alerts_total;
    out->population = s->P;
    out->threshold = s->T;
    out->elapsed_ms = ms;
    out->node_updates_per_s = ms > 0 ? (double)s->P * (double)rounds / (ms * 1e-3) : 0.0;
    out->hbm_bytes_alg = alg_bytes(s) * (double)s->P * (double)rounds;
    out->status = s->done ? GP_STATUS_CONVERGED : GP_STATUS_MAX_ROUNDS;
    out->reserved = 0;
    return GP_OK;
}

int gp_read_state(gp_sim* s, int64_t first, int64_t count, int32_t* c, double* sv, double* wv, uint8_t* flags) {
    if (!s) {
        set_err("gp_read_state: null handle");
        return GP_EINVAL;
    }
    if (first < 0 || count < 0 || first + count > s->P) {
        set_err("gp_read_state: range [%lld, %lld) outside [0, %lld)", (long long)first, (long long)(first + count),
                (long long)s->P);
        return GP_EINVAL;
    }
    if (count == 0) return GP_OK;
    if (s->mode == MODE_RCCL) {
        const Slab& sl = s->slab[0];
        if (first < sl.S.lo || first + count > sl.hi) {
            set_err("gp_read_state: range [%lld, %lld) outside this rank's slab [%u, %u)", (long long)first,
                    (long long)(first + count), sl.S.lo, sl.hi);
            return GP_EINVAL;
        }
    }
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipStreamSynchronize(s->stream));
    const int cur = (int)(s->rounds_done & 1);
    for (const Slab& sl : s->slab) {
        const DevState& S = sl.S;
        const int64_t a = std::max<int64_t>(first, S.lo), b = std::min<int64_t>(first + count, sl.hi);
        if (a >= b) continue;
        const int64_t n = b - a, q0 = a - first;
        if (S.alg == PUSHSUM) {
            std::vector<double2> sw((size_t)n);
            std::vector<uint8_t> nb((size_t)n);
            HIP_TRY(hipMemcpy(sw.data(), S.sw[cur] + (a - S.base), sizeof(double2) * n, hipMemcpyDeviceToHost));
            const uint8_t* nbsrc = S.topo == FULL ? S.nb[0] : S.nb[cur];
            HIP_TRY(hipMemcpy(nb.data(), nbsrc + (a - S.base), n, hipMemcpyDeviceToHost));
            for (int64_t q = 0; q < n; ++q) {
                if (c) c[q0 + q] = 0;
                if (sv) sv[q0 + q] = sw[q].x;
                if (wv) wv[q0 + q] = sw[q].y;
                if (flags) {
                    const uint8_t bb = nb[q];
                    flags[q0 + q] = (uint8_t)(((bb & B_ACTIVE) ? 1 : 0) | ((bb & B_CONV) ? 2 : 0) |
                                              (((bb >> CNT_SHIFT) & 3) << 2));
                }
            }
        } else {
            std::vector<int32_t> cc((size_t)n);
            HIP_TRY(hipMemcpy(cc.data(), S.c + (a - S.lo), sizeof(int32_t) * n, hipMemcpyDeviceToHost));
            for (int64_t q = 0; q < n; ++q) {
                const int64_t i = a + q;
                const int32_t ci = cc[q];
                if (c) c[q0 + q] = ci;
                if (sv) sv[q0 + q] = 0.0;
                if (wv) wv[q0 + q] = 0.0;
                if (flags) {
                    const bool act = (i == (int64_t)S.seed_node || ci >= 1) && ci <= 10;
                    flags[q0 + q] = (uint8_t)((act ? 1 : 0) | (ci >= 11 ? 2 : 0));
                }
            }
        }
    }
    return GP_OK;
}

int gp_neighbors(gp_sim* s, int64_t node, int64_t* out, int64_t cap) {
    if (!s || node < 0 || node >= s->P) {
        set_err("gp_neighbors: bad handle or node");
        return GP_EINVAL;
    }
    const DevState& S = s->slab[0].S;
    const uint32_t j = (uint32_t)node;
    std::vector<int64_t> nb;
    if (S.topo == FULL) {
        const int64_t deg = s->P - 1;
        for (int64_t k = 0; k < std::min(deg, cap); ++k) out[k] = full_target(j, (uint32_t)k);
        return (int)deg;
    }
    uint32_t mask = S.topo == LINE ? present_mask<LINE>(j, S.G) : present_mask<GRID3D>(j, S.G);
    for (uint32_t d = 0; d < 6; ++d)
        if (mask & (1u << d)) nb.push_back(S.topo == LINE ? nbr<LINE>(j, d, S.G) : nbr<GRID3D>(j, d, S.G));
    if (S.topo == IMP3D) nb.push_back(uniform(S.k0, S.k1, S_TOPO, j, 0, S.G.P - 1));  // Program.fs:259
    for (int64_t k = 0; k < std::min<int64_t>((int64_t)nb.size(), cap); ++k) out[k] = nb[(size_t)k];
    return (int)nb.size();
}

int gp_get_info(gp_sim* s, gp_info* o) {
    if (!s || !o) {
        set_err("gp_get_info: null argument");
        return GP_EINVAL;
    }
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipMemcpyAsync(s->host_ctl, s->slab[0].S.ctl, sizeof(Ctl), hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    o->population = s->P;
    o->threshold = s->T;
    o->grid = s->g;
    o->seed_node = s->slab[0].S.seed_node;
    o->rounds = s->rounds_done;
    o->alerts_total = s->alerts_total;
    o->active = s->slab[0].S.alg == PUSHSUM ? (int64_t)s->host_ctl->active_total : -1;
    o->topology = s->cfg.topology;
    o->algorithm = s->cfg.algorithm;
    o->device = s->device;
    o->num_gpus = s->world;
    if (s->mode == MODE_RCCL) {
        o->slab_first = s->slab[0].S.lo;
        o->slab_count = s->slab[0].S.nloc;
    } else {
        o->slab_first = 0;
        o->slab_count = s->P;
    }
    return GP_OK;
}

#ifdef GP_EXPERIMENTS
// Experiments build, tests: round kernel launches per round (DevState::rregions), -1 without a handle.
int gp_debug_round_regions(gp_sim* s) { return s && !s->slab.empty() ? (int)s->slab[0].S.rregions : -1; }
#endif

int gp_sync(gp_sim* s) {
    if (!s) {
        set_err("gp_sync: null handle");
        return GP_EINVAL;
    }
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipStreamSynchronize(s->stream));
    return GP_OK;
}

int gp_kernel_stats(gp_sim* s, double* total_ms, int64_t* launches, char* name, int32_t name_cap, int32_t reset) {
    if (!s) {
        set_err("gp_kernel_stats: null handle");
        return GP_EINVAL;
    }
    if (total_ms) *total_ms = s->kernel_ms;
    if (launches) *launches = s->launches;
    if (name && name_cap > 0) std::snprintf(name, (size_t)name_cap, "%s", bulk_kernel_name(s->slab[0].S));
    if (reset) {
        s->kernel_ms = 0.0;
        s->launches = 0;
    }
    return GP_OK;
}

double gp_alg_bytes_per_node(gp_sim* s) { return s ? alg_bytes(s) : 0.0; }

void gp_destroy(gp_sim* s) {
    if (!s) return;
    (void)hipSetDevice(s->device);
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    if (s->xstream) (void)hipStreamSynchronize(s->xstream);
    for (auto& e : s->ev) (void)hipEventDestroy(e);
    for (int h = 0; h < XMAXH; ++h) {
        if (s->ev_send[h]) (void)hipEventDestroy(s->ev_send[h]);
        if (s->ev_xfer[h]) (void)hipEventDestroy(s->ev_xfer[h]);
    }
    if (s->comm) (void)ncclCommDestroy(s->comm);
    free_all(s);
    if (s->host_ctl) (void)hipHostFree(s->host_ctl);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    if (s->xstream) (void)hipStreamDestroy(s->xstream);
    delete s;
}

}  // extern "C"
