// gp_wave.hip -- wave-autonomous per-round kernels for line / 3D / Imp3D (gfx950).
//
// One synchronous round of SRS v1 in PULL form.  Every wave
// owns whole 256-node chunks (4 nodes per lane, node = c0 + 64k + lane) and
// never meets another wave at a barrier, so 8 waves per SIMD keep their loads
// in flight independently:
//
//   1. own (s, w), own node byte, the six lattice neighbours' direction bytes
//      and the chunk's in-list offsets are loaded up front (coalesced: every
//      load instruction covers 64 consecutive nodes);
//   2. Imp3D: one flattened, lane-balanced sweep over the chunk's in-edges
//      (receiver-sorted CSR) decides "the sender used its random edge this
//      round" -- Philox of the sender once every node is active, the
//      ballot-packed bitmap during activation, the exchange tag for senders on
//      another rank -- and gathers the senders' (s, w) with all loads of the
//      sweep in flight together; messages are parked in wave-private LDS;
//   3. per node: gather (s, w) of the lattice neighbours that chose this node,
//      fold in canonical order (own half, lattice slots, random edges by
//      ascending sender), ratio test, draw the next round's direction.
//
// Slab-aware: node ids are global; a rank owns [lo, lo + nloc) and its node
// arrays start at id `base` (= lo - halo), so lattice neighbours in the
// adjacent rank's boundary plane read the halo copy the exchange left there.
// Built with -ffp-contract=off: the fold must round exactly like the oracle.
#include "gp_wavecommon.hpp"

namespace gp {
namespace {
constexpr int WNPT = 4;                 // nodes per lane per chunk
constexpr int CH = 64 * WNPT;           // nodes per chunk
}  // namespace

// The chunk kernels are an experiment variant (measured slower than the tiled
// kernels): built into the experiments library only.
#ifdef GP_EXPERIMENTS
namespace {
using namespace wk;

// Did sender i use its random edge in round r?  (i local to this rank.)
__device__ __forceinline__ bool local_sent_random(const WaveArgs& a, uint32_t i, uint32_t r, bool all_active,
                                                  uint32_t stream) {
    if (all_active) {
        const uint32_t di = popc6(present_mask<IMP3D>(i, a.G)) + 1u;
        return uniform(a.k0, a.k1, stream, i, r, di) == di - 1u;
    }
    return (a.rbc[(i >> 6) - (a.lo >> 6)] >> (i & 63)) & 1ull;
}

}  // namespace

// ---------------------------------------------------------------- push-sum
template <int TOPO>
__global__ __launch_bounds__(BULK_THREADS) void k_ps_wave(WaveArgs a, uint32_t r) {
    __shared__ WaveLds Lw[WPB];
    Ctl* ctl = a.ctl;
    if (ld_agent(&ctl->done)) return;
    const bool all_active = ld_agent(&ctl->all_active) != 0;
    const int lane = threadIdx.x & 63;
    WaveLds& L = Lw[threadIdx.x >> 6];
    const double2* __restrict__ swc = a.swc;
    double2* __restrict__ swn = a.swn;
    const uint8_t* __restrict__ nbc = a.nbc;
    const Geom G = a.G;
    const uint32_t lo = a.lo, nloc = a.nloc, base = a.base;
    constexpr uint32_t ND = TOPO == LINE ? 2 : 6;
    uint32_t alerts = 0, newly = 0;

    const uint32_t wg = blockIdx.x * WPB + (threadIdx.x >> 6), wn = gridDim.x * WPB;
    for (uint32_t ch = wg; ch < a.nchunks; ch += wn) {
        // chunks sit on global multiples of CH (64-aligned ballot words); the
        // slab's first and last chunk may be partial: valid ids [cv, c1)
        const uint32_t c0 = ((lo / CH) + ch) * CH;
        const uint32_t cv = max(lo, c0);
        const uint32_t c1 = min(lo + nloc, c0 + CH);
        // ---- 1. loads that depend on nothing
        double2 own[WNPT];
        uint32_t bown[WNPT], from[WNPT], off[WNPT];
#pragma unroll
        for (int k = 0; k < WNPT; ++k) {
            const uint32_t j = c0 + k * 64 + lane;
            const bool valid = j >= cv && j < c1;
            const uint32_t jl = (valid ? j : cv) - base;
            own[k] = swc[jl];
            bown[k] = nbc[jl];
            const uint32_t mask = valid ? present_mask<TOPO>(j, G) : 0u;
            uint32_t f = 0;
#pragma unroll
            for (uint32_t d = 0; d < ND; ++d) {
                const bool has = (mask >> d) & 1u;
                const uint32_t nl = (has ? nbr<TOPO>(j, d, G) : cv) - base;
                const uint32_t nbd = nbc[nl] & DIR_MASK;
                f |= (has && nbd == (d ^ 1u)) ? (1u << d) : 0u;
            }
            from[k] = f;
            if (TOPO == IMP3D) off[k] = a.in_off[min(max(j, cv), c1) - lo];
        }
        // ---- 2. Imp3D in-edges: flattened decide + gather, parked in LDS
        uint32_t e0 = 0, e1 = 0;
        if (TOPO == IMP3D) {
            e0 = __builtin_amdgcn_readlane(off[0], 0);
            e1 = a.in_off[c1 - lo];
            const uint32_t nst = min(e1 - e0, ECAP);
            uint32_t nmsg = 0;
            for (uint32_t q0 = 0; q0 < nst; q0 += EU * 64) {
                uint32_t src[EU];
                bool sent[EU];
                double2 val[EU];
#pragma unroll
                for (int m = 0; m < EU; ++m) {
                    const uint32_t q = q0 + m * 64 + lane;
                    src[m] = q < nst ? a.in_src[e0 + q] : lo;
                }
#pragma unroll
                for (int m = 0; m < EU; ++m) {
                    const uint32_t q = q0 + m * 64 + lane;
                    const uint32_t i = src[m];
                    bool s = false;
                    if (q < nst) {
                        if (i - lo >= nloc) s = a.rtag[e0 + q] == r;  // sender on another rank
                        else s = local_sent_random(a, i, r, all_active, S_PUSHSUM);
                    }
                    sent[m] = s;
                }
#pragma unroll
                for (int m = 0; m < EU; ++m) {
                    const uint32_t q = q0 + m * 64 + lane;
                    const uint32_t i = src[m];
                    val[m] = make_double2(0.0, 0.0);
                    if (sent[m]) val[m] = (i - lo >= nloc) ? a.rmsg[e0 + q] : swc[i - base];
                }
#pragma unroll
                for (int m = 0; m < EU; ++m) {
                    const uint32_t q = q0 + m * 64 + lane;
                    const unsigned long long bal = __ballot(sent[m]);
                    const uint32_t slot = nmsg + lane_prefix(bal);
                    nmsg += (uint32_t)__popcll(bal);
                    if (q < nst) L.code[q] = !sent[m] ? CODE_NONE : (slot < MCAP ? slot : CODE_GLOBAL);
                    if (sent[m] && slot < MCAP) L.msg[slot] = val[m];
                }
            }
            wave_lds_sync();
        }
        // ---- 3. per node: lattice gathers, fold, ratio test, next direction
#pragma unroll
        for (int k = 0; k < WNPT; ++k) {
            const uint32_t j = c0 + k * 64 + lane;
            const bool valid = j >= cv && j < c1;
            const uint32_t mask = valid ? present_mask<TOPO>(j, G) : 0u;
            const uint32_t deg = popc6(mask) + (TOPO == IMP3D ? 1u : 0u);
            const uint32_t b = bown[k];
            bool active = (b & B_ACTIVE) != 0;
            const double2 sv = own[k];
            const bool halve = active && deg > 0;
            double acc_s = halve ? sv.x * 0.5 : sv.x;
            double acc_w = halve ? sv.y * 0.5 : sv.y;
            const uint32_t f = from[k];
            double2 m[ND];
#pragma unroll
            for (uint32_t d = 0; d < ND; ++d) {
                const bool s = (f >> d) & 1u;
                const uint32_t nl = (s ? nbr<TOPO>(j, d, G) : cv) - base;
                m[d] = s ? swc[nl] : make_double2(0.0, 0.0);
            }
#pragma unroll
            for (uint32_t d = 0; d < ND; ++d) {
                if ((f >> d) & 1u) {
                    acc_s = acc_s + m[d].x * 0.5;
                    acc_w = acc_w + m[d].y * 0.5;
                }
            }
            bool recv = f != 0;
            if (TOPO == IMP3D) {
                const uint32_t eb = off[k];
                const uint32_t nx = k + 1 < WNPT ? __builtin_amdgcn_readlane(off[k + 1 < WNPT ? k + 1 : k], 0) : e1;
                uint32_t ee = __shfl_down(eb, 1, 64);
                if (lane == 63) ee = nx;
                for (uint32_t e = eb; e < ee; ++e) {
                    const uint32_t q = e - e0;
                    bool s;
                    double2 mi = make_double2(0.0, 0.0);
                    if (q < ECAP) {
                        const uint32_t code = L.code[q];
                        s = code != CODE_NONE;
                        if (code < MCAP) {
                            mi = L.msg[code];
                        } else if (s) {  // parked-message overflow: reload
                            const uint32_t i = a.in_src[e];
                            mi = (i - lo >= nloc) ? a.rmsg[e] : swc[i - base];
                        }
                    } else {  // beyond the staged edges (chunk in-degree > ECAP): decide here
                        const uint32_t i = a.in_src[e];
                        if (i - lo >= nloc) {
                            s = a.rtag[e] == r;
                            if (s) mi = a.rmsg[e];
                        } else {
                            s = local_sent_random(a, i, r, all_active, S_PUSHSUM);
                            if (s) mi = swc[i - base];
                        }
                    }
                    if (s) {
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
            uint32_t dir = DIR_NONE;
            if (active && deg > 0) dir = slot_to_dir(mask, uniform(a.k0, a.k1, S_PUSHSUM, j, r + 1, deg));
            if (valid) {
                const uint32_t jl = j - base;
                a.nbn[jl] = (uint8_t)(flags | dir);
                swn[jl] = make_double2(acc_s, acc_w);
            }
            if (TOPO == IMP3D && !all_active) {
                const unsigned long long bits = __ballot(valid && dir == DIR_RANDOM);
                if (lane == 0) {  // the slab's first chunk may start below lo: no word there
                    const int64_t wi = (int64_t)((c0 + k * 64) >> 6) - (int64_t)(lo >> 6);
                    if (wi >= 0) a.rbn[wi] = bits;
                }
            }
            __builtin_amdgcn_sched_barrier(0);  // one node's gathers live at a time (VGPR budget)
        }
        if (TOPO == IMP3D) wave_lds_sync();  // the next chunk's sweep overwrites L
    }
    block_add2(alerts, newly, &ctl->round_alerts, &ctl->round_active);
}

// ---------------------------------------------------------------- gossip
// Deliveries to j = lattice senders pointing here + Imp3D random-edge senders
// + the injector; all dropped if j was converged at round start (Program.fs:87).
template <int TOPO>
__global__ __launch_bounds__(BULK_THREADS) void k_gossip_wave(WaveArgs a, uint32_t r) {
    __shared__ WaveLds Lw[WPB];
    Ctl* ctl = a.ctl;
    if (ld_agent(&ctl->done)) return;
    const long long inj = ld_agent(&ctl->inj_target);
    const int lane = threadIdx.x & 63;
    WaveLds& L = Lw[threadIdx.x >> 6];
    const uint8_t* __restrict__ nbc = a.nbc;
    const Geom G = a.G;
    const uint32_t lo = a.lo, nloc = a.nloc, base = a.base;
    constexpr uint32_t ND = TOPO == LINE ? 2 : 6;
    uint8_t* codes = reinterpret_cast<uint8_t*>(L.code);
    uint32_t alerts = 0;

    const uint32_t wg = blockIdx.x * WPB + (threadIdx.x >> 6), wn = gridDim.x * WPB;
    for (uint32_t ch = wg; ch < a.nchunks; ch += wn) {
        // chunks sit on global multiples of CH (64-aligned ballot words); the
        // slab's first and last chunk may be partial: valid ids [cv, c1)
        const uint32_t c0 = ((lo / CH) + ch) * CH;
        const uint32_t cv = max(lo, c0);
        const uint32_t c1 = min(lo + nloc, c0 + CH);
        int32_t c0v[WNPT];
        uint32_t inc[WNPT], off[WNPT];
#pragma unroll
        for (int k = 0; k < WNPT; ++k) {
            const uint32_t j = c0 + k * 64 + lane;
            const bool valid = j >= cv && j < c1;
            c0v[k] = a.c[(valid ? j : cv) - lo];
            const uint32_t mask = valid ? present_mask<TOPO>(j, G) : 0u;
            uint32_t n = (valid && (long long)j == inj) ? 1u : 0u;
#pragma unroll
            for (uint32_t d = 0; d < ND; ++d) {
                const bool has = (mask >> d) & 1u;
                const uint32_t nl = (has ? nbr<TOPO>(j, d, G) : cv) - base;
                n += (has && (nbc[nl] & DIR_MASK) == (d ^ 1u)) ? 1u : 0u;
            }
            inc[k] = n;
            if (TOPO == IMP3D) off[k] = a.in_off[min(max(j, cv), c1) - lo];
        }
        uint32_t e0 = 0, e1 = 0;
        if (TOPO == IMP3D) {
            e0 = __builtin_amdgcn_readlane(off[0], 0);
            e1 = a.in_off[c1 - lo];
            const uint32_t nst = min(e1 - e0, ECAP);
            for (uint32_t q0 = 0; q0 < nst; q0 += EU * 64) {
                uint32_t src[EU];
#pragma unroll
                for (int m = 0; m < EU; ++m) {
                    const uint32_t q = q0 + m * 64 + lane;
                    src[m] = q < nst ? a.in_src[e0 + q] : lo;
                }
#pragma unroll
                for (int m = 0; m < EU; ++m) {
                    const uint32_t q = q0 + m * 64 + lane;
                    if (q < nst) {
                        const uint32_t i = src[m];
                        bool s;
                        if (i - lo >= nloc) s = a.rtag[e0 + q] == r;
                        else s = local_sent_random(a, i, r, false, S_GOSSIP);
                        codes[q] = (uint8_t)s;
                    }
                }
            }
            wave_lds_sync();
        }
#pragma unroll
        for (int k = 0; k < WNPT; ++k) {
            const uint32_t j = c0 + k * 64 + lane;
            const bool valid = j >= cv && j < c1;
            const uint32_t mask = valid ? present_mask<TOPO>(j, G) : 0u;
            uint32_t n = inc[k];
            if (TOPO == IMP3D) {
                const uint32_t eb = off[k];
                const uint32_t nx = k + 1 < WNPT ? __builtin_amdgcn_readlane(off[k + 1 < WNPT ? k + 1 : k], 0) : e1;
                uint32_t ee = __shfl_down(eb, 1, 64);
                if (lane == 63) ee = nx;
                for (uint32_t e = eb; e < ee; ++e) {
                    const uint32_t q = e - e0;
                    if (q < ECAP) {
                        n += codes[q];
                    } else {
                        const uint32_t i = a.in_src[e];
                        n += (i - lo >= nloc) ? (a.rtag[e] == r ? 1u : 0u)
                                              : (local_sent_random(a, i, r, false, S_GOSSIP) ? 1u : 0u);
                    }
                }
            }
            int32_t c1v = c0v[k];
            if (valid && c1v < (int32_t)GOSSIP_DONE && n) {
                c1v += (int32_t)n;
                a.c[j - lo] = c1v;
                alerts += c1v > 10;  // the receipt that finds rumours == 10 (Program.fs:92-94)
            }
            uint32_t dir = DIR_NONE;
            const bool active = valid && ((j == a.seed_node) || c1v >= 1) && c1v <= 10;
            if (active) {
                const uint32_t deg = popc6(mask) + (TOPO == IMP3D ? 1u : 0u);
                if (deg > 0) dir = slot_to_dir(mask, uniform(a.k0, a.k1, S_GOSSIP, j, r + 1, deg));
            }
            if (valid) a.nbn[j - base] = (uint8_t)dir;
            if (TOPO == IMP3D) {
                const unsigned long long bits = __ballot(valid && dir == DIR_RANDOM);
                if (lane == 0) {  // the slab's first chunk may start below lo: no word there
                    const int64_t wi = (int64_t)((c0 + k * 64) >> 6) - (int64_t)(lo >> 6);
                    if (wi >= 0) a.rbn[wi] = bits;
                }
            }
        }
        if (TOPO == IMP3D) wave_lds_sync();
    }
    block_add2(alerts, 0u, &ctl->round_alerts, nullptr);
}

// Resident 256-thread blocks per CU of the round kernel (grid = this x CUs: one
// continuous sweep, so the x-1 plane a chunk gathers from was just streamed).
int wave_blocks_per_cu(int topo, int alg) {
    const void* f;
    if (alg == PUSHSUM)
        f = topo == LINE ? (const void*)k_ps_wave<LINE> : topo == GRID3D ? (const void*)k_ps_wave<GRID3D>
                                                                        : (const void*)k_ps_wave<IMP3D>;
    else
        f = topo == LINE ? (const void*)k_gossip_wave<LINE>
                         : topo == GRID3D ? (const void*)k_gossip_wave<GRID3D> : (const void*)k_gossip_wave<IMP3D>;
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, f, BULK_THREADS, 0) != hipSuccess || n < 1) n = 1;
    return n;
}

hipError_t launch_round_wave(const WaveArgs& a, int topo, int alg, uint32_t round, int grid, hipStream_t st) {
    const dim3 g(grid), b(BULK_THREADS);
    if (alg == PUSHSUM) {
        switch (topo) {
            case LINE: hipLaunchKernelGGL(k_ps_wave<LINE>, g, b, 0, st, a, round); break;
            case GRID3D: hipLaunchKernelGGL(k_ps_wave<GRID3D>, g, b, 0, st, a, round); break;
            default: hipLaunchKernelGGL(k_ps_wave<IMP3D>, g, b, 0, st, a, round); break;
        }
    } else {
        switch (topo) {
            case LINE: hipLaunchKernelGGL(k_gossip_wave<LINE>, g, b, 0, st, a, round); break;
            case GRID3D: hipLaunchKernelGGL(k_gossip_wave<GRID3D>, g, b, 0, st, a, round); break;
            default: hipLaunchKernelGGL(k_gossip_wave<IMP3D>, g, b, 0, st, a, round); break;
        }
    }
    return hipGetLastError();
}
#endif  // GP_EXPERIMENTS

uint32_t wave_chunks(uint32_t lo, uint32_t nloc) {
    return (uint32_t)(((uint64_t)lo + nloc + CH - 1) / CH - lo / CH);
}

WaveArgs make_wave_args(const DevState& S, uint32_t round) {
    const int cur = round & 1;
    WaveArgs a;
    a.swc = S.sw[cur];
    a.swn = S.sw[cur ^ 1];
    a.nbc = S.nb[cur];
    a.nbn = S.nb[cur ^ 1];
    a.rbc = S.rbits[cur];
    a.rbn = S.rbits[cur ^ 1];
    a.in_off = S.in_off;
    a.in_src = S.in_src;
    a.rtag = S.rtag;
    a.rmsg = S.rmsg;
    a.c = S.c;
    a.rcnt = S.rcnt;
    a.rq_cur = S.rq[round & 1];
    a.rq_next = S.rq[(round + 1) & 1];
    a.rnd = S.rnd;
    a.ctl = S.ctl;
    a.G = S.G;
    a.k0 = S.k0;
    a.k1 = S.k1;
    a.seed_node = S.seed_node;
    a.lo = S.lo;
    a.nloc = S.nloc;
    a.base = S.base;
    a.nchunks = wave_chunks(S.lo, S.nloc);
    a.x_lo = a.x_hi = a.zsegs = a.yblocks = a.xs_len = a.nitems = 0;
    if (S.G.g2) {  // column kernels (3D / Imp3D)
        const uint32_t g = S.G.g;
        a.x_lo = S.lo / S.G.g2;
        a.x_hi = (S.lo + S.nloc) / S.G.g2;
        a.zsegs = (g + 63) / 64;
        a.yblocks = (g + 3) / 4;
        const uint32_t planes = a.x_hi - a.x_lo;
        const uint32_t xs = S.col_xsegs ? S.col_xsegs : 1u;
        a.xs_len = (planes + xs - 1) / xs;
        const uint32_t nseg = a.xs_len ? (planes + a.xs_len - 1) / a.xs_len : 0u;
        a.nitems = a.zsegs * a.yblocks * nseg;
    }
    return a;
}

}  // namespace gp
