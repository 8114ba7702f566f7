// gp_col.hip -- column-march round kernels for the 3D / Imp3D lattice (gfx950).
//
// Gossip: one synchronous round of SRS v1 in PULL form with 2.5-D
// blocking (push-sum runs the tile kernel, gp_round.hip).  A wave owns a patch of 4 y-rows x 64 z-columns (one node per lane
// and row; node id = x*g^2 + y*g + z, lanes = consecutive z, so every row of a
// patch is one coalesced 64-node segment) and marches it along x through its
// x-segment.  Planes x and x+1 of the patch stay in registers and plane x+2 is
// prefetched a step ahead, so of the six lattice senders of a node
//   x+1 and (inside the patch) y+-1 are register selects,
//   x-1 was streamed by this same wave one step ago (L2), and
//   z+-1 sit in the lines this wave just loaded (L1),
// and only the two y-halo rows touch another wave's data.  Per node and round
// the compulsory stream is the rumour counter + node byte in and out; the
// lattice costs no HBM traffic of its own.  Imp3D random-edge deliveries are
// integer counts, so their order is free: a sender whose next direction is its
// random edge counts the rumour at its target a round ahead (rq, an atomic) when
// the target is on this rank; for a target on another rank it sets the edge's bit
// in the send bitmap, and the target's rank adds the rumour (k_apply_bits,
// gp_xchg.hip).  No per-edge pass runs.
//
// Work items (patch, x-segment) are dealt XCD-contiguously: the waves of one
// XCD own one y-band of every plane, so y-halo rows come from the XCD's L2.
// Built with -ffp-contract=off: the fold must round exactly like the oracle.
#include "gp_wavecommon.hpp"

// gossip column kernel: waves per SIMD (measured 5..7 with the batched step loads,
// profiles/r02/col_batch/: Imp3D best at 5, 3D at 7)
#define GP_COL_MINW(TOPO) ((TOPO) == IMP3D ? 5 : 7)
// wave priority raised (s_setprio 2) while a column step issues its loads, dropped for the
// step's ALU work (as the push-sum tile kernel).  C3, same box, alternated: 0.596-0.603 ->
// 0.589-0.590 ms/round (profiles/r04/setprio_c3c4.txt)
constexpr int COL_PRIO = 2;

namespace gp {
namespace {

using namespace wk;
constexpr int NR = 4;  // y rows per patch

// XCD-contiguous deal of n work items over the grid's waves (speed only).
__device__ __forceinline__ void item_range(uint32_t n, uint32_t& it, uint32_t& end, uint32_t& step) {
    const uint32_t wid = threadIdx.x >> 6;
    if ((gridDim.x & 7) == 0) {
        const uint32_t xcd = blockIdx.x & 7;
        it = (uint32_t)((uint64_t)n * xcd / 8) + (blockIdx.x >> 3) * WPB + wid;
        end = (uint32_t)((uint64_t)n * (xcd + 1) / 8);
        step = (gridDim.x >> 3) * WPB;
    } else {
        it = blockIdx.x * WPB + wid;
        end = n;
        step = gridDim.x * WPB;
    }
}

__device__ __forceinline__ uint32_t byte_of(uint32_t packed, int k) { return (packed >> (8 * k)) & 0xFFu; }

}  // namespace

// ---------------------------------------------------------------- gossip
// Deliveries to j = lattice senders pointing here + Imp3D random-edge senders
// + the injector; all dropped if j was converged at round start (Program.fs:87).
// REMOTE (Imp3D slabs of a multi-rank run): a random-edge target on another rank gets
// its rumour through the send bitmap (a.rtg names the bit, gp_xchg.hpp).
template <int TOPO, bool REMOTE>
__global__ __launch_bounds__(BULK_THREADS, GP_COL_MINW(TOPO)) void k_gossip_col(WaveArgs a, uint32_t r) {
    Ctl* ctl = a.ctl;
    if (ld_agent(&ctl->done)) return;
    const long long inj = ld_agent(&ctl->inj_target);
    const int lane = threadIdx.x & 63;
    const uint8_t* __restrict__ nbc = a.nbc;
    const uint32_t g = a.G.g, g2 = a.G.g2, base = a.base, lo = a.lo;
    uint32_t alerts = 0;

    uint32_t it, it_end, it_step;
    item_range(a.nitems, it, it_end, it_step);
    for (; it < it_end; it += it_step) {
        const uint32_t zs = it % a.zsegs;
        const uint32_t t = it / a.zsegs;
        const uint32_t yb = t % a.yblocks;
        const uint32_t xa = a.x_lo + (t / a.yblocks) * a.xs_len;
        const uint32_t xb = min(a.x_hi, xa + a.xs_len);
        const uint32_t z = zs * 64 + (uint32_t)lane;
        const uint32_t y0 = yb * NR;
        const bool zv = z < g;
        bool rv[NR];
        uint32_t yo[NR], myz[NR];
#pragma unroll
        for (int k = 0; k < NR; ++k) {
            const uint32_t y = y0 + k;
            rv[k] = zv && y < g;
            yo[k] = rv[k] ? y * g + z : 0u;
            myz[k] = (y + 1 < g ? 4u : 0u) | (y > 0 ? 8u : 0u) | (z + 1 < g ? 16u : 0u) | (z > 0 ? 32u : 0u);
        }
        // planes xa - 1, xa, xa + 1 of the patch (unconditional loads, pinned, then masked:
        // see the x-step below)
        uint32_t pb = 0, cb = 0, nb = 0;
        {
            uint32_t lp[NR], lc[NR], ln[NR];
#pragma unroll
            for (int k = 0; k < NR; ++k) {
                const uint32_t jl = xa * g2 + yo[k] - base;
                lc[k] = nbc[jl];
                lp[k] = nbc[xa > 0 ? jl - g2 : jl];
                ln[k] = nbc[xa + 1 < g ? jl + g2 : jl];
            }
#pragma unroll
            for (int k = 0; k < NR; ++k) asm volatile("" : "+v"(lc[k]), "+v"(lp[k]), "+v"(ln[k]));
#pragma unroll
            for (int k = 0; k < NR; ++k) {
                cb |= (rv[k] ? lc[k] : (uint32_t)DIR_NONE) << (8 * k);
                pb |= ((rv[k] && xa > 0) ? lp[k] : (uint32_t)DIR_NONE) << (8 * k);
                nb |= ((rv[k] && xa + 1 < g) ? ln[k] : (uint32_t)DIR_NONE) << (8 * k);
            }
        }
        for (uint32_t x = xa; x < xb; ++x) {
            const uint32_t px = x * g2;
            const bool pf = x + 1 < xb && x + 2 < g;
            // Every load of the step is issued unconditionally (indices clamped to a
            // valid node of this plane), pinned by an asm use only after all are in
            // flight, and masked afterwards: as `cond ? load : NONE` the compiler
            // turned each into a branch and waited for it there -- a dozen serialized
            // round trips per step.
            // z +- 1 senders: the neighbour lanes' bytes of plane x (cb, by DPP); only the
            // wave's end lanes load theirs (lane 0: z - 1, lane 63: z + 1, one register).
            const uint32_t pxb = px - base;
            uint32_t lnn[NR], led[NR], lrc[NR], lrd[NR];
            int32_t cv[NR];
            const bool ledge = (lane == 0 && z > 0) || (lane == 63 && z + 1 < g);
            __builtin_amdgcn_s_setprio(COL_PRIO);
#pragma unroll
            for (int k = 0; k < NR; ++k) {
                const uint32_t jl = pxb + yo[k];  // yo = 0 on invalid lanes: the plane's first node
                lnn[k] = nbc[(pf ? 2u * g2 : 0u) + jl];
                cv[k] = a.c[px + yo[k] - lo];
                led[k] = nbc[(rv[k] && ledge) ? (lane == 0 ? jl - 1 : jl + 1) : jl];
                lrc[k] = lrd[k] = 0u;
                if (TOPO == IMP3D) {
                    lrc[k] = a.rq8 ? (uint32_t)reinterpret_cast<const uint8_t*>(a.rq_cur)[px + yo[k] - lo]
                                   : a.rq_cur[px + yo[k] - lo];
                    lrd[k] = REMOTE ? a.rtg[px + yo[k] - lo] : a.rnd[px + yo[k] - lo];
                }
            }
            const bool hmv = zv && y0 > 0, hpv = zv && y0 + NR < g;
            uint32_t hym = nbc[hmv ? pxb + (y0 - 1) * g + z : pxb];
            uint32_t hyp = nbc[hpv ? pxb + (y0 + NR) * g + z : pxb];
#pragma unroll
            for (int k = 0; k < NR; ++k)
                asm volatile("" : "+v"(lnn[k]), "+v"(cv[k]), "+v"(led[k]), "+v"(lrc[k]), "+v"(lrd[k]));
            asm volatile("" : "+v"(hym), "+v"(hyp));
            __builtin_amdgcn_s_setprio(0);
            if (!hmv) hym = DIR_NONE;
            if (!hpv) hyp = DIR_NONE;
            // lane - 1's and lane + 1's bytes of plane x (wave_shr:1 / wave_shl:1)
            const uint32_t cbl = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)cb, 0x138, 0xF, 0xF, false);
            const uint32_t cbr = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)cb, 0x130, 0xF, 0xF, false);
            uint32_t nnb = 0, zbm = 0, zbp = 0;
            uint32_t rcv[NR];
#pragma unroll
            for (int k = 0; k < NR; ++k) {
                nnb |= ((pf && rv[k]) ? lnn[k] : (uint32_t)DIR_NONE) << (8 * k);
                if (!rv[k]) cv[k] = (int32_t)GOSSIP_DONE;
                const uint32_t bm = lane == 0 ? led[k] : byte_of(cbl, k);
                const uint32_t bp = lane == 63 ? led[k] : byte_of(cbr, k);
                zbm |= ((rv[k] && z > 0) ? bm : (uint32_t)DIR_NONE) << (8 * k);
                zbp |= ((rv[k] && z + 1 < g) ? bp : (uint32_t)DIR_NONE) << (8 * k);
                rcv[k] = (TOPO == IMP3D && rv[k]) ? lrc[k] : 0u;
            }
#pragma unroll
            for (int k = 0; k < NR; ++k) {
                const uint32_t j = px + yo[k];
                const uint32_t mask = rv[k] ? (myz[k] | (x > 0 ? 1u : 0u) | (x + 1 < g ? 2u : 0u)) : 0u;
                uint32_t n = (rv[k] && (long long)j == inj) ? 1u : 0u;
                n += ((mask & 1u) && (byte_of(pb, k) & DIR_MASK) == 1u) ? 1u : 0u;
                n += ((mask & 2u) && (byte_of(nb, k) & DIR_MASK) == 0u) ? 1u : 0u;
                n += ((mask & 4u) && ((k + 1 < NR ? byte_of(cb, k + 1) : hyp) & DIR_MASK) == 3u) ? 1u : 0u;
                n += ((mask & 8u) && ((k > 0 ? byte_of(cb, k - 1) : hym) & DIR_MASK) == 2u) ? 1u : 0u;
                n += ((mask & 16u) && (byte_of(zbp, k) & DIR_MASK) == 5u) ? 1u : 0u;
                n += ((mask & 32u) && (byte_of(zbm, k) & DIR_MASK) == 4u) ? 1u : 0u;
                n += rcv[k];
                int32_t c1v = cv[k];
                if (rv[k] && c1v < (int32_t)GOSSIP_DONE && n) {
                    c1v += (int32_t)n;
                    a.c[j - lo] = c1v;
                    alerts += c1v > 10;  // the receipt that finds rumours == 10 (Program.fs:92-94)
                }
                uint32_t dir = DIR_NONE;
                const bool active = rv[k] && ((j == a.seed_node) || c1v >= 1) && c1v <= 10;
                if (active) {
                    const uint32_t deg = popc6(mask) + (TOPO == IMP3D ? 1u : 0u);
                    if (deg > 0) dir = slot_to_dir(mask, uniform(a.k0, a.k1, S_GOSSIP, j, r + 1, deg));
                }
                if (rv[k]) a.nbn[j - base] = (uint8_t)dir;
                if (TOPO == IMP3D && rv[k]) {
                    // this round's count consumed, and a send on the random edge next round
                    // counted at its target now (the receiver drops it at round start if
                    // converged, Program.fs:87); a target on another rank gets it through
                    // the exchange (k_pack reads this direction byte)
                    if (lrc[k]) {
                        if (a.rq8) reinterpret_cast<uint8_t*>(a.rq_cur)[j - lo] = 0u;
                        else a.rq_cur[j - lo] = 0u;
                    }
                    if (REMOTE) {  // local target (t - lo), or the edge's bit of the send bitmap
                        if (dir == DIR_RANDOM) {
                            if (lrd[k] & 0x80000000u) atomicOr(&a.sbits[(lrd[k] & 0x7FFFFFFFu) >> 5], 1u << (lrd[k] & 31u));
                            else rq_add(a.rq_next, a.rq8, lrd[k]);
                        }
                    } else if (dir == DIR_RANDOM && lrd[k] - lo < a.nloc) {
                        rq_add(a.rq_next, a.rq8, lrd[k] - lo);
                    }
                }
            }
            pb = cb;
            cb = nb;
            nb = nnb;
        }
    }
    block_add2(alerts, 0u, &ctl->round_alerts, nullptr);
}

// Imp3D gossip, round 0: the seed's send on its random edge (only the seed can be
// sending), counted at its target when the target is on this rank (otherwise the
// exchange of round 0 carries it).
__global__ void k_col_seed_init(WaveArgs a, const uint8_t* nb0) {
    const uint32_t i = a.seed_node;
    if (i - a.lo >= a.nloc || (nb0[i - a.base] & DIR_MASK) != DIR_RANDOM) return;
    if (a.rtg) {  // several ranks: a remote target's bit travels with round 0's exchange
        const uint32_t e = a.rtg[i - a.lo];
        if (e & 0x80000000u) atomicOr(&a.sbits[(e & 0x7FFFFFFFu) >> 5], 1u << (e & 31u));
        else rq_add(a.rq_cur, a.rq8, e);
        return;
    }
    const uint32_t t = a.rnd[i - a.lo] - a.lo;
    if (t < a.nloc) rq_add(a.rq_cur, a.rq8, t);
}

int col_blocks_per_cu(int topo, int alg) {
    (void)alg;
    const void* f = topo == GRID3D ? (const void*)k_gossip_col<GRID3D, false> : (const void*)k_gossip_col<IMP3D, false>;
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, f, BULK_THREADS, 0) != hipSuccess || n < 1) n = 1;
    return n;
}

hipError_t launch_round_col(const WaveArgs& a, int topo, int alg, uint32_t round, int grid, hipStream_t st) {
    const dim3 g(grid), b(BULK_THREADS);
    if (alg == PUSHSUM) {
        return hipErrorInvalidValue;  // (push-sum: the tile kernel)
    } else {
        if (topo == GRID3D) {
            hipLaunchKernelGGL((k_gossip_col<GRID3D, false>), g, b, 0, st, a, round);
        } else {
            if (!a.rq_cur || !a.rq_next || !a.rnd) return hipErrorInvalidValue;
            if (a.rtg) hipLaunchKernelGGL((k_gossip_col<IMP3D, true>), g, b, 0, st, a, round);
            else hipLaunchKernelGGL((k_gossip_col<IMP3D, false>), g, b, 0, st, a, round);
        }
    }
    return hipGetLastError();
}

hipError_t launch_col_seed_init(const DevState& S, hipStream_t st) {
    if (S.topo != IMP3D) return hipSuccess;
    WaveArgs a = make_wave_args(S, 0);
    hipLaunchKernelGGL(k_col_seed_init, dim3(1), dim3(1), 0, st, a, S.nb[0]);
    return hipGetLastError();
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
    a.rq_cur = S.rq[round & 1];
    a.rq_next = S.rq[(round + 1) & 1];
    a.rq8 = S.rq8;
    a.rnd = S.rnd;
    a.rtg = S.rtg;
    a.sbits = S.sbits;
    a.ctl = S.ctl;
    a.G = S.G;
    a.k0 = S.k0;
    a.k1 = S.k1;
    a.seed_node = S.seed_node;
    a.lo = S.lo;
    a.nloc = S.nloc;
    a.base = S.base;
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
