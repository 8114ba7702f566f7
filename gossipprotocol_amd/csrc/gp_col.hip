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
// integer counts: counted by their senders a round ahead (one rank) or by the
// receivers' delivery pass k_gossip_redges (several ranks).
//
// Work items (patch, x-segment) are dealt XCD-contiguously: the waves of one
// XCD own one y-band of every plane, so y-halo rows come from the XCD's L2.
// The random-edge bitmap of these kernels has one 64-bit word per row segment:
// word ((x - x_lo) * g + y) * zsegs + z / 64, bit z % 64 (col_rb_word).
// Built with -ffp-contract=off: the fold must round exactly like the oracle.
#include "gp_wavecommon.hpp"

// gossip column kernel: waves per SIMD (measured 5..7 with the batched step loads,
// profiles/r02/col_batch/: Imp3D best at 5, 3D at 7); GP_COL_WAVES (experiments)
// sets one value for both
#ifdef GP_COL_WAVES
#define GP_COL_MINW(TOPO) GP_COL_WAVES
#else
#define GP_COL_MINW(TOPO) ((TOPO) == IMP3D ? 5 : 7)
#endif

namespace gp {
namespace {

using namespace wk;
constexpr int NR = 4;  // y rows per patch

__device__ __forceinline__ uint32_t col_rb_word(const WaveArgs& a, uint32_t x, uint32_t y, uint32_t z) {
    return ((x - a.x_lo) * a.G.g + y) * a.zsegs + (z >> 6);
}

// Did sender i (on this rank) use its random edge in round r?  Its direction
// draw of round r (counter (i, r), SRS v1 B.2) must pick the random slot -- the
// last one, deg - 1 -- and, unless every node is active, it must have been
// active: the bitmap bit (= active and that draw).  Redrawing first reads the
// bitmap (a random 8-byte load, one 128-byte line) only for the ~1/7 of in-edges
// whose draw selects the random slot.
__device__ __forceinline__ bool col_sent_random(const WaveArgs& a, uint32_t i, uint32_t r, bool all_active,
                                                uint32_t stream) {
    const Geom& G = a.G;
    const uint32_t x = fastdiv(i, G.div_g2);
    const uint32_t rem = i - x * G.g2;
    const uint32_t y = fastdiv(rem, G.div_g);
    const uint32_t z = rem - y * G.g;
    const uint32_t di = popc6(mask_xyz(x, y, z, G.g - 1)) + 1u;
    if (uniform(a.k0, a.k1, stream, i, r, di) != di - 1u) return false;
    return all_active || ((a.rbc[col_rb_word(a, x, y, z)] >> (z & 63)) & 1ull);
}

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
template <int TOPO>
__global__ __launch_bounds__(BULK_THREADS, GP_COL_MINW(TOPO)) void k_gossip_col(WaveArgs a, uint32_t r) {
    Ctl* ctl = a.ctl;
    if (ld_agent(&ctl->done)) return;
    const long long inj = ld_agent(&ctl->inj_target);
    const int lane = threadIdx.x & 63;
    const uint8_t* __restrict__ nbc = a.nbc;
    const uint32_t g = a.G.g, g2 = a.G.g2, base = a.base, lo = a.lo;
    const bool push = a.rq_cur != nullptr;  // one rank: senders count random-edge deliveries (no k_gossip_redges)
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
#pragma unroll
            for (int k = 0; k < NR; ++k) {
                const uint32_t jl = pxb + yo[k];  // yo = 0 on invalid lanes: the plane's first node
                lnn[k] = nbc[(pf ? 2u * g2 : 0u) + jl];
                cv[k] = a.c[px + yo[k] - lo];
                led[k] = nbc[(rv[k] && ledge) ? (lane == 0 ? jl - 1 : jl + 1) : jl];
                lrc[k] = lrd[k] = 0u;
                if (TOPO == IMP3D) {
                    if (push) {
                        lrc[k] = a.rq_cur[px + yo[k] - lo];
                        lrd[k] = a.rnd[px + yo[k] - lo];
                    } else {
                        lrc[k] = a.rcnt[px + yo[k] - lo];
                    }
                }
            }
            const bool hmv = zv && y0 > 0, hpv = zv && y0 + NR < g;
            uint32_t hym = nbc[hmv ? pxb + (y0 - 1) * g + z : pxb];
            uint32_t hyp = nbc[hpv ? pxb + (y0 + NR) * g + z : pxb];
#pragma unroll
            for (int k = 0; k < NR; ++k)
                asm volatile("" : "+v"(lnn[k]), "+v"(cv[k]), "+v"(led[k]), "+v"(lrc[k]), "+v"(lrd[k]));
            asm volatile("" : "+v"(hym), "+v"(hyp));
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
                if (TOPO == IMP3D && push && rv[k]) {
                    // one rank, push form: this round's count consumed, and a send on the
                    // random edge next round counted at its target now (the receiver
                    // drops it at round start if converged, Program.fs:87)
                    if (lrc[k]) a.rq_cur[j - lo] = 0u;
                    if (dir == DIR_RANDOM) atomicAdd(&a.rq_next[lrd[k] - lo], 1u);
                }
                if (TOPO == IMP3D && !push) {  // several ranks: the delivery pass reads these bits
                    const unsigned long long bits = __ballot(rv[k] && dir == DIR_RANDOM);
                    if (lane == 0 && y0 + k < g) a.rbn[col_rb_word(a, x, y0 + k, zs * 64)] = bits;
                }
            }
            pb = cb;
            cb = nb;
            nb = nnb;
        }
    }
    block_add2(alerts, 0u, &ctl->round_alerts, nullptr);
}

// Imp3D gossip, before the column kernel: per local receiver, how many of its
// in-edge senders sent it a rumour on their random edge this round.  Tiles of
// RE_TILE receivers: the tile's in-edges (receiver-sorted, contiguous) are
// decided RE_FU per thread -- senders loaded together, their direction draws as
// one Philox batch, the bitmap read only for the ~1/7 that pick the random slot
// (col_sent_random), remote senders by the exchange tag -- into a byte per edge
// in LDS, then every receiver sums its edge range.  Inside the x-march these
// were three dependent memory round trips per patch step.
constexpr uint32_t RE_TILE = 1024;
constexpr int RE_FU = 6;  // staged in-edges per thread: 1536 per tile (mean 1024, 16 sigma)

// Tiles are software-pipelined one step deep: tile t's edge range and senders
// were loaded during the previous tile of this block, so a tile costs one
// exposed memory round trip (the bitmap reads of its picks) instead of three
// (range -> senders -> bitmap).  Loads are unconditional where possible
// (clamped indices) and the barriers wait for LDS only, so the next tile's
// loads stay in flight across them.
__device__ __forceinline__ void redges_src(const WaveArgs& a, uint32_t e_lo, uint32_t e_hi, uint32_t (&src)[RE_FU]) {
    const uint32_t cnt = e_hi - e_lo;
#pragma unroll
    for (int m = 0; m < RE_FU; ++m) {
        const uint32_t q = threadIdx.x + m * BULK_THREADS;
        src[m] = a.in_src[cnt ? e_lo + min(q, cnt - 1u) : 0u];  // lanes with q >= cnt: never used
    }
}

__device__ __forceinline__ void lds_barrier_only() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

#ifndef GP_RE_MINW
#define GP_RE_MINW 5  // delivery pass: waves per SIMD (5: 96 VGPRs, no spills; 4 measured slower, profiles/r02/c3_redges/minw.txt)
#endif
__global__ __launch_bounds__(BULK_THREADS, GP_RE_MINW) void k_gossip_redges(WaveArgs a, uint32_t r) {
    __shared__ uint8_t sent[BULK_THREADS * RE_FU];
    if (ld_agent(&a.ctl->done)) return;
    const uint32_t lo = a.lo, nloc = a.nloc;
    const Geom& G = a.G;
    constexpr int NPT = RE_TILE / BULK_THREADS;
    const uint32_t ntl = (nloc + RE_TILE - 1) / RE_TILE;
    uint32_t t = blockIdx.x;
    if (t >= ntl) return;
    uint32_t e_lo = a.in_off[t * RE_TILE], e_hi = a.in_off[min(nloc, t * RE_TILE + RE_TILE)];
    uint32_t src[RE_FU];
    redges_src(a, e_lo, e_hi, src);
    for (;;) {
        const uint32_t j0 = t * RE_TILE, j1 = min(nloc, j0 + RE_TILE);  // local receiver ids
        const uint32_t tn = t + gridDim.x;
        const bool more = tn < ntl;  // block-uniform
        const uint32_t cnt = e_hi - e_lo;
        const bool staged = cnt <= (uint32_t)(BULK_THREADS * RE_FU);
        uint32_t eb[NPT], ee[NPT];
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
            const uint32_t jl = min(j0 + k * BULK_THREADS + threadIdx.x, j1 - 1u);
            eb[k] = a.in_off[jl];
            ee[k] = a.in_off[jl + 1];
        }
        uint32_t n_lo = 0, n_hi = 0;
        if (more) {
            n_lo = a.in_off[tn * RE_TILE];
            n_hi = a.in_off[min(nloc, tn * RE_TILE + RE_TILE)];
        }
        if (staged) {
            uint32_t di[RE_FU], wrd[RE_FU], zb[RE_FU], X[RE_FU], Y[RE_FU];
#pragma unroll
            for (int m = 0; m < RE_FU; ++m) {
                const uint32_t i = src[m];
                const uint32_t x = fastdiv(i, G.div_g2);
                const uint32_t rem = i - x * G.g2;
                const uint32_t y = fastdiv(rem, G.div_g);
                const uint32_t z = rem - y * G.g;
                di[m] = popc6(mask_xyz(x, y, z, G.g - 1)) + 1u;
                wrd[m] = i - lo < nloc ? col_rb_word(a, x, y, z) : 0u;
                zb[m] = z & 63u;
            }
            philox2_batch<RE_FU>(src, r, S_GOSSIP, a.k0, a.k1, X, Y);
            unsigned long long w[RE_FU];
#pragma unroll
            for (int m = 0; m < RE_FU; ++m) {
                const uint32_t q = threadIdx.x + m * BULK_THREADS;
                const uint32_t i = src[m];
                w[m] = 0ull;
                if (q < cnt) {
                    if (i - lo >= nloc) w[m] = a.rtag[e_lo + q] == r ? ~0ull : 0ull;  // sender on another rank
                    else if (uniform_from(X[m], Y[m], di[m]) == di[m] - 1u) w[m] = a.rbc[wrd[m]];
                }
            }
            // the next tile's senders, behind this tile's bitmap reads (issued on every
            // path -- the last tile reloads its own -- so the wait below counts them)
            redges_src(a, more ? n_lo : e_lo, more ? n_hi : e_hi, src);
#pragma unroll
            for (int m = 0; m < RE_FU; ++m) sent[threadIdx.x + m * BULK_THREADS] = (uint8_t)((w[m] >> zb[m]) & 1ull);
        } else {
            redges_src(a, more ? n_lo : e_lo, more ? n_hi : e_hi, src);
        }
        lds_barrier_only();
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
            const uint32_t jl = j0 + k * BULK_THREADS + threadIdx.x;
            if (jl >= j1) continue;
            uint32_t n = 0;
            if (staged) {
                for (uint32_t e = eb[k]; e < ee[k]; ++e) n += sent[e - e_lo];
            } else {  // rare: tile in-degree above the staging capacity
                for (uint32_t e = eb[k]; e < ee[k]; ++e) {
                    const uint32_t i = a.in_src[e];
                    if (i - lo >= nloc) n += a.rtag[e] == r ? 1u : 0u;
                    else n += col_sent_random(a, i, r, false, S_GOSSIP) ? 1u : 0u;
                }
            }
            a.rcnt[jl] = (uint16_t)n;
        }
        if (!more) break;
        lds_barrier_only();
        t = tn;
        e_lo = n_lo;
        e_hi = n_hi;
    }
}

// Random-edge bits of round 0 in the column layout (only the seed can be sending).
// Every word is written exactly once (the seed's word with its bit), so no
// store can race the seed's bit away.
__global__ __launch_bounds__(BULK_THREADS) void k_col_rbits_init(WaveArgs a, const uint8_t* nb0, uint32_t words) {
    const uint32_t i = a.seed_node;
    uint32_t sw = 0xFFFFFFFFu;
    unsigned long long sbit = 0ull;
    if (i - a.lo < a.nloc && (nb0[i - a.base] & DIR_MASK) == DIR_RANDOM) {
        const Geom& G = a.G;
        const uint32_t x = fastdiv(i, G.div_g2);
        const uint32_t rem = i - x * G.g2;
        const uint32_t y = fastdiv(rem, G.div_g);
        const uint32_t z = rem - y * G.g;
        sw = col_rb_word(a, x, y, z);
        sbit = 1ull << (z & 63);
    }
    if (a.rbn)  // (gossip, one rank, push form: no bitmap)
        for (uint32_t w = blockIdx.x * BULK_THREADS + threadIdx.x; w < words; w += gridDim.x * BULK_THREADS)
            a.rbn[w] = w == sw ? sbit : 0ull;
    // one rank, push form: the seed's round-0 send on its random edge, counted at the target
    if (a.rq_cur && sbit && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&a.rq_cur[a.rnd[i - a.lo] - a.lo], 1u);
}

uint32_t col_rbits_words(uint32_t planes, uint32_t g) { return planes * g * ((g + 63) / 64) + 16u; }

int col_blocks_per_cu(int topo, int alg) {
    (void)alg;
    const void* f = topo == GRID3D ? (const void*)k_gossip_col<GRID3D> : (const void*)k_gossip_col<IMP3D>;
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
            hipLaunchKernelGGL(k_gossip_col<GRID3D>, g, b, 0, st, a, round);
        } else {
            if (!a.rq_cur) {  // several ranks: receivers decide their in-edges (exchange tags for remote senders)
                if (!a.rcnt) return hipErrorInvalidValue;
                const uint32_t ge = std::min<uint32_t>((a.nloc + RE_TILE - 1) / RE_TILE, 256u * 16u);
                hipLaunchKernelGGL(k_gossip_redges, dim3(std::max(1u, ge)), b, 0, st, a, round);
            }
            hipLaunchKernelGGL(k_gossip_col<IMP3D>, g, b, 0, st, a, round);
        }
    }
    return hipGetLastError();
}

hipError_t launch_col_rbits_init(const DevState& S, hipStream_t st) {
    WaveArgs a = make_wave_args(S, 0);
    a.rbn = S.rbits[0];  // the bits of round 0's sends
    hipLaunchKernelGGL(k_col_rbits_init, dim3(256), dim3(BULK_THREADS), 0, st, a, S.nb[0], S.rbits_words);
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
