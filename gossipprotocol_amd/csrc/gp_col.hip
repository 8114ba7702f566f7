// gp_col.hip -- column-march round kernels for the 3D / Imp3D lattice (gfx950).
//
// One synchronous round of SRS v1 in PULL form with 2.5-D
// blocking.  A wave owns a patch of 4 y-rows x 64 z-columns (one node per lane
// and row; node id = x*g^2 + y*g + z, lanes = consecutive z, so every row of a
// patch is one coalesced 64-node segment) and marches it along x through its
// x-segment.  Planes x and x+1 of the patch stay in registers and plane x+2 is
// prefetched a step ahead, so of the six lattice senders of a node
//   x+1 and (inside the patch) y+-1 are register selects,
//   x-1 was streamed by this same wave one step ago (L2), and
//   z+-1 sit in the lines this wave just loaded (L1),
// and only the two y-halo rows touch another wave's data.  Per node and round
// the compulsory stream is own (s, w) + node byte in and out; the lattice
// costs no HBM traffic of its own.  Imp3D in-edges are swept per step exactly
// like the chunk kernel (gp_wave.hip): flattened over the patch's four row
// segments, decided by Philox / bitmap / exchange tag, gathered with all loads
// of the sweep in flight, parked in wave-private LDS, folded per node in
// canonical order.
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

// In-edge sweep of one patch-step: rows k = 0..NR-1 own the edges
// [e0[k], e0[k] + cnt) of the CSR; flat index q = P[k] + (e - e0[k]).
// PUSH: park (s, w) of senders that used their random edge; gossip: 0/1 codes.
template <bool PUSH>
__device__ __forceinline__ void sweep_in_edges(const WaveArgs& a, WaveLds& L, const uint32_t (&e0)[NR],
                                               const uint32_t (&P)[NR + 1], uint32_t r, bool all_active,
                                               uint32_t stream) {
    const int lane = threadIdx.x & 63;
    const uint32_t lo = a.lo, nloc = a.nloc, base = a.base;
    const uint32_t nst = min(P[NR], ECAP);
    uint32_t nmsg = 0;
    for (uint32_t q0 = 0; q0 < nst; q0 += EU * 64) {
        uint32_t eidx[EU], src[EU];
        bool sent[EU];
#pragma unroll
        for (int m = 0; m < EU; ++m) {
            const uint32_t q = q0 + m * 64 + lane;
            const uint32_t k = (q >= P[1] ? 1u : 0u) + (q >= P[2] ? 1u : 0u) + (q >= P[3] ? 1u : 0u);
            const uint32_t eb = k == 0 ? e0[0] : k == 1 ? e0[1] : k == 2 ? e0[2] : e0[3];
            const uint32_t pb = k == 0 ? P[0] : k == 1 ? P[1] : k == 2 ? P[2] : P[3];
            eidx[m] = eb + (q - pb);
            src[m] = q < nst ? a.in_src[eidx[m]] : lo;
        }
        // decisions: every sender's direction draw of round r as one Philox batch
        // (interleaved chains), the bitmap read only where the draw picks the
        // random slot (col_sent_random)
        {
            const Geom& G = a.G;
            uint32_t xs[EU], ys[EU], wrd[EU], di[EU];
#pragma unroll
            for (int m = 0; m < EU; ++m) {
                const uint32_t i = src[m];
                const uint32_t x = fastdiv(i, G.div_g2);
                const uint32_t rem = i - x * G.g2;
                const uint32_t y = fastdiv(rem, G.div_g);
                const uint32_t z = rem - y * G.g;
                di[m] = popc6(mask_xyz(x, y, z, G.g - 1)) + 1u;
                wrd[m] = z;
                xs[m] = x;
                ys[m] = y;
            }
            uint32_t X[EU], Y[EU];
            philox2_batch<EU>(src, r, stream, a.k0, a.k1, X, Y);
#pragma unroll
            for (int m = 0; m < EU; ++m) {
                const uint32_t q = q0 + m * 64 + lane;
                bool s = false;
                if (q < nst) {
                    const uint32_t i = src[m];
                    if (i - lo >= nloc) {
                        s = a.rtag[eidx[m]] == r;  // sender on another rank
                    } else if (uniform_from(X[m], Y[m], di[m]) == di[m] - 1u) {
                        const uint32_t z = wrd[m];
                        s = all_active || ((a.rbc[col_rb_word(a, xs[m], ys[m], z)] >> (z & 63)) & 1ull);
                    }
                }
                sent[m] = s;
            }
        }
        if (PUSH) {
            double2 val[EU];
#pragma unroll
            for (int m = 0; m < EU; ++m) {
                const uint32_t i = src[m];
                val[m] = make_double2(0.0, 0.0);
                if (sent[m]) val[m] = (i - lo >= nloc) ? a.rmsg[eidx[m]] : a.swc[i - base];
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
        } else {
#pragma unroll
            for (int m = 0; m < EU; ++m) {
                const uint32_t q = q0 + m * 64 + lane;
                if (q < nst) L.code[q] = sent[m] ? 1u : 0u;
            }
        }
    }
    wave_lds_sync();
}

// Row k's CSR bounds of the patch-step: per-lane offset and the row's end.
[[maybe_unused]] __device__ __forceinline__ void row_offsets(const WaveArgs& a, uint32_t rs, uint32_t nz, bool row_ok, uint32_t& off,
                                            uint32_t& rend) {
    const int lane = threadIdx.x & 63;
    if (row_ok) {
        off = a.in_off[rs + min((uint32_t)lane, nz) - a.lo];
        rend = a.in_off[rs + nz - a.lo];
    } else {
        off = 0;
        rend = 0;
    }
}

}  // namespace

// ---------------------------------------------------------------- push-sum
// Experiment variant (push-sum runs the tiled kernel):
// experiments library only.
#ifdef GP_EXPERIMENTS
template <int TOPO>
__global__ __launch_bounds__(BULK_THREADS) void k_ps_col(WaveArgs a, uint32_t r) {
    __shared__ WaveLds Lw[WPB];
    Ctl* ctl = a.ctl;
    if (ld_agent(&ctl->done)) return;
    const bool all_active = ld_agent(&ctl->all_active) != 0;
    const int lane = threadIdx.x & 63;
    WaveLds& L = Lw[threadIdx.x >> 6];
    const double2* __restrict__ swc = a.swc;
    double2* __restrict__ swn = a.swn;
    const uint8_t* __restrict__ nbc = a.nbc;
    const uint32_t g = a.G.g, g2 = a.G.g2, base = a.base, lo = a.lo, nloc = a.nloc;
    uint32_t alerts = 0, newly = 0;

    uint32_t it, it_end, it_step;
    item_range(a.nitems, it, it_end, it_step);
    for (; it < it_end; it += it_step) {
        const uint32_t zs = it % a.zsegs;
        const uint32_t t = it / a.zsegs;
        const uint32_t yb = t % a.yblocks;
        const uint32_t xa = a.x_lo + (t / a.yblocks) * a.xs_len;
        const uint32_t xb = min(a.x_hi, xa + a.xs_len);
        const uint32_t z = zs * 64 + (uint32_t)lane;
        const uint32_t nz = min(64u, g - zs * 64);
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
        // planes xa (cur) and xa+1 (nxt), direction bytes of xa-1 (pb)
        double2 cur[NR], nxt[NR];
        uint32_t pb = 0, cb = 0, nb = 0;
#pragma unroll
        for (int k = 0; k < NR; ++k) {
            const uint32_t jl = xa * g2 + yo[k] - base;
            cur[k] = rv[k] ? swc[jl] : make_double2(0.0, 1.0);
            cb |= (rv[k] ? (uint32_t)nbc[jl] : (uint32_t)DIR_NONE) << (8 * k);
            pb |= ((rv[k] && xa > 0) ? (uint32_t)nbc[jl - g2] : (uint32_t)DIR_NONE) << (8 * k);
            const bool hn = rv[k] && xa + 1 < g;
            nxt[k] = hn ? swc[jl + g2] : make_double2(0.0, 1.0);
            nb |= (hn ? (uint32_t)nbc[jl + g2] : (uint32_t)DIR_NONE) << (8 * k);
        }
        for (uint32_t x = xa; x < xb; ++x) {
            const uint32_t px = x * g2;
            // prefetch plane x+2 (the nxt of the next step)
            const bool pf = x + 1 < xb && x + 2 < g;
            double2 nn[NR];
            uint32_t nnb = 0;
#pragma unroll
            for (int k = 0; k < NR; ++k) {
                const bool h = pf && rv[k];
                const uint32_t jl = px + 2 * g2 + yo[k] - base;
                nn[k] = h ? swc[jl] : make_double2(0.0, 1.0);
                nnb |= (h ? (uint32_t)nbc[jl] : (uint32_t)DIR_NONE) << (8 * k);
            }
            // halo direction bytes of plane x: rows y0-1, y0+NR and columns z-+1
            const uint32_t hym = (zv && y0 > 0) ? nbc[px + (y0 - 1) * g + z - base] : DIR_NONE;
            const uint32_t hyp = (zv && y0 + NR < g) ? nbc[px + (y0 + NR) * g + z - base] : DIR_NONE;
            uint32_t zbm = 0, zbp = 0;
#pragma unroll
            for (int k = 0; k < NR; ++k) {
                const uint32_t jl = px + yo[k] - base;
                zbm |= ((rv[k] && z > 0) ? (uint32_t)nbc[jl - 1] : (uint32_t)DIR_NONE) << (8 * k);
                zbp |= ((rv[k] && z + 1 < g) ? (uint32_t)nbc[jl + 1] : (uint32_t)DIR_NONE) << (8 * k);
            }
            uint32_t off[NR], rend[NR], e0[NR], P[NR + 1];
            if (TOPO == IMP3D) {
#pragma unroll
                for (int k = 0; k < NR; ++k) row_offsets(a, px + (y0 + k) * g + zs * 64, nz, y0 + k < g, off[k], rend[k]);
                P[0] = 0;
#pragma unroll
                for (int k = 0; k < NR; ++k) {
                    e0[k] = __builtin_amdgcn_readlane(off[k], 0);
                    P[k + 1] = P[k] + (rend[k] - e0[k]);
                }
                sweep_in_edges<true>(a, L, e0, P, r, all_active, S_PUSHSUM);
            }
#pragma unroll
            for (int k = 0; k < NR; ++k) {
                const uint32_t j = px + yo[k];
                const uint32_t jl = j - base;
                const uint32_t mask = rv[k] ? (myz[k] | (x > 0 ? 1u : 0u) | (x + 1 < g ? 2u : 0u)) : 0u;
                uint32_t f = 0;
                f |= ((mask & 1u) && (byte_of(pb, k) & DIR_MASK) == 1u) ? 1u : 0u;
                f |= ((mask & 2u) && (byte_of(nb, k) & DIR_MASK) == 0u) ? 2u : 0u;
                f |= ((mask & 4u) && ((k + 1 < NR ? byte_of(cb, k + 1) : hyp) & DIR_MASK) == 3u) ? 4u : 0u;
                f |= ((mask & 8u) && ((k > 0 ? byte_of(cb, k - 1) : hym) & DIR_MASK) == 2u) ? 8u : 0u;
                f |= ((mask & 16u) && (byte_of(zbp, k) & DIR_MASK) == 5u) ? 16u : 0u;
                f |= ((mask & 32u) && (byte_of(zbm, k) & DIR_MASK) == 4u) ? 32u : 0u;
                const uint32_t b = byte_of(cb, k);
                const uint32_t deg = popc6(mask) + (TOPO == IMP3D ? 1u : 0u);
                bool active = (b & B_ACTIVE) != 0;
                const double2 sv = cur[k];
                const bool halve = active && deg > 0;
                double acc_s = halve ? sv.x * 0.5 : sv.x;
                double acc_w = halve ? sv.y * 0.5 : sv.y;
                const double2 z2 = make_double2(0.0, 0.0);
                double2 m[6];
                m[0] = (f & 1u) ? swc[jl - g2] : z2;
                m[1] = (f & 2u) ? nxt[k] : z2;
                if (k + 1 < NR) m[2] = (f & 4u) ? cur[k + 1 < NR ? k + 1 : k] : z2;
                else m[2] = (f & 4u) ? swc[jl + g] : z2;
                if (k > 0) m[3] = (f & 8u) ? cur[k > 0 ? k - 1 : k] : z2;
                else m[3] = (f & 8u) ? swc[jl - g] : z2;
                m[4] = (f & 16u) ? swc[jl + 1] : z2;
                m[5] = (f & 32u) ? swc[jl - 1] : z2;
#pragma unroll
                for (int d = 0; d < 6; ++d) {
                    if ((f >> d) & 1u) {
                        acc_s = acc_s + m[d].x * 0.5;
                        acc_w = acc_w + m[d].y * 0.5;
                    }
                }
                bool recv = f != 0;
                if (TOPO == IMP3D) {
                    const uint32_t ebk = off[k];
                    uint32_t ee = __shfl_down(ebk, 1, 64);
                    if (lane == 63) ee = rend[k];
                    for (uint32_t e = ebk; e < ee; ++e) {
                        const uint32_t q = P[k] + (e - e0[k]);
                        bool s;
                        double2 mi = z2;
                        if (q < ECAP) {
                            const uint32_t code = L.code[q];
                            s = code != CODE_NONE;
                            if (code < MCAP) {
                                mi = L.msg[code];
                            } else if (s) {  // parked-message overflow: reload
                                const uint32_t i = a.in_src[e];
                                mi = (i - lo >= nloc) ? a.rmsg[e] : swc[i - base];
                            }
                        } else {  // beyond the staged edges: decide here
                            const uint32_t i = a.in_src[e];
                            if (i - lo >= nloc) {
                                s = a.rtag[e] == r;
                                if (s) mi = a.rmsg[e];
                            } else {
                                s = col_sent_random(a, i, r, all_active, S_PUSHSUM);
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
                if (rv[k]) {
                    a.nbn[jl] = (uint8_t)(flags | dir);
                    swn[jl] = make_double2(acc_s, acc_w);
                }
                if (TOPO == IMP3D && !all_active) {
                    const unsigned long long bits = __ballot(rv[k] && dir == DIR_RANDOM);
                    if (lane == 0 && y0 + k < g) a.rbn[col_rb_word(a, x, y0 + k, zs * 64)] = bits;
                }
            }
            if (TOPO == IMP3D) wave_lds_sync();  // the next step's sweep overwrites L
            // rotate the plane window
            pb = cb;
            cb = nb;
            nb = nnb;
#pragma unroll
            for (int k = 0; k < NR; ++k) {
                cur[k] = nxt[k];
                nxt[k] = nn[k];
            }
        }
    }
    block_add2(alerts, newly, &ctl->round_alerts, &ctl->round_active);
}
#endif  // GP_EXPERIMENTS

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
                if (TOPO == IMP3D) {
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
    for (uint32_t w = blockIdx.x * BULK_THREADS + threadIdx.x; w < words; w += gridDim.x * BULK_THREADS)
        a.rbn[w] = w == sw ? sbit : 0ull;
    // one rank, push form: the seed's round-0 send on its random edge, counted at the target
    if (a.rq_cur && sbit && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&a.rq_cur[a.rnd[i - a.lo] - a.lo], 1u);
}

uint32_t col_rbits_words(uint32_t planes, uint32_t g) { return planes * g * ((g + 63) / 64) + 16u; }

int col_blocks_per_cu(int topo, int alg) {
    const void* f;
    f = topo == GRID3D ? (const void*)k_gossip_col<GRID3D> : (const void*)k_gossip_col<IMP3D>;
#ifdef GP_EXPERIMENTS
    if (alg == PUSHSUM) f = topo == GRID3D ? (const void*)k_ps_col<GRID3D> : (const void*)k_ps_col<IMP3D>;
#else
    (void)alg;
#endif
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, f, BULK_THREADS, 0) != hipSuccess || n < 1) n = 1;
    return n;
}

hipError_t launch_round_col(const WaveArgs& a, int topo, int alg, uint32_t round, int grid, hipStream_t st) {
    const dim3 g(grid), b(BULK_THREADS);
    if (alg == PUSHSUM) {
#ifdef GP_EXPERIMENTS
        if (topo == GRID3D) hipLaunchKernelGGL(k_ps_col<GRID3D>, g, b, 0, st, a, round);
        else hipLaunchKernelGGL(k_ps_col<IMP3D>, g, b, 0, st, a, round);
#else
        return hipErrorInvalidValue;
#endif
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

}  // namespace gp
