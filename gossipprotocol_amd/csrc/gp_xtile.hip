// gp_xtile.hip -- x-marching tiled push-sum round kernel for the 3D / Imp3D
// lattice (gfx950).
//
// The tile kernel (gp_round.hip) with a different tile geometry: a tile is a
// window of TILE consecutive ids inside one x-plane, and a workgroup marches
// its window through the planes of its x-segment.  Thread t always owns the
// same four (y, z) positions, so the node's x-1 and x+1 lattice neighbours are
// the same thread's nodes of the previous and next plane: their (s, w) and
// node bytes are kept in registers (x-1: last step's own values; x+1: loaded
// at the start of the step and consumed at its end, then reused as the next
// step's own values).  Compared with the tile kernel this removes the x+-1
// (s, w) gathers and the x+-1 byte staging, and the main (s, w) stream is
// always one plane ahead of its use.  y+-1 / z+-1 neighbours and the Imp3D
// in-edges are handled exactly like the tile kernel (LDS-staged row bytes,
// gathers of the actual senders, flattened in-edge pass).
//
// During activation (not every node active yet) a local random-edge sender is
// recognised from its node byte (direction == random edge); this kernel keeps
// no ballot bitmap.  Built with -ffp-contract=off (canonical fold order).
#include "gp_internal.hpp"

namespace gp {
namespace {

constexpr int TPB = BULK_THREADS;  // 256
constexpr int NPT = 4;
constexpr int TILE = TPB * NPT;    // ids per plane window
constexpr int HMAX = 1625;
constexpr int W_ROWS = (TILE + 2 * HMAX) / 4 + 4;
constexpr int SRC_CAP = 1536;
constexpr int MSG_CAP = 384;
constexpr uint16_t POS_NONE = 0xFFFF, POS_GLOBAL = 0xFFFE;

struct XTileLds {
    uint32_t rows[W_ROWS];       // direction bytes of [j0 - g, j1 + g)
    uint32_t off[TILE + 1];      // in_off[j0 .. j1]
    uint32_t src[SRC_CAP];       // in_src[in_off[j0] .. in_off[j1])
    uint16_t pos[SRC_CAP];       // staged in-edge -> parked message slot
    double2 msg[MSG_CAP];
    uint32_t out[TILE / 4 + 2];  // next-round node bytes from the 4-aligned id T4
    uint32_t red[2][TPB / 64];
};

template <typename T>
__device__ __forceinline__ T ld_agent(const T* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint32_t lds_byte(const uint32_t* w, uint32_t idx) {
    return reinterpret_cast<const uint8_t*>(w)[idx];
}

__device__ __forceinline__ uint32_t stage_bytes(uint32_t* lds, const uint8_t* nb, int64_t lo, int64_t hi,
                                                uint32_t ext_lo, uint32_t ext_hi) {
    if (lo < (int64_t)ext_lo) lo = ext_lo;
    if (hi > (int64_t)ext_hi) hi = ext_hi;
    const uint32_t ws = (uint32_t)lo & ~3u;
    const int nw = hi > lo ? (int)(((uint32_t)hi + 3u - ws) >> 2) : 0;
    const uint32_t* src = reinterpret_cast<const uint32_t*>(nb + ws);
    for (int w = threadIdx.x; w < nw; w += TPB) lds[w] = src[w];
    return ws;
}

__device__ __forceinline__ uint32_t byte_of(uint32_t packed, int k) { return (packed >> (8 * k)) & 0xFFu; }

}  // namespace

template <int TOPO, bool REMOTE>
__global__ __launch_bounds__(TPB, 4) void k_ps_xtile(RoundArgs a, uint32_t r) {
    __shared__ XTileLds L;
    Ctl* ctl = a.ctl;
    if (ld_agent(&ctl->done)) return;
    const bool all_active = ld_agent(&ctl->all_active) != 0;
    const double2* __restrict__ swc = a.swc;
    double2* __restrict__ swn = a.swn;
    const uint8_t* __restrict__ nbc = a.nbc;
    const uint32_t* __restrict__ in_src = a.in_src;
    const Geom G = a.G;
    const uint32_t g = G.g, g2 = G.g2;
    const uint32_t x_lo = a.lo / g2, x_hi = (a.lo + a.nloc) / g2;
    const uint32_t nwin = (g2 + TILE - 1) / TILE;
    const uint32_t xs_len = a.xs_len;
    const uint32_t nseg = (x_hi - x_lo + xs_len - 1) / xs_len;
    const uint32_t nitems = nwin * nseg;
    uint32_t alerts = 0, newly = 0;
    const int lane = threadIdx.x & 63;

    // XCD-contiguous deal of the (window, segment) items (speed only)
    uint32_t it, it_end, it_step;
    if ((gridDim.x & 7) == 0) {
        const uint32_t xcd = blockIdx.x & 7;
        it = (uint32_t)((uint64_t)nitems * xcd / 8) + (blockIdx.x >> 3);
        it_end = (uint32_t)((uint64_t)nitems * (xcd + 1) / 8);
        it_step = gridDim.x >> 3;
    } else {
        it = blockIdx.x;
        it_end = nitems;
        it_step = gridDim.x;
    }
    for (; it < it_end; it += it_step) {
        const uint32_t w = it % nwin;
        const uint32_t xa = x_lo + (it / nwin) * xs_len;
        const uint32_t xb = min(x_hi, xa + xs_len);
        const uint32_t ws = w * TILE;
        const uint32_t nt = min((uint32_t)TILE, g2 - ws);  // ids in this window
        // the same (y, z) positions in every plane: own / x-1 values rotate through registers
        double2 prv[NPT], cur[NPT], nxt[NPT];
        uint32_t pb = 0, cb = 0, nbx = 0;
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
            const uint32_t jl = k * TPB + threadIdx.x;
            const bool valid = jl < nt;
            const uint32_t j = xa * g2 + ws + (valid ? jl : 0u);
            cur[k] = valid ? swc[j] : make_double2(0.0, 1.0);
            cb |= (valid ? (uint32_t)nbc[j] : (uint32_t)DIR_NONE) << (8 * k);
            const bool hp = valid && xa > 0;
            prv[k] = hp ? swc[j - g2] : make_double2(0.0, 1.0);
            pb |= (hp ? (uint32_t)nbc[j - g2] : (uint32_t)DIR_NONE) << (8 * k);
        }
        for (uint32_t x = xa; x < xb; ++x) {
            const uint32_t j0 = x * g2 + ws, j1 = j0 + nt;
            const uint32_t T4 = j0 & ~3u;
            uint32_t e_lo = 0, e_hi = 0;
            if (TOPO == IMP3D) {
                e_lo = a.in_off[j0];
                e_hi = a.in_off[j1];
            }
            // plane x+1 of this window: the fold's x+1 senders now, own values next step
            const bool hn = x + 1 < g;
            nbx = 0;
#pragma unroll
            for (int k = 0; k < NPT; ++k) {
                const uint32_t jl = k * TPB + threadIdx.x;
                const bool v = hn && jl < nt;
                const uint32_t j = j0 + (jl < nt ? jl : 0u) + g2;
                nxt[k] = v ? swc[j] : make_double2(0.0, 1.0);
                nbx |= (v ? (uint32_t)nbc[j] : (uint32_t)DIR_NONE) << (8 * k);
            }
            const uint32_t b_rows = stage_bytes(L.rows, a.nbc, (int64_t)j0 - g, (int64_t)j1 + g, a.ext_lo, a.ext_hi);
            const uint32_t cnt = e_hi - e_lo;
            const bool staged = cnt <= (uint32_t)SRC_CAP;
            if (TOPO == IMP3D) {
                for (uint32_t q = threadIdx.x; q <= nt; q += TPB) L.off[q] = a.in_off[j0 + q];
                if (staged)
                    for (uint32_t q = threadIdx.x; q < cnt; q += TPB) L.src[q] = in_src[e_lo + q];
            }
            __syncthreads();
            if (TOPO == IMP3D) {
                if (staged) {
                    // flattened in-edge pass: all decisions, then all gathers (see gp_round.hip)
                    constexpr int FU = SRC_CAP / TPB;
                    constexpr uint32_t WCAP = MSG_CAP / (TPB / 64);
                    uint32_t isrc[FU];
                    bool snt[FU];
#pragma unroll
                    for (int m = 0; m < FU; ++m) {
                        const uint32_t q = threadIdx.x + m * TPB;
                        isrc[m] = q < cnt ? L.src[q] : a.lo;
                    }
#pragma unroll
                    for (int m = 0; m < FU; ++m) {
                        const uint32_t q = threadIdx.x + m * TPB;
                        const uint32_t i = isrc[m];
                        bool sent = false;
                        if (q < cnt) {
                            if (REMOTE && i - a.lo >= a.nloc) {
                                sent = a.rtag[e_lo + q] == r;
                            } else if (all_active) {
                                const uint32_t di = popc6(present_mask<IMP3D>(i, G)) + 1u;
                                sent = uniform(a.k0, a.k1, S_PUSHSUM, i, r, di) == di - 1u;
                            } else {
                                sent = (nbc[i] & DIR_MASK) == DIR_RANDOM;
                            }
                        }
                        snt[m] = sent;
                    }
                    double2 v[FU];
#pragma unroll
                    for (int m = 0; m < FU; ++m) {
                        v[m] = make_double2(0.0, 0.0);
                        if (snt[m]) {
                            const uint32_t q = threadIdx.x + m * TPB;
                            v[m] = (REMOTE && isrc[m] - a.lo >= a.nloc) ? a.rmsg[e_lo + q] : swc[isrc[m]];
                        }
                    }
                    const uint32_t wbase = (threadIdx.x >> 6) * WCAP;
                    uint32_t wn = 0;
#pragma unroll
                    for (int m = 0; m < FU; ++m) {
                        const uint32_t q = threadIdx.x + m * TPB;
                        const unsigned long long bal = __ballot(snt[m]);
                        const uint32_t slot = wn + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
                        wn += (uint32_t)__popcll(bal);
                        if (q < cnt) L.pos[q] = !snt[m] ? POS_NONE : (slot < WCAP ? (uint16_t)(wbase + slot) : POS_GLOBAL);
                        if (snt[m] && slot < WCAP) L.msg[wbase + slot] = v[m];
                    }
                }
                __syncthreads();
            }
#pragma unroll
            for (int k = 0; k < NPT; ++k) {
                const uint32_t jl = k * TPB + threadIdx.x;
                const uint32_t j = j0 + jl;
                const bool valid = jl < nt;
                if (valid) {
                    const uint32_t rem = ws + jl;  // position inside plane x
                    const uint32_t y = fastdiv(rem, G.div_g);
                    const uint32_t z = rem - y * g;
                    const uint32_t gm = g - 1;
                    const uint32_t mask = (x > 0 ? 1u : 0u) | (x < gm ? 2u : 0u) | (y < gm ? 4u : 0u) |
                                          (y > 0 ? 8u : 0u) | (z < gm ? 16u : 0u) | (z > 0 ? 32u : 0u);
                    const uint32_t deg = popc6(mask) + (TOPO == IMP3D ? 1u : 0u);
                    const uint32_t b = byte_of(cb, k);
                    uint32_t from = 0;
                    if ((mask & 1u) && (byte_of(pb, k) & DIR_MASK) == 1u) from |= 1u;
                    if ((mask & 2u) && (byte_of(nbx, k) & DIR_MASK) == 0u) from |= 2u;
                    if ((mask & 4u) && (lds_byte(L.rows, j + g - b_rows) & DIR_MASK) == 3u) from |= 4u;
                    if ((mask & 8u) && (lds_byte(L.rows, j - g - b_rows) & DIR_MASK) == 2u) from |= 8u;
                    if ((mask & 16u) && (lds_byte(L.rows, j + 1 - b_rows) & DIR_MASK) == 5u) from |= 16u;
                    if ((mask & 32u) && (lds_byte(L.rows, j - 1 - b_rows) & DIR_MASK) == 4u) from |= 32u;
                    bool active = (b & B_ACTIVE) != 0;
                    const double2 sv = cur[k];
                    const bool halve = active && deg > 0;
                    double acc_s = halve ? sv.x * 0.5 : sv.x;
                    double acc_w = halve ? sv.y * 0.5 : sv.y;
                    const double2 z2 = make_double2(0.0, 0.0);
                    double2 m[6];
                    m[0] = (from & 1u) ? prv[k] : z2;
                    m[1] = (from & 2u) ? nxt[k] : z2;
                    m[2] = (from & 4u) ? swc[j + g] : z2;
                    m[3] = (from & 8u) ? swc[j - g] : z2;
                    m[4] = (from & 16u) ? swc[j + 1] : z2;
                    m[5] = (from & 32u) ? swc[j - 1] : z2;
#pragma unroll
                    for (int d = 0; d < 6; ++d) {
                        if ((from >> d) & 1u) {
                            acc_s = acc_s + m[d].x * 0.5;
                            acc_w = acc_w + m[d].y * 0.5;
                        }
                    }
                    bool recv = from != 0;
                    if (TOPO == IMP3D) {
                        const uint32_t e_b = L.off[jl], e_e = L.off[jl + 1];
                        for (uint32_t e = e_b; e < e_e; ++e) {
                            bool sent = false;
                            double2 mi = z2;
                            if (staged) {
                                const uint16_t p = L.pos[e - e_lo];
                                sent = p != POS_NONE;
                                if (p < (uint16_t)MSG_CAP) {
                                    mi = L.msg[p];
                                } else if (p == POS_GLOBAL) {
                                    const uint32_t i = L.src[e - e_lo];
                                    mi = (REMOTE && i - a.lo >= a.nloc) ? a.rmsg[e] : swc[i];
                                }
                            } else {  // rare: window in-degree above SRC_CAP
                                const uint32_t i = in_src[e];
                                if (REMOTE && i - a.lo >= a.nloc) {
                                    sent = a.rtag[e] == r;
                                    if (sent) mi = a.rmsg[e];
                                } else {
                                    if (all_active) {
                                        const uint32_t di = popc6(present_mask<IMP3D>(i, G)) + 1u;
                                        sent = uniform(a.k0, a.k1, S_PUSHSUM, i, r, di) == di - 1u;
                                    } else {
                                        sent = (nbc[i] & DIR_MASK) == DIR_RANDOM;
                                    }
                                    if (sent) mi = swc[i];
                                }
                            }
                            if (sent) {
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
                            uint32_t cn = (b >> CNT_SHIFT) & 3u;
                            cn = fabs(r_new - r_old) > 1e-10 ? 0u : cn + 1u;
                            flags = (flags & ~(3u << CNT_SHIFT)) | (cn << CNT_SHIFT);
                            if (cn == 3) {
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
                    reinterpret_cast<uint8_t*>(L.out)[j - T4] = (uint8_t)(flags | dir);
                    swn[j] = make_double2(acc_s, acc_w);
                }
            }
            __syncthreads();
            for (uint32_t wd = threadIdx.x; wd * 4 < nt + (j0 - T4); wd += TPB) {
                const uint32_t jw = T4 + wd * 4;
                if (jw >= j0 && jw + 4 <= j1) {
                    reinterpret_cast<uint32_t*>(a.nbn + T4)[wd] = L.out[wd];
                } else {
                    for (uint32_t bb = 0; bb < 4; ++bb)
                        if (jw + bb >= j0 && jw + bb < j1)
                            a.nbn[jw + bb] = reinterpret_cast<const uint8_t*>(L.out)[wd * 4 + bb];
                }
            }
            __syncthreads();
            // rotate the plane ring
            pb = cb;
            cb = nbx;
#pragma unroll
            for (int k = 0; k < NPT; ++k) {
                prv[k] = cur[k];
                cur[k] = nxt[k];
            }
        }
    }
    uint32_t xx = alerts, yy = newly;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        xx += __shfl_xor(xx, o, 64);
        yy += __shfl_xor(yy, o, 64);
    }
    if (lane == 0) {
        L.red[0][threadIdx.x >> 6] = xx;
        L.red[1][threadIdx.x >> 6] = yy;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        xx = 0;
        yy = 0;
        for (int q = 0; q < TPB / 64; ++q) {
            xx += L.red[0][q];
            yy += L.red[1][q];
        }
        if (xx) atomicAdd(&ctl->round_alerts, (unsigned long long)xx);
        if (yy) atomicAdd(&ctl->round_active, (unsigned long long)yy);
    }
}

hipError_t launch_round_xtile(const RoundArgs& a, int topo, bool remote, uint32_t round, int grid, hipStream_t st) {
    const dim3 gr(grid), b(TPB);
    if (topo == GRID3D) hipLaunchKernelGGL((k_ps_xtile<GRID3D, false>), gr, b, 0, st, a, round);
    else if (remote) hipLaunchKernelGGL((k_ps_xtile<IMP3D, true>), gr, b, 0, st, a, round);
    else hipLaunchKernelGGL((k_ps_xtile<IMP3D, false>), gr, b, 0, st, a, round);
    return hipGetLastError();
}

uint32_t xtile_windows(uint32_t g2) { return (g2 + TILE - 1) / TILE; }

}  // namespace gp
