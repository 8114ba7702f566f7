// gp_pscol.hip -- push-sum round kernel for the 3D / Imp3D lattice (gfx950):
// column march with a one-step software pipeline.
//
// One synchronous push-sum round of SRS v1 (Program.fs:101-131)
// in PULL form.  A 256-thread workgroup owns a patch of 16 y-rows x 64
// z-columns (wave w: rows 4w..4w+3, lane = z) and marches it along x through
// its x-segment.  Every (s, w) and node byte of the slab is read from HBM once,
// by the workgroup that owns it; the lattice messages of a node then come from
//   x-1, x+1       this lane's registers (planes x-1, x, x+1 are kept),
//   y+-1           this lane's registers inside the wave, the neighbour wave's
//                  boundary row through LDS, or a halo row of the next patch
//                  (gathered by LDS-DMA only where that node sends inward),
//   z+-1           the neighbour lanes' registers by DPP (wave ends: gathered
//                  halo columns).
// Imp3D random edges: the in-lists are stored in patch order (a step = one
// plane of a patch owns one contiguous edge range, pc_src), so a step stages
// its ~1024 in-edge senders with coalesced loads, redraws each sender's
// direction (its Philox draw of this round picks the random slot iff it sent
// on it; during activation also the ballot bitmap), and gathers the ~1/7 used
// messages by LDS-DMA into per-wave compacted slots (sender addresses permuted
// to the first lanes by ds_permute, one DMA per 64 edges).
//
// Pipeline (one barrier per step): step i issues the loads of plane i+2 and of
// step i+2's in-edge senders and halo bytes, decides step i+1 (edge draws,
// message gathers, halo gathers, boundary rows to LDS), folds plane i, writes
// it, and waits at the barrier -- every load of a step has the step's compute
// to land in.  The fold is the canonical one: own half, lattice slots in slot
// order (x-1, x+1, y+1, y-1, z+1, z-1; absent messages add +0.0, exact), random
// edges by ascending sender, fma(m, 0.5, acc) under the 2^-1020 guard (as
// k_ps_tile); ratio test; next-round direction by one Philox batch.
// Built with -ffp-contract=off: the fold must round exactly like the oracle.
#include "gp_wavecommon.hpp"

#ifndef GP_PC_MINW
#define GP_PC_MINW 4  // waves per SIMD (= resident workgroups per CU; LDS allows 5)
#endif

namespace gp {
namespace {

using namespace wk;

#ifndef GP_PC_NR
#define GP_PC_NR 2
#endif
constexpr int PC_NR = GP_PC_NR;              // y rows per wave
constexpr uint32_t PC_ROWS = WPB * PC_NR;    // y rows per patch
constexpr uint32_t PC_RSH = PC_ROWS == 16 ? 4 : PC_ROWS == 8 ? 3 : 2;
static_assert((1u << PC_RSH) == PC_ROWS, "patch rows: a power of two");
constexpr uint32_t PC_Q = PC_ROWS * 64;      // receivers per step
constexpr int PC_F0 = PC_Q / BULK_THREADS;   // in-edges per thread at the mean in-degree (1)
constexpr int PC_FU = PC_F0 + 1;             // staged in-edges per thread: 11-16 sigma above the mean
constexpr uint32_t PC_NW = PC_FU * WPB;      // 64-bit used-edge words per step
constexpr uint32_t PC_MW = 16 + 16 * PC_NR;  // message slots per wave and step (mean 64 PC_NR / 7 used)
#ifndef GP_PC_AHEAD
#define GP_PC_AHEAD 2
#endif
constexpr int PC_AHEAD = GP_PC_AHEAD;        // steps between a step's in-edge decisions (message gathers) and its fold
constexpr int PC_NE = PC_AHEAD + 1;          // LDS sets of in-edge data in use

struct PsColLds {
    // in-edge data of a step, set step % PC_NE
    double2 msg[PC_NE][WPB * PC_MW];         // used random-edge messages, compacted per wave
    unsigned long long bits[PC_NE][PC_NW + 1];  // bit q % 64 of word q / 64: in-edge q of the step was used; then 0
    uint32_t wb[PC_NE][PC_NW];               // slot of the first used edge of each word
    uint32_t ind[PC_NE][PC_Q / 8];           // the step's in-degrees, a nibble per receiver
    // plane data by parity
    double2 ydn[2][WPB][64];                 // [b]: (s, w) of row y0 + 4b - 1 where it sends +y
    double2 yup[2][WPB][64];                 // [b]: (s, w) of row y0 + 4b + 4 where it sends -y
    uint8_t ydnf[2][WPB][64];                //       ... and whether it does
    uint8_t yupf[2][WPB][64];
    double2 hz[2][WPB][8];                   // [w][2k + side]: z0 - 1 (side 0) / z0 + 64 (side 1) of row k
    uint8_t hzf[2][WPB][8];
    uint32_t red[2][WPB];
};

typedef __attribute__((address_space(1))) void gvoid_t;
typedef __attribute__((address_space(3))) void lvoid_t;

__device__ __forceinline__ void dma16(const void* g, void* lds_wave_base) {
    __builtin_amdgcn_global_load_lds((gvoid_t*)g, (lvoid_t*)lds_wave_base, 16, 0, 0);
}
__device__ __forceinline__ uint32_t byte_of(uint32_t packed, int k) { return (packed >> (8 * k)) & 0xFFu; }

template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}
// v of lane + 1 (CTRL 0x130, wave_shl:1) or lane - 1 (0x138, wave_shr:1)
template <int CTRL>
__device__ __forceinline__ double2 dpp_double2(double2 v) {
    auto mv = [](double d) {
        const uint64_t u = __builtin_bit_cast(uint64_t, d);
        const uint32_t lo = dpp_u32<CTRL>((uint32_t)u), hi = dpp_u32<CTRL>((uint32_t)(u >> 32));
        return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
    };
    return make_double2(mv(v.x), mv(v.y));
}

__device__ __forceinline__ void st_stream(double2* p, double2 v) {
    __builtin_nontemporal_store(v.x, &p->x);
    __builtin_nontemporal_store(v.y, &p->y);
}

__device__ __forceinline__ uint32_t col_word(const PsColArgs& a, uint32_t x, uint32_t y, uint32_t z) {
    return ((x - a.x_lo) * a.G.g + y) * a.zs + (z >> 6);
}

// One work item: patch (yb, zsg), planes [xa, xb).
template <int TOPO, bool REMOTE>
__device__ __forceinline__ void pscol_item(const PsColArgs& a, uint32_t r, PsColLds& L, uint32_t yb, uint32_t zsg,
                                           uint32_t xa, uint32_t xb, bool all_active, uint32_t& alerts,
                                           uint32_t& newly, bool& tiny) {
    const Geom G = a.G;
    const uint32_t g = G.g, g2 = G.g2;
    const double2* __restrict__ swc = a.swc;
    const uint8_t* __restrict__ nbc = a.nbc;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const uint32_t z0 = zsg * 64, z = z0 + lane, zc = min(z, g - 1);
    const bool zv = z < g;
    const uint32_t y0 = yb * PC_ROWS, yw = y0 + PC_NR * wv;
    bool rv[PC_NR];
    uint32_t yo[PC_NR], myz[PC_NR];
#pragma unroll
    for (int k = 0; k < PC_NR; ++k) {
        const uint32_t y = yw + k;
        rv[k] = zv && y < g;
        yo[k] = min(y, g - 1) * g + zc;  // clamped: loads of invalid lanes stay in the plane
        myz[k] = (y + 1 < g ? 4u : 0u) | (y > 0 ? 8u : 0u) | (z + 1 < g ? 16u : 0u) | (z > 0 ? 32u : 0u);
    }
    // halo rows of the patch: wave 0 the row y0 - 1, wave 3 the row y0 + PC_ROWS
    const bool hw = (wv == 0 && y0 > 0) || (wv == WPB - 1 && y0 + PC_ROWS < g);  // wave-uniform
    const uint32_t hoff = (hw ? (wv == 0 ? y0 - 1 : y0 + PC_ROWS) : min(yw, g - 1)) * g + zc;
    const bool hv = hw && zv;
    // halo columns: lane l < 2 PC_NR of every wave, row k = l / 2, side l % 2 (z0 - 1 / z0 + 64)
    const uint32_t zk = (lane >> 1) & (PC_NR - 1u), zside = lane & 1u;
    const bool zhv = lane < 2 * PC_NR && yw + zk < g && (zside ? z0 + 64 < g : z0 > 0);
    const uint32_t zhoff = min(yw + zk, g - 1) * g + (zside ? min(z0 + 64, g - 1) : (z0 > 0 ? z0 - 1 : 0u));
    // steps of this patch: step(x) = sbase + x - x_lo; pc_soff read one step ahead of use
    const uint32_t nx = a.x_hi - a.x_lo;
    const int64_t sbase = (int64_t)(yb * a.zs + zsg) * nx - (int64_t)a.x_lo;
    auto soff_at = [&](int64_t x) -> uint32_t {
        int64_t s = sbase + x;
        s = s < 0 ? 0 : (s > (int64_t)a.nsteps ? (int64_t)a.nsteps : s);
        return a.soff[s];
    };
    // planes the node arrays hold: [pl_lo, pl_hi)
    const uint32_t pl_lo = a.ext_lo / g2, pl_hi = a.ext_hi / g2;

    double2 sp[PC_NR], sc[PC_NR], sn[PC_NR];
    uint32_t bp = 0x07070707u, bc = 0x07070707u, bn = 0x07070707u;
#pragma unroll
    for (int k = 0; k < PC_NR; ++k) sp[k] = sc[k] = sn[k] = make_double2(0.0, 1.0);
    uint32_t raw[PC_FU];
#pragma unroll
    for (int m = 0; m < PC_FU; ++m) raw[m] = 0u;
    uint32_t hb = DIR_NONE, zhb = DIR_NONE;
    uint32_t dslot = 0, dslot_n = 0;  // direction slots of planes i, i + 1 (a byte per row)
    const int64_t ia = (int64_t)xa - (PC_AHEAD + 1 > 3 ? PC_AHEAD + 1 : 3);
    // first edges of the steps i .. i + PC_AHEAD + 2 (pc_soff read ahead of use)
    uint32_t ev[PC_AHEAD + 3];
#pragma unroll
    for (int t = 0; t < PC_AHEAD + 3; ++t) ev[t] = TOPO == IMP3D ? soff_at(ia + t) : 0u;

    for (int64_t i = ia; i < (int64_t)xb; ++i) {
        // ---- (2a) decide step i + PC_AHEAD's in-edges: sender draws, message gathers
        const int64_t ex_ = i + PC_AHEAD;
        if (TOPO == IMP3D && ex_ >= (int64_t)xa && ex_ < (int64_t)xb) {
            const int es = (int)(ex_ % PC_NE);
            const uint32_t e_b = ev[PC_AHEAD];
            {
                if (wv == 0 && lane < PC_Q / 32)  // the step's nibble in-degrees (PC_Q / 2 bytes)
                    dma16(a.ind4 + ((uint64_t)(sbase + ex_) * (PC_Q / 2) + lane * 16), &L.ind[es][0]);
                const uint32_t cnt = ev[PC_AHEAD + 1] - e_b;
                uint32_t isrc[PC_FU];
                bool sent[PC_FU];
#pragma unroll
                for (int m = 0; m < PC_FU; ++m) isrc[m] = raw[m] & 0x3FFFFFFFu;
                uint32_t x[PC_FU], y[PC_FU];
                {
                    // the first PC_F0 edges per thread cover the mean in-degree of a step; the
                    // last is drawn only by waves that hold an edge there
                    uint32_t n0[PC_F0], x0[PC_F0], y0_[PC_F0];
#pragma unroll
                    for (int m = 0; m < PC_F0; ++m) n0[m] = isrc[m];
                    philox2_batch<PC_F0>(n0, r, S_PUSHSUM, a.k0, a.k1, x0, y0_);
#pragma unroll
                    for (int m = 0; m < PC_F0; ++m) {
                        x[m] = x0[m];
                        y[m] = y0_[m];
                    }
                    x[PC_F0] = y[PC_F0] = 0u;
                    if (cnt > (uint32_t)PC_F0 * BULK_THREADS + (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x & ~63u)) {
                        uint32_t n1[1] = {isrc[PC_F0]}, x1[1], y1[1];
                        philox2_batch<1>(n1, r, S_PUSHSUM, a.k0, a.k1, x1, y1);
                        x[PC_F0] = x1[0];
                        y[PC_F0] = y1[0];
                    }
                }
                bool pick[PC_FU];
#pragma unroll
                for (int m = 0; m < PC_FU; ++m) {
                    const uint32_t q = threadIdx.x + m * BULK_THREADS;
                    const uint32_t di = (raw[m] >> 30) + 4u;
                    // every node active: a remote sender's draw decides too (no tag)
                    const bool local = !REMOTE || all_active || isrc[m] - a.lo < a.nloc;
                    pick[m] = q < cnt && local && uniform_from(x[m], y[m], di) == di - 1u;
                }
                if (all_active) {
#pragma unroll
                    for (int m = 0; m < PC_FU; ++m) sent[m] = pick[m];
                } else {
                    // activation: the pick must also have been active -- the ballot bitmap of
                    // round r's sends (column layout), read for the picks only, all in flight
                    unsigned long long wb_[PC_FU];
                    uint32_t zb[PC_FU];
#pragma unroll
                    for (int m = 0; m < PC_FU; ++m) {
                        const uint32_t i_ = pick[m] ? isrc[m] : a.lo;
                        const uint32_t xs = fastdiv(i_, G.div_g2);
                        const uint32_t rem = i_ - xs * g2;
                        const uint32_t ys = fastdiv(rem, G.div_g);
                        const uint32_t zs_ = rem - ys * g;
                        zb[m] = zs_ & 63u;
                        wb_[m] = a.rbc[col_word(a, xs, ys, zs_)];
                    }
#pragma unroll
                    for (int m = 0; m < PC_FU; ++m) asm volatile("" : "+v"(wb_[m])::"memory");
#pragma unroll
                    for (int m = 0; m < PC_FU; ++m) sent[m] = pick[m] && ((wb_[m] >> zb[m]) & 1ull);
                }
                if (REMOTE && !all_active) {  // sender on another rank, activation: the exchange tagged its message
#pragma unroll
                    for (int m = 0; m < PC_FU; ++m) {
                        const uint32_t q = threadIdx.x + m * BULK_THREADS;
                        if (q < cnt && isrc[m] - a.lo >= a.nloc) sent[m] = a.rtag[e_b + q] == r;
                    }
                }
                // used edges: ballot word per (m, wave); messages compacted into the wave's
                // slots -- each used edge's source address goes to lane `rank` by ds_permute,
                // then one LDS-DMA of the first `count` lanes
                uint32_t run = 0;
#pragma unroll
                for (int m = 0; m < PC_FU; ++m) {
                    const unsigned long long bal = __ballot(sent[m]);
                    const uint32_t nb_ = (uint32_t)__popcll(bal);
                    const uint32_t rk = lane_prefix(bal);
                    if (lane == 0) {
                        L.bits[es][m * WPB + wv] = bal;
                        L.wb[es][m * WPB + wv] = wv * PC_MW + run;
                    }
                    if (nb_ && run < PC_MW) {  // wave-uniform
                        const uint32_t q = threadIdx.x + m * BULK_THREADS;
                        const double2* srcp = (REMOTE && isrc[m] - a.lo >= a.nloc) ? a.rmsg + (e_b + q) : swc + isrc[m];
                        const uint64_t ad = reinterpret_cast<uint64_t>(srcp);
                        const uint32_t dst = sent[m] ? rk : nb_ + (lane - rk);
                        const uint32_t alo = (uint32_t)__builtin_amdgcn_ds_permute((int)(dst * 4u), (int)(uint32_t)ad);
                        const uint32_t ahi = (uint32_t)__builtin_amdgcn_ds_permute((int)(dst * 4u), (int)(uint32_t)(ad >> 32));
                        if (lane < nb_ && run + lane < PC_MW)
                            dma16(reinterpret_cast<const void*>(((uint64_t)ahi << 32) | alo), &L.msg[es][wv * PC_MW + run]);
                    }
                    run += nb_;
                }
                if (threadIdx.x == 0) L.bits[es][PC_NW] = 0ull;
            }
        }
        // ---- (2b) decide plane i + 1: halo gathers, direction draws, boundary rows
        const int64_t dx = i + 1;
        if (dx >= (int64_t)xa && dx < (int64_t)xb) {
            const int par = (int)(dx & 1);
            const uint32_t px = (uint32_t)dx * g2;
            // halo rows and columns of plane i + 1: gathered only where that node sends into the patch
            {
                const bool up = wv == 0;  // wave 0: row y0 - 1 sending +y (dir 2); wave 3: row y0 + 16 sending -y (dir 3)
                const bool need = hv && (hb & DIR_MASK) == (up ? 2u : 3u);
                if (hw) {
                    if (up) L.ydnf[par][0][lane] = need ? 1 : 0;
                    else L.yupf[par][WPB - 1][lane] = need ? 1 : 0;
                    if (need) {
                        if (up) dma16(swc + px + hoff, &L.ydn[par][0][0]);
                        else dma16(swc + px + hoff, &L.yup[par][WPB - 1][0]);
                    }
                } else if (wv == 0 || wv == WPB - 1) {
                    if (wv == 0) L.ydnf[par][0][lane] = 0;
                    else L.yupf[par][WPB - 1][lane] = 0;
                }
                const bool zneed = zhv && (zhb & DIR_MASK) == (zside ? 5u : 4u);
                if (lane < 2 * PC_NR) L.hzf[par][wv][lane] = zneed ? 1 : 0;
                if (zneed) dma16(swc + px + zhoff, &L.hz[par][wv][0]);
            }
            // next-round direction slots of plane i + 1's nodes, U(deg) of their draws (counter
            // (j, r + 1), independent of the state), consumed by the fold of the next step
            {
                const uint32_t xbn = (dx > 0 ? 1u : 0u) | (dx + 1 < (int64_t)g ? 2u : 0u);
                uint32_t node[PC_NR], x[PC_NR], y[PC_NR];
#pragma unroll
                for (int k = 0; k < PC_NR; ++k) node[k] = px + yo[k];
                philox2_batch<PC_NR>(node, r + 1, S_PUSHSUM, a.k0, a.k1, x, y);
                dslot_n = 0;
#pragma unroll
                for (int k = 0; k < PC_NR; ++k)
                    dslot_n |= uniform_from(x[k], y[k], popc6(myz[k] | xbn) + (TOPO == IMP3D ? 1u : 0u)) << (8 * k);
            }
            // boundary rows of plane i + 1 (sn) for the neighbour waves
            if (wv > 0) {
                const bool s0 = rv[0] && (byte_of(bn, 0) & DIR_MASK) == 3u;  // row 0 sends -y
                L.yupf[par][wv - 1][lane] = s0 ? 1 : 0;
                if (s0) L.yup[par][wv - 1][lane] = sn[0];
            }
            if (wv < WPB - 1) {
                const bool s3 = rv[PC_NR - 1] && (byte_of(bn, PC_NR - 1) & DIR_MASK) == 2u;  // row 3 sends +y
                L.ydnf[par][wv + 1][lane] = s3 ? 1 : 0;
                if (s3) L.ydn[par][wv + 1][lane] = sn[PC_NR - 1];
            }
        }

        // ---- (1) loads for the next steps: plane i + 2, in-edge senders of step i + 2, halo bytes of plane i + 2
        const int64_t p2 = i + 2;
        const bool pl_ok = p2 >= (int64_t)xa - 1 && p2 <= (int64_t)xb && p2 >= (int64_t)pl_lo && p2 < (int64_t)pl_hi;
        const uint32_t p2c = (uint32_t)(pl_ok ? p2 : (int64_t)pl_lo);
        double2 sn2[PC_NR];
        uint32_t bn2 = 0x07070707u, hb2 = DIR_NONE, zhb2 = DIR_NONE;
        {
            uint32_t lb[PC_NR];
#pragma unroll
            for (int k = 0; k < PC_NR; ++k) {
                sn2[k] = swc[p2c * g2 + yo[k]];
                lb[k] = nbc[p2c * g2 + yo[k]];
            }
            uint32_t lh = nbc[p2c * g2 + hoff];
            uint32_t lz = nbc[p2c * g2 + zhoff];
            if (pl_ok) {
#pragma unroll
                for (int k = 0; k < PC_NR; ++k) bn2 = (bn2 & ~(0xFFu << (8 * k))) | ((rv[k] ? lb[k] : DIR_NONE) << (8 * k));
                hb2 = hv ? lh : DIR_NONE;
                zhb2 = zhv ? lz : DIR_NONE;
            }
        }
        uint32_t raw2[PC_FU];  // in-edge senders of step i + PC_AHEAD + 1
        uint32_t e_new = 0;
        if (TOPO == IMP3D) {
            const uint32_t e_c = ev[PC_AHEAD + 1], cnt2 = ev[PC_AHEAD + 2] - e_c;
            const bool ed_ok = i + PC_AHEAD + 1 >= (int64_t)xa && i + PC_AHEAD + 1 < (int64_t)xb;
#pragma unroll
            for (int m = 0; m < PC_FU; ++m) {
                const uint32_t q = threadIdx.x + m * BULK_THREADS;
                raw2[m] = __builtin_nontemporal_load(a.src + e_c + (cnt2 && ed_ok ? min(q, cnt2 - 1u) : 0u));
            }
            e_new = soff_at(i + PC_AHEAD + 3);
        }

        // ---- (3) fold plane i
        if (i >= (int64_t)xa) {
            const uint32_t xi = (uint32_t)i;
            const int par = (int)(i & 1);
            const int es = (int)(i % PC_NE);
            const uint32_t e_a = ev[0];
            const uint32_t px = xi * g2;
            const uint32_t xbits = (xi > 0 ? 1u : 0u) | (xi + 1 < g ? 2u : 0u);
            // Imp3D: receiver q's in-edges are [pre(q), pre(q) + d(q)) of the step, pre = the
            // exclusive prefix of the nibble in-degrees: every wave sums the 16 chunks of 64
            // receivers (lane L: receivers 16L..16L+15) and keeps the chunk prefixes; the part
            // inside a chunk comes from ballots of the degree bits (every d <= 14, checked at
            // create)
            uint32_t cinc = 0;
            if (TOPO == IMP3D) {
                const uint2 w2 = lane < PC_Q / 16 ? reinterpret_cast<const uint2*>(L.ind[es])[lane] : make_uint2(0u, 0u);
                auto nsum = [](uint32_t w_) { return (((w_ & 0x0F0F0F0Fu) + ((w_ >> 4) & 0x0F0F0F0Fu)) * 0x01010101u) >> 24; };
                uint32_t incl = nsum(w2.x) + nsum(w2.y);
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const uint32_t t = __shfl_up(incl, o, 64);
                    if (lane >= (uint32_t)o) incl += t;
                }
                const uint32_t ex = __shfl_up(incl, 1, 64);
                cinc = lane == 0 ? 0u : ex;
            }
            // z +- 1 senders: the neighbour lanes' bytes and (s, w) by DPP; the wave's end
            // lanes take the gathered halo columns
            const uint32_t bcl = dpp_u32<0x138>(bc), bcr = dpp_u32<0x130>(bc);
            const uint2 hzf = *reinterpret_cast<const uint2*>(&L.hzf[par][wv][0]);  // flag bytes 2k + side (8 max)
            uint32_t pend = 0;  // per row, 8 bits: 0-5 mask, 6 draw a direction; bits 4k..: flags
            uint32_t pfl = 0;
            const double2 zero = make_double2(0.0, 0.0);
#pragma unroll
            for (int k = 0; k < PC_NR; ++k) {
                const uint32_t b = byte_of(bc, k);
                const uint32_t mask = rv[k] ? (myz[k] | xbits) : 0u;
                const uint32_t hzk = k < 2 ? hzf.x : hzf.y;
                bool fz1, fz0;  // z + 1 sends -z (dir 5), z - 1 sends +z (dir 4)
                if (lane == 63u) fz1 = byte_of(hzk, (2 * k + 1) & 3) != 0;
                else fz1 = (byte_of(bcr, k) & DIR_MASK) == 5u;
                if (lane == 0u) fz0 = byte_of(hzk, (2 * k) & 3) != 0;
                else fz0 = (byte_of(bcl, k) & DIR_MASK) == 4u;
                bool fy1, fy0;  // y + 1 sends -y (dir 3), y - 1 sends +y (dir 2)
                if (k + 1 < PC_NR) fy1 = (byte_of(bc, k + 1 < PC_NR ? k + 1 : k) & DIR_MASK) == 3u;
                else fy1 = L.yupf[par][wv][lane] != 0;
                if (k > 0) fy0 = (byte_of(bc, k > 0 ? k - 1 : k) & DIR_MASK) == 2u;
                else fy0 = L.ydnf[par][wv][lane] != 0;
                const bool fx0 = (byte_of(bp, k) & DIR_MASK) == 1u, fx1 = (byte_of(bn, k) & DIR_MASK) == 0u;
                const uint32_t from = mask & ((fx0 ? 1u : 0u) | (fx1 ? 2u : 0u) | (fy1 ? 4u : 0u) | (fy0 ? 8u : 0u) |
                                              (fz1 ? 16u : 0u) | (fz0 ? 32u : 0u));
                // messages (all lanes run the DPP; wave-end lanes take the halo column)
                double2 mz1 = dpp_double2<0x130>(sc[k]), mz0 = dpp_double2<0x138>(sc[k]);
                if (lane == 63u) mz1 = L.hz[par][wv][2 * k + 1];
                if (lane == 0u) mz0 = L.hz[par][wv][2 * k];
                const double2 my1 = k + 1 < PC_NR ? sc[k + 1 < PC_NR ? k + 1 : k] : L.yup[par][wv][lane];
                const double2 my0 = k > 0 ? sc[k > 0 ? k - 1 : k] : L.ydn[par][wv][lane];

                // this node's in-edge range (every lane takes part in the ballots)
                uint32_t epre = 0, edeg = 0;
                if (TOPO == IMP3D) {
                    const uint32_t ql = (PC_NR * wv + k) * 64u + lane;
                    const uint32_t d = (reinterpret_cast<const uint8_t*>(L.ind[es])[ql >> 1] >> ((ql & 1u) * 4u)) & 15u;
                    uint32_t ex = lane_prefix(__ballot(d & 1u)) + 2u * lane_prefix(__ballot(d & 2u));
                    if (__ballot(d >= 4u)) ex += 4u * lane_prefix(__ballot(d & 4u)) + 8u * lane_prefix(__ballot(d & 8u));
                    epre = (uint32_t)__builtin_amdgcn_readlane((int)cinc, (int)(4u * (PC_NR * wv + k))) + ex;
                    edeg = d;
                }
                if (rv[k]) {
                    const uint32_t deg = popc6(mask) + (TOPO == IMP3D ? 1u : 0u);
                    bool active = (b & B_ACTIVE) != 0;
                    const double2 sv = sc[k];
                    const double hf = (active && deg > 0) ? 0.5 : 1.0;  // exact either way
                    double acc_s = sv.x * hf, acc_w = sv.y * hf;
                    // fma(m, 0.5, acc) rounds once, exactly like acc + m * 0.5 while m * 0.5 is
                    // exact (|m| >= 2^-1021): every node checks its round-start (s, w), the
                    // values its messages carry, against 2^-1020 (Ctl::tiny fails the batch)
                    auto fold = [&](const double2 mi) {
                        acc_s = __builtin_fma(mi.x, 0.5, acc_s);
                        acc_w = __builtin_fma(mi.y, 0.5, acc_w);
                    };
                    tiny |= (sv.y < 0x1p-1020) | (sv.x != 0.0 && sv.x < 0x1p-1020);
                    bool recv = from != 0;
                    fold((from & 1u) ? sp[k] : zero);
                    fold((from & 2u) ? sn[k] : zero);
                    fold((from & 4u) ? my1 : zero);
                    fold((from & 8u) ? my0 : zero);
                    fold((from & 16u) ? mz1 : zero);
                    fold((from & 32u) ? mz0 : zero);
                    if (TOPO == IMP3D) {
                        // used in-edges: the node's window of the step bitmap, 32 bits at a time,
                        // walked set bit by set bit (ascending sender = canonical order)
                        const uint32_t* bw = reinterpret_cast<const uint32_t*>(L.bits[es]);
                        const uint32_t qe = epre + edeg;
                        for (uint32_t q0 = epre; q0 < qe; q0 += 32u) {
                            uint32_t win = __builtin_amdgcn_alignbit(bw[(q0 >> 5) + 1], bw[q0 >> 5], q0 & 31u);
                            if (qe - q0 < 32u) win &= (1u << (qe - q0)) - 1u;
                            while (win) {
                                const uint32_t q = q0 + (uint32_t)__builtin_ctz(win);
                                win &= win - 1u;
                                const uint32_t wd = q >> 6;
                                const unsigned long long below = L.bits[es][wd] & ((1ull << (q & 63u)) - 1ull);
                                const uint32_t slot = L.wb[es][wd] + (uint32_t)__popcll(below);
                                // (unconditional LDS read with a clamped slot: as two branches the
                                // compiler merged the LDS and HBM reads into one flat load)
                                double2 mi = L.msg[es][min(slot, WPB * PC_MW - 1u)];
                                asm volatile("" : "+v"(mi.x), "+v"(mi.y));
                                if (slot >= ((wd % WPB) + 1u) * PC_MW) {  // the wave's slots overflowed (never expected): HBM
                                    const uint32_t i_ = a.src[e_a + q] & 0x3FFFFFFFu;
                                    mi = (REMOTE && i_ - a.lo >= a.nloc) ? a.rmsg[e_a + q] : swc[i_];
                                }
                                fold(mi);
                                recv = true;
                            }
                        }
                    }
                    uint32_t flags = b & (B_ACTIVE | B_CONV | (3u << CNT_SHIFT));
                    if (recv) {
                        if (!(b & B_CONV)) {
                            uint32_t cnt3 = (b >> CNT_SHIFT) & 3u;
                            cnt3 = ratio_moved(sv.x, sv.y, acc_s, acc_w) ? 0u : cnt3 + 1u;
                            flags = (flags & ~(3u << CNT_SHIFT)) | (cnt3 << CNT_SHIFT);
                            if (cnt3 == 3) {
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
                    pend |= (mask | (active && deg > 0 ? 64u : 0u)) << (8 * k);
                    pfl |= (flags >> 3) << (8 * k);
                    st_stream(a.swn + px + yo[k], make_double2(acc_s, acc_w));
                }
            }
            // next-round directions: the slots drawn a step ahead (dslot)
#pragma unroll
            for (int k = 0; k < PC_NR; ++k) {
                const uint32_t pk = byte_of(pend, k), mask = pk & 63u;
                uint32_t dir = DIR_NONE;
                if (pk & 64u) dir = slot_to_dir_fast(mask, byte_of(dslot, k));
                if (rv[k]) a.nbn[px + yo[k]] = (uint8_t)((byte_of(pfl, k) << 3) | dir);
                if (TOPO == IMP3D && !all_active) {  // activation: ballot bitmap of next round's random-edge sends
                    const unsigned long long bits = __ballot(rv[k] && dir == DIR_RANDOM);
                    if (lane == 0 && yw + k < g) a.rbn[col_word(a, xi, yw + k, z0)] = bits;
                }
            }
        }

        __syncthreads();  // this step's loads, gathers and LDS writes are complete

        // ---- (4) rotate the window
#pragma unroll
        for (int k = 0; k < PC_NR; ++k) {
            sp[k] = sc[k];
            sc[k] = sn[k];
            sn[k] = sn2[k];
        }
        dslot = dslot_n;
        bp = bc;
        bc = bn;
        bn = bn2;
        hb = hb2;
        zhb = zhb2;
        if (TOPO == IMP3D) {
#pragma unroll
            for (int m = 0; m < PC_FU; ++m) raw[m] = raw2[m];
#pragma unroll
            for (int t = 0; t + 1 < PC_AHEAD + 3; ++t) ev[t] = ev[t + 1];
            ev[PC_AHEAD + 2] = e_new;
        }
    }
}

// Block sums of alerts / newly active (valid in thread 0).
__device__ __forceinline__ void pc_block_counts(uint32_t (*red)[WPB], uint32_t& x, uint32_t& y) {
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        x += __shfl_xor(x, o, 64);
        y += __shfl_xor(y, o, 64);
    }
    if (lane == 0) {
        red[0][wv] = x;
        red[1][wv] = y;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        x = 0;
        y = 0;
        for (int w = 0; w < WPB; ++w) {
            x += red[0][w];
            y += red[1][w];
        }
    }
}

template <int TOPO, bool REMOTE>
__global__ __launch_bounds__(BULK_THREADS, GP_PC_MINW) void k_ps_col(PsColArgs a, uint32_t r) {
    __shared__ PsColLds L;
    Ctl* ctl = a.ctl;
    if (ld_agent(&ctl->done)) return;
    const bool all_active = ld_agent(&ctl->all_active) != 0;
    uint32_t alerts = 0, newly = 0;
    bool tiny = false;
    // work items dealt per XCD (blocks b with equal b % 8): XCD c owns the y-band of
    // patches yb in [YB c / 8, YB (c + 1) / 8) of every z-segment and x-segment, so
    // the halo rows a patch gathers were streamed by its y-neighbours on the same XCD
    const uint32_t c = blockIdx.x & 7u, kk = blockIdx.x >> 3;
    const uint32_t yb0 = a.yb * c / 8, nyb = a.yb * (c + 1) / 8 - yb0;
    if (nyb && kk < nyb * a.zs * a.nseg) {
        const uint32_t yb = yb0 + kk % nyb, t = kk / nyb;
        const uint32_t zsg = t % a.zs, seg = t / a.zs;
        const uint32_t xa = a.x_lo + seg * a.xs_len, xb = min(a.x_hi, xa + a.xs_len);
        if (xa < xb) pscol_item<TOPO, REMOTE>(a, r, L, yb, zsg, xa, xb, all_active, alerts, newly, tiny);
    }
    if (__ballot(tiny) && (threadIdx.x & 63u) == 0) atomicOr(&ctl->tiny, 1u);
    pc_block_counts(L.red, alerts, newly);
    if (threadIdx.x == 0) {
        if (a.fuse == 2) {
            block_done_close_sharded(ctl, a.G.P, a.G.T, r, alerts, newly);
        } else {
            if (alerts) atomicAdd(&ctl->round_alerts, (unsigned long long)alerts);
            if (newly) atomicAdd(&ctl->round_active, (unsigned long long)newly);
        }
    }
}

// ---------------------------------------------------------------- setup kernels
// Patch key of receiver t (its owner's slab: planes [x_lo, x_lo + nx), key base kb):
// kb + ((yb * zsegs + zs) * nx + x - x_lo) * PC_Q + (y % PC_ROWS) * 64 + z % 64.
__global__ __launch_bounds__(BULK_THREADS) void k_pc_keys(const uint32_t* __restrict__ rnd, uint32_t n,
                                                          uint32_t* __restrict__ key, Geom G, PcKeyPlan kp) {
    for (uint32_t i = blockIdx.x * BULK_THREADS + threadIdx.x; i < n; i += gridDim.x * BULK_THREADS) {
        const uint32_t t = rnd[i];
        const uint32_t x = fastdiv(t, G.div_g2);
        const uint32_t rem = t - x * G.g2;
        const uint32_t y = fastdiv(rem, G.div_g);
        const uint32_t z = rem - y * G.g;
        int w = 0;
        for (int v = 1; v < kp.W; ++v) w += x >= kp.x_lo[v] ? 1 : 0;
        const uint32_t nx = kp.x_lo[w + 1] - kp.x_lo[w];
        key[i] = kp.kbase[w] + (((y >> PC_RSH) * kp.zs + (z >> 6)) * nx + (x - kp.x_lo[w])) * PC_Q +
                 (y & (PC_ROWS - 1u)) * 64u + (z & 63u);
    }
}

// Per-step first edges (relative to the rank's first edge) and nibble in-degrees
// of one slab from the global per-key counts / offsets; largest in-degree and
// largest step edge count into stat[0], stat[1] (atomicMax).
__global__ __launch_bounds__(BULK_THREADS) void k_pc_slab(const uint32_t* __restrict__ off_all,
                                                          const uint32_t* __restrict__ counts, uint32_t kbase,
                                                          uint32_t nsteps, uint32_t edge0, uint32_t* __restrict__ soff,
                                                          uint8_t* __restrict__ ind4, uint32_t* stat) {
    uint32_t mdeg = 0, mstep = 0;
    const uint32_t nb = nsteps * (PC_Q / 2);
    for (uint32_t b = blockIdx.x * BULK_THREADS + threadIdx.x; b < nb; b += gridDim.x * BULK_THREADS) {
        const uint32_t d0 = counts[kbase + 2 * b], d1 = counts[kbase + 2 * b + 1];
        mdeg = max(mdeg, max(d0, d1));
        ind4[b] = (uint8_t)(min(d0, 15u) | (min(d1, 15u) << 4));
    }
    for (uint32_t s = blockIdx.x * BULK_THREADS + threadIdx.x; s <= nsteps; s += gridDim.x * BULK_THREADS) {
        const uint32_t o = off_all[kbase + s * PC_Q];
        soff[s] = o - edge0;
        if (s < nsteps) mstep = max(mstep, off_all[kbase + (s + 1) * PC_Q] - o);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mdeg = max(mdeg, (uint32_t)__shfl_xor(mdeg, o, 64));
        mstep = max(mstep, (uint32_t)__shfl_xor(mstep, o, 64));
    }
    if ((threadIdx.x & 63u) == 0) {
        atomicMax(&stat[0], mdeg);
        atomicMax(&stat[1], mstep);
    }
}

}  // namespace

uint32_t pscol_step_capacity() { return PC_FU * BULK_THREADS; }
uint32_t pscol_patch_rows() { return PC_ROWS; }
uint32_t pscol_step_receivers() { return PC_Q; }

int pscol_blocks_per_cu(int topo, bool remote) {
    const void* f = topo == GRID3D ? (const void*)k_ps_col<GRID3D, false>
                    : remote       ? (const void*)k_ps_col<IMP3D, true>
                                   : (const void*)k_ps_col<IMP3D, false>;
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, f, BULK_THREADS, 0) != hipSuccess || n < 1) n = 1;
    return n;
}

PsColArgs make_pscol_args(const DevState& S, uint32_t round) {
    const int cur = round & 1;
    PsColArgs a{};
    a.swc = S.sw[cur] - S.base;
    a.swn = S.sw[cur ^ 1] - S.base;
    a.nbc = S.nb[cur] - S.base;
    a.nbn = S.nb[cur ^ 1] - S.base;
    a.rbc = S.rbits[cur];
    a.rbn = S.rbits[cur ^ 1];
    a.src = S.pc_src;
    a.soff = S.pc_soff;
    a.ind4 = S.pc_ind4;
    a.rtag = S.rtag;
    a.rmsg = S.rmsg;
    a.ctl = S.ctl;
    a.G = S.G;
    a.k0 = S.k0;
    a.k1 = S.k1;
    a.lo = S.lo;
    a.nloc = S.nloc;
    a.ext_lo = S.ext_lo;
    a.ext_hi = S.ext_hi;
    const uint32_t g = S.G.g;
    a.x_lo = S.lo / S.G.g2;
    a.x_hi = (S.lo + S.nloc) / S.G.g2;
    a.zs = (g + 63) / 64;
    a.yb = (g + PC_ROWS - 1) / PC_ROWS;
    const uint32_t planes = a.x_hi - a.x_lo;
    const uint32_t xs = S.col_xsegs ? S.col_xsegs : 1u;
    a.xs_len = (planes + xs - 1) / xs;
    a.nseg = a.xs_len ? (planes + a.xs_len - 1) / a.xs_len : 0u;
    a.nsteps = S.pc_nsteps;
    a.fuse = S.fuse_finalize;
    return a;
}

// Blocks of the push-sum column kernel: 8 x the largest per-XCD item count.
uint32_t pscol_grid(const DevState& S) {
    const PsColArgs a = make_pscol_args(S, 0);
    uint32_t mx = 0;
    for (uint32_t c = 0; c < 8; ++c) mx = std::max(mx, (a.yb * (c + 1) / 8 - a.yb * c / 8) * a.zs * a.nseg);
    return 8u * std::max(1u, mx);
}

hipError_t launch_round_pscol(const DevState& S, uint32_t round, hipStream_t st) {
    const PsColArgs a = make_pscol_args(S, round);
    const dim3 g(pscol_grid(S)), b(BULK_THREADS);
    const bool remote = S.rtag != nullptr;
    if (S.topo == GRID3D) hipLaunchKernelGGL((k_ps_col<GRID3D, false>), g, b, 0, st, a, round);
    else if (remote) hipLaunchKernelGGL((k_ps_col<IMP3D, true>), g, b, 0, st, a, round);
    else hipLaunchKernelGGL((k_ps_col<IMP3D, false>), g, b, 0, st, a, round);
    return hipGetLastError();
}

hipError_t launch_pc_keys(const uint32_t* rnd, uint32_t n, uint32_t* key, const Geom& G, const PcKeyPlan& kp, int grid,
                          hipStream_t st) {
    hipLaunchKernelGGL(k_pc_keys, dim3(grid), dim3(BULK_THREADS), 0, st, rnd, n, key, G, kp);
    return hipGetLastError();
}

hipError_t launch_pc_slab(const uint32_t* off_all, const uint32_t* counts, uint32_t kbase, uint32_t nsteps,
                          uint32_t edge0, uint32_t* soff, uint8_t* ind4, uint32_t* stat, int grid, hipStream_t st) {
    hipLaunchKernelGGL(k_pc_slab, dim3(grid), dim3(BULK_THREADS), 0, st, off_all, counts, kbase, nsteps, edge0, soff,
                       ind4, stat);
    return hipGetLastError();
}

}  // namespace gp
