// gp_block.hip -- push-sum on a small 3D lattice held in LDS across rounds (gfx950).
//
// C2 (BASELINE config 2: 3D push-sum, n = 1e6, g = 100) is 17 bytes of state per
// node, 17 MB in all -- less than the chip's LDS (256 CUs x 160 KiB).  A round of
// the tile kernel re-streams that state through HBM and the Infinity Cache in a
// fresh launch (20.7 us per round, bound by one tile's latency); here one
// cooperative launch runs a whole batch of rounds with the lattice resident in LDS:
//
//   * the lattice is cut into NB = nbx * nby * nbz boxes (at most one per CU), one
//     1024-thread workgroup each; a box's node bytes and (s, w) live in LDS;
//   * per round a box writes its six boundary layers (node byte + (s, w)) to a
//     face buffer in global memory with device-coherent stores, the grid meets at a
//     barrier (grid_sync), and every box reads its neighbours' facing layers into
//     LDS halo arrays with device-coherent loads -- the only global traffic of a
//     round (~28 KB per box at C2);
//   * each node then folds exactly as the tile kernel (gp_round.hip) does: own half,
//     lattice messages in the receiver's slot order (Program.fs:246-257), the ratio
//     test of Program.fs:114-123 (SRS v1 B.4), the next direction by Philox -- with
//     acc + m * 0.5, the oracle's own rounding;
//   * the round's alert / newly-active counts go to a per-round accumulator; after
//     the next barrier every box reads it, so every box knows the cumulative alert
//     count and stops after the round that reaches T (Program.fs:51-56), and box 0
//     records the round in the control block (hist, totals, done) for the host.
//
// At the end of the launch the state is written back to the round's (s, w) / node
// byte buffers, so everything else (gp_read_state, the next batch) sees the usual
// layout.  Every barrier wait has a time limit: a grid that is not co-resident
// (hipLaunchCooperativeKernel refuses such a launch) or a lost block sets `err` and
// every block leaves -- the batch fails loudly instead of hanging the device.
#include <algorithm>

#include "gp_internal.hpp"

namespace gp {

namespace {

constexpr int BK_THREADS = 1024;
constexpr int BK_NPT = 5;  // nodes per thread: boxes of at most 5120 nodes
constexpr int EPOCH = BLOCK_EPOCH;  // rounds between grid barriers

struct BlockArgs {
    const double2* sw_in;   // round r0's state (id-indexed)
    double2* sw_out;        // the state after the last executed round
    double2* sw_alt;        // the other buffer (the state if the executed count is even)
    const uint8_t* nb_in;
    uint8_t* nb_out;
    uint8_t* nb_alt;
    double2* ck_sw;         // the epoch checkpoint: the input buffers (id-indexed)
    uint8_t* ck_nb;
    uint32_t* fb;           // face node bytes, one word each [2][NB][6][fmax]
    double2* fs;            // face (s, w) [2][NB][6][fmax]
    unsigned int* bar;      // barrier arrivals (zeroed before the launch)
    unsigned long long* acc;  // [3][EPOCH][2]: per-round alerts, newly active (zeroed before the launch)
    unsigned int* err;      // set by a barrier that timed out
    Ctl* ctl;
    Geom G;
    uint32_t k0, k1;
    uint32_t r0, nrounds;
    uint32_t nbx, nby, nbz, fmax, vmax;
};

__device__ __forceinline__ uint32_t split(uint32_t g, uint32_t i, uint32_t n) {
    return (uint32_t)((uint64_t)g * i / n);
}

__device__ __forceinline__ uint64_t now_10ns() { return __builtin_amdgcn_s_memrealtime(); }  // 100 MHz

// Grid barrier k (k = 1, 2, ...).  Faces are written and read with device-coherent
// (agent-scope, relaxed atomic) stores and loads, so no cache write-back or invalidate is
// needed: each wave waits for its face stores to be performed (vmcnt) before the
// workgroup barrier, thread 0 then arrives.  Arrivals are counted per group of blocks
// (blockIdx % 8: the blocks of one XCD) and the last of a group arrives on the global
// word, so no word takes more than ~NB / 8 returning atomics per barrier (one word takes
// ~88 per microsecond); counters are never reset inside a launch.  Waits at most ~2 s.
// Measured at C2 (profiles/r05/c2/): agent-scope release / acquire fences in every wave
// (an L2 write-back and invalidate each) 133 us per round; one per block 37 us; this form
// 19 us, of which 9.5 us is faces and barrier (no-node-work ablation).  Rejected: non-
// returning arrivals with the waiters polling all 8 group counters (11.4 us ablation), and
// computing the box interior while the barrier completes (22 us: the two passes over the
// node slots cost more than the wait they hide).
__device__ __forceinline__ bool grid_sync(unsigned int* bar, unsigned int k, unsigned int nb, unsigned int* err) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    __shared__ unsigned int ok;
    if (threadIdx.x == 0) {
        ok = 1u;
        const unsigned int grp = blockIdx.x & 7u;
        const unsigned int members = (nb - grp + 7u) / 8u;
        const unsigned int groups = nb < 8u ? nb : 8u;
        unsigned int* gc = bar + 16u * (1u + grp);  // a 64-byte line per group counter
        const unsigned int prev = __hip_atomic_fetch_add(gc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev + 1u == k * members) __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t t0 = now_10ns();
        while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < k * groups) {
            if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) || now_10ns() - t0 > 200000000ull) {
                __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = 0u;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __syncthreads();
    return ok != 0u;
}


}  // namespace

__global__ __launch_bounds__(BK_THREADS) void k_ps_block(BlockArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const uint32_t g = a.G.g, g2 = a.G.g2, gm = g - 1u;
    const uint32_t NB = gridDim.x;
    const uint32_t b = blockIdx.x;
    const uint32_t ix = b / (a.nby * a.nbz), iy = (b / a.nbz) % a.nby, iz = b % a.nbz;
    const uint32_t x0 = split(g, ix, a.nbx), x1 = split(g, ix + 1, a.nbx);
    const uint32_t y0 = split(g, iy, a.nby), y1 = split(g, iy + 1, a.nby);
    const uint32_t z0 = split(g, iz, a.nbz), z1 = split(g, iz + 1, a.nbz);
    const uint32_t dx = x1 - x0, dy = y1 - y0, dz = z1 - z0, dyz = dy * dz, V = dx * dyz;
    const uint32_t F = a.fmax;
    // LDS: (s, w) of the box, then of the six halos, then a zero sentinel (one array, so a
    // neighbour is one index: in the box, in a halo, or the sentinel); node bytes likewise
    // (sentinel DIR_NONE); the next round's node bytes; packed box coordinates
    const uint32_t NS = a.vmax + 6 * F;  // the sentinel's index
    double2* swl = reinterpret_cast<double2*>(lds);         // [NS + 1]
    double2* hsw = swl + a.vmax;
    uint8_t* bl = reinterpret_cast<uint8_t*>(swl + NS + 1);  // [NS + 1]
    uint8_t* hb = bl + a.vmax;
    uint8_t* bn = bl + ((NS + 1 + 3) & ~3u);                // [vmax]
    uint32_t* ct = reinterpret_cast<uint32_t*>(bn + ((a.vmax + 3) & ~3u));  // [vmax] lx | ly << 10 | lz << 20
    __shared__ uint32_t red[2][BK_THREADS / 64];
    __shared__ unsigned int bad;  // a face never came (err set): the launch ends
    __shared__ unsigned long long ecnt[2 * EPOCH];  // the epoch's per-round counts
    static_assert(2 * EPOCH <= BK_THREADS, "one count per thread");
    constexpr unsigned long long SIGN = 1ull << 63;
    // face sizes and whether the neighbour in direction f exists (slot order: x-1, x+1, y+1, y-1, z+1, z-1)
    const uint32_t fsz[6] = {dyz, dyz, dx * dz, dx * dz, dx * dy, dx * dy};
    const bool has[6] = {ix > 0, ix + 1 < a.nbx, iy + 1 < a.nby, iy > 0, iz + 1 < a.nbz, iz > 0};
    const uint32_t nbr_b[6] = {b - a.nby * a.nbz, b + a.nby * a.nbz, b + a.nbz, b - a.nbz, b + 1, b - 1};

    // the box's state into LDS
    for (uint32_t v = threadIdx.x; v < V; v += BK_THREADS) {
        const uint32_t lx = v / dyz, ly = (v - lx * dyz) / dz, lz = v - lx * dyz - ly * dz;
        const uint32_t j = (x0 + lx) * g2 + (y0 + ly) * g + (z0 + lz);
        swl[v] = a.sw_in[j];
        bl[v] = a.nb_in[j];
        ct[v] = lx | (ly << 10) | (lz << 20);  // (no divisions per node and round)
    }
    if (threadIdx.x == 0) {
        swl[NS] = make_double2(0.0, 0.0);
        bl[NS] = DIR_NONE;
        bad = 0u;
    }
    unsigned long long total = __hip_atomic_load(&a.ctl->alerts_total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned long long act = __hip_atomic_load(&a.ctl->active_total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t done_rounds = 0;  // rounds executed by this launch
    bool stop = __hip_atomic_load(&a.ctl->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
    __syncthreads();
    // One node of round r: the tile kernel's fold (own half, the lattice messages in the
    // receiver's slot order -- Program.fs:246-257 -- acc + m * 0.5, the oracle's rounding;
    // a direction without a message adds +0.0, exact for the non-negative s and w), the
    // ratio test (Program.fs:114-123), the next direction by Philox.
    auto node = [&](uint32_t v, uint32_t draw, double2& res, uint32_t& alerts, uint32_t& newly) {
        const uint32_t c = ct[v];
        const uint32_t lx = c & 1023u, ly = (c >> 10) & 1023u, lz = c >> 20;
        const uint32_t x = x0 + lx, y = y0 + ly, z = z0 + lz;
        const uint32_t mask = mask_xyz(x, y, z, gm);
        const uint32_t bt = bl[v];
        const double2 sv = swl[v];
        const bool active = (bt & B_ACTIVE) != 0;
        const uint32_t deg = popc6(mask);
        const bool halve = active && deg > 0;
        double acc_s = halve ? sv.x * 0.5 : sv.x;
        double acc_w = halve ? sv.y * 0.5 : sv.y;
        // every neighbour's byte first (in the box, in a halo, or the DIR_NONE sentinel), then the
        // (s, w) of those that send here (direction d ^ 1), folded in slot order
        const bool in[6] = {lx > 0, lx + 1 < dx, ly + 1 < dy, ly > 0, lz + 1 < dz, lz > 0};
        const uint32_t vn[6] = {v - dyz, v + dyz, v + dz, v - dz, v + 1, v - 1};
        const uint32_t hn[6] = {ly * dz + lz, ly * dz + lz, lx * dz + lz, lx * dz + lz, lx * dy + ly, lx * dy + ly};
        uint32_t u[6], from = 0;
#pragma unroll
        for (int d = 0; d < 6; ++d) {
            u[d] = !((mask >> d) & 1u) ? NS : in[d] ? vn[d] : a.vmax + d * F + hn[d];
            from |= (bl[u[d]] & DIR_MASK) == (uint32_t)(d ^ 1) ? 1u << d : 0u;
        }
        // all six reads issued together (a non-sender reads the zero sentinel NS): one LDS round
        // trip instead of one per sender (a read under a branch is waited on where it stands;
        // measured C2 7.70 -> 7.92e10 node-updates/s, profiles/r06/c2_sel)
        double2 m[6];
#pragma unroll
        for (int d = 0; d < 6; ++d) m[d] = swl[(from >> d) & 1u ? u[d] : NS];
#pragma unroll
        for (int d = 0; d < 6; ++d) {
            acc_s = acc_s + m[d].x * 0.5;  // the oracle's rounding (no fused multiply-add)
            acc_w = acc_w + m[d].y * 0.5;
        }
        uint32_t flags = bt & (B_ACTIVE | B_CONV | (3u << CNT_SHIFT));
        bool act_n = active;
        if (from) {
            if (!(bt & B_CONV)) {
                uint32_t c3 = (bt >> CNT_SHIFT) & 3u;
                c3 = ratio_moved(sv.x, sv.y, acc_s, acc_w) ? 0u : c3 + 1u;
                flags = (flags & ~(3u << CNT_SHIFT)) | (c3 << CNT_SHIFT);
                if (c3 == 3) {
                    flags |= B_CONV;
                    ++alerts;
                }
            }
            if (!active) {
                ++newly;
                flags |= B_ACTIVE;
                act_n = true;
            }
        }
        uint32_t dir = DIR_NONE;
        if (act_n && deg > 0) dir = slot_to_dir_fast(mask, draw);
        res = make_double2(acc_s, acc_w);
        bn[v] = (uint8_t)(flags | dir);
    };
    // The Philox draws of round r for this thread's node slots (the next direction's slot in
    // [0, deg), Program.fs:101-131 via SRS v1 B.3), 3 bits per slot: they depend on the node and
    // the round only, so they are computed between the face stores and the face loads.
    auto draws = [&](uint32_t r) -> uint32_t {
        uint32_t id[4], x[4], y[4], dg[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t c = ct[min(q * BK_THREADS + threadIdx.x, V - 1u)];
            const uint32_t lx = c & 1023u, ly = (c >> 10) & 1023u, lz = c >> 20;
            id[q] = (x0 + lx) * g2 + (y0 + ly) * g + (z0 + lz);
            dg[q] = popc6(mask_xyz(x0 + lx, y0 + ly, z0 + lz, gm));
        }
        philox2_batch(id, r + 1, S_PUSHSUM, a.k0, a.k1, x, y);
        uint32_t pk = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) pk |= uniform_from(x[q], y[q], dg[q]) << (3 * q);
        if (V > 4u * BK_THREADS) {  // (a fifth slot: boxes of more than 4096 nodes)
            const uint32_t c = ct[min(4u * BK_THREADS + threadIdx.x, V - 1u)];
            const uint32_t lx = c & 1023u, ly = (c >> 10) & 1023u, lz = c >> 20;
            const uint32_t dd = popc6(mask_xyz(x0 + lx, y0 + ly, z0 + lz, gm));
            pk |= uniform(a.k0, a.k1, S_PUSHSUM, (x0 + lx) * g2 + (y0 + ly) * g + (z0 + lz), r + 1, dd) << 12;
        }
        return pk;
    };
    // One round r as executed step `step` of this launch: (1) the box's boundary layers -> its face
    // buffer (parity step & 1), every word tagged with the step; (2) the neighbours' facing layers
    // of this step -> LDS halos (waiting for them by their tags); (3) every node of the box; (4)
    // commit to LDS, the round's counts into its accumulator slot (count, or not: a replay).
    // False if a neighbour's face never came (err set).
    auto one_round = [&](uint32_t r, uint32_t step, unsigned long long* slot) -> bool {
        const size_t fp = (size_t)(step & 1u) * NB;
        // every face word carries the step that wrote it: the sign bit of s and of w (both >= 0)
        // tells step s from step s - 2 (the two steps that share a face buffer), the node-byte
        // word carries step + 1 in its upper bits
        const unsigned long long tb = (unsigned long long)(((step >> 1) & 1u) ^ 1u) << 63;
        const uint32_t tw = (step + 1u) << 8;
        {
            const size_t fo = (fp + b) * 6 * F;
#pragma unroll
            for (int f = 0; f < 6; ++f) {
                if (!has[f]) continue;
                for (uint32_t t = threadIdx.x; t < fsz[f]; t += BK_THREADS) {
                    uint32_t v;
                    if (f < 2) {  // x layer: t = ly * dz + lz
                        v = (f == 0 ? 0u : dx - 1u) * dyz + t;
                    } else if (f < 4) {  // y layer: t = lx * dz + lz
                        const uint32_t lx = t / dz, lz = t - lx * dz;
                        v = lx * dyz + (f == 2 ? dy - 1u : 0u) * dz + lz;
                    } else {  // z layer: t = lx * dy + ly
                        const uint32_t lx = t / dy, ly = t - lx * dy;
                        v = lx * dyz + ly * dz + (f == 4 ? dz - 1u : 0u);
                    }
                    // device-coherent stores (agent-scope atomics), each word single-copy atomic
                    const double2 mm = swl[v];
                    unsigned long long* q = reinterpret_cast<unsigned long long*>(a.fs + fo + f * F + t);
                    __hip_atomic_store(&q[0], __builtin_bit_cast(unsigned long long, mm.x) | tb, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(&q[1], __builtin_bit_cast(unsigned long long, mm.y) | tb, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(&a.fb[fo + f * F + t], (uint32_t)bl[v] | tw, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
        // the neighbours' facing layers of this step -> LDS halos: each thread loads its entry of
        // every face at once (device-coherent loads) and loads again the entries whose tags are
        // not yet this step's -- the face words themselves are the synchronisation
        const uint32_t pk = draws(r);  // (while this step's face stores, and the neighbours', land)
        for (uint32_t t = threadIdx.x; t < F; t += BK_THREADS) {
            unsigned long long sx[6], wx[6];
            uint32_t bw[6], pend = 0;
#pragma unroll
            for (int f = 0; f < 6; ++f) pend |= (has[f] && t < fsz[f]) ? 1u << f : 0u;
            const uint32_t want = pend;
            uint64_t t0 = 0;
            while (true) {
#pragma unroll
                for (int f = 0; f < 6; ++f)
                    if ((pend >> f) & 1u) {
                        const size_t fo = ((fp + nbr_b[f]) * 6 + (f ^ 1)) * F + t;
                        unsigned long long* fq = reinterpret_cast<unsigned long long*>(a.fs + fo);
                        sx[f] = __hip_atomic_load(&fq[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        wx[f] = __hip_atomic_load(&fq[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        bw[f] = __hip_atomic_load(&a.fb[fo], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
#pragma unroll
                for (int f = 0; f < 6; ++f)
                    if (((pend >> f) & 1u) && (sx[f] & SIGN) == tb && (wx[f] & SIGN) == tb && (bw[f] & ~0xffu) == tw)
                        pend &= ~(1u << f);
                if (!pend) break;
                if (!t0) t0 = now_10ns();
                if (__hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) || now_10ns() - t0 > 200000000ull) {
                    __hip_atomic_fetch_or(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    bad = 1u;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
#pragma unroll
            for (int f = 0; f < 6; ++f)
                if ((want >> f) & 1u) {
                    hb[f * F + t] = (uint8_t)bw[f];
                    hsw[f * F + t] = make_double2(__builtin_bit_cast(double, sx[f] & ~SIGN),
                                                  __builtin_bit_cast(double, wx[f] & ~SIGN));
                }
        }
        __syncthreads();
        if (bad) return false;
        // the round for this thread's nodes: the new (s, w) of node slot q in n[q] (named
        // registers, selected by q: the slot loop is not unrolled -- unrolled, the compiler
        // interleaved all slots and spilled); the new node bytes go to bn
        uint32_t alerts = 0, newly = 0;
        double2 n0 = make_double2(0.0, 0.0), n1 = n0, n2 = n0, n3 = n0, n4 = n0;
        static_assert(BK_NPT == 5, "one named register pair per node slot");
#pragma unroll 1
        for (int q = 0; q < BK_NPT; ++q) {
            const uint32_t v = q * BK_THREADS + threadIdx.x;
            if (v >= V) break;
            double2 res;
            node(v, (pk >> (3 * q)) & 7u, res, alerts, newly);
            if (q == 0) n0 = res;
            else if (q == 1) n1 = res;
            else if (q == 2) n2 = res;
            else if (q == 3) n3 = res;
            else n4 = res;
        }
        __syncthreads();  // every node has read the round-start state
        {
            const double2 nq[BK_NPT] = {n0, n1, n2, n3, n4};
#pragma unroll
            for (int q = 0; q < BK_NPT; ++q) {
                const uint32_t v = q * BK_THREADS + threadIdx.x;
                if (v < V) {
                    swl[v] = nq[q];
                    bl[v] = bn[v];
                }
            }
        }
        uint32_t xa = alerts, xn = newly;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            xa += __shfl_xor(xa, o, 64);
            xn += __shfl_xor(xn, o, 64);
        }
        if ((threadIdx.x & 63u) == 0) {
            red[0][threadIdx.x >> 6] = xa;
            red[1][threadIdx.x >> 6] = xn;
        }
        __syncthreads();  // (also: the commit is complete before the next round's face stores)
        if (threadIdx.x == 0 && slot) {
            xa = xn = 0;
            for (int w = 0; w < BK_THREADS / 64; ++w) {
                xa += red[0][w];
                xn += red[1][w];
            }
            if (xa) __hip_atomic_fetch_add(&slot[0], (unsigned long long)xa, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (xn) __hip_atomic_fetch_add(&slot[1], (unsigned long long)xn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return true;
    };
    // the box's state to / from the checkpoint (the launch's input buffers, id-indexed): written at
    // every epoch's start, read back only for a replay (device-coherent loads: the lines the launch
    // read at its start may still sit in this CU's vector L1)
    auto box_io = [&](bool save) {
        for (uint32_t v = threadIdx.x; v < V; v += BK_THREADS) {
            const uint32_t lx = v / dyz, ly = (v - lx * dyz) / dz, lz = v - lx * dyz - ly * dz;
            const uint32_t j = (x0 + lx) * g2 + (y0 + ly) * g + (z0 + lz);
            unsigned long long* q = reinterpret_cast<unsigned long long*>(a.ck_sw + j);
            if (save) {
                q[0] = __builtin_bit_cast(unsigned long long, swl[v].x);
                q[1] = __builtin_bit_cast(unsigned long long, swl[v].y);
                a.ck_nb[j] = bl[v];
            } else {
                const unsigned long long sx = __hip_atomic_load(&q[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned long long wx = __hip_atomic_load(&q[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                swl[v] = make_double2(__builtin_bit_cast(double, sx), __builtin_bit_cast(double, wx));
                bl[v] = __hip_atomic_load(&a.ck_nb[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        __syncthreads();
    };
    // Epochs of up to EPOCH rounds: inside one, boxes wait only for their neighbours (a box runs at
    // most one round ahead of each neighbour); at its end the grid meets once, every box reads the
    // epoch's per-round counts and finds the round R (if any) in which the cumulative alerts reach
    // T.  The boxes have then run past R, so each reloads the epoch's starting state (checkpoint)
    // and runs the epoch's rounds again up to R -- the same arithmetic, so the same state -- and the
    // launch ends after round R (Program.fs:51-56).
    // (One box: epochs of one round -- it checks after every round, nothing to replay.)
    const uint32_t E = NB > 1 ? (uint32_t)EPOCH : 1u;
    uint32_t step = 0, epoch = 0;
    for (uint32_t e0 = 0; e0 < a.nrounds && !stop; e0 += E, ++epoch) {
        const uint32_t n = min(E, a.nrounds - e0);
        unsigned long long* slots = a.acc + 2 * EPOCH * (epoch % 3u);
        if (NB > 1 && e0 > 0) box_io(true);  // (epoch 0: the checkpoint is the input)
        bool ok = true;
        for (uint32_t k = 0; k < n && ok; ++k) ok = one_round(a.r0 + e0 + k, step++, slots + 2 * k);
        if (!ok) break;
        // the epoch's barrier (a grid barrier for several boxes): every count of its rounds is in
        if (NB > 1 && !grid_sync(a.bar, epoch + 1u, NB, a.err)) break;
        if (NB == 1) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
        // the epoch's counts into LDS (one load per thread), then every thread scans them
        if (threadIdx.x < 2 * n) ecnt[threadIdx.x] = __hip_atomic_load(&slots[threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        uint32_t last = n;  // rounds of the epoch that count
        bool conv = false;
        unsigned long long tot = total, ac = act;
        for (uint32_t k = 0; k < n; ++k) {
            tot += ecnt[2 * k];
            ac += ecnt[2 * k + 1];
            if (tot >= a.G.T) {
                last = k + 1;
                conv = true;
                break;
            }
        }
        if (b == 0) {
            Ctl* ctl = a.ctl;
            if (threadIdx.x < last) ctl->hist[(a.r0 + e0 + threadIdx.x) % HIST] = ecnt[2 * threadIdx.x];
            if (threadIdx.x == 0) {
                __hip_atomic_store(&ctl->alerts_total, tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&ctl->active_total, ac, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (ac >= a.G.P) __hip_atomic_store(&ctl->all_active, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (tot >= a.G.T) __hip_atomic_store(&ctl->done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            // the slots of epoch + 2 (every box read them, for epoch - 1, before arriving here)
            unsigned long long* zz = a.acc + 2 * EPOCH * ((epoch + 2u) % 3u);
            if (threadIdx.x < 2 * EPOCH) __hip_atomic_store(&zz[threadIdx.x], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (conv) {  // converged in round a.r0 + e0 + last - 1: back to the epoch's start, replay
            if (last < n) {
                box_io(false);
                for (uint32_t k = 0; k < last && ok; ++k) ok = one_round(a.r0 + e0 + k, step++, nullptr);
                if (!ok) break;
            }
            done_rounds += last;
            total = tot;
            stop = true;
            break;
        }
        done_rounds += n;
        total = tot;
        act = ac;
    }
    // the state after the last executed round, into that round's buffers (the tile kernel's
    // convention: round r writes buffer (r + 1) & 1)
    __syncthreads();
    double2* swo = (done_rounds & 1u) ? a.sw_out : a.sw_alt;
    uint8_t* nbo = (done_rounds & 1u) ? a.nb_out : a.nb_alt;
    for (uint32_t v = threadIdx.x; v < V; v += BK_THREADS) {
        const uint32_t lx = v / dyz, ly = (v - lx * dyz) / dz, lz = v - lx * dyz - ly * dz;
        const uint32_t j = (x0 + lx) * g2 + (y0 + ly) * g + (z0 + lz);
        swo[j] = swl[v];
        nbo[j] = bl[v];
    }
}

// ---------------------------------------------------------------- host side
// The box grid of a g^3 lattice for `cus` workgroups: the most boxes (at most one per
// CU, a box of at most BK_NPT * 1024 nodes) with the smallest largest box, whose LDS
// (17 bytes per node and per halo node) fits; false if none does.
bool block_plan(uint32_t g, int cus, BlockPlan& p) {
    bool found = false;
    uint64_t best_v = ~0ull;
    for (uint32_t nx = 1; nx <= g && nx <= (uint32_t)cus; ++nx)
        for (uint32_t ny = 1; ny <= g && nx * ny <= (uint32_t)cus; ++ny)
            for (uint32_t nz = 1; nz <= g && nx * ny * nz <= (uint32_t)cus; ++nz) {
                const uint64_t bx = (g + nx - 1) / nx, by = (g + ny - 1) / ny, bz = (g + nz - 1) / nz;
                const uint64_t v = bx * by * bz;
                const uint64_t f = std::max(by * bz, std::max(bx * bz, bx * by));
                const uint64_t ns = v + 6 * f + 1;
                const uint64_t lds = 16 * ns + ((ns + 3) & ~3ull) + ((v + 3) & ~3ull) + 4 * v + 64;
                if (v > (uint64_t)BK_NPT * BK_THREADS || lds > 150 * 1024 || bx > 1023 || by > 1023 || bz > 1023)
                    continue;
                // estimated round time: node slots per thread (ceil(v / 1024)) plus a grid barrier
                // (~3 slots) when there are several boxes; then the fewest boxes (less face traffic)
                const uint64_t nbk = (uint64_t)nx * ny * nz;
                const uint64_t key = (((v + BK_THREADS - 1) / BK_THREADS + (nbk > 1 ? 3 : 0)) << 32) | nbk;
                if (!found || key < best_v) {
                    found = true;
                    best_v = key;
                    p.nbx = nx;
                    p.nby = ny;
                    p.nbz = nz;
                    p.vmax = (uint32_t)v;
                    p.fmax = (uint32_t)f;
                    p.lds = (uint32_t)lds;
                }
            }
    return found;
}

size_t block_face_bytes(const BlockPlan& p) {
    const size_t nb = (size_t)p.nbx * p.nby * p.nbz;
    return 2 * nb * 6 * p.fmax * (16 + 4);
}

hipError_t launch_round_block(const DevState& S, const BlockPlan& p, uint32_t r0, uint32_t nrounds, void* face,
                              void* scratch, hipStream_t st) {
    BlockArgs a{};
    const int cur = r0 & 1;
    a.sw_in = S.sw[cur];
    a.sw_out = S.sw[cur ^ 1];
    a.sw_alt = S.sw[cur];
    a.nb_in = S.nb[cur];
    a.nb_out = S.nb[cur ^ 1];
    a.nb_alt = S.nb[cur];
    a.ck_sw = S.sw[cur];
    a.ck_nb = S.nb[cur];
    const size_t nb = (size_t)p.nbx * p.nby * p.nbz;
    a.fs = static_cast<double2*>(face);
    a.fb = reinterpret_cast<uint32_t*>(a.fs + 2 * nb * 6 * p.fmax);
    // scratch (words): [0] barrier (groups arrived), [1] error flag, [16 (1 + grp)] the arrivals
    // of block group grp (a 64-byte line each), [144, 144 + 12 EPOCH) 3 x EPOCH x 2 accumulators,
    // then a 64-byte line of step flags per box
    a.bar = static_cast<unsigned int*>(scratch);
    a.err = a.bar + 1;
    a.acc = reinterpret_cast<unsigned long long*>(a.bar + 144);

    a.ctl = S.ctl;
    a.G = S.G;
    a.k0 = S.k0;
    a.k1 = S.k1;
    a.r0 = r0;
    a.nrounds = nrounds;
    a.nbx = p.nbx;
    a.nby = p.nby;
    a.nbz = p.nbz;
    a.fmax = p.fmax;
    a.vmax = p.vmax;
    hipError_t e = hipMemsetAsync(scratch, 0, BLOCK_SCRATCH_BYTES, st);
    if (e == hipSuccess) e = hipMemsetAsync(face, 0, block_face_bytes(p), st);  // (no face word carries a step)
    if (e != hipSuccess) return e;
    void* args[] = {&a};
    return hipLaunchCooperativeKernel(reinterpret_cast<const void*>(&k_ps_block), dim3((uint32_t)nb),
                                      dim3(BK_THREADS), args, p.lds, st);
}

hipError_t block_kernel_setup(const BlockPlan& p) {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ps_block), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)p.lds);
}

// Whether the plan's boxes can all be resident at once on `cus` CUs (the cooperative launch's
// condition), from the runtime's occupancy for this LDS size; false also if the query fails.
bool block_plan_resident(const BlockPlan& p, int cus) {
    if (block_kernel_setup(p) != hipSuccess) return false;
    int per = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, reinterpret_cast<const void*>(&k_ps_block), BK_THREADS,
                                                     p.lds) != hipSuccess)
        return false;
    return (uint64_t)p.nbx * p.nby * p.nbz <= (uint64_t)per * (uint64_t)cus;
}

}  // namespace gp
