// gp_kernels.hip -- CDNA4 (gfx950) kernels of the synchronous gossip /
// push-sum round (SRS v1).
//
// Design:
//   * the per-round bulk kernels for line / 3D / Imp3D live in gp_round.hip;
//     this file holds setup kernels, the full-topology round and the finalize
//     kernel;
//   * state is double-buffered (round r reads buffer r&1, writes r&1^1), so the
//     bulk kernels need no inter-workgroup synchronisation;
//   * a single-workgroup finalize kernel closes the round: alert bookkeeping
//     (scheduler, Program.fs:41-61), done flag, and the gossip injector
//     (Actor2, Program.fs:141-163) for the next round.
// Built with -ffp-contract=off: the push-sum fold must round exactly like the
// CPU oracle.
#include "gp_internal.hpp"
#include "gp_fullbin.hpp"

namespace gp {

// ---------------------------------------------------------------- helpers
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Sum over a 256-thread block; result valid in thread 0.
__device__ __forceinline__ void block_sum2(uint32_t& a, uint32_t& b, uint32_t (*lds)[BULK_THREADS / 64]) {
    a = wave_sum(a);
    b = wave_sum(b);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) {
        lds[0][wid] = a;
        lds[1][wid] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        a = 0;
        b = 0;
#pragma unroll
        for (int i = 0; i < BULK_THREADS / 64; ++i) {
            a += lds[0][i];
            b += lds[1][i];
        }
    }
}

template <typename T>
__device__ __forceinline__ T ld_agent(const T* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ void st_agent(T* p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int TOPO>
__device__ __forceinline__ uint32_t degree_of(uint32_t mask) {
    return popc6(mask) + (TOPO == IMP3D ? 1u : 0u);
}

// Direction node j sends in during `round` (slot U(deg) of its neighbour array,
// Program.fs:86 / 103 / 128).
template <int TOPO>
__device__ __forceinline__ uint32_t draw_dir(const DevState& S, uint32_t stream, uint32_t j, uint32_t mask,
                                             uint32_t round) {
    const uint32_t deg = degree_of<TOPO>(mask);
    if (deg == 0) return DIR_NONE;
    return slot_to_dir(mask, uniform(S.k0, S.k1, stream, j, round, deg));
}

// ---------------------------------------------------------------- init
// InitialSum x / weight 1.0 / count 1 / rumours 0 (Program.fs:67-71,78,174);
// only the seed (Program.fs:193) is active in round 0.
// Slab-aware: the rank's nodes [lo, lo + nloc); node arrays at id - base.
template <int TOPO, int ALG>
__global__ __launch_bounds__(BULK_THREADS) void k_init(DevState S) {
    for (uint32_t lj = blockIdx.x * BULK_THREADS + threadIdx.x; lj < S.nloc; lj += gridDim.x * BULK_THREADS) {
        const uint32_t j = S.lo + lj;
        const uint32_t jb = j - S.base;
        const bool seed = j == S.seed_node;
        uint32_t dir = DIR_NONE;
        if (TOPO != FULL && seed) {
            const uint32_t mask = present_mask<TOPO>(j, S.G);
            dir = draw_dir<TOPO>(S, ALG == GOSSIP ? S_GOSSIP : S_PUSHSUM, j, mask, 0);
        }
        if (ALG == PUSHSUM) {
            S.sw[0][jb] = make_double2((double)j, 1.0);
            S.nb[0][jb] = (uint8_t)((1u << CNT_SHIFT) | (seed ? B_ACTIVE : 0u) | dir);
        } else {
            S.c[lj] = 0;
            if (TOPO != FULL) S.nb[0][jb] = (uint8_t)dir;
            else S.inc[lj] = 0;
        }
    }
}

__global__ __launch_bounds__(BULK_THREADS) void k_iota(uint32_t* v, uint32_t n) {
    for (uint32_t i = blockIdx.x * BULK_THREADS + threadIdx.x; i < n; i += gridDim.x * BULK_THREADS) v[i] = i;
}

__global__ __launch_bounds__(BULK_THREADS) void k_histogram(const uint32_t* keys, uint32_t n, uint32_t* counts) {
    for (uint32_t i = blockIdx.x * BULK_THREADS + threadIdx.x; i < n; i += gridDim.x * BULK_THREADS)
        atomicAdd(&counts[keys[i]], 1u);
}

// Injector list = ids 0..T-1 (Program.fs:147-148) as a bitmap + per-chunk counts.
__global__ __launch_bounds__(BULK_THREADS) void k_injector_init(DevState S) {
    const uint32_t T = S.G.T;
    const uint32_t nwords = S.nchunks * (INJ_CHUNK / 32);
    for (uint32_t w = blockIdx.x * BULK_THREADS + threadIdx.x; w < nwords; w += gridDim.x * BULK_THREADS) {
        const uint64_t lo = (uint64_t)w * 32;
        uint32_t bits = 0;
        if (lo + 32 <= T) bits = 0xFFFFFFFFu;
        else if (lo < T) bits = (1u << (uint32_t)(T - lo)) - 1u;
        S.live_bits[w] = bits;
    }
    for (uint32_t c = blockIdx.x * BULK_THREADS + threadIdx.x; c < S.nchunks; c += gridDim.x * BULK_THREADS) {
        const uint64_t lo = (uint64_t)c * INJ_CHUNK;
        const uint64_t hi = lo + INJ_CHUNK < T ? lo + INJ_CHUNK : T;
        S.chunk_live[c] = (uint32_t)(hi - lo);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) S.ctl->live = T;
}

// ---------------------------------------------------------------- full topology
// Gossip: every active node sends to a uniform j != i (Program.fs:211-216,86-88).
__global__ __launch_bounds__(BULK_THREADS) void k_full_gossip_send(DevState S, uint32_t r) {
    if (ld_agent(&S.ctl->done)) return;
    const uint32_t P = S.G.P;
    for (uint32_t i = blockIdx.x * BULK_THREADS + threadIdx.x; i < P; i += gridDim.x * BULK_THREADS) {
        const int32_t ci = S.c[i];
        if (((i == S.seed_node) || ci >= 1) && ci <= 10) {
            const uint32_t t = full_target(i, uniform(S.k0, S.k1, S_GOSSIP, i, r, P - 1));
            atomicAdd(&S.inc[t], 1);  // integer: order-independent, bit-exact
        }
    }
}

__global__ __launch_bounds__(BULK_THREADS) void k_full_gossip_recv(DevState S, uint32_t r) {
    __shared__ uint32_t red[2][BULK_THREADS / 64];
    (void)r;
    Ctl* ctl = S.ctl;
    if (ld_agent(&ctl->done)) return;
    const uint32_t P = S.G.P;
    uint32_t alerts = 0, unused = 0;
    for (uint32_t j = blockIdx.x * BULK_THREADS + threadIdx.x; j < P; j += gridDim.x * BULK_THREADS) {
        const int32_t d = S.inc[j];
        if (!d) continue;
        S.inc[j] = 0;
        const int32_t c0 = S.c[j];
        if (c0 < (int32_t)GOSSIP_DONE) {
            S.c[j] = c0 + d;
            alerts += c0 + d > 10;
        }
    }
    block_sum2(alerts, unused, red);
    if (threadIdx.x == 0 && alerts) atomicAdd(&ctl->round_alerts, (unsigned long long)alerts);
}

// ---------------------------------------------------------------- finalize
// Block-wide inclusive scan over FIN_THREADS values (one per thread).
__device__ uint32_t block_incl_scan(uint32_t v, uint32_t* lds) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    if (lane == 63) lds[wid] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (int i = 0; i < FIN_THREADS / 64; ++i) {
            const uint32_t t = lds[i];
            lds[i] = run;
            run += t;
        }
    }
    __syncthreads();
    v += lds[wid];
    __syncthreads();
    return v;
}

// The injector's list L (Program.fs:147-148) is a bitmap over ids 0..T-1 plus
// per-chunk live counts, replicated on every rank.  inj_find: the id of the
// k-th live element (block-wide two-level search), or -1.
__device__ long long inj_find(const DevState& S, uint32_t k) {
    __shared__ uint32_t lds[FIN_THREADS / 64];
    __shared__ uint32_t sh_chunk, sh_k;
    __shared__ long long sh_id;
    if (threadIdx.x == 0) {
        sh_chunk = 0xFFFFFFFFu;
        sh_id = -1;
    }
    __syncthreads();
    // phase A: which chunk holds the k-th live id
    const uint32_t nch = S.nchunks;
    const uint32_t per = (nch + FIN_THREADS - 1) / FIN_THREADS;
    const uint32_t c_lo = threadIdx.x * per;
    const uint32_t c_hi = c_lo + per < nch ? c_lo + per : nch;
    uint32_t local = 0;
    for (uint32_t c = c_lo; c < c_hi; ++c) local += S.chunk_live[c];
    const uint32_t incl = block_incl_scan(local, lds);
    const uint32_t excl = incl - local;
    if (k >= excl && k < incl) {
        uint32_t run = excl;
        for (uint32_t c = c_lo; c < c_hi; ++c) {
            const uint32_t n = S.chunk_live[c];
            if (k < run + n) {
                sh_chunk = c;
                sh_k = k - run;
                break;
            }
            run += n;
        }
    }
    __syncthreads();
    if (sh_chunk >= nch) return -1;  // unreachable when chunk_live sums to live
    // phase B: which bit of the chunk's 2048 words
    const uint32_t chunk = sh_chunk, kk = sh_k;
    constexpr uint32_t WPT = (INJ_CHUNK / 32) / FIN_THREADS;  // words per thread (2)
    const uint32_t* words = S.live_bits + (size_t)chunk * (INJ_CHUNK / 32);
    uint32_t wv[WPT];
    uint32_t wl = 0;
#pragma unroll
    for (uint32_t q = 0; q < WPT; ++q) {
        wv[q] = words[threadIdx.x * WPT + q];
        wl += (uint32_t)__popc(wv[q]);
    }
    const uint32_t wincl = block_incl_scan(wl, lds);
    const uint32_t wexcl = wincl - wl;
    if (kk >= wexcl && kk < wincl) {
        uint32_t rem = kk - wexcl;
#pragma unroll
        for (uint32_t q = 0; q < WPT; ++q) {
            const uint32_t pc = (uint32_t)__popc(wv[q]);
            if (rem < pc) {
                uint32_t m = wv[q];
                for (uint32_t z = 0; z < rem; ++z) m &= m - 1;  // drop `rem` lowest set bits
                const uint32_t bit = (uint32_t)__ffs(m) - 1;
                sh_id = (long long)chunk * INJ_CHUNK + (threadIdx.x * WPT + q) * 32 + bit;
                break;
            }
            rem -= pc;
        }
    }
    __syncthreads();
    return sh_id;
}

// Remove id from L (Program.fs:158); one thread.
__device__ void inj_remove(const DevState& S, long long id, uint32_t live) {
    const uint32_t chunk = (uint32_t)(id / INJ_CHUNK);
    const uint32_t word = (uint32_t)((id % INJ_CHUNK) / 32), bit = (uint32_t)(id % 32);
    uint32_t* w = S.live_bits + (size_t)chunk * (INJ_CHUNK / 32) + word;
    *w = *w & ~(1u << bit);
    S.chunk_live[chunk] -= 1;
    st_agent(&S.ctl->live, (unsigned long long)(live - 1));
}

// Scheduler bookkeeping of round `round_done` from this round's global counts
// (Program.fs:51-56); returns 1 when the run is over.  One thread.
__device__ int close_round(const DevState& S, uint32_t round_done, unsigned long long a, unsigned long long na) {
    return close_round_ctl(S.ctl, S.G.P, S.G.T, round_done, a, na);
}

// Single rank: closes round `round_done` (if has_done) and prepares round
// `round_next`: scheduler bookkeeping and, for gossip on line / 3D / Imp3D, one
// injector step (Program.fs:150-159): k = U(|L|), t = k-th live id; if t
// converged remove it, else deliver one rumour to t in round_next.
__global__ __launch_bounds__(FIN_THREADS) void k_finalize(DevState S, uint32_t round_done, uint32_t round_next,
                                                          int has_done, int injector) {
    __shared__ int sh_skip;
    Ctl* ctl = S.ctl;
    if (threadIdx.x == 0) {
        int skip = (int)ld_agent(&ctl->done);
        if (!skip && has_done)
            skip = close_round(S, round_done, atomicExch(&ctl->round_alerts, 0ull),
                               atomicExch(&ctl->round_active, 0ull));
        sh_skip = skip;
    }
    __syncthreads();
    if (sh_skip || !injector) return;
    const uint32_t live = (uint32_t)ld_agent(&ctl->live);
    long long target = -1;
    if (live) {
        const long long id = inj_find(S, uniform(S.k0, S.k1, S_INJECT, 0, round_next, live));
        if (threadIdx.x == 0 && id >= 0) {
            if (S.c[id - S.lo] >= (int32_t)GOSSIP_DONE) inj_remove(S, id, live);  // converged: remove
            else target = id;                                                    // Process2 to the pick
        }
    }
    if (threadIdx.x == 0) st_agent(&ctl->inj_target, target);
}

// Multi-rank, part 1: this rank's counts of round `round_done` go to xchg[0..1];
// the injector pick for round_next (identical on every rank: L is replicated)
// goes to inj_pick and xchg[2] = 1 iff this rank owns it and it has converged.
// xchg is then summed over ranks (RCCL all-reduce) before part 2.
__global__ __launch_bounds__(FIN_THREADS) void k_finalize_pre(DevState S, uint32_t round_next, int injector) {
    Ctl* ctl = S.ctl;
    const int skip = (int)ld_agent(&ctl->done);
    if (threadIdx.x == 0) {
        ctl->xchg[0] = skip ? 0ull : atomicExch(&ctl->round_alerts, 0ull);
        ctl->xchg[1] = skip ? 0ull : atomicExch(&ctl->round_active, 0ull);
        ctl->xchg[2] = 0ull;
        // an exchange buffer of this rank overflowed (send or receive side): summed
        // over ranks, so every rank fails the batch (gp_step), not only the sender
        ctl->xchg[3] = (ld_agent(&ctl->overflow) ? 1ull : 0ull) + (ld_agent(&ctl->tiny) ? 65536ull : 0ull);
        ctl->inj_pick = -1;
    }
    if (skip || !injector) return;
    const uint32_t live = (uint32_t)ld_agent(&ctl->live);
    if (!live) return;
    const long long id = inj_find(S, uniform(S.k0, S.k1, S_INJECT, 0, round_next, live));
    if (threadIdx.x == 0 && id >= 0) {
        ctl->inj_pick = id;
        if ((uint64_t)(id - S.lo) < S.nloc && S.c[id - S.lo] >= (int32_t)GOSSIP_DONE) ctl->xchg[2] = 1ull;
    }
}

// Multi-rank, part 2: global bookkeeping from the summed xchg, then apply the
// injector pick (remove from the replicated L if converged, else deliver).
__global__ void k_finalize_post(DevState S, uint32_t round_done, int has_done, int injector) {
    Ctl* ctl = S.ctl;
    if (threadIdx.x != 0) return;
    if (ctl->xchg[3] & 0xFFFFull) ctl->overflow = 1u;  // some rank's exchange overflowed: this run is invalid
    if (ctl->xchg[3] >> 16) ctl->tiny = 1u;            // some rank saw a value below the FMA fold's bound
    if (ld_agent(&ctl->done)) return;
    if (has_done && close_round(S, round_done, ctl->xchg[0], ctl->xchg[1])) return;
    long long target = -1;
    const long long id = ctl->inj_pick;
    if (injector && id >= 0) {
        if (ctl->xchg[2]) inj_remove(S, id, (uint32_t)ld_agent(&ctl->live));
        else target = id;
    }
    st_agent(&ctl->inj_target, target);
}

// ---------------------------------------------------------------- launchers
hipError_t launch_init(const DevState& S, int grid, hipStream_t st) {
#define GP_INIT(T, A) hipLaunchKernelGGL((k_init<T, A>), dim3(grid), dim3(BULK_THREADS), 0, st, S)
    if (S.alg == PUSHSUM) {
        switch (S.topo) {
            case LINE: GP_INIT(LINE, PUSHSUM); break;
            case FULL: GP_INIT(FULL, PUSHSUM); break;
            case GRID3D: GP_INIT(GRID3D, PUSHSUM); break;
            default: GP_INIT(IMP3D, PUSHSUM); break;
        }
    } else {
        switch (S.topo) {
            case LINE: GP_INIT(LINE, GOSSIP); break;
            case FULL: GP_INIT(FULL, GOSSIP); break;
            case GRID3D: GP_INIT(GRID3D, GOSSIP); break;
            default: GP_INIT(IMP3D, GOSSIP); break;
        }
    }
#undef GP_INIT
    return hipGetLastError();
}

hipError_t launch_injector_init(const DevState& S, int grid, hipStream_t st) {
    hipLaunchKernelGGL(k_injector_init, dim3(grid), dim3(BULK_THREADS), 0, st, S);
    return hipGetLastError();
}

hipError_t launch_iota(uint32_t* v, uint32_t n, int grid, hipStream_t st) {
    hipLaunchKernelGGL(k_iota, dim3(grid), dim3(BULK_THREADS), 0, st, v, n);
    return hipGetLastError();
}

hipError_t launch_histogram(const uint32_t* keys, uint32_t n, uint32_t* counts, int grid, hipStream_t st) {
    hipLaunchKernelGGL(k_histogram, dim3(grid), dim3(BULK_THREADS), 0, st, keys, n, counts);
    return hipGetLastError();
}

hipError_t launch_bulk(const DevState& S, uint32_t round, int grid, hipStream_t st) {
    const dim3 g(grid), b(BULK_THREADS);
    if (S.topo != FULL) {
        if (S.kernel == KERNEL_TILE)
            return S.tile_wide ? wide::launch_round_tile(S, round, grid, st) : launch_round_tile(S, round, grid, st);
        if (S.kernel == KERNEL_COL) return launch_round_col(make_wave_args(S, round), S.topo, S.alg, round, grid, st);
        return hipErrorInvalidValue;
    }
    if (S.alg == PUSHSUM) {
        return launch_full_pushsum_round(S, round, grid, st);
    } else {
        hipLaunchKernelGGL(k_full_gossip_send, g, b, 0, st, S, round);
        hipLaunchKernelGGL(k_full_gossip_recv, g, b, 0, st, S, round);
    }
    return hipGetLastError();
}

const char* bulk_kernel_name(const DevState& S) {
    static const char* ps[2][4] = {{"k_ps_tile<LINE>", "k_fb_send+split+fold", "k_ps_tile<GRID3D>", "k_ps_tile<IMP3D>"},
                                   {"k_ps_tile<LINE>", "k_fb_send+split+fold", "k_ps_col<GRID3D>", "k_ps_col<IMP3D>"}};
    static const char* go[2][4] = {{"k_gossip_tile<LINE>", "k_full_gossip_send+recv", "k_gossip_tile<GRID3D>",
                                    "k_gossip_tile<IMP3D>"},
                                   {"k_gossip_tile<LINE>", "k_full_gossip_send+recv", "k_gossip_col<GRID3D>",
                                    "k_gossip_col<IMP3D>"}};
    if (S.topo == FULL && S.alg == PUSHSUM && S.fb_fused) return "k_fb_split+fold<send>";  // one rank, fused
    if (S.kernel == KERNEL_BLOCK) return "k_ps_block<GRID3D>";  // LDS-resident, one launch per batch
    const int v = S.kernel == KERNEL_COL ? 1 : 0;
    if (v == 0 && S.tile_wide && S.topo != FULL) {  // the 1024-thread size class (gp_round_wide.hip)
        static const char* w[2][4] = {{"wide::k_gossip_tile<LINE>", "", "wide::k_gossip_tile<GRID3D>",
                                       "wide::k_gossip_tile<IMP3D>"},
                                      {"wide::k_ps_tile<LINE>", "", "wide::k_ps_tile<GRID3D>", "wide::k_ps_tile<IMP3D>"}};
        return w[S.alg == PUSHSUM ? 1 : 0][S.topo];
    }
    return S.alg == PUSHSUM ? ps[v][S.topo] : go[v][S.topo];
}

// Experiments build, GP_CHECK_CLOSE=1 (tests): the alert bookkeeping recounted
// from the node state after a batch, to cross-check the round closes (the fused
// close orders its shard counts by returning relaxed atomics at the device
// coherence point, gp_internal.hpp).  Every node alerts once: push-sum when it
// converges (Program.fs:118-121), gossip on the receipt that takes it past 10
// rumours (Program.fs:92-94).
__global__ __launch_bounds__(256) void k_count_alerted(const uint8_t* nb, const int32_t* c, uint32_t n,
                                                       unsigned long long* out) {
    uint32_t k = 0;
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256)
        k += c ? (c[i] > 10 ? 1u : 0u) : ((nb[i] & B_CONV) ? 1u : 0u);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) k += __shfl_xor(k, o, 64);
    if ((threadIdx.x & 63) == 0 && k) atomicAdd(out, (unsigned long long)k);
}

hipError_t launch_count_alerted(const uint8_t* nb, const int32_t* c, uint32_t n, unsigned long long* out, int grid,
                                hipStream_t st) {
    hipLaunchKernelGGL(k_count_alerted, dim3(grid), dim3(256), 0, st, nb, c, n, out);
    return hipGetLastError();
}

hipError_t launch_finalize_pre(const DevState& S, uint32_t round_next, hipStream_t st) {
    const int injector = (S.alg == GOSSIP && S.topo != FULL) ? 1 : 0;
    hipLaunchKernelGGL(k_finalize_pre, dim3(1), dim3(FIN_THREADS), 0, st, S, round_next, injector);
    return hipGetLastError();
}

hipError_t launch_finalize_post(const DevState& S, uint32_t round_done, uint32_t round_next, hipStream_t st) {
    const int has_done = round_next > 0;
    const int injector = (S.alg == GOSSIP && S.topo != FULL) ? 1 : 0;
    hipLaunchKernelGGL(k_finalize_post, dim3(1), dim3(64), 0, st, S, round_done, has_done, injector);
    return hipGetLastError();
}

hipError_t launch_finalize(const DevState& S, uint32_t round_done, uint32_t round_next, hipStream_t st) {
    const int has_done = round_next > 0;
    const int injector = (S.alg == GOSSIP && S.topo != FULL) ? 1 : 0;
    hipLaunchKernelGGL(k_finalize, dim3(1), dim3(FIN_THREADS), 0, st, S, round_done, round_next, has_done,
                       injector);
    return hipGetLastError();
}

}  // namespace gp

namespace gp {
// Full-topology push-sum round on one rank (gp_fullbin.hip).
hipError_t launch_full_pushsum_round(const DevState& S, uint32_t round, int grid, hipStream_t st) {
    FullBinArgs a{};
    const int cur = round & 1;
    a.swc = S.sw[cur];
    a.swn = S.sw[cur ^ 1];
    a.nb = S.nb[0];
    a.ctl = S.ctl;
    a.overflow = &S.ctl->overflow;
    a.P = S.G.P;
    a.k0 = S.k0;
    a.k1 = S.k1;
    a.s1 = S.fb_s1;
    a.nb1 = S.fb_nb1;
    a.nb2 = S.fb_nb2;
    a.cap1 = S.fb_cap1;
    a.cap2 = S.fb_cap2;
    a.cnt1 = S.fb_cnt1;
    a.cnt2 = S.fb_cnt2;
    a.hdr1 = S.fb_hdr1;
    a.pay1 = S.fb_pay1;
    a.hdr2 = S.fb_hdr2;
    a.pay2 = S.fb_pay2;
    a.lo = S.lo;      // one rank: 0
    a.nloc = S.nloc;  // one rank: P
    a.t_lo = 0;
    a.t_hi = S.fb_nb2;
    a.W = 1;
    a.fused = S.fb_fused;
    return launch_full_bin_round(a, round, grid, st);
}
}  // namespace gp
