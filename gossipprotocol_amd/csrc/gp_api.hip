// gp_api.hip -- C-ABI of libgossip_hip.so (include/gossip_hip.h) and the host
// orchestrator of the synchronous round loop.
//
// Replaces, in /root/reference/Project2/Program.fs:
//   * actor population + topology build (Program.fs:169-176,180-191,209-216,238-261)
//     -> gp_create: SoA device state, implicit neighbours, Imp3D in-lists;
//   * message loop + scheduler (Program.fs:41-61,84-131,141-163) -> gp_step / gp_run:
//     per round one bulk kernel + one finalize kernel, queued in batches with one
//     host synchronisation per batch (never per round).
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/gossip_hip.h"
#include "gp_internal.hpp"

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

constexpr int64_t BATCH = 1024;  // rounds queued per host synchronisation (<= HIST)
static_assert(BATCH <= HIST, "alert ring must cover a batch");

}  // namespace

struct gp_sim {
    gp_config cfg{};
    DevState S{};
    int device = 0;
    hipStream_t stream = nullptr;
    int grid = 1;
    int64_t P = 0, T = 0, g = 0;
    int64_t rounds_done = 0;
    int64_t alerts_total = 0;
    bool done = false;
    Ctl* host_ctl = nullptr;  // pinned mirror of the device control block
    std::vector<void*> allocs;
    // kernel timing
    bool timing = false;
    std::vector<hipEvent_t> ev;
    double kernel_ms = 0.0;
    int64_t launches = 0;
};

namespace {

int dev_alloc(gp_sim* s, void** p, size_t bytes) {
    if (bytes == 0) bytes = 4;
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

void free_all(gp_sim* s) {
    for (void* p : s->allocs) (void)hipFree(p);
    s->allocs.clear();
}

uint32_t bits_for(uint64_t maxval) {
    uint32_t b = 1;
    while (b < 32 && (maxval >> b) != 0) ++b;
    return b;
}

// Imp3D: draw rnd[] (Program.fs:258-260), then build the receiver-sorted
// in-lists: a stable sort of (rnd[i], i) by rnd keeps every receiver's
// senders in ascending id order; in_off = exclusive scan of the in-degrees.
int build_imp3d(gp_sim* s) {
    DevState& S = s->S;
    const uint32_t P = S.G.P;
    int rc;
    if ((rc = dev_alloc_t(s, &S.rnd, P)) || (rc = dev_alloc_t(s, &S.in_off, (size_t)P + 1)) ||
        (rc = dev_alloc_t(s, &S.in_src, P)))
        return rc;
    uint32_t *iota = nullptr, *keys_sorted = nullptr, *counts = nullptr;
    HIP_TRY(hipMalloc(&iota, sizeof(uint32_t) * P));
    HIP_TRY(hipMalloc(&keys_sorted, sizeof(uint32_t) * P));
    HIP_TRY(hipMalloc(&counts, sizeof(uint32_t) * ((size_t)P + 1)));
    HIP_TRY(launch_topo_rnd(S, s->grid, s->stream));
    HIP_TRY(launch_iota(iota, P, s->grid, s->stream));
    const uint32_t bits = bits_for(P > 1 ? P - 2 : 0);
    size_t tmp_bytes = 0;
    HIP_TRY(sort_pairs(nullptr, tmp_bytes, S.rnd, keys_sorted, iota, S.in_src, P, bits, s->stream));
    void* tmp = nullptr;
    HIP_TRY(hipMalloc(&tmp, tmp_bytes ? tmp_bytes : 4));
    HIP_TRY(sort_pairs(tmp, tmp_bytes, S.rnd, keys_sorted, iota, S.in_src, P, bits, s->stream));
    HIP_TRY(hipMemsetAsync(counts, 0, sizeof(uint32_t) * ((size_t)P + 1), s->stream));
    HIP_TRY(launch_histogram(S.rnd, P, counts, s->grid, s->stream));
    size_t scan_bytes = 0;
    HIP_TRY(exclusive_scan_u32(nullptr, scan_bytes, counts, S.in_off, P + 1, s->stream));
    void* scan_tmp = nullptr;
    HIP_TRY(hipMalloc(&scan_tmp, scan_bytes ? scan_bytes : 4));
    HIP_TRY(exclusive_scan_u32(scan_tmp, scan_bytes, counts, S.in_off, P + 1, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    HIP_TRY(hipFree(scan_tmp));
    HIP_TRY(hipFree(tmp));
    HIP_TRY(hipFree(counts));
    HIP_TRY(hipFree(keys_sorted));
    HIP_TRY(hipFree(iota));
    return GP_OK;
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

// One synchronous round r (bulk kernel[s]) followed by the finalize kernel.
int launch_round(gp_sim* s, uint32_t r, hipEvent_t e0, hipEvent_t e1) {
    DevState& S = s->S;
    if (e0) HIP_TRY(hipEventRecord(e0, s->stream));
    if (S.topo == FULL && S.alg == PUSHSUM) {
        HIP_TRY(launch_full_pushsum_send(S, r, s->grid, s->stream));
        HIP_TRY(sort_pairs(S.sort_tmp, S.sort_tmp_bytes, S.key[0], S.key[1], S.val[0], S.val[1], S.G.P, S.key_bits,
                           s->stream));
        HIP_TRY(hipMemsetAsync(S.head, 0xFF, sizeof(uint32_t) * S.G.P, s->stream));
        HIP_TRY(launch_full_pushsum_mark(S, s->grid, s->stream));
    }
    HIP_TRY(launch_bulk(S, r, s->grid, s->stream));
    if (e1) HIP_TRY(hipEventRecord(e1, s->stream));
    HIP_TRY(launch_finalize(S, r, r + 1, s->stream));
    return GP_OK;
}

double alg_bytes(const gp_sim* s) {
    const DevState& S = s->S;
    if (S.alg == PUSHSUM) {
        // sw r+w 32, node byte r+w 2 (+ Imp3D in-list: offset 4 + sender 4)
        if (S.topo == IMP3D) return 42.0;
        if (S.topo != FULL) return 34.0;
        // send: byte 1 + key 4; sort: (key+val) r+w per pass; mark: key 4 + head 4;
        // recv: sw r+w 32 + byte 1 + head 4 + key/val 8 + gathered sw 16
        const double passes = (S.key_bits + 7) / 8;
        return 5.0 + 16.0 * passes + 8.0 + 4.0 + 61.0;
    }
    // gossip: counter r+w 8, direction byte r+w 2 (+ Imp3D in-list 8)
    if (S.topo == IMP3D) return 18.0;
    if (S.topo != FULL) return 10.0;
    return 4.0 + 8.0 + 8.0 + 8.0;  // send: c + atomic RMW; recv: inc r+w, c r+w
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
    if (*P > 0xFFFFFF00ll) {
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
    *out = nullptr;
    if (cfg->algorithm != GP_GOSSIP && cfg->algorithm != GP_PUSHSUM) {
        set_err("option invalid: algorithm id %d", cfg->algorithm);
        return GP_EINVAL;
    }
    if (cfg->num_gpus > 1) {
        set_err("num_gpus > 1: run one process per GPU and use gp_create_rank");
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
    s->timing = (cfg->flags & GP_FLAG_KERNEL_TIMING) != 0;
    auto fail = [&](int code) {
        gp_destroy(s);
        return code;
    };
    if (hipSetDevice(s->device) != hipSuccess || hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess) {
        set_err("hipSetDevice/hipStreamCreate failed on device %d", s->device);
        return fail(GP_EHIP);
    }
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, s->device);
    const int64_t blocks = (P + BULK_THREADS - 1) / BULK_THREADS;
    // 64 workgroups per CU: measured best for the tiled round kernels (tools/ablate.py:
    // 2048 -> 27.5, 8192 -> 22.1, 16384 -> 21.2 ms/round at P = 1e9)
    int64_t cap = (int64_t)prop.multiProcessorCount * 64;
    // round-kernel variant: column march for lattices with enough patches to fill
    // the chip, the chunk kernel otherwise (line, small g); GP_KERNEL overrides
    // (measured, profiles/r01: push-sum -> tiled; gossip on a large lattice -> column march)
    int kernel = KERNEL_TILE;
    const bool lattice = cfg->topology == GP_3D || cfg->topology == GP_IMP3D;
    if (lattice && cfg->algorithm == GP_GOSSIP && g >= 200) kernel = KERNEL_COL;
    if (const char* e = std::getenv("GP_KERNEL")) {
        if (!std::strcmp(e, "tile")) kernel = KERNEL_TILE;
        else if (!std::strcmp(e, "wave")) kernel = KERNEL_WAVE;
        else if (!std::strcmp(e, "col") && lattice) kernel = KERNEL_COL;
    }
    uint32_t col_xsegs = 1;
    if (cfg->topology != GP_FULL && kernel != KERNEL_TILE) {
        // exactly the resident grid (a persistent sweep), a multiple of the 8 XCDs
        const int bpc = kernel == KERNEL_COL ? col_blocks_per_cu(cfg->topology, cfg->algorithm)
                                             : wave_blocks_per_cu(cfg->topology, cfg->algorithm);
        cap = (int64_t)prop.multiProcessorCount * bpc;
        if (kernel == KERNEL_COL) {
            // x segments per patch: enough work items for every resident wave, >= 16 planes each
            const int64_t patches = ((g + 63) / 64) * ((g + 3) / 4);
            const int64_t waves = cap * (BULK_THREADS / 64);
            int64_t xs = std::max<int64_t>(1, waves / std::max<int64_t>(1, patches));
            xs = std::min<int64_t>(xs, std::max<int64_t>(1, g / 16));
            col_xsegs = (uint32_t)xs;
        }
    }
    if (const char* e = std::getenv("GP_GRID")) cap = std::max<int64_t>(1, std::atoll(e));
    if (const char* e = std::getenv("GP_XSEGS")) col_xsegs = (uint32_t)std::max(1, std::atoi(e));
    s->grid = (int)std::max<int64_t>(1, std::min(kernel == KERNEL_COL ? cap : blocks, cap));

    DevState& S = s->S;
    S.topo = cfg->topology;
    S.alg = cfg->algorithm;
    S.G.P = (uint32_t)P;
    S.G.T = (uint32_t)T;
    S.G.g = (uint32_t)g;
    S.G.g2 = (uint32_t)(g * g);
    S.G.div_g = make_fastdiv(S.G.g ? S.G.g : 1);
    S.G.div_g2 = make_fastdiv(S.G.g2 ? S.G.g2 : 1);
    S.lo = 0;
    S.nloc = (uint32_t)P;
    S.base = 0;
    S.ext_lo = 0;
    S.ext_hi = (uint32_t)P;
    S.rtag = nullptr;
    S.rmsg = nullptr;
    S.kernel = kernel;
    S.col_xsegs = col_xsegs;
    S.tile_walk = 0;
    if (const char* e = std::getenv("GP_WALK")) S.tile_walk = (uint32_t)std::atoi(e);
    S.k0 = (uint32_t)cfg->seed;
    S.k1 = (uint32_t)(cfg->seed >> 32);
    // choice = Random().Next(0, nodes) (Program.fs:193,221,263)
    S.seed_node = uniform(S.k0, S.k1, S_START, 0, 0, (uint32_t)T);

    const size_t Pn = (size_t)P;
    if ((rc = dev_alloc_t(s, &S.ctl, 1))) return fail(rc);
    const size_t Pnb = Pn + 1024;  // node-byte arrays: tiles read/write whole words past P
    if (S.alg == PUSHSUM) {
        if ((rc = dev_alloc_t(s, &S.sw[0], Pn)) || (rc = dev_alloc_t(s, &S.sw[1], Pn)) ||
            (rc = dev_alloc_t(s, &S.nb[0], Pnb)))
            return fail(rc);
        if (S.topo != FULL && (rc = dev_alloc_t(s, &S.nb[1], Pnb))) return fail(rc);
    } else {
        if ((rc = dev_alloc_t(s, &S.c, Pn))) return fail(rc);
        if (S.topo == FULL) {
            if ((rc = dev_alloc_t(s, &S.inc, Pn))) return fail(rc);
        } else {
            if ((rc = dev_alloc_t(s, &S.nb[0], Pnb)) || (rc = dev_alloc_t(s, &S.nb[1], Pnb))) return fail(rc);
            S.nchunks = (uint32_t)((T + INJ_CHUNK - 1) / INJ_CHUNK);
            if ((rc = dev_alloc_t(s, &S.live_bits, (size_t)S.nchunks * (INJ_CHUNK / 32))) ||
                (rc = dev_alloc_t(s, &S.chunk_live, S.nchunks)))
                return fail(rc);
        }
    }
    if (S.topo == FULL && S.alg == PUSHSUM) {
        if ((rc = dev_alloc_t(s, &S.key[0], Pn)) || (rc = dev_alloc_t(s, &S.key[1], Pn)) ||
            (rc = dev_alloc_t(s, &S.val[0], Pn)) || (rc = dev_alloc_t(s, &S.val[1], Pn)) ||
            (rc = dev_alloc_t(s, &S.head, Pn)))
            return fail(rc);
        S.key_bits = bits_for((uint64_t)P);
        if (launch_iota(S.val[0], S.G.P, s->grid, s->stream) != hipSuccess) {
            set_err("iota launch failed");
            return fail(GP_EHIP);
        }
        size_t tb = 0;
        if (sort_pairs(nullptr, tb, S.key[0], S.key[1], S.val[0], S.val[1], S.G.P, S.key_bits, s->stream) !=
            hipSuccess) {
            set_err("rocprim sort sizing failed");
            return fail(GP_EHIP);
        }
        S.sort_tmp_bytes = tb;
        if ((rc = dev_alloc(s, &S.sort_tmp, tb))) return fail(rc);
    }
    if (S.topo == IMP3D) {
        S.rbits_words = S.kernel == KERNEL_COL ? col_rbits_words(S.nloc / S.G.g2, S.G.g) : rbits_words_for(S.lo, S.nloc);
        if ((rc = dev_alloc_t(s, &S.rbits[0], S.rbits_words)) || (rc = dev_alloc_t(s, &S.rbits[1], S.rbits_words)))
            return fail(rc);
        if ((rc = build_imp3d(s))) return fail(rc);
    }

    if (hipHostMalloc((void**)&s->host_ctl, sizeof(Ctl), hipHostMallocDefault) != hipSuccess) {
        set_err("hipHostMalloc failed");
        return fail(GP_ENOMEM);
    }
    std::memset(s->host_ctl, 0, sizeof(Ctl));
    s->host_ctl->active_total = 1;  // the seed
    s->host_ctl->all_active = P <= 1 ? 1u : 0u;
    s->host_ctl->inj_target = -1;
    if (hipMemcpyAsync(S.ctl, s->host_ctl, sizeof(Ctl), hipMemcpyHostToDevice, s->stream) != hipSuccess ||
        launch_init(S, s->grid, s->stream) != hipSuccess) {
        set_err("init launch failed");
        return fail(GP_EHIP);
    }
    if (S.topo == IMP3D && (S.kernel == KERNEL_COL ? launch_col_rbits_init(S, s->stream)
                                                   : launch_rbits_init(S, s->grid, s->stream)) != hipSuccess) {
        set_err("random-edge bitmap init failed");
        return fail(GP_EHIP);
    }
    if (S.alg == GOSSIP && S.topo != FULL && launch_injector_init(S, s->grid, s->stream) != hipSuccess) {
        set_err("injector init launch failed");
        return fail(GP_EHIP);
    }
    if (launch_finalize(S, 0, 0, s->stream) != hipSuccess) {  // prepare round 0
        set_err("finalize launch failed");
        return fail(GP_EHIP);
    }
    hipError_t e = hipStreamSynchronize(s->stream);
    if (e != hipSuccess) {
        set_err("initialisation failed: %s", hipGetErrorString(e));
        return fail(GP_EHIP);
    }
    if (s->timing) {
        s->ev.resize(2 * BATCH);
        for (auto& x : s->ev)
            if (hipEventCreate(&x) != hipSuccess) {
                set_err("hipEventCreate failed");
                return fail(GP_EHIP);
            }
    }
    *out = s;
    return GP_OK;
}

int gp_get_unique_id(uint8_t unique_id[128]) {
    (void)unique_id;
    set_err("multi-GPU ranks are not available in this build");
    return GP_ESTATE;
}

int gp_create_rank(const gp_config* cfg, int32_t rank, int32_t world, const uint8_t unique_id[128], gp_sim** out) {
    (void)unique_id;
    if (world == 1 && rank == 0) return gp_create(cfg, out);
    set_err("multi-GPU ranks are not available in this build");
    return GP_ESTATE;
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
        for (int64_t k = 0; k < batch; ++k) {
            const uint32_t r = (uint32_t)(s->rounds_done + k);
            hipEvent_t e0 = s->timing ? s->ev[2 * k] : nullptr;
            hipEvent_t e1 = s->timing ? s->ev[2 * k + 1] : nullptr;
            int rc = launch_round(s, r, e0, e1);
            if (rc) return rc;
        }
        HIP_TRY(hipMemcpyAsync(s->host_ctl, s->S.ctl, sizeof(Ctl), hipMemcpyDeviceToHost, s->stream));
        HIP_TRY(hipStreamSynchronize(s->stream));
        const Ctl& hc = *s->host_ctl;
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
        if (s->timing) {
            for (int64_t k = 0; k < ex; ++k) {
                float ms = 0.f;
                HIP_TRY(hipEventElapsedTime(&ms, s->ev[2 * k], s->ev[2 * k + 1]));
                s->kernel_ms += ms;
                ++s->launches;
            }
        }
        s->rounds_done += ex;
        s->alerts_total = cum;
        s->done = hc.done != 0;
        executed += ex;
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
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipStreamSynchronize(s->stream));
    const DevState& S = s->S;
    const int cur = (int)(s->rounds_done & 1);
    if (S.alg == PUSHSUM) {
        std::vector<double2> sw((size_t)count);
        std::vector<uint8_t> nb((size_t)count);
        HIP_TRY(hipMemcpy(sw.data(), S.sw[cur] + first, sizeof(double2) * count, hipMemcpyDeviceToHost));
        const uint8_t* nbsrc = S.topo == FULL ? S.nb[0] : S.nb[cur];
        HIP_TRY(hipMemcpy(nb.data(), nbsrc + first, count, hipMemcpyDeviceToHost));
        for (int64_t q = 0; q < count; ++q) {
            if (c) c[q] = 0;
            if (sv) sv[q] = sw[q].x;
            if (wv) wv[q] = sw[q].y;
            if (flags) {
                const uint8_t b = nb[q];
                flags[q] = (uint8_t)(((b & B_ACTIVE) ? 1 : 0) | ((b & B_CONV) ? 2 : 0) | (((b >> CNT_SHIFT) & 3) << 2));
            }
        }
    } else {
        std::vector<int32_t> cc((size_t)count);
        HIP_TRY(hipMemcpy(cc.data(), S.c + first, sizeof(int32_t) * count, hipMemcpyDeviceToHost));
        for (int64_t q = 0; q < count; ++q) {
            const int64_t i = first + q;
            const int32_t ci = cc[q];
            if (c) c[q] = ci;
            if (sv) sv[q] = 0.0;
            if (wv) wv[q] = 0.0;
            if (flags) {
                const bool act = (i == (int64_t)S.seed_node || ci >= 1) && ci <= 10;
                flags[q] = (uint8_t)((act ? 1 : 0) | (ci >= 11 ? 2 : 0));
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
    const DevState& S = s->S;
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
    if (S.topo == IMP3D) {
        uint32_t r = 0;
        HIP_TRY(hipSetDevice(s->device));
        HIP_TRY(hipStreamSynchronize(s->stream));
        HIP_TRY(hipMemcpy(&r, S.rnd + j, sizeof r, hipMemcpyDeviceToHost));
        nb.push_back(r);
    }
    for (int64_t k = 0; k < std::min<int64_t>((int64_t)nb.size(), cap); ++k) out[k] = nb[(size_t)k];
    return (int)nb.size();
}

int gp_get_info(gp_sim* s, gp_info* o) {
    if (!s || !o) {
        set_err("gp_get_info: null argument");
        return GP_EINVAL;
    }
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipMemcpyAsync(s->host_ctl, s->S.ctl, sizeof(Ctl), hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    o->population = s->P;
    o->threshold = s->T;
    o->grid = s->g;
    o->seed_node = s->S.seed_node;
    o->rounds = s->rounds_done;
    o->alerts_total = s->alerts_total;
    o->active = s->S.alg == PUSHSUM ? (int64_t)s->host_ctl->active_total : -1;
    o->topology = s->S.topo;
    o->algorithm = s->S.alg;
    o->device = s->device;
    o->num_gpus = 1;
    o->slab_first = 0;
    o->slab_count = s->P;
    return GP_OK;
}

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
    if (name && name_cap > 0) {
        std::snprintf(name, (size_t)name_cap, "%s", bulk_kernel_name(s->S));
    }
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
    for (auto& e : s->ev) (void)hipEventDestroy(e);
    free_all(s);
    if (s->host_ctl) (void)hipHostFree(s->host_ctl);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    delete s;
}

}  // extern "C"
