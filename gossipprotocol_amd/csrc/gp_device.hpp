// gp_device.hpp -- host/device helpers shared by the HIP kernels of
// libgossip_hip.so: counter-based RNG, exact fast division, the implicit
// topology and the packed per-node byte.  gfx950 only.
//
// Reference mapping (Program.fs = /root/reference/Project2/Program.fs):
//   Philox draws replace `new Random()` (Program.fs:86,103,128,130,152,193,221,259,263);
//   the lattice slot order is Program.fs:246-257; line Program.fs:182-191;
//   full Program.fs:211-216.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define GP_HD __host__ __device__ __forceinline__

namespace gp {

// ---------------------------------------------------------------- enums
enum Topology : int { LINE = 0, FULL = 1, GRID3D = 2, IMP3D = 3 };
enum Algorithm : int { GOSSIP = 0, PUSHSUM = 1 };
// Philox streams (ctr word 2)
enum Stream : uint32_t { S_TOPO = 0, S_START = 1, S_GOSSIP = 2, S_PUSHSUM = 3, S_INJECT = 4 };

// ---------------------------------------------------------------- node byte
// One byte per node per buffer: bits 0-2 = direction this node sends in during
// the round the buffer belongs to (0..5 lattice, 6 Imp3D random edge, 7 none);
// push-sum only: bit 3 active, bit 4 converged, bits 5-6 stability count.
constexpr uint8_t DIR_MASK = 7, DIR_NONE = 7, DIR_RANDOM = 6;
constexpr uint8_t B_ACTIVE = 8, B_CONV = 16;
constexpr int CNT_SHIFT = 5;
constexpr uint32_t GOSSIP_DONE = 11;  // rumours >= 11 stops sending (Program.fs:85)

// a ^ b ^ k (k wave-uniform).  gfx950 has a three-input bitwise op with a
// lookup table, v_bitop3_b32 (0x96 = a ^ b ^ c); the compiler does not form it
// and emits two v_xor_b32 instead.
GP_HD uint32_t xor3(uint32_t a, uint32_t b, uint32_t k) {
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "s"(k));
    return r;
#else
    return a ^ b ^ k;
#endif
}

// ---------------------------------------------------------------- Philox4x32-10
// Random123 Philox4x32 with 10 rounds; ctr = (node_lo, round, stream, node_hi),
// key = (seed_lo, seed_hi).  Only output words 0 and 1 are consumed.
GP_HD void philox2(uint32_t node, uint32_t round, uint32_t stream, uint32_t k0, uint32_t k1,
                   uint32_t& x, uint32_t& y) {
    uint32_t c0 = node, c1 = round, c2 = stream, c3 = 0;
#if defined(__HIP_DEVICE_COMPILE__)
    // The key is wave-uniform: recompute its schedule per call on the scalar
    // unit instead of letting the compiler keep 20 round keys live across a
    // kernel (they end up spilled to VGPR lanes and cost a v_readlane each).
    asm volatile("" : "+s"(k0), "+s"(k1));
#endif
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t n0 = xor3((uint32_t)(p1 >> 32), c1, k0);
        const uint32_t n2 = xor3((uint32_t)(p0 >> 32), c3, k1);
        c1 = (uint32_t)p1;
        c3 = (uint32_t)p0;
        c0 = n0;
        c2 = n2;
    }
    x = c0;
    y = c1;
}

// N independent Philox4x32-10 draws (same round and stream, nodes node[0..N))
// in one straight-line block: the rounds of the N chains interleave, so their
// multiply latencies overlap; the wave-uniform key schedule is computed once
// per round for all chains.  Bit-identical to N calls of philox2.
template <int N>
GP_HD void philox2_batch(const uint32_t (&node)[N], uint32_t round, uint32_t stream, uint32_t k0, uint32_t k1,
                         uint32_t (&x)[N], uint32_t (&y)[N]) {
    uint32_t c0[N], c1[N], c2[N], c3[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        c0[i] = node[i];
        c1[i] = round;
        c2[i] = stream;
        c3[i] = 0;
    }
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+s"(k0), "+s"(k1));  // see philox2: keep the key schedule off the hoisting path
#endif
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
#pragma unroll
        for (int i = 0; i < N; ++i) {
            const uint64_t p0 = (uint64_t)0xD2511F53u * c0[i];
            const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2[i];
            const uint32_t n0 = xor3((uint32_t)(p1 >> 32), c1[i], k0);
            const uint32_t n2 = xor3((uint32_t)(p0 >> 32), c3[i], k1);
            c1[i] = (uint32_t)p1;
            c3[i] = (uint32_t)p0;
            c0[i] = n0;
            c2[i] = n2;
        }
    }
#pragma unroll
    for (int i = 0; i < N; ++i) {
        x[i] = c0[i];
        y[i] = c1[i];
    }
}

// U(m) = floor(((y<<32)|x) * m / 2^64) for m < 2^32 (exact, no 128-bit type).
GP_HD uint32_t uniform_from(uint32_t x, uint32_t y, uint32_t m) {
    const uint64_t lo = (uint64_t)x * m;
    const uint64_t hi = (uint64_t)y * m + (lo >> 32);
    return (uint32_t)(hi >> 32);
}

GP_HD uint32_t uniform(uint32_t k0, uint32_t k1, uint32_t stream, uint32_t node, uint32_t round,
                       uint32_t m) {
    uint32_t x, y;
    philox2(node, round, stream, k0, k1, x, y);
    return uniform_from(x, y, m);
}

// ---------------------------------------------------------------- push-sum ratio test
// The stability test of Program.fs:114-123 as SRS v1 states it: did the ratio
// move, |RN(s2 / w2) - RN(s / w)| > 1e-10 (both quotients and their difference
// rounded to double)?  Two fp64 divisions are ~30 VALU instructions, a large
// share of a node's work, so a division-free test decides first whenever it can
// prove the answer "moved":
//   N = s2 w - s w2 (b = fma(s2, w, -RN(s w2)), m = RN(w w2)):  |b| > 2^-18 m
// implies |s2/w2 - s/w| = |N| / (w w2) > 2^-20 + 2^-33 >= 1e-10 (1 + 2^-52) +
// 2^-53 (|s2/w2| + |s/w|), i.e. even after rounding both quotients (each off by
// at most 2^-53 of a ratio < 2^32: every ratio is a weighted mean of node ids,
// ids < 2^32) and their difference, the exact test says "moved".  Margins: the
// error of b is at most 2^-53 (|N| + s w2 (1 + 2^-53)) <= 2^-53 |N| + 2^-21 w w2,
// that of m 2^-53 m; the products stay normal (the m and s w2 guards), and s, w
// are >= 0 / > 0.  Everything else -- slow ratio changes, the converging tail --
// takes the exact divisions.  Requires -ffp-contract=off (explicit fma only).
GP_HD bool ratio_moved(double s, double w, double s2, double w2) {
    const double a = s * w2;
    const double b = __builtin_fma(s2, w, -a);
    const double m = w * w2;
    if (m >= 0x1p-900 && (s == 0.0 || a >= 0x1p-900) && __builtin_fabs(b) > 0x1p-18 * m) return true;
    return __builtin_fabs(s2 / w2 - s / w) > 1e-10;
}

// ---------------------------------------------------------------- fast division
// Exact n / d for 32-bit n and a runtime-constant d (libdivide's u32 scheme).
struct FastDiv {
    uint32_t d;
    uint32_t magic;
    uint32_t shift;
    uint32_t mode;  // 0: power of two (shift only), 1: mulhi+shift, 2: mulhi+add+shift
};

inline FastDiv make_fastdiv(uint32_t d) {
    FastDiv f{d, 0, 0, 0};
    if (d == 0) return f;
    const uint32_t l = 31u - (uint32_t)__builtin_clz(d);
    if ((d & (d - 1)) == 0) {
        f.shift = l;
        f.mode = 0;
        return f;
    }
    const uint64_t num = 1ull << (32 + l);
    uint32_t proposed = (uint32_t)(num / d);
    const uint32_t rem = (uint32_t)(num % d);
    const uint32_t e = d - rem;
    if (e < (1u << l)) {
        f.shift = l;
        f.mode = 1;
    } else {
        proposed += proposed;
        const uint32_t twice_rem = rem + rem;
        if (twice_rem >= d || twice_rem < rem) proposed += 1;
        f.shift = l;
        f.mode = 2;
    }
    f.magic = 1u + proposed;
    return f;
}

GP_HD uint32_t mulhi32(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }

GP_HD uint32_t fastdiv(uint32_t n, const FastDiv& f) {
    if (f.mode == 0) return n >> f.shift;
    const uint32_t q = mulhi32(f.magic, n);
    if (f.mode == 1) return q >> f.shift;
    const uint32_t t = ((n - q) >> 1) + q;
    return t >> f.shift;
}

// ---------------------------------------------------------------- topology
// 3D directions in the reference's slot order (Program.fs:246-257):
// 0 x-1, 1 x+1, 2 y+1, 3 y-1, 4 z+1, 5 z-1 (id = x*g^2 + y*g + z).
// Line directions (Program.fs:182-191): 0 = i-1, 1 = i+1.
// The opposite direction is d ^ 1 in both numberings.
struct Geom {
    uint32_t P;  // population
    uint32_t T;  // alert threshold
    uint32_t g, g2;
    FastDiv div_g, div_g2;
};

// Bit d set iff direction d exists for node j.  Imp3D adds the random slot
// after the lattice slots (Program.fs:258-260) -- not part of the mask.
template <int TOPO>
GP_HD uint32_t present_mask(uint32_t j, const Geom& G) {
    if (TOPO == LINE) return (j > 0 ? 1u : 0u) | (j + 1 < G.P ? 2u : 0u);
    const uint32_t x = fastdiv(j, G.div_g2);
    const uint32_t rem = j - x * G.g2;
    const uint32_t y = fastdiv(rem, G.div_g);
    const uint32_t z = rem - y * G.g;
    const uint32_t gm = G.g - 1;
    return (x > 0 ? 1u : 0u) | (x < gm ? 2u : 0u) | (y < gm ? 4u : 0u) | (y > 0 ? 8u : 0u) |
           (z < gm ? 16u : 0u) | (z > 0 ? 32u : 0u);
}

template <int TOPO>
GP_HD uint32_t nbr(uint32_t j, uint32_t d, const Geom& G) {
    if (TOPO == LINE) return d == 0 ? j - 1 : j + 1;
    switch (d) {
        case 0: return j - G.g2;
        case 1: return j + G.g2;
        case 2: return j + G.g;
        case 3: return j - G.g;
        case 4: return j + 1;
        default: return j - 1;
    }
}

GP_HD uint32_t popc6(uint32_t m) {
#if defined(__HIP_DEVICE_COMPILE__)
    return (uint32_t)__popc(m);
#else
    return (uint32_t)__builtin_popcount(m);
#endif
}

// Slot k (0-based, in slot order) -> direction.  k == popc(mask) is the Imp3D
// random slot.
GP_HD uint32_t slot_to_dir(uint32_t mask, uint32_t k) {
#pragma unroll
    for (uint32_t d = 0; d < 6; ++d) {
        if (mask & (1u << d)) {
            if (k == 0) return d;
            --k;
        }
    }
    return DIR_RANDOM;
}

// slot_to_dir with the interior-node case (all six lattice slots present) first.
GP_HD uint32_t slot_to_dir_fast(uint32_t mask, uint32_t k) {
    if (mask == 63u) return k < 6u ? k : (uint32_t)DIR_RANDOM;
    return slot_to_dir(mask, k);
}

// Present-direction mask from lattice coordinates (same bits as present_mask).
GP_HD uint32_t mask_xyz(uint32_t x, uint32_t y, uint32_t z, uint32_t gm) {
    return (x > 0 ? 1u : 0u) | (x < gm ? 2u : 0u) | (y < gm ? 4u : 0u) | (y > 0 ? 8u : 0u) | (z < gm ? 16u : 0u) |
           (z > 0 ? 32u : 0u);
}

// Full topology slot k of node i (Program.fs:211-216: all j != i, ascending).
GP_HD uint32_t full_target(uint32_t i, uint32_t k) { return k < i ? k : k + 1; }

}  // namespace gp
