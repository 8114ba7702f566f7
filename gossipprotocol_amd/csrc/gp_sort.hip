// gp_sort.hip -- rocPRIM device primitives used once, at create (never per round):
//   * Imp3D setup: stable sort of the random edges (rnd[i] -> i) by target, so
//     each receiver's in-list holds its senders in ascending id order (the
//     canonical fold order of SRS v1 B.4), and the scan of the in-degrees into
//     the in-list offsets.  Per-round message binning is hand-written
//     (gp_fullbin.hip).
// Kept in its own translation unit because rocPRIM's templates dominate the
// library's compile time.
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "gp_internal.hpp"

namespace gp {

hipError_t sort_pairs(void* tmp, size_t& tmp_bytes, const uint32_t* kin, uint32_t* kout, const uint32_t* vin,
                      uint32_t* vout, uint32_t n, uint32_t bits, hipStream_t st) {
    return rocprim::radix_sort_pairs(tmp, tmp_bytes, kin, kout, vin, vout, n, 0u, bits, st);
}

hipError_t exclusive_scan_u32(void* tmp, size_t& tmp_bytes, const uint32_t* in, uint32_t* out, uint32_t n,
                              hipStream_t st) {
    return rocprim::exclusive_scan(tmp, tmp_bytes, in, out, 0u, (size_t)n, rocprim::plus<uint32_t>(), st);
}

}  // namespace gp
