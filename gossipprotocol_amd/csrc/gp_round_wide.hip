// gp_round_wide.hip -- the tiled round kernels of gp_round.hip compiled a second
// time as the small-population size class: 1024 threads per 1024-node tile, one
// node per thread, 8 waves per SIMD (gp::wide::launch_round_tile).
//
// A tile then costs one dependent memory round trip in its node phase instead of
// four (gp_round.hip's 256 threads x 4 nodes), which is what bounds a round when
// the network has only a few tiles per resident block: C2 (3D push-sum, P = 10^6,
// 977 tiles) measured 26.4 -> 21.0 us per round (profiles/r04/c2_tile_shape.txt).
// At 10^9 nodes the 4-nodes-per-thread kernel is faster (more waves' worth of
// memory-level parallelism per VGPR), so gp_api.hip's choose_kernel picks by size.
#define GP_ROUND_WIDE 1
#define GP_TPB 1024
#define GP_NPT 1
#define GP_MINB 8
#include "gp_round.hip"
