// Exactly-W peer loads for the xGMI collectives.  W (the world size) is a kernel argument, hence wave-uniform: the
// switch below is one scalar branch, and each case issues its NR loads back to back (all in flight at once, one
// per peer link) before summing them in rank order 0..W-1 -- bitwise the same on every rank.  No rank's slab is
// read that is not summed (a fixed MAXR-deep unroll would re-read a slab over the link for q >= W).
#pragma once
#include <hip/hip_runtime.h>

namespace dca {
typedef float rs_f4 __attribute__((ext_vector_type(4)));

template <int NR, class F>
__device__ __forceinline__ rs_f4 rank_sum_n(F&& ld) {
  rs_f4 p[NR];
#pragma unroll
  for (int q = 0; q < NR; ++q) p[q] = ld(q);
  rs_f4 s = p[0];
#pragma unroll
  for (int q = 1; q < NR; ++q) s += p[q];
  return s;
}
// sum over q in [0, W) of ld(q), W in [1, 8]
template <class F>
__device__ __forceinline__ rs_f4 rank_sum(int W, F&& ld) {
  switch (W) {
    case 1: return rank_sum_n<1>(ld);
    case 2: return rank_sum_n<2>(ld);
    case 3: return rank_sum_n<3>(ld);
    case 4: return rank_sum_n<4>(ld);
    case 5: return rank_sum_n<5>(ld);
    case 6: return rank_sum_n<6>(ld);
    case 7: return rank_sum_n<7>(ld);
    default: return rank_sum_n<8>(ld);
  }
}
}  // namespace dca
