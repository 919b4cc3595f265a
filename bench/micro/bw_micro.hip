// HBM ceilings of the byte patterns of ResNet-50's short-K 1x1 GEMMs (no MFMA, no LDS): every thread streams rows of
// a [M, KIN] bf16 input and writes rows of a [M, KOUT] bf16 output (a row's input bytes are folded into its output
// so no load is dead), so the read : write ratio is KIN : KOUT, like C[M, N] = A[M, K] B^T at K = KIN, N = KOUT.
// Variants: default / non-temporal loads and stores, rows in flight per thread.  This is the bandwidth a stream
// GEMM epilogue can at best reach for that shape; bench/gemm_shortk.py measures the GEMM itself.
// Standalone: hipcc --offload-arch=gfx950 -O3 bw_micro.hip -o bw_micro;  ./bw_micro   (one JSON line per case)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));  \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

typedef unsigned v4u __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ v4u ld(const v4u* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(v4u* p, v4u v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// thread t of the grid handles rows r = t / CPR + U * stride ... (CPR = 16-B chunks per output row); each output
// chunk c of row r gets input chunk c % IPR of the same row (+ the row index so nothing is constant-folded)
template <int U, bool NTL, bool NTS>
__global__ void __launch_bounds__(256) k_stream(const v4u* __restrict__ in, v4u* __restrict__ out, long M, int IPR,
                                                int CPR) {
  const long total = M * CPR;
  const long stride = (long)gridDim.x * 256;
  for (long base = (long)blockIdx.x * 256 + threadIdx.x; base < total; base += stride * U) {
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = base + u * stride;
      const long r = i / CPR;
      const int c = (int)(i - r * CPR);
      v[u] = i < total ? ld<NTL>(in + r * IPR + (c % IPR)) : v4u{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = base + u * stride;
      if (i < total) st<NTS>(out + i, v[u] + (unsigned)i);
    }
  }
}

template <int U, bool NTL, bool NTS>
static float run(const v4u* in, v4u* out, long M, int kin, int kout, int grid) {
  const int IPR = kin * 2 / 16, CPR = kout * 2 / 16;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  std::vector<float> t;
  for (int it = 0; it < 25; ++it) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL((k_stream<U, NTL, NTS>), dim3(grid), dim3(256), 0, 0, in, out, M, IPR, CPR);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, a, b));
    if (it >= 5) t.push_back(ms * 1e3f);
  }
  std::sort(t.begin(), t.end());
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return t[t.size() / 2];
}

int main() {
  struct Shape {
    long M;
    int kin, kout;
  } shapes[] = {{802816, 64, 256}, {802816, 256, 64}, {200704, 128, 512}, {802816, 64, 64}, {200704, 512, 128}};
  size_t maxb = 0;
  for (auto& s : shapes) maxb = std::max(maxb, (size_t)s.M * std::max(s.kin, s.kout) * 2);
  v4u *in = nullptr, *out = nullptr;
  CK(hipMalloc(&in, maxb));
  CK(hipMalloc(&out, maxb));
  CK(hipMemset(in, 1, maxb));
  CK(hipMemset(out, 0, maxb));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  for (auto& s : shapes) {
    const double bytes = (double)s.M * (s.kin + s.kout) * 2;
    for (int wpc : {4, 8, 16}) {
      const int grid = wpc * ncu;
      struct V {
        const char* name;
        float us;
      } vs[] = {
          {"u4", run<4, false, false>(in, out, s.M, s.kin, s.kout, grid)},
          {"u4_nts", run<4, false, true>(in, out, s.M, s.kin, s.kout, grid)},
          {"u4_ntl_nts", run<4, true, true>(in, out, s.M, s.kin, s.kout, grid)},
          {"u8_nts", run<8, false, true>(in, out, s.M, s.kin, s.kout, grid)},
          {"u2_nts", run<2, false, true>(in, out, s.M, s.kin, s.kout, grid)},
      };
      for (auto& v : vs)
        printf("{\"M\": %ld, \"kin\": %d, \"kout\": %d, \"wg_per_cu\": %d, \"variant\": \"%s\", \"us\": %.1f, "
               "\"tbps\": %.2f}\n",
               s.M, s.kin, s.kout, wpc, v.name, v.us, bytes / v.us / 1e6);
      fflush(stdout);
    }
  }
  CK(hipFree(in));
  CK(hipFree(out));
  return 0;
}
