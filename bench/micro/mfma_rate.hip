// MFMA issue-rate micro-benchmark: how many cycles a bf16 MFMA takes at one and at two waves per SIMD, in the
// patterns the 256 x 256 GEMM kernels use (k_gemm_w4: 64 independent 16x16x32 accumulators per wave and k32 step,
// one operand shared by 8 consecutive MFMAs; k_gemm_pp: two wave groups per SIMD).  Operands are random bf16 in
// registers (no memory traffic in the loop); every workgroup holds 4 or 8 waves on one CU (256 workgroups).
// Reported: wall us, the in-kernel clock (s_memtime / s_memrealtime) and cycles per MFMA per SIMD.
// Standalone: hipcc --offload-arch=gfx950 -O3 mfma_rate.hip -o mfma_rate;  ./mfma_rate   (one JSON line per case)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));  \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

// MODE 0: 8 x 8 accumulators of 16x16x32, A shared by 8 consecutive MFMAs (k_gemm_w4's order)
// MODE 1: the same with a barrier every 64 MFMAs
// MODE 2: 4 x 4 accumulators of 32x32x16 (same 128 x 128 tile per wave, 16 MFMAs of 32 cycles per k16... 32 per k32)
template <int MODE, int NN, int NT>
__global__ void __launch_bounds__(NT, 1) k_mfma(const s16x8* __restrict__ src, float* __restrict__ out, int iters,
                                                 unsigned long long* __restrict__ stamps) {
  const int t = threadIdx.x;
  s16x8 fa[8], fb[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    fa[i] = src[(blockIdx.x * 16 + i) * 64 + (t & 63)];
    fb[i] = src[(blockIdx.x * 16 + 8 + i) * 64 + (t & 63)];
  }
  const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  float sum = 0.f;
  if constexpr (MODE <= 1) {
    f32x4 acc[8][NN];
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int n = 0; n < NN; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int m = 0; m < 8; ++m)
#pragma unroll
        for (int n = 0; n < NN; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[m], fb[n], acc[m][n], 0, 0, 0);
      if (MODE == 1) __builtin_amdgcn_s_barrier();
    }
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int n = 0; n < NN; ++n) sum += acc[m][n][0] + acc[m][n][3];
  } else {
    f32x16 acc[4][NN / 2];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < NN / 2; ++n)
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[m][n][j] = 0.f;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int n = 0; n < NN / 2; ++n)
            acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[m + 4 * s], fb[n + 4 * s], acc[m][n], 0, 0, 0);
    }
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < NN / 2; ++n) sum += acc[m][n][0] + acc[m][n][15];
  }
  const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (t == 0) {
    stamps[blockIdx.x * 2] = c1 - c0;
    stamps[blockIdx.x * 2 + 1] = r1 - r0;
  }
  out[blockIdx.x * blockDim.x + t] = sum;
}

template <int MODE, int NN, int threads>
static void run( const s16x8* src, float* out, unsigned long long* stamps, const char* name) {
  const int iters = 2000, blocks = 256;
  hipLaunchKernelGGL((k_mfma<MODE, NN, threads>), dim3(blocks), dim3(threads), 0, 0, src, out, 10, stamps);
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a));
  hipLaunchKernelGGL((k_mfma<MODE, NN, threads>), dim3(blocks), dim3(threads), 0, 0, src, out, iters, stamps);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  unsigned long long h[512];
  CK(hipMemcpy(h, stamps, sizeof(h), hipMemcpyDeviceToHost));
  double cyc = 0, rt = 0;
  for (int i = 0; i < blocks; ++i) {
    cyc += h[2 * i];
    rt += h[2 * i + 1];
  }
  cyc /= blocks;
  rt /= blocks;
  const int waves_per_simd = threads / 256;
  const double mfma_per_wave = (double)iters * 8 * NN;  // in 16x16x32 units (a 32x32x16 = 2 units, 4 NN per iter)
  const double per_simd = mfma_per_wave * waves_per_simd;
  const double flop = 2.0 * 256 * threads / 64 * mfma_per_wave * 16 * 16 * 32;
  printf("{\"case\": \"%s\", \"waves_per_simd\": %d, \"us\": %.1f, \"ghz\": %.3f, \"cyc_per_mfma16\": %.2f, \"tflops\": %.1f}\n",
         name, waves_per_simd, ms * 1e3, cyc / (rt * 10.0), cyc / per_simd, flop / (ms * 1e-3) / 1e12);
}

int main() {
  const size_t n = 256 * 16 * 64;
  s16x8* src;
  float* out;
  unsigned long long* stamps;
  CK(hipMalloc(&src, n * sizeof(s16x8)));
  CK(hipMalloc(&out, 256 * 512 * sizeof(float)));
  CK(hipMalloc(&stamps, 512 * sizeof(unsigned long long)));
  short* h = (short*)malloc(n * sizeof(s16x8));
  unsigned s = 12345u;
  for (size_t i = 0; i < n * 8; ++i) {  // random bf16 in [-2, 2)
    s = s * 1664525u + 1013904223u;
    const float f = ((s >> 8) * (1.f / 16777216.f)) * 4.f - 2.f;
    unsigned u;
    memcpy(&u, &f, 4);
    h[i] = (short)(u >> 16);
  }
  CK(hipMemcpy(src, h, n * sizeof(s16x8), hipMemcpyHostToDevice));
  run<0, 8, 256>(src, out, stamps, "16x16x32_1wave_8x8");
  run<1, 8, 256>(src, out, stamps, "16x16x32_1wave_8x8_barrier");
  run<0, 4, 256>(src, out, stamps, "16x16x32_1wave_8x4");
  run<0, 4, 512>(src, out, stamps, "16x16x32_2wave_8x4");
  run<2, 8, 256>(src, out, stamps, "32x32x16_1wave_4x4");
  run<2, 4, 512>(src, out, stamps, "32x32x16_2wave_4x2");
  run<0, 8, 256>(src, out, stamps, "16x16x32_1wave_8x8_again");
  return 0;
}
