// Microbenchmark: ds_read_b128 at 2-byte-aligned LDS addresses on gfx950 (correctness + cost vs aligned).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(512) k_check(unsigned* bad, int sh) {
  __shared__ __attribute__((aligned(16))) unsigned short lds[16384];
  for (int i = threadIdx.x; i < 16384; i += 512) lds[i] = (unsigned short)(i * 7 + 3);
  __syncthreads();
  const int base = (threadIdx.x * 24) % 16000 + sh;
  u16x8 v;
  __builtin_memcpy(&v, lds + base, 16);
  for (int j = 0; j < 8; ++j)
    if (v[j] != (unsigned short)((base + j) * 7 + 3)) atomicAdd(bad, 1u);
}

template <int SH>
__global__ void __launch_bounds__(512) k_time(f4* out, int iters, long long* cyc) {
  __shared__ __attribute__((aligned(16))) unsigned short lds[16384];
  for (int i = threadIdx.x; i < 16384; i += 512) lds[i] = (unsigned short)i;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // wgrad-like pattern: 16 rows (c) x 4 chunks (q), row stride 296 bf16
  const unsigned short* p = lds + (lane & 15) * 296 + (lane >> 4) * 8 + w * 16 + SH;
  f4 acc = {0, 0, 0, 0};
  long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      bf16x8 b;
      __builtin_memcpy(&b, p + s * 32, 16);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, b, acc, 0, 0, 0);
    }
    asm volatile("" ::: "memory");
  }
  long long t1 = clock64();
  out[threadIdx.x + blockIdx.x * 512] = acc;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  unsigned* bad;
  f4* out;
  long long* cyc;
  hipMalloc(&bad, 4);
  hipMalloc(&out, 64 * 512 * sizeof(f4));
  hipMalloc(&cyc, 64 * 8);
  for (int sh = 0; sh < 8; ++sh) {
    hipMemset(bad, 0, 4);
    hipLaunchKernelGGL(k_check, dim3(1), dim3(512), 0, 0, bad, sh);
    unsigned h = 0;
    hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost);
    printf("shift %d elements: mismatches %u\n", sh, h);
  }
  long long c0, c1, c2;
  hipLaunchKernelGGL(k_time<0>, dim3(32), dim3(512), 0, 0, out, 1000, cyc);
  hipDeviceSynchronize();
  hipLaunchKernelGGL(k_time<0>, dim3(32), dim3(512), 0, 0, out, 1000, cyc);
  hipMemcpy(&c0, cyc, 8, hipMemcpyDeviceToHost);
  hipLaunchKernelGGL(k_time<1>, dim3(32), dim3(512), 0, 0, out, 1000, cyc);
  hipMemcpy(&c1, cyc, 8, hipMemcpyDeviceToHost);
  hipLaunchKernelGGL(k_time<2>, dim3(32), dim3(512), 0, 0, out, 1000, cyc);
  hipMemcpy(&c2, cyc, 8, hipMemcpyDeviceToHost);
  printf("cycles per (8 reads + 8 mfma) x 1000: aligned %lld, +2B %lld, +4B %lld\n", c0, c1, c2);
  return 0;
}
