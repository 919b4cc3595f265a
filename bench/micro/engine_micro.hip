// Calibration micro-benchmarks of the NetResDeep engine's building blocks (kernel-boundary floor, in-kernel
// granule exchange, xGMI one-shot protocol).  Diagnostic only: built as libdca_micro.so by
// `python -m distributeddataparallel_cifar10_amd.build micro` and used by bench/stamps.py, bench/xchg_bench.py and
// bench/xgmi_allreduce_bench.py.  Nothing here is linked into the production engine library.
#include <algorithm>
#include <string>

#include "../../distributeddataparallel_cifar10_amd/csrc/netresdeep_kernels.hip"
#include "../../distributeddataparallel_cifar10_amd/csrc/xgmi_allreduce.hip"

namespace {
thread_local std::string g_err;
#define HIPCK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      g_err = std::string(#x) + ": " + hipGetErrorString(e_);                      \
      return -1;                                                                   \
    }                                                                              \
  } while (0)
}  // namespace

namespace dca {
__global__ void k_mb_empty(int) {}
// Memory round-trip calibration kernels (8 float4 = 32 KiB per workgroup unless noted):
//   1: all WGs read the same 32 KiB (never written) + serial LDS reduce by thread 0
//   2: one float per thread, WG-private, then store
//   3: WG-private 32 KiB (never written), per-thread sums stored
//   4: WG-private 32 KiB written by the PREVIOUS kernel at the same WG index (ping-pong)
//   5: like 4 but reading the region written by WG (w+1) % grid (another XCD under round-robin dispatch)
//   6: every WG reads the same 32 KiB that WG 0 of the previous kernel wrote (BN-partials pattern)
__global__ void __launch_bounds__(NT) k_mb_load(const f32x4* src, f32x4* dst, int kind) {
  const int t = threadIdx.x, w = blockIdx.x, g = gridDim.x;
  if (kind == 2) {
    const float v = ((const float*)src)[w * NT + t];
    ((float*)dst)[w * NT + t] = v + 1.f;
    return;
  }
  const int base = kind == 1 || kind == 6 ? 0 : (kind == 5 ? ((w + 1) % g) : w) * 2048;
  f32x4 v[8];
#pragma unroll
  for (int m = 0; m < 8; ++m) v[m] = src[base + t + NT * m];
  if (kind == 1) {
    float s = 0.f;
#pragma unroll
    for (int m = 0; m < 8; ++m) s += v[m].x + v[m].y + v[m].z + v[m].w;
    __shared__ float r[NT];
    r[t] = s;
    __syncthreads();
    if (t == 0) {
      float a = 0.f;
      for (int k = 0; k < NT; ++k) a += r[k];
      ((float*)dst)[w] = a;
    }
    return;
  }
  if (kind == 3) {
    f32x4 s = v[0];
#pragma unroll
    for (int m = 1; m < 8; ++m) s += v[m];
    dst[w * NT + t] = s;
    return;
  }
  if (kind == 6 && w != 0) {
    f32x4 s = v[0];
#pragma unroll
    for (int m = 1; m < 8; ++m) s += v[m];
    dst[4096 + w * NT + t] = s;  // scratch, away from the region the next kernel reads
    return;
  }
#pragma unroll
  for (int m = 0; m < 8; ++m) dst[(kind == 6 ? 0 : w * 2048) + t + NT * m] = v[m] + 1.f;
}
// In-kernel all-gather of 64 floats per workgroup among G co-resident workgroups, `rounds` times
// (the BN-statistics exchange of a persistent design).  Data-as-flag granules {tag, value} (8-byte relaxed
// agent-scope atomic stores/loads, i.e. sc1 write-through / L2-bypassing): no fences needed.  Parity
// double-buffered by round.  Every spin is bounded; a timeout sets *err and the kernel still completes.
template <int NTH>
__global__ void __launch_bounds__(NTH) k_mb_xchg(unsigned long long* gran, unsigned* err, int rounds, int sleep) {
  const int t = threadIdx.x, w = blockIdx.x, G = gridDim.x;
  __shared__ float red[64];
  float keep = 0.f;
  for (int r = 0; r < rounds; ++r) {
    const unsigned long long tag = (unsigned long long)(r + 1) << 32;
    unsigned long long* buf = gran + (size_t)(r & 1) * G * 64;
    if (t < 64) {
      const float v = (float)(w + t) + keep;
      __hip_atomic_store(buf + w * 64 + t, tag | __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      float acc = 0.f;
      for (unsigned spins = 0;; ++spins) {
        bool ok = true;
        acc = 0.f;
        for (int k = 0; k < G; ++k) {
          const unsigned long long x = __hip_atomic_load(buf + k * 64 + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok &= (x & 0xffffffff00000000ull) == tag;
          acc += __uint_as_float((unsigned)x);
        }
        if (__all(ok)) break;
        if (spins > (1u << 20)) {
          atomicOr(err, 1u);
          break;
        }
        if (sleep) __builtin_amdgcn_s_sleep(1);
      }
      red[t] = acc;
    }
    __syncthreads();
    keep = red[t & 63] * 1e-9f;
    __syncthreads();
  }
  if (t == 0 && keep == 12345.f) err[1] = 1;  // keep the chain live
}
// Same exchange, but the sweep is spread over all waves of the workgroup and uses plain (non-volatile)
// sc1 buffer loads, so every wave has all of its granule loads in flight at once.
template <int NTH>
__global__ void __launch_bounds__(NTH) k_mb_xchg2(unsigned long long* gran, unsigned* err, int rounds) {
  constexpr int NW = NTH / 64, KMAX = 8;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, w = blockIdx.x, G = gridDim.x;
  __shared__ float red[NW][64];
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(gran, (short)0, 2 * G * 64 * 8, 0x00020000);
  float keep = 0.f;
  for (int r = 0; r < rounds; ++r) {
    const unsigned tag = (unsigned)(r + 1);
    const int boff = (r & 1) * G * 64;
    if (wave == 0) {
      const float v = (float)(w + lane) + keep;
      __hip_atomic_store(gran + boff + w * 64 + lane, ((unsigned long long)tag << 32) | __float_as_uint(v),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    float acc = 0.f;
    for (unsigned spins = 0;; ++spins) {
      bool ok = true;
      acc = 0.f;
      unsigned lo[KMAX], hi[KMAX];
#pragma unroll
      for (int kk = 0; kk < KMAX; ++kk) {
        const int k = wave + NW * kk;
        if (k < G) {
          const auto x = __builtin_amdgcn_raw_buffer_load_b64(rs, (boff + k * 64 + lane) * 8, 0, 16);
          lo[kk] = x[0];
          hi[kk] = x[1];
        } else {
          lo[kk] = 0u;
          hi[kk] = tag;
        }
      }
#pragma unroll
      for (int kk = 0; kk < KMAX; ++kk) {
        ok &= hi[kk] == tag;
        acc += __uint_as_float(lo[kk]);
      }
      if (__all(ok)) break;
      if (spins > (1u << 20)) {
        atomicOr(err, 1u);
        break;
      }
    }
    red[wave][lane] = acc;
    __syncthreads();
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NW; ++k) s += red[k][lane];
    keep = s * 1e-9f;
    __syncthreads();
  }
  if (t == 0 && keep == 12345.f) err[1] = 1;
}
}  // namespace dca

extern "C" {

const char* dca_micro_last_error() { return g_err.c_str(); }

// Persistent-exchange calibration: G workgroups of `nth` threads, `rounds` all-gather rounds.
// Writes the kernel time (us, median of `iters`) and the timeout flag.
int dca_microbench_xchg(int G, int nth, int rounds, int iters, int sleep, float* us, int* err_out) {
  hipStream_t s;
  HIPCK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  unsigned long long* gran;
  unsigned* err;
  HIPCK(hipMalloc(&gran, (size_t)2 * G * 64 * 8));
  HIPCK(hipMalloc(&err, 16));
  HIPCK(hipMemset(err, 0, 16));
  hipEvent_t a, b;
  HIPCK(hipEventCreate(&a));
  HIPCK(hipEventCreate(&b));
  float best = 1e30f;
  for (int it = 0; it < iters; ++it) {
    HIPCK(hipMemsetAsync(gran, 0, (size_t)2 * G * 64 * 8, s));
    HIPCK(hipEventRecord(a, s));
    if (sleep == 2 && nth == 1024) hipLaunchKernelGGL(dca::k_mb_xchg2<1024>, dim3(G), dim3(1024), 0, s, gran, err, rounds);
    else if (sleep == 2) hipLaunchKernelGGL(dca::k_mb_xchg2<256>, dim3(G), dim3(256), 0, s, gran, err, rounds);
    else if (nth == 1024) hipLaunchKernelGGL(dca::k_mb_xchg<1024>, dim3(G), dim3(1024), 0, s, gran, err, rounds, sleep);
    else hipLaunchKernelGGL(dca::k_mb_xchg<256>, dim3(G), dim3(256), 0, s, gran, err, rounds, sleep);
    HIPCK(hipEventRecord(b, s));
    HIPCK(hipEventSynchronize(b));
    float ms = 0.f;
    HIPCK(hipEventElapsedTime(&ms, a, b));
    best = std::min(best, ms);
  }
  unsigned herr[2];
  HIPCK(hipMemcpy(herr, err, 8, hipMemcpyDeviceToHost));
  *us = best * 1e3f;
  *err_out = (int)herr[0];
  (void)hipFree(gran);
  (void)hipFree(err);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  (void)hipStreamDestroy(s);
  return 0;
}

// xGMI all-reduce protocol cost without peers in other processes: W ranks simulated in THIS process, one
// stream and one uncached region each (so all ranks' kernels are co-resident, as on W separate GPUs), `iters`
// all-reduces of FLAT_N floats per rank.  Writes mean microseconds per all-reduce; *err_out = timeout flag.
int dca_microbench_xgmi(int W, int iters, float* us, int* err_out) {
  // W <= 3: with GPU_MAX_HW_QUEUES=4 a 4th user stream can share a hardware queue with another, which serialises
  // two ranks' kernels and deadlocks the flag wait until its deadline (measured: the W=4 run never finished).
  if (W < 1 || W > dca::xg::MAXR || W > 3 || iters < 1) {
    g_err = "microbench_xgmi: 1 <= W <= 3 (co-resident streams per process), iters >= 1";
    return -1;
  }
  hipStream_t st[3];
  char* reg[3];
  float *src, *dst;
  unsigned* err;
  dca::xg::Peers P{};
  for (int q = 0; q < W; ++q) {
    HIPCK(hipStreamCreateWithFlags(&st[q], hipStreamNonBlocking));
    HIPCK(hipExtMallocWithFlags((void**)&reg[q], dca::xg::REGION_BYTES, hipDeviceMallocUncached));
    HIPCK(hipMemset(reg[q], 0, dca::xg::REGION_BYTES));
    P.base[q] = reg[q];
  }
  HIPCK(hipMalloc(&src, sizeof(float) * dca::FLAT_ALLOC * W));
  HIPCK(hipMalloc(&dst, sizeof(float) * dca::FLAT_ALLOC * W));
  HIPCK(hipMemset(src, 0, sizeof(float) * dca::FLAT_ALLOC * W));
  HIPCK(hipMalloc(&err, 16));
  HIPCK(hipMemset(err, 0, 16));
  HIPCK(hipDeviceSynchronize());
  hipEvent_t a, b;
  HIPCK(hipEventCreate(&a));
  HIPCK(hipEventCreate(&b));
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    HIPCK(hipDeviceSynchronize());
    HIPCK(hipEventRecord(a, st[0]));
    for (int q = 1; q < W; ++q) HIPCK(hipStreamWaitEvent(st[q], a, 0));
    for (int i = 0; i < iters; ++i)
      for (int q = 0; q < W; ++q) {
        dca::Ctx cx{};
        cx.ws = W;
        cx.rank = q;
        hipLaunchKernelGGL(dca::xg::k_xgmi_ar_sgd<true>, dim3(dca::xg::AR_NB), dim3(dca::xg::AR_T), 0, st[q], cx, P,
                           (const float*)(src + (size_t)q * dca::FLAT_ALLOC), dst + (size_t)q * dca::FLAT_ALLOC, err,
                           0, 2ull * 100000000ull);
      }
    for (int q = 1; q < W; ++q) {
      hipEvent_t e;
      HIPCK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      HIPCK(hipEventRecord(e, st[q]));
      HIPCK(hipStreamWaitEvent(st[0], e, 0));
      (void)hipEventDestroy(e);
    }
    HIPCK(hipEventRecord(b, st[0]));
    HIPCK(hipEventSynchronize(b));
    float ms = 0.f;
    HIPCK(hipEventElapsedTime(&ms, a, b));
    best = std::min(best, 1e3f * ms / (float)iters);
  }
  unsigned h = 0;
  HIPCK(hipMemcpy(&h, err, sizeof(unsigned), hipMemcpyDeviceToHost));
  *us = best;
  *err_out = h ? 1 : 0;
  for (int q = 0; q < W; ++q) {
    (void)hipStreamDestroy(st[q]);
    (void)hipFree(reg[q]);
  }
  (void)hipFree(src);
  (void)hipFree(dst);
  (void)hipFree(err);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return 0;
}

// Launch-floor calibration: a hipGraph of `nk` dependent kernels of `kind` (0 empty; 1..6 see k_mb_load)
// with `grid` workgroups, replayed `iters` times.  Writes microseconds per kernel to *us.
int dca_microbench(int kind, int nk, int grid, int iters, float* us) {
  hipStream_t s;
  HIPCK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  char* buf;
  const size_t half = (size_t)(grid + 1) * 2048 * 16 + (1 << 16);
  HIPCK(hipMalloc(&buf, 2 * half));
  HIPCK(hipMemset(buf, 0, 2 * half));
  hipGraph_t g;
  HIPCK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int k = 0; k < nk; ++k) {
    const bool odd = (k & 1) && kind >= 4;
    const dca::f32x4* src = (const dca::f32x4*)(buf + (odd ? half : 0));
    dca::f32x4* dst = (dca::f32x4*)(buf + (odd ? 0 : half));
    if (kind == 0) hipLaunchKernelGGL(dca::k_mb_empty, dim3(grid), dim3(dca::NT), 0, s, k);
    else hipLaunchKernelGGL(dca::k_mb_load, dim3(grid), dim3(dca::NT), 0, s, src, dst, kind);
  }
  HIPCK(hipStreamEndCapture(s, &g));
  hipGraphExec_t ex;
  HIPCK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
  hipEvent_t a, b;
  HIPCK(hipEventCreate(&a));
  HIPCK(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w) HIPCK(hipGraphLaunch(ex, s));
  HIPCK(hipEventRecord(a, s));
  for (int it = 0; it < iters; ++it) HIPCK(hipGraphLaunch(ex, s));
  HIPCK(hipEventRecord(b, s));
  HIPCK(hipEventSynchronize(b));
  float ms = 0.f;
  HIPCK(hipEventElapsedTime(&ms, a, b));
  *us = 1e3f * ms / (float)(iters * nk);
  (void)hipGraphExecDestroy(ex);
  (void)hipGraphDestroy(g);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  (void)hipFree(buf);
  (void)hipStreamDestroy(s);
  return 0;
}

}  // extern "C"
