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

// BN-statistics exchange variants of the sliced engine, with emulated per-round compute and jitter (512-thread
// workgroups, 64 fp32 partials per workgroup and round, every workgroup needs the 64 sums over all G):
//   V0: one hop, 8-byte {value, tag} granules, every workgroup sweeps G x 512 B (the round-2 engine);
//   V1: one hop, 4-byte self-tagged values (tag in the 2 low mantissa bits), sweep G x 256 B;
//   V2: two hops, 8-byte granules: group k = L % 8 (one XCD under round-robin dispatch) is summed by its leader
//       (L = k, sweeps G / 8 x 512 B) and published as a group record; every workgroup sweeps the 8 records (4 KB);
//   V3: V2 with 4-byte self-tagged values (leader sweeps G / 8 x 256 B, everyone 8 x 256 B).
// work / jitter in 10-ns ticks (s_memrealtime): round r of workgroup L "computes" work + hash(L, r) % jitter.
__device__ __forceinline__ unsigned mb_tag4(int r) { return 1u + (unsigned)((r >> 1) % 3); }
__device__ __forceinline__ void mb_st4(unsigned* p, unsigned tag4, float v) {
  __hip_atomic_store(p, (__float_as_uint(v) & ~3u) | tag4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void mb_st8(unsigned long long* p, unsigned tag, float v) {
  __hip_atomic_store(p, ((unsigned long long)tag << 32) | __float_as_uint(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
// 8-byte granule sweep: lanes 32 hf + j read slots 2j, 2j+1 of unit (2 wv + hf + 16 k); result per wave in cred
template <int KS>
__device__ bool mb_sweep8(const unsigned long long* base, int nunit, int ustride, int wv, int lane, unsigned tag,
                          float* cred, unsigned* err) {
  const int j = lane & 31, hf = lane >> 5;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, 0x7ffffff0, 0x00020000);
  float s0 = 0.f, s1 = 0.f;
  for (unsigned spins = 0;; ++spins) {
    asm volatile("" ::: "memory");
    typedef unsigned v4u_ __attribute__((ext_vector_type(4)));
    v4u_ x[KS];
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      const int u = 2 * wv + hf + 16 * k, uc = u < nunit ? u : nunit - 1;
      x[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, (uc * ustride + 2 * j) * 8, 0, 16);
    }
    bool ok = true;
    s0 = s1 = 0.f;
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      const bool valid = 2 * wv + hf + 16 * k < nunit;
      ok &= !valid || (x[k][1] == tag && x[k][3] == tag);
      s0 += valid ? __uint_as_float(x[k][0]) : 0.f;
      s1 += valid ? __uint_as_float(x[k][2]) : 0.f;
    }
    if (__all(ok)) break;
    if (spins > (1u << 20)) {
      if (lane == 0) atomicOr(err, 1u);
      break;
    }
  }
  s0 += __shfl_xor(s0, 32);
  s1 += __shfl_xor(s1, 32);
  if (lane < 32) {
    cred[wv * 64 + 2 * lane] = s0;
    cred[wv * 64 + 2 * lane + 1] = s1;
  }
  return true;
}
// 4-byte self-tagged sweep: lanes 16 sub + q read slots 4q .. 4q+3 of unit (4 wv + sub + 32 k)
template <int KS>
__device__ bool mb_sweep4(const unsigned* base, int nunit, int ustride, int wv, int lane, unsigned tag4, float* cred,
                          unsigned* err) {
  const int q = lane & 15, sub = lane >> 4;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, 0x7ffffff0, 0x00020000);
  float s[4];
  for (unsigned spins = 0;; ++spins) {
    asm volatile("" ::: "memory");
    typedef unsigned v4u_ __attribute__((ext_vector_type(4)));
    v4u_ x[KS];
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      const int u = 4 * wv + sub + 32 * k, uc = u < nunit ? u : nunit - 1;
      x[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, (uc * ustride + 4 * q) * 4, 0, 16);
    }
    bool ok = true;
#pragma unroll
    for (int i = 0; i < 4; ++i) s[i] = 0.f;
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      const bool valid = 4 * wv + sub + 32 * k < nunit;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        ok &= !valid || (x[k][i] & 3u) == tag4;
        s[i] += valid ? __uint_as_float(x[k][i]) : 0.f;
      }
    }
    if (__all(ok)) break;
    if (spins > (1u << 20)) {
      if (lane == 0) atomicOr(err, 1u);
      break;
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    s[i] += __shfl_xor(s[i], 16);
    s[i] += __shfl_xor(s[i], 32);
  }
  if (lane < 16) {
#pragma unroll
    for (int i = 0; i < 4; ++i) cred[wv * 64 + 4 * q + i] = s[i];
  }
  return true;
}
__device__ __forceinline__ unsigned mb_xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
  return v;
}
// V4: census of the workgroups' XCDs (HW_REG_XCC_ID) at kernel start; per round the members of one XCD hand their
// partials to that XCD's leader through the XCD's L2 (plain granule stores, sc1 = L1-bypassing loads served by the
// shared L2), the leaders publish XCD records write-through (sc1), every workgroup sweeps the <= 8 records.
__device__ void mb_bnx_v4(unsigned* buf, unsigned* err, int rounds, int work, int jitter) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, L = blockIdx.x, G = gridDim.x;
  __shared__ float cred[8 * 64];
  __shared__ int xcl[256];
  __shared__ int mlist[256];
  __shared__ int s_info[16];  // [2] this workgroup leads its XCD, [8 + v] members of xcc v
  unsigned long long* cen = (unsigned long long*)buf + (size_t)2 * 256 * 64 + 2 * 8 * 64;
  const unsigned myx = mb_xcc_id();
  if (t == 0) mb_st8(cen + L, 1u, __uint_as_float(myx));
  for (int k = t; k < G; k += 512) {
    unsigned long long x;
    for (unsigned spins = 0;; ++spins) {
      x = __hip_atomic_load(cen + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((x >> 32) == 1u) break;
      if (spins > (1u << 20)) {
        atomicOr(err, 1u);
        break;
      }
    }
    xcl[k] = (int)(unsigned)x & 7;
  }
  __syncthreads();
  if (t < 8) {
    int n = 0;
    for (int k = 0; k < G; ++k) n += xcl[k] == t;
    s_info[8 + t] = n;
  }
  if (t < G && xcl[t] == (int)myx) {
    int m = 0;
    for (int k = 0; k < t; ++k) m += xcl[k] == (int)myx;
    mlist[m] = t;
    if (t == L) s_info[2] = m == 0;
  }
  __syncthreads();
  const int nm = s_info[8 + myx] < 32 ? s_info[8 + myx] : 32;  // (<= 32 members per XCD for G <= 256)
  const bool leader = s_info[2] != 0;
  float keep = 0.f;
  for (int r = 0; r < rounds; ++r) {
    {
      unsigned h = (unsigned)L * 2654435761u ^ (unsigned)r * 40503u;
      h ^= h >> 13;
      h *= 0x5bd1e995u;
      h ^= h >> 15;
      const unsigned long long dl = (unsigned long long)work + (jitter > 0 ? h % (unsigned)jitter : 0u);
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while (__builtin_amdgcn_s_memrealtime() - t0 < dl) __builtin_amdgcn_s_sleep(1);
    }
    const float v = (float)((L + lane) & 7) + keep;
    const int par = r & 1;
    const unsigned tag = (unsigned)(r + 1);
    unsigned long long* A8 = (unsigned long long*)buf + (size_t)par * 256 * 64;
    unsigned long long* B8 = (unsigned long long*)buf + (size_t)2 * 256 * 64 + par * 8 * 64;
    if (wv == 0)  // plain 8-byte store: stays in this XCD's L2, where the leader's sc1 loads read it
      __hip_atomic_store(A8 + L * 64 + lane, ((unsigned long long)tag << 32) | __float_as_uint(v), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_WORKGROUP);
    if (leader) {
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)A8, (short)0, 0x7ffffff0, 0x00020000);
      const int j = lane & 31, hf = lane >> 5;
      float s0 = 0.f, s1 = 0.f;
      for (unsigned spins = 0;; ++spins) {
        asm volatile("" ::: "memory");
        typedef unsigned v4u_ __attribute__((ext_vector_type(4)));
        v4u_ x[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int u = 2 * wv + hf + 16 * k, uc = mlist[u < nm ? u : nm - 1];
          x[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, (uc * 64 + 2 * j) * 8, 0, 16);
        }
        bool ok = true;
        s0 = s1 = 0.f;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const bool valid = 2 * wv + hf + 16 * k < nm;
          ok &= !valid || (x[k][1] == tag && x[k][3] == tag);
          s0 += valid ? __uint_as_float(x[k][0]) : 0.f;
          s1 += valid ? __uint_as_float(x[k][2]) : 0.f;
        }
        if (__all(ok)) break;
        if (spins > (1u << 20)) {
          if (lane == 0) atomicOr(err, 1u);
          break;
        }
      }
      s0 += __shfl_xor(s0, 32);
      s1 += __shfl_xor(s1, 32);
      if (lane < 32) {
        cred[wv * 64 + 2 * lane] = s0;
        cred[wv * 64 + 2 * lane + 1] = s1;
      }
      __syncthreads();
      if (wv == 0) {
        float s = 0.f;
        for (int k = 0; k < 8; ++k) s += cred[k * 64 + lane];
        mb_st8(B8 + myx * 64 + lane, tag, s);
      }
      __syncthreads();
    }
    // every workgroup: the records of the XCDs that have members (waves 0..3: xcc 2 wv + hf)
    if (wv < 4) {
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)B8, (short)0, 0x7ffffff0, 0x00020000);
      const int j = lane & 31, hf = lane >> 5, xv = 2 * wv + hf;
      const bool valid = s_info[8 + xv] > 0;
      float s0 = 0.f, s1 = 0.f;
      for (unsigned spins = 0;; ++spins) {
        asm volatile("" ::: "memory");
        typedef unsigned v4u_ __attribute__((ext_vector_type(4)));
        const v4u_ x = __builtin_amdgcn_raw_buffer_load_b128(rs, (xv * 64 + 2 * j) * 8, 0, 16);
        const bool ok = !valid || (x[1] == tag && x[3] == tag);
        s0 = valid ? __uint_as_float(x[0]) : 0.f;
        s1 = valid ? __uint_as_float(x[2]) : 0.f;
        if (__all(ok)) break;
        if (spins > (1u << 20)) {
          if (lane == 0) atomicOr(err, 1u);
          break;
        }
      }
      s0 += __shfl_xor(s0, 32);
      s1 += __shfl_xor(s1, 32);
      if (lane < 32) {
        cred[wv * 64 + 2 * lane] = s0;
        cred[wv * 64 + 2 * lane + 1] = s1;
      }
    }
    __syncthreads();
    float s = 0.f;
    for (int k = 0; k < 4; ++k) s += cred[k * 64 + lane];
    keep = s * 1e-9f;
    __syncthreads();
  }
  if (t == 0 && keep == 12345.f) err[1] = 1;
}

template <int V>
__global__ void __launch_bounds__(512) k_mb_bnx(unsigned* buf, unsigned* err, int rounds, int work, int jitter) {
  if constexpr (V == 4) {
    mb_bnx_v4(buf, err, rounds, work, jitter);
    return;
  }
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, L = blockIdx.x, G = gridDim.x;
  __shared__ float cred[8 * 64];
  const int NG = 8, M = (G + NG - 1) / NG, grp = L % NG;
  float keep = 0.f;
  for (int r = 0; r < rounds; ++r) {
    {  // emulated compute of this round
      unsigned h = (unsigned)L * 2654435761u ^ (unsigned)r * 40503u;
      h ^= h >> 13;
      h *= 0x5bd1e995u;
      h ^= h >> 15;
      const unsigned long long dl = (unsigned long long)work + (jitter > 0 ? h % (unsigned)jitter : 0u);
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while (__builtin_amdgcn_s_memrealtime() - t0 < dl) __builtin_amdgcn_s_sleep(1);
    }
    const float v = (float)((L + lane) & 7) + keep;
    const int par = r & 1;
    const unsigned tag = (unsigned)(r + 1), tag4 = mb_tag4(r);
    unsigned long long* A8 = (unsigned long long*)buf + (size_t)par * 256 * 64;
    unsigned* A4 = buf + (size_t)par * 256 * 64;
    unsigned long long* B8 = (unsigned long long*)buf + (size_t)2 * 256 * 64 + par * NG * 64;
    unsigned* B4 = buf + (size_t)2 * 256 * 64 + par * NG * 64;
    int nred = 8;  // waves whose cred rows hold the final partials
    if (wv == 0) {
      if (V == 0 || V == 2) mb_st8(A8 + L * 64 + lane, tag, v);
      else mb_st4(A4 + L * 64 + lane, tag4, v);
    }
    if (V == 0) {
      if (G <= 64) mb_sweep8<4>(A8, G, 64, wv, lane, tag, cred, err);
      else if (G <= 128) mb_sweep8<8>(A8, G, 64, wv, lane, tag, cred, err);
      else mb_sweep8<16>(A8, G, 64, wv, lane, tag, cred, err);
    } else if (V == 1) {
      if (G <= 64) mb_sweep4<2>(A4, G, 64, wv, lane, tag4, cred, err);
      else if (G <= 128) mb_sweep4<4>(A4, G, 64, wv, lane, tag4, cred, err);
      else mb_sweep4<8>(A4, G, 64, wv, lane, tag4, cred, err);
    } else {
      if (L < NG) {  // group leader: sum the group's M members (units L + 8 m), publish the group record
        if (V == 2) {
          if (M <= 16) mb_sweep8<1>(A8 + grp * 64, M, NG * 64, wv, lane, tag, cred, err);
          else mb_sweep8<2>(A8 + grp * 64, M, NG * 64, wv, lane, tag, cred, err);
        } else {
          if (wv < 4 || M > 16) mb_sweep4<1>(A4 + grp * 64, M, NG * 64, wv, lane, tag4, cred, err);
        }
        __syncthreads();
        if (wv == 0) {
          const int nw = V == 2 ? 8 : (M > 16 ? 8 : 4);
          float s = 0.f;
          for (int k = 0; k < nw; ++k) s += cred[k * 64 + lane];
          if (V == 2) mb_st8(B8 + grp * 64 + lane, tag, s);
          else mb_st4(B4 + grp * 64 + lane, tag4, s);
        }
        __syncthreads();
      }
      if (V == 2) {
        if (wv < 4) mb_sweep8<1>(B8, NG, 64, wv, lane, tag, cred, err);
        nred = 4;
      } else {
        if (wv < 2) mb_sweep4<1>(B4, NG, 64, wv, lane, tag4, cred, err);
        nred = 2;
      }
    }
    __syncthreads();
    float s = 0.f;
    for (int k = 0; k < nred; ++k) s += cred[k * 64 + lane];
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

// BN-exchange variants (k_mb_bnx): G workgroups, `rounds` rounds, emulated work / jitter in 10-ns ticks.
// Writes the best kernel time over `iters` (us) and the timeout flag.
int dca_microbench_bnx(int variant, int G, int rounds, int work, int jitter, int iters, float* us, int* err_out) {
  if (G < 8 || G > 256 || G % 8 || variant < 0 || variant > 4) {
    g_err = "microbench_bnx: G in [8, 256], multiple of 8; variant 0..4";
    return -1;
  }
  hipStream_t s;
  HIPCK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const size_t bytes = (size_t)2 * 256 * 64 * 8 + 2 * 8 * 64 * 8 + 256 * 8;
  unsigned* buf;
  unsigned* err;
  HIPCK(hipMalloc(&buf, bytes));
  HIPCK(hipMalloc(&err, 16));
  HIPCK(hipMemset(err, 0, 16));
  hipEvent_t a, b;
  HIPCK(hipEventCreate(&a));
  HIPCK(hipEventCreate(&b));
  float best = 1e30f;
  for (int it = 0; it < iters; ++it) {
    HIPCK(hipMemsetAsync(buf, 0, bytes, s));
    HIPCK(hipEventRecord(a, s));
    switch (variant) {
      case 0: hipLaunchKernelGGL(dca::k_mb_bnx<0>, dim3(G), dim3(512), 0, s, buf, err, rounds, work, jitter); break;
      case 1: hipLaunchKernelGGL(dca::k_mb_bnx<1>, dim3(G), dim3(512), 0, s, buf, err, rounds, work, jitter); break;
      case 2: hipLaunchKernelGGL(dca::k_mb_bnx<2>, dim3(G), dim3(512), 0, s, buf, err, rounds, work, jitter); break;
      case 4: hipLaunchKernelGGL(dca::k_mb_bnx<4>, dim3(G), dim3(512), 0, s, buf, err, rounds, work, jitter); break;
      default: hipLaunchKernelGGL(dca::k_mb_bnx<3>, dim3(G), dim3(512), 0, s, buf, err, rounds, work, jitter); break;
    }
    HIPCK(hipGetLastError());
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
  (void)hipFree(buf);
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
