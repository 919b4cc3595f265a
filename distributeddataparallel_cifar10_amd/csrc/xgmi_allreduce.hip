// One-shot gradient all-reduce over xGMI peer-to-peer reads, fused with the averaging SGD step.
//
// Replaces the reference's DDP Reducer all-reduce (reference main.py:63, SURVEY.md 2.4 CC5 + CC4) for ranks of
// ONE node.  The whole NetResDeep gradient is 304 KB (fp32): a ring all-reduce over 8 GPUs is 14 dependent
// latency-bound steps, while the 8 MI355X of a node are fully connected by xGMI (7 point-to-point links per GPU),
// so every rank simply reads all 7 peers' gradients at once -- one link per peer, ~38 KB per link per 1/8 of the
// buffer -- and sums them in registers (SURVEY.md 5.8 cost model: one-shot wins for buckets this small).
//
// Shared region (one per rank, exported with hipIpcGetMemHandle and mapped by every peer):
//   [flags: MAXR ranks x AR_NB workgroups ints, padded to 4 KiB][slab parity 0][slab parity 1]
// allocated uncached (hipDeviceMallocUncached) so no L2 line of it is ever stale on any GPU.
//
// Protocol of workgroup b (it owns float4 chunk b of the flat buffer [0, FLAT_N), on every rank):
//   1. ep = my_flags[me][b] + 1 (the epoch this workgroup last published, plus one); slab parity = ep & 1
//   2. copy my chunk b of cx.grads into my slab[parity] (write-through store); wait for it (vmcnt) + barrier
//   3. store ep into flags[me][b] of EVERY rank (itself included)
//   4. wait until my flags[q][b] >= ep for all ranks q (bounded by a real-time deadline -> error bit, no hang)
//   5. read chunk b of all W slabs[parity] (cache-bypassing loads); sum in rank order 0..W-1 (bitwise identical
//      on every rank); write the sum to cx.grads; SGD with 1/W averaging + derived weight copies; the
//      running-stat segment [OFF_RS, FLAT_N) is rank 0's BN buffers (others contribute 0): CC4.
// Memory ordering without L2 write-backs: the slab and flag stores are system-coherent write-through stores
// (cache policy sc0 sc1) to uncached memory, a `s_waitcnt vmcnt(0)` + workgroup barrier orders them before the
// flag store, and the slab loads are sc0 sc1 loads that bypass every cache.  (A __threadfence_system() per wave
// -- buffer_wbl2 of the whole XCD L2 + buffer_inv -- measured ~48 us per all-reduce with 2 ranks on one GPU.)
// Reuse safety: a rank writes slab[parity] again at epoch ep+2 only after its workgroup b passed step 4 of
// epoch ep+1, i.e. after every peer started epoch ep+1, i.e. (stream order) after every peer finished reading
// epoch ep.  Parities alternate, so epoch ep+1's writes never touch what epoch ep's readers read.
#pragma once
#include "common.h"
#include "rank_sum.h"

namespace dca {
namespace xg {

constexpr int MAXR = 8;                                  // ranks of one xGMI node
constexpr int AR_T = 256;                                // threads per workgroup: one float4 each
constexpr int AR_V4 = FLAT_N / 4;                        // 19035 float4 (FLAT_N is a multiple of 4)
constexpr int AR_NB = (AR_V4 + AR_T - 1) / AR_T;         // 75 workgroups
constexpr size_t FLAG_BYTES = 8192;                      // >= MAXR * max(AR_NB, pks::NSEG) * 4
constexpr size_t SLAB_FLOATS = (size_t)AR_NB * AR_T * 4;  // 76800 >= FLAT_N
constexpr size_t REGION_BYTES = FLAG_BYTES + 2 * SLAB_FLOATS * 4;
static_assert(MAXR * AR_NB * 4 <= (int)FLAG_BYTES, "flag area too small");
static_assert(FLAT_N % 4 == 0, "flat buffer must be float4 granular");

struct Peers {
  char* base[MAXR];           // every rank's shared region, mapped into this process (own one at base[rank])
  unsigned long long* ticks;  // optional [2]: s_memrealtime ticks spent in the kernel by workgroup 0, calls
};

typedef unsigned v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int flag_load(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void flag_store(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// Epochs count calls and wrap modulo 2^32 (after ~2^31 steps a plain signed compare would overflow): "flag f has
// not reached epoch ep yet" as a wrap-aware serial-number comparison; next_ep is the wrapping increment.
__device__ __forceinline__ bool flag_before(int f, int ep) { return (int)((unsigned)f - (unsigned)ep) < 0; }
__device__ __forceinline__ int next_ep(int f) { return (int)((unsigned)f + 1u); }
// The exchange word's bit 31: a peer-flag wait of this rank expired (set here, read and cleared by the host).
__device__ __forceinline__ int failed(const unsigned* err) {
  return (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 0x80000000u) ? 1 : 0;
}
// Wait until flag *f has reached epoch ep; on expiry of `deadline` (s_memrealtime ticks) set bit 31 of *err.
__device__ __forceinline__ void wait_flag(const int* f, int ep, unsigned long long deadline, unsigned* err) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (flag_before(flag_load(f), ep)) {
    __builtin_amdgcn_s_sleep(1);
    if (__builtin_amdgcn_s_memrealtime() - t0 > deadline) {
      atomicOr(err, 0x80000000u);
      break;
    }
  }
}
__device__ __forceinline__ float* slab(const Peers& P, int q, int parity) {
  return (float*)(P.base[q] + FLAG_BYTES) + (size_t)parity * SLAB_FLOATS;
}

// src: this rank's gradient (cx.grads); `sgd` 0 = sum into `sum_out` only (self-test), 1 = training step.
// `deadline_ticks`: wait limit in s_memrealtime ticks (100 MHz); on expiry err bit 31 is set and the workgroup
// neither sums nor updates (the host raises on the word at its next check).  With the word already set on entry it
// does not publish either: the flag stops advancing, so every peer's next wait for this rank expires as well and all
// ranks fail together (seg_exchange in netresdeep_pks.hip: same rule).
template <bool BF>
__global__ void __launch_bounds__(AR_T) k_xgmi_ar_sgd(Ctx cx, Peers P, const float* src, float* sum_out,
                                                      unsigned* err, int sgd, unsigned long long deadline_ticks) {
  const int b = blockIdx.x, t = threadIdx.x, W = cx.ws, me = cx.rank;
  const int v = b * AR_T + t;
  const bool live = v < AR_V4;
  int* myflags = (int*)P.base[me];
  __shared__ int s_ep, s_fail;
  const unsigned long long t_in = __builtin_amdgcn_s_memrealtime();
  if (t == 0) {
    s_ep = next_ep(flag_load(myflags + me * AR_NB + b));
    s_fail = failed(err);
  }
  const f32x4 g = live ? *(const f32x4*)(src + 4 * v) : f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();
  const int ep = s_ep, par = ep & 1;
  if (s_fail) return;
  constexpr int SYS = 17;  // cache policy sc0 | sc1: system-coherent (write-through store / cache-bypassing load)
  const __amdgpu_buffer_rsrc_t mine =
      __builtin_amdgcn_make_buffer_rsrc(slab(P, me, par), (short)0, (int)(SLAB_FLOATS * 4), 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, g), mine, 16 * v, 0, SYS);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's slab store is performed
  __syncthreads();                                    // ... and every thread's of this workgroup
  if (t < W) flag_store((int*)P.base[t] + me * AR_NB + b, ep);
  if (t < W) wait_flag(myflags + t * AR_NB + b, ep, deadline_ticks, err);
  __syncthreads();
  if (t == 0) s_fail = failed(err);
  __syncthreads();
  if (b == 0 && t == 0 && P.ticks != nullptr) {  // exposed all-reduce time of this rank (metrics)
    atomicAdd(P.ticks, __builtin_amdgcn_s_memrealtime() - t_in);
    atomicAdd(P.ticks + 1, 1ull);
  }
  if (!live || s_fail) return;
  // exactly W loads in flight at once (one per peer link), cache-bypassing, summed in rank order (rank_sum.h)
  const f32x4 s = rank_sum(W, [&](int q) {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(slab(P, q, par), (short)0, (int)(SLAB_FLOATS * 4), 0x00020000);
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * v, 0, SYS));
  });
  if (!sgd) {
    *(f32x4*)(sum_out + 4 * v) = s;
    return;
  }
  *(f32x4*)(cx.grads + 4 * v) = s;  // the all-reduced (summed) gradient, as after an RCCL all-reduce
  const int e0 = 4 * v;
  if (e0 >= OFF_RS) {  // CC4 segment (OFF_RS is float4 aligned): rank 0's running stats become the base
    *(f32x4*)(cx.rs_base + (e0 - OFF_RS)) = s;
    return;
  }
  f32x4 w = *(const f32x4*)(cx.params + e0);
  w -= cx.lr * s * cx.inv_ws;  // same rounding as k_apply_sgd (the RCCL path)
  *(f32x4*)(cx.params + e0) = w;
#pragma unroll
  for (int k = 0; k < 4; ++k) derive_param<BF>(cx, e0 + k, w[k]);
}

}  // namespace xg
}  // namespace dca
