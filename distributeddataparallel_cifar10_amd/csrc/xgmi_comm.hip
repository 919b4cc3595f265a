// Generic xGMI all-reduce for the flat gradient buckets of ANY model (FlatBucketDDP, ResNet-50/101, PPE).
//
// Replaces the reference's DDP Reducer bucket all-reduce (reference main.py:63, ppe_main_ddp.py:114; SURVEY.md
// 2.4 CC5, 5.8) inside one node.  The 8 MI355X of a node are fully connected by xGMI -- 7 point-to-point links per
// GPU, not a switch -- so a ring all-reduce is bound by ONE link per step.  Here every rank reads its peers'
// buffers directly, one link per peer, all links at once:
//   * one-shot: every rank reads the whole bucket from all W-1 peers and sums.  One flag round trip; (W-1)*S
//     bytes in per rank.  Wins for small buckets (latency-bound).
//   * two-shot: rank r reduces segment r (1/W of the bucket) from all peers (reduce-scatter by peer reads),
//     publishes it, then every rank reads every other segment from its owner (all-gather by peer reads).  Two
//     flag round trips; 2*(W-1)/W*S bytes in per rank, spread over all W-1 links: the direct-mesh bound
//     S/(W/2 * link) instead of the ring's 2(W-1)/W*S/link.
// Sums are taken in rank order 0..W-1 on every rank (one-shot) or once by the segment owner (two-shot), so every
// rank ends with bitwise-identical gradients.  The wire format is fp32 or bf16 (halves the link bytes; the sum is
// accumulated in fp32 and the final averaged value rounded once to bf16, identically on every rank).
//
// Shared region (one per rank, hipDeviceMallocUncached, exported with hipIpcGetMemHandle, mapped by every peer):
//   [in-flags  MAXR x NB_MAX ints][out-flags MAXR x NB_MAX ints]  (FLAG_BYTES)
//   [in slab parity 0][in slab parity 1][out slab parity 0][out slab parity 1]   (slab_bytes each)
// Element i of a bucket always sits at element i of a slab.
//
// Failing together: a workgroup that finds the error word set on entry returns at once (no publish, no wait, dst
// keeps the rank's own values); one whose wait expires does not sum.  The flag then stops advancing, so every
// peer's next wait for this rank expires too and all ranks report the error -- publishing ahead instead would let a
// slow peer pass its wait on a later call's slab and sum mixed calls without noticing.
// Protocol of workgroup b (the communicator launches exactly `nb` workgroups for every call, so every workgroup
// advances its epoch on every call and ep is uniform across the grid and across ranks):
//   1. ep = in_flags[me][b] + 1, parity = ep & 1
//   2. publish: copy piece b of the bucket (one-shot: piece b of the whole bucket; two-shot: piece b of EVERY
//      rank's segment) into my in slab[parity] with write-through stores; s_waitcnt vmcnt(0) + barrier
//   3. store ep into in_flags[me][b] of every rank; wait until my in_flags[q][b] >= ep for all q
//   4. one-shot: read piece b from all W in slabs (cache-bypassing), sum in rank order, scale, write dst -> done.
//      two-shot: read piece b of MY segment from all W in slabs, sum in rank order, scale, write it to dst and to
//      my out slab[parity] (write-through); vmcnt(0) + barrier; store ep into out_flags[me][b] of every rank;
//      wait until my out_flags[q][b] >= ep for all q; read piece b of segment q from rank q's out slab into dst.
//   Waits are bounded by s_memrealtime: on expiry bit 0 of *err is set and the workgroup stops (no hang; the host
//   raises when it reads the error word).
// Reuse safety (as csrc/xgmi_allreduce.hip): workgroup b writes a slab of parity p at call k only after it passed
// a wait of call k-1, i.e. after every peer STARTED call k-1, i.e. (stream order) after every peer finished call
// k-2 -- the last call that read parity p.  This holds whatever the bucket partition of each call is.
// In-place (src == dst) is safe: workgroup b only writes dst elements that it published itself in step 2.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rank_sum.h"

namespace dca {
namespace comm {

constexpr int MAXR = 8;      // ranks of one xGMI node
constexpr int T = 512;       // threads per workgroup (8 waves)
constexpr int NB_MAX = 1024;  // workgroups per call, upper bound
constexpr size_t FLAG_BYTES = 2 * MAXR * NB_MAX * 4;  // 64 KiB
constexpr int SYS = 17;      // cache policy sc0 | sc1: system coherent (write-through store, cache-bypassing load)
constexpr int RSRC_FLAGS = 0x00020000;

typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned u4 __attribute__((ext_vector_type(4)));
typedef unsigned u2 __attribute__((ext_vector_type(2)));

struct Args {
  char* base[MAXR];  // every rank's region mapped in this process (own one at base[me])
  const float* src;
  float* dst;
  long long n;       // elements of the bucket
  long long slab_bytes;
  unsigned* err;
  unsigned long long deadline;  // s_memrealtime ticks (100 MHz)
  float scale;       // applied to the sum (1/W for an average)
  int W, me, nb;
};

__device__ __forceinline__ int* in_flags(char* base) { return (int*)base; }
__device__ __forceinline__ int* out_flags(char* base) { return (int*)base + MAXR * NB_MAX; }
__device__ __forceinline__ char* in_slab(const Args& a, int q, int par) {
  return a.base[q] + FLAG_BYTES + (size_t)par * a.slab_bytes;
}
__device__ __forceinline__ char* out_slab(const Args& a, int q, int par) {
  return a.base[q] + FLAG_BYTES + (size_t)(2 + par) * a.slab_bytes;
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(char* p, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)bytes, RSRC_FLAGS);
}

__device__ __forceinline__ unsigned bf16_bits(float x) {  // round to nearest even; NaN stays NaN
  unsigned u = __builtin_bit_cast(unsigned, x);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (u >> 16) | 0x40u;
  return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}
__device__ __forceinline__ float bf16_float(unsigned h) { return __builtin_bit_cast(float, h << 16); }
__device__ __forceinline__ u2 pack_bf16(f4 v) {
  return u2{bf16_bits(v[0]) | (bf16_bits(v[1]) << 16), bf16_bits(v[2]) | (bf16_bits(v[3]) << 16)};
}
__device__ __forceinline__ f4 unpack_bf16(u2 w) {
  return f4{bf16_float(w[0] & 0xffffu), bf16_float(w[0] >> 16), bf16_float(w[1] & 0xffffu), bf16_float(w[1] >> 16)};
}
__device__ __forceinline__ f4 round_bf16(f4 v) { return unpack_bf16(pack_bf16(v)); }

// float4 v of the bucket (the last one may be partial: n % 4 != 0)
__device__ __forceinline__ f4 load_src(const float* s, long long v, long long n) {
  if (4 * v + 4 <= n) return *(const f4*)(s + 4 * v);
  f4 r = {0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < 4; ++k)
    if (4 * v + k < n) r[k] = s[4 * v + k];
  return r;
}
__device__ __forceinline__ void store_dst(float* d, long long v, long long n, f4 x) {
  if (4 * v + 4 <= n) {
    *(f4*)(d + 4 * v) = x;
    return;
  }
  for (int k = 0; k < 4; ++k)
    if (4 * v + k < n) d[4 * v + k] = x[k];
}

// slab traffic: element offset 4v, wire fp32 (16 B) or bf16 (8 B)
template <bool BF>
__device__ __forceinline__ void slab_put(__amdgpu_buffer_rsrc_t r, long long v, f4 x) {
  if (BF)
    __builtin_amdgcn_raw_buffer_store_b64(pack_bf16(x), r, (int)(8 * v), 0, SYS);
  else
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, x), r, (int)(16 * v), 0, SYS);
}
template <bool BF>
__device__ __forceinline__ f4 slab_get(__amdgpu_buffer_rsrc_t r, long long v) {
  if (BF) return unpack_bf16(__builtin_amdgcn_raw_buffer_load_b64(r, (int)(8 * v), 0, SYS));
  return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(16 * v), 0, SYS));
}

__device__ __forceinline__ bool err_set(const Args& a) {
  return __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
}
// Raise flag[me][b] = ep on every rank, then wait for flag[q][b] >= ep on all q (thread q polls rank q's flag in
// MY region).  Called by the whole workgroup after its slab stores; returns after a workgroup barrier, false
// (workgroup-uniform) when a wait of this rank expired: the slabs read next may hold other epochs.
__device__ __forceinline__ bool exchange(const Args& a, bool out, int ep, int* s_fail) {
  const int t = threadIdx.x, b = blockIdx.x;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's write-through slab stores are performed
  __syncthreads();                                    // ... and every thread's of this workgroup
  if (t < a.W) {
    int* f = (out ? out_flags(a.base[t]) : in_flags(a.base[t])) + a.me * NB_MAX + b;
    __hip_atomic_store(f, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const int* mine = (out ? out_flags(a.base[a.me]) : in_flags(a.base[a.me])) + t * NB_MAX + b;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while ((int)((unsigned)__hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - (unsigned)ep) < 0) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > a.deadline) {
        atomicOr(a.err, 1u);
        break;
      }
    }
  }
  __syncthreads();
  if (t == 0) *s_fail = err_set(a);
  __syncthreads();
  return !*s_fail;
}

// Sum float4 v over all W ranks' slabs (rank order), exactly W loads in flight at once (one per peer link).
template <bool BF>
__device__ __forceinline__ f4 gather_sum(const __amdgpu_buffer_rsrc_t* rs, int W, long long v) {
  return rank_sum(W, [&](int q) { return slab_get<BF>(rs[q], v); });
}
// Two-shot all-gather: element i of every other rank's piece b, exactly W - 1 peer loads in flight per thread.
template <bool BF, int NR>
__device__ __forceinline__ void allgather_n(const Args& a, const __amdgpu_buffer_rsrc_t* rout, const long long* lo,
                                            const long long* hi, long long len) {
  for (long long i = threadIdx.x; i < len; i += T) {
    f4 got[NR];
#pragma unroll
    for (int q = 0; q < NR; ++q) {
      const long long v = lo[q] + i < hi[q] ? lo[q] + i : lo[q];  // clamped: unconditional loads
      if (q != a.me) got[q] = slab_get<BF>(rout[q], v);
    }
#pragma unroll
    for (int q = 0; q < NR; ++q)
      if (q != a.me && lo[q] + i < hi[q]) store_dst(a.dst, lo[q] + i, a.n, got[q]);
  }
}

template <bool BF, bool TWO>
__global__ void __launch_bounds__(T) k_allreduce(Args a) {
  const int t = threadIdx.x, b = blockIdx.x, W = a.W, me = a.me;
  const long long nv = (a.n + 3) / 4;
  __shared__ int s_ep, s_fail;
  if (t == 0) {
    s_ep = __hip_atomic_load(in_flags(a.base[me]) + me * NB_MAX + b, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM) + 1u;  // wraps mod 2^32 (wrap-aware wait below)
    s_fail = err_set(a);
  }
  __syncthreads();
  if (s_fail) return;
  const int ep = s_ep, par = ep & 1;
  const long long wire = BF ? 2 : 4;
  const long long sb = (nv * 4) * wire;  // slab bytes in use
  __amdgpu_buffer_rsrc_t rin[MAXR];
#pragma unroll
  for (int q = 0; q < MAXR; ++q) rin[q] = rsrc(in_slab(a, q < W ? q : me, par), sb);  // q >= W: never read

  if (!TWO) {
    const long long piece = (nv + a.nb - 1) / a.nb, lo = b * piece, hi = lo + piece < nv ? lo + piece : nv;
    for (long long v = lo + t; v < hi; v += T) slab_put<BF>(rin[me], v, load_src(a.src, v, a.n));
    if (!exchange(a, false, ep, &s_fail)) return;
    for (long long v = lo + t; v < hi; v += T) {
      f4 s = gather_sum<BF>(rin, W, v) * a.scale;
      store_dst(a.dst, v, a.n, BF ? round_bf16(s) : s);
    }
    return;
  }
  // two-shot: segment q = [q*seg, min((q+1)*seg, nv)); piece b of a segment = [b*piece, (b+1)*piece) within it
  const long long seg = (nv + W - 1) / W, piece = (seg + a.nb - 1) / a.nb;
  auto range = [&](int q, long long& lo, long long& hi) {
    const long long s0 = q * seg, s1 = s0 + seg < nv ? s0 + seg : nv;
    lo = s0 + b * piece;
    hi = lo + piece < s1 ? lo + piece : s1;
  };
  for (int q = 0; q < W; ++q) {
    long long lo, hi;
    range(q, lo, hi);
    for (long long v = lo + t; v < hi; v += T) slab_put<BF>(rin[me], v, load_src(a.src, v, a.n));
  }
  if (!exchange(a, false, ep, &s_fail)) return;
  const __amdgpu_buffer_rsrc_t rmine = rsrc(out_slab(a, me, par), sb);
  {
    long long lo, hi;
    range(me, lo, hi);
    for (long long v = lo + t; v < hi; v += T) {
      f4 s = gather_sum<BF>(rin, W, v) * a.scale;
      if (BF) s = round_bf16(s);
      slab_put<BF>(rmine, v, s);
      store_dst(a.dst, v, a.n, s);
    }
  }
  if (!exchange(a, true, ep, &s_fail)) return;
  // all-gather: piece b of every other segment from its owner, W-1 loads in flight per thread
  __amdgpu_buffer_rsrc_t rout[MAXR];
  long long lo[MAXR], hi[MAXR], len = 0;
#pragma unroll
  for (int q = 0; q < MAXR; ++q) {
    rout[q] = rsrc(out_slab(a, q < W ? q : me, par), sb);  // q >= W: never read
    if (q < W) {
      range(q, lo[q], hi[q]);
      len = hi[q] - lo[q] > len ? hi[q] - lo[q] : len;
    } else {
      lo[q] = hi[q] = 0;
    }
  }
  switch (W) {  // wave-uniform: exactly the W - 1 peers are read
    case 1: break;
    case 2: allgather_n<BF, 2>(a, rout, lo, hi, len); break;
    case 3: allgather_n<BF, 3>(a, rout, lo, hi, len); break;
    case 4: allgather_n<BF, 4>(a, rout, lo, hi, len); break;
    case 5: allgather_n<BF, 5>(a, rout, lo, hi, len); break;
    case 6: allgather_n<BF, 6>(a, rout, lo, hi, len); break;
    case 7: allgather_n<BF, 7>(a, rout, lo, hi, len); break;
    default: allgather_n<BF, 8>(a, rout, lo, hi, len); break;
  }
}

}  // namespace comm
}  // namespace dca
