// Layer kernels of the ops layer (ops/): channels-last (NHWC) bf16 activations, fp32 statistics / parameters.
//
// Reference ops they implement: conv2d via im2col + MFMA GEMM (K1/K4/K19/K22: the GEMM is
// ops_gemm.hip), BatchNorm2d train forward/backward with the ReLU and residual add fused (K5-K7, K17, K18, K20),
// max_pool2d forward/backward (K3, K16), global average pool (ResNet family), cross-entropy forward+backward
// (K11, K12), SGD with momentum / weight decay over a flat buffer (K24), and the fp8 e4m3 quantisation used by
// the fp8 GEMM path (amax + scale computed on the device: no host sync).
//
// Every reduction has a fixed order (per-block partials, then one finalize): results are deterministic.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ops_gemm.hip"

namespace dca {
namespace ops {

typedef unsigned short bf16_t;

__device__ __forceinline__ float ld_bf(const bf16_t* p) { return bf2f(*p); }

// ---------------------------------------------------------------------------------------------------------
// im2col / col2im (NHWC).  Column index k = (kh * KW + kw) * C + c, rows = output pixels (n, oh, ow); columns
// k >= KH*KW*C up to the padded width Kp are zero.
// ---------------------------------------------------------------------------------------------------------
struct ConvGeom {
  int N, H, W, C;        // input
  int KH, KW, stride, pad;
  int Ho, Wo;            // output
  int K, Kp;             // K = KH*KW*C, Kp = padded column count (multiple of 8)
};

__device__ __forceinline__ void unpack8(uint4 u, float* f) {
  const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = __uint_as_float((w[j >> 1] >> ((j & 1) * 16)) << 16);
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  unsigned w[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) w[j] = (unsigned)f2bf_rne(f[2 * j]) | ((unsigned)f2bf_rne(f[2 * j + 1]) << 16);
  return uint4{w[0], w[1], w[2], w[3]};
}

__global__ void __launch_bounds__(256) k_im2col(const bf16_t* __restrict__ x, bf16_t* __restrict__ cols, ConvGeom g) {
  const int groups = g.Kp >> 3;  // 8 columns per thread
  const long total = (long)g.N * g.Ho * g.Wo * groups;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int kg = (int)(i % groups);
    const long row = i / groups;
    const int ow = (int)(row % g.Wo), oh = (int)((row / g.Wo) % g.Ho), n = (int)(row / ((long)g.Wo * g.Ho));
    const int k0 = kg * 8;
    uint4 out;
    if ((g.C & 7) == 0) {  // 8 consecutive k share (kh, kw): one 16-B load
      const int tap = k0 / g.C, c = k0 % g.C, kh = tap / g.KW, kw = tap % g.KW;
      const int h = oh * g.stride - g.pad + kh, w = ow * g.stride - g.pad + kw;
      const bool in = k0 < g.K && h >= 0 && h < g.H && w >= 0 && w < g.W;
      out = in ? *(const uint4*)(x + (((long)n * g.H + h) * g.W + w) * g.C + c) : uint4{0u, 0u, 0u, 0u};
    } else {
      unsigned wd[4] = {0u, 0u, 0u, 0u};
      for (int e = 0; e < 8; ++e) {
        const int k = k0 + e;
        if (k >= g.K) break;
        const int tap = k / g.C, c = k % g.C, kh = tap / g.KW, kw = tap % g.KW;
        const int h = oh * g.stride - g.pad + kh, w = ow * g.stride - g.pad + kw;
        if (h >= 0 && h < g.H && w >= 0 && w < g.W)
          wd[e >> 1] |= (unsigned)x[(((long)n * g.H + h) * g.W + w) * g.C + c] << ((e & 1) * 16);
      }
      out = uint4{wd[0], wd[1], wd[2], wd[3]};
    }
    *(uint4*)(cols + row * g.Kp + k0) = out;
  }
}

// dX[n,h,w,c] = sum over the (kh, kw) taps whose output pixel read (h, w): gather form, no atomics.
// C % 8 == 0: one thread per pixel and 8 channels (16-B loads / stores, fp32 sums); else one per element.
// accumulate: dx += (the other consumer's input gradient already in dx, fused instead of a separate add)
__global__ void __launch_bounds__(256) k_col2im(const bf16_t* __restrict__ dcols, bf16_t* __restrict__ dx, ConvGeom g,
                                                int accumulate) {
  const int vec = (g.C & 7) == 0 ? 8 : 1;
  const int cgs = g.C / vec;
  const long total = (long)g.N * g.H * g.W * cgs;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int c = (int)(i % cgs) * vec;
    const long pix = i / cgs;
    const int w = (int)(pix % g.W), h = (int)((pix / g.W) % g.H), n = (int)(pix / ((long)g.W * g.H));
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int kh = 0; kh < g.KH; ++kh) {
      const int th = h + g.pad - kh;
      if (th < 0 || th % g.stride) continue;
      const int oh = th / g.stride;
      if (oh >= g.Ho) continue;
      for (int kw = 0; kw < g.KW; ++kw) {
        const int tw = w + g.pad - kw;
        if (tw < 0 || tw % g.stride) continue;
        const int ow = tw / g.stride;
        if (ow >= g.Wo) continue;
        const long o = (((long)n * g.Ho + oh) * g.Wo + ow) * g.Kp + (kh * g.KW + kw) * g.C + c;
        if (vec == 8) {
          float d[8];
          unpack8(*(const uint4*)(dcols + o), d);
#pragma unroll
          for (int j = 0; j < 8; ++j) s[j] += d[j];
        } else {
          s[0] += ld_bf(dcols + o);
        }
      }
    }
    const long xo = pix * g.C + c;
    if (accumulate) {
      float o[8];
      if (vec == 8) unpack8(*(const uint4*)(dx + xo), o);
      else o[0] = ld_bf(dx + xo);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += o[j];
    }
    if (vec == 8) *(uint4*)(dx + xo) = pack8(s);
    else dx[xo] = f2bf_rne(s[0]);
  }
}

// ---------------------------------------------------------------------------------------------------------
// BatchNorm (training) over x[M][C] (M = N*H*W), fused with ReLU and a residual add.
//   res_mode 0: out = act(z)            1: out = act(z) + r  (NetResDeep: skip after the ReLU)
//   res_mode 2: out = act(z + r)        (ResNet bottleneck)            z = (x - mean) * invstd * gamma + beta
// Statistics: per-block partial sums of (x - shift) and (x - shift)^2 in fp32 (shift = running_mean, close to
// the batch mean: a single pass without cancellation trouble), then one finalize.
// ---------------------------------------------------------------------------------------------------------
constexpr int BN_ROWS = 256;  // rows per partial block (threads: 64 channel lanes x 4 row lanes)
constexpr int BN_U = 4;        // rows per thread with their loads in flight together (apply / backward kernels)

// 16-B activation loads / stores, optionally non-temporal (NT): the large BN passes stream tensors far bigger than
// the Infinity Cache, where keeping them out of the caches measured 8-20 % faster (bench/micro/bn_micro.hip); the
// smaller ones are re-read while still cache-resident and stay on the default policy
typedef unsigned bn_v4u __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ uint4 bn_ld16(const bf16_t* p) {
  if constexpr (NT) {
    const bn_v4u v = __builtin_nontemporal_load((const bn_v4u*)p);
    return uint4{v.x, v.y, v.z, v.w};
  } else {
    return *(const uint4*)p;
  }
}
template <bool NT>
__device__ __forceinline__ void bn_st16(bf16_t* p, uint4 v) {
  if constexpr (NT) __builtin_nontemporal_store(bn_v4u{v.x, v.y, v.z, v.w}, (bn_v4u*)p);
  else *(uint4*)p = v;
}
// How a BN backward recovers dz from dy (compile time, so each pass carries only its own loads and registers):
//   BWD_PLAIN no activation; BWD_RELU ReLU recomputed from x; BWD_RES ReLU(bn(x) + r) recomputed (reads r);
//   BWD_MASK the forward's stored ReLU bit mask.  BWD_RES / BWD_MASK (res_mode 2) also produce dr = dz.
enum { BWD_PLAIN = 0, BWD_RELU = 1, BWD_RES = 2, BWD_MASK = 3 };

// grid (ceil(C/64), ceil(M/BN_ROWS)); part[blockIdx.y][C] = (sum, sumsq)
__global__ void __launch_bounds__(256) k_bn_stats(const bf16_t* __restrict__ x, const float* __restrict__ shift,
                                                  float2* __restrict__ part, int M, int C) {
  __shared__ float2 red[4][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6, c = blockIdx.x * 64 + cl;
  const int r0 = blockIdx.y * BN_ROWS;
  float s = 0.f, q = 0.f;
  if (c < C) {
    const float k = shift[c];
    for (int r = r0 + rl; r < min(M, r0 + BN_ROWS); r += 4) {
      const float v = ld_bf(x + (long)r * C + c) - k;
      s += v;
      q += v * v;
    }
  }
  red[rl][cl] = float2{s, q};
  __syncthreads();
  if (rl == 0 && c < C) {
    float2 a = red[0][cl];
    for (int j = 1; j < 4; ++j) {
      a.x += red[j][cl].x;
      a.y += red[j][cl].y;
    }
    part[(long)blockIdx.y * C + c] = a;
  }
}

// Reduce the per-block partials of 16 channels per workgroup: 16 part-lanes x 16 channels, 8 loads in flight
// per thread, then a fixed-order LDS combine (deterministic).  Returns the (sum, sumsq) of channel c in lane 0..15.
// Sum of the per-tile partials of channel c.  A workgroup covers CW channels x (256 / CW) partial lanes: few
// channels per workgroup (narrow layers) keep enough workgroups and short serial loops -- the reduction is
// latency-bound (layer-1 BNs of ResNet-50 at batch 256: 6272 partials x 64 channels).  Tree combine in LDS.
// NTH threads per workgroup (256; 1024 for the one-channel-per-workgroup form, whose 64-128 workgroups otherwise
// walk thousands of partial rows in 3-4 dependent load rounds).
template <int CW, int NTH = 256>
__device__ __forceinline__ float2 reduce_parts(const float2* __restrict__ part, int nparts, int C, int c, float2* red) {
  constexpr int PL = NTH / CW;
  const int pl = threadIdx.x / CW, cl = threadIdx.x % CW;
  float sx = 0.f, sy = 0.f;
  if (c < C) {
    for (int p0 = pl; p0 < nparts; p0 += PL * 8) {
      float2 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int p = p0 + PL * u;
        v[u] = part[(long)min(p, nparts - 1) * C + c];  // clamped, unconditional: all 8 loads in flight
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const bool in = p0 + PL * u < nparts;
        sx += in ? v[u].x : 0.f;
        sy += in ? v[u].y : 0.f;
      }
    }
  }
  red[threadIdx.x] = float2{sx, sy};
  __syncthreads();
#pragma unroll
  for (int h = PL / 2; h > 0; h >>= 1) {
    if (pl < h) {
      const float2 o = red[threadIdx.x + h * CW];
      red[threadIdx.x].x += o.x;
      red[threadIdx.x].y += o.y;
    }
    __syncthreads();
  }
  return red[cl];
}

// channels per finalize workgroup for C channels (grid C / CW)
#define BN_FIN_DISPATCH(C, CALL) \
  do {                                 \
    if ((C) >= 2048) { CALL(16); }     \
    else if ((C) >= 1024) { CALL(8); } \
    else if ((C) >= 512) { CALL(4); }  \
    else if ((C) >= 256) { CALL(2); }  \
    else { CALL(1); }                  \
  } while (0)

template <int CW, int NTH = 256>
__global__ void __launch_bounds__(NTH) k_bn_finalize(const float2* __restrict__ part, int nparts, int M, int C,
                                                     float* __restrict__ running_mean, float* __restrict__ running_var,
                                                     float2* __restrict__ stats, float eps, float momentum) {
  __shared__ float2 red[NTH];
  const int c = blockIdx.x * CW + (threadIdx.x % CW);
  const float2 a = reduce_parts<CW, NTH>(part, nparts, C, c, red);
  if (threadIdx.x >= CW || c >= C) return;
  const float k = running_mean[c];
  const float dm = a.x / M;
  const float var = fmaxf(a.y / M - dm * dm, 0.f);
  const float mean = k + dm;
  stats[c] = float2{mean, rsqrtf(var + eps)};
  if (momentum > 0.f) {
    const float unb = M > 1 ? var * M / (M - 1) : var;
    running_mean[c] = (1.f - momentum) * k + momentum * mean;
    running_var[c] = (1.f - momentum) * running_var[c] + momentum * unb;
  }
}


// Inference (BatchNorm2d in eval mode): the running statistics are the normalisation statistics.
// stats[c] = (running_mean, rsqrt(running_var + eps)); grid ceil(C/256), 256 threads.
__global__ void __launch_bounds__(256) k_bn_eval_stats(const float* __restrict__ running_mean,
                                                       const float* __restrict__ running_var,
                                                       float2* __restrict__ stats, int C, float eps) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c < C) stats[c] = float2{running_mean[c], rsqrtf(running_var[c] + eps)};
}

// A residual that is itself a training BatchNorm output, applied on the fly (res_mode 2): r' = r * rsc + rsh per
// channel from its own batch statistics, so the ResNet downsample branch's BN never writes its output (the branch
// returns its conv output y and this pass reads that instead of the BN'd copy: one full pass over a 4x-width
// tensor per downsample block saved).  stats == nullptr: r is used as it is.
struct BnRes {
  const float2* stats;
  const float* gamma;
  const float* beta;
};

// out = fused(x); vectorised by 8 channels (C % 8 == 0)
// Optionally also emits an fp8 e4m3 copy of the output for an fp8 consumer GEMM, with DELAYED scaling: the scale
// 448 / amax comes from the previous step's amax of this tensor (amax_prev), and this step's amax is recorded in
// amax_out for the next step -- no extra pass over the activation, no host sync.
template <int CL, int ROWS = BN_ROWS, bool NT = false, bool RAFF = false>
__global__ void __launch_bounds__(256) k_bn_apply(const bf16_t* __restrict__ x, const bf16_t* __restrict__ r,
                                                  bf16_t* __restrict__ out, const float2* __restrict__ stats,
                                                  const float* __restrict__ gamma, const float* __restrict__ beta,
                                                  long M, int C, int relu, int res_mode, uint8_t* __restrict__ q,
                                                  const float* __restrict__ amax_prev, unsigned* __restrict__ amax_out,
                                                  uint8_t* __restrict__ mk, BnRes rb) {
  // grid (ceil(C/(8 CL)), ceil(M/ROWS)): CL channel groups of 8 x 256/CL row lanes, z = x * sc + sh per channel
  __shared__ float red[256];
  const int cgl = threadIdx.x % CL, rl = threadIdx.x / CL, c0 = blockIdx.x * (8 * CL) + cgl * 8;
  const long r0 = (long)blockIdx.y * ROWS;
  float qs = 1.f, amax = 0.f;
  if (q) qs = *amax_prev > 0.f ? 448.f / *amax_prev : 1.f;
  if (c0 < C) {
    float sc[8], sh[8], rsc[8], rsh[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float2 st = stats[c0 + j];
      sc[j] = st.y * gamma[c0 + j];
      sh[j] = beta[c0 + j] - st.x * sc[j];
      if constexpr (RAFF) {  // (its own instantiation: the plain passes keep their registers and schedule)
        const float2 rs = rb.stats[c0 + j];
        rsc[j] = rs.y * rb.gamma[c0 + j];
        rsh[j] = rb.beta[c0 + j] - rs.x * rsc[j];
      }
    }
    const long rend = M < r0 + ROWS ? M : r0 + ROWS;
    for (long base = r0 + rl; base < rend; base += (256 / CL) * BN_U) {
    uint4 X[BN_U], R[BN_U];
#pragma unroll
    for (int u = 0; u < BN_U; ++u) {  // all loads in flight first (clamped rows)
      const long rw = base + (256 / CL) * u, o = (rw < rend ? rw : rend - 1) * C + c0;
      X[u] = bn_ld16<NT>(x + o);
      if (res_mode) R[u] = bn_ld16<NT>(r + o);
    }
#pragma unroll
    for (int u = 0; u < BN_U; ++u) {
      const long row = base + (256 / CL) * u;
      if (row >= rend) break;
      const long o = row * C + c0;
      float v[8], rv[8];
      unpack8(X[u], v);
      if (res_mode) unpack8(R[u], rv);
      if constexpr (RAFF) {
#pragma unroll
        for (int j = 0; j < 8; ++j) rv[j] = rv[j] * rsc[j] + rsh[j];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float z = v[j] * sc[j] + sh[j];
        if (res_mode == 2) z += rv[j];
        if (relu) z = z > 0.f ? z : 0.f;
        if (res_mode == 1) z += rv[j];
        v[j] = z;
      }
      const uint4 ov = pack8(v);
      bn_st16<NT>(out + o, ov);
      if (mk) {  // ReLU mask, one bit per element (bit j: channel c0 + j), for the backward
        unsigned b = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) b |= (v[j] > 0.f ? 1u : 0u) << j;
        mk[o >> 3] = (uint8_t)b;
      }
      if (q) {
        float f[8];
        unpack8(ov, f);  // quantise the value as stored (bf16)
        int w[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          float c[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            amax = fmaxf(amax, fabsf(f[4 * h + j]));
            c[j] = fminf(fmaxf(f[4 * h + j] * qs, -448.f), 448.f);
          }
          w[h] = __builtin_amdgcn_cvt_pk_fp8_f32(c[0], c[1], 0, false);
          w[h] = __builtin_amdgcn_cvt_pk_fp8_f32(c[2], c[3], w[h], true);
        }
        *(uint2*)(q + o) = uint2{(unsigned)w[0], (unsigned)w[1]};
      }
    }
    }
  }
  if (q) {
    red[threadIdx.x] = amax;
    __syncthreads();
    for (int o = 128; o; o >>= 1) {
      if (threadIdx.x < o) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + o]);
      __syncthreads();
    }
    if (threadIdx.x == 0) atomicMax(amax_out, __float_as_uint(red[0]));
  }
}

// dz = dy * act'(.) recomputed from x (and r) -- or, when the forward stored it (BWD_MASK), the ReLU bit mask
// (1/16 of the bytes of r; exactly the forward's mask); partial sums of dz and dz * xhat per channel.
// grid (ceil(C/(8 CL)), ceil(M/BN_ROWS)); 256 threads = CL channel groups (8 channels, one 16-B load per tensor per
// row) x 256/CL row lanes; all rows' loads of a thread are independent (issued back to back).
template <int CL, int MODE, bool NT>
__global__ void __launch_bounds__(256) k_bn_bwd_stats(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                      const bf16_t* __restrict__ r, const float2* __restrict__ stats,
                                                      const float* __restrict__ gamma, const float* __restrict__ beta,
                                                      float2* __restrict__ part, int M, int C,
                                                      const uint8_t* __restrict__ mk) {
  __shared__ float2 red[256 / CL][8 * CL];
  const int cgl = threadIdx.x % CL, rl = threadIdx.x / CL, c0 = blockIdx.x * (8 * CL) + cgl * 8;
  const int r0 = blockIdx.y * BN_ROWS;
  float s[8], q[8], mu[8], is[8], ga[8], be[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = min(c0 + j, C - 1);
    s[j] = q[j] = 0.f;
    mu[j] = stats[c].x;
    is[j] = stats[c].y;
    ga[j] = gamma[c];
    be[j] = beta[c];
  }
  if (c0 < C) {
    const int rend = min(M, r0 + BN_ROWS);
    // BN_U rows per thread in flight: every load issued (clamped rows, unconditional) before any is used
    for (int base = r0 + rl; base < rend; base += (256 / CL) * BN_U) {
      uint4 X[BN_U], D[BN_U], R[BN_U];
      unsigned MB[BN_U];
#pragma unroll
      for (int u = 0; u < BN_U; ++u) {
        const long o = (long)min(base + (256 / CL) * u, rend - 1) * C + c0;
        X[u] = bn_ld16<NT>(x + o);
        D[u] = bn_ld16<NT>(dy + o);
        if constexpr (MODE == BWD_MASK) MB[u] = mk[o >> 3];
        if constexpr (MODE == BWD_RES) R[u] = bn_ld16<NT>(r + o);
      }
#pragma unroll
      for (int u = 0; u < BN_U; ++u) {
        if (base + (256 / CL) * u >= rend) break;
        float xv[8], dv[8], rv[8];
        unpack8(X[u], xv);
        unpack8(D[u], dv);
        if constexpr (MODE == BWD_RES) unpack8(R[u], rv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xh = (xv[j] - mu[j]) * is[j];
          float d = dv[j];
          if constexpr (MODE == BWD_MASK) {
            d = (MB[u] >> j) & 1u ? d : 0.f;
          } else if constexpr (MODE != BWD_PLAIN) {
            float z = xh * ga[j] + be[j];
            if constexpr (MODE == BWD_RES) z += rv[j];
            d = z > 0.f ? d : 0.f;
          }
          s[j] += d;
          q[j] = __builtin_fmaf(d, xh, q[j]);  // explicit: the same rounding in every MODE instantiation
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[rl][cgl * 8 + j] = float2{s[j], q[j]};
  __syncthreads();
  const int c = blockIdx.x * (8 * CL) + threadIdx.x;
  if (threadIdx.x < 8 * CL && c < C) {
    float2 a = red[0][threadIdx.x];
    for (int k = 1; k < 256 / CL; ++k) {
      a.x += red[k][threadIdx.x].x;
      a.y += red[k][threadIdx.x].y;
    }
    part[(long)blockIdx.y * C + c] = a;
  }
}

// dgamma = sum(dz * xhat), dbeta = sum(dz) (written, or added when accumulate: shared modules); sums for dx.
// grid ceil(C/16), 256 threads.
template <int CW, int NTH = 256>
__global__ void __launch_bounds__(NTH) k_bn_bwd_finalize(const float2* __restrict__ part, int nparts, int C,
                                                         float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                         float2* __restrict__ sums, int accumulate) {
  __shared__ float2 red[NTH];
  const int c = blockIdx.x * CW + (threadIdx.x % CW);
  const float2 a = reduce_parts<CW, NTH>(part, nparts, C, c, red);
  if (threadIdx.x >= CW || c >= C) return;
  sums[c] = a;
  dgamma[c] = accumulate ? dgamma[c] + a.y : a.y;
  dbeta[c] = accumulate ? dbeta[c] + a.x : a.x;
}

// BN partial rows reduced with coalesced reads and an agent ticket per 64-channel column block (replaces the
// per-channel k_bn_finalize / k_bn_bwd_finalize, which read one 8-byte word per lane from rows C x 8 bytes apart:
// 18.6 us for 6272 x 256 partials, 770 us per ResNet-50 step in all, profiles/rocprof_resnet50_r5u.txt).
// Grid (ceil(C / 64), gy), 256 threads = 64 channels x 4 row lanes: one load instruction reads 512 contiguous bytes
// of a partial row, 16 loads in flight per thread.  Workgroup (x, y) sums rows [y rpb, (y + 1) rpb) of channels
// 64 x .., stores the (sum, sumsq) write-through into row y rpb (already read by it; the partial rows are scratch)
// and takes column block x's ticket; the last of the gy workgroups sums the gy row sums in a fixed order (bitwise
// reproducible) and finishes: MODE 0 like k_bn_finalize (a0 / a1 = running mean / var, out = stats), MODE 1 like
// k_bn_bwd_finalize (a0 / a1 = dgamma / dbeta, out = sums).  ticket[gridDim.x] is zero at launch; the last
// workgroups reset it.
constexpr int BNT_U = 16;  // loads in flight per thread
__host__ __device__ inline int bn_fin_rpb(int nparts) {  // rows per workgroup: <= 128 row sums per column block
  const int unit = 4 * BNT_U;
  return unit * ((nparts + unit * 128 - 1) / (unit * 128));
}
template <int MODE>
__global__ void __launch_bounds__(256) k_bn_fin_ticket(float2* __restrict__ part, int nparts, int rpb, int M, int C,
                                                       float* __restrict__ a0, float* __restrict__ a1,
                                                       float2* __restrict__ out, float eps, float momentum,
                                                       int accumulate, unsigned* __restrict__ ticket) {
  __shared__ float2 red[256];
  __shared__ unsigned s_last;
  const int t = threadIdx.x, cl = t & 63, rl = t >> 6, c = blockIdx.x * 64 + cl;
  const int r0 = blockIdx.y * rpb, r1 = min(nparts, r0 + rpb);
  float sx = 0.f, sy = 0.f;
  if (c < C) {
    for (int p0 = r0 + rl; p0 < r1; p0 += 4 * BNT_U) {
      float2 v[BNT_U];
#pragma unroll
      for (int u = 0; u < BNT_U; ++u) v[u] = part[(long)min(p0 + 4 * u, r1 - 1) * C + c];  // clamped: all in flight
#pragma unroll
      for (int u = 0; u < BNT_U; ++u) {
        const bool in = p0 + 4 * u < r1;
        sx += in ? v[u].x : 0.f;
        sy += in ? v[u].y : 0.f;
      }
    }
  }
  red[t] = float2{sx, sy};
  __syncthreads();
  if (t < 64 && c < C) {
    float2 a = red[t];
#pragma unroll
    for (int j = 1; j < 4; ++j) {
      a.x += red[t + 64 * j].x;
      a.y += red[t + 64 * j].y;
    }
    float* dst = (float*)(part + (long)r0 * C + c);
    __hip_atomic_store(dst, a.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(dst + 1, a.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the write-through row sums are performed
  __syncthreads();
  if (t == 0)
    s_last = __hip_atomic_fetch_add(ticket + blockIdx.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
             gridDim.y - 1;
  __syncthreads();
  if (!s_last) return;
  // the last workgroup of this column block: 4 row lanes each sum a quarter of the row sums, combined in fixed order
  const int gy = gridDim.y, q = (gy + 3) >> 2, b0 = rl * q, b1 = min(gy, b0 + q);
  float ax = 0.f, ay = 0.f;
  if (c < C) {
    for (int b = b0; b < b1; b += BNT_U) {
      float vx[BNT_U], vy[BNT_U];
#pragma unroll
      for (int u = 0; u < BNT_U; ++u) {
        const float* s = (const float*)(part + (long)min(b + u, b1 - 1) * rpb * C + c);
        vx[u] = __hip_atomic_load(s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        vy[u] = __hip_atomic_load(s + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
#pragma unroll
      for (int u = 0; u < BNT_U; ++u) {
        const bool in = b + u < b1;
        ax += in ? vx[u] : 0.f;
        ay += in ? vy[u] : 0.f;
      }
    }
  }
  red[t] = float2{ax, ay};
  __syncthreads();
  if (t < 64 && c < C) {
    const float2 a{((red[t].x + red[t + 64].x) + red[t + 128].x) + red[t + 192].x,
                   ((red[t].y + red[t + 64].y) + red[t + 128].y) + red[t + 192].y};
    if constexpr (MODE == 0) {
      const float k = a0[c];
      const float dm = a.x / M;
      const float var = fmaxf(a.y / M - dm * dm, 0.f);
      const float mean = k + dm;
      out[c] = float2{mean, rsqrtf(var + eps)};
      if (momentum > 0.f) {
        const float unb = M > 1 ? var * M / (M - 1) : var;
        a0[c] = (1.f - momentum) * k + momentum * mean;
        a1[c] = (1.f - momentum) * a1[c] + momentum * unb;
      }
    } else {
      out[c] = a;
      a0[c] = accumulate ? a0[c] + a.y : a.y;
      a1[c] = accumulate ? a1[c] + a.x : a.x;
    }
  }
  if (t == 0) __hip_atomic_store(ticket + blockIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// dx = gamma * invstd * (dz - mean(dz) - xhat * mean(dz * xhat)); BWD_RES / BWD_MASK also write dr = dz.
// grid (ceil(C/(8 CL)), ceil(M/ROWS)): CL channel groups x 256/CL row lanes, per-channel coefficients folded once per
// thread (dx = A*dz + B*x + D), one 16-B load / store per tensor per row.
template <int CL, int MODE, int ROWS, bool NT>
__global__ void __launch_bounds__(256) k_bn_bwd_apply(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                      const bf16_t* __restrict__ r, const float2* __restrict__ stats,
                                                      const float* __restrict__ gamma, const float* __restrict__ beta,
                                                      const float2* __restrict__ sums, bf16_t* __restrict__ dx,
                                                      bf16_t* __restrict__ dr, long M, int C,
                                                      const uint8_t* __restrict__ mk) {
  const int cgl = threadIdx.x % CL, rl = threadIdx.x / CL, c0 = blockIdx.x * (8 * CL) + cgl * 8;
  if (c0 >= C) return;
  const long r0 = (long)blockIdx.y * ROWS;
  const float inv_m = 1.f / (float)M;
  float mu[8], is[8], ga[8], be[8], ca[8], cb[8], cd[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float2 st = stats[c0 + j], sm = sums[c0 + j];
    mu[j] = st.x;
    is[j] = st.y;
    ga[j] = gamma[c0 + j];
    be[j] = beta[c0 + j];
    // dx = g*is*(dz - sx/M - (x - mu)*is * sy/M) = ca*dz + cb*x + cd
    ca[j] = ga[j] * is[j];
    cb[j] = -ca[j] * is[j] * sm.y * inv_m;
    cd[j] = -ca[j] * sm.x * inv_m - cb[j] * mu[j];
  }
  const long rend = M < r0 + ROWS ? M : r0 + ROWS;
  for (long base = r0 + rl; base < rend; base += (256 / CL) * BN_U) {
    uint4 X[BN_U], D[BN_U], R[BN_U];
    unsigned MB[BN_U];
#pragma unroll
    for (int u = 0; u < BN_U; ++u) {  // all loads in flight first (clamped rows)
      const long row = base + (256 / CL) * u, o = (row < rend ? row : rend - 1) * C + c0;
      X[u] = bn_ld16<NT>(x + o);
      D[u] = bn_ld16<NT>(dy + o);
      if constexpr (MODE == BWD_MASK) MB[u] = mk[o >> 3];
      if constexpr (MODE == BWD_RES) R[u] = bn_ld16<NT>(r + o);
    }
#pragma unroll
    for (int u = 0; u < BN_U; ++u) {
      const long row = base + (256 / CL) * u;
      if (row >= rend) break;
      const long o = row * C + c0;
      float xv[8], d[8], rv[8];
      unpack8(X[u], xv);
      unpack8(D[u], d);
      if constexpr (MODE == BWD_RES) unpack8(R[u], rv);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float dz = d[j];
        if constexpr (MODE == BWD_MASK) {
          dz = (MB[u] >> j) & 1u ? dz : 0.f;
        } else if constexpr (MODE != BWD_PLAIN) {
          float z = (xv[j] - mu[j]) * is[j] * ga[j] + be[j];
          if constexpr (MODE == BWD_RES) z += rv[j];
          dz = z > 0.f ? dz : 0.f;
        }
        rv[j] = dz;
        // explicit FMAs: every MODE instantiation rounds alike (a select folded into a product can otherwise be
        // contracted differently, so BWD_MASK on dout and BWD_PLAIN on the written dout * mask differed in dx)
        d[j] = __builtin_fmaf(ca[j], dz, __builtin_fmaf(cb[j], xv[j], cd[j]));
      }
      bn_st16<NT>(dx + o, pack8(d));
      if constexpr (MODE == BWD_RES) bn_st16<NT>(dr + o, pack8(rv));
      if constexpr (MODE == BWD_MASK)
        if (dr) bn_st16<NT>(dr + o, pack8(rv));  // (none: the consumer takes dout and the mask instead)
    }
  }
}

// ---------------------------------------------------------------------------------------------------------
// Max pooling (NHWC, window KxK, stride S, padding P) with the argmax tap kept as a byte; backward gathers.
// ---------------------------------------------------------------------------------------------------------
struct PoolGeom {
  int N, H, W, C, K, S, P, Ho, Wo;
};

// C % 8 == 0: one thread per output pixel and 8 channels (16-B loads, 8-B argmax stores); else per element
// IT: index type.  unsigned (32-bit) when every element offset of x and y fits -- the per-thread index decode is
// then 32-bit division instead of the 64-bit division sequence, which made the ResNet-50 pools ALU-bound.
template <typename IT>
__global__ void __launch_bounds__(256) k_maxpool_fwd(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                     uint8_t* __restrict__ arg, PoolGeom g) {
  const int vec = (g.C & 7) == 0 ? 8 : 1;
  const IT cgs = (IT)(g.C / vec), Wo = (IT)g.Wo, Ho = (IT)g.Ho;
  const IT total = (IT)g.N * Ho * Wo * cgs;
  for (IT i = (IT)blockIdx.x * 256 + threadIdx.x; i < total; i += (IT)gridDim.x * 256) {
    const int c = (int)(i % cgs) * vec;
    const IT p = i / cgs, pr = p / Wo;
    const int ow = (int)(p - pr * Wo), oh = (int)(pr % Ho), n = (int)(pr / Ho);
    float best[8];
    int bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      best[j] = -INFINITY;
      bi[j] = 0;
    }
    for (int kh = 0; kh < g.K; ++kh) {
      const int h = oh * g.S - g.P + kh;
      if (h < 0 || h >= g.H) continue;
      for (int kw = 0; kw < g.K; ++kw) {
        const int w = ow * g.S - g.P + kw;
        if (w < 0 || w >= g.W) continue;
        const IT xo = (((IT)n * g.H + h) * g.W + w) * g.C + c;
        float v[8];
        if (vec == 8) unpack8(*(const uint4*)(x + xo), v);
        else v[0] = ld_bf(x + xo);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (j < vec && (v[j] > best[j] || (v[j] != v[j] && best[j] == best[j]))) {  // first max wins; NaN propagates
            best[j] = v[j];
            bi[j] = kh * g.K + kw;
          }
        }
      }
    }
    const IT o = p * g.C + c;
    if (vec == 8) {
      *(uint4*)(y + o) = pack8(best);
      *(uint2*)(arg + o) = uint2{(unsigned)bi[0] | ((unsigned)bi[1] << 8) | ((unsigned)bi[2] << 16) | ((unsigned)bi[3] << 24),
                                 (unsigned)bi[4] | ((unsigned)bi[5] << 8) | ((unsigned)bi[6] << 16) | ((unsigned)bi[7] << 24)};
    } else {
      y[o] = f2bf_rne(best[0]);
      arg[o] = (uint8_t)bi[0];
    }
  }
}

// 3x3 / stride 2 / pad 1 forward with H = 2 Ho, W = 2 Wo, C % 8 == 0: the generic kernel's runtime tap loops issue
// their 9 loads one after another (a memory latency each); here all 9 are unrolled and in flight together.  Only
// the top row / left column of a window can fall into the padding (H = 2 Ho): those taps load the window centre
// and are skipped in the compare, which runs in the same tap order (first max wins, NaN propagates).
// BN = true (the ResNet stem, k_bn_pool_fwd): x is the conv output y and every tap is first taken through the
// training BatchNorm + ReLU and rounded to bf16 exactly as k_bn_apply stores it, so pooled values and argmax bytes
// equal those of k_bn_apply followed by the plain pool -- without writing and re-reading the N x H x W x C
// activation (822 MB per ResNet-50 step at batch 256).
__device__ __forceinline__ float rbf16(float f) { return bf2f(f2bf_rne(f)); }
template <typename IT, bool BN>
__device__ __forceinline__ void maxpool_k3s2_fwd(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                 uint8_t* __restrict__ arg, const PoolGeom& g,
                                                 const float2* __restrict__ stats, const float* __restrict__ gamma,
                                                 const float* __restrict__ beta) {
  const IT cgs = (IT)(g.C >> 3), Wo = (IT)g.Wo, Ho = (IT)g.Ho;
  const IT total = (IT)g.N * Ho * Wo * cgs;
  for (IT i = (IT)blockIdx.x * 256 + threadIdx.x; i < total; i += (IT)gridDim.x * 256) {
    const int c = (int)(i % cgs) * 8;
    const IT p = i / cgs, pr = p / Wo;
    const int ow = (int)(p - pr * Wo), oh = (int)(pr % Ho), n = (int)(pr / Ho);
    const IT ctr = (((IT)n * g.H + 2 * oh) * g.W + 2 * ow) * g.C + c;  // window centre (always in range)
    const IT rs = (IT)g.W * g.C;
    const bool top = oh > 0, left = ow > 0;
    uint4 u[9];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const bool ok = (kh > 0 || top) && (kw > 0 || left);
        const IT o = ok ? ctr + (IT)(kh * rs) - rs + (IT)(kw * g.C) - (IT)g.C : ctr;
        u[kh * 3 + kw] = *(const uint4*)(x + o);
      }
    float sc[8], sh[8];
    if constexpr (BN) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {  // k_bn_apply's per-channel coefficients
        const float2 st = stats[c + j];
        sc[j] = st.y * gamma[c + j];
        sh[j] = beta[c + j] - st.x * sc[j];
      }
    }
    float best[8];
    int bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      best[j] = -INFINITY;
      bi[j] = 0;
    }
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      if (!((t >= 3 || top) && (t % 3 > 0 || left))) continue;
      float v[8];
      unpack8(u[t], v);
      if constexpr (BN) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float z = v[j] * sc[j] + sh[j];
          z = z > 0.f ? z : 0.f;
          v[j] = rbf16(z);
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (v[j] > best[j] || (v[j] != v[j] && best[j] == best[j])) {
          best[j] = v[j];
          bi[j] = t;
        }
    }
    const IT o = p * g.C + c;
    *(uint4*)(y + o) = pack8(best);
    *(uint2*)(arg + o) = uint2{(unsigned)bi[0] | ((unsigned)bi[1] << 8) | ((unsigned)bi[2] << 16) | ((unsigned)bi[3] << 24),
                               (unsigned)bi[4] | ((unsigned)bi[5] << 8) | ((unsigned)bi[6] << 16) | ((unsigned)bi[7] << 24)};
  }
}
template <typename IT>
__global__ void __launch_bounds__(256) k_maxpool_fwd_k3s2(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                          uint8_t* __restrict__ arg, PoolGeom g) {
  maxpool_k3s2_fwd<IT, false>(x, y, arg, g, nullptr, nullptr, nullptr);
}
template <typename IT>
__global__ void __launch_bounds__(256) k_bn_pool_fwd(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                     uint8_t* __restrict__ arg, PoolGeom g,
                                                     const float2* __restrict__ stats, const float* __restrict__ gamma,
                                                     const float* __restrict__ beta) {
  maxpool_k3s2_fwd<IT, true>(x, y, arg, g, stats, gamma, beta);
}

// 3x3 / stride 2 / pad 1 backward with H = 2 Ho, W = 2 Wo, C % 8 == 0 (the ResNet stem pool): output pixel
// (n, oh, ow) and 8 channels own the 2x2 input block (2oh..2oh+1, 2ow..2ow+1).  Even input rows/cols are reached
// only by the centre tap of their own output; odd ones also by the next output's first tap.  Every dy / argmax
// record is loaded once per thread (4 loads -> 4 blocks, instead of 2.25 loads per store in the input-driven
// kernel).  Sums are taken in ascending tap order, as in k_maxpool_bwd.  e[k][j]: input pixel k = 2 a + b of the
// block (row offset a, column offset b), channel c + j, in fp32 (the pool backward rounds them to bf16).
template <typename IT>
__device__ __forceinline__ void maxpool_k3s2_block_grad(const bf16_t* __restrict__ dy,
                                                        const uint8_t* __restrict__ arg, const PoolGeom& g, IT p,
                                                        int c, int oh, int ow, float (&e)[4][8]) {
  const bool hr = oh + 1 < g.Ho, hc = ow + 1 < g.Wo;
  // records (oh, ow), (oh, ow+1), (oh+1, ow), (oh+1, ow+1); missing neighbours read the own record with an
  // impossible tap (255) so all loads are unconditional
  const IT o00 = p * g.C + c;
  const IT o01 = hc ? o00 + g.C : o00;
  const IT o10 = hr ? o00 + (IT)g.Wo * g.C : o00;
  const IT o11 = hr && hc ? o00 + ((IT)g.Wo + 1) * g.C : o00;
  float d00[8], d01[8], d10[8], d11[8];
  unpack8(*(const uint4*)(dy + o00), d00);
  unpack8(*(const uint4*)(dy + o01), d01);
  unpack8(*(const uint4*)(dy + o10), d10);
  unpack8(*(const uint4*)(dy + o11), d11);
  const uint2 a00 = *(const uint2*)(arg + o00), a01 = *(const uint2*)(arg + o01);
  const uint2 a10 = *(const uint2*)(arg + o10), a11 = *(const uint2*)(arg + o11);
  const unsigned m01 = hc ? 0u : 0xffu, m10 = hr ? 0u : 0xffu, m11 = hr && hc ? 0u : 0xffu;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int sh = (j & 3) * 8;
    const unsigned t00 = ((j < 4 ? a00.x : a00.y) >> sh) & 0xffu;
    const unsigned t01 = (((j < 4 ? a01.x : a01.y) >> sh) & 0xffu) | m01;
    const unsigned t10 = (((j < 4 ? a10.x : a10.y) >> sh) & 0xffu) | m10;
    const unsigned t11 = (((j < 4 ? a11.x : a11.y) >> sh) & 0xffu) | m11;
    e[0][j] = t00 == 4u ? d00[j] : 0.f;
    float s = 0.f;
    s += t01 == 3u ? d01[j] : 0.f;
    s += t00 == 5u ? d00[j] : 0.f;
    e[1][j] = s;
    s = 0.f;
    s += t10 == 1u ? d10[j] : 0.f;
    s += t00 == 7u ? d00[j] : 0.f;
    e[2][j] = s;
    s = 0.f;
    s += t11 == 0u ? d11[j] : 0.f;
    s += t10 == 2u ? d10[j] : 0.f;
    s += t01 == 6u ? d01[j] : 0.f;
    s += t00 == 8u ? d00[j] : 0.f;
    e[3][j] = s;
  }
}
template <typename IT>
__global__ void __launch_bounds__(256) k_maxpool_bwd_k3s2(const bf16_t* __restrict__ dy,
                                                          const uint8_t* __restrict__ arg, bf16_t* __restrict__ dx,
                                                          PoolGeom g) {
  const IT cgs = (IT)(g.C >> 3), Wo = (IT)g.Wo, Ho = (IT)g.Ho;
  const IT total = (IT)g.N * Ho * Wo * cgs;
  for (IT i = (IT)blockIdx.x * 256 + threadIdx.x; i < total; i += (IT)gridDim.x * 256) {
    const int c = (int)(i % cgs) * 8;
    const IT p = i / cgs, pr = p / Wo;
    const int ow = (int)(p - pr * Wo), oh = (int)(pr % Ho), n = (int)(pr / Ho);
    float e[4][8];
    maxpool_k3s2_block_grad<IT>(dy, arg, g, p, c, oh, ow, e);
    const IT x00 = (((IT)n * g.H + 2 * oh) * g.W + 2 * ow) * g.C + c;
    const IT xr = (IT)g.W * g.C;
    *(uint4*)(dx + x00) = pack8(e[0]);
    *(uint4*)(dx + x00 + g.C) = pack8(e[1]);
    *(uint4*)(dx + x00 + xr) = pack8(e[2]);
    *(uint4*)(dx + x00 + xr + g.C) = pack8(e[3]);
  }
}

// The stem's BN backward through the fused pool (k_bn_pool_fwd): dz of an input pixel is the pool backward's value
// (maxpool_k3s2_block_grad, rounded to bf16 as k_maxpool_bwd_k3s2 stores it) times the ReLU mask recomputed from
// y, as BWD_RELU does -- so neither dz nor the post-ReLU activation is ever written (the unfused backward wrote dz
// and read it twice: 1.1 GB per ResNet-50 step at batch 256).
// Statistics: grid (C / 64, ceil(Npo / 64)) over the Npo output pixels, 256 threads = 8 channel groups x 32 pixel
// lanes x 2 output pixels; part[blockIdx.y][C] = (sum dz, sum dz * xhat) of the block's 256 input pixels.
constexpr int BNP_OPB = 64;  // output pixels per statistics workgroup
template <typename IT>
__global__ void __launch_bounds__(256) k_bn_pool_bwd_stats(const bf16_t* __restrict__ dp, const uint8_t* __restrict__ arg,
                                                           const bf16_t* __restrict__ x, const float2* __restrict__ stats,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, float2* __restrict__ part,
                                                           PoolGeom g) {
  __shared__ float2 red[32][64];
  const int cgl = threadIdx.x & 7, pl = threadIdx.x >> 3, c = blockIdx.x * 64 + cgl * 8;
  const IT npo = (IT)g.N * g.Ho * g.Wo;
  float s[8], q[8], mu[8], is[8], ga[8], be[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    s[j] = q[j] = 0.f;
    mu[j] = stats[c + j].x;
    is[j] = stats[c + j].y;
    ga[j] = gamma[c + j];
    be[j] = beta[c + j];
  }
#pragma unroll
  for (int u = 0; u < BNP_OPB / 32; ++u) {
    const IT p = (IT)blockIdx.y * BNP_OPB + pl + 32 * u;
    if (p >= npo) break;
    const IT pr = p / (IT)g.Wo;
    const int ow = (int)(p - pr * (IT)g.Wo), oh = (int)(pr % (IT)g.Ho), n = (int)(pr / (IT)g.Ho);
    const IT x00 = (((IT)n * g.H + 2 * oh) * g.W + 2 * ow) * g.C + c, xr = (IT)g.W * g.C;
    const uint4 X[4] = {*(const uint4*)(x + x00), *(const uint4*)(x + x00 + g.C), *(const uint4*)(x + x00 + xr),
                        *(const uint4*)(x + x00 + xr + g.C)};
    float e[4][8];
    maxpool_k3s2_block_grad<IT>(dp, arg, g, p, c, oh, ow, e);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float xv[8];
      unpack8(X[k], xv);
#pragma unroll
      for (int j = 0; j < 8; ++j) {  // k_bn_bwd_stats<.., BWD_RELU, ..>'s arithmetic on the stored dz
        const float xh = (xv[j] - mu[j]) * is[j];
        float d = rbf16(e[k][j]);
        const float z = xh * ga[j] + be[j];
        d = z > 0.f ? d : 0.f;
        s[j] += d;
        q[j] = __builtin_fmaf(d, xh, q[j]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[pl][cgl * 8 + j] = float2{s[j], q[j]};
  __syncthreads();
  if (threadIdx.x < 64) {
    float2 a = red[0][threadIdx.x];
    for (int k = 1; k < 32; ++k) {
      a.x += red[k][threadIdx.x].x;
      a.y += red[k][threadIdx.x].y;
    }
    part[(long)blockIdx.y * g.C + blockIdx.x * 64 + threadIdx.x] = a;
  }
}
// dx = gamma * invstd * (dz - mean(dz) - xhat * mean(dz * xhat)) over the 2x2 input block of every output pixel
// (k_bn_bwd_apply's coefficients and FMAs); M = N H W input pixels.
template <typename IT>
__global__ void __launch_bounds__(256) k_bn_pool_bwd_apply(const bf16_t* __restrict__ dp, const uint8_t* __restrict__ arg,
                                                           const bf16_t* __restrict__ x, const float2* __restrict__ stats,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta,
                                                           const float2* __restrict__ sums, bf16_t* __restrict__ dx,
                                                           PoolGeom g) {
  const IT cgs = (IT)(g.C >> 3), Wo = (IT)g.Wo, Ho = (IT)g.Ho;
  const IT total = (IT)g.N * Ho * Wo * cgs;
  const float inv_m = 1.f / (float)((long)g.N * g.H * g.W);
  for (IT i = (IT)blockIdx.x * 256 + threadIdx.x; i < total; i += (IT)gridDim.x * 256) {
    const int c = (int)(i % cgs) * 8;
    const IT p = i / cgs, pr = p / Wo;
    const int ow = (int)(p - pr * Wo), oh = (int)(pr % Ho), n = (int)(pr / Ho);
    const IT x00 = (((IT)n * g.H + 2 * oh) * g.W + 2 * ow) * g.C + c, xr = (IT)g.W * g.C;
    const IT xo[4] = {x00, x00 + g.C, x00 + xr, x00 + xr + g.C};
    uint4 X[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) X[k] = *(const uint4*)(x + xo[k]);
    float e[4][8];
    maxpool_k3s2_block_grad<IT>(dp, arg, g, p, c, oh, ow, e);
    float mu[8], is[8], ga[8], be[8], ca[8], cb[8], cd[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float2 st = stats[c + j], sm = sums[c + j];
      mu[j] = st.x;
      is[j] = st.y;
      ga[j] = gamma[c + j];
      be[j] = beta[c + j];
      ca[j] = ga[j] * is[j];
      cb[j] = -ca[j] * is[j] * sm.y * inv_m;
      cd[j] = -ca[j] * sm.x * inv_m - cb[j] * mu[j];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float xv[8], d[8];
      unpack8(X[k], xv);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float dz = rbf16(e[k][j]);
        const float z = (xv[j] - mu[j]) * is[j] * ga[j] + be[j];
        dz = z > 0.f ? dz : 0.f;
        d[j] = __builtin_fmaf(ca[j], dz, __builtin_fmaf(cb[j], xv[j], cd[j]));
      }
      *(uint4*)(dx + xo[k]) = pack8(d);
    }
  }
}

// one thread per input pixel and 8 channels (C % 8 == 0: 16-B dy loads, 8-B argmax loads), else per element
template <typename IT>
__global__ void __launch_bounds__(256) k_maxpool_bwd(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ arg,
                                                     bf16_t* __restrict__ dx, PoolGeom g) {
  const int vec = (g.C & 7) == 0 ? 8 : 1;
  const IT cgs = (IT)(g.C / vec), W = (IT)g.W, H = (IT)g.H;
  const IT total = (IT)g.N * H * W * cgs;
  for (IT i = (IT)blockIdx.x * 256 + threadIdx.x; i < total; i += (IT)gridDim.x * 256) {
    const int c = (int)(i % cgs) * vec;
    const IT p = i / cgs, pr = p / W;
    const int w = (int)(p - pr * W), h = (int)(pr % H), n = (int)(pr / H);
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int kh = 0; kh < g.K; ++kh) {
      const int th = h + g.P - kh;
      if (th < 0 || th % g.S) continue;
      const int oh = th / g.S;
      if (oh >= g.Ho) continue;
      for (int kw = 0; kw < g.K; ++kw) {
        const int tw = w + g.P - kw;
        if (tw < 0 || tw % g.S) continue;
        const int ow = tw / g.S;
        if (ow >= g.Wo) continue;
        const IT o = (((IT)n * g.Ho + oh) * g.Wo + ow) * g.C + c;
        const int tap = kh * g.K + kw;
        if (vec == 8) {
          float d[8];
          unpack8(*(const uint4*)(dy + o), d);
          const uint2 a = *(const uint2*)(arg + o);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const unsigned aj = ((j < 4 ? a.x : a.y) >> ((j & 3) * 8)) & 0xffu;
            s[j] += aj == (unsigned)tap ? d[j] : 0.f;
          }
        } else if (arg[o] == tap) {
          s[0] += ld_bf(dy + o);
        }
      }
    }
    const IT xo = p * g.C + c;
    if (vec == 8) *(uint4*)(dx + xo) = pack8(s);
    else dx[xo] = f2bf_rne(s[0]);
  }
}

// global average pool [N][HW][C] -> [N][C] (fp32 out) and its backward (broadcast / HW, bf16 out)
// TO: float (fp32 features) or bf16_t (the bf16 operand of the following fc GEMM, no separate cast pass)
template <typename TO>
__global__ void __launch_bounds__(256) k_avgpool_fwd(const bf16_t* __restrict__ x, TO* __restrict__ y, int N,
                                                     int HW, int C) {
  const int c = blockIdx.x * 256 + threadIdx.x, n = blockIdx.y;
  if (c >= C) return;
  float s = 0.f;
  for (int p = 0; p < HW; ++p) s += ld_bf(x + ((long)n * HW + p) * C + c);
  if constexpr (sizeof(TO) == 2) y[(long)n * C + c] = f2bf_rne(s / HW);
  else y[(long)n * C + c] = s / HW;
}
// C % 8 == 0: one thread per pixel and 8 channels (dy: two 16-B fp32 loads or one 16-B bf16 load, one 16-B store),
// 32-bit index decode
template <typename TD>
__global__ void __launch_bounds__(256) k_avgpool_bwd8(const TD* __restrict__ dy, bf16_t* __restrict__ dx, int N,
                                                      int HW, int C) {
  const unsigned cg = (unsigned)C >> 3, per_n = (unsigned)HW * cg, total = (unsigned)N * per_n;
  const float hw = (float)HW;
  for (unsigned i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
    const unsigned n = i / per_n, c = (i % cg) * 8u;
    float v[8];
    if constexpr (sizeof(TD) == 2) {
      unpack8(*(const uint4*)(dy + n * (unsigned)C + c), v);
    } else {
      const f32x4 a = *(const f32x4*)(dy + n * (unsigned)C + c), b = *(const f32x4*)(dy + n * (unsigned)C + c + 4);
      for (int j = 0; j < 4; ++j) {
        v[j] = a[j];
        v[4 + j] = b[j];
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] /= hw;
    *(uint4*)(dx + 8ul * i) = pack8(v);
  }
}
__global__ void __launch_bounds__(256) k_avgpool_bwd(const float* __restrict__ dy, bf16_t* __restrict__ dx, int N,
                                                     int HW, int C) {
  const long total = (long)N * HW * C;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int c = (int)(i % C);
    const long n = i / ((long)HW * C);
    dx[i] = f2bf_rne(dy[n * C + c] / HW);
  }
}

// ---------------------------------------------------------------------------------------------------------
// Cross-entropy (mean over the batch): per-row loss and dlogits = (softmax - onehot) / B.  One wave per row.
// ---------------------------------------------------------------------------------------------------------
// loss_mean (optional): the batch mean of the row losses, computed by the last row's workgroup to finish (agent-scope
// ticket; the rows' losses are stored write-through and read back with sc1 loads -- the guide's in-launch
// reduction), summed in a fixed order (bitwise reproducible), so the mean needs no separate reduction kernel.
// *ticket must be 0 at launch; the last workgroup resets it.
__global__ void __launch_bounds__(64) k_cross_entropy(const float* __restrict__ logits, const long* __restrict__ labels,
                                                      float* __restrict__ loss, float* __restrict__ dlogits, int B,
                                                      int K, float grad_scale, float* __restrict__ loss_mean,
                                                      unsigned* __restrict__ ticket) {
  const int b = blockIdx.x, l = threadIdx.x;
  const float* row = logits + (long)b * K;
  float m = -INFINITY;
  for (int k = l; k < K; k += 64) m = fmaxf(m, row[k]);
  for (int o = 32; o; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  float s = 0.f;
  for (int k = l; k < K; k += 64) s += __expf(row[k] - m);
  for (int o = 32; o; o >>= 1) s += __shfl_xor(s, o);
  long y = labels[b];
  y = y < 0 ? 0 : (y >= K ? K - 1 : y);
  const float lse = m + __logf(s);
  if (l == 0) __hip_atomic_store(loss + b, lse - row[y], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (dlogits) {
    const float inv = 1.f / s;
    for (int k = l; k < K; k += 64)
      dlogits[(long)b * K + k] = (__expf(row[k] - m) * inv - (k == y ? 1.f : 0.f)) * grad_scale;
  }
  if (loss_mean == nullptr) return;
  __shared__ unsigned s_last;
  if (l == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the write-through loss store is performed
    s_last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(B - 1);
  }
  __syncthreads();
  if (!s_last) return;
  float a = 0.f;
  for (int r = l; r < B; r += 64) a += __hip_atomic_load(loss + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (int o = 32; o; o >>= 1) a += __shfl_xor(a, o);
  if (l == 0) {
    *loss_mean = a / (float)B;
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// out[i] = x[i] * s[0] (s: a device scalar, e.g. the incoming gradient of a loss)
__global__ void __launch_bounds__(256) k_scale_dev(const float* __restrict__ x, const float* __restrict__ sp,
                                                  float* __restrict__ out, long n) {
  const float sc = *sp;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) out[i] = x[i] * sc;
}

__global__ void __launch_bounds__(256) k_cast_bf16(const float* __restrict__ x, bf16_t* __restrict__ y, long n) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) y[i] = f2bf_rne(x[i]);
}

// out[r * L + j] (+)= src[r * S + idx[j]] (fp32; e.g. the space-to-depth stem's weight gradient remapped to torch's
// layout, accumulated into the flat DDP gradient view)
__global__ void __launch_bounds__(256) k_gather_cols(const float* __restrict__ src, int S, const long* __restrict__ idx,
                                                    int L, float* __restrict__ out, int rows, int accumulate) {
  const long total = (long)rows * L;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long r = i / L, j = i % L;
    const float v = src[r * S + idx[j]];
    out[i] = accumulate ? out[i] + v : v;
  }
}

// *ptrs[i] += 1 for i < n (BatchNorm num_batches_tracked of every BN of a model: one launch per step)
__global__ void __launch_bounds__(64) k_add_i64(long long* const* __restrict__ ptrs, int n) {
  for (int i = threadIdx.x; i < n; i += 64) *ptrs[i] += 1;
}

// Preamble of a GEMM layer's backward: dy [R][N] (fp32 or bf16) with an optional ReLU mask (y > 0, y [R][N] bf16 or
// fp32) -> dyb [R][N] bf16 (the GEMMs' operand; optional) and db [N] fp32 = the column sums (the bias gradient).
// 2-D grid: blockIdx.x = a 64-column block (one wave-wide coalesced row segment), blockIdx.y = a chunk of rpb rows;
// the 256 threads are 64 columns x 4 row lanes.  Each block writes its 64 column partials write-through; the last
// block of a column block to finish (that column block's agent ticket) sums the gridDim.y partials in chunk order --
// one launch, bitwise reproducible, enough workgroups to fill the chip.  ticket[gridDim.x] is zero at launch and
// reset by the last blocks.
template <typename TD, typename TY>
__global__ void __launch_bounds__(256) k_dy_prep(const TD* __restrict__ dy, const TY* __restrict__ y,
                                                bf16_t* __restrict__ dyb, float* __restrict__ part,
                                                float* __restrict__ db, unsigned* __restrict__ ticket, int R, int N,
                                                int rpb, int accumulate) {
  __shared__ float red[256];
  __shared__ unsigned s_last;
  const int t = threadIdx.x, cl = t & 63, rlane = t >> 6;
  const int c = blockIdx.x * 64 + cl;
  const long r0 = (long)blockIdx.y * rpb, r1 = r0 + rpb < R ? r0 + rpb : R;
  float acc = 0.f;
  if (c < N) {
#pragma unroll 4
    for (long r = r0 + rlane; r < r1; r += 4) {
      float v;
      if constexpr (sizeof(TD) == 2) v = bf2f(dy[r * N + c]);
      else v = dy[r * N + c];
      if (y != nullptr) {
        float yv;
        if constexpr (sizeof(TY) == 2) yv = bf2f(y[r * N + c]);
        else yv = y[r * N + c];
        v = yv > 0.f ? v : 0.f;
      }
      if (dyb != nullptr) dyb[r * N + c] = f2bf_rne(v);
      acc += v;
    }
  }
  red[t] = acc;
  __syncthreads();
  if (t < 64 && c < N)
    __hip_atomic_store(part + (long)blockIdx.y * N + c, red[t] + red[t + 64] + red[t + 128] + red[t + 192],
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0)
    s_last = __hip_atomic_fetch_add(ticket + blockIdx.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
             gridDim.y - 1;
  __syncthreads();
  if (!s_last) return;
  // last block of this column block: 4 lanes per column each sum a quarter of the chunks, combined in fixed order
  const int gy = gridDim.y, q = (gy + 3) >> 2, b0 = rlane * q, b1 = b0 + q < gy ? b0 + q : gy;
  float a = 0.f;
  if (c < N) {
#pragma unroll 8
    for (int b = b0; b < b1; ++b) a += __hip_atomic_load(part + (long)b * N + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  red[t] = a;
  __syncthreads();
  if (t < 64 && c < N) {
    const float s = ((red[t] + red[t + 64]) + red[t + 128]) + red[t + 192];
    db[c] = accumulate ? db[c] + s : s;  // accumulate: straight into a flat DDP gradient view (grad sink)
  }
  if (t == 0) __hip_atomic_store(ticket + blockIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------------------------------------------------
// SGD over a flat fp32 buffer, torch.optim.SGD semantics: d = g + wd*p; buf = first ? d : mu*buf + d; p -= lr*buf
// (mu == 0: no buffer).  `first` is a device flag (the step counter lives on the device: no host sync).
// ---------------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_sgd(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ buf,
                                             long n, float lr, float mu, float wd, int* __restrict__ first) {
  const bool init = first ? *first != 0 : false;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    float d = g[i];
    if (wd != 0.f) d += wd * p[i];
    if (mu != 0.f) {
      d = init ? d : mu * buf[i] + d;
      buf[i] = d;
    }
    p[i] -= lr * d;
  }
}
__global__ void k_clear_flag(int* f) { *f = 0; }

// ---------------------------------------------------------------------------------------------------------
// fp8 e4m3 (OCP) quantisation with a per-tensor scale computed on the device:
//   amax = max |x|  (k_amax: per-block max, then atomicMax on the float bits -- non-negative floats order as
//   unsigned ints);  q = sat(x * 448 / amax);  the GEMM multiplies by amax / 448 (inv scale) in its epilogue.
// ---------------------------------------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ float ld_any(const T* p, long i);
template <> __device__ __forceinline__ float ld_any<float>(const float* p, long i) { return p[i]; }
template <> __device__ __forceinline__ float ld_any<bf16_t>(const bf16_t* p, long i) { return bf2f(p[i]); }

template <typename T>
__global__ void __launch_bounds__(256) k_amax(const T* __restrict__ x, long n, unsigned* __restrict__ amax_bits) {
  __shared__ float red[256];
  float m = 0.f;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) m = fmaxf(m, fabsf(ld_any(x, i)));
  red[threadIdx.x] = m;
  __syncthreads();
  for (int o = 128; o; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + o]);
    __syncthreads();
  }
  if (threadIdx.x == 0) atomicMax(amax_bits, __float_as_uint(red[0]));
}

template <typename T>
__global__ void __launch_bounds__(256) k_quant_fp8(const T* __restrict__ x, uint8_t* __restrict__ q, long n,
                                                   const unsigned* __restrict__ amax_bits) {
  const float amax = __uint_as_float(*amax_bits);
  const float sc = amax > 0.f ? 448.f / amax : 1.f;
  const long n4 = n >> 2;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = fminf(fmaxf(ld_any(x, 4 * i + j) * sc, -448.f), 448.f);
    int w = __builtin_amdgcn_cvt_pk_fp8_f32(v[0], v[1], 0, false);
    w = __builtin_amdgcn_cvt_pk_fp8_f32(v[2], v[3], w, true);
    ((int*)q)[i] = w;
  }
  for (long i = 4 * n4 + (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float v = fminf(fmaxf(ld_any(x, i) * sc, -448.f), 448.f);
    q[i] = (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(v, 0.f, 0, false) & 0xff);
  }
}

// alpha for an fp8 GEMM: (amax_a / 448) * (amax_b / 448) * extra  -> one float on the device
__global__ void k_fp8_alpha(const unsigned* amax_a, const unsigned* amax_b, float extra, float* alpha) {
  const float a = __uint_as_float(*amax_a), b = __uint_as_float(*amax_b);
  *alpha = (a > 0.f ? a / 448.f : 1.f) * (b > 0.f ? b / 448.f : 1.f) * extra;
}

// ---------------------------------------------------------------------------------------------------------
// Per-step weight packing: every layer's fp32 master weight [Cout][Cin][KH][KW] (torch layout -- the parameter
// itself) becomes its bf16 GEMM operands in ONE launch for the whole model, instead of a chain of
// permute / pad / cast ops per layer:
//   fwd   [Cout][Kp]            column (kh*KW + kw)*Cin_pad + c, zero for padded channels (Cin_pad = 8 for a
//                               3-channel stem) -> forward and strided-dgrad operand
//   dgrad [Cin][KH*KW*Cout]     taps flipped, ci/co swapped -> the stride-1 input gradient as an implicit conv
// and, for fp8 layers, the per-layer amax (k_pack_weights) then the e4m3 copy q = sat(w * 448 / amax)
// (k_pack_fp8).  grid (blocks per layer, layers); every block grid-strides over its layer's fwd elements.
// ---------------------------------------------------------------------------------------------------------
struct PackDesc {
  const float* w;
  bf16_t* fwd;
  bf16_t* dgrad;    // or null
  uint8_t* q8;      // or null
  unsigned* amax;   // float bits, zeroed before k_pack_weights (q8 layers only)
  int co, ci, ci_pad, kh, kw, kp;
};

// Index math is 32-bit: a layer's weight count is far below 2^31 (asserted on the host), and the 64-bit division
// sequences made this launch ALU-bound.
__device__ __forceinline__ bool pack_src(const PackDesc& d, unsigned i, unsigned& src, int& n, int& c, int& a,
                                         int& b) {
  n = (int)(i / (unsigned)d.kp);
  const int k = (int)(i - (unsigned)n * d.kp);
  const int tap = k / d.ci_pad;
  c = k - tap * d.ci_pad;
  a = tap / d.kw;
  b = tap - a * d.kw;
  if (c >= d.ci || tap >= d.kh * d.kw) return false;
  src = (((unsigned)n * d.ci + c) * d.kh + a) * d.kw + b;
  return true;
}

__global__ void __launch_bounds__(256) k_pack_weights(const PackDesc* __restrict__ descs) {
  const PackDesc d = descs[blockIdx.y];
  const unsigned total = (unsigned)d.co * d.kp;
  float m = 0.f;
  for (unsigned i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
    unsigned src;
    int n, c, a, b;
    const float v = pack_src(d, i, src, n, c, a, b) ? d.w[src] : 0.f;
    d.fwd[i] = f2bf_rne(v);
    m = fmaxf(m, fabsf(v));
  }
  if (d.dgrad) {
    // second pass: dgrad[c*taps + tflip][n] = w[n][c][taps-1-tflip] is a transpose of the [Cout][Cin*taps] weight
    // matrix (taps flipped inside each channel group), done through 32 x 32 LDS tiles so both the fp32 reads and
    // the bf16 writes are coalesced (a direct gather reads one cache line per element).
    __shared__ float tile[32][33];
    const unsigned taps = d.kh * d.kw, co = d.co, R = (unsigned)d.ci * taps;
    const unsigned tn = (co + 31) / 32, tr = (R + 31) / 32;
    const unsigned tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    for (unsigned t = blockIdx.x; t < tn * tr; t += gridDim.x) {  // block-uniform trip count
      const unsigned n0 = (t / tr) * 32, r0 = (t % tr) * 32;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const unsigned n = n0 + ty + 8 * j, r = r0 + tx;
        tile[ty + 8 * j][tx] = n < co && r < R ? d.w[n * R + r] : 0.f;
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const unsigned r = r0 + ty + 8 * j, n = n0 + tx;
        if (r < R && n < co) {
          const unsigned c = r / taps, tap = r - c * taps;
          d.dgrad[(c * taps + (taps - 1 - tap)) * co + n] = f2bf_rne(tile[tx][ty + 8 * j]);
        }
      }
      __syncthreads();
    }
  }
  if (d.q8) {
    __shared__ float red[256];
    red[threadIdx.x] = m;
    __syncthreads();
    for (int o = 128; o; o >>= 1) {
      if (threadIdx.x < o) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + o]);
      __syncthreads();
    }
    if (threadIdx.x == 0) atomicMax(d.amax, __float_as_uint(red[0]));
  }
}

__global__ void __launch_bounds__(256) k_pack_fp8(const PackDesc* __restrict__ descs) {
  const PackDesc d = descs[blockIdx.y];
  if (!d.q8) return;
  const float amax = __uint_as_float(*d.amax);
  const float sc = amax > 0.f ? 448.f / amax : 1.f;
  const unsigned total = (unsigned)d.co * d.kp;
  for (unsigned i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
    unsigned src;
    int n, c, a, b;
    const float v = pack_src(d, i, src, n, c, a, b) ? fminf(fmaxf(d.w[src] * sc, -448.f), 448.f) : 0.f;
    d.q8[i] = (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(v, 0.f, 0, false) & 0xff);
  }
}

// Network input: NCHW fp32 [N][C][HW] (C <= 8) -> NHWC bf16 [N][HW][8], channels C..7 zero (the 8-channel-padded
// stem input of the implicit-GEMM stem).  One thread per pixel: C strided fp32 reads, one 16-B store.
__global__ void __launch_bounds__(256) k_nchw_to_nhwc8(const float* __restrict__ x, bf16_t* __restrict__ y, int N,
                                                       int C, long HW) {
  const long total = (long)N * HW;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long n = i / HW, p = i - n * HW;
    float v[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) v[c] = c < C ? x[(n * C + c) * HW + p] : 0.f;
    *(uint4*)(y + i * 8) = pack8(v);
  }
}

// Space-to-depth input of a stride-2 stem convolution (C <= 4 channels): y[n][Y][X][(2 ph + pw) C + c] =
// x[n][c][2Y + ph - P][2X + pw - P] (zero outside the image; channels 4C .. 15 zero), 16 bf16 channels per pixel.
// A KxK / 2 conv with padding P - 1 over x is then a ceil((K+1)/2)^2 stride-1 conv with no padding over y (ops
// functional.stem_s2d_weight_index): ResNet's 7x7/2 stem becomes 4x4 taps x 16 channels = K 256 instead of
// 7 x 7 x 8 = 392, with two 16-B chunks per tap instead of one.
__global__ void __launch_bounds__(256) k_nchw_to_s2d16(const float* __restrict__ x, bf16_t* __restrict__ y, int N,
                                                       int C, int H, int W, int Hs, int Ws, int P) {
  const long total = (long)N * Hs * Ws;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long n = i / ((long)Hs * Ws);
    const int rem = (int)(i - n * Hs * Ws), Y = rem / Ws, X = rem - Y * Ws;
    float v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = 0.f;
#pragma unroll
    for (int ph = 0; ph < 2; ++ph)
#pragma unroll
      for (int pw = 0; pw < 2; ++pw) {
        const int h = 2 * Y + ph - P, w = 2 * X + pw - P;
        if (h < 0 || h >= H || w < 0 || w >= W) continue;
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (c < C) v[(2 * ph + pw) * C + c] = x[((n * C + c) * H + h) * W + w];
      }
    uint4* o = (uint4*)(y + i * 16);
    o[0] = pack8(v);
    o[1] = pack8(v + 8);
  }
}

// Gathered bf16 copies of fp32 weights: out[i] = bf16(w[idx[i]]), 0 where idx[i] < 0 -- the per-parity-class
// input-gradient matrices of strided convolutions and the space-to-depth stem matrix (index tables built once on
// the host).  grid (blocks, descriptors).
struct GatherDesc {
  const float* w;
  const int* idx;
  bf16_t* out;
  long n;
};
__global__ void __launch_bounds__(256) k_pack_gather(const GatherDesc* __restrict__ descs) {
  const GatherDesc d = descs[blockIdx.y];
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < d.n; i += (long)gridDim.x * 256) {
    const int k = d.idx[i];
    d.out[i] = f2bf_rne(k >= 0 ? d.w[k] : 0.f);
  }
}

}  // namespace ops
}  // namespace dca
