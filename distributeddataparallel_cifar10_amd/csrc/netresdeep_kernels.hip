// Fused NetResDeep training step for CDNA4 (gfx950 / MI355X).
//
// One training step = 22 dependent kernels (world_size 1), all captured in one hipGraph by engine.cpp:
//   k_stem_block0           : uint8 gather + normalise + conv1+bias+ReLU+maxpool (MFMA) -> x0, then trunk conv 0
//   k_fwd_block  (i=1..9)   : finalise BN(i-1) batch stats, apply BN+ReLU+residual while staging the LDS tile,
//                             trunk conv i on MFMA, per-tile BN partials (mean, M2) in the epilogue
//   k_head                  : BN(9)+ReLU+residual, maxpool, fc1+ReLU, fc2, cross-entropy fwd+bwd, fc bwd to the
//                             pooled features, maxpool bwd -> g10, first BN-backward partial sums
//   k_bwd_block  (i=9..0)   : BN-backward (grid-wide sums finalised in the prologue) -> dgrad conv on MFMA
//                             (+ residual), next block's BN-backward partials in the epilogue; horizontally fused
//                             extra workgroups compute the wgrad of block i+1 (or the fc1/fc2 grads for i=9);
//                             i=0 also does the stem backward and block-0 wgrad in-tile
//   k_reduce                : deterministic reduction of the wgrad partial slabs, SGD (fused at world_size 1),
//                             rebuild of the MFMA-layout weight copies, loss/cursor bookkeeping
// With world_size > 1, k_reduce only writes gradients; engine.cpp all-reduces them over RCCL (bucket A overlaps
// the trunk backward) and k_apply_sgd updates.
//
// Reference semantics mirrored: model/resnet.py:5-37 (weight-shared ResBlock, skip after ReLU), main.py:27-39
// (SGD lr, CrossEntropy mean), BatchNorm2d train-mode statistics and running-stat EMA applied 10x per forward.
#include "common.h"

namespace dca {

// ------------------------------------------------------------------------------------------------------------
// LDS record helpers.  A "record" is the 32 channels of one pixel (or of one weight row): 8 chunks of 16 B in
// fp32 mode, 4 chunks in bf16 mode.  Chunks are XOR-swizzled by a per-record key so that the 16-lane groups of
// ds_read_b128 (16 different pixels, same chunk) spread over all 64 banks.
// ------------------------------------------------------------------------------------------------------------
template <bool BF> struct Rec {
  static constexpr int NCH = BF ? 4 : 8;
  static constexpr int BYTES = NCH * 16;
  static constexpr int ESZ = BF ? 2 : 4;
};
template <bool BF> __device__ __forceinline__ int swz(int key) {
  if constexpr (BF) return (0x1230 >> (((key >> 2) & 3) << 2)) & 3;  // G = {0,3,2,1}
  else return key & 7;
}
template <bool BF> __device__ __forceinline__ int rec_off(int rec, int key, int chunk) {
  return ((rec * Rec<BF>::NCH) + (chunk ^ swz<BF>(key))) << 4;
}
__device__ __forceinline__ unsigned short bfbits(float f) {
  return __builtin_bit_cast(unsigned short, (__bf16)f);
}
__device__ __forceinline__ unsigned pk2(float a, float b) {
  return (unsigned)bfbits(a) | ((unsigned)bfbits(b) << 16);
}
__device__ __forceinline__ f32x4 ld4(const float* p) { return *(const f32x4*)p; }
__device__ __forceinline__ void st4(float* p, f32x4 v) { *(f32x4*)p = v; }
__device__ __forceinline__ f32x4 z4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }
__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// store 4 consecutive channels (4*c4 .. 4*c4+3) into a record
template <bool BF> __device__ __forceinline__ void st4_rec(char* base, int rec, int key, int c4, f32x4 v) {
  if constexpr (BF) {
    const int off = rec_off<BF>(rec, key, c4 >> 1) + ((c4 & 1) << 3);
    uint2 p;
    p.x = pk2(v.x, v.y);
    p.y = pk2(v.z, v.w);
    *(uint2*)(base + off) = p;
  } else {
    *(f32x4*)(base + rec_off<BF>(rec, key, c4)) = v;
  }
}
// store one channel into a record
template <bool BF> __device__ __forceinline__ void st1_rec(char* base, int rec, int key, int ch, float v) {
  if constexpr (BF) {
    *(unsigned short*)(base + rec_off<BF>(rec, key, ch >> 3) + ((ch & 7) << 1)) = bfbits(v);
  } else {
    *(float*)(base + rec_off<BF>(rec, key, ch >> 2) + ((ch & 3) << 2)) = v;
  }
}
// zero the 16-B chunks of `nrec` records starting at record `rec0`, every `stride` records
template <bool BF> __device__ __forceinline__ void zero_recs(char* base, int rec0, int nrec, int stride) {
  for (int idx = threadIdx.x; idx < nrec * Rec<BF>::NCH; idx += NT) {
    const int r = rec0 + (idx / Rec<BF>::NCH) * stride;
    *(uint4*)(base + ((r * Rec<BF>::NCH + idx % Rec<BF>::NCH) << 4)) = uint4{0u, 0u, 0u, 0u};
  }
}
// derived weight [9][32 out][32 in] (plain, compute type) -> swizzled LDS records (key = out)
template <bool BF> __device__ __forceinline__ void stage_weights(char* ws, const void* src) {
  const uint4* s = (const uint4*)src;
  for (int idx = threadIdx.x; idx < 288 * Rec<BF>::NCH; idx += NT) {
    const int rec = idx / Rec<BF>::NCH, ch = idx % Rec<BF>::NCH;
    *(uint4*)(ws + rec_off<BF>(rec, rec & 31, ch)) = s[idx];
  }
}

// ------------------------------------------------------------------------------------------------------------
// 3x3 / pad-1 / 32->32 convolution of an R-row tile on MFMA.
//   xs: (R+2) x 18 records (halo rows/cols, zero padded), ws: 9 taps x 32 output-channel records.
//   Wave w owns output tiles t = w + 4j (row t>>1, output-channel half t&1); one 16x16 MFMA tile =
//   16 pixels of one row x 16 output channels.  acc[j][i] = out[row][pixel 4q+i][16h + (lane&15)].
// bf16: v_mfma_f32_16x16x32_bf16, one MFMA per tap (K = 32 input channels).
// fp32: v_mfma_f32_16x16x4_f32 (exact fp32), K permuted so each lane reads 4 consecutive channels with one
//       ds_read_b128 that feeds 4 MFMAs (k-slot q of step s <-> channel 16hf + 4q + s, same on A and B).
// ------------------------------------------------------------------------------------------------------------
template <bool BF, int R>
__device__ __forceinline__ void conv_core(const char* xs, const char* ws, f32x4 (&acc)[R / 2], int wave, int lane) {
  const int c = lane & 15, q = lane >> 4;
#pragma unroll
  for (int j = 0; j < R / 2; ++j) acc[j] = z4();
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int kh = tap / 3, kw = tap % 3;
#pragma unroll
    for (int j = 0; j < R / 2; ++j) {
      const int tt = wave + 4 * j, rr = tt >> 1, h = tt & 1;
      const int col = c + kw, rec = (rr + kh) * 18 + col;
      const int wrec = tap * 32 + h * 16 + c;
      if constexpr (BF) {
        const bf16x8 a = *(const bf16x8*)(xs + rec_off<BF>(rec, col, q));
        const bf16x8 b = *(const bf16x8*)(ws + rec_off<BF>(wrec, h * 16 + c, q));
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[j], 0, 0, 0);
      } else {
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          const f32x4 a = *(const f32x4*)(xs + rec_off<BF>(rec, col, 4 * hf + q));
          const f32x4 b = *(const f32x4*)(ws + rec_off<BF>(wrec, h * 16 + c, 4 * hf + q));
          acc[j] = mfma4(a.x, b.x, acc[j]);
          acc[j] = mfma4(a.y, b.y, acc[j]);
          acc[j] = mfma4(a.z, b.z, acc[j]);
          acc[j] = mfma4(a.w, b.w, acc[j]);
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------------------
// Weight-gradient GEMM of the shared trunk conv over a ROWS x 16 pixel tile:
//   dW[co][ci][tap] += sum_p dy[p][co] * x[p + off(tap)][ci]
// dyT: [32 co][DS] (pixel-contiguous), xT: [3 kw][32 ci][XS] with xT[kw][ci][r][c] = x[r-1][c+kw-1].
// 36 output tiles (2 co halves x 9 taps x 2 ci halves), 9 per wave; written as raw MFMA fragments
// (tile, lane, reg) to a private slab -> fully coalesced f32x4 stores, reduced later by k_reduce.
// ------------------------------------------------------------------------------------------------------------
template <bool BF, int ROWS>
__device__ __forceinline__ void wgrad_core(const char* dyT, int DS, const char* xT, int XS, float* slab, int wave,
                                           int lane) {
  constexpr int ESZ = Rec<BF>::ESZ;
  const int c = lane & 15, q = lane >> 4;
  f32x4 acc[9];
#pragma unroll
  for (int j = 0; j < 9; ++j) acc[j] = z4();
  if constexpr (BF) {
#pragma unroll 2
    for (int s = 0; s < ROWS / 2; ++s) {
      const int row = 2 * s + (q >> 1), c0 = 8 * (q & 1);
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        const int tt = wave + 4 * j, mt = tt & 1, nt = tt >> 1, tap = nt >> 1, cih = nt & 1;
        const int kh = tap / 3, kw = tap % 3;
        const bf16x8 a = *(const bf16x8*)(dyT + ((16 * mt + c) * DS + row * 16 + c0) * ESZ);
        const bf16x8 b = *(const bf16x8*)(xT + ((kw * 32 + 16 * cih + c) * XS + (row + kh) * 16 + c0) * ESZ);
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[j], 0, 0, 0);
      }
    }
  } else {
    for (int row = 0; row < ROWS; ++row) {
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        const int tt = wave + 4 * j, mt = tt & 1, nt = tt >> 1, tap = nt >> 1, cih = nt & 1;
        const int kh = tap / 3, kw = tap % 3;
        const f32x4 a = *(const f32x4*)(dyT + ((16 * mt + c) * DS + row * 16 + 4 * q) * ESZ);
        const f32x4 b = *(const f32x4*)(xT + ((kw * 32 + 16 * cih + c) * XS + (row + kh) * 16 + 4 * q) * ESZ);
        acc[j] = mfma4(a.x, b.x, acc[j]);
        acc[j] = mfma4(a.y, b.y, acc[j]);
        acc[j] = mfma4(a.z, b.z, acc[j]);
        acc[j] = mfma4(a.w, b.w, acc[j]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 9; ++j) st4(slab + (((wave + 4 * j) * 64 + lane) << 2), acc[j]);
}

// ------------------------------------------------------------------------------------------------------------
// BatchNorm statistic reductions (deterministic, fixed order).
// ------------------------------------------------------------------------------------------------------------
// forward: per-tile (mean, M2) with equal counts -> batch mean and biased variance (Chan's combination)
__device__ void reduce_fstats(const float2* part, int nparts, float cnt, float* red, float* s_mean, float* s_var) {
  const int t = threadIdx.x, c = t & 31, g = t >> 5;
  float sm = 0.f;
  for (int w = g; w < nparts; w += 8) sm += part[w * 32 + c].x;
  red[t] = sm;
  __syncthreads();
  if (t < 32) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += red[k * 32 + t];
    s_mean[t] = s / (float)nparts;
  }
  __syncthreads();
  const float mean = s_mean[c];
  float m2 = 0.f;
  for (int w = g; w < nparts; w += 8) {
    const float2 p = part[w * 32 + c];
    const float d = p.x - mean;
    m2 += p.y + cnt * d * d;
  }
  red[t] = m2;
  __syncthreads();
  if (t < 32) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += red[k * 32 + t];
    s_var[t] = s / ((float)nparts * cnt);
  }
  __syncthreads();
}
// backward: per-tile (sum dz, sum dz*xhat) -> totals
__device__ void reduce_bsums(const float2* part, int nparts, float* red, float* s_a, float* s_b) {
  const int t = threadIdx.x, c = t & 31, g = t >> 5;
  float sa = 0.f, sb = 0.f;
  for (int w = g; w < nparts; w += 8) {
    const float2 p = part[w * 32 + c];
    sa += p.x;
    sb += p.y;
  }
  red[t] = sa;
  red[256 + t] = sb;
  __syncthreads();
  if (t < 32) {
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      a += red[k * 32 + t];
      b += red[256 + k * 32 + t];
    }
    s_a[t] = a;
    s_b[t] = b;
  }
  __syncthreads();
}
// running-stat EMA of one BN application (reference: nn.BatchNorm2d momentum 0.1, unbiased running_var)
__device__ __forceinline__ void bn_running_update(const Ctx& cx, int t, float mean, float var_b, bool from_base) {
  const float ntot = (float)cx.B * 256.f;
  const float unb = var_b * ntot / (ntot - 1.f);
  const float rm0 = from_base ? cx.rs_base[t] : cx.rm[t];
  const float rv0 = from_base ? cx.rs_base[32 + t] : cx.rv[t];
  const float m = cx.bn_mom;
  cx.rm[t] = rm0 * (1.f - m) + mean * m;
  cx.rv[t] = rv0 * (1.f - m) + unb * m;
}

// forward epilogue: store y tile, per-tile BN partials (mean, M2) for this tile's R*16 pixels
template <int R>
__device__ __forceinline__ void fwd_epilogue(const f32x4 (&acc)[R / 2], float* ytile, float2* part, float* red,
                                             float* s_tmp, int wave, int lane) {
  const int t = threadIdx.x, c = lane & 15, q = lane >> 4;
#pragma unroll
  for (int j = 0; j < R / 2; ++j) {
    const int tt = wave + 4 * j, rr = tt >> 1, ch = 16 * (tt & 1) + c;
    float* yp = ytile + (rr * 16 + 4 * q) * 32 + ch;
    yp[0] = acc[j].x;
    yp[32] = acc[j].y;
    yp[64] = acc[j].z;
    yp[96] = acc[j].w;
    float s = acc[j].x + acc[j].y + acc[j].z + acc[j].w;
    s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    if (q == 0) red[tt * 16 + c] = s;
  }
  __syncthreads();
  if (t < 32) {
    const int h = t >> 4, cc = t & 15;
    float s = 0.f;
#pragma unroll
    for (int rr = 0; rr < R; ++rr) s += red[(rr * 2 + h) * 16 + cc];
    s_tmp[t] = s / (float)(R * 16);
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < R / 2; ++j) {
    const int tt = wave + 4 * j, ch = 16 * (tt & 1) + c;
    const float m = s_tmp[ch];
    const float d0 = acc[j].x - m, d1 = acc[j].y - m, d2 = acc[j].z - m, d3 = acc[j].w - m;
    float s = d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3;
    s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    if (q == 0) red[tt * 16 + c] = s;
  }
  __syncthreads();
  if (t < 32) {
    const int h = t >> 4, cc = t & 15;
    float s = 0.f;
#pragma unroll
    for (int rr = 0; rr < R; ++rr) s += red[(rr * 2 + h) * 16 + cc];
    part[t] = make_float2(s_tmp[t], s);
  }
}

__device__ __forceinline__ size_t act_off(int blk, int B) { return (size_t)blk * B * 8192; }

// ============================================================================================================
// Forward, block 0: stem (gather+normalise+conv1+bias+ReLU+maxpool) fused with the first trunk conv.
// ============================================================================================================
template <bool BF, int R>
__global__ void __launch_bounds__(NT) k_stem_block0(Ctx cx) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int RR = R + 2, IR = 2 * RR + 2, IW = 34, RB = Rec<BF>::BYTES, TPI = 16 / R;
  using TA = typename std::conditional<BF, unsigned short, float>::type;
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63, c = lane & 15, q = lane >> 4;
  const int wg = blockIdx.x, n = wg / TPI, r0 = (wg % TPI) * R;
  char* ws = smem;
  char* xs = ws + 288 * RB;
  float* xin = (float*)(xs + RR * 18 * RB);   // [3][IR][IW]
  TA* swl = (TA*)(xin + 3 * IR * IW);         // [32][32]
  float* s_bias = (float*)(swl + 32 * 32);
  float* red = s_bias + 32;
  float* s_tmp = red + 512;

  const uint8_t* src = cx.data + (size_t)sample_id(cx, n) * 3072;
  const float nmean[3] = {0.4915f, 0.4823f, 0.4468f};  // reference main.py:56-57
  const float nstd[3] = {0.2470f, 0.2435f, 0.2616f};
  for (int idx = t; idx < 3 * IR * IW; idx += NT) {
    const int ch = idx / (IR * IW), rem = idx % (IR * IW), ir = rem / IW, ic = rem % IW;
    const int y = 2 * r0 - 3 + ir, x = ic - 1;
    float v = 0.f;
    if (y >= 0 && y < 32 && x >= 0 && x < 32) v = ((float)src[ch * 1024 + y * 32 + x] / 255.f - nmean[ch]) / nstd[ch];
    xin[idx] = v;
  }
  stage_weights<BF>(ws, cx.wt_f);
  {
    const uint4* s = (const uint4*)cx.sw;
    for (int idx = t; idx < 32 * 32 * (int)sizeof(TA) / 16; idx += NT) ((uint4*)swl)[idx] = s[idx];
  }
  if (t < 32) s_bias[t] = cx.params[OFF_C1B + t];
  zero_recs<BF>(xs, 0, RR, 18);
  zero_recs<BF>(xs, 17, RR, 18);
  __syncthreads();

  // per-lane im2col offsets (k = ci*9 + kh*3 + kw)
  constexpr int NK = BF ? 8 : 7;
  int koff[NK];
  bool kval[NK];
#pragma unroll
  for (int s = 0; s < NK; ++s) {
    const int k = BF ? 8 * q + s : 4 * s + q;
    kval[s] = k < 27;
    const int ci = k / 9, kh = (k % 9) / 3, kw = k % 3;
    koff[s] = kval[s] ? ci * IR * IW + kh * IW + kw : 0;
  }
  float* X0 = cx.X + (size_t)n * 8192;
  uint8_t* code_out = cx.SCODE + (size_t)n * 8192;
  for (int u = wave; u < 4 * RR; u += 4) {
    const int prl = u >> 2, chalf = (u >> 1) & 1, h = u & 1;
    const int co = 16 * h + c;
    const int base0 = (2 * prl) * IW + 16 * chalf + c;
    f32x4 a0 = z4(), a1 = z4();
    if constexpr (BF) {
      const bf16x8 b = *(const bf16x8*)(swl + co * 32 + 8 * q);
      bf16x8 v0, v1;
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        v0[s] = (__bf16)(kval[s] ? xin[koff[s] + base0] : 0.f);
        v1[s] = (__bf16)(kval[s] ? xin[koff[s] + base0 + IW] : 0.f);
      }
      a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(v0, b, a0, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(v1, b, a1, 0, 0, 0);
    } else {
#pragma unroll
      for (int s = 0; s < 7; ++s) {
        const float bw = kval[s] ? swl[co * 32 + 4 * s + q] : 0.f;
        const float v0 = kval[s] ? xin[koff[s] + base0] : 0.f;
        const float v1 = kval[s] ? xin[koff[s] + base0 + IW] : 0.f;
        a0 = mfma4(v0, bw, a0);
        a1 = mfma4(v1, bw, a1);
      }
    }
    const float bias = s_bias[co];
    const int pr_img = r0 - 1 + prl;
    const bool rvalid = pr_img >= 0 && pr_img < 16;
#pragma unroll
    for (int pp = 0; pp < 2; ++pp) {
      const float v00 = fmaxf(a0[2 * pp] + bias, 0.f), v01 = fmaxf(a0[2 * pp + 1] + bias, 0.f);
      const float v10 = fmaxf(a1[2 * pp] + bias, 0.f), v11 = fmaxf(a1[2 * pp + 1] + bias, 0.f);
      float best = v00;
      int code = 0;
      if (v01 > best) { best = v01; code = 1; }
      if (v10 > best) { best = v10; code = 2; }
      if (v11 > best) { best = v11; code = 3; }
      if (best > 0.f) code |= 4;
      const int pc = 8 * chalf + 2 * q + pp;
      st1_rec<BF>(xs, prl * 18 + pc + 1, pc + 1, co, rvalid ? best : 0.f);
      if (prl >= 1 && prl <= R) {
        X0[(pr_img * 16 + pc) * 32 + co] = best;
        code_out[(pr_img * 16 + pc) * 32 + co] = (uint8_t)code;
      }
    }
  }
  __syncthreads();
  f32x4 acc[R / 2];
  conv_core<BF, R>(xs, ws, acc, wave, lane);
  fwd_epilogue<R>(acc, cx.Y + (size_t)n * 8192 + r0 * 512, cx.FPART + (size_t)wg * 32, red, s_tmp, wave, lane);
}

// ============================================================================================================
// Forward, blocks 1..9: x_i = relu(BN(y_{i-1})) + x_{i-1} staged into LDS, then y_i = conv(x_i).
// ============================================================================================================
template <bool BF, int R>
__global__ void __launch_bounds__(NT) k_fwd_block(Ctx cx, int i) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int RR = R + 2, TPI = 16 / R, NF = RR * 128 / NT, RB = Rec<BF>::BYTES;
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int wg = blockIdx.x, n = wg / TPI, r0 = (wg % TPI) * R;
  const int nparts = cx.B * TPI;
  char* ws = smem;
  char* xs = ws + 288 * RB;
  float* red = (float*)(xs + RR * 18 * RB);
  float* s_mean = red + 512;
  float* s_var = s_mean + 32;
  float* s_scale = s_var + 32;
  float* s_shift = s_scale + 32;

  const float* Yp = cx.Y + act_off(i - 1, cx.B) + (size_t)n * 8192;
  const float* Xp = cx.X + act_off(i - 1, cx.B) + (size_t)n * 8192;
  f32x4 yv[NF], xv[NF];
#pragma unroll
  for (int m = 0; m < NF; ++m) {
    const int f = t + NT * m, tr = f >> 7, col = (f >> 3) & 15, c4 = f & 7, row = r0 - 1 + tr;
    if (row >= 0 && row < 16) {
      const int off = (row * 16 + col) * 32 + 4 * c4;
      yv[m] = ld4(Yp + off);
      xv[m] = ld4(Xp + off);
    } else {
      yv[m] = z4();
      xv[m] = z4();
    }
  }
  stage_weights<BF>(ws, cx.wt_f);
  zero_recs<BF>(xs, 0, RR, 18);
  zero_recs<BF>(xs, 17, RR, 18);
  reduce_fstats(cx.FPART + (size_t)(i - 1) * cx.pstride * 32, nparts, (float)(R * 16), red, s_mean, s_var);
  if (t < 32) {
    const float mean = s_mean[t], var = s_var[t], invstd = rsqrtf(var + cx.bn_eps);
    const float gam = cx.params[OFF_BNW + t], bet = cx.params[OFF_BNB + t];
    s_scale[t] = gam * invstd;
    s_shift[t] = bet - mean * gam * invstd;
    if (wg == 0) {
      cx.STATS[(i - 1) * 32 + t] = make_float2(mean, invstd);
      bn_running_update(cx, t, mean, var, (i == 1) && cx.ws > 1);
      if (t == 0) *cx.nbt += 1;
    }
  }
  __syncthreads();
  float* Xo = cx.X + act_off(i, cx.B) + (size_t)n * 8192;
#pragma unroll
  for (int m = 0; m < NF; ++m) {
    const int f = t + NT * m, tr = f >> 7, col = (f >> 3) & 15, c4 = f & 7, row = r0 - 1 + tr;
    f32x4 xn = z4();
    if (row >= 0 && row < 16) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int ch = 4 * c4 + e;
        xn[e] = fmaxf(yv[m][e] * s_scale[ch] + s_shift[ch], 0.f) + xv[m][e];
      }
      if (tr >= 1 && tr <= R) st4(Xo + (row * 16 + col) * 32 + 4 * c4, xn);
    }
    st4_rec<BF>(xs, tr * 18 + col + 1, col + 1, c4, xn);
  }
  __syncthreads();
  f32x4 acc[R / 2];
  conv_core<BF, R>(xs, ws, acc, wave, lane);
  fwd_epilogue<R>(acc, cx.Y + act_off(i, cx.B) + (size_t)n * 8192 + r0 * 512,
                  cx.FPART + ((size_t)i * cx.pstride + wg) * 32, red, s_mean, wave, lane);
}

// ============================================================================================================
// Head: BN(9)+ReLU+residual -> maxpool -> fc1+ReLU -> fc2 -> cross-entropy (fwd + bwd) -> back to g10,
// plus the first BN-backward partial sums.  One workgroup per image.
// ============================================================================================================
template <int R>
__global__ void __launch_bounds__(NT) k_head(Ctx cx) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TPI = 16 / R;
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int n = blockIdx.x, nparts = cx.B * TPI;
  float* x10 = (float*)smem;        // [256][32]  (reused as dz)
  float* dzx = x10 + 8192;          // [256][32]
  float* P = dzx + 8192;            // [2048] NCHW-flatten order (c*64 + ph*8 + pw)
  float* dpl = P + 2048;            // [2048]
  uint8_t* code = (uint8_t*)(dpl + 2048);  // [64 pooled px][32]
  float* red = (float*)(code + 2048);
  float* s_mean = red + 512;
  float* s_var = s_mean + 32;
  float* s_scale = s_var + 32;
  float* s_shift = s_scale + 32;
  float* s_invstd = s_shift + 32;
  float* hv = s_invstd + 32;   // fc1 pre-activation [32]
  float* sdh = hv + 32;        // [32]
  float* logit = sdh + 32;     // [16]
  float* sdl = logit + 16;     // [16]

  const float* Yp = cx.Y + act_off(9, cx.B) + (size_t)n * 8192;
  const float* Xp = cx.X + act_off(9, cx.B) + (size_t)n * 8192;
  f32x4 yv[8];
#pragma unroll
  for (int m = 0; m < 8; ++m) yv[m] = ld4(Yp + 4 * (t + NT * m));
  reduce_fstats(cx.FPART + (size_t)9 * cx.pstride * 32, nparts, (float)(R * 16), red, s_mean, s_var);
  if (t < 32) {
    const float mean = s_mean[t], var = s_var[t], invstd = rsqrtf(var + cx.bn_eps);
    const float gam = cx.params[OFF_BNW + t], bet = cx.params[OFF_BNB + t];
    s_scale[t] = gam * invstd;
    s_shift[t] = bet - mean * gam * invstd;
    s_invstd[t] = invstd;
    if (n == 0) {
      cx.STATS[9 * 32 + t] = make_float2(mean, invstd);
      bn_running_update(cx, t, mean, var, false);
      if (t == 0) *cx.nbt += 1;
    }
  }
  __syncthreads();
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const int f = t + NT * m, c4 = f & 7;
    const f32x4 xv = ld4(Xp + 4 * f);
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = fmaxf(yv[m][e] * s_scale[4 * c4 + e] + s_shift[4 * c4 + e], 0.f) + xv[e];
    st4(x10 + 4 * f, o);
  }
  __syncthreads();
  // 2x2 max-pool with first-max tie break (PyTorch scan order)
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const int o = t + NT * m, ch = o & 31, pp = o >> 5, ph = pp >> 3, pw = pp & 7;
    const int p00 = ((2 * ph) * 16 + 2 * pw) * 32 + ch;
    const float v00 = x10[p00], v01 = x10[p00 + 32], v10 = x10[p00 + 512], v11 = x10[p00 + 544];
    float best = v00;
    int id = 0;
    if (v01 > best) { best = v01; id = 1; }
    if (v10 > best) { best = v10; id = 2; }
    if (v11 > best) { best = v11; id = 3; }
    P[ch * 64 + pp] = best;
    code[pp * 32 + ch] = (uint8_t)id;
  }
  __syncthreads();
  // fc1: wave w computes outputs j = 8w .. 8w+7 (coalesced 1 KiB rows of W1)
  const float* W1 = cx.params + OFF_FC1W;
#pragma unroll 2
  for (int jj = 0; jj < 8; ++jj) {
    const int j = 8 * wave + jj;
    float s = 0.f;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const f32x4 w4 = ld4(W1 + j * 2048 + 4 * lane + 256 * m);
      const f32x4 p4 = ld4(P + 4 * lane + 256 * m);
      s += w4.x * p4.x + w4.y * p4.y + w4.z * p4.z + w4.w * p4.w;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) hv[j] = s + cx.params[OFF_FC1B + j];
  }
  __syncthreads();
  if (t < 10) {
    float s = cx.params[OFF_FC2B + t];
    for (int j = 0; j < 32; ++j) s += cx.params[OFF_FC2W + t * 32 + j] * fmaxf(hv[j], 0.f);
    logit[t] = s;
  }
  __syncthreads();
  if (t == 0) {
    const int label = cx.labels[sample_id(cx, n)];
    float mx = logit[0];
    for (int o = 1; o < 10; ++o) mx = fmaxf(mx, logit[o]);
    float se = 0.f;
    for (int o = 0; o < 10; ++o) se += expf(logit[o] - mx);
    const float lse = mx + logf(se);
    cx.HLOSS[n] = lse - logit[label];
    const float invB = 1.f / (float)cx.B;
    for (int o = 0; o < 10; ++o) sdl[o] = (expf(logit[o] - lse) - (o == label ? 1.f : 0.f)) * invB;
  }
  __syncthreads();
  if (t < 32) {
    float s = 0.f;
    for (int o = 0; o < 10; ++o) s += cx.params[OFF_FC2W + o * 32 + t] * sdl[o];
    const float dh = hv[t] > 0.f ? s : 0.f;
    sdh[t] = dh;
    cx.HDH[n * 32 + t] = dh;
    cx.HH[n * 32 + t] = fmaxf(hv[t], 0.f);
    if (t < 10) cx.HDL[n * 10 + t] = sdl[t];
  }
#pragma unroll
  for (int m = 0; m < 2; ++m) st4(cx.HP + (size_t)n * 2048 + 4 * (t + NT * m), ld4(P + 4 * (t + NT * m)));
  __syncthreads();
  // dp = W1^T dh  (coalesced over k)
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const int k = t + NT * m;
    float s = 0.f;
#pragma unroll 8
    for (int j = 0; j < 32; ++j) s += W1[j * 2048 + k] * sdh[j];
    dpl[k] = s;
  }
  __syncthreads();
  // g10 = maxpool-backward(dp); dz9 = g10 * [z9 > 0]; per-tile sums of dz and dz*xhat
  float* G0 = cx.G + (size_t)n * 8192;  // ping-pong slot 0 holds g10
  float* dzl = x10;
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const int f = t + NT * m, pix = f >> 3, c4 = f & 7, row = pix >> 4, col = pix & 15;
    const int pp = (row >> 1) * 8 + (col >> 1), pos = (row & 1) * 2 + (col & 1);
    f32x4 g, dz, dzxv;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int ch = 4 * c4 + e;
      g[e] = (code[pp * 32 + ch] == pos) ? dpl[ch * 64 + pp] : 0.f;
      const float y = yv[m][e];
      const float z = y * s_scale[ch] + s_shift[ch];
      const float xh = (y - s_mean[ch]) * s_invstd[ch];
      dz[e] = z > 0.f ? g[e] : 0.f;
      dzxv[e] = dz[e] * xh;
    }
    st4(G0 + 4 * f, g);
    st4(dzl + 4 * f, dz);
    st4(dzx + 4 * f, dzxv);
  }
  __syncthreads();
  {
    const int ch = t & 31, k = t >> 5;
    if (k < TPI) {
      float sa = 0.f, sb = 0.f;
      for (int p = k * R * 16; p < (k + 1) * R * 16; ++p) {
        sa += dzl[p * 32 + ch];
        sb += dzx[p * 32 + ch];
      }
      cx.BPART[(size_t)(n * TPI + k) * 32 + ch] = make_float2(sa, sb);
    }
  }
}

// ============================================================================================================
// Backward workgroup roles
// ============================================================================================================
// fc1/fc2 weight gradients from the head's saved per-image vectors (sum over the batch, fixed order)
__device__ void fc_grads_role(const Ctx& cx, int f) {
  const int t = threadIdx.x, j = t >> 3, k = 64 * f + 8 * (t & 7);
  f32x4 a0 = z4(), a1 = z4();
  for (int b = 0; b < cx.B; ++b) {
    const float dh = cx.HDH[b * 32 + j];
    const f32x4 p0 = ld4(cx.HP + (size_t)b * 2048 + k), p1 = ld4(cx.HP + (size_t)b * 2048 + k + 4);
    a0 += dh * p0;
    a1 += dh * p1;
  }
  st4(cx.grads + OFF_FC1W + j * 2048 + k, a0);
  st4(cx.grads + OFF_FC1W + j * 2048 + k + 4, a1);
  if (f == 0) {
    for (int idx = t; idx < 32 + 320 + 10; idx += NT) {
      float s = 0.f;
      if (idx < 32) {
        for (int b = 0; b < cx.B; ++b) s += cx.HDH[b * 32 + idx];
        cx.grads[OFF_FC1B + idx] = s;
      } else if (idx < 352) {
        const int o = (idx - 32) >> 5, jj = (idx - 32) & 31;
        for (int b = 0; b < cx.B; ++b) s += cx.HDL[b * 10 + o] * cx.HH[b * 32 + jj];
        cx.grads[OFF_FC2W + o * 32 + jj] = s;
      } else {
        const int o = idx - 352;
        for (int b = 0; b < cx.B; ++b) s += cx.HDL[b * 10 + o];
        cx.grads[OFF_FC2B + o] = s;
      }
    }
  }
}

// wgrad of trunk block `blk` over RW rows of one image, from DY[blk] and X[blk] (stored by earlier kernels)
template <bool BF, int RW>
__device__ void wgrad_role(const Ctx& cx, int blk, int wv, char* smem) {
  constexpr int ESZ = Rec<BF>::ESZ, PADE = 16 / ESZ;
  constexpr int DS = RW * 16 + PADE, XS = (RW + 2) * 16 + PADE;
  using TA = typename std::conditional<BF, unsigned short, float>::type;
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int n = wv / (16 / RW), r0 = (wv % (16 / RW)) * RW;
  TA* dyT = (TA*)smem;
  TA* xT = dyT + 32 * DS;
  for (int idx = t; idx < 3 * 32 * XS * ESZ / 16; idx += NT) ((uint4*)xT)[idx] = uint4{0u, 0u, 0u, 0u};
  const float* dyp = cx.DY + act_off(blk, cx.B) + (size_t)n * 8192 + r0 * 512;
  const float* xp = cx.X + act_off(blk, cx.B) + (size_t)n * 8192;
  __syncthreads();
  for (int f = t; f < RW * 128; f += NT) {
    const int pix = f >> 3, c4 = f & 7;
    const f32x4 v = ld4(dyp + 4 * f);
#pragma unroll
    for (int e = 0; e < 4; ++e) dyT[(4 * c4 + e) * DS + pix] = BF ? (TA)bfbits(v[e]) : (TA)v[e];
  }
  for (int f = t; f < (RW + 2) * 128; f += NT) {
    const int tr = f >> 7, col = (f >> 3) & 15, c4 = f & 7, row = r0 - 1 + tr;
    if (row < 0 || row >= 16) continue;
    const f32x4 v = ld4(xp + (row * 16 + col) * 32 + 4 * c4);
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int cc = col + 1 - kw;
      if (cc < 0 || cc >= 16) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        TA* dst = xT + (kw * 32 + 4 * c4 + e) * XS + tr * 16 + cc;
        *dst = BF ? (TA)bfbits(v[e]) : (TA)v[e];
      }
    }
  }
  __syncthreads();
  const int nw_blk = cx.B * (16 / RW);
  wgrad_core<BF, RW>((const char*)dyT, DS, (const char*)xT, XS,
                     cx.WSLAB + ((size_t)(blk - 1) * nw_blk + wv) * WSLAB_N, wave, lane);
}

// dgrad role: BN-backward of block i -> dgrad conv -> g_i; epilogue prepares block i-1 (or the stem, i == 0)
template <bool BF, int R, int RW>
__device__ void dgrad_role(const Ctx& cx, int i, int wg, char* smem) {
  constexpr int RR = R + 2, TPI = 16 / R, NF = RR * 128 / NT, RB = Rec<BF>::BYTES;
  constexpr int ESZ = Rec<BF>::ESZ, PADE = 16 / ESZ;
  constexpr int DS0 = R * 16 + PADE, XS0 = RR * 16 + PADE;          // block-0 in-tile wgrad
  constexpr int IRb = 2 * R + 2, IW = 34, DSP = 2 * R * 32 + PADE;   // stem backward
  using TA = typename std::conditional<BF, unsigned short, float>::type;
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63, c = lane & 15, q = lane >> 4;
  const int n = wg / TPI, r0 = (wg % TPI) * R;
  const int nparts = cx.B * TPI;
  const int rd = (9 - i) & 1, wr = (10 - i) & 1;

  char* ws = smem;
  char* dys = ws + 288 * RB;
  float* gown = (float*)(dys + RR * 18 * RB);  // [R*16][32]
  float* yprev = gown + R * 512;               // [R*16][32]
  float* red = yprev + R * 512;                // [512]
  float* s_a = red + 512;
  float* s_b = s_a + 32;
  float* s_mean = s_b + 32;
  float* s_inv = s_mean + 32;
  float* s_scale = s_inv + 32;
  float* s_shift = s_scale + 32;
  float* s_k1 = s_shift + 32;
  float* s_pm = s_k1 + 32;
  float* s_pi = s_pm + 32;
  float* s_gam = s_pi + 32;
  float* s_bet = s_gam + 32;
  char* ext = (char*)(s_bet + 32);              // block-0 extras
  TA* dyT = (TA*)ext;                           // [32][DS0]
  TA* xT = dyT + 32 * DS0;                      // [3][32][XS0]
  float* xin = (float*)(xT + 3 * 32 * XS0);     // [3][IRb][IW]
  TA* dsT = (TA*)(xin + 3 * IRb * IW);          // [32][DSP]

  const size_t img = (size_t)n * 8192;
  const float* gin = cx.G + (size_t)rd * cx.B * 8192 + img;
  const float* yi = cx.Y + act_off(i, cx.B) + img;
  f32x4 gv[NF], yv[NF];
#pragma unroll
  for (int m = 0; m < NF; ++m) {
    const int f = t + NT * m, tr = f >> 7, col = (f >> 3) & 15, c4 = f & 7, row = r0 - 1 + tr;
    if (row >= 0 && row < 16) {
      const int off = (row * 16 + col) * 32 + 4 * c4;
      gv[m] = ld4(gin + off);
      yv[m] = ld4(yi + off);
    } else {
      gv[m] = z4();
      yv[m] = z4();
    }
  }
  if (i >= 1) {
    const float* yp = cx.Y + act_off(i - 1, cx.B) + img + r0 * 512;
    for (int f = t; f < R * 128; f += NT) st4(yprev + 4 * f, ld4(yp + 4 * f));
  }
  stage_weights<BF>(ws, cx.wt_d);
  zero_recs<BF>(dys, 0, RR, 18);
  zero_recs<BF>(dys, 17, RR, 18);
  if (i == 0) {
    for (int idx = t; idx < 3 * 32 * XS0 * ESZ / 16; idx += NT) ((uint4*)xT)[idx] = uint4{0u, 0u, 0u, 0u};
    for (int idx = t; idx < 32 * DSP * ESZ / 16; idx += NT) ((uint4*)dsT)[idx] = uint4{0u, 0u, 0u, 0u};
    // stem input rows 2r0-1 .. 2r0+2R (normalised, zero padded)
    const uint8_t* src = cx.data + (size_t)sample_id(cx, n) * 3072;
    const float nmean[3] = {0.4915f, 0.4823f, 0.4468f};
    const float nstd[3] = {0.2470f, 0.2435f, 0.2616f};
    for (int idx = t; idx < 3 * IRb * IW; idx += NT) {
      const int ch = idx / (IRb * IW), rem = idx % (IRb * IW), ir = rem / IW, ic = rem % IW;
      const int y = 2 * r0 - 1 + ir, x = ic - 1;
      float v = 0.f;
      if (y >= 0 && y < 32 && x >= 0 && x < 32)
        v = ((float)src[ch * 1024 + y * 32 + x] / 255.f - nmean[ch]) / nstd[ch];
      xin[idx] = v;
    }
  }
  reduce_bsums(cx.BPART + (size_t)rd * cx.pstride * 32, nparts, red, s_a, s_b);
  if (t < 32) {
    const float2 st = cx.STATS[i * 32 + t];
    const float gam = cx.params[OFF_BNW + t], bet = cx.params[OFF_BNB + t];
    const float N = (float)cx.B * 256.f;
    s_mean[t] = st.x;
    s_inv[t] = st.y;
    s_scale[t] = gam * st.y;
    s_shift[t] = bet - st.x * gam * st.y;
    s_k1[t] = gam * st.y / N;
    s_gam[t] = gam;
    s_bet[t] = bet;
    if (i >= 1) {
      const float2 sp = cx.STATS[(i - 1) * 32 + t];
      s_pm[t] = sp.x;
      s_pi[t] = sp.y;
    }
    if (wg == 0) {  // shared BN affine grads accumulate over the 10 applications
      const float pw = (i == 9) ? 0.f : cx.grads[OFF_BNW + t];
      const float pb = (i == 9) ? 0.f : cx.grads[OFF_BNB + t];
      cx.grads[OFF_BNW + t] = pw + s_b[t];
      cx.grads[OFF_BNB + t] = pb + s_a[t];
    }
  }
  __syncthreads();
  {
    const float N = (float)cx.B * 256.f;
    float* dyo = cx.DY + act_off(i, cx.B) + img;
    const float* x0p = cx.X + img;  // block 0 input (for the in-tile wgrad, i == 0)
#pragma unroll
    for (int m = 0; m < NF; ++m) {
      const int f = t + NT * m, tr = f >> 7, col = (f >> 3) & 15, c4 = f & 7, row = r0 - 1 + tr;
      f32x4 dy = z4();
      if (row >= 0 && row < 16) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int ch = 4 * c4 + e;
          const float y = yv[m][e];
          const float xh = (y - s_mean[ch]) * s_inv[ch];
          const float z = y * s_scale[ch] + s_shift[ch];
          const float dz = z > 0.f ? gv[m][e] : 0.f;
          dy[e] = s_k1[ch] * (N * dz - s_a[ch] - xh * s_b[ch]);
        }
        if (tr >= 1 && tr <= R) {
          const int po = ((tr - 1) * 16 + col) * 32 + 4 * c4;
          st4(gown + po, gv[m]);
          if (i >= 1) st4(dyo + (row * 16 + col) * 32 + 4 * c4, dy);
          else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              dyT[(4 * c4 + e) * DS0 + (tr - 1) * 16 + col] = BF ? (TA)bfbits(dy[e]) : (TA)dy[e];
          }
        }
        if (i == 0) {
          const f32x4 xv = ld4(x0p + (row * 16 + col) * 32 + 4 * c4);
#pragma unroll
          for (int kw = 0; kw < 3; ++kw) {
            const int cc = col + 1 - kw;
            if (cc < 0 || cc >= 16) continue;
#pragma unroll
            for (int e = 0; e < 4; ++e)
              xT[(kw * 32 + 4 * c4 + e) * XS0 + tr * 16 + cc] = BF ? (TA)bfbits(xv[e]) : (TA)xv[e];
          }
        }
      }
      st4_rec<BF>(dys, tr * 18 + col + 1, col + 1, c4, dy);
    }
  }
  __syncthreads();
  f32x4 acc[R / 2];
  conv_core<BF, R>(dys, ws, acc, wave, lane);

  if (i >= 1) {
    float* gout = cx.G + (size_t)wr * cx.B * 8192 + img + r0 * 512;
#pragma unroll
    for (int j = 0; j < R / 2; ++j) {
      const int tt = wave + 4 * j, rr = tt >> 1, ch = 16 * (tt & 1) + c;
      const float scp = s_gam[ch] * s_pi[ch], shp = s_bet[ch] - s_pm[ch] * s_gam[ch] * s_pi[ch];
      float sa = 0.f, sb = 0.f;
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) {
        const int po = (rr * 16 + 4 * q + ii) * 32 + ch;
        const float g = gown[po] + acc[j][ii];
        gout[po] = g;
        const float y = yprev[po];
        const float z = y * scp + shp;
        const float dz = z > 0.f ? g : 0.f;
        sa += dz;
        sb += dz * (y - s_pm[ch]) * s_pi[ch];
      }
      sa += __shfl_xor(sa, 16);
      sa += __shfl_xor(sa, 32);
      sb += __shfl_xor(sb, 16);
      sb += __shfl_xor(sb, 32);
      if (q == 0) {
        red[tt * 16 + c] = sa;
        red[256 + tt * 16 + c] = sb;
      }
    }
    __syncthreads();
    if (t < 32) {
      const int h = t >> 4, cc = t & 15;
      float sa = 0.f, sb = 0.f;
#pragma unroll
      for (int rr = 0; rr < R; ++rr) {
        sa += red[(rr * 2 + h) * 16 + cc];
        sb += red[256 + (rr * 2 + h) * 16 + cc];
      }
      cx.BPART[((size_t)wr * cx.pstride + wg) * 32 + t] = make_float2(sa, sb);
    }
    return;
  }

  // ---- i == 0: stem backward (maxpool-bwd routed by the saved argmax, ReLU mask) + stem & block-0 wgrads ----
  const uint8_t* codep = cx.SCODE + img + r0 * 512;
#pragma unroll
  for (int j = 0; j < R / 2; ++j) {
    const int tt = wave + 4 * j, rr = tt >> 1, ch = 16 * (tt & 1) + c;
    float db = 0.f;
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      const int col = 4 * q + ii, po = (rr * 16 + col) * 32 + ch;
      const float g = gown[po] + acc[j][ii];
      const int code = codep[po];
      if (code & 4) {
        const int pos = code & 3;
        const int sr = 2 * rr + (pos >> 1), sc = 2 * col + (pos & 1);
        dsT[ch * DSP + sr * 32 + sc] = BF ? (TA)bfbits(g) : (TA)g;
        db += g;
      }
    }
    db += __shfl_xor(db, 16);
    db += __shfl_xor(db, 32);
    if (q == 0) red[tt * 16 + c] = db;
  }
  __syncthreads();
  float* sslab = cx.SSLAB + (size_t)wg * SSLAB_N;
  if (t < 32) {
    const int h = t >> 4, cc = t & 15;
    float s = 0.f;
#pragma unroll
    for (int rr = 0; rr < R; ++rr) s += red[(rr * 2 + h) * 16 + cc];
    sslab[1024 + t] = s;
  }
  // stem wgrad: D[co][k] = sum_p ds[p][co] * im2col[p][k]; wave -> tile (mt = wave&1, nt = wave>>1)
  {
    const int mt = wave & 1, nt = wave >> 1, kidx = 16 * nt + c, co = 16 * mt + c;
    const bool kv = kidx < 27;
    const int ci = kidx / 9, kh = (kidx % 9) / 3, kw = kidx % 3;
    const float* xb = xin + (kv ? ci * IRb * IW + kh * IW + kw : 0);
    f32x4 acc2 = z4();
    for (int s = 0; s < 2 * R; ++s) {
      if constexpr (BF) {
        const bf16x8 a = *(const bf16x8*)(dsT + co * DSP + s * 32 + 8 * q);
        bf16x8 b;
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) b[jj] = (__bf16)(kv ? xb[s * IW + 8 * q + jj] : 0.f);
        acc2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc2, 0, 0, 0);
      } else {
#pragma unroll
        for (int b2 = 0; b2 < 2; ++b2) {
          const f32x4 a = *(const f32x4*)(dsT + co * DSP + s * 32 + 16 * b2 + 4 * q);
#pragma unroll
          for (int st = 0; st < 4; ++st) {
            const float bv = kv ? xb[s * IW + 16 * b2 + 4 * q + st] : 0.f;
            acc2 = mfma4(a[st], bv, acc2);
          }
        }
      }
    }
    st4(sslab + ((wave * 64 + lane) << 2), acc2);
  }
  // block-0 trunk wgrad, in tile
  const int nw_blk = cx.B * (16 / RW);
  wgrad_core<BF, R>((const char*)dyT, DS0, (const char*)xT, XS0, cx.WSLAB + ((size_t)9 * nw_blk + wg) * WSLAB_N,
                    wave, lane);
}

template <bool BF, int R, int RW>
__global__ void __launch_bounds__(NT) k_bwd_block(Ctx cx, int i) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nparts = cx.B * (16 / R);
  int bid = blockIdx.x;
  if (bid < nparts) {
    dgrad_role<BF, R, RW>(cx, i, bid, smem);
    return;
  }
  bid -= nparts;
  if (i == 9) {
    fc_grads_role(cx, bid);
    return;
  }
  wgrad_role<BF, RW>(cx, i + 1, bid, smem);
}

// ============================================================================================================
// Gradient reduction + (optionally fused) SGD + derived weight layouts + bookkeeping.
// ============================================================================================================
template <bool BF>
__device__ __forceinline__ void put_w(void* dst, int idx, float w) {
  if constexpr (BF) ((unsigned short*)dst)[idx] = bfbits(w);
  else ((float*)dst)[idx] = w;
}

template <bool BF>
__global__ void __launch_bounds__(NT) k_reduce(Ctx cx, int nslab, int nsslab) {
  __shared__ f32x4 red[NT];
  const int t = threadIdx.x, bid = blockIdx.x;
  if (bid < N_TRUNK_RED_WG + N_STEM_RED_WG) {
    const bool stem = bid >= N_TRUNK_RED_WG;
    const int chunk = stem ? bid - N_TRUNK_RED_WG : bid;
    const int slot = t & 15, grp = t >> 4, e0 = chunk * 64 + slot * 4;
    const float* src = stem ? cx.SSLAB : cx.WSLAB;
    const int stride = stem ? SSLAB_N : WSLAB_N, cnt = stem ? nsslab : nslab;
    f32x4 s = z4();
    for (int k = grp; k < cnt; k += 16) s += ld4(src + (size_t)k * stride + e0);
    red[t] = s;
    __syncthreads();
    if (t < 16) {
      f32x4 tot = z4();
#pragma unroll
      for (int g = 0; g < 16; ++g) tot += red[g * 16 + t];
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) {
        const int e = chunk * 64 + t * 4 + ii;
        int pidx = -1, kind = 0, d0 = 0, d1 = 0;
        if (!stem) {
          const int tt = e >> 8, ln = (e >> 2) & 63, mt = tt & 1, nt = tt >> 1, tap = nt >> 1, cih = nt & 1;
          const int co = 16 * mt + 4 * (ln >> 4) + ii, ci = 16 * cih + (ln & 15);
          pidx = OFF_CONVW + co * 288 + ci * 9 + tap;
          kind = 1;
          d0 = (tap * 32 + co) * 32 + ci;
          d1 = ((8 - tap) * 32 + ci) * 32 + co;
        } else if (e < 1024) {
          const int tt = e >> 8, ln = (e >> 2) & 63, mt = tt & 1, nt = tt >> 1;
          const int co = 16 * mt + 4 * (ln >> 4) + ii, k = 16 * nt + (ln & 15);
          if (k < 27) {
            pidx = OFF_C1W + co * 27 + k;
            kind = 2;
            d0 = co * 32 + k;
          }
        } else if (e < 1056) {
          pidx = OFF_C1B + (e - 1024);
        }
        if (pidx < 0) continue;
        const float g = tot[ii];
        cx.grads[pidx] = g;
        if (cx.fuse_sgd) {
          const float w = cx.params[pidx] - cx.lr * g;
          cx.params[pidx] = w;
          if (kind == 1) {
            put_w<BF>(cx.wt_f, d0, w);
            put_w<BF>(cx.wt_d, d1, w);
          } else if (kind == 2) {
            put_w<BF>(cx.sw, d0, w);
          }
        }
      }
    }
    return;
  }
  const int ob = bid - N_TRUNK_RED_WG - N_STEM_RED_WG;
  const int nother = gridDim.x - N_TRUNK_RED_WG - N_STEM_RED_WG - 1;
  if (ob < nother) {  // SGD of fc1/fc2/BN (their grads were written directly by the backward kernels)
    constexpr int NA = BUCKET_A_END / 4, NBN = (OFF_C1W - OFF_BNW) / 4;
    for (int v = ob * NT + t; v < NA + NBN; v += nother * NT) {
      const int e = v < NA ? 4 * v : OFF_BNW + 4 * (v - NA);
      const f32x4 g = ld4(cx.grads + e);
      st4(cx.params + e, ld4(cx.params + e) - cx.lr * g);
    }
    return;
  }
  // bookkeeping workgroup
  if (t == 0) {
    float s = 0.f;
    for (int b = 0; b < cx.B; ++b) s += cx.HLOSS[b];
    *cx.loss_acc += (double)(s / (float)cx.B);
    *cx.cursor += cx.B;
    *cx.step_count += 1;
  }
  if (!cx.fuse_sgd && t < 64) {  // CC4: rank 0's running stats ride the bucket-B all-reduce (others add 0)
    const float v = t < 32 ? cx.rm[t] : cx.rv[t - 32];
    cx.grads[OFF_RS + t] = cx.rank == 0 ? v : 0.f;
  }
}

// SGD after the gradient all-reduce (world_size > 1), or mode 0 = derive weight layouts / init state only.
template <bool BF>
__global__ void __launch_bounds__(NT) k_apply_sgd(Ctx cx, int mode) {
  const int gid = blockIdx.x * NT + threadIdx.x, gsz = gridDim.x * NT;
  for (int e = gid; e < OFF_RS; e += gsz) {
    float w = cx.params[e];
    if (mode) {
      w -= cx.lr * cx.grads[e] * cx.inv_ws;
      cx.params[e] = w;
    }
    if (e >= OFF_CONVW && e < OFF_CONVW + 9216) {
      const int r = e - OFF_CONVW, co = r / 288, ci = (r / 9) % 32, tap = r % 9;
      put_w<BF>(cx.wt_f, (tap * 32 + co) * 32 + ci, w);
      put_w<BF>(cx.wt_d, ((8 - tap) * 32 + ci) * 32 + co, w);
    } else if (e >= OFF_C1W && e < OFF_C1W + 864) {
      const int r = e - OFF_C1W, co = r / 27, k = r % 27;
      put_w<BF>(cx.sw, co * 32 + k, w);
    }
  }
  if (gid < 64) {
    if (mode) cx.rs_base[gid] = cx.grads[OFF_RS + gid];
    else cx.rs_base[gid] = gid < 32 ? cx.rm[gid] : cx.rv[gid - 32];
  }
  if (!mode && gid < 32 * 5) put_w<BF>(cx.sw, (gid / 5) * 32 + 27 + gid % 5, 0.f);
}

// ------------------------------------------------------------------------------------------------------------
// explicit instantiations used by engine.cpp
// ------------------------------------------------------------------------------------------------------------
#define DCA_INST(BF, R, RW)                                                   \
  template __global__ void k_stem_block0<BF, R>(Ctx);                         \
  template __global__ void k_fwd_block<BF, R>(Ctx, int);                      \
  template __global__ void k_bwd_block<BF, R, RW>(Ctx, int);
DCA_INST(false, 4, 8)
DCA_INST(true, 4, 16)
DCA_INST(false, 2, 8)
DCA_INST(true, 2, 16)
template __global__ void k_head<4>(Ctx);
template __global__ void k_head<2>(Ctx);
template __global__ void k_reduce<false>(Ctx, int, int);
template __global__ void k_reduce<true>(Ctx, int, int);
template __global__ void k_apply_sgd<false>(Ctx, int);
template __global__ void k_apply_sgd<true>(Ctx, int);

}  // namespace dca
