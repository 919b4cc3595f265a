// Shared definitions for the NetResDeep CDNA4 (gfx950) training engine.
//
// Layout conventions (see README "Engine design"):
//   * activations are NHWC fp32: [B][16][16][32]; the stem input is the uint8 CIFAR image CHW [3][32][32]
//   * parameters live in ONE flat fp32 buffer (the module's nn.Parameters are views into it, so the state_dict
//     always reflects what the kernels train); gradients use the same layout.  The layout is ordered by
//     gradient-ready time so DDP buckets are contiguous slices: bucket A = fc1/fc2 (ready after the head),
//     bucket B = trunk conv + BN + stem (ready after the last backward kernel) + the BN running-stat segment.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dca {

constexpr int C = 32;     // channels of every trunk tensor (NetResDeep n_chans1)
constexpr int NT = 256;   // threads per workgroup (4 waves of 64)
constexpr int NBLK = 10;  // ResBlock applications (n_blocks)

// ---- flat parameter layout (floats).  Every tensor starts on a 16-byte boundary. -----------------------
constexpr int OFF_FC1W = 0;        // [32][2048]
constexpr int OFF_FC2W = 65536;    // [10][32]
constexpr int OFF_FC1B = 65856;    // [32]
constexpr int OFF_FC2B = 65888;    // [10] (+2 pad)
constexpr int BUCKET_A_END = 65900;
constexpr int OFF_CONVW = 65900;   // [32][32][3][3]  (the ONE shared trunk conv)
constexpr int OFF_BNW = 75116;     // [32]
constexpr int OFF_BNB = 75148;     // [32]
constexpr int OFF_C1W = 75180;     // [32][3][3][3]
constexpr int OFF_C1B = 76044;     // [32]
constexpr int OFF_RS = 76076;      // [64] running_mean|running_var segment (grads buffer only: CC4 broadcast)
constexpr int FLAT_N = 76140;
constexpr int FLAT_ALLOC = 76160;  // padded allocation

constexpr int WSLAB_N = 9216;      // trunk-conv wgrad partial (MFMA fragment order)
constexpr int SSLAB_N = 1088;      // stem wgrad partial: 1024 fragment (32co x 32k) + 32 bias + pad
constexpr int N_FC_WG = 32;        // workgroups computing the fc1/fc2 weight gradients (inside bwd block 9)
constexpr int N_TRUNK_RED_WG = 144;  // 9216 / 64
constexpr int N_STEM_RED_WG = 17;    // 1088 / 64

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// Everything a kernel needs, passed by value (kernarg segment).
struct Ctx {
  int B;          // images in this step (ragged last batch supported)
  int ws, rank;   // data-parallel world size / rank
  int fuse_sgd;   // 1: the reduction kernel applies SGD directly (world_size 1)
  float lr, bn_mom, bn_eps, inv_ws;
  float* params;  // flat fp32 [FLAT_ALLOC]
  float* grads;   // flat fp32 [FLAT_ALLOC]
  void* wt_f;     // derived conv weight, forward   [9 tap][32 co][32 ci]  (compute type)
  void* wt_d;     // derived conv weight, dgrad     [9 tap][32 ci][32 co]  (flipped taps)
  void* sw;       // derived stem weight            [32 co][32 k]  (k = ci*9+kh*3+kw, 27..31 zero)
  float* rm;      // BN running_mean (module buffer)
  float* rv;      // BN running_var  (module buffer)
  long long* nbt; // BN num_batches_tracked
  float* rs_base; // [64] rank-0 running stats at the start of the step (world_size > 1)
  const uint8_t* data;  // [N][3][32][32] uint8 dataset, device resident
  const int* labels;    // [N]
  const int* indices;   // [epoch_len] sampler order for this rank
  int* cursor;          // device scalar: position of this step's batch in `indices`
  int n_data;           // images in `data` (gathers are clamped: a bad cursor must never fault the GPU)
  int n_idx;            // capacity of `indices`
  double* loss_acc;     // device scalar: sum of per-step mean losses
  int* step_count;      // device scalar
  // activations & scratch
  float* X;        // [10][B][16][16][32]   block inputs x_0..x_9
  float* Y;        // [10][B][16][16][32]   conv outputs y_0..y_9
  float* DY;       // [10][B][16][16][32]   BN-backward outputs dy_1..dy_9 (for the deferred wgrad)
  float* G;        // [2][B][16][16][32]    residual-stream gradient ping-pong
  uint8_t* SCODE;  // [B][16][16][32]       stem pool argmax (bits 0-1) | relu-positive (bit 2)
  float2* FPART;   // [10][nparts][32]      forward BN partials (mean, M2) per tile
  float2* STATS;   // [10][32]              (mean, invstd)
  float2* BPART;   // [2][nparts][32]       backward BN partials (sum dz, sum dz*xhat)
  float* WSLAB;    // [nslab][9216]         trunk wgrad partials
  float* SSLAB;    // [nparts][1088]        stem wgrad partials
  float* HP;       // [B][2048] pooled features (fc1 input)
  float* HH;       // [B][32]   relu(fc1)
  float* HDH;      // [B][32]   d fc1-preactivation
  float* HDL;      // [B][10]   d logits
  float* HLOSS;    // [B]       per-image CE loss
  int pstride;     // FPART/BPART stride per block (>= max nparts)
};

// sample id of image n of the current batch, clamped into range
__device__ __forceinline__ int sample_id(const Ctx& cx, int n) {
  int pos = *cx.cursor + n;
  pos = pos < 0 ? 0 : (pos >= cx.n_idx ? cx.n_idx - 1 : pos);
  int id = cx.indices[pos];
  return id < 0 ? 0 : (id >= cx.n_data ? cx.n_data - 1 : id);
}

__device__ __forceinline__ unsigned short f2bf(float f) {
  unsigned u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);  // round to nearest even (finite inputs)
  return (unsigned short)(u >> 16);
}
__device__ __forceinline__ unsigned pack2bf(float a, float b) {
  return (unsigned)f2bf(a) | ((unsigned)f2bf(b) << 16);
}

}  // namespace dca
