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
constexpr int RED_CHUNK = 32;        // floats reduced per k_reduce workgroup (8 float4 slots x 32 slab groups)
constexpr int N_TRUNK_RED_WG = WSLAB_N / RED_CHUNK;  // 288
constexpr int N_STEM_RED_WG = SSLAB_N / RED_CHUNK;   // 34

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s4v __attribute__((ext_vector_type(4)));  // 4 bf16 bit patterns (16x16x16 MFMA operand)

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
  float* HPART;    // [nparts][32] per-tile partial fc1 pre-activations
  uint8_t* HCODE;  // [B][64][32] head max-pool argmax
  int pstride;     // FPART/BPART stride per block (>= max nparts)
  void* w1b;                   // [32][2048] bf16 copy of fc1.weight (persistent engine's head; kept by every SGD)
  void* swf;                   // [2 co half][3 k group][64 lanes][4] bf16 conv1 weights as 16x16x16 MFMA B fragments
  unsigned long long* stamps;  // [32 kernel slots][256 wg][8 stamps][2] (diagnostic DCA_STAMPS builds only)
  // sliced persistent engine (netresdeep_pks.hip): bf16 hi / lo splits of the conv weights in the kernel's LDS
  // record layout (record = 32 bf16, 64 B, 16-B chunks swizzled: pkw_elem), so a plane is staged by a straight
  // LDS-DMA copy; u16 offsets
  //   [0, 9216) fwd hi, record tap*32 + co, element ci | [9216, 18432) fwd lo |
  //   [18432, 27648) dgrad hi, record (8 - tap)*32 + ci, element co | [27648, 36864) dgrad lo |
  //   [36864, 38400) conv1 MFMA B fragments hi (swf_slot order) | [38400, 39936) lo
  unsigned short* pkw;
};
constexpr int PKW_REC = 32;             // u16 per record
constexpr int PKW_PLANE = 288 * PKW_REC;  // 9216
// u16 offset of element e of record r (chunk e >> 3 at position (e >> 3) ^ 2((r >> 2) & 1): netresdeep_pks.hip
// rec_chunk)
__host__ __device__ inline int pkw_elem(int r, int e) {
  return r * PKW_REC + ((((e >> 3) ^ ((r >> 1) & 2)) << 3) | (e & 7));
}
constexpr int PKW_DGRAD = 2 * PKW_PLANE;
constexpr int PKW_STEM = 4 * PKW_PLANE;   // 46080
constexpr int PKW_N = PKW_STEM + 2 * 1536;

// In-kernel phase stamps (diagnostic build, -DDCA_STAMPS): thread 0 of each workgroup records
// (s_memtime, s_memrealtime) at phase boundaries.  Never compiled into the production library.
#ifdef DCA_STAMPS
#define DCA_STAMP(cx, slot, wg, k)                                                                        \
  do {                                                                                                     \
    if (threadIdx.x == 0 && (wg) < 256) {                                                                  \
      unsigned long long t0_, t1_;                                                                         \
      __builtin_amdgcn_sched_barrier(0);                                                                   \
      asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0_), "=s"(t1_)::"memory"); \
      __builtin_amdgcn_sched_barrier(0);                                                                   \
      unsigned long long* p_ = (cx).stamps + ((((size_t)(slot) * 256 + (wg)) * 8 + (k)) << 1);           \
      p_[0] = t0_;                                                                                         \
      p_[1] = t1_;                                                                                         \
    }                                                                                                      \
  } while (0)
#else
#define DCA_STAMP(cx, slot, wg, k) \
  do {                             \
  } while (0)
#endif

// sample id of image n of the current batch, clamped into range
__device__ __forceinline__ int sample_id(const Ctx& cx, int n) {
  int pos = *cx.cursor + n;
  pos = pos < 0 ? 0 : (pos >= cx.n_idx ? cx.n_idx - 1 : pos);
  int id = cx.indices[pos];
  return id < 0 ? 0 : (id >= cx.n_data ? cx.n_data - 1 : id);
}

// conv1 weight element (co, k = ci * 9 + tap) -> its slot in the persistent stem's MFMA B fragments
__device__ __forceinline__ int swf_slot(int co, int k) {
  const int ci = k / 9, tap = k % 9;
  return (((co >> 4) * 3 + (tap >> 2)) * 64 + 16 * (tap & 3) + (co & 15)) * 4 + ci;
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

namespace dca {
constexpr int RED_F = 1600;  // floats of per-workgroup reduction scratch in LDS
// Dynamic-LDS plan of every kernel, shared by the device carve-up and the host launch sizes (bytes; every
// region a multiple of 16 so carve offsets stay 16-byte aligned -- cdna guide Guideline 17).
template <bool BF, int R, int RW>
struct LdsPlan {
  static constexpr size_t RB = BF ? 64 : 128, ESZ = BF ? 2 : 4, PADE = 16 / ESZ, RR = R + 2;
  static constexpr size_t RED = RED_F * 4;  // reduction scratch
  static constexpr size_t IR = 2 * RR + 2, IW = 34;
  static constexpr size_t stem = 288 * RB + RR * 18 * RB + 3 * IR * IW * 4 + 32 * 32 * ESZ + 32 * 4 + RED + 32 * 4;
  static constexpr size_t fwd = 288 * RB + RR * 18 * RB + RED + 4 * 32 * 4;
  static constexpr size_t head1 = R * 512 * 4 + 128 * R * 4 + RED + 5 * 32 * 4;
  static constexpr size_t head2 = 256 * 4 + 320 * 4 + 96 * 4 + 128 * R + 128 * R * 4 + RED + 4 * 32 * 4;
  static constexpr size_t dgrad = 288 * RB + RR * 18 * RB + 2 * R * 512 * 4 + RED + 11 * 32 * 4;
  static constexpr size_t DS0 = R * 16 + PADE, XS0 = RR * 16 + PADE, IRb = 2 * R + 2, DSP = 2 * R * 32 + PADE;
  static constexpr size_t dgrad0 = dgrad + 32 * DS0 * ESZ + 3 * 32 * XS0 * ESZ + 3 * IRb * IW * 4 + 32 * DSP * ESZ;
  static constexpr size_t DS = RW * 16 + PADE, XS = (RW + 2) * 16 + PADE;
  static constexpr size_t wgrad = 32 * DS * ESZ + 3 * 32 * XS * ESZ;
  static constexpr size_t fc = (64 * 32 + 64 * 64 + 64 * 32 + 64 * 16) * 4;  // batch <= 64
};
constexpr int BMAX_LIMIT = 64;  // per-rank batch supported by the unrolled staging paths
}  // namespace dca
