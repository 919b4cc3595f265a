// General MFMA GEMM for the ops layer (ops/): C[M,N] = alpha * sum_k A(m,k) * B(n,k)  (+ bias[n]) (+ beta*C) (ReLU)
//
// Operands are bf16 (v_mfma_f32_16x16x32_bf16) or OCP fp8 e4m3 (v_mfma_scale_f32_16x16x128_f8f6f4 with unit
// E8M0 block scales: the MX-scaled form is the one that runs at the fp8 rate on CDNA4; the per-tensor fp8
// scales are folded into alpha).  Accumulation is fp32; the output is fp32 or bf16.
//
// Operand access: A(m,k) = A[m*lda + k] (ta = 0, K contiguous -- the MFMA-natural "NT" form) or A[k*lda + m]
// (ta = 1, bf16 only: the loader transposes while writing LDS); B(n,k) likewise with tb.  This covers, for a
// channels-last 1x1 convolution / linear layer with X[M,Cin], W[Cout,Cin], dY[M,Cout]:
//   forward  Y  = X  . W^T   (ta 0, tb 0)      dgrad dX = dY . W   (ta 0, tb 1)
//   wgrad    dW = dY^T . X   (ta 1, tb 1, split-K over the pixel dimension into an fp32 slab + reduce kernel)
//
// Tiling (CDNA4, 64-wide waves): 128x128 output tile per 256-thread workgroup (4 waves as 2x2, each 64x64 =
// 4x4 MFMA 16x16 tiles, 64 fp32 accumulator VGPRs), K-tile = 128 bytes per row (64 bf16 / 128 fp8), LDS
// double-buffered (64 KiB -> 2 workgroups per CU), register-staged prefetch of tile k+1 during the MFMAs of
// tile k, one barrier per K-tile.  LDS rows are 128 B with 16-B chunks XOR-swizzled by (row >> 1) & 7, so a
// ds_read_b128 of 16 lanes (16 rows, one chunk) covers all 64 banks once.  Workgroup ids are remapped so that
// consecutive output tiles (which share their A rows) run on the same XCD and share its L2.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace dca {
namespace ops {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef int i32x8 __attribute__((ext_vector_type(8)));

constexpr int GT = 256;          // threads per GEMM workgroup
constexpr int GBM = 128;
constexpr int GBK_BYTES = 128;   // bytes of K per row per K-tile
constexpr int G_TILE_BYTES = GBM * GBK_BYTES;  // 16 KiB per operand per buffer


struct GemmArgs {
  const void* A;
  const void* B;
  void* C;             // output (fp32 or bf16), row stride ldc
  const float* bias;   // [N] or null
  float* ws;           // split-K slab [splits][M][N] fp32 (splits > 1)
  int M, N, K;         // K in elements
  int lda, ldb, ldc;   // strides in elements
  float alpha, beta;   // beta: C += beta * C_old (fp32/bf16 read of the output)
  int ta, tb;          // transposed operand access (bf16 only)
  int fp8;             // 1: operands are fp8 e4m3 (ta = tb = 0)
  int relu, out_bf16;
  int splits, k_per_split;  // split-K (k_per_split a multiple of the K-tile)
  const float* alpha_dev;   // optional device-side factor (fp8 per-tensor scales: no host sync)
  // implicit-GEMM convolution (bf16, NHWC input with C % 8 == 0; no im2col buffer):
  //   conv = 1: A(m = output pixel, k = (kh*KW + kw)*C + c) gathered from A = x        (forward / dgrad)
  //   conv = 2: B(n = (kh*KW + kw)*C + c, k = output pixel) gathered from B = x        (weight gradient)
  int conv;
  int cN, cH, cW, cC, cKH, cKW, cS, cP, cHo, cWo;
  // fused BatchNorm statistics of the output (splits == 1): col_stats[tile_m][N] = (sum, sumsq) over the tile's
  // rows of (out - stats_shift[col]), the layout k_bn_finalize reduces
  float2* col_stats;
  const float* stats_shift;
  // fp8 per-tensor scales as device amax bits (q = x * 448 / amax): alpha *= (amax_a / 448) * (amax_b / 448)
  const unsigned* amax_a;
  const unsigned* amax_b;
  // weight-gradient layout remap (wperm_T > 0): output column n = tap * wperm_Cpad + c of the GEMM is stored at
  // row * (wperm_C * wperm_T) + c * wperm_T + tap -- torch's [Cout][Cin][KH][KW] -- and dropped for padded
  // channels (c >= wperm_C); always through the fp32 slab + reduce kernel.
  int wperm_C, wperm_Cpad, wperm_T;
  // single = 1: one LDS operand buffer (2 barriers per K-tile) so short-K GEMMs run with half the LDS and
  // twice the workgroups per CU (set by the launcher when a split has <= 4 K-tiles)
  int single;
  int stages;  // k_gemm_glds: LDS buffers in the K pipeline (2..4; tiles in flight = stages - 1), when !single
  // output row remap (orow_S > 0): GEMM row m = pixel (n, i, j) of an orow_Ho x orow_Wo grid is stored at row
  // (n * orow_H + orow_S * i + orow_ph) * orow_W + orow_S * j + orow_pw of C -- the sub-pixel (parity class)
  // input gradients of a strided convolution written straight into dX
  int orow_S, orow_ph, orow_pw, orow_H, orow_W, orow_Ho, orow_Wo;
  // masked accumulation source (beta != 0, bf16 output): C = alpha A B + beta * (beta_src * mask) instead of
  // beta * C_old -- the residual gradient dout * [ReLU(bn3 + r) > 0] of a bottleneck, read from dout and the bn3
  // forward's bit mask (bit j of byte e / 8: element e of beta_src's [M][ldc] layout) so bn3's backward never writes
  // it out.  k_gemm_stream applies it in the epilogue; other kernels get a masked copy into C first (dca_ops_gemm).
  const void* beta_src;
  const uint8_t* beta_mask;
};

__device__ __forceinline__ float amax_scale(const unsigned* a) {
  if (!a) return 1.f;
  const float v = __uint_as_float(*a);
  return v > 0.f ? v * (1.f / 448.f) : 1.f;
}
__device__ __forceinline__ float gemm_alpha(const GemmArgs& g) {
  return g.alpha * (g.alpha_dev ? *g.alpha_dev : 1.f) * amax_scale(g.amax_a) * amax_scale(g.amax_b);
}

__device__ __forceinline__ int lds_off(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }

__device__ __forceinline__ unsigned short f2bf_rne(float f) {
  return __builtin_bit_cast(unsigned short, (__bf16)f);
}
__device__ __forceinline__ float bf2f(unsigned short h) { return __uint_as_float((unsigned)h << 16); }

// Stage of one operand tile held in registers between its global load and its LDS write (NI x 16 B per thread:
// 4 for a 128-row tile, 2 for a 64-row tile).
template <int NI>
struct StageT {
  uint4 v[NI];
};
using Stage = StageT<4>;

// Non-transposed operand: rows r0.., K bytes kb0.. (row-major, K contiguous).  Thread t owns chunks
// idx = t + 256 i: row idx >> 3, chunk idx & 7.  Rows past R are clamped (their results are never stored);
// bytes past the K range are zero.  A chunk that straddles the K end, or a row stride that is not 16-B
// aligned, takes the element-wise path (esz-byte loads).
template <int ESZ, int NI = 4>
__device__ __forceinline__ void load_nt(StageT<NI>& s, const char* base, int r0, int R, size_t ld_bytes, int kb0,
                                        int kb_end) {
  const bool vec_ok = (ld_bytes & 15) == 0;
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int idx = threadIdx.x + GT * i, row = idx >> 3, ch = idx & 7;
    int rg = r0 + row;
    rg = rg < R ? rg : R - 1;
    const int kb = kb0 + ch * 16;
    const char* rowp = base + (size_t)rg * ld_bytes;
    if (vec_ok && kb + 16 <= kb_end) {
      s.v[i] = *(const uint4*)(rowp + kb);
    } else {
      unsigned w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
      for (int e = 0; e < 16 / ESZ; ++e) {
        const int b = kb + e * ESZ;
        unsigned x = 0u;
        if (b < kb_end) x = ESZ == 2 ? (unsigned)*(const unsigned short*)(rowp + b) : (unsigned)*(const uint8_t*)(rowp + b);
        w[(e * ESZ) >> 2] |= x << (((e * ESZ) & 3) * 8);
      }
      s.v[i] = uint4{w[0], w[1], w[2], w[3]};
    }
  }
}
template <int NI = 4>
__device__ __forceinline__ void store_nt(const StageT<NI>& s, char* lds) {
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int idx = threadIdx.x + GT * i;
    *(uint4*)(lds + lds_off(idx >> 3, idx & 7)) = s.v[i];
  }
}
// Transposed bf16 operand: element (r, k) at base[k*ld + r].  Thread t owns 8 consecutive r (group t & 15) at 4
// consecutive k (4 (t >> 4) .. +3): 4 row loads of 16 B, transposed in registers into 8 LDS writes of 8 B (the
// 4 k values of one r).  Vector loads where the 8 rows are in range and 16-B aligned, element-wise otherwise
// (rows past R clamped, never stored).  s.v[i] = the 8 r values at k = k0 + 4 (t >> 4) + i.
__device__ __forceinline__ void load_t(Stage& s, const unsigned short* base, int r0, int R, size_t ld, int k0,
                                       int k_end) {
  const bool vec_ok = (ld & 7) == 0;
  const int rg = r0 + (threadIdx.x & 15) * 8;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = k0 + 4 * (threadIdx.x >> 4) + i;
    if (k >= k_end) {
      s.v[i] = uint4{0u, 0u, 0u, 0u};
    } else if (vec_ok && rg + 8 <= R) {
      s.v[i] = *(const uint4*)(base + (size_t)k * ld + rg);
    } else {
      unsigned w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int r = rg + e < R ? rg + e : R - 1;
        w[e >> 1] |= (unsigned)base[(size_t)k * ld + r] << ((e & 1) * 16);
      }
      s.v[i] = uint4{w[0], w[1], w[2], w[3]};
    }
  }
}
__device__ __forceinline__ void store_t(const Stage& s, char* lds) {
  const int kq = 4 * (threadIdx.x >> 4), rb = (threadIdx.x & 15) * 8;
  const unsigned w[4][4] = {{s.v[0].x, s.v[0].y, s.v[0].z, s.v[0].w}, {s.v[1].x, s.v[1].y, s.v[1].z, s.v[1].w},
                            {s.v[2].x, s.v[2].y, s.v[2].z, s.v[2].w}, {s.v[3].x, s.v[3].y, s.v[3].z, s.v[3].w}};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int sh = (j & 1) * 16;
    const unsigned e0 = (w[0][j >> 1] >> sh) & 0xffffu, e1 = (w[1][j >> 1] >> sh) & 0xffffu;
    const unsigned e2 = (w[2][j >> 1] >> sh) & 0xffffu, e3 = (w[3][j >> 1] >> sh) & 0xffffu;
    *(uint2*)(lds + lds_off(rb + j, kq >> 3) + (kq & 7) * 2) = uint2{e0 | (e1 << 16), e2 | (e3 << 16)};
  }
}

// x / d and x % d for 0 <= x < 2^24 by a float reciprocal and one correction (a runtime-divisor integer division
// is ~20-40 instructions; these decodes run once per tile row)
__device__ __forceinline__ int fdiv_rc(int x, int d, float inv, int& r) {
  int q = (int)((float)x * inv);
  r = x - q * d;
  if (r < 0) {
    --q;
    r += d;
  }
  if (r >= d) {
    ++q;
    r -= d;
  }
  return q;
}
// valid-tap mask of an implicit-conv row whose window starts at (ih0, iw0): bit kh * KW + kw, from the valid
// kh / kw ranges (rep = sum over kh of 1 << kh * KW spreads the kw bits over the kernel rows)
__device__ __forceinline__ unsigned tap_mask(int ih0, int iw0, int H, int W, int KH, int KW, unsigned rep) {
  const int khlo = ih0 < 0 ? -ih0 : 0, khhi = min(KH, H - ih0);
  const int kwlo = iw0 < 0 ? -iw0 : 0, kwhi = min(KW, W - iw0);
  const unsigned long long rows =
      khhi > khlo ? ((1ull << (khhi * KW)) - 1ull) & ~((1ull << (khlo * KW)) - 1ull) : 0ull;
  const unsigned cols = kwhi > kwlo ? ((1u << kwhi) - 1u) & ~((1u << kwlo) - 1u) : 0u;
  return (unsigned)rows & (cols * rep);
}

// Implicit-GEMM gathers.  Per-thread row decompositions are computed once per tile (the rows a thread loads
// are fixed across the K loop); every load is unconditional from a clamped address, then selected to zero.
struct ConvRows {  // conv = 1: the 4 output pixels (A rows) this thread loads
  int nh[4], ih[4], iw[4];
};
__device__ __forceinline__ void conv_rows(ConvRows& cr, const GemmArgs& g, int m0) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int m = m0 + ((threadIdx.x + GT * i) >> 3);
    m = m < g.M ? m : g.M - 1;
    int ow, t, oh, n;
    if (g.M < (1 << 24)) {  // float-reciprocal decode (runtime-divisor divisions are ~20-40 instructions each)
      t = fdiv_rc(m, g.cWo, 1.f / (float)g.cWo, ow);
      n = fdiv_rc(t, g.cHo, 1.f / (float)g.cHo, oh);
    } else {
      ow = m % g.cWo, t = m / g.cWo, oh = t % g.cHo, n = t / g.cHo;
    }
    cr.nh[i] = n * g.cH;
    cr.ih[i] = oh * g.cS - g.cP;
    cr.iw[i] = ow * g.cS - g.cP;
  }
}
// ESZ = 2: 8 bf16 channels of one tap per 16-B chunk (C % 8 == 0); ESZ = 1: 16 fp8 channels (C % 16 == 0)
template <int ESZ>
__device__ __forceinline__ void load_conv_a(Stage& s, const char* x, const ConvRows& cr, const GemmArgs& g, int k0,
                                            int k_end) {
  const int k = k0 + (threadIdx.x & 7) * (16 / ESZ);  // one tap per chunk
  int c, kw;  // (K < 2^24: checked by the launcher for implicit convs)
  const int tap = fdiv_rc(k, g.cC, 1.f / (float)g.cC, c), kh = fdiv_rc(tap, g.cKW, 1.f / (float)g.cKW, kw);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int h = cr.ih[i] + kh, w = cr.iw[i] + kw;
    const bool ok = k < k_end && h >= 0 && h < g.cH && w >= 0 && w < g.cW;
    const long off = ok ? (((long)(cr.nh[i] + h) * g.cW + w) * g.cC + c) * ESZ : 0;
    const uint4 v = *(const uint4*)(x + off);
    s.v[i] = ok ? v : uint4{0u, 0u, 0u, 0u};
  }
}
struct ConvCols {  // conv = 2: the 4 column groups (8 consecutive n = 8 channels of one tap) this thread loads
  int kh[4], kw[4], c[4];
  bool in[4];
};
__device__ __forceinline__ void conv_cols(ConvCols& cc, const GemmArgs& g, int n0) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int n = n0 + ((threadIdx.x + GT * i) & 15) * 8;
    const int tap = n / g.cC;
    cc.c[i] = n - tap * g.cC;
    cc.kh[i] = tap / g.cKW;
    cc.kw[i] = tap - cc.kh[i] * g.cKW;
    cc.in[i] = n < g.N;
  }
}
__device__ __forceinline__ void load_conv_b(Stage& s, const unsigned short* x, const ConvCols& cc, const GemmArgs& g,
                                            int k0, int k_end) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int p = k0 + 4 * (threadIdx.x >> 4) + i;  // output pixel = GEMM k (load_t's thread layout)
    const bool pin = p < k_end;
    p = pin ? p : k0;
    const int ow = p % g.cWo, t = p / g.cWo, oh = t % g.cHo, n = t / g.cHo;
    const int h = oh * g.cS - g.cP + cc.kh[i], w = ow * g.cS - g.cP + cc.kw[i];
    const bool ok = pin && cc.in[i] && h >= 0 && h < g.cH && w >= 0 && w < g.cW;
    const long off = ok ? ((long)(n * g.cH + h) * g.cW + w) * g.cC + cc.c[i] : 0;
    const uint4 v = *(const uint4*)(x + off);
    s.v[i] = ok ? v : uint4{0u, 0u, 0u, 0u};
  }
}

__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

// (tm, tn) of the t-th tile in grouped order: bands of GROUP tile rows, column-major inside a band, so the tiles
// one XCD runs together (consecutive t after xcd_remap) cover a compact block of C: with 32 x 32 tiles an XCD's
// 64 co-resident tiles share 8 A row-tiles and 8 B column-tiles instead of 2 and 32
constexpr int TILE_GROUP = 8;
__device__ __forceinline__ void tile_coords(int t, int ntm, int ntn, int& tm, int& tn) {
  const int per = TILE_GROUP * ntn, band = t / per, first = band * TILE_GROUP;
  const int rows = ntm - first < TILE_GROUP ? ntm - first : TILE_GROUP, r = t - band * per;
  tm = first + r % rows;
  tn = r / rows;
}

template <int BN_>
struct GemmTile {
  static constexpr int B_BYTES = BN_ * GBK_BYTES;              // B tile per buffer
  static constexpr int BUF = G_TILE_BYTES + B_BYTES;           // A + B per buffer
  static constexpr int LDS = 2 * BUF;                          // double buffered
  static constexpr int EPI = GBM / 2 * BN_ * 4;                // fp32 epilogue staging: one 64-row half
  static constexpr int LDS_SINGLE = BUF > EPI ? BUF : EPI;     // single-buffer launch
  static constexpr int NF = BN_ / 32;                          // 16-wide MFMA column fragments per wave
  static constexpr int WCW = BN_ / 2;                          // columns per wave (2 x 2 waves)
  static_assert(LDS >= EPI, "epilogue half tile must fit in the K-loop LDS");
};

// BN_ = 128: the general tile.  BN_ = 64: narrow-N GEMMs (e.g. 64-channel convolutions) -- half the B tile, no
// wasted MFMA columns, 48 KiB LDS (3 workgroups per CU); its B operand must be K-contiguous (no tb / conv 2).
// K loop: register prefetch of tile k+1 during the MFMAs of tile k, written to the other LDS buffer after them.
// (A two-tile-deep prefetch measured neutral to 20 % slower: 196 VGPRs = 1 wave per SIMD, bench/gemm_bench.py.)
// Shared epilogue of the GEMM kernels (acc = this wave's 64 x BN_/2 fp32 fragments of the 128 x BN_ tile).
template <int BN_, int NW>
struct WaveGrid {  // NW waves as 2 (rows of 64) x NW/2 (column slices) over the 128 x BN_ tile
  static constexpr int WC = NW / 2, WCW = BN_ / WC, NF = WCW / 16, NT = NW * 64;
  static_assert(NF >= 1, "bad wave grid");
};

template <int BN_, int NW = 4>
__device__ __forceinline__ void gemm_epilogue(const GemmArgs& g, f32x4 (&acc)[4][WaveGrid<BN_, NW>::NF], char* smem,
                                              int m0, int n0, int tm, int ksplit) {
  using T = WaveGrid<BN_, NW>;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wr = wave / T::WC, wc = wave % T::WC;
  // Epilogue.  Split-K partials go straight to the fp32 slab.  Otherwise the 128x128 fp32 tile is staged in
  // LDS (the K-loop buffers are free: 64 KiB exactly; 16-column groups XOR-swizzled by (row >> 2) & 3 so the
  // fragment writes of one instruction hit distinct banks), then written back row-contiguously, 16 B per lane,
  // with alpha / bias / beta / ReLU applied -- and, when asked, the per-column BN partial sums of the tile.
  if (g.splits > 1 || g.wperm_T > 0) {
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < T::NF; ++n) {
        const int col = n0 + wc * T::WCW + n * 16 + (lane & 15);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int row = m0 + wr * 64 + m * 16 + (lane >> 4) * 4 + j;
          if (row < g.M && col < g.N) g.ws[((size_t)ksplit * g.M + row) * g.N + col] = acc[m][n][j];
        }
      }
    return;
  }
  // Two 64-row halves (32 KiB of fp32 staging for a 128-column tile): the waves owning rows half*64.. stage
  // their fragments, then all 256 threads write 8 columns (one 16-B bf16 / two 16-B fp32 stores) per row.
  float* ct = (float*)smem;
  auto cidx = [](int r, int c) { return r * BN_ + (c ^ (((r >> 2) & 3) << 4)); };
  const float alpha = gemm_alpha(g);
  constexpr int CG = BN_ / 8, RL = T::NT / CG;  // column groups of 8, row lanes
  const int cg = threadIdx.x % CG, col0 = n0 + cg * 8;
  float bias8[8], shift8[8], s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int col = min(col0 + e, g.N - 1);
    bias8[e] = g.bias ? g.bias[col] : 0.f;
    shift8[e] = g.col_stats ? g.stats_shift[col] : 0.f;
    s1[e] = s2[e] = 0.f;
  }
  const bool full8 = col0 + 8 <= g.N && (g.ldc & 7) == 0;
#pragma unroll 1
  for (int half = 0; half < 2; ++half) {
    if (wr == half) {
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < T::NF; ++n)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            ct[cidx(m * 16 + (lane >> 4) * 4 + j, wc * T::WCW + n * 16 + (lane & 15))] = acc[m][n][j];
    }
    __syncthreads();
    for (int r = 0; r < GBM / 2 / RL; ++r) {
      const int lr = threadIdx.x / CG + RL * r, row = m0 + half * 64 + lr;
      if (row >= g.M || col0 >= g.N) continue;
      const f32x4 a0 = *(const f32x4*)(ct + cidx(lr, cg * 8)), a1 = *(const f32x4*)(ct + cidx(lr, cg * 8 + 4));
      const float av[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
      float v[8];
      size_t orow = (size_t)row;
      if (g.orow_S > 0) {
        const int j = row % g.orow_Wo, t = row / g.orow_Wo, i = t % g.orow_Ho, n = t / g.orow_Ho;
        orow = ((size_t)n * g.orow_H + g.orow_S * i + g.orow_ph) * g.orow_W + g.orow_S * j + g.orow_pw;
      }
      const size_t o = orow * g.ldc + col0;
      float old[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (g.beta != 0.f) {  // accumulate into the existing output: one 16-B (two for fp32) load per row chunk
        if (full8 && g.out_bf16) {
          const uint4 u = *(const uint4*)((const unsigned short*)g.C + o);
          const unsigned w4[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
          for (int e = 0; e < 8; ++e) old[e] = __uint_as_float((w4[e >> 1] >> ((e & 1) * 16)) << 16);
        } else if (full8) {
          const f32x4 a = *(const f32x4*)((const float*)g.C + o), b = *(const f32x4*)((const float*)g.C + o + 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            old[e] = a[e];
            old[e + 4] = b[e];
          }
        } else {
          for (int e = 0; e < 8 && col0 + e < g.N; ++e)
            old[e] = g.out_bf16 ? bf2f(((const unsigned short*)g.C)[o + e]) : ((const float*)g.C)[o + e];
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float x = av[e] * alpha + bias8[e] + g.beta * old[e];
        if (g.relu) x = x > 0.f ? x : 0.f;
        v[e] = x;
      }
      if (g.out_bf16) {
        unsigned short h[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) h[e] = f2bf_rne(v[e]);
        if (g.col_stats) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {  // statistics of the values as stored (bf16)
            const float d = bf2f(h[e]) - shift8[e];
            s1[e] += d;
            s2[e] += d * d;
          }
        }
        if (full8) {
          *(uint4*)((unsigned short*)g.C + o) =
              uint4{h[0] | ((unsigned)h[1] << 16), h[2] | ((unsigned)h[3] << 16), h[4] | ((unsigned)h[5] << 16),
                    h[6] | ((unsigned)h[7] << 16)};
        } else {
          for (int e = 0; e < 8 && col0 + e < g.N; ++e) ((unsigned short*)g.C)[o + e] = h[e];
        }
      } else {
        if (g.col_stats) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float d = v[e] - shift8[e];
            s1[e] += d;
            s2[e] += d * d;
          }
        }
        if (full8) {
          *(f32x4*)((float*)g.C + o) = f32x4{v[0], v[1], v[2], v[3]};
          *(f32x4*)((float*)g.C + o + 4) = f32x4{v[4], v[5], v[6], v[7]};
        } else {
          for (int e = 0; e < 8 && col0 + e < g.N; ++e) ((float*)g.C)[o + e] = v[e];
        }
      }
    }
    __syncthreads();
  }
  if (g.col_stats) {  // combine the row lanes of each column group (fixed order), one float2 per column
    float2* red = (float2*)smem;  // [RL row lanes][BN_ cols]
#pragma unroll
    for (int e = 0; e < 8; ++e) red[(threadIdx.x / CG) * BN_ + cg * 8 + e] = float2{s1[e], s2[e]};
    __syncthreads();
    if (threadIdx.x < BN_) {
      const int col = n0 + threadIdx.x;
      float2 t = red[threadIdx.x];
      for (int k = 1; k < RL; ++k) {
        t.x += red[k * BN_ + threadIdx.x].x;
        t.y += red[k * BN_ + threadIdx.x].y;
      }
      if (col < g.N) g.col_stats[(size_t)tm * g.N + col] = t;
    }
  }
}

template <bool FP8, int BN_>
__global__ void __launch_bounds__(GT) k_gemm(GemmArgs g) {
  using T = GemmTile<BN_>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int ntm = (g.M + GBM - 1) / GBM, ntn = (g.N + BN_ - 1) / BN_;
  const int tile = xcd_remap(blockIdx.x, ntm * ntn);
  int tm, tn;
  tile_coords(tile, ntm, ntn, tm, tn);
  const int m0 = tm * GBM, n0 = tn * BN_;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wr = wave >> 1, wc = wave & 1;
  constexpr int ESZ = FP8 ? 1 : 2;
  const int ksplit = blockIdx.y;
  const int k_begin = ksplit * g.k_per_split;
  const int k_end = min(g.K, k_begin + g.k_per_split);
  constexpr int KT = GBK_BYTES / ESZ;  // elements per K-tile
  const int nk = (k_end - k_begin + KT - 1) / KT;

  f32x4 acc[4][T::NF];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < T::NF; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  ConvRows cr;
  ConvCols cc;
  if (g.conv == 1) conv_rows(cr, g, m0);
  if constexpr (BN_ == 128) {
    if (g.conv == 2) conv_cols(cc, g, n0);
  }
  using SB = StageT<BN_ / 32>;
  auto load = [&](Stage& sa, SB& sb, int kt) {
    const int k0 = k_begin + kt * KT;
    if (g.conv == 1) load_conv_a<ESZ>(sa, (const char*)g.A, cr, g, k0, k_end);
    else if (g.ta) load_t(sa, (const unsigned short*)g.A, m0, g.M, g.lda, k0, k_end);
    else load_nt<ESZ>(sa, (const char*)g.A, m0, g.M, (size_t)g.lda * ESZ, k0 * ESZ, k_end * ESZ);
    if constexpr (BN_ == 128) {
      if (g.conv == 2) load_conv_b(sb, (const unsigned short*)g.B, cc, g, k0, k_end);
      else if (g.tb) load_t(sb, (const unsigned short*)g.B, n0, g.N, g.ldb, k0, k_end);
      else load_nt<ESZ>(sb, (const char*)g.B, n0, g.N, (size_t)g.ldb * ESZ, k0 * ESZ, k_end * ESZ);
    } else {
      load_nt<ESZ, BN_ / 32>(sb, (const char*)g.B, n0, g.N, (size_t)g.ldb * ESZ, k0 * ESZ, k_end * ESZ);
    }
  };
  auto store = [&](const Stage& sa, const SB& sb, int buf) {
    char* la = smem + buf * T::BUF;
    char* lb = la + G_TILE_BYTES;
    if (g.ta && g.conv != 1) store_t(sa, la);
    else store_nt(sa, la);
    if constexpr (BN_ == 128) {
      if (g.tb || g.conv == 2) store_t(sb, lb);
      else store_nt(sb, lb);
    } else {
      store_nt<BN_ / 32>(sb, lb);
    }
  };

  Stage sa1;
  SB sb1;
  if (nk > 0) {
    load(sa1, sb1, 0);
    store(sa1, sb1, 0);
  }
  __syncthreads();
  const bool single = g.single != 0;
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = single ? 0 : (kt & 1);
    if (kt + 1 < nk) load(sa1, sb1, kt + 1);  // global loads in flight during the MFMAs below
    const char* la = smem + buf * T::BUF;
    const char* lb = la + G_TILE_BYTES;
    if constexpr (!FP8) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        s16x8 af[4], bfr[T::NF];
#pragma unroll
        for (int m = 0; m < 4; ++m)
          af[m] = *(const s16x8*)(la + lds_off(wr * 64 + m * 16 + (lane & 15), s * 4 + (lane >> 4)));
#pragma unroll
        for (int n = 0; n < T::NF; ++n)
          bfr[n] = *(const s16x8*)(lb + lds_off(wc * T::WCW + n * 16 + (lane & 15), s * 4 + (lane >> 4)));
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int n = 0; n < T::NF; ++n)
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m], bfr[n], acc[m][n], 0, 0, 0);
      }
    } else {
      i32x8 af[4], bfr[T::NF];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int row = wr * 64 + m * 16 + (lane & 15), c = 2 * (lane >> 4);
        const uint4 lo = *(const uint4*)(la + lds_off(row, c)), hi = *(const uint4*)(la + lds_off(row, c + 1));
        af[m] = i32x8{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
      }
#pragma unroll
      for (int n = 0; n < T::NF; ++n) {
        const int row = wc * T::WCW + n * 16 + (lane & 15), c = 2 * (lane >> 4);
        const uint4 lo = *(const uint4*)(lb + lds_off(row, c)), hi = *(const uint4*)(lb + lds_off(row, c + 1));
        bfr[n] = i32x8{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
      }
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < T::NF; ++n)  // fp8 e4m3 x fp8 e4m3, unit E8M0 scales (127)
          acc[m][n] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[m], bfr[n], acc[m][n], 0, 0, 0, 127, 0, 127);
    }
    if (kt + 1 < nk) {
      if (single) __syncthreads();  // every wave is done reading the buffer it is about to overwrite
      store(sa1, sb1, single ? 0 : buf ^ 1);
    }
    __syncthreads();
  }

  gemm_epilogue<BN_, 4>(g, acc, smem, m0, n0, tm, ksplit);
}


// ---------------------------------------------------------------------------------------------------------
// k_gemm_glds: the same tile / fragments / epilogue as k_gemm for K-contiguous operands (ta = tb = 0, or the
// implicit conv gather of A), but staged global -> LDS with global_load_lds_dwordx4 (no VGPR staging, no
// ds_write pass): tile k+1's loads stay in flight during tile k's MFMAs, retired by a counted vmcnt and a raw
// s_barrier (a __syncthreads() would drain them: CDNA4 guide, "Pipelining across barriers").
// The LDS image must be lane-linear per wave instruction (8 rows x 128 B), so the XOR swizzle of lds_off is
// applied to the SOURCE chunk each lane loads (an involution: the fragment reads use lds_off unchanged).
// Out-of-range chunks (K tail, conv padding) load from a zeroed global word.
// ---------------------------------------------------------------------------------------------------------
__device__ __attribute__((aligned(16))) unsigned char g_gemm_zero16[16];


__device__ __forceinline__ void glds16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}
// 16 B per lane from a buffer descriptor straight into LDS (wave-linear at lds_wave_base); an offset past the
// descriptor's range loads zeros
__device__ __forceinline__ void blds16(__amdgpu_buffer_rsrc_t rs, char* lds_wave_base, unsigned voff, unsigned soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)lds_wave_base, 16, voff, soff, 0, 0);
}
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <bool FP8, int BN_, int NW>
__global__ void __launch_bounds__(NW * 64) k_gemm_glds(GemmArgs g) {
  using T = GemmTile<BN_>;
  using Wg = WaveGrid<BN_, NW>;
  constexpr int RA = GBM / NW, RB = BN_ / NW;  // A / B tile rows staged by each wave
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int ntm = (g.M + GBM - 1) / GBM, ntn = (g.N + BN_ - 1) / BN_;
  const int tile = xcd_remap(blockIdx.x, ntm * ntn);
  int tm, tn;
  tile_coords(tile, ntm, ntn, tm, tn);
  const int m0 = tm * GBM, n0 = tn * BN_;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), wr = wave / Wg::WC, wc = wave % Wg::WC;
  constexpr int ESZ = FP8 ? 1 : 2;
  constexpr int KT = GBK_BYTES / ESZ;
  constexpr int NAI = RA / 8, NBI = RB / 8;  // A / B wave instructions (8 rows each) per tile
  constexpr int NI = NAI + NBI;              // glds per thread per tile
  const int ksplit = blockIdx.y;
  const int k_begin = ksplit * g.k_per_split;
  const int k_end = min(g.K, k_begin + g.k_per_split);
  const int nk = (k_end - k_begin + KT - 1) / KT;
  const int lr = lane >> 3, lj = lane & 7;

  const bool c64 = g.conv == 1 && g.cC % KT == 0;
  constexpr unsigned OOB = 0x80000000u;
  const long long a_bytes = g.conv == 1 ? (long long)g.cN * g.cH * g.cW * g.cC * ESZ
                                        : ((long long)(g.M - 1) * g.lda + g.K) * ESZ;
  const long long b_bytes = ((long long)(g.N - 1) * g.ldb + g.K) * ESZ;
  const int ntaps = g.cKH * g.cKW;
  const bool fast = a_bytes < OOB && b_bytes < OOB && (g.conv == 0 || (c64 && ntaps <= 32 && g.M < (1 << 24)));

  // per-lane rows: A row wave*32 + i*8 + lr, B row wave*(BN_/4) + i*8 + lr
  const char* arow[NAI];
  int nh[NAI], ih[NAI], iw[NAI];
#pragma unroll
  for (int i = 0; i < NAI; ++i) {
    int m = m0 + wave * RA + i * 8 + lr;
    m = m < g.M ? m : g.M - 1;
    arow[i] = (const char*)g.A + (size_t)m * g.lda * ESZ;
    if (g.conv == 1 && !fast) {
      const int ow = m % g.cWo, t = m / g.cWo, oh = t % g.cHo, n = t / g.cHo;
      nh[i] = n * g.cH;
      ih[i] = oh * g.cS - g.cP;
      iw[i] = ow * g.cS - g.cP;
    }
  }
  const char* brow[NBI];
#pragma unroll
  for (int i = 0; i < NBI; ++i) {
    int n = n0 + wave * RB + i * 8 + lr;
    n = n < g.N ? n : g.N - 1;
    brow[i] = (const char*)g.B + (size_t)n * g.ldb * ESZ;
  }
  const int kb_end = k_end * ESZ;

  // Fast path (plain K-contiguous operands, or the implicit conv with C % 64 == 0): buffer_load ... lds with the
  // per-lane byte offsets computed once here, so a K-tile costs one add per load (plus, for the conv, a tap
  // validity test against a per-row mask) and the tap / channel position advances without divisions.  The
  // profile of the general path (profiles/gemm_pmc_r2.txt): ~7 VALU and ~8 SALU per MFMA on the 3x3 conv, the
  // issue bound of that kernel.  Out-of-range lanes (rows past M / N, padding taps, the K tail) get an offset
  // past the descriptor's range, which loads zeros.
  const __amdgpu_buffer_rsrc_t ars = __builtin_amdgcn_make_buffer_rsrc((void*)g.A, (short)0, (int)(fast ? a_bytes : 0),
                                                                       0x00020000);
  const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc((void*)g.B, (short)0, (int)(fast ? b_bytes : 0),
                                                                       0x00020000);
  unsigned aoff[NAI], amask[NAI], boff[NBI];
  int s_tap = 0, s_kh = 0, s_kw = 0, s_c0b = 0, s_tapoff = 0;  // conv: position of the next tile to issue
  if (fast) {
    const float inv_wo = g.conv == 1 ? 1.f / (float)g.cWo : 0.f, inv_ho = g.conv == 1 ? 1.f / (float)g.cHo : 0.f;
    unsigned rep = 0u;
    if (g.conv == 1)
      for (int kh = 0; kh < g.cKH; ++kh) rep |= 1u << (kh * g.cKW);
#pragma unroll
    for (int i = 0; i < NAI; ++i) {
      const int r = wave * RA + i * 8 + lr, m = m0 + r;
      const unsigned cb = (unsigned)(lj ^ ((r >> 1) & 7)) << 4;
      if (g.conv == 1) {  // float-reciprocal row decode, range-based tap mask (no per-tap loop)
        int ow, oh;
        const int t = fdiv_rc(m < g.M ? m : 0, g.cWo, inv_wo, ow), n = fdiv_rc(t, g.cHo, inv_ho, oh);
        const int ih0 = oh * g.cS - g.cP, iw0 = ow * g.cS - g.cP;
        const long long ro = (((long long)n * g.cH + ih0) * g.cW + iw0) * g.cC * ESZ;
        aoff[i] = (unsigned)(ro + cb);  // wraps for padding rows; only used when the tap is valid
        amask[i] = m < g.M ? tap_mask(ih0, iw0, g.cH, g.cW, g.cKH, g.cKW, rep) : 0u;
      } else {
        aoff[i] = m < g.M ? (unsigned)((long long)m * g.lda * ESZ) + cb : OOB;
      }
    }
#pragma unroll
    for (int i = 0; i < NBI; ++i) {
      const int r = wave * RB + i * 8 + lr, n = n0 + r;
      boff[i] = n < g.N ? (unsigned)((long long)n * g.ldb * ESZ) + ((unsigned)(lj ^ ((r >> 1) & 7)) << 4) : OOB;
    }
    if (g.conv == 1) {
      s_tap = k_begin / g.cC;
      s_c0b = (k_begin - s_tap * g.cC) * ESZ;
      s_kh = s_tap / g.cKW;
      s_kw = s_tap - s_kh * g.cKW;
      s_tapoff = (s_kh * g.cW + s_kw) * g.cC * ESZ;
    }
  }
  auto lane_cb = [&](int r) { return (int)((unsigned)(lj ^ ((r >> 1) & 7)) << 4); };
  auto issue_fast = [&](int kt, int buf) {
    const int kb0 = (k_begin + kt * KT) * ESZ;
    const bool tail = kb_end - kb0 < GBK_BYTES;  // (uniform) the last, partial K-tile
    char* la = smem + buf * T::BUF;
    char* lb = la + G_TILE_BYTES;
    if (g.conv == 1) {
      const unsigned sadd = (unsigned)(s_tapoff + s_c0b), bit = 1u << s_tap;
#pragma unroll
      for (int i = 0; i < NAI; ++i) {
        bool ok = (amask[i] & bit) != 0u;
        if (tail) ok = ok && kb0 + lane_cb(wave * RA + i * 8 + lr) < kb_end;
        blds16(ars, la + (wave * RA + i * 8) * 128, ok ? aoff[i] + sadd : OOB, 0u);
      }
      s_c0b += GBK_BYTES;
      if (s_c0b == g.cC * ESZ) {
        s_c0b = 0;
        ++s_tap;
        if (++s_kw == g.cKW) {
          s_kw = 0;
          ++s_kh;
        }
        s_tapoff = (s_kh * g.cW + s_kw) * g.cC * ESZ;
      }
    } else {
#pragma unroll
      for (int i = 0; i < NAI; ++i) {
        unsigned v = aoff[i];
        if (tail && kb0 + lane_cb(wave * RA + i * 8 + lr) >= kb_end) v = OOB;
        blds16(ars, la + (wave * RA + i * 8) * 128, v, (unsigned)kb0);
      }
    }
#pragma unroll
    for (int i = 0; i < NBI; ++i) {
      unsigned v = boff[i];
      if (tail && kb0 + lane_cb(wave * RB + i * 8 + lr) >= kb_end) v = OOB;
      blds16(brs, lb + (wave * RB + i * 8) * 128, v, (unsigned)kb0);
    }
  };
  auto issue = [&](int kt, int buf) {
    if (fast) {
      issue_fast(kt, buf);
      return;
    }
    const int kb0 = (k_begin + kt * KT) * ESZ;
    char* la = smem + buf * T::BUF;
    char* lb = la + G_TILE_BYTES;
    int tc0 = 0, tkh = 0, tkw = 0;
    if (c64) {
      const int k0 = kb0 / ESZ, tap = k0 / g.cC;
      tc0 = k0 - tap * g.cC;
      tkh = tap / g.cKW;
      tkw = tap - tkh * g.cKW;
    }
#pragma unroll
    for (int i = 0; i < NAI; ++i) {
      const int r = wave * RA + i * 8 + lr;
      const int kb = kb0 + ((lj ^ ((r >> 1) & 7)) << 4);
      const void* src = g_gemm_zero16;
      if (g.conv == 1) {
        int c, kh, kw;
        if (c64) {  // the whole K-tile is one tap: wave-uniform decode, per-lane channel offset only
          c = tc0 + (kb - kb0) / ESZ;
          kh = tkh;
          kw = tkw;
        } else {
          const int k = kb / ESZ, tap = k / g.cC;
          c = k - tap * g.cC;
          kh = tap / g.cKW;
          kw = tap - kh * g.cKW;
        }
        const int h = ih[i] + kh, w = iw[i] + kw;
        if (kb < kb_end && h >= 0 && h < g.cH && w >= 0 && w < g.cW)
          src = (const char*)g.A + (((size_t)(nh[i] + h) * g.cW + w) * g.cC + c) * ESZ;
      } else if (kb < kb_end) {
        src = arow[i] + kb;
      }
      glds16(src, la + (wave * RA + i * 8) * 128);
    }
#pragma unroll
    for (int i = 0; i < NBI; ++i) {
      const int r = wave * RB + i * 8 + lr;
      const int kb = kb0 + ((lj ^ ((r >> 1) & 7)) << 4);
      glds16(kb < kb_end ? (const void*)(brow[i] + kb) : (const void*)g_gemm_zero16,
             lb + (wave * RB + i * 8) * 128);
    }
  };

  f32x4 acc[4][Wg::NF];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < Wg::NF; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  // S LDS buffers, S - 1 tiles in flight.  S = 1 (single): tile k is issued after tile k-1's closing barrier.
  const int S = g.single ? 1 : (g.stages >= 2 && g.stages <= 4 ? g.stages : 2);
  for (int t0 = 0; t0 < S - 1 && t0 < nk; ++t0) issue(t0, t0);
  // buffer indices stepped incrementally: kt % S with a runtime S compiled to ~40 SALU of signed division per
  // K-tile (the loop's issue bound on short-N shapes, profiles/gemm_stream_pmc_r2.txt)
  int buf = 0, ibuf = S - 1;  // kt % S, (kt + S - 1) % S
  for (int kt = 0; kt < nk; ++kt, buf = buf + 1 == S ? 0 : buf + 1, ibuf = ibuf + 1 == S ? 0 : ibuf + 1) {
    const int nt = kt + S - 1;
    if (nt < nk) issue(nt, ibuf);  // into the buffer every wave finished reading before the last barrier
    switch (min(nk - 1, nt) - kt) {   // this thread's loads of tile kt have landed (later tiles' in flight)
      case 0: wait_vmcnt<0>(); break;
      case 1: wait_vmcnt<NI>(); break;
      case 2: wait_vmcnt<2 * NI>(); break;
      default: wait_vmcnt<3 * NI>(); break;
    }
    __builtin_amdgcn_s_barrier();  // ... and every thread's
    asm volatile("" ::: "memory");
    const char* la = smem + buf * T::BUF;
    const char* lb = la + G_TILE_BYTES;
    if constexpr (!FP8) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        s16x8 af[4], bfr[Wg::NF];
#pragma unroll
        for (int m = 0; m < 4; ++m)
          af[m] = *(const s16x8*)(la + lds_off(wr * 64 + m * 16 + (lane & 15), s * 4 + (lane >> 4)));
#pragma unroll
        for (int n = 0; n < Wg::NF; ++n)
          bfr[n] = *(const s16x8*)(lb + lds_off(wc * Wg::WCW + n * 16 + (lane & 15), s * 4 + (lane >> 4)));
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int n = 0; n < Wg::NF; ++n)
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m], bfr[n], acc[m][n], 0, 0, 0);
      }
    } else {
      i32x8 af[4], bfr[Wg::NF];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int row = wr * 64 + m * 16 + (lane & 15), c = 2 * (lane >> 4);
        const uint4 lo = *(const uint4*)(la + lds_off(row, c)), hi = *(const uint4*)(la + lds_off(row, c + 1));
        af[m] = i32x8{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
      }
#pragma unroll
      for (int n = 0; n < Wg::NF; ++n) {
        const int row = wc * Wg::WCW + n * 16 + (lane & 15), c = 2 * (lane >> 4);
        const uint4 lo = *(const uint4*)(lb + lds_off(row, c)), hi = *(const uint4*)(lb + lds_off(row, c + 1));
        bfr[n] = i32x8{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
      }
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < Wg::NF; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[m], bfr[n], acc[m][n], 0, 0, 0, 127, 0, 127);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave is done reading buf before it is refilled
    asm volatile("" ::: "memory");
  }
  gemm_epilogue<BN_, NW>(g, acc, smem, m0, n0, tm, ksplit);
}

// Epilogue of the 256-row tiles (k_gemm_pp): four 64-row quarters of the fp32 tile are staged in LDS by
// stage(q) (64 x BN fp32, 16-column groups XOR-swizzled by (row >> 2) & 3 -- the kernels' cidx), then written back
// row-contiguously, 16 B per lane, with alpha / bias / beta / ReLU and the optional BN column statistics (one
// partial row per 128 output rows, the k_bn_finalize layout).  stage is called with a compile-time q (unrolled:
// the accumulator indices must stay static).
template <int NT, int BN = 256, class StageFn>
__device__ __forceinline__ void store_quarters_256(const GemmArgs& g, char* smem, int m0, int n0, int tm, StageFn stage) {
  float* ct = (float*)smem;
  auto cidx = [](int r, int c) { return r * BN + (c ^ (((r >> 2) & 3) << 4)); };
  const float alpha = gemm_alpha(g);
  constexpr int CG = BN / 8, RL = NT / CG;  // column groups of 8, row lanes
  const int cg = threadIdx.x % CG, col0 = n0 + cg * 8;
  float bias8[8], shift8[8], s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int col = min(col0 + e, g.N - 1);
    bias8[e] = g.bias ? g.bias[col] : 0.f;
    shift8[e] = g.col_stats ? g.stats_shift[col] : 0.f;
    s1[e] = s2[e] = 0.f;
  }
  const bool full8 = col0 + 8 <= g.N && (g.ldc & 7) == 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    stage(q);
    __syncthreads();
    for (int r = 0; r < 64 / RL; ++r) {
      const int lrow = threadIdx.x / CG + RL * r, row = m0 + q * 64 + lrow;
      if (row >= g.M || col0 >= g.N) continue;
      const f32x4 a0 = *(const f32x4*)(ct + cidx(lrow, cg * 8)), a1 = *(const f32x4*)(ct + cidx(lrow, cg * 8 + 4));
      const float av[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
      const size_t o = (size_t)row * g.ldc + col0;
      float old[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (g.beta != 0.f) {
        if (full8 && g.out_bf16) {
          const uint4 u = *(const uint4*)((const unsigned short*)g.C + o);
          const unsigned w4[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
          for (int e = 0; e < 8; ++e) old[e] = __uint_as_float((w4[e >> 1] >> ((e & 1) * 16)) << 16);
        } else {
          for (int e = 0; e < 8 && col0 + e < g.N; ++e)
            old[e] = g.out_bf16 ? bf2f(((const unsigned short*)g.C)[o + e]) : ((const float*)g.C)[o + e];
        }
      }
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float x = av[e] * alpha + bias8[e] + g.beta * old[e];
        if (g.relu) x = x > 0.f ? x : 0.f;
        v[e] = x;
      }
      if (g.out_bf16) {
        unsigned short hb[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) hb[e] = f2bf_rne(v[e]);
        if (g.col_stats) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float d = bf2f(hb[e]) - shift8[e];
            s1[e] += d;
            s2[e] += d * d;
          }
        }
        if (full8) {
          *(uint4*)((unsigned short*)g.C + o) =
              uint4{hb[0] | ((unsigned)hb[1] << 16), hb[2] | ((unsigned)hb[3] << 16), hb[4] | ((unsigned)hb[5] << 16),
                    hb[6] | ((unsigned)hb[7] << 16)};
        } else {
          for (int e = 0; e < 8 && col0 + e < g.N; ++e) ((unsigned short*)g.C)[o + e] = hb[e];
        }
      } else {
        if (g.col_stats) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float d = v[e] - shift8[e];
            s1[e] += d;
            s2[e] += d * d;
          }
        }
        if (full8) {
          *(f32x4*)((float*)g.C + o) = f32x4{v[0], v[1], v[2], v[3]};
          *(f32x4*)((float*)g.C + o + 4) = f32x4{v[4], v[5], v[6], v[7]};
        } else {
          for (int e = 0; e < 8 && col0 + e < g.N; ++e) ((float*)g.C)[o + e] = v[e];
        }
      }
    }
    __syncthreads();
    if (g.col_stats && (q & 1)) {  // one partial row per 128 output rows (the k_bn_finalize layout)
      float2* red = (float2*)smem;  // [RL][BN]
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[(threadIdx.x / CG) * BN + cg * 8 + e] = float2{s1[e], s2[e]};
        s1[e] = s2[e] = 0.f;
      }
      __syncthreads();
      for (int c = threadIdx.x; c < BN; c += NT) {
        const int col = n0 + c;
        float2 t = red[c];
        for (int k = 1; k < RL; ++k) {
          t.x += red[k * BN + c].x;
          t.y += red[k * BN + c].y;
        }
        const int prow = 2 * tm + (q >> 1);
        if (col < g.N && prow * 128 < g.M) g.col_stats[(size_t)prow * g.N + col] = t;
      }
      __syncthreads();
    }
  }
}

// ---------------------------------------------------------------------------------------------------------
// k_gemm_pp: 256 x 256 output tile, 512 threads as two wave groups that ping-pong (bf16, K-contiguous operands or
// the C % 64 implicit conv; no split-K / row remap).  Group r (waves 4r .. 4r+3) owns rows 128r .., wave (r, c)
// a 128 x 64 sub-tile (32 accumulators of 16 x 16).  Every K-tile is two k32 steps; per step a group first reads
// its A / B fragments from LDS (L) and then issues its 32 MFMAs (M).  Group 1 starts one barrier late, so in
// every barrier interval one group runs MFMAs while the other reads fragments and issues LDS-DMA: each SIMD holds
// one wave of each group (waves w and w + 4), so its MFMA pipe is fed by whichever group is in M.
// Interval I_j (between barriers j and j + 1): group 0 runs L(s) in I_2s and M(s) in I_2s+1, group 1 L(s) in
// I_2s+1 and M(s) in I_2s+2 (step s = 2 kt + h).  Staging, two LDS buffers (tile kt in buffer kt & 1):
//   * tile kt + 1 is issued in I_4kt (group 0 before L(2kt), group 1 in M(2kt - 1)); its buffer last held tile
//     kt - 1, read for the last time in I_4kt-1 and retired there (lgkmcnt(0) before that barrier).  Plain GEMMs:
//     group 1 issues in I_4kt+1 instead, before L(2kt), so no LDS-DMA issue delays an MFMA phase (50176 x 256 x
//     2304: 86 -> 73 us; the implicit conv keeps I_4kt -- its gather lands later: profiles/gemm_pp_issue_ab_r6.log);
//   * every issuing thread waits vmcnt(0) before the barrier ending I_4kt+3 (group 0 after M(2kt + 1), group 1
//     after L(2kt + 1)), so tile kt + 1 is complete and visible when group 0 reads it in I_4kt+4.
// Operand addressing as k_gemm_glds' fast path (per-lane offsets computed once, incremental tap for the conv).
// ---------------------------------------------------------------------------------------------------------
constexpr int PP_BM = 256, PP_NT = 512;
constexpr int PP_TILE = PP_BM * GBK_BYTES;  // A: 32 KiB per buffer
template <int BN>
struct PpTile {  // BN = 256: a group's 4 waves side by side (128 x 64 each); BN = 128: 2 x 2 waves of 64 x 64
  static constexpr int WMG = BN == 256 ? 1 : 2, WNG = 4 / WMG, MF = 8 / WMG;
  static constexpr int BTILE = BN * GBK_BYTES, BUF = PP_TILE + BTILE, LDS = 2 * BUF;
  static constexpr int NIB = BN / 64;  // B glds per thread and K-tile (wave: B rows (BN / 8) wave ..)
  static_assert(LDS >= 64 * BN * 4, "epilogue staging fits");
};
constexpr int PP_LDS = PpTile<256>::LDS;  // 128 KiB

template <int PP_BN>
__global__ void __launch_bounds__(PP_NT) k_gemm_pp(GemmArgs g) {
  using TT = PpTile<PP_BN>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int ntm = (g.M + PP_BM - 1) / PP_BM, ntn = (g.N + PP_BN - 1) / PP_BN;
  const int tile = xcd_remap(blockIdx.x, ntm * ntn);
  int tm, tn;
  tile_coords(tile, ntm, ntn, tm, tn);
  const int m0 = tm * PP_BM, n0 = tn * PP_BN;
  // (wave index made provably uniform: every LDS-DMA's M0 base is then plain SALU arithmetic instead of a VALU
  // address + v_readfirstlane per instruction -- 4096^3 127 -> 123 us, profiles/gemm_pmc_r7.txt)
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), wr = wave >> 2;
  const int wi = (wave & 3) / TT::WNG, wj = (wave & 3) % TT::WNG;  // wave position inside its group
  const int wrow = wr * 128 + wi * (128 / TT::WMG), wcol = wj * 64;
  constexpr int ESZ = 2, KT = GBK_BYTES / ESZ;
  const int k_begin = 0, k_end = g.K, nk = (g.K + KT - 1) / KT;
  const int lr = lane >> 3, lj = lane & 7;
  constexpr int NI = 4;  // glds per thread and operand per K-tile (wave: rows 32 wave .. + 32)
  constexpr unsigned OOB = 0x80000000u;
  const long long a_bytes = g.conv == 1 ? (long long)g.cN * g.cH * g.cW * g.cC * ESZ
                                        : ((long long)(g.M - 1) * g.lda + g.K) * ESZ;
  const long long b_bytes = ((long long)(g.N - 1) * g.ldb + g.K) * ESZ;
  const __amdgpu_buffer_rsrc_t ars = __builtin_amdgcn_make_buffer_rsrc((void*)g.A, (short)0, (int)a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc((void*)g.B, (short)0, (int)b_bytes, 0x00020000);
  unsigned aoff[NI], amask[NI], boff[TT::NIB];
  int s_tap = 0, s_kh = 0, s_kw = 0, s_c0b = 0, s_tapoff = 0;
  const float inv_wo = g.conv == 1 ? 1.f / (float)g.cWo : 0.f, inv_ho = g.conv == 1 ? 1.f / (float)g.cHo : 0.f;
  unsigned rep = 0u;
  if (g.conv == 1)
    for (int kh = 0; kh < g.cKH; ++kh) rep |= 1u << (kh * g.cKW);
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int r = wave * 32 + i * 8 + lr, m = m0 + r;
    const unsigned cb = (unsigned)(lj ^ ((r >> 1) & 7)) << 4;
    if (g.conv == 1) {  // float-reciprocal row decode (M < 2^24: launcher), range-built tap mask
      int ow, oh;
      const int t = fdiv_rc(m < g.M ? m : 0, g.cWo, inv_wo, ow), n = fdiv_rc(t, g.cHo, inv_ho, oh);
      const int ih0 = oh * g.cS - g.cP, iw0 = ow * g.cS - g.cP;
      aoff[i] = (unsigned)((((long long)n * g.cH + ih0) * g.cW + iw0) * g.cC * ESZ + cb);
      amask[i] = m < g.M ? tap_mask(ih0, iw0, g.cH, g.cW, g.cKH, g.cKW, rep) : 0u;
    } else {
      amask[i] = 0u;
      aoff[i] = m < g.M ? (unsigned)((long long)m * g.lda * ESZ) + cb : OOB;
    }
  }
#pragma unroll
  for (int i = 0; i < TT::NIB; ++i) {
    const int r = wave * (PP_BN / 8) + i * 8 + lr, n = n0 + r;
    boff[i] = n < g.N ? (unsigned)((long long)n * g.ldb * ESZ) + ((unsigned)(lj ^ ((r >> 1) & 7)) << 4) : OOB;
  }
  auto lane_cb = [&](int r) { return (int)((unsigned)(lj ^ ((r >> 1) & 7)) << 4); };
  // this thread's LDS-DMA of tile kt into buffer kt & 1 (tiles issued in increasing order: the conv tap state)
  auto issue = [&](int kt) {
    const int kb0 = (k_begin + kt * KT) * ESZ;
    const bool tail = k_end * ESZ - kb0 < GBK_BYTES;
    char* la = smem + (kt & 1) * TT::BUF;
    char* lb = la + PP_TILE;
    if (g.conv == 1) {
      const unsigned sadd = (unsigned)(s_tapoff + s_c0b), bit = 1u << s_tap;
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        bool ok = (amask[i] & bit) != 0u;
        if (tail) ok = ok && kb0 + lane_cb(wave * 32 + i * 8 + lr) < k_end * ESZ;
        blds16(ars, la + (wave * 32 + i * 8) * 128, ok ? aoff[i] + sadd : OOB, 0u);
      }
      s_c0b += GBK_BYTES;
      if (s_c0b == g.cC * ESZ) {
        s_c0b = 0;
        ++s_tap;
        if (++s_kw == g.cKW) {
          s_kw = 0;
          ++s_kh;
        }
        s_tapoff = (s_kh * g.cW + s_kw) * g.cC * ESZ;
      }
    } else {
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        unsigned v = aoff[i];
        if (tail && kb0 + lane_cb(wave * 32 + i * 8 + lr) >= k_end * ESZ) v = OOB;
        blds16(ars, la + (wave * 32 + i * 8) * 128, v, (unsigned)kb0);
      }
    }
#pragma unroll
    for (int i = 0; i < TT::NIB; ++i) {
      const int r = wave * (PP_BN / 8) + i * 8;
      unsigned v = boff[i];
      if (tail && kb0 + lane_cb(r + lr) >= k_end * ESZ) v = OOB;
      blds16(brs, lb + r * 128, v, (unsigned)kb0);
    }
  };
  auto bar = [] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  constexpr int MF = TT::MF;
  f32x4 acc[MF][4];
#pragma unroll
  for (int m = 0; m < MF; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  s16x8 af[MF], bfr[4];
  auto load_frags = [&](int kt, int h) {
    const char* la = smem + (kt & 1) * TT::BUF;
    const char* lb = la + PP_TILE;
#pragma unroll
    for (int m = 0; m < MF; ++m) af[m] = *(const s16x8*)(la + lds_off(wrow + m * 16 + (lane & 15), h * 4 + (lane >> 4)));
#pragma unroll
    for (int n = 0; n < 4; ++n) bfr[n] = *(const s16x8*)(lb + lds_off(wcol + n * 16 + (lane & 15), h * 4 + (lane >> 4)));
  };
  auto mfmas = [&] {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int m = 0; m < MF; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m], bfr[n], acc[m][n], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // prologue: tile 0 complete and visible to everyone
  if (nk > 0) issue(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  bar();
  if (wr == 0) {
#pragma unroll 1
    for (int st = 0; st < 2 * nk; ++st) {
      const int kt = st >> 1, h = st & 1;
      if (h == 0 && kt + 1 < nk) issue(kt + 1);  // I_4kt: buffer (kt+1) & 1 retired in I_4kt-1
      load_frags(kt, h);
      bar();                                      // end of L(st)
      mfmas();
      if (h == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // my part of tile kt + 1 landed
      bar();                                      // end of M(st)
    }
    bar();  // group 1 runs one barrier behind
  } else {
    const bool cv = g.conv == 1;
    if (nk > 1) issue(1);  // I_0: group 1's part of tile 1 (group 0 issued its part before L(0))
    bar();                 // end of I_0
#pragma unroll 1
    for (int st = 0; st < 2 * nk; ++st) {
      const int kt = st >> 1, h = st & 1;
      // plain GEMM: I_4kt+1 (an L phase, not the MFMA phase): tile kt + 1 into buffer (kt + 1) & 1, last read in
      // I_4kt-1; implicit conv: I_4kt+4, tile kt + 2 (a gather lands later: one more interval of slack)
      if (!cv && h == 0 && kt >= 1 && kt + 1 < nk) issue(kt + 1);
      load_frags(kt, h);
      if (h == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // my part of tile kt + 1 landed (I_4kt+3)
      bar();  // end of L(st)
      if (cv && h == 1 && kt + 2 < nk) issue(kt + 2);
      mfmas();
      bar();  // end of M(st)
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // epilogue: four 64-row quarters staged in LDS (fp32, 64 KiB), written row-contiguously (store_quarters_256)
  float* ct = (float*)smem;
  auto cidx = [](int r, int c) { return r * PP_BN + (c ^ (((r >> 2) & 3) << 4)); };
  store_quarters_256<PP_NT, PP_BN>(g, smem, m0, n0, tm, [&](int q) {
    // quarter q = rows 64 q ..: group q >> 1; BN = 256: its accumulators (q & 1) * 4 ..; BN = 128: wave wi = q & 1
    if (wr == (q >> 1) && (TT::WMG == 1 || wi == (q & 1))) {
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            ct[cidx(m * 16 + (lane >> 4) * 4 + j, wcol + n * 16 + (lane & 15))] =
                acc[TT::WMG == 1 ? (q & 1) * 4 + m : m][n][j];
    }
  });
}

// ---------------------------------------------------------------------------------------------------------
// k_gemm_pp4: k_gemm_pp's 256 x 256 tile and ping-pong wave groups on a ring of four k32 slots (32 KiB each: A
// [256][64 B] | B [256][64 B]) instead of two 64-deep K-tile buffers.  The PMC comparison with hipBLASLt
// (profiles/gemm_pmc_r7.txt) put k_gemm_pp's loss in the barrier intervals that carry a whole K-tile's LDS-DMA
// issue (8 pieces per thread in one interval, longer than the other group's 32 MFMAs).  Here every interval of a
// group issues 4 pieces (2 A + 2 B: 16 rows x 64 B each) of the step two ahead, into the slot its own group finished
// reading two steps ago, so the issue cost is spread evenly and each DMA still has three to four barrier intervals
// (~1,500-2,000 MFMA cycles) to land:
//   group 0, step s: L = issue(s + 2), fragment reads of s | barrier | M = 32 MFMAs of s, vmcnt retires s + 1 |
//   barrier;  group 1 runs one barrier behind and retires s + 1 at the end of its L interval (the barrier that ends
//   it is the one before group 0 reads s + 1).
// Slot (s + 2) & 3 last held step s - 2, read by group 1 in interval 2s - 3 and retired by its M interval 2s - 2.
// Rows of 64 B with 16-B chunks XOR-swizzled by (row >> 1) & 3 (the fragment reads' lane groups conflict-free);
// the swizzle is applied to each lane's source chunk (the DMA image is lane-linear).  K % 64 == 0 (launcher).
// ---------------------------------------------------------------------------------------------------------
__device__ __forceinline__ int pp4_off(int row, int chunk) { return row * 64 + ((chunk ^ ((row >> 1) & 3)) << 4); }
constexpr int PP4_SLOT = 2 * PP_BM * 64;  // 32 KiB
constexpr int PP4_LDS = 4 * PP4_SLOT;     // 128 KiB

template <bool CONV>
__global__ void __launch_bounds__(PP_NT) k_gemm_pp4(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int ntm = (g.M + PP_BM - 1) / PP_BM, ntn = (g.N + PP_BM - 1) / PP_BM;
  const int tile = xcd_remap(blockIdx.x, ntm * ntn);
  int tm, tn;
  tile_coords(tile, ntm, ntn, tm, tn);
  const int m0 = tm * PP_BM, n0 = tn * PP_BM;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), wr = wave >> 2;
  const int wrow = wr * 128, wcol = (wave & 3) * 64;
  constexpr int ESZ = 2;
  const int nsteps = g.K / 32;
  constexpr unsigned OOB = 0x80000000u;
  const long long a_bytes = CONV ? (long long)g.cN * g.cH * g.cW * g.cC * ESZ : ((long long)(g.M - 1) * g.lda + g.K) * ESZ;
  const long long b_bytes = ((long long)(g.N - 1) * g.ldb + g.K) * ESZ;
  const __amdgpu_buffer_rsrc_t ars = __builtin_amdgcn_make_buffer_rsrc((void*)g.A, (short)0, (int)a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc((void*)g.B, (short)0, (int)b_bytes, 0x00020000);
  // staging: wave w loads rows 32 w + 16 i + (lane >> 2), i = 0, 1, of A and of B; chunk position lane & 3
  const int lq = lane >> 2, lc = lane & 3;
  unsigned aoff[2], amask[2], boff[2];
  int s_tap = 0, s_kh = 0, s_kw = 0, s_c0b = 0, s_tapoff = 0;
  unsigned rep = 0u;
  float inv_wo = 0.f, inv_ho = 0.f;
  if constexpr (CONV) {
    inv_wo = 1.f / (float)g.cWo;
    inv_ho = 1.f / (float)g.cHo;
    for (int kh = 0; kh < g.cKH; ++kh) rep |= 1u << (kh * g.cKW);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = wave * 32 + i * 16 + lq, m = m0 + r, n = n0 + r;
    const unsigned cb = (unsigned)(lc ^ ((r >> 1) & 3)) << 4;
    if constexpr (CONV) {
      int ow, oh;
      const int t = fdiv_rc(m < g.M ? m : 0, g.cWo, inv_wo, ow), nn = fdiv_rc(t, g.cHo, inv_ho, oh);
      const int ih0 = oh * g.cS - g.cP, iw0 = ow * g.cS - g.cP;
      aoff[i] = (unsigned)((((long long)nn * g.cH + ih0) * g.cW + iw0) * g.cC * ESZ + cb);
      amask[i] = m < g.M ? tap_mask(ih0, iw0, g.cH, g.cW, g.cKH, g.cKW, rep) : 0u;
    } else {
      amask[i] = 0u;
      aoff[i] = m < g.M ? (unsigned)((long long)m * g.lda * ESZ) + cb : OOB;
    }
    boff[i] = n < g.N ? (unsigned)((long long)n * g.ldb * ESZ) + cb : OOB;
  }
  // this thread's 4 DMA pieces of step st into slot st & 3 (steps issued in increasing order: the conv tap state)
  auto issue = [&](int st) {
    char* la = smem + (st & 3) * PP4_SLOT;
    char* lb = la + PP_BM * 64;
    const unsigned kb0 = (unsigned)st * 64u;
    if constexpr (CONV) {
      const unsigned sadd = (unsigned)(s_tapoff + s_c0b), bit = 1u << s_tap;
#pragma unroll
      for (int i = 0; i < 2; ++i)
        blds16(ars, la + (wave * 32 + i * 16) * 64, (amask[i] & bit) ? aoff[i] + sadd : OOB, 0u);
      s_c0b += 64;
      if (s_c0b == g.cC * ESZ) {
        s_c0b = 0;
        ++s_tap;
        if (++s_kw == g.cKW) {
          s_kw = 0;
          ++s_kh;
        }
        s_tapoff = (s_kh * g.cW + s_kw) * g.cC * ESZ;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 2; ++i) blds16(ars, la + (wave * 32 + i * 16) * 64, aoff[i], kb0);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) blds16(brs, lb + (wave * 32 + i * 16) * 64, boff[i], kb0);
  };
  auto bar = [] {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  f32x4 acc[8][4];
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  s16x8 af[8], bfr[4];
  const int frow = lane & 15, fch = lane >> 4;
  auto load_frags = [&](int st) {
    const char* la = smem + (st & 3) * PP4_SLOT;
    const char* lb = la + PP_BM * 64;
#pragma unroll
    for (int m = 0; m < 8; ++m) af[m] = *(const s16x8*)(la + pp4_off(wrow + m * 16 + frow, fch));
#pragma unroll
    for (int n = 0; n < 4; ++n) bfr[n] = *(const s16x8*)(lb + pp4_off(wcol + n * 16 + frow, fch));
  };
  auto mfmas = [&] {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m], bfr[n], acc[m][n], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // prologue: steps 0 and 1 complete and visible
  issue(0);
  if (nsteps > 1) issue(1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  bar();
  if (wr == 0) {
#pragma unroll 1
    for (int st = 0; st < nsteps; ++st) {
      const bool more = st + 2 < nsteps;
      if (more) issue(st + 2);
      load_frags(st);
      bar();  // end of L(st)
      mfmas();
      if (more) wait_vmcnt<4>();  // step st + 1 landed (this thread's part); st + 2 in flight
      else wait_vmcnt<0>();
      bar();  // end of M(st)
    }
    bar();  // group 1 runs one barrier behind
  } else {
    bar();  // end of interval 0
#pragma unroll 1
    for (int st = 0; st < nsteps; ++st) {
      const bool more = st + 2 < nsteps;
      if (more) issue(st + 2);
      load_frags(st);
      if (more) wait_vmcnt<4>();  // step st + 1 landed before the barrier group 0 reads it behind
      else wait_vmcnt<0>();
      bar();  // end of L(st)
      mfmas();
      bar();  // end of M(st)
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  float* ct = (float*)smem;
  auto cidx = [](int r, int c) { return r * PP_BM + (c ^ (((r >> 2) & 3) << 4)); };
  store_quarters_256<PP_NT, 256>(g, smem, m0, n0, tm, [&](int q) {
    if (wr == (q >> 1)) {
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            ct[cidx(m * 16 + (lane >> 4) * 4 + j, wcol + n * 16 + (lane & 15))] = acc[(q & 1) * 4 + m][n][j];
    }
  });
}

// ---------------------------------------------------------------------------------------------------------
// k_gemm_stream: persistent kernel for the short-K, output-heavy GEMMs of channels-last 1x1 convolutions (ResNet-50
// at batch 256: M = 5e4..8e5 pixels, N = 128..2048, K = 64..256).  Those calls move ~3x more bytes out than in and
// have 1-4 K-tiles per 128 x 128 tile, so the one-tile-per-workgroup kernels serialise load -> MFMA -> LDS-staged
// epilogue and reach 1.6-2.8 TB/s (profiles/gemm_shortk_r2.log).  Here a workgroup walks a static list of tiles as
// one flat stream of K-tiles, double-buffered by LDS-DMA, so the next tile's operands are in flight during this
// tile's MFMAs and epilogue.
//   * 4 waves, each 128 (M) x 32 (N) (or 128 x 16: 64-column tiles).  The MFMA operands are swapped (weights = src0, activations = src1), so a
//     lane's accumulators are consecutive output COLUMNS of one row, and the 32 weight rows of a wave slab are
//     staged in LDS in the order n = 8 (i >> 2) + 4 f + (i & 3) (fragment f, MFMA row i): lane (q, j) then holds
//     columns 8q .. 8q + 7 of row j of every 16-row fragment -- one 16-B bf16 store per row, no LDS staging.
//   * Epilogue straight from registers: alpha, bias, + beta * C_old (the residual-join input gradients),
//     bf16 (packed cvt), buffer stores (rows past M dropped by the
//     descriptor); the BN column statistics are summed over the wave's 128 rows in packed-fp32 registers and a
//     16-lane DPP row reduction, and written by lane j = 15 to col_stats[tm][n] (same layout as the other kernels).
//     The accumulators start from the MFMA's zero C operand on a tile's first K-tile (no per-tile clearing).
//   * vmcnt is in issue order for loads, stores and LDS-DMA alike: after an epilogue the wait is vmcnt(NST) (its
//     8 C + statistics stores stay in flight) before the next tile's DMA is issued.
//   * Implicit convolutions (C % 64 == 0, one tap per K-step) use the same stream: the 3x3 convolutions of
//     ResNet-50's layers 1-2 (N = 64 / 128) were issue-bound on the one-tile kernel (16 VALU + 12 SALU per MFMA,
//     profiles/gemm_stream_pmc_r2.txt).
//   * XCD-aware static schedule: workgroup b runs on XCD b % 8; XCD x owns tiles [x T / 8, (x + 1) T / 8) in the
//     grouped order, dealt round-robin to its workgroups, so its co-resident tiles share A row-tiles in its L2.
// Requirements (checked by the launcher): bf16 NT operands (or the C % 64 implicit conv), N % 64 == 0 (NF = 1) or
// N % 128 == 0 (NF = 2), K % 64 == 0, bf16 output, no ReLU, 16-B aligned rows, operand / output byte ranges < 2^31,
// at most 32 taps.
// ---------------------------------------------------------------------------------------------------------
constexpr int ST_NT = 256;
constexpr int ST_BUF = 2 * G_TILE_BYTES;  // A + B tile, 128 rows x 128 B each
typedef unsigned st_v4u __attribute__((ext_vector_type(4)));
typedef unsigned st_v2u __attribute__((ext_vector_type(2)));

// NF: 16-column MFMA fragments per wave.  MW: waves along M -- the tile is 128 MW rows x 64 NF (4 / MW) columns and
// wave (wm, wn) owns rows 128 wm .., so each wave's statistics are exactly one 128-row partial row of col_stats
// (MW = 2, NF = 2: 256 x 64 tiles for the 64-channel layers, 10 fragment reads per 16 MFMAs).
// CONV: A is the implicit im2col of an NHWC input with C % 64 == 0 (one tap per K-step; per-row tap-validity masks
// computed once per tile, padding taps load zeros through an offset past the descriptor).
template <int NF, int MW, bool CONV>
__global__ void __launch_bounds__(ST_NT, 2) k_gemm_stream(GemmArgs g) {
  constexpr int NWN = 4 / MW, WN = 16 * NF, TN = NWN * WN, TM = GBM * MW;  // waves along N, columns per wave / tile
  constexpr int NAI = 4 * MW;               // A DMA instructions per wave and K-step (TM rows, 8 per instruction)
  constexpr int NBI = TN / 32;              // B DMA instructions per wave and K-step (TN rows over 4 waves)
  constexpr int NI = NAI + NBI;             // DMA instructions per lane and K-step
  constexpr int BUF = TM * 128 + TN * 128;  // LDS bytes per buffer: A | B
  constexpr int NST = 8 + 2 * NF;           // stores per lane and epilogue: 8 output rows + the statistics
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr unsigned OOB = 0x80000000u;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), j = lane & 15, q = lane >> 4;
  const int wm = w / NWN, wn = w % NWN;
  const int ntm = (g.M + TM - 1) / TM, ntn = g.N / TN, T = ntm * ntn, nk = g.K / 64;
  const int nstat = (g.M + GBM - 1) / GBM;  // col_stats rows (128-row blocks)
  float* sbias = (float*)(smem + 2 * BUF);  // [N] bias | [N] statistics shift
  float* sshift = sbias + g.N;
  for (int c = threadIdx.x; c < g.N; c += ST_NT) {
    sbias[c] = g.bias ? g.bias[c] : 0.f;
    sshift[c] = g.col_stats ? g.stats_shift[c] : 0.f;
  }
  const float alpha = gemm_alpha(g);
  __syncthreads();  // (also drains these loads: the pipeline's vmcnt accounting starts from zero)
  const int nxwg = gridDim.x >> 3, xcd = blockIdx.x & 7, loc = blockIdx.x >> 3;
  const int t_beg = (int)((long long)xcd * T / 8), t_end = (int)((long long)(xcd + 1) * T / 8);
  const int my_tiles = t_end - t_beg > loc ? (t_end - t_beg - loc + nxwg - 1) / nxwg : 0;
  const int steps = my_tiles * nk;
  const long long a_bytes = CONV ? (long long)g.cN * g.cH * g.cW * g.cC * 2 : ((long long)(g.M - 1) * g.lda + g.K) * 2;
  const __amdgpu_buffer_rsrc_t ars = __builtin_amdgcn_make_buffer_rsrc((void*)g.A, (short)0, (int)a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)g.B, (short)0, (int)(((long long)(g.N - 1) * g.ldb + g.K) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(
      g.C, (short)0, (int)((long long)g.M * g.ldc * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t srs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)g.col_stats, (short)0, g.col_stats ? (int)((long long)nstat * g.N * 8) : 0, 0x00020000);
  // beta != 0: C_old from C, or (masked source) from beta_src with the bit mask
  const bool mold = !CONV && g.beta_mask != nullptr;  // (plain GEMMs only: the launcher never sends it a conv)
  const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
      mold ? (void*)g.beta_src : g.C, (short)0, (int)((long long)g.M * g.ldc * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t mrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)g.beta_mask, (short)0, mold ? (int)((long long)g.M * g.ldc / 8) : 0, 0x00020000);
  const unsigned lda2 = (unsigned)g.lda * 2u, ldb2 = (unsigned)g.ldb * 2u;
  const int cpt = CONV ? g.cC / 64 : 1;  // K-steps per tap
  const float inv_wo = CONV ? 1.f / (float)g.cWo : 0.f, inv_ho = CONV ? 1.f / (float)g.cHo : 0.f;
  unsigned rep = 0u;  // bit kh * KW set for every kh: spreads a kw mask over the kernel rows
  if constexpr (CONV)
    for (int kh = 0; kh < g.cKH; ++kh) rep |= 1u << (kh * g.cKW);

  // issue side: A row offsets (and conv tap masks) of the tile whose K-steps are being issued
  unsigned aoff[NAI], amask[NAI];
  int itm = 0, itn = 0;
  // issue() is called for s = 0, 1, 2, ... in order: the (tile, K-step, tap) position advances incrementally
  // (no per-step division: runtime divisions compile to ~20 SALU each)
  int i_k = 0, i_kt = 0, i_tap = 0, i_cs = 0, i_toff = 0;
  auto issue = [&](int s) {
    const int k = i_k, kt = i_kt;
    if (kt == 0) {
      tile_coords(t_beg + loc + k * nxwg, ntm, ntn, itm, itn);
#pragma unroll
      for (int i = 0; i < NAI; ++i) {
        const int r = 8 * NAI * w + 8 * i + (lane >> 3), m = itm * TM + r;
        const unsigned cb = (unsigned)((lane & 7) ^ ((r >> 1) & 7)) << 4;
        if constexpr (CONV) {
          // row decode by float-reciprocal division (exact after one correction: m < 2^24, launcher-checked) and
          // the tap mask from the valid kh / kw ranges: rows(kh) & (cols(kw) x rep) -- the per-tap loop and two
          // integer divisions per row were ~200 VALU per K-step (PMC, profiles/gemm_stream_pmc_r2.txt)
          int ow, oh;
          const int t2 = fdiv_rc(m < g.M ? m : 0, g.cWo, inv_wo, ow), n = fdiv_rc(t2, g.cHo, inv_ho, oh);
          const int ih0 = oh * g.cS - g.cP, iw0 = ow * g.cS - g.cP;
          aoff[i] = (unsigned)((((long long)n * g.cH + ih0) * g.cW + iw0) * g.cC * 2) + cb;  // wraps for padding
          amask[i] = m < g.M ? tap_mask(ih0, iw0, g.cH, g.cW, g.cKH, g.cKW, rep) : 0u;
        } else {
          aoff[i] = m < g.M ? (unsigned)m * lda2 + cb : OOB;
        }
      }
    }
    char* la = smem + (s & 1) * BUF;
    char* lb = la + TM * 128;
    const unsigned kb0 = (unsigned)kt * 128u;
    if constexpr (CONV) {
      const int tap = i_tap;
      const unsigned toff = (unsigned)i_toff;
#pragma unroll
      for (int i = 0; i < NAI; ++i)
        blds16(ars, la + (8 * NAI * w + 8 * i) * 128, (amask[i] >> tap) & 1u ? aoff[i] + toff : OOB, 0u);
      // next K-step: 64 more channels of this tap, or the next tap (kw, then kh), or tap 0 of the next tile
      if (++i_cs < cpt) {
        i_toff += 128;
      } else {
        i_cs = 0;
        ++i_tap;
        const int kh = i_tap / g.cKW;  // (once per tap)
        i_toff = ((kh * g.cW + (i_tap - kh * g.cKW)) * g.cC) * 2;
      }
      if (kt + 1 == nk) i_tap = i_cs = i_toff = 0;
    } else {
#pragma unroll
      for (int i = 0; i < NAI; ++i) blds16(ars, la + (8 * NAI * w + 8 * i) * 128, aoff[i], kb0);
    }
#pragma unroll
    for (int ib = 0; ib < NBI; ++ib) {  // LDS row WN v + 16 f + i holds weight row WN v + 4 NF (i >> 2) + 4 f + (i & 3)
      const int r = 8 * NBI * w + 8 * ib + (lane >> 3), v = r / WN, rl = r % WN, f = rl >> 4, i = rl & 15;
      const unsigned cb = (unsigned)((lane & 7) ^ ((r >> 1) & 7)) << 4;
      const int n = itn * TN + WN * v + 4 * NF * (i >> 2) + 4 * f + (i & 3);
      blds16(brs, lb + (8 * NBI * w + 8 * ib) * 128, (unsigned)n * ldb2 + cb, kb0);
    }
    if (++i_kt == nk) {
      i_kt = 0;
      ++i_k;
    }
  };

  // DPP sum over the 16 lanes of a row (lane j = 15 of each row ends with the total)
  auto rowsum16 = [](float x) {
    x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x111, 0xf, 0xf, true));
    x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x112, 0xf, 0xf, true));
    x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x114, 0xf, 0xf, true));
    x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x118, 0xf, 0xf, true));
    return x;
  };
  f32x4 acc[8][NF];
  // one K-step from LDS buffer `buf`; FIRST: the tile's first K-step (accumulators start from the MFMA's zero C)
  auto compute = [&](int buf, auto first) {
    const char* la = smem + buf * BUF;
    const char* lb = la + TM * 128;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      s16x8 xf[8], wf[NF];
#pragma unroll
      for (int m = 0; m < 8; ++m) xf[m] = *(const s16x8*)(la + lds_off(GBM * wm + 16 * m + j, 4 * s2 + q));
#pragma unroll
      for (int f = 0; f < NF; ++f) wf[f] = *(const s16x8*)(lb + lds_off(WN * wn + 16 * f + j, 4 * s2 + q));
#pragma unroll
      for (int m = 0; m < 8; ++m)
#pragma unroll
        for (int f = 0; f < NF; ++f)
          acc[m][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              wf[f], xf[m], (decltype(first)::value && s2 == 0) ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[m][f], 0, 0, 0);
    }
  };
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
  // output image (STG: 128 x 128 tiles, the output-heavy N % 128 == 0 calls; the 256 x 64 tiles of the read-heavy
  // N = 64 calls store straight from the accumulators -- staging them spilled): TM rows of RB bytes = CPR 16-B
  // chunks; chunk c of row r at c ^ img_sw(r), so the 16 rows of a fragment store and the 16 chunks of a read-out
  // pass each hit 16 distinct 16-B bank groups
  constexpr bool STG = NF == 2 && MW == 1;
  constexpr int RB = 2 * TN, CPR = TN / 8;
  static_assert(TM * CPR == 8 * ST_NT, "8 read-out passes");
  auto img_sw = [](int r) { return CPR == 16 ? (r & 15) : ((r >> 1) & 7); };
  st_v4u old[8];  // beta != 0: this tile's C_old rows (lane (q, j): row 16 m + j, columns c0 .. c0 + 4 NF - 1)
  unsigned omk[8];  // masked source: the mask byte of those columns (c0 % 8 == 0 for NF = 2, 0 or 4 for NF = 1)
  auto load_old = [&](int tm, int tn) {
    const int c0 = tn * TN + WN * wn + 4 * NF * q;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int row = tm * TM + GBM * wm + 16 * m + j;
      const unsigned o = row < g.M ? ((unsigned)row * (unsigned)g.ldc + c0) * 2u : OOB;
      if constexpr (NF == 2) {
        old[m] = __builtin_amdgcn_raw_buffer_load_b128(ors, o, 0, 0);
      } else {
        const st_v2u v = __builtin_amdgcn_raw_buffer_load_b64(ors, o, 0, 0);
        old[m] = st_v4u{v[0], v[1], 0u, 0u};
      }
    }
    if (mold) {  // issued after the 8 C_old loads: the waits below count 16
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const int row = tm * TM + GBM * wm + 16 * m + j;
        const unsigned o = row < g.M ? ((unsigned)row * (unsigned)g.ldc + c0) >> 3 : OOB;
        omk[m] = __builtin_amdgcn_raw_buffer_load_b8(mrs, o, 0, 0);
      }
    }
  };
  // epilogue of tile (tm, tn): lane (q, j) owns columns c0 .. c0 + 4 NF - 1 of rows tm*128 + 16 m + j.
  // more: the DMA of the next K-step was issued after the C_old loads.  FULL: no row past M.
  auto epilogue = [&](int tm, int tn, bool more, char* stg, auto full, auto acc_old) {
    constexpr bool FULL = decltype(full)::value, BETA = decltype(acc_old)::value;
    constexpr int NP = 2 * NF;  // column pairs per lane
    const int c0 = tn * TN + WN * wn + 4 * NF * q;
    if constexpr (BETA) {
      if (more) wait_vmcnt<NI>();
      else wait_vmcnt<0>();
    }
    f2 b2[NP], sh2[NP], s1[NP], sq[NP];
#pragma unroll
    for (int e = 0; e < NP; ++e) {
      b2[e] = *(const f2*)(sbias + c0 + 2 * e);
      sh2[e] = *(const f2*)(sshift + c0 + 2 * e);
      s1[e] = sq[e] = f2{0.f, 0.f};
    }
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int row = tm * TM + GBM * wm + 16 * m + j;
      const bool in = FULL || row < g.M;
      unsigned pk[NP];
#pragma unroll
      for (int e = 0; e < NP; ++e) {  // columns 2e, 2e + 1 = fragment e >> 1, elements 2 (e & 1) + {0, 1}
        const f32x4& a = acc[m][e >> 1];
        f2 x = f2{a[2 * (e & 1)], a[2 * (e & 1) + 1]} * alpha + b2[e];
        if constexpr (BETA) {
          f2 ov = f2{__uint_as_float(old[m][e] << 16), __uint_as_float(old[m][e] & 0xffff0000u)};
          if (mold) {
            const unsigned b = omk[m] >> ((c0 & 7) + 2 * e);
            ov = f2{(b & 1u) ? ov[0] : 0.f, (b & 2u) ? ov[1] : 0.f};
          }
          x += ov * g.beta;
        }
        pk[e] = __builtin_bit_cast(unsigned, __builtin_convertvector(x, bf2));
        // statistics of the values as stored (bf16)
        f2 d = f2{__uint_as_float(pk[e] << 16), __uint_as_float(pk[e] & 0xffff0000u)} - sh2[e];
        if (!FULL && !in) d = f2{0.f, 0.f};
        s1[e] += d;
        sq[e] += d * d;
      }
      if constexpr (STG) {  // into the LDS image of the tile: row rl (2 TN bytes), 16-B chunk 4 wn + q, swizzled
        const int rl = GBM * wm + 16 * m + j;
        *(st_v4u*)(stg + rl * RB + (((4 * wn + q) ^ img_sw(rl)) << 4)) = st_v4u{pk[0], pk[1], pk[2], pk[3]};
      } else {
        const unsigned o = in ? ((unsigned)row * (unsigned)g.ldc + c0) * 2u : OOB;
        if constexpr (NF == 2) __builtin_amdgcn_raw_buffer_store_b128(st_v4u{pk[0], pk[1], pk[2], pk[3]}, crs, o, 0, 2);
        else __builtin_amdgcn_raw_buffer_store_b64(st_v2u{pk[0], pk[1]}, crs, o, 0, 2);  // (nt: streamed output)
      }
    }
    if constexpr (STG) {
      // whole rows out of the LDS image: a wave instruction stores 4 rows x 256 or 8 rows x 128 contiguous bytes
      // (16 rows x 64 B straight from the accumulators is the fragment-shaped form the MI355X guide measures at 2x
      // TA_BUSY)
      __syncthreads();
#pragma unroll
      for (int ps = 0; ps < 8; ++ps) {
        const int idx = ST_NT * ps + (int)threadIdx.x, rl = idx / CPR, ch = idx % CPR, row = tm * TM + rl;
        const st_v4u v = *(const st_v4u*)(stg + rl * RB + ((ch ^ img_sw(rl)) << 4));
        const unsigned o = row < g.M ? ((unsigned)row * (unsigned)g.ldc + tn * TN + 8 * ch) * 2u : OOB;
        __builtin_amdgcn_raw_buffer_store_b128(v, crs, o, 0, 2);  // (nt: streamed output)
      }
    }
    float r1[2 * NP], r2[2 * NP];
#pragma unroll
    for (int e = 0; e < NP; ++e) {
      r1[2 * e] = rowsum16(s1[e][0]);
      r1[2 * e + 1] = rowsum16(s1[e][1]);
      r2[2 * e] = rowsum16(sq[e][0]);
      r2[2 * e + 1] = rowsum16(sq[e][1]);
    }
    const unsigned so = j == 15 ? ((unsigned)(tm * MW + wm) * (unsigned)g.N + c0) * 8u : OOB;
#pragma unroll
    for (int p = 0; p < NP; ++p)
      __builtin_amdgcn_raw_buffer_store_b128(
          st_v4u{__float_as_uint(r1[2 * p]), __float_as_uint(r2[2 * p]), __float_as_uint(r1[2 * p + 1]),
                 __float_as_uint(r2[2 * p + 1])},
          srs, so + 16u * p, 0, 0);
    if constexpr (STG) __syncthreads();  // the image is read out before its buffer takes the next DMA
  };

  // the stream: step s = (tile k, K-step kt), s = k * nk + kt; the DMA of step s + 1 is in flight during step s.
  // beta != 0: the tile's C_old rows are loaded at the top of its last K-step, ahead of the next step's DMA, so
  // their latency hides under that step's MFMAs
  const bool bta = g.beta != 0.f;
  if (steps > 0) issue(0);
  for (int k = 0; k < my_tiles; ++k) {
    int tm, tn;
    tile_coords(t_beg + loc + k * nxwg, ntm, ntn, tm, tn);
    for (int kt = 0; kt < nk; ++kt) {
      const int s = k * nk + kt;
      const bool lo = bta && kt == nk - 1;
      if (kt == 0 && k > 0) {  // outstanding: this step's DMA, then the previous epilogue's stores
        wait_vmcnt<NST>();
        if (lo) load_old(tm, tn);
        if (s + 1 < steps) issue(s + 1);
      } else if (lo) {  // outstanding: this step's DMA | C_old (8) | next DMA (NI)
        load_old(tm, tn);
        if (s + 1 < steps) {
          issue(s + 1);
          if (mold) wait_vmcnt<16 + NI>();
          else wait_vmcnt<8 + NI>();
        } else {
          if (mold) wait_vmcnt<16>();
          else wait_vmcnt<8>();
        }
      } else if (s + 1 < steps) {
        issue(s + 1);
        wait_vmcnt<NI>();
      } else {
        wait_vmcnt<0>();
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (kt == 0) compute(s & 1, std::true_type{});
      else compute(s & 1, std::false_type{});
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // every wave is done reading this buffer before it is refilled
      asm volatile("" ::: "memory");
    }
    // (STG: the tile's last K-step buffer, free after the barrier above, holds the output image)
    const bool full = tm * TM + GBM * wm + GBM <= g.M, more = (k + 1) * nk < steps;
    char* stg = smem + (((k + 1) * nk - 1) & 1) * BUF;
    if (bta) {
      if (full) epilogue(tm, tn, more, stg, std::true_type{}, std::true_type{});
      else epilogue(tm, tn, more, stg, std::false_type{}, std::true_type{});
    } else {
      if (full) epilogue(tm, tn, more, stg, std::true_type{}, std::false_type{});
      else epilogue(tm, tn, more, stg, std::false_type{}, std::false_type{});
    }
  }
}

// ---------------------------------------------------------------------------------------------------------
// k_direct_conv<C, KH, KW>: stride-1 implicit convolutions with 64 output channels whose input rows are too narrow
// for the LDS-staged implicit-GEMM kernels to stream well:
//   * <16, 4, 4>: the space-to-depth ResNet stem (ops/functional.py stem_s2d_index): 4 x 4 taps over the 16-channel
//     s2d input, no padding.  The generic kernels stage A through LDS in 16-B chunks per tap and ran it at 402 us
//     (1.3 TB/s) at batch 256;
//   * <64, 3, 3>: the 64-channel 3 x 3 / pad 1 convolutions of ResNet-50's layer 1 and their input gradients
//     (122-142 us each on the one-tile glds kernel at batch 256: 1.5 TB/s, 415 TF).
// Design:
//   * persistent workgroups walk 128-pixel M blocks (XCD-contiguous ranges); the 64 x K weight matrix stays in LDS
//     (K = KH KW C: 32 KB for the stem), rows permuted as in k_gemm_stream so a lane ends with 16 consecutive
//     output channels of one pixel;
//   * each wave owns 32 pixels of a block as two 16-pixel fragments and loads their A operands straight from
//     global memory into registers: K-slice s (32 k) of pixel j is 16 B = 8 channels per lane (k = 32 s + 8 q);
//     an input pixel is read by KH KW taps of up to KH KW output pixels, so these loads hit L1 / L2 after the first;
//     padding taps load zeros through an out-of-range offset.  The next fragment's loads are in flight during this
//     fragment's MFMAs and epilogue (two register buffers);
//   * epilogue from registers: alpha, bias, bf16, 32 B per pixel and lane (nt stores); the BN column statistics of
//     the block are summed over both fragments in registers, over 16 pixels by DPP, over the 4 waves in LDS in wave
//     order: one col_stats row per 128-row block (the layout k_bn_finalize reduces).
// Requirements (launcher): conv == 1, stride 1, N = 64, K = KH KW C, bf16 out, no beta / ReLU / split / remap,
// byte ranges < 2^31.
// ---------------------------------------------------------------------------------------------------------
constexpr int DC_NT = 256;
template <int C, int KH, int KW>
struct DirectConv {
  static constexpr int K = KH * KW * C, NS = K / 32;                 // K, 32-wide K slices
  static constexpr int LDS = K * 128 + 2 * 64 * 4 + 4 * 64 * 8;      // weights | bias, shift | statistics
  static_assert(K % 64 == 0 && (C % 8) == 0 && (32 % C == 0 || C % 32 == 0), "slices of whole 8-channel chunks");
};
template <int C, int KH, int KW>
__global__ void __launch_bounds__(DC_NT, 2) k_direct_conv(GemmArgs g) {
  using T = DirectConv<C, KH, KW>;
  constexpr int NS = T::NS;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr unsigned OOB = 0x80000000u;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), j = lane & 15, q = lane >> 4;
  char* lw = smem;  // weights: K-tile kt (64 k) at kt * 8 KB, row r (128 B, XOR-swizzled chunks: lds_off)
  float* sbias = (float*)(smem + T::K * 128);
  float* sshift = sbias + 64;
  float* sst = sshift + 64;  // [4 waves][64] x (sum, sumsq)
  // weight row r = 16 f + i of the LDS image holds output channel 16 (i >> 2) + 4 f + (i & 3): lane (q, j) of
  // fragment f then holds channels 16 q + 4 f .. + 3, i.e. channels 16 q .. 16 q + 15 over the 4 fragments
  const unsigned short* Bp = (const unsigned short*)g.B;
  for (int e = threadIdx.x; e < T::K / 64 * 64 * 8; e += DC_NT) {
    const int c = e & 7, r = (e >> 3) & 63, kt = e >> 9, f = r >> 4, i = r & 15;
    const int co = 16 * (i >> 2) + 4 * f + (i & 3);
    *(uint4*)(lw + kt * 8192 + lds_off(r, c)) = *(const uint4*)(Bp + (size_t)co * g.ldb + kt * 64 + c * 8);
  }
  if (threadIdx.x < 64) {
    sbias[threadIdx.x] = g.bias ? g.bias[threadIdx.x] : 0.f;
    sshift[threadIdx.x] = g.col_stats ? g.stats_shift[threadIdx.x] : 0.f;
  }
  const float alpha = gemm_alpha(g);
  __syncthreads();
  const int nblk = (g.M + GBM - 1) / GBM, nxwg = gridDim.x >> 3, xcd = blockIdx.x & 7, loc = blockIdx.x >> 3;
  const int b_beg = (int)((long long)xcd * nblk / 8), b_end = (int)((long long)(xcd + 1) * nblk / 8);
  const int nmy = b_end - b_beg > loc ? (b_end - b_beg - loc + nxwg - 1) / nxwg : 0;
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)g.A, (short)0, (int)((long long)g.cN * g.cH * g.cW * C * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(
      g.C, (short)0, (int)((long long)g.M * g.ldc * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t srs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)g.col_stats, (short)0, g.col_stats ? (int)((long long)nblk * 64 * 8) : 0, 0x00020000);
  const bool stats = g.col_stats != nullptr;
  const float inv_wo = 1.f / (float)g.cWo, inv_ho = 1.f / (float)g.cHo;
  typedef unsigned v4u_ __attribute__((ext_vector_type(4)));
  // K-slice s of this lane: 8 channels c0 = (32 s + 8 q) % C of tap t = (32 s + 8 q) / C = (kh, kw)
  auto slice_tap = [&](int s) { return (32 * s + 8 * q) / C; };
  auto slice_off = [&](int s) {  // byte offset of the slice's chunk relative to the pixel's (ih0, iw0) corner
    const int t = slice_tap(s), c0 = (32 * s + 8 * q) % C;
    return (((t / KW) * g.cW + (t % KW)) * C + c0) * 2;
  };
  // fragment (block i of this workgroup's list, half m): pixel 128 b + 32 w + 16 m + j
  auto load_frag = [&](v4u_(&dst)[NS], int i, int m) {
    const int b = b_beg + loc + i * nxwg;
    const int p = b * GBM + 32 * w + 16 * m + j;
    int base = 0;
    unsigned valid = 0u;  // bit t: tap t inside the input
    if (i < nmy && p < g.M) {
      int ow, oh;
      const int t2 = fdiv_rc(p, g.cWo, inv_wo, ow), n = fdiv_rc(t2, g.cHo, inv_ho, oh);
      const int ih0 = oh - g.cP, iw0 = ow - g.cP;
      base = ((n * g.cH + ih0) * g.cW + iw0) * C * 2;  // (negative for a padded corner: used only when valid)
#pragma unroll
      for (int t = 0; t < KH * KW; ++t) {
        const int ih = ih0 + t / KW, iw = iw0 + t % KW;
        valid |= (ih >= 0 && ih < g.cH && iw >= 0 && iw < g.cW) ? 1u << t : 0u;
      }
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const unsigned o = (valid >> slice_tap(s)) & 1u ? (unsigned)(base + slice_off(s)) : OOB;
      dst[s] = __builtin_amdgcn_raw_buffer_load_b128(xrs, o, 0, 0);
    }
  };
  auto rowsum16 = [](float x) {
    x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x111, 0xf, 0xf, true));
    x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x112, 0xf, 0xf, true));
    x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x114, 0xf, 0xf, true));
    x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x118, 0xf, 0xf, true));
    return x;
  };
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
  f2 s1[8], sq[8];  // this lane's statistics of channels 16 q + 2 e, + 1 over the block's fragments so far
  // one fragment: MFMAs, output, statistics
  auto frag = [&](const v4u_(&a)[NS], int b, int m) {
    f32x4 acc[4];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const char* lk = lw + (s >> 1) * 8192;
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        const s16x8 wf = *(const s16x8*)(lk + lds_off(16 * f + j, 4 * (s & 1) + q));
        acc[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, __builtin_bit_cast(s16x8, a[s]),
                                                         s == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[f], 0, 0, 0);
      }
    }
    const int p = b * GBM + 32 * w + 16 * m + j;
    const bool in = p < g.M;
    unsigned pk[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {  // channels 16 q + 2 e, + 1 = fragment e >> 1, elements 2 (e & 1) + {0, 1}
      const int c = 16 * q + 2 * e;
      const f32x4& v = acc[e >> 1];
      const f2 x = f2{v[2 * (e & 1)], v[2 * (e & 1) + 1]} * alpha + f2{sbias[c], sbias[c + 1]};
      pk[e] = __builtin_bit_cast(unsigned, __builtin_convertvector(x, bf2));
      f2 d = f2{__uint_as_float(pk[e] << 16), __uint_as_float(pk[e] & 0xffff0000u)} - f2{sshift[c], sshift[c + 1]};
      if (!in) d = f2{0.f, 0.f};
      s1[e] += d;
      sq[e] += d * d;
    }
    const unsigned o = in ? ((unsigned)p * (unsigned)g.ldc + 16u * q) * 2u : OOB;
    __builtin_amdgcn_raw_buffer_store_b128(v4u_{pk[0], pk[1], pk[2], pk[3]}, crs, o, 0, 2);
    __builtin_amdgcn_raw_buffer_store_b128(v4u_{pk[4], pk[5], pk[6], pk[7]}, crs, o + 16u, 0, 2);
  };
  auto block_stats = [&](int b) {  // the block's statistics row; resets the running sums
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float a0 = rowsum16(s1[e][0]), a1 = rowsum16(s1[e][1]);
      const float b0 = rowsum16(sq[e][0]), b1 = rowsum16(sq[e][1]);
      if (j == 15) *(float4*)(sst + 2 * (w * 64 + 16 * q + 2 * e)) = float4{a0, b0, a1, b1};
      s1[e] = sq[e] = f2{0.f, 0.f};
    }
    __syncthreads();
    if (threadIdx.x < 64) {
      float s = 0.f, s2 = 0.f;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        s += sst[2 * (v * 64 + threadIdx.x)];
        s2 += sst[2 * (v * 64 + threadIdx.x) + 1];
      }
      __builtin_amdgcn_raw_buffer_store_b64(st_v2u{__float_as_uint(s), __float_as_uint(s2)}, srs,
                                            ((unsigned)b * 64u + threadIdx.x) * 8u, 0, 0);
    }
    __syncthreads();
  };
#pragma unroll
  for (int e = 0; e < 8; ++e) s1[e] = sq[e] = f2{0.f, 0.f};
  v4u_ a0[NS], a1[NS];
  if (nmy > 0) load_frag(a0, 0, 0);
  for (int i = 0; i < nmy; ++i) {
    const int b = b_beg + loc + i * nxwg;
    load_frag(a1, i, 1);      // this block's second fragment, in flight during the first one's work
    frag(a0, b, 0);
    load_frag(a0, i + 1, 0);  // the next block's first fragment (past the end: zeros, no traffic)
    frag(a1, b, 1);
    if (stats) block_stats(b);
  }
}

// ---------------------------------------------------------------------------------------------------------
// k_conv3x3_rows: the 64-channel 3 x 3 / pad 1 / stride 1 convolutions on rows of at most 64 pixels (ResNet-50's
// layer 1 at 56 x 56: forward and input gradient).  k_direct_conv<64, 3, 3> loads each output pixel's 576 k straight
// from global memory into MFMA registers: every input pixel is fetched 9 times and each wave-load touches 64
// separate 16-B pieces, so its vector L1 makes one access per lane (PMC: 63.5 M L1 accesses per call, ~0.85 per
// cycle and CU over the kernel, MFMA busy 0.19; profiles/conv3x3_rows_r9.txt).  Here a workgroup walks consecutive
// output rows (n, oh) and keeps their input rows in an LDS ring:
//   * 4 row slots of 66 pixels x 128 B (pixel iw at slot position iw + 1; position 0 and those past W stay zero),
//     16-B chunks XOR-swizzled by position & 7 (one ds_read_b128 lane group = 16 pixels of one chunk covers the 64
//     banks once); each input row is fetched once per workgroup with coalesced 16-B loads, issued one output row
//     ahead and written to its slot after that row's MFMAs (slot (r + 2) & 3 held row r - 2, no longer read);
//   * wave w owns output channels 16 w .. 16 w + 15: its 16 x 576 weight fragment (18 K-slices) stays in 72 VGPRs
//     for the kernel's life, and per slice it reads the row's 16-pixel A fragments from LDS (one ds_read_b128 per
//     MFMA).  The taps of a padding row (oh = 0 / H - 1) are skipped, uniformly per row;
//   * epilogue: alpha, bias, bf16 into a double-buffered LDS output image (64 pixels x 128 B), stored as whole
//     128-B pixel rows after the row's barrier (one barrier per output row); the BN column statistics (sum, sumsq
//     of out - shift) stay in registers over the workgroup's rows and are written once, row v of col_stats for
//     workgroup v, with the rows from grid to nblk - 1 zeroed (k_bn_finalize sums every row).
// Requirements (launcher): those of k_direct_conv<64, 3, 3>, W <= 64, grid <= nblk when col_stats.
// ---------------------------------------------------------------------------------------------------------
constexpr int CR_NT = 256, CR_SLOT = 66 * 128, CR_OUT = 64 * 128;
constexpr int CR_LDS = 4 * CR_SLOT + 2 * CR_OUT;
__device__ __forceinline__ int cr_off(int px, int chunk) { return px * 128 + ((chunk ^ (px & 7)) << 4); }

// The row kernels' BN column statistics: lane (q, j) of wave w holds the sums of channels 16 w + 4 q + e over its
// pixels; summed over j by DPP, written as row vid of col_stats ([nblk][NC][2]), and the rows from grid to nblk - 1
// zeroed.
template <int NC = 64>
__device__ __forceinline__ void rows_stats_out(const GemmArgs& g, const float (&s1)[4], const float (&sq)[4], int vid,
                                               int grid, int w, int q, int j) {
  auto rowsum16 = [](float x) {
    x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x111, 0xf, 0xf, true));
    x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x112, 0xf, 0xf, true));
    x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x114, 0xf, 0xf, true));
    x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x118, 0xf, 0xf, true));
    return x;
  };
  const int nblk = (g.M + GBM - 1) / GBM;
  const __amdgpu_buffer_rsrc_t srs =
      __builtin_amdgcn_make_buffer_rsrc((void*)g.col_stats, (short)0, (int)((long long)nblk * NC * 8), 0x00020000);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float a = rowsum16(s1[e]), b = rowsum16(sq[e]);
    if (j == 15)
      __builtin_amdgcn_raw_buffer_store_b64(st_v2u{__float_as_uint(a), __float_as_uint(b)}, srs,
                                            ((unsigned)vid * NC + 16u * w + 4u * q + e) * 8u, 0, 0);
  }
  for (int row = grid + vid; row < nblk; row += grid)
    if (threadIdx.x < NC)
      __builtin_amdgcn_raw_buffer_store_b64(st_v2u{0u, 0u}, srs, ((unsigned)row * NC + threadIdx.x) * 8u, 0, 0);
}

// C = 64: 4 waves (3 workgroups per CU), rows <= 64 pixels; C = 128 (layer 2, 28 x 28): 8 waves of 16 output
// channels each, 144 weight VGPRs per lane (one workgroup per CU), rows <= 32 pixels.  16-B chunks of a pixel row
// XOR-swizzled by pixel & (C / 8 - 1).  A ds_read_b128 lane group holds lanes j in {0-3, 12-15} of one lane quarter
// q and j in {4-11} of its partner q ^ 1.  With 128-B rows (C = 64) that is conflict-free for every tap shift as
// is; with 256-B rows (C = 128) no pixel swizzle is (PMC: 25 % of the LDS cycles were conflicts), so for C = 128
// lane j takes pixel cr_pix(j) = j < 8 ? j ^ 4 : j -- one half of a group then reads pixels {0-3, 8-11} + s, the
// other {4-7, 12-15} + s, sets closed under + 8 -- and quarter q of K-slice h reads chunk cr_chunk(h, q) = 8 (q & 1)
// + 4 (q >> 1) + h, so the halves' chunks differ by 8: x ^ 8 = x + 8 (mod 16) keeps each half inside its own bank
// positions for every tap shift (brute-force checked over all shifts).
template <int C>
struct RowConv {
  static constexpr int NT = 4 * C, CH = C / 8, PXB = 2 * C, NS = 9 * C / 32, HS = C / 32;
  static constexpr int SPX = C == 64 ? 66 : 34, SLOT = SPX * PXB, OUT = (SPX - 2) * PXB, LDS = 4 * SLOT + 2 * OUT;
  static constexpr int NL = ((SPX - 2) * CH + NT - 1) / NT;  // 16-B row pieces per thread
};
template <int C>
__device__ __forceinline__ int crc_off(int px, int chunk) {
  return px * (2 * C) + ((chunk ^ (px & (C / 8 - 1))) << 4);
}
template <int C>
__device__ __forceinline__ int cr_pix(int j) { return C == 64 ? j : (j < 8 ? j ^ 4 : j); }
template <int C>
__device__ __forceinline__ int cr_chunk(int h, int q) { return C == 64 ? 4 * h + q : 8 * (q & 1) + 4 * (q >> 1) + h; }
template <int NF, int C = 64>  // NF: 16-pixel fragments per row, ceil(W / 16)
__global__ void __launch_bounds__(4 * C, C == 64 ? 3 : 1) k_conv3x3_rows(GemmArgs g) {
  using T = RowConv<C>;
  constexpr int NT = T::NT, NS = T::NS, NL = T::NL;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  typedef unsigned v4u_ __attribute__((ext_vector_type(4)));
  constexpr unsigned OOB = 0x80000000u;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), j = lane & 15, q = lane >> 4;
  const int H = g.cH, W = g.cW, R = g.cN * g.cH;  // output rows (n, oh); stride 1 / pad 1: input rows alike
  const int grid = gridDim.x;
  // XCD-contiguous row ranges: the workgroups of one XCD take neighbouring ranges (shared boundary rows in its L2)
  const int vid = (grid & 7) == 0 ? (int)(blockIdx.x & 7) * (grid >> 3) + (int)(blockIdx.x >> 3) : (int)blockIdx.x;
  const int r_beg = (int)((long long)vid * R / grid), r_end = (int)((long long)(vid + 1) * R / grid);
  for (int e = threadIdx.x; e < 4 * T::SLOT / 16; e += NT) *(v4u_*)(smem + e * 16) = v4u_{0u, 0u, 0u, 0u};
  // weights: lane (q, j) of slice s = (tap, h) holds channel 16 w + j, k = tap * C + 8 cr_chunk(h, q) .. + 7
  const unsigned short* Bp = (const unsigned short*)g.B;
  const int pj = cr_pix<C>(j);  // this lane's pixel within a 16-pixel fragment
  s16x8 wf[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s)
    wf[s] = *(const s16x8*)(Bp + (size_t)(16 * w + j) * g.ldb + (s / T::HS) * C + 8 * cr_chunk<C>(s % T::HS, q));
  const float alpha = gemm_alpha(g);
  float bias[4], shift[4], s1[4], sq[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int c = 16 * w + 4 * q + e;
    bias[e] = g.bias ? g.bias[c] : 0.f;
    shift[e] = g.col_stats ? g.stats_shift[c] : 0.f;
    s1[e] = sq[e] = 0.f;
  }
  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)g.A, (short)0, (int)((long long)R * W * T::PXB), 0x00020000);
  const __amdgpu_buffer_rsrc_t crs =
      __builtin_amdgcn_make_buffer_rsrc(g.C, (short)0, (int)((long long)g.M * g.ldc * 2), 0x00020000);
  // input row gr: W * CH pieces of 16 B (pixel e / CH, chunk e % CH), NL per thread
  auto row_load = [&](v4u_(&st)[NL], int gr) {
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int e = threadIdx.x + NT * i;
      const unsigned o =
          (gr >= 0 && gr < R && e < W * T::CH) ? (unsigned)gr * (unsigned)W * T::PXB + (unsigned)e * 16u : OOB;
      st[i] = __builtin_amdgcn_raw_buffer_load_b128(xrs, o, 0, 0);
    }
  };
  auto row_store = [&](const v4u_(&st)[NL], int gr) {
    if (gr < 0 || gr >= R) return;
    char* sl = smem + (gr & 3) * T::SLOT;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int e = threadIdx.x + NT * i;
      if (e < W * T::CH) *(v4u_*)(sl + crc_off<C>(e / T::CH + 1, e % T::CH)) = st[i];
    }
  };
  v4u_ st[NL];
  __syncthreads();  // ring zeroed before any row lands in it
  for (int d = -1; d <= 1; ++d) {
    row_load(st, r_beg + d);
    row_store(st, r_beg + d);
  }
  __syncthreads();
  for (int r = r_beg; r < r_end; ++r) {
    const int oh = r % H;
    const bool pre = r + 1 < r_end;  // the next output row needs input row r + 2
    if (pre) row_load(st, r + 2);
    f32x4 acc[NF];
#pragma unroll
    for (int f = 0; f < NF; ++f) acc[f] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      if (oh - 1 + kh < 0 || oh - 1 + kh >= H) continue;
      const char* sl = smem + ((r - 1 + kh) & 3) * T::SLOT;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
#pragma unroll
        for (int h = 0; h < T::HS; ++h) {
          const int s = (kh * 3 + kw) * T::HS + h;
#pragma unroll
          for (int f = 0; f < NF; ++f) {
            const s16x8 a = *(const s16x8*)(sl + crc_off<C>(16 * f + pj + kw, cr_chunk<C>(h, q)));
            acc[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[s], a, acc[f], 0, 0, 0);
          }
        }
      }
    }
    // lane (q, j) of fragment f: channels 16 w + 4 q + e of pixel 16 f + cr_pix(j)
    char* ob = smem + 4 * T::SLOT + (r & 1) * T::OUT;
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const int px = 16 * f + pj;
      unsigned short hv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        hv[e] = f2bf_rne(acc[f][e] * alpha + bias[e]);
        const float d = px < W ? bf2f(hv[e]) - shift[e] : 0.f;
        s1[e] += d;
        sq[e] += d * d;
      }
      *(uint2*)(ob + crc_off<C>(px, 2 * w + (q >> 1)) + (q & 1) * 8) =
          uint2{hv[0] | ((unsigned)hv[1] << 16), hv[2] | ((unsigned)hv[3] << 16)};
    }
    if (pre) row_store(st, r + 2);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int e = threadIdx.x + NT * i;
      if (e < W * T::CH) {
        const int px = e / T::CH, c = e % T::CH;
        const v4u_ v = *(const v4u_*)(ob + crc_off<C>(px, c));
        __builtin_amdgcn_raw_buffer_store_b128(v, crs, ((unsigned)(r * W + px) * (unsigned)g.ldc + 8u * c) * 2u, 0, 2);
      }
    }
  }
  if (g.col_stats) rows_stats_out<C>(g, s1, sq, vid, grid, w, q, j);
}

// k_conv_s2d_rows: the space-to-depth ResNet stem (ops/functional.py stem_s2d_index: 4 x 4 taps over a 16-channel
// input, no padding, stride 1, 64 outputs) in the row-ring form of k_conv3x3_rows, replacing k_direct_conv<16, 4, 4>
// (207 us at batch 256, the same one-access-per-lane vector-L1 pattern):
//   * 5 row slots of up to 128 input pixels x 32 B (no swizzle needed: the 16 lanes of a ds_read_b128 group read 16
//     pixels' alternating 16-B halves, 256 distinct bytes); output row (n, oh) reads input rows oh .. oh + 3 of image
//     n, the next one's new row is fetched during its MFMAs; the first row of a workgroup or of an image loads all
//     four (one extra barrier);
//   * wave w: channels 16 w .. + 15, its 16 x 256 weight fragment (8 K-slices; slice s = taps 2 s, 2 s + 1 of kernel
//     row s >> 1) in 32 VGPRs; NF = ceil(Wo / 16) A fragments per slice from LDS;
//   * epilogue as k_conv3x3_rows (double-buffered LDS output image of up to 128 pixels, statistics per workgroup).
// Requirements (launcher): Wi <= 128 (Wo <= 125), grid <= nblk when col_stats.
constexpr int CS_SLOT = 128 * 32, CS_OUT = 128 * 128, CS_LDS = 5 * CS_SLOT + 2 * CS_OUT;
template <int NF>
__global__ void __launch_bounds__(CR_NT, 3) k_conv_s2d_rows(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  typedef unsigned v4u_ __attribute__((ext_vector_type(4)));
  constexpr unsigned OOB = 0x80000000u;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), j = lane & 15, q = lane >> 4;
  const int Hi = g.cH, Wi = g.cW, Ho = g.cHo, Wo = g.cWo, R = g.cN * Ho;
  const int grid = gridDim.x;
  const int vid = (grid & 7) == 0 ? (int)(blockIdx.x & 7) * (grid >> 3) + (int)(blockIdx.x >> 3) : (int)blockIdx.x;
  const int r_beg = (int)((long long)vid * R / grid), r_end = (int)((long long)(vid + 1) * R / grid);
  // slots past Wi are read by the tail fragments' taps (discarded pixels): keep them finite
  for (int e = threadIdx.x; e < 5 * CS_SLOT / 16; e += CR_NT) *(v4u_*)(smem + e * 16) = v4u_{0u, 0u, 0u, 0u};
  const unsigned short* Bp = (const unsigned short*)g.B;
  s16x8 wf[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) wf[s] = *(const s16x8*)(Bp + (size_t)(16 * w + j) * g.ldb + 32 * s + 8 * q);
  const float alpha = gemm_alpha(g);
  float bias[4], shift[4], s1[4], sq[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int c = 16 * w + 4 * q + e;
    bias[e] = g.bias ? g.bias[c] : 0.f;
    shift[e] = g.col_stats ? g.stats_shift[c] : 0.f;
    s1[e] = sq[e] = 0.f;
  }
  const int RI = g.cN * Hi;  // input rows
  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)g.A, (short)0, (int)((long long)RI * Wi * 32), 0x00020000);
  const __amdgpu_buffer_rsrc_t crs =
      __builtin_amdgcn_make_buffer_rsrc(g.C, (short)0, (int)((long long)g.M * g.ldc * 2), 0x00020000);
  auto row_load = [&](int gi) {  // input row gi: Wi * 2 pieces of 16 B, one per thread
    const unsigned o = (gi < RI && (int)threadIdx.x < Wi * 2) ? ((unsigned)gi * (unsigned)Wi * 32u + threadIdx.x * 16u) : OOB;
    return __builtin_amdgcn_raw_buffer_load_b128(xrs, o, 0, 0);
  };
  auto row_store = [&](const v4u_& v, int gi) {
    if (gi < RI && (int)threadIdx.x < Wi * 2) *(v4u_*)(smem + (gi % 5) * CS_SLOT + threadIdx.x * 16) = v;
  };
  __syncthreads();  // ring zeroed
  for (int r = r_beg; r < r_end; ++r) {
    const int n = r / Ho, oh = r - n * Ho, gi0 = n * Hi + oh;  // input rows gi0 .. gi0 + 3
    if (r == r_beg || oh == 0) {  // a workgroup's or an image's first row: all four rows (the last barrier freed them)
      v4u_ v[4];
#pragma unroll
      for (int d = 0; d < 4; ++d) v[d] = row_load(gi0 + d);
#pragma unroll
      for (int d = 0; d < 4; ++d) row_store(v[d], gi0 + d);
      __syncthreads();
    }
    const bool pre = r + 1 < r_end && oh + 1 < Ho;  // the next row of this image needs input row gi0 + 4
    v4u_ nx;
    if (pre) nx = row_load(gi0 + 4);
    f32x4 acc[NF];
#pragma unroll
    for (int f = 0; f < NF; ++f) acc[f] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 8; ++s) {  // kernel row s >> 1, column 2 (s & 1) + (q >> 1), channels 8 (q & 1) .. + 7
      const char* sl = smem + ((gi0 + (s >> 1)) % 5) * CS_SLOT + (2 * (s & 1) + (q >> 1)) * 32 + (q & 1) * 16;
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        const s16x8 a = *(const s16x8*)(sl + (16 * f + j) * 32);
        acc[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[s], a, acc[f], 0, 0, 0);
      }
    }
    char* ob = smem + 5 * CS_SLOT + (r & 1) * CS_OUT;
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const int px = 16 * f + j;
      unsigned short hv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        hv[e] = f2bf_rne(acc[f][e] * alpha + bias[e]);
        const float d = px < Wo ? bf2f(hv[e]) - shift[e] : 0.f;
        s1[e] += d;
        sq[e] += d * d;
      }
      *(uint2*)(ob + cr_off(px, 2 * w + (q >> 1)) + (q & 1) * 8) =
          uint2{hv[0] | ((unsigned)hv[1] << 16), hv[2] | ((unsigned)hv[3] << 16)};
    }
    if (pre) row_store(nx, gi0 + 4);  // slot of row gi0 - 1, last read by the previous output row
    __syncthreads();
    for (int e = threadIdx.x; e < Wo * 8; e += CR_NT) {
      const int px = e >> 3, c = e & 7;
      const v4u_ v = *(const v4u_*)(ob + cr_off(px, c));
      __builtin_amdgcn_raw_buffer_store_b128(v, crs, ((unsigned)(r * Wo + px) * (unsigned)g.ldc + 8u * c) * 2u, 0, 2);
    }
  }
  if (g.col_stats) rows_stats_out(g, s1, sq, vid, grid, w, q, j);
}

// Split-K combine: C = alpha * sum_s ws[s] (+bias) (+beta*C) (ReLU).  256 threads = 64 consecutive elements x 4
// split lanes (lane l sums slabs l, l+4, ...; the 4 partials are added in lane order: deterministic), so
// thousands of slabs of a small weight gradient are read by many threads with 256-B row segments.
// With wperm_T > 0 the column is remapped to torch's weight layout (see GemmArgs) and padded channels dropped.
constexpr int RED_EL = 64, RED_LANES = 4;
// Masked accumulation source for the GEMM kernels without the epilogue form (dca_ops_gemm): C[m][n] =
// beta_src[m][n] * bit(m * ldc + n) over the M x N output (bf16), before a plain beta = 1 GEMM.
__global__ void __launch_bounds__(256) k_masked_copy(const unsigned short* __restrict__ src,
                                                     const unsigned char* __restrict__ mk,
                                                     unsigned short* __restrict__ dst, int M, int N, int ldc) {
  const long total = (long)M * (N / 8);
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long row = i / (N / 8), c8 = (i % (N / 8)) * 8, o = row * ldc + c8;
    const uint4 v = *(const uint4*)(src + o);
    const unsigned b = mk[o >> 3];
    unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k)
      w[k] = ((b >> (2 * k)) & 1u ? (w[k] & 0xffffu) : 0u) | ((b >> (2 * k + 1)) & 1u ? (w[k] & 0xffff0000u) : 0u);
    *(uint4*)(dst + o) = uint4{w[0], w[1], w[2], w[3]};
  }
}

__global__ void __launch_bounds__(256) k_gemm_splitk_reduce(GemmArgs g) {
  __shared__ float red[RED_LANES][RED_EL];
  const size_t total = (size_t)g.M * g.N;
  const float alpha = gemm_alpha(g);
  const int el = threadIdx.x % RED_EL, sl = threadIdx.x / RED_EL;
  for (size_t base = (size_t)blockIdx.x * RED_EL; base < total; base += (size_t)gridDim.x * RED_EL) {
    const size_t i = base + el;
    float v = 0.f;
    if (i < total) {
      const float* p = g.ws + i;
      int s = sl;
#pragma unroll 4
      for (; s < g.splits; s += RED_LANES) v += p[(size_t)s * total];
    }
    red[sl][el] = v;
    __syncthreads();
    if (sl == 0 && i < total) {
      v = (red[0][el] + red[1][el]) + (red[2][el] + red[3][el]);
      const int row = (int)(i / g.N), col = (int)(i % g.N);
      size_t o = (size_t)row * g.ldc + col;
      bool keep = true;
      if (g.wperm_T > 0) {
        const int tap = col / g.wperm_Cpad, c = col - tap * g.wperm_Cpad;
        keep = c < g.wperm_C && tap < g.wperm_T;
        o = ((size_t)row * g.wperm_C + c) * g.wperm_T + tap;
      }
      if (keep) {
        v *= alpha;
        if (g.bias) v += g.bias[col];
        if (g.beta != 0.f) v += g.beta * (g.out_bf16 ? bf2f(((const unsigned short*)g.C)[o]) : ((const float*)g.C)[o]);
        if (g.relu) v = v > 0.f ? v : 0.f;
        if (g.out_bf16) ((unsigned short*)g.C)[o] = f2bf_rne(v);
        else ((float*)g.C)[o] = v;
      }
    }
    __syncthreads();
  }
}

}  // namespace ops
}  // namespace dca
