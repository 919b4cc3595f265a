// Weight-gradient GEMM for the ops layer:  C[m][n] = sum_k A[k][m] * B[k][n]  over a split-K range, written
// to the fp32 split-K slab (k_gemm_splitk_reduce then sums the slabs and remaps to torch's weight layout).
//
//   A = dY [P][lda] bf16   (k = output pixel, m = output channel)
//   B = X  [P][ldb] bf16   (n = input channel), or conv == 2: the implicit im2col of an NHWC input,
//                          n = tap * C + c, gathered 8 channels (16 B) of one tap at a time
//
// Both operands are K-OUTER (pixel-major): the MFMA wants 8 consecutive k per lane, which are 8 different
// rows of the natural layout.  Instead of transposing in registers on the way into LDS (what the general
// k_gemm does for ta/tb operands: 8-byte LDS writes and bit shuffles), the tiles are stored in LDS exactly as
// they come from HBM -- [64 pixels][BM or BN channels], 16-B chunks, coalesced row loads -- and the MFMA
// fragments are read with the CDNA4 transposing LDS read ds_read_b64_tr_b16 (2 reads = one 16x16x32 operand).
//
// K permutation: the MFMA only needs A and B to agree on which physical k each (lane group g, element j)
// holds.  Element j < 4 of group g is pixel row 4g + j (read 0 covers rows 0..15), element j >= 4 is row
// 16 + 4g + (j - 4) (read 1 covers rows 16..31); so the two 16-lane groups of a 32-lane half read 8
// consecutive rows, and with a row stride of 8 banks (mod 64) those 8 rows x 32 B hit 64 distinct banks.
//
// Tiles BM x BN in {64,128}^2 (no MFMA work wasted on the 64-channel layers), 4 waves (WAVES_M x WAVES_N),
// K-tile 64 pixels, LDS double-buffered with register prefetch of the next tile during the MFMAs, one barrier
// per K-tile.  Work items (tile, split) are dealt out so that the tiles of one K range share an XCD (its L2
// holds the dY / X rows they all read).
#pragma once
#include "ops_gemm.hip"

namespace dca {
namespace ops {

typedef short s16x4 __attribute__((ext_vector_type(4)));

// q = p / d, r = p % d for 0 <= p < 2^24 via a float reciprocal and one correction step (the pixel decode of the
// implicit-im2col gather runs per row per K-tile: integer division would make the loader VALU-bound)
__device__ __forceinline__ int fdivmod(int p, int d, float inv, int& r) {
  int q = (int)((float)p * inv);
  r = p - q * d;
  if (r < 0) {
    --q;
    r += d;
  } else if (r >= d) {
    ++q;
    r -= d;
  }
  return q;
}

__device__ __forceinline__ s16x4 lds_tr16(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((s16x4 __attribute__((address_space(3)))*)(p));
}

template <int BM, int BN, int WAVES_M>
struct WgradTile {
  static constexpr int WAVES_N = 4 / WAVES_M;
  static constexpr int FM = BM / (16 * WAVES_M), FN = BN / (16 * WAVES_N);
  static constexpr int BK = 64;  // (128-pixel K-tiles measured slower on the 64-channel 3x3: profiles/wgrad_bk128_ab_r5o.log)
  static constexpr int SA = BM * 2 + 32, SB = BN * 2 + 32;  // LDS row strides: 8 banks mod 64
  static constexpr int A_BYTES = BK * SA, B_BYTES = BK * SB, BUF = A_BYTES + B_BYTES, LDS = 2 * BUF;
  static constexpr int CA = BM / 8, CB = BN / 8;             // 16-B chunks per row
  static constexpr int NA = BK * CA / 256, NB = BK * CB / 256;
  static_assert(FM >= 1 && FN >= 1 && NA >= 1 && NB >= 1, "bad wgrad tile");
};

template <int BM, int BN, int WAVES_M>
__global__ void __launch_bounds__(256) k_wgrad(GemmArgs g) {
  using T = WgradTile<BM, BN, WAVES_M>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int ntm = (g.M + BM - 1) / BM, ntn = (g.N + BN - 1) / BN, ntiles = ntm * ntn;
  const int work = xcd_remap(blockIdx.x, ntiles * g.splits);
  const int tile = work % ntiles, ksplit = work / ntiles;
  const int m0 = (tile / ntn) * BM, n0 = (tile % ntn) * BN;
  const int k_begin = ksplit * g.k_per_split, k_end = min(g.K, k_begin + g.k_per_split);
  const int nk = (k_end - k_begin + T::BK - 1) / T::BK;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / T::WAVES_N, wn = wave % T::WAVES_N;
  const unsigned short* A = (const unsigned short*)g.A;
  const unsigned short* B = (const unsigned short*)g.B;

  // per-thread fixed column chunk (256 % C{A,B} == 0): rows t / C + (256 / C) * i
  const int cha = threadIdx.x % T::CA, ra = threadIdx.x / T::CA;
  const int chb = threadIdx.x % T::CB, rb = threadIdx.x / T::CB;
  const int ma = m0 + cha * 8, nb = n0 + chb * 8;
  const bool a_in = ma < g.M, b_in = nb < g.N;
  int ckh = 0, ckw = 0, cc = 0;
  if (g.conv == 2) {
    const int tap = nb / g.cC;
    cc = nb - tap * g.cC;
    ckh = tap / g.cKW;
    ckw = tap - ckh * g.cKW;
  }

  // Loader state per row slot i (rows k = k0 + r + RS i of K-tile k0): for the implicit im2col B the row's pixel
  // decode (img, oh, ow) advanced by 64 pixels with scalar deltas -- no per-tile division (the loader was ~7 VALU
  // per MFMA, PMC, VALU-bound); plain rows keep one multiply (measured: pointer stepping was no faster).
  // Every load is unconditional from a valid address and selected to zero afterwards.
  constexpr int RSA = 256 / T::CA, RSB = 256 / T::CB;
  int bimg[T::NB], boh[T::NB], bow[T::NB];
  const float inv_wo = 1.f / (float)g.cWo, inv_ho = 1.f / (float)g.cHo;
  const int hw = g.cHo * g.cWo, d_img = T::BK / hw, d_rem = T::BK - d_img * hw, d_oh = d_rem / g.cWo,
            d_ow = d_rem - d_oh * g.cWo;
#pragma unroll
  for (int i = 0; i < T::NB; ++i) {
    const int k = min(k_begin + rb + RSB * i, g.K - 1);
    if (g.conv == 2) {
      const int t = fdivmod(k, g.cWo, inv_wo, bow[i]);
      bimg[i] = fdivmod(t, g.cHo, inv_ho, boh[i]);
    } else {
      bimg[i] = boh[i] = bow[i] = 0;
    }
  }
  uint4 sa[T::NA], sb[T::NB];
  auto load = [&](int kt) {
    const int k0 = k_begin + kt * T::BK;
#pragma unroll
    for (int i = 0; i < T::NA; ++i) {
      const int k = k0 + ra + RSA * i;
      const bool ok = a_in && k < k_end;
      const uint4 v = *(const uint4*)(A + (ok ? (size_t)k * g.lda + ma : 0));
      sa[i] = ok ? v : uint4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int i = 0; i < T::NB; ++i) {
      bool ok = b_in && k0 + rb + RSB * i < k_end;
      const unsigned short* src;
      if (g.conv == 2) {
        const int h = boh[i] * g.cS - g.cP + ckh, w = bow[i] * g.cS - g.cP + ckw;
        ok = ok && h >= 0 && h < g.cH && w >= 0 && w < g.cW;
        src = B + ((size_t)(bimg[i] * g.cH + h) * g.cW + w) * g.cC + cc;
        // next tile: 64 pixels on
        bow[i] += d_ow;
        const int c1 = bow[i] >= g.cWo;
        bow[i] -= c1 ? g.cWo : 0;
        boh[i] += d_oh + c1;
        const int c2 = boh[i] >= g.cHo;
        boh[i] -= c2 ? g.cHo : 0;
        bimg[i] += d_img + c2;
      } else {
        src = B + (ok ? (size_t)(k0 + rb + RSB * i) * g.ldb + nb : 0);
      }
      const uint4 v = *(const uint4*)(ok ? src : B);
      sb[i] = ok ? v : uint4{0u, 0u, 0u, 0u};
    }
  };
  auto store = [&](int buf) {
    char* la = smem + buf * T::BUF;
    char* lb = la + T::A_BYTES;
#pragma unroll
    for (int i = 0; i < T::NA; ++i) *(uint4*)(la + (ra + (256 / T::CA) * i) * T::SA + cha * 16) = sa[i];
#pragma unroll
    for (int i = 0; i < T::NB; ++i) *(uint4*)(lb + (rb + (256 / T::CB) * i) * T::SB + chb * 16) = sb[i];
  };

  f32x4 acc[T::FM][T::FN];
#pragma unroll
  for (int i = 0; i < T::FM; ++i)
#pragma unroll
    for (int j = 0; j < T::FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // transposed-read lane address: lane 4q+p of its 16-lane group g -> row 4g + q (+16 for read 1), cols 4p..4p+3
  const int grp = lane >> 4, q = (lane >> 2) & 3, p4 = (lane & 3) * 4;
  const int a_col = (wm * T::FM * 16 + p4) * 2, b_col = (wn * T::FN * 16 + p4) * 2;

  if (nk > 0) {
    load(0);
    store(0);
  }
  __syncthreads();
  const bool single = g.single != 0;  // one LDS buffer: half the LDS, twice the workgroups per CU
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = single ? 0 : (kt & 1);
    if (kt + 1 < nk) load(kt + 1);
    const char* la = smem + buf * T::BUF;
    const char* lb = la + T::A_BYTES;
#pragma unroll
    for (int s = 0; s < T::BK / 32; ++s) {
      const int r0 = s * 32 + 4 * grp + q;  // read 0 row; read 1 is r0 + 16
      s16x8 af[T::FM], bfr[T::FN];
#pragma unroll
      for (int i = 0; i < T::FM; ++i) {
        const char* pa = la + r0 * T::SA + a_col + i * 32;
        const s16x4 lo = lds_tr16(pa), hi = lds_tr16(pa + 16 * T::SA);
        af[i] = s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < T::FN; ++j) {
        const char* pb = lb + r0 * T::SB + b_col + j * 32;
        const s16x4 lo = lds_tr16(pb), hi = lds_tr16(pb + 16 * T::SB);
        bfr[j] = s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int i = 0; i < T::FM; ++i)
#pragma unroll
        for (int j = 0; j < T::FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) {
      if (single) __syncthreads();  // every wave is done reading the buffer it is about to overwrite
      store(single ? 0 : buf ^ 1);
    }
    __syncthreads();
  }

  // slab [split][M][N]: C fragment (row 4 (lane >> 4) + j, col lane & 15)
#pragma unroll
  for (int i = 0; i < T::FM; ++i)
#pragma unroll
    for (int j = 0; j < T::FN; ++j) {
      const int col = n0 + wn * T::FN * 16 + j * 16 + (lane & 15);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = m0 + wm * T::FM * 16 + i * 16 + (lane >> 4) * 4 + e;
        if (row < g.M && col < g.N) g.ws[((size_t)ksplit * g.M + row) * g.N + col] = acc[i][j][e];
      }
    }
}

// ---------------------------------------------------------------------------------------------------------
// k_wgrad_pp: weight gradients on a 256 x PBN tile (PBN = 256 | 128 | 64), 512 threads as two wave groups on the
// k_gemm_pp ping-pong schedule (one group issues its MFMAs while the other reads its fragments and issues LDS-DMA;
// each SIMD holds one wave of each group), operands staged by LDS-DMA instead of a register pass (k_wgrad: 4 waves,
// register-staged, one barrier per K-tile: ~400 TF on ResNet-50's shapes).
//   * The 256-wide side is the larger GEMM dimension: SW = false -> rows = M (output channels, A = dY), columns = N
//     (B = X or its implicit im2col); SW = true (M < 256 <= N, e.g. a 64-channel 3x3 conv, N = 576) -> rows = N
//     (from B), columns = M (from A), and the epilogue writes the transposed fragment (4 consecutive n per lane: one
//     16-B store).
//   * K-tile = 64 pixel rows; an operand row of W channels is 2W bytes in LDS, stored row-linear with 16-B chunk c of
//     row r at chunk position c ^ swz(r) (2 (r & 7) for rows of >= 256 B, 2 ((r >> 1) & 3) for 128-B rows): the DMA
//     image stays wave-linear (1 KiB per wave instruction) because the swizzle is applied to the SOURCE chunk each
//     lane loads.  Fragments by ds_read_b64_tr_b16 with k_wgrad's lane map (lanes 4q + p of 16-lane group g: row
//     4g + q, +16 for the high half, columns 4p ..): the 32 lanes of one LDS cycle read 8 consecutive rows x 32 B,
//     which the swizzle spreads over all 64 banks.
//   * Group r owns rows 128 r ..; waves: PBN = 256 -> 128 x 64 (32 accumulators), 128 -> 2 x 2 of 64 x 64 (16),
//     64 -> 4 x 1 of 32 x 64 (8).  Split-K over pixels into the fp32 slab (k_gemm_splitk_reduce remaps it).
//   * Out-of-range chunks (M / N edges, K tail, conv padding) load through an offset past the descriptor: zeros.
// ---------------------------------------------------------------------------------------------------------
constexpr int WP_BM = 256, WP_NT = 512, WP_KT = 64;
template <int PBN>
struct WpTile {
  static constexpr int WMG = PBN == 256 ? 1 : (PBN == 128 ? 2 : 4), WNG = 4 / WMG, MF = 8 / WMG;
  static constexpr int R_RB = WP_BM * 2, C_RB = PBN * 2;            // LDS row bytes: row side | column side
  static constexpr int R_CPR = R_RB / 16, C_CPR = C_RB / 16;        // 16-B chunks per row
  static constexpr int R_RPI = 1024 / R_RB, C_RPI = 1024 / C_RB;    // rows per wave DMA instruction
  static constexpr int R_BYTES = WP_KT * R_RB, C_BYTES = WP_KT * C_RB, BUF = R_BYTES + C_BYTES, LDS = 2 * BUF;
  static constexpr int NIR = R_BYTES / 16 / WP_NT, NIC = C_BYTES / 16 / WP_NT;  // DMA per thread and K-tile
  static_assert(NIR * WP_NT * 16 == R_BYTES && NIC * WP_NT * 16 == C_BYTES, "wgrad pp staging");
};
template <int RB>
__device__ __forceinline__ int wp_swz(int r) { return RB >= 256 ? 2 * (r & 7) : 2 * ((r >> 1) & 3); }
template <int RB>
__device__ __forceinline__ int wp_off(int r, int colbyte) {
  return r * RB + ((((colbyte >> 4) ^ wp_swz<RB>(r)) << 4) | (colbyte & 15));
}

// One operand side of k_wgrad_pp: NI DMA slots per thread and K-tile (fixed tile row and logical chunk each), plain
// pixel-major rows (offset stepped by 64 rows per tile) or the implicit im2col of an NHWC input (pixel decode
// stepped by 64 pixels per tile: k_wgrad's incremental decode, no division in the loop).
template <int NI, int RB, int RPI>
struct WpSide {
  unsigned off[NI];
  int row[NI], img[NI], oh[NI], ow[NI], kh[NI], kw[NI], cc[NI];
  __device__ __forceinline__ void init(const GemmArgs& g, bool implicit, int e0, int extent, int ld, int k_begin,
                                       int wave, int lane) {
    constexpr int CPR = RB / 16;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int r = (wave * NI + i) * RPI + lane / CPR, c = (lane % CPR) ^ wp_swz<RB>(r);
      const int e = e0 + 8 * c;  // first channel (GEMM index) of this lane's chunk
      row[i] = r;
      img[i] = oh[i] = ow[i] = kh[i] = kw[i] = cc[i] = 0;
      if (implicit) {
        const int ee = e < extent ? e : 0, tap = ee / g.cC;
        cc[i] = e < extent ? ee - tap * g.cC : -1;  // -1: past the extent (never valid)
        kh[i] = tap / g.cKW;
        kw[i] = tap - kh[i] * g.cKW;
        const float inv_wo = 1.f / (float)g.cWo, inv_ho = 1.f / (float)g.cHo;
        const int t = fdivmod(min(k_begin + r, g.K - 1), g.cWo, inv_wo, ow[i]);
        img[i] = fdivmod(t, g.cHo, inv_ho, oh[i]);
        off[i] = 0u;
      } else {
        off[i] = e < extent ? (unsigned)((long long)(k_begin + r) * ld * 2 + e * 2) : 0x80000000u;
      }
    }
  }
  __device__ __forceinline__ void issue(const GemmArgs& g, bool implicit, __amdgpu_buffer_rsrc_t rs, char* lds,
                                        int kt, int k0, int k_end, int ld, int wave, int d_img, int d_oh, int d_ow) {
    constexpr unsigned OOB = 0x80000000u;
    if (implicit) {
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int h = oh[i] * g.cS - g.cP + kh[i], w = ow[i] * g.cS - g.cP + kw[i];
        const bool ok = cc[i] >= 0 && k0 + row[i] < k_end && h >= 0 && h < g.cH && w >= 0 && w < g.cW;
        blds16(rs, lds + (wave * NI + i) * 1024, ok ? (unsigned)((((img[i] * g.cH + h) * g.cW + w) * g.cC + cc[i]) * 2) : OOB,
               0u);
        ow[i] += d_ow;
        const int c1 = ow[i] >= g.cWo;
        ow[i] -= c1 ? g.cWo : 0;
        oh[i] += d_oh + c1;
        const int c2 = oh[i] >= g.cHo;
        oh[i] -= c2 ? g.cHo : 0;
        img[i] += d_img + c2;
      }
    } else {
      const unsigned so = (unsigned)((long long)kt * WP_KT * ld * 2);
#pragma unroll
      for (int i = 0; i < NI; ++i) blds16(rs, lds + (wave * NI + i) * 1024, k0 + row[i] < k_end ? off[i] : OOB, so);
    }
  }
};

template <int PBN, bool SW>
__global__ void __launch_bounds__(WP_NT) k_wgrad_pp(GemmArgs g) {
  using T = WpTile<PBN>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int RX = SW ? g.N : g.M, CX = SW ? g.M : g.N;  // extents of the row side / column side
  const int ntm = (RX + WP_BM - 1) / WP_BM, ntn = (CX + PBN - 1) / PBN, ntiles = ntm * ntn;
  const int work = xcd_remap(blockIdx.x, ntiles * g.splits);
  const int tile = work % ntiles, ksplit = work / ntiles;
  const int r0t = (tile / ntn) * WP_BM, c0t = (tile % ntn) * PBN;
  const int k_begin = ksplit * g.k_per_split, k_end = min(g.K, k_begin + g.k_per_split);
  const int nk = (k_end - k_begin + WP_KT - 1) / WP_KT;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), wr = wave >> 2;
  const int wi = (wave & 3) / T::WNG, wj = (wave & 3) % T::WNG;
  const int wrow = wr * 128 + wi * (128 / T::WMG), wcol = wj * 64;  // this wave's sub-tile in the 256 x PBN tile
  const bool conv = g.conv == 2;  // B (the row side when SW) is the implicit im2col of an NHWC input
  const long long a_bytes = (long long)g.K * g.lda * 2;
  const long long b_bytes = conv ? (long long)g.cN * g.cH * g.cW * g.cC * 2 : (long long)g.K * g.ldb * 2;
  const __amdgpu_buffer_rsrc_t ars = __builtin_amdgcn_make_buffer_rsrc((void*)g.A, (short)0, (int)a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc((void*)g.B, (short)0, (int)b_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rrs = SW ? brs : ars, crs = SW ? ars : brs;
  const int rld = SW ? g.ldb : g.lda, cld = SW ? g.lda : g.ldb;
  const bool r_imp = SW && conv, c_imp = !SW && conv;
  int d_img = 0, d_oh = 0, d_ow = 0;
  if (conv) {
    const int hw = g.cHo * g.cWo, rem = WP_KT % hw;
    d_img = WP_KT / hw;
    d_oh = rem / g.cWo;
    d_ow = rem - d_oh * g.cWo;
  }
  WpSide<T::NIR, T::R_RB, T::R_RPI> rside;
  WpSide<T::NIC, T::C_RB, T::C_RPI> cside;
  rside.init(g, r_imp, r0t, RX, rld, k_begin, wave, lane);
  cside.init(g, c_imp, c0t, CX, cld, k_begin, wave, lane);
  // this thread's LDS-DMA of K-tile kt into buffer kt & 1 (every thread issues its tiles in increasing order)
  auto issue = [&](int kt) {
    const int k0 = k_begin + kt * WP_KT;
    char* lr = smem + (kt & 1) * T::BUF;
    rside.issue(g, r_imp, rrs, lr, kt, k0, k_end, rld, wave, d_img, d_oh, d_ow);
    cside.issue(g, c_imp, crs, lr + T::R_BYTES, kt, k0, k_end, cld, wave, d_img, d_oh, d_ow);
  };
  auto bar = [] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  constexpr int MF = T::MF;
  f32x4 acc[MF][4];
#pragma unroll
  for (int m = 0; m < MF; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  s16x8 af[MF], bfr[4];
  const int grp = lane >> 4, q = (lane >> 2) & 3, p4 = (lane & 3) * 4;
  auto load_frags = [&](int kt, int h) {
    const char* lr = smem + (kt & 1) * T::BUF;
    const char* lc = lr + T::R_BYTES;
    const int r0 = h * 32 + 4 * grp + q;  // high half: r0 + 16 (same swizzle)
#pragma unroll
    for (int m = 0; m < MF; ++m) {
      const char* pa = lr + wp_off<T::R_RB>(r0, (wrow + m * 16 + p4) * 2);
      const s16x4 lo = lds_tr16(pa), hi = lds_tr16(pa + 16 * T::R_RB);
      af[m] = s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const char* pb = lc + wp_off<T::C_RB>(r0, (wcol + n * 16 + p4) * 2);
      const s16x4 lo = lds_tr16(pb), hi = lds_tr16(pb + 16 * T::C_RB);
      bfr[n] = s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
  };
  auto mfmas = [&] {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int m = 0; m < MF; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m], bfr[n], acc[m][n], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // the k_gemm_pp schedule (its comment block has the interval bookkeeping)
  if (nk > 0) issue(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  bar();
  if (wr == 0) {
#pragma unroll 1
    for (int st = 0; st < 2 * nk; ++st) {
      const int kt = st >> 1, h = st & 1;
      if (h == 0 && kt + 1 < nk) issue(kt + 1);
      load_frags(kt, h);
      bar();
      mfmas();
      if (h == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      bar();
    }
    bar();
  } else {
    if (nk > 1) issue(1);
    bar();
#pragma unroll 1
    for (int st = 0; st < 2 * nk; ++st) {
      const int kt = st >> 1, h = st & 1;
      load_frags(kt, h);
      if (h == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      bar();
      if (h == 1 && kt + 2 < nk) issue(kt + 2);
      mfmas();
      bar();
    }
  }

  // slab [split][M][N] straight from the accumulators: fragment (row-side 4 (lane >> 4) + e, column-side lane & 15)
#pragma unroll
  for (int m = 0; m < MF; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int cidx = c0t + wcol + n * 16 + (lane & 15), ridx = r0t + wrow + m * 16 + (lane >> 4) * 4;
      if constexpr (SW) {  // (m = cidx, n = ridx .. ridx + 3): one 16-B store (N % 8 == 0)
        if (cidx < g.M && ridx < g.N) *(f32x4*)(g.ws + ((size_t)ksplit * g.M + cidx) * g.N + ridx) = acc[m][n];
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (ridx + e < g.M && cidx < g.N) g.ws[((size_t)ksplit * g.M + ridx + e) * g.N + cidx] = acc[m][n][e];
      }
    }
}

// ---------------------------------------------------------------------------------------------------------
// k_wgrad3x3_rows: weight gradient of the 64-channel 3 x 3 / pad 1 / stride 1 convolutions on rows of at most 64
// pixels (ResNet-50's layer 1), dW[co][tap * 64 + c] = sum_p dY[p][co] X[p + tap][c], in the row form of
// k_conv3x3_rows (ops_gemm.hip): a workgroup walks consecutive output rows (n, oh) with the three input rows in an
// LDS ring (4 slots of 66 pixels x 128 B, pixel iw at position iw + 1) and the dY row in a double buffer, each row
// fetched once per workgroup with coalesced 16-B loads one row ahead.  k_wgrad re-gathers the implicit im2col per
// K-tile (13 VALU per MFMA, MFMA busy 0.19: profiles/conv3x3_rows_r9.txt).
//   * wave w owns input channels 16 w .. + 15 of all 9 taps and all 64 output channels: 9 x 4 accumulator tiles
//     (144 registers) for the workgroup's whole row range;
//   * per 32-pixel chunk: the 4 dY fragments (16 co x 32 pixels) and per valid tap one X fragment (32 pixels x 16
//     channels, shifted by kw) are read with ds_read_b64_tr_b16 (two per fragment: pixels 8 q .. + 3 and + 4 .. + 7
//     of lane group q), i.e. 26 transposed reads for 36 MFMAs; the 16-B chunks of a pixel row are XOR-swizzled by
//     wr_sw(pixel) so the 8 pixel rows x 32 B of a 32-lane half hit 64 distinct banks for every shift;
//   * padding rows are skipped per row; pixels past W are zero in the dY image;
//   * the workgroup's partial 64 x 576 sums go to split slab vid of the fp32 workspace (k_gemm_splitk_reduce sums
//     them in a fixed order: deterministic).
// Requirements (launcher): bf16, C = Cout = 64 (W <= 64) or 128 (W <= 32), grid <= the slab's splits (x 2 for 128).
// ---------------------------------------------------------------------------------------------------------
__device__ __forceinline__ int wr_off(int px, int chunk) {
  return px * 128 + ((chunk ^ ((((px >> 1) & 3) << 1) ^ (((px >> 3) & 1) << 2))) << 4);
}
// X pixel rows of C channels: C = 64 as wr_off; C = 128 (256-B rows, one bank window per pixel): chunk XOR 2 f(px)
// with f = (px & 3) | ((px >> 3) & 1) << 2, injective on the 8 pixels {b .. b + 3, b + 8 .. b + 11} of a 32-lane half
template <int C>
__device__ __forceinline__ int wx_off(int px, int chunk) {
  if constexpr (C == 64) return wr_off(px, chunk);
  else return px * 256 + ((chunk ^ (((px & 3) | (((px >> 3) & 1) << 2)) << 1)) << 4);
}
// C = 64: 4 waves, rows <= 64 pixels; C = 128 (layer 2, 28 x 28): 8 waves (input channels 16 w .. + 15 each), rows
// <= 32 pixels, and the 128 output channels split over two workgroups (half = blockIdx.x % 2: 64 each, 144
// accumulators per lane), one workgroup per CU
template <int C>
struct WgradRows {
  static constexpr int NT = 4 * C, HALVES = C / 64, SPX = C == 64 ? 66 : 34, XCH = C / 8;
  static constexpr int SLOT = SPX * 2 * C, DY = (SPX - 2) * 128, LDS = 4 * SLOT + 2 * DY;
  static constexpr int NLX = ((SPX - 2) * XCH + NT - 1) / NT, NLD = ((SPX - 2) * 8 + NT - 1) / NT;
};
constexpr int WR_LDS = WgradRows<64>::LDS;
template <int NPC, int C = 64>  // NPC: 32-pixel chunks per row, ceil(W / 32)
__global__ void __launch_bounds__(4 * C, C == 64 ? 2 : 1) k_wgrad3x3_rows(GemmArgs g) {
  using T = WgradRows<C>;
  constexpr int NT = T::NT, NLX = T::NLX, NLD = T::NLD;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  typedef unsigned v4u_ __attribute__((ext_vector_type(4)));
  constexpr unsigned OOB = 0x80000000u;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), j = lane & 15, q = lane >> 4;
  const int ra = j >> 2, rp = j & 3;  // transposed read: lane 4 ra + rp of its group addresses block row ra, cols 4 rp..
  const int H = g.cH, W = g.cW, R = g.cN * g.cH;
  const int half = (int)blockIdx.x % T::HALVES, bid = (int)blockIdx.x / T::HALVES, grid = gridDim.x / T::HALVES;
  const int vid = (grid & 7) == 0 ? (bid & 7) * (grid >> 3) + (bid >> 3) : bid;
  const int r_beg = (int)((long long)vid * R / grid), r_end = (int)((long long)(vid + 1) * R / grid);
  char* dyb = smem + 4 * T::SLOT;
  for (int e = threadIdx.x; e < T::LDS / 16; e += NT) *(v4u_*)(smem + e * 16) = v4u_{0u, 0u, 0u, 0u};
  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)g.B, (short)0, (int)((long long)R * W * 2 * C), 0x00020000);
  const __amdgpu_buffer_rsrc_t drs =
      __builtin_amdgcn_make_buffer_rsrc((void*)g.A, (short)0, (int)((long long)R * W * g.lda * 2), 0x00020000);
  auto x_load = [&](v4u_(&st)[NLX], int gr) {
#pragma unroll
    for (int i = 0; i < NLX; ++i) {
      const int e = threadIdx.x + NT * i;
      const unsigned o =
          (gr >= 0 && gr < R && e < W * T::XCH) ? (unsigned)gr * (unsigned)W * (2u * C) + (unsigned)e * 16u : OOB;
      st[i] = __builtin_amdgcn_raw_buffer_load_b128(xrs, o, 0, 0);
    }
  };
  auto x_store = [&](const v4u_(&st)[NLX], int gr) {
    if (gr < 0 || gr >= R) return;
    char* sl = smem + (gr & 3) * T::SLOT;
#pragma unroll
    for (int i = 0; i < NLX; ++i) {
      const int e = threadIdx.x + NT * i;
      if (e < W * T::XCH) *(v4u_*)(sl + wx_off<C>(e / T::XCH + 1, e % T::XCH)) = st[i];
    }
  };
  auto d_load = [&](v4u_(&st)[NLD], int r) {  // this workgroup's 64 output channels of dY row r
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int e = threadIdx.x + NT * i;
      const unsigned o = (r < R && e < W * 8) ? ((unsigned)(r * W + (e >> 3)) * (unsigned)g.lda + 64u * half +
                                                 8u * (unsigned)(e & 7)) * 2u
                                              : OOB;
      st[i] = __builtin_amdgcn_raw_buffer_load_b128(drs, o, 0, 0);
    }
  };
  auto d_store = [&](const v4u_(&st)[NLD], int r) {
    char* db = dyb + (r & 1) * T::DY;
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int e = threadIdx.x + NT * i;
      if (e < W * 8) *(v4u_*)(db + wr_off(e >> 3, e & 7)) = st[i];
    }
  };
  // one 16 x 32 operand: pixels px .. px + 7 (as 8 q + 0..3, + 4..7) of the 16 channels from byte column 32 cb
  auto frag_d = [&](const char* base, int px, int cb) {
    const int ch = 2 * cb + (rp >> 1), within = 8 * (rp & 1);
    const s16x4 lo = lds_tr16(base + wr_off(px + ra, ch) + within);
    const s16x4 hi = lds_tr16(base + wr_off(px + 4 + ra, ch) + within);
    return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  };
  auto frag_x = [&](const char* base, int px, int cb) {
    const int ch = 2 * cb + (rp >> 1), within = 8 * (rp & 1);
    const s16x4 lo = lds_tr16(base + wx_off<C>(px + ra, ch) + within);
    const s16x4 hi = lds_tr16(base + wx_off<C>(px + 4 + ra, ch) + within);
    return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  };
  f32x4 acc[9][4];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int m = 0; m < 4; ++m) acc[t][m] = f32x4{0.f, 0.f, 0.f, 0.f};
  v4u_ xs[NLX], ds[NLD];
  __syncthreads();  // zeroed before any row lands
  for (int d = -1; d <= 1; ++d) {
    x_load(xs, r_beg + d);
    x_store(xs, r_beg + d);
  }
  d_load(ds, r_beg);
  d_store(ds, r_beg);
  __syncthreads();
  for (int r = r_beg; r < r_end; ++r) {
    const int oh = r % H;
    const bool pre = r + 1 < r_end;
    if (pre) {
      x_load(xs, r + 2);
      d_load(ds, r + 1);
    }
    const char* db = dyb + (r & 1) * T::DY;
#pragma unroll
    for (int pc = 0; pc < NPC; ++pc) {
      const int px0 = 32 * pc + 8 * q;
      s16x8 a[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) a[m] = frag_d(db, px0, m);
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        if (oh - 1 + kh < 0 || oh - 1 + kh >= H) continue;
        const char* sl = smem + ((r - 1 + kh) & 3) * T::SLOT;
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const s16x8 b = frag_x(sl, px0 + kw, w);
#pragma unroll
          for (int m = 0; m < 4; ++m)
            acc[kh * 3 + kw][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[m], b, acc[kh * 3 + kw][m], 0, 0, 0);
        }
      }
    }
    if (pre) {
      x_store(xs, r + 2);  // slot of row r - 2, last read by the previous output row
      d_store(ds, r + 1);  // the other dY buffer, last read by the previous output row
    }
    __syncthreads();
  }
  // lane (q, j) of tile (t, m): output channel 64 half + 16 m + 4 q + e, input channel 16 w + j of tap t
  float* wsp = g.ws + (size_t)vid * C * 9 * C;
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int e = 0; e < 4; ++e) wsp[(64 * half + 16 * m + 4 * q + e) * (9 * C) + t * C + 16 * w + j] = acc[t][m][e];
}

// ---------------------------------------------------------------------------------------------------------
// k_wgrad_s2d_rows: weight gradient of the space-to-depth stem conv (4 x 4 taps over 16 channels, no padding, 64
// outputs; ops/functional.py stem_s2d_index), dW[co][tap * 16 + c] = sum_p dY[p][co] X[p + tap][c], in the row form
// of k_conv_s2d_rows (ops_gemm.hip; k_wgrad<64, 128, 1> ran it at 226 us at batch 256):
//   * input rows in 5 LDS slots of 128 pixels x 32 B (the first row of a workgroup or an image loads all four, later
//     ones one row ahead), the dY row in a double buffer of 128 pixels x 128 B;
//   * wave w owns kernel row kh = w: 4 taps x 4 output-channel tiles (64 accumulators), reading only input row
//     oh + w; a tap's X fragment (32 pixels x the 16 channels) and the 4 dY fragments come from ds_read_b64_tr_b16,
//     two per fragment, with the K order of k_wgrad (element e < 4 of lane group q = pixel 4 q + e, e >= 4 = pixel
//     16 + 4 q + e - 4), so a 32-lane half reads 8 consecutive pixels: 256 contiguous bytes of an X slot, and 8 dY
//     rows whose 16-B chunks are XOR-swizzled by ((pixel >> 1) & 3) << 1 (conflict-free);
//   * pixels past Wo are zero in the dY image; partial sums to split slab vid (k_gemm_splitk_reduce).
// Requirements (launcher): C = 16, KH = KW = 4, pad 0, stride 1, Cout = 64, Wi <= 128, grid <= the slab's splits.
// ---------------------------------------------------------------------------------------------------------
__device__ __forceinline__ int ws2_off(int px, int chunk) { return px * 128 + ((chunk ^ (((px >> 1) & 3) << 1)) << 4); }
constexpr int WS_SLOT = 128 * 32, WS_DY = 128 * 128, WS_LDS = 5 * WS_SLOT + 2 * WS_DY;
template <int NPC>  // 32-pixel chunks per output row: ceil(Wo / 32)
__global__ void __launch_bounds__(CR_NT, 3) k_wgrad_s2d_rows(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  typedef unsigned v4u_ __attribute__((ext_vector_type(4)));
  constexpr unsigned OOB = 0x80000000u;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), j = lane & 15, q = lane >> 4;
  const int ra = j >> 2, rp = j & 3;
  const int Hi = g.cH, Wi = g.cW, Ho = g.cHo, Wo = g.cWo, R = g.cN * Ho, RI = g.cN * Hi;
  const int grid = gridDim.x;
  const int vid = (grid & 7) == 0 ? (int)(blockIdx.x & 7) * (grid >> 3) + (int)(blockIdx.x >> 3) : (int)blockIdx.x;
  const int r_beg = (int)((long long)vid * R / grid), r_end = (int)((long long)(vid + 1) * R / grid);
  char* dyb = smem + 5 * WS_SLOT;
  for (int e = threadIdx.x; e < WS_LDS / 16; e += CR_NT) *(v4u_*)(smem + e * 16) = v4u_{0u, 0u, 0u, 0u};
  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)g.B, (short)0, (int)((long long)RI * Wi * 32), 0x00020000);
  const __amdgpu_buffer_rsrc_t drs =
      __builtin_amdgcn_make_buffer_rsrc((void*)g.A, (short)0, (int)((long long)R * Wo * g.lda * 2), 0x00020000);
  auto x_load = [&](int gi) {  // input row gi: Wi * 2 pieces of 16 B, one per thread
    const unsigned o =
        (gi < RI && (int)threadIdx.x < Wi * 2) ? ((unsigned)gi * (unsigned)Wi * 32u + threadIdx.x * 16u) : OOB;
    return __builtin_amdgcn_raw_buffer_load_b128(xrs, o, 0, 0);
  };
  auto x_store = [&](const v4u_& v, int gi) {
    if (gi < RI && (int)threadIdx.x < Wi * 2) *(v4u_*)(smem + (gi % 5) * WS_SLOT + threadIdx.x * 16) = v;
  };
  auto d_load = [&](v4u_(&st)[4], int r) {  // dY row r: Wo * 8 pieces, up to 4 per thread
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = threadIdx.x + CR_NT * i;
      const unsigned o = (r < R && e < Wo * 8)
                             ? ((unsigned)(r * Wo + (e >> 3)) * (unsigned)g.lda + 8u * (unsigned)(e & 7)) * 2u : OOB;
      st[i] = __builtin_amdgcn_raw_buffer_load_b128(drs, o, 0, 0);
    }
  };
  auto d_store = [&](const v4u_(&st)[4], int r) {
    char* db = dyb + (r & 1) * WS_DY;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = threadIdx.x + CR_NT * i;
      if (e < Wo * 8) *(v4u_*)(db + ws2_off(e >> 3, e & 7)) = st[i];
    }
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int m = 0; m < 4; ++m) acc[t][m] = f32x4{0.f, 0.f, 0.f, 0.f};
  v4u_ ds[4], xn;
  __syncthreads();  // zeroed before any row lands
  d_load(ds, r_beg);
  d_store(ds, r_beg);
  for (int r = r_beg; r < r_end; ++r) {
    const int n = r / Ho, oh = r - n * Ho, gi0 = n * Hi + oh;
    if (r == r_beg || oh == 0) {  // a workgroup's or an image's first row: all four input rows
      v4u_ v[4];
#pragma unroll
      for (int d = 0; d < 4; ++d) v[d] = x_load(gi0 + d);
#pragma unroll
      for (int d = 0; d < 4; ++d) x_store(v[d], gi0 + d);
      __syncthreads();
    }
    const bool pre = r + 1 < r_end, prex = pre && oh + 1 < Ho;
    if (pre) d_load(ds, r + 1);
    if (prex) xn = x_load(gi0 + 4);
    const char* db = dyb + (r & 1) * WS_DY;
    const char* sl = smem + ((gi0 + w) % 5) * WS_SLOT;  // this wave's kernel row
#pragma unroll 1
    for (int pc = 0; pc < NPC; ++pc) {
      const int p0 = 32 * pc + 4 * q + ra;
      s16x8 a[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int ch = 2 * m + (rp >> 1), within = 8 * (rp & 1);
        const s16x4 lo = lds_tr16(db + ws2_off(p0, ch) + within), hi = lds_tr16(db + ws2_off(p0 + 16, ch) + within);
        a[m] = s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int kw = 0; kw < 4; ++kw) {
        const s16x4 lo = lds_tr16(sl + (p0 + kw) * 32 + 8 * rp), hi = lds_tr16(sl + (p0 + 16 + kw) * 32 + 8 * rp);
        const s16x8 b = s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int m = 0; m < 4; ++m) acc[kw][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[m], b, acc[kw][m], 0, 0, 0);
      }
    }
    if (prex) x_store(xn, gi0 + 4);  // slot of row gi0 - 1, last read by the previous output row
    if (pre) d_store(ds, r + 1);     // the other dY buffer, last read by the previous output row
    __syncthreads();
  }
  // lane (q, j) of tile (kw, m): output channel 16 m + 4 q + e, column (4 w + kw) * 16 + j
  float* wsp = g.ws + (size_t)vid * 64 * 256;
#pragma unroll
  for (int kw = 0; kw < 4; ++kw)
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int e = 0; e < 4; ++e) wsp[(16 * m + 4 * q + e) * 256 + (4 * w + kw) * 16 + j] = acc[kw][m][e];
}

}  // namespace ops
}  // namespace dca
