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
  static constexpr int BK = 64;
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
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
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
    for (int s = 0; s < 2; ++s) {
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

}  // namespace ops
}  // namespace dca
