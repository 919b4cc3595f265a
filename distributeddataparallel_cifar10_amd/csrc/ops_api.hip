// C ABI of the ops layer (libdca_ops.so), driven from ops/_native.py with torch-allocated tensors and the
// caller's HIP stream.  Every entry point validates what the kernels assume about shapes before launching
// (a bad shape is an error string, never an out-of-bounds access on the GPU).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <tuple>
#include <cstring>
#include <string>
#include <cstdlib>
#include <cstdint>

#include "ops_nn.hip"
#include "ops_wgrad.hip"

namespace {
thread_local std::string g_err;
#define OPCK(x)                                              \
  do {                                                       \
    hipError_t e_ = (x);                                     \
    if (e_ != hipSuccess) {                                  \
      g_err = std::string(#x) + ": " + hipGetErrorString(e_); \
      return -1;                                             \
    }                                                        \
  } while (0)
#define REQUIRE(c, msg)  \
  do {                   \
    if (!(c)) {          \
      g_err = msg;       \
      return -1;         \
    }                    \
  } while (0)

inline int grid_for(long work, int per_block = 256, int cap = 8192) {
  long b = (work + per_block - 1) / per_block;
  return (int)std::max(1L, std::min(b, (long)cap));
}
bool g_lds_set = false;
// Dispatch policy.  Every rule below was chosen by measurement (docs/ARCHITECTURE.md "GEMM dispatch"); the A/B
// environment switches of rounds 1-4 are gone (round 5), except DCA_OPS_STREAM, kept as the diagnostic A/B of the
// persistent short-K kernel that is still being tuned (0 never, 1 every eligible shape, unset: the shape rule).
// 3x3/2 max-pool specialisations: unrolled forward, output-driven backward (324 -> 107 us backward at batch 256)
constexpr bool POOL_K3S2 = true;
// bf16 implicit-conv glds (C % 64 == 0): neutral at batch 64, +2..6 % per conv GEMM at batch 256
constexpr bool GLDS_CONV = true;
// single-buffer weight-gradient kernel: the loop is latency-bound, so more resident workgroups per CU win
// (batch-256 census: M = 64 weight gradients 845 -> 580 us, 835 -> 556 us)
constexpr bool WGRAD_SINGLE = true;
// glds single-buffer mode (32 KiB LDS: ~1.5x the resident workgroups) for short K: K-tiles per split <= 9.
// Batch-256 census vs double-buffered: K <= 576 0.78-0.91x time, K = 1152 0.93x, K = 1024-4608 0.97-1.23x.
constexpr int GLDS_SINGLE_NK = 9;
// narrow (128 x 64) short-K GEMMs on the single-buffer glds kernel: 0.89-0.90x the register-staged time at
// batch 256 (802816 x 64 x {64, 256})
constexpr bool GLDS_NARROW = true;
// register-staged kernel: single LDS buffer up to this many K-tiles per split
constexpr int REG_SINGLE_NK = 4;
// glds K pipeline: 2 LDS buffers (3-4 measured 1.4-1.6x slower on the long-K shapes: fewer resident waves)
constexpr int GLDS_STAGES = 2;
inline int getenv_pp4() {  // A/B knob: DCA_OPS_PP4=0 keeps the two-buffer k_gemm_pp (and its K >= 1024 rule)
  static const int v = [] {
    const char* e = getenv("DCA_OPS_PP4");
    return e ? atoi(e) : 1;
  }();
  return v;
}
inline int getenv_conv_rows() {  // A/B knob: DCA_OPS_CONV_ROWS=0 keeps the layer-1 3x3 convs and the stem on
                                 // k_direct_conv
  static const int v = [] {
    const char* e = getenv("DCA_OPS_CONV_ROWS");
    return e ? atoi(e) : 1;
  }();
  return v;
}
inline int getenv_wgrad_rows() {  // A/B knob: DCA_OPS_WGRAD_ROWS=0 keeps the 64-channel 3x3 weight gradient on k_wgrad
  static const int v = [] {
    const char* e = getenv("DCA_OPS_WGRAD_ROWS");
    return e ? atoi(e) : 1;
  }();
  return v;
}
inline int getenv_stream() {  // persistent short-K GEMM (k_gemm_stream): DCA_OPS_STREAM = 0 never, 1 whenever
  static const int v = [] {    // eligible, 2 (default) by the shape rule at the launch site
    const char* e = getenv("DCA_OPS_STREAM");
    return e ? atoi(e) : 2;
  }();
  return v;
}
// implicit 3x3 convolutions (N = 128) on k_gemm_stream (129.5 -> 117.5 us at batch 256), and the strided 1x1
// (downsample) ones with N % 128 == 0 and M >= 16384 (256x56x56x256 -> 512: 177 -> 126 us, 256x28x28x512 -> 1024:
// 116 -> 101 us; 256x14x14x1024 -> 2048, M = 12544, stays on pp4: 82 vs 95 us; profiles/stream_downsample_ab_r8f.log)
constexpr bool STREAM_CONV = true;
// weight gradients with M >= 256 (and the swapped 1x1 forms) on the ping-pong LDS-DMA kernel k_wgrad_pp
// (0.71-0.92x the k_wgrad time on every routed shape); the 64-wide / swapped implicit forms stay on k_wgrad
// (1.4-1.7x slower on k_wgrad_pp, profiles/wgrad_pp_r3.log)
inline int nparts_rows(long M) { return (int)((M + dca::ops::BN_ROWS - 1) / dca::ops::BN_ROWS); }
// BN kernels: 16 channel lanes (256 contiguous bytes per row and wave instruction) when C % 128 == 0, else 8
// finalize threads per workgroup: 1024 when one workgroup reduces one channel's partial rows (C < 256)
#define BN_FIN_NTH(CW) ((CW) == 1 ? 1024 : 256)

// Per-shape policy of the large BN passes (bench/micro/bn_micro.hip, profiles/bn_micro_r4s.log; same box, ResNet-50
// batch-256 shapes): tensors of >= 2^26 elements stream with non-temporal loads / stores (statistics 181.6 -> 145.5 us,
// residual apply 251.6 -> 209.5 us at 802816 x 256); the 16-lane backward apply of >= 2^25 elements also takes 128
// rows per workgroup (twice the workgroups: 104.5 -> 84.2 us at 50176 x 1024).  Smaller tensors keep the default
// cache policy and 256 rows (they are re-read while still in the Infinity Cache).  Same box, whole step: 10,292 ->
// 10,494 img/s (profiles/resnet50_bntune_ab_r4t.log).
using namespace dca::ops;
inline bool bn_nt(long M, int C) { return C % 128 == 0 && (long)M * C >= (1L << 26); }
inline bool bn_bwd_apply_fine(long M, int C) { return C % 128 == 0 && (long)M * C >= (1L << 25); }
inline int bn_bwd_mode(int relu, int res_mode, const void* mask) {
  if (mask) return BWD_MASK;
  if (relu) return res_mode == 2 ? BWD_RES : BWD_RELU;
  return BWD_PLAIN;
}
template <int CL, typename... A>
void bn_stats_launch(int mode, bool nt, dim3 g, hipStream_t st, A... a) {
#define BST(MO)                                                                                  \
  if (nt) hipLaunchKernelGGL((k_bn_bwd_stats<CL, MO, true>), g, dim3(256), 0, st, a...);         \
  else hipLaunchKernelGGL((k_bn_bwd_stats<CL, MO, false>), g, dim3(256), 0, st, a...)
  switch (mode) {
    case BWD_PLAIN: BST(BWD_PLAIN); break;
    case BWD_RELU: BST(BWD_RELU); break;
    case BWD_RES: BST(BWD_RES); break;
    default: BST(BWD_MASK); break;
  }
#undef BST
}
template <int CL, typename... A>
void bn_bwd_apply_launch(int mode, bool fine, long M, int C, hipStream_t st, A... a) {
  const unsigned gx = (unsigned)((C + 8 * CL - 1) / (8 * CL));
  const dim3 g128(gx, (unsigned)((M + 127) / 128)), g256(gx, (unsigned)((M + 255) / 256));
#define BAP(MO)                                                                                          \
  if (fine) hipLaunchKernelGGL((k_bn_bwd_apply<CL, MO, 128, true>), g128, dim3(256), 0, st, a...);      \
  else hipLaunchKernelGGL((k_bn_bwd_apply<CL, MO, 256, false>), g256, dim3(256), 0, st, a...)
  switch (mode) {
    case BWD_PLAIN: BAP(BWD_PLAIN); break;
    case BWD_RELU: BAP(BWD_RELU); break;
    case BWD_RES: BAP(BWD_RES); break;
    default: BAP(BWD_MASK); break;
  }
#undef BAP
}
template <bool RAFF, typename... A>
void bn_apply_launch_t(long M, int C, hipStream_t st, A... a) {
  if (C % 128 != 0) {
    hipLaunchKernelGGL((k_bn_apply<8, BN_ROWS, false, RAFF>), dim3((C + 63) / 64, nparts_rows(M)), dim3(256), 0, st, a...);
  } else if (bn_nt(M, C)) {
    hipLaunchKernelGGL((k_bn_apply<16, 128, true, RAFF>), dim3(C / 128, (unsigned)((M + 127) / 128)), dim3(256), 0, st,
                       a...);
  } else {
    hipLaunchKernelGGL((k_bn_apply<16, BN_ROWS, false, RAFF>), dim3(C / 128, nparts_rows(M)), dim3(256), 0, st, a...);
  }
}
// (the residual's on-the-fly BN -- the last argument, BnRes -- selects its own instantiation)
template <typename... A>
void bn_apply_launch(long M, int C, hipStream_t st, A... a) {
  const BnRes rb = std::get<sizeof...(A) - 1>(std::tuple<A...>(a...));
  if (rb.stats) bn_apply_launch_t<true>(M, C, st, a...);
  else bn_apply_launch_t<false>(M, C, st, a...);
}
// BN partial-row reduction (MODE 0 forward statistics, MODE 1 backward sums): with ticket words (ceil(C / 64), zero)
// the coalesced ticketed kernel (k_bn_fin_ticket; the partial rows are overwritten), else the per-channel one
template <int MODE>
void bn_fin_launch(float* part, int nparts, long M, int C, float* a0, float* a1, float* out, float eps, float momentum,
                   int accumulate, unsigned* ticket, hipStream_t st) {
  if (ticket) {
    const int rpb = bn_fin_rpb(nparts);
    const dim3 grid((unsigned)((C + 63) / 64), (unsigned)((nparts + rpb - 1) / rpb));
    hipLaunchKernelGGL((k_bn_fin_ticket<MODE>), grid, dim3(256), 0, st, (float2*)part, nparts, rpb, (int)M, C, a0, a1,
                       (float2*)out, eps, momentum, accumulate, ticket);
    return;
  }
  if constexpr (MODE == 0) {
#define FIN(CW) hipLaunchKernelGGL((k_bn_finalize<CW, BN_FIN_NTH(CW)>), dim3((C + CW - 1) / CW), dim3(BN_FIN_NTH(CW)), 0, \
                                   st, (const float2*)part, nparts, (int)M, C, a0, a1, (float2*)out, eps, momentum)
    BN_FIN_DISPATCH(C, FIN);
#undef FIN
  } else {
#define FIN(CW) hipLaunchKernelGGL((k_bn_bwd_finalize<CW, BN_FIN_NTH(CW)>), dim3((C + CW - 1) / CW), dim3(BN_FIN_NTH(CW)), \
                                   0, st, (const float2*)part, nparts, C, a0, a1, (float2*)out, accumulate)
    BN_FIN_DISPATCH(C, FIN);
#undef FIN
  }
}
}  // namespace

using namespace dca::ops;

extern "C" {

const char* dca_ops_last_error() { return g_err.c_str(); }
int dca_ops_abi_version() { return 13; }

// Must match ops/_native.py::GemmArgs.
int dca_ops_gemm(const GemmArgs* a, void* stream) {
  GemmArgs g = *a;
  hipStream_t st = (hipStream_t)stream;
  REQUIRE(g.M > 0 && g.N > 0 && g.K > 0, "gemm: empty problem");
  REQUIRE(!g.fp8 || (!g.ta && !g.tb), "gemm: fp8 operands must be K-contiguous (ta = tb = 0)");
  REQUIRE(!g.fp8 || (g.K % 16 == 0 && (g.conv == 1 || g.lda % 16 == 0) && g.ldb % 16 == 0),
          "gemm: fp8 needs K, lda, ldb % 16 == 0");
  REQUIRE(g.conv == 1 || g.ta || g.lda >= g.K, "gemm: lda < K");
  REQUIRE(g.conv == 2 || !g.tb || g.ldb >= g.N, "gemm: ldb < N (transposed B)");
  REQUIRE(g.conv == 2 || g.tb || g.ldb >= g.K, "gemm: ldb < K");
  REQUIRE(g.conv == 1 || !g.ta || g.lda >= g.M, "gemm: lda < M (transposed A)");
  REQUIRE(g.ldc >= g.N, "gemm: ldc < N");
  REQUIRE(g.conv >= 0 && g.conv <= 2, "gemm: bad conv mode");
  REQUIRE(g.conv != 1 || g.K < (1 << 24), "gemm: implicit conv K >= 2^24");
  if (g.conv) {
    REQUIRE(g.cC > 0 && (g.fp8 ? (g.conv == 1 && g.cC % 16 == 0) : g.cC % 8 == 0),
            "gemm: implicit conv needs C % 8 == 0 (bf16) or an fp8 forward with C % 16 == 0");
    // a sub-pixel input-gradient class (orow_S > 0) relies on the gather's bounds checks for its one-sided
    // padding, so its output grid is only bounded; otherwise the usual convolution arithmetic
    REQUIRE(g.orow_S > 0 ? (g.conv == 1 && g.cHo >= 1 && g.cWo >= 1 && g.cHo <= g.cH && g.cWo <= g.cW)
                         : (g.cHo == (g.cH + 2 * g.cP - g.cKH) / g.cS + 1 && g.cWo == (g.cW + 2 * g.cP - g.cKW) / g.cS + 1),
            "gemm: inconsistent conv geometry");
    const long pix = (long)g.cN * g.cHo * g.cWo, kc = (long)g.cKH * g.cKW * g.cC;
    REQUIRE(g.conv != 1 || (g.M == pix && g.K == kc && !g.ta), "gemm: conv A shape mismatch");
    REQUIRE(g.conv != 2 || (g.K == pix && g.N == kc && !g.tb), "gemm: conv B shape mismatch");
  }
  REQUIRE(!g.col_stats || (g.stats_shift && g.splits <= 1), "gemm: column stats need a shift and no split-K");
  REQUIRE(!g.beta_mask || (g.beta_src && g.beta_src != g.C && g.beta != 0.f && g.out_bf16 && !g.ta &&
                           g.splits <= 1 && g.wperm_T <= 0 && g.orow_S <= 0 && g.N % 8 == 0 && g.ldc % 8 == 0 &&
                           ((uintptr_t)g.beta_src & 15) == 0),
          "gemm: a masked accumulation source needs a separate 16-B aligned bf16 source, beta != 0 and a plain "
          "bf16 output with N, ldc % 8 == 0");
  REQUIRE(g.orow_S <= 0 || (g.splits <= 1 && g.wperm_T <= 0 && g.orow_Ho > 0 && g.orow_Wo > 0 &&
                            (long)g.orow_Ho * g.orow_Wo > 0 && g.M % ((long)g.orow_Ho * g.orow_Wo) == 0 &&
                            g.orow_S * (g.orow_Ho - 1) + g.orow_ph < g.orow_H &&
                            g.orow_S * (g.orow_Wo - 1) + g.orow_pw < g.orow_W),
          "gemm: output row remap needs the epilogue path and a consistent pixel grid");
  if (!g_lds_set) {
    OPCK(hipFuncSetAttribute((const void*)k_gemm<false, 128>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             GemmTile<128>::LDS));
    OPCK(hipFuncSetAttribute((const void*)k_gemm<true, 128>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             GemmTile<128>::LDS));
    OPCK(hipFuncSetAttribute((const void*)k_gemm<false, 64>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             GemmTile<64>::LDS));
    OPCK(hipFuncSetAttribute((const void*)k_gemm<true, 64>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             GemmTile<64>::LDS));
    {
      constexpr int l00 = WgradTile<64, 64, 2>::LDS, l01 = WgradTile<64, 128, 1>::LDS;
      constexpr int l10 = WgradTile<128, 64, 4>::LDS, l11 = WgradTile<128, 128, 2>::LDS;
      OPCK(hipFuncSetAttribute((const void*)k_wgrad<64, 64, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, l00));
      OPCK(hipFuncSetAttribute((const void*)k_wgrad<64, 128, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, l01));
      OPCK(hipFuncSetAttribute((const void*)k_wgrad<128, 64, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, l10));
      OPCK(hipFuncSetAttribute((const void*)k_wgrad<128, 128, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, l11));
#define WPP_ATTR(PBN, SW) \
  OPCK(hipFuncSetAttribute((const void*)k_wgrad_pp<PBN, SW>, hipFuncAttributeMaxDynamicSharedMemorySize, WpTile<PBN>::LDS))
      WPP_ATTR(256, false);
      WPP_ATTR(128, false);
      WPP_ATTR(128, true);
#undef WPP_ATTR
#define GLDS_ATTR(F8, BNV, NWV)                                                                          \
  OPCK(hipFuncSetAttribute((const void*)k_gemm_glds<F8, BNV, NWV>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                           4 * GemmTile<BNV>::BUF))
      GLDS_ATTR(false, 128, 4);
      GLDS_ATTR(true, 128, 4);
      GLDS_ATTR(false, 64, 4);
      GLDS_ATTR(true, 64, 4);
      GLDS_ATTR(false, 128, 8);
      GLDS_ATTR(true, 128, 8);
      GLDS_ATTR(false, 64, 8);
      GLDS_ATTR(true, 64, 8);
#undef GLDS_ATTR
    }
    OPCK(hipFuncSetAttribute((const void*)k_gemm_pp<256>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             PpTile<256>::LDS));
    OPCK(hipFuncSetAttribute((const void*)k_gemm_pp4<false>, hipFuncAttributeMaxDynamicSharedMemorySize, PP4_LDS));
    OPCK(hipFuncSetAttribute((const void*)k_gemm_pp4<true>, hipFuncAttributeMaxDynamicSharedMemorySize, PP4_LDS));
    OPCK(hipFuncSetAttribute((const void*)k_gemm_stream<2, 1, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             2 * (2 * G_TILE_BYTES + 8192) + 2 * 2048 * 4));
    OPCK(hipFuncSetAttribute((const void*)k_gemm_stream<2, 1, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             2 * (2 * G_TILE_BYTES + 8192) + 2 * 2048 * 4));
    OPCK(hipFuncSetAttribute((const void*)k_gemm_stream<2, 2, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             2 * (2 * G_TILE_BYTES + 8192) + 2 * 2048 * 4));
    OPCK(hipFuncSetAttribute((const void*)k_gemm_stream<2, 2, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             2 * (2 * G_TILE_BYTES + 8192) + 2 * 2048 * 4));
    g_lds_set = true;
  }
  const int kt = GBK_BYTES / (g.fp8 ? 1 : 2);
  if (g.splits < 1) g.splits = 1;
  REQUIRE(g.wperm_T <= 0 || (g.ws && !g.col_stats && g.wperm_C > 0 && g.wperm_Cpad >= g.wperm_C),
          "gemm: weight-layout remap needs a workspace and no column stats");
  if (g.splits > 1) {
    REQUIRE(g.ws != nullptr, "gemm: split-K needs a workspace");
    int kps = (g.K + g.splits - 1) / g.splits;
    kps = (kps + kt - 1) / kt * kt;
    g.k_per_split = kps;
    g.splits = (g.K + kps - 1) / kps;
  } else {
    g.k_per_split = g.K;
  }
  // weight gradients (both operands pixel-major, bf16, 16-B aligned channel rows): the transposed-read kernel,
  // always through the slab + reduce pass
  const bool wgrad = !g.fp8 && g.ta && (g.tb || g.conv == 2) && g.M % 8 == 0 && g.N % 8 == 0 && g.lda % 8 == 0 &&
                     (g.conv == 2 || g.ldb % 8 == 0) && g.ws != nullptr;
  if (wgrad) {
    REQUIRE(g.conv != 2 || (long)g.cN * g.cHo * g.cWo < (1L << 24), "gemm: weight-gradient pixel count >= 2^24");
    // the 64-channel 3 x 3 / pad 1 weight gradient on rows <= 64 pixels: the row-ring kernel (k_wgrad3x3_rows), one
    // split slab per workgroup
    if (g.conv == 2 && g.cC == 64 && g.cKH == 3 && g.cKW == 3 && g.cP == 1 && g.cS == 1 && g.cW <= 64 &&
        g.cHo == g.cH && g.cWo == g.cW && g.M == 64 && g.N == 576 && g.K == g.cN * g.cH * g.cW && g.lda % 8 == 0 &&
        g.lda >= 64 && ((uintptr_t)g.A & 15) == 0 && ((uintptr_t)g.B & 15) == 0 &&
        (long long)g.cN * g.cH * g.cW * g.lda * 2 < (1LL << 31) && (long long)g.cN * g.cH * g.cW * 128 < (1LL << 31) &&
        getenv_conv_rows() && getenv_wgrad_rows()) {
      static int ncu_w = 0;
      if (!ncu_w) {
        int dev = 0;
        OPCK(hipGetDevice(&dev));
        OPCK(hipDeviceGetAttribute(&ncu_w, hipDeviceAttributeMultiprocessorCount, dev));
      }
      const long cg = std::min<long>(std::min<long>(g.splits, 2L * ncu_w), (long)g.cN * g.cH);
      g.splits = (int)cg;
      const dim3 cgd((unsigned)cg), cb(CR_NT);
      if (g.cW <= 32) hipLaunchKernelGGL(k_wgrad3x3_rows<1>, cgd, cb, WR_LDS, st, g);
      else hipLaunchKernelGGL(k_wgrad3x3_rows<2>, cgd, cb, WR_LDS, st, g);
      hipLaunchKernelGGL(k_gemm_splitk_reduce, dim3(grid_for((long)g.M * g.N, RED_EL, 4096)), dim3(256), 0, st, g);
      OPCK(hipGetLastError());
      return 0;
    }
    // the 128-channel 3 x 3 / pad 1 weight gradient on rows <= 32 pixels (layer 2): k_wgrad3x3_rows<1, 128>,
    // two workgroups (output-channel halves) per split slab, one workgroup per CU
    if (g.conv == 2 && g.cC == 128 && g.cKH == 3 && g.cKW == 3 && g.cP == 1 && g.cS == 1 && g.cW <= 32 &&
        g.cHo == g.cH && g.cWo == g.cW && g.M == 128 && g.N == 1152 && g.K == g.cN * g.cH * g.cW && g.lda % 8 == 0 &&
        g.lda >= 128 && ((uintptr_t)g.A & 15) == 0 && ((uintptr_t)g.B & 15) == 0 &&
        (long long)g.cN * g.cH * g.cW * g.lda * 2 < (1LL << 31) && (long long)g.cN * g.cH * g.cW * 256 < (1LL << 31) &&
        getenv_conv_rows() && getenv_wgrad_rows()) {
      static int ncu_w2 = 0;
      if (!ncu_w2) {
        int dev = 0;
        OPCK(hipGetDevice(&dev));
        OPCK(hipDeviceGetAttribute(&ncu_w2, hipDeviceAttributeMultiprocessorCount, dev));
      }
      const long cg = std::min<long>(std::min<long>(g.splits, ncu_w2 / 2), (long)g.cN * g.cH);
      g.splits = (int)cg;
      const dim3 cgd((unsigned)(2 * cg)), cb(WgradRows<128>::NT);
      hipLaunchKernelGGL((k_wgrad3x3_rows<1, 128>), cgd, cb, WgradRows<128>::LDS, st, g);
      hipLaunchKernelGGL(k_gemm_splitk_reduce, dim3(grid_for((long)g.M * g.N, RED_EL, 4096)), dim3(256), 0, st, g);
      OPCK(hipGetLastError());
      return 0;
    }
    // the space-to-depth stem's weight gradient (4 x 4 taps over 16 channels) on rows <= 128 input pixels:
    // k_wgrad_s2d_rows, one split slab per workgroup
    if (g.conv == 2 && g.cC == 16 && g.cKH == 4 && g.cKW == 4 && g.cP == 0 && g.cS == 1 && g.cW <= 128 &&
        g.cHo == g.cH - 3 && g.cWo == g.cW - 3 && g.M == 64 && g.N == 256 && g.K == g.cN * g.cHo * g.cWo &&
        g.lda % 8 == 0 && g.lda >= 64 && ((uintptr_t)g.A & 15) == 0 && ((uintptr_t)g.B & 15) == 0 &&
        (long long)g.cN * g.cHo * g.cWo * g.lda * 2 < (1LL << 31) && (long long)g.cN * g.cH * g.cW * 32 < (1LL << 31) &&
        getenv_conv_rows() && getenv_wgrad_rows()) {
      static int ncu_s2 = 0;
      if (!ncu_s2) {
        int dev = 0;
        OPCK(hipGetDevice(&dev));
        OPCK(hipDeviceGetAttribute(&ncu_s2, hipDeviceAttributeMultiprocessorCount, dev));
      }
      const long cg = std::min<long>(std::min<long>(g.splits, 3L * ncu_s2), (long)g.cN * g.cHo);
      g.splits = (int)cg;
      const dim3 cgd((unsigned)cg), cb(CR_NT);
      switch ((g.cWo + 31) >> 5) {
        case 1: hipLaunchKernelGGL(k_wgrad_s2d_rows<1>, cgd, cb, WS_LDS, st, g); break;
        case 2: hipLaunchKernelGGL(k_wgrad_s2d_rows<2>, cgd, cb, WS_LDS, st, g); break;
        case 3: hipLaunchKernelGGL(k_wgrad_s2d_rows<3>, cgd, cb, WS_LDS, st, g); break;
        default: hipLaunchKernelGGL(k_wgrad_s2d_rows<4>, cgd, cb, WS_LDS, st, g); break;
      }
      hipLaunchKernelGGL(k_gemm_splitk_reduce, dim3(grid_for((long)g.M * g.N, RED_EL, 4096)), dim3(256), 0, st, g);
      OPCK(hipGetLastError());
      return 0;
    }
    // the ping-pong kernel: the larger of M (output channels) / N (input channels x taps) along its 256-row side
    // (SW: N), the smaller one as a 256 / 128 column tile; 32-bit operand offsets, 16-B aligned rows.  The split
    // count is cut to about one workgroup per CU (one fits per CU).  Shape rule from bench/wgrad_bench.py at batch
    // 256 (profiles/wgrad_pp_r3.log): M >= 256, N >= 128 -> 0.71-0.92x the k_wgrad time (3x3 256x2304x50176 123.4
    // -> 92.1 us); swapped only for plain (1x1) operands with 64 < M <= 128 (0.89-0.92x); the swapped implicit 3x3
    // convolutions (1.5-1.7x) and the 64-wide column tile (1.0-1.7x) measured slower and stay on k_wgrad
    const long long a_by = (long long)g.K * g.lda * 2;
    const long long b_by = g.conv == 2 ? (long long)g.cN * g.cH * g.cW * g.cC * 2 : (long long)g.K * g.ldb * 2;
    const bool sw = g.M < 256;
    const int big = sw ? g.N : g.M, small = sw ? g.M : g.N;
    const bool pp_shape = sw ? (g.conv != 2 && small > 64 && small <= 128 && big >= 256) : (big >= 256 && small >= 128);
    if (pp_shape && a_by < (1LL << 31) && b_by < (1LL << 31) && ((uintptr_t)g.A & 15) == 0 &&
        ((uintptr_t)g.B & 15) == 0 && (g.conv != 2 || g.cC % 8 == 0)) {
      const int pbn = sw ? 128 : ((small % 256 == 0 || small > 1024) ? 256 : 128);
      const long tiles = (long)((big + WP_BM - 1) / WP_BM) * ((small + pbn - 1) / pbn);
      const long want = std::max<long>(1, (256 + tiles - 1) / tiles);
      if (want < g.splits) {  // fewer, longer splits (the slab was sized for g.splits: smaller is fine)
        int kps = (int)((g.K + want - 1) / want);
        kps = (kps + WP_KT - 1) / WP_KT * WP_KT;
        g.k_per_split = kps;
        g.splits = (g.K + kps - 1) / kps;
      }
      const dim3 grid((unsigned)(tiles * g.splits)), blk(WP_NT);
      // (the four-slot k32 ring schedule of k_gemm_pp4 measured 20-30 % slower here: each interval would carry
      // 24 transposed fragment reads and 6 DMA pieces, longer than the other group's 32 MFMAs;
      // profiles/gemm_ring_ab_r7.log)
      if (sw) {
        hipLaunchKernelGGL((k_wgrad_pp<128, true>), grid, blk, WpTile<128>::LDS, st, g);
      } else if (pbn == 256) {
        hipLaunchKernelGGL((k_wgrad_pp<256, false>), grid, blk, WpTile<256>::LDS, st, g);
      } else {
        hipLaunchKernelGGL((k_wgrad_pp<128, false>), grid, blk, WpTile<128>::LDS, st, g);
      }
      hipLaunchKernelGGL(k_gemm_splitk_reduce, dim3(grid_for((long)g.M * g.N, RED_EL, 4096)), dim3(256), 0, st, g);
      OPCK(hipGetLastError());
      return 0;
    }
    const int bm = g.M <= 64 ? 64 : 128, bn = g.N <= 64 ? 64 : 128;
    const long items = (long)((g.M + bm - 1) / bm) * ((g.N + bn - 1) / bn) * g.splits;
    REQUIRE(items < (1L << 31), "gemm: too many work items");
    const dim3 grid((unsigned)items);
    // single LDS buffer: more resident workgroups per CU for these latency-bound loops
    g.single = WGRAD_SINGLE ? 1 : 0;
    const int sh = g.single ? 1 : 0;
    const int l00 = WgradTile<64, 64, 2>::LDS >> sh, l01 = WgradTile<64, 128, 1>::LDS >> sh;
    const int l10 = WgradTile<128, 64, 4>::LDS >> sh, l11 = WgradTile<128, 128, 2>::LDS >> sh;
    if (bm == 64 && bn == 64) hipLaunchKernelGGL((k_wgrad<64, 64, 2>), grid, dim3(256), l00, st, g);
    else if (bm == 64) hipLaunchKernelGGL((k_wgrad<64, 128, 1>), grid, dim3(256), l01, st, g);
    else if (bn == 64) hipLaunchKernelGGL((k_wgrad<128, 64, 4>), grid, dim3(256), l10, st, g);
    else hipLaunchKernelGGL((k_wgrad<128, 128, 2>), grid, dim3(256), l11, st, g);
    hipLaunchKernelGGL(k_gemm_splitk_reduce, dim3(grid_for((long)g.M * g.N, RED_EL, 4096)), dim3(256), 0, st, g);
    OPCK(hipGetLastError());
    return 0;
  }
  // persistent stream kernel (k_gemm_stream), bf16 -> bf16, K % 64 == 0, no split / remap / ReLU:
  //   plain NT, N % 128 == 0: by default for K <= 512 and M >= 16384, accumulating (beta) calls only for K <= 128
  //     (the output-heavy 1x1 convolutions and their input gradients; profiles/gemm_shortk_r2.log);
  //   N = 64: 256 x 64 tiles (802816 x 64 x 256: 123.4 -> 109.1 us);
  //   implicit conv with C % 64 == 0, N = 128: M >= 16384 (ResNet-50's layer-2 3x3 convolutions and their input
  //     gradients: 129.5 -> 117.5 us at batch 256).  The N = 64 conv stays on the one-tile kernel unless forced
  //     (DCA_OPS_STREAM=1, diagnostic): 174 us there, 218 us with 128 x 64 stream tiles, 283 us with 256 x 64
  // stride-1 implicit convs with 64 outputs on narrow input rows -> k_direct_conv: the space-to-depth ResNet stem
  // (4 x 4 taps over 16 channels) and the 64-channel 3 x 3 / pad 1 convolutions (layer 1 forward and input gradient)
  // the 128-channel 3 x 3 / pad 1 convs on rows <= 32 pixels (ResNet-50's layer 2 at 28 x 28, forward and input
  // gradient) -> the row-ring kernel k_conv3x3_rows<NF, 128> (one 8-wave workgroup per CU)
  if (g.conv == 1 && g.cC == 128 && g.cKH == 3 && g.cKW == 3 && g.cP == 1 && g.cS == 1 && g.cW <= 32 &&
      g.cHo == g.cH && g.cWo == g.cW && g.N == 128 && g.K == 1152 && !g.fp8 && !g.tb && g.splits == 1 &&
      g.wperm_T <= 0 && g.orow_S <= 0 && g.out_bf16 && !g.relu && g.beta == 0.f && !g.beta_mask && g.ldb >= g.K &&
      g.ldb % 8 == 0 && g.ldc >= 128 && g.ldc % 8 == 0 && ((uintptr_t)g.A & 15) == 0 && ((uintptr_t)g.B & 15) == 0 &&
      ((uintptr_t)g.C & 15) == 0 && (long long)g.cN * g.cH * g.cW * 256 < (1LL << 31) &&
      (long long)g.M * g.ldc * 2 < (1LL << 31) && g.M < (1 << 24) && getenv_conv_rows()) {
    static int ncu_r = 0;
    if (!ncu_r) {
      int dev = 0;
      OPCK(hipGetDevice(&dev));
      OPCK(hipDeviceGetAttribute(&ncu_r, hipDeviceAttributeMultiprocessorCount, dev));
    }
    long cg = std::min<long>(ncu_r, (long)g.cN * g.cH);
    if (g.col_stats) cg = std::min<long>(cg, (g.M + GBM - 1) / GBM);
    constexpr int lds = RowConv<128>::LDS;
    const dim3 cgd((unsigned)cg), cb(RowConv<128>::NT);
    if (g.cW <= 16) hipLaunchKernelGGL((k_conv3x3_rows<1, 128>), cgd, cb, lds, st, g);
    else hipLaunchKernelGGL((k_conv3x3_rows<2, 128>), cgd, cb, lds, st, g);
    OPCK(hipGetLastError());
    return 0;
  }
  const bool dc_stem = g.cC == 16 && g.cKH == 4 && g.cKW == 4 && g.cP == 0;
  const bool dc_3x3 = g.cC == 64 && g.cKH == 3 && g.cKW == 3 && g.cP == 1;
  // (the kernel loops over the compile-time K = KH KW C: an mnk override or a padded K must not reach it)
  if (g.conv == 1 && (dc_stem || dc_3x3) && g.K == g.cKH * g.cKW * g.cC && g.cS == 1 && g.N == 64 && !g.fp8 && !g.tb && g.splits == 1 && g.wperm_T <= 0 && g.orow_S <= 0 && g.out_bf16 && !g.relu &&
      g.beta == 0.f && !g.beta_mask && g.ldb >= g.K && g.ldb % 8 == 0 && g.ldc >= 64 && g.ldc % 8 == 0 &&
      ((uintptr_t)g.A & 15) == 0 && ((uintptr_t)g.B & 15) == 0 && ((uintptr_t)g.C & 15) == 0 &&
      (long long)g.cN * g.cH * g.cW * g.cC * 2 < (1LL << 31) && (long long)g.M * g.ldc * 2 < (1LL << 31) &&
      g.M < (1 << 24)) {
    static int ncu_s = 0;
    if (!ncu_s) {
      int dev = 0;
      OPCK(hipGetDevice(&dev));
      OPCK(hipDeviceGetAttribute(&ncu_s, hipDeviceAttributeMultiprocessorCount, dev));
    }
    const long blocks = (g.M + GBM - 1) / GBM;
    long grid = std::min<long>(2L * ncu_s, (blocks + 7) / 8 * 8);
    grid = std::max<long>(8, grid / 8 * 8);
    if (dc_3x3 && g.cW <= 64 && getenv_conv_rows()) {  // row-ring form (k_conv3x3_rows): the layer-1 shapes
      long cg = std::min<long>(3L * ncu_s, (long)g.cN * g.cH);
      if (g.col_stats) cg = std::min<long>(cg, blocks);  // one statistics row per workgroup
      const dim3 cgd((unsigned)cg), cb(CR_NT);
      switch ((g.cW + 15) >> 4) {
        case 1: hipLaunchKernelGGL(k_conv3x3_rows<1>, cgd, cb, CR_LDS, st, g); break;
        case 2: hipLaunchKernelGGL(k_conv3x3_rows<2>, cgd, cb, CR_LDS, st, g); break;
        case 3: hipLaunchKernelGGL(k_conv3x3_rows<3>, cgd, cb, CR_LDS, st, g); break;
        default: hipLaunchKernelGGL(k_conv3x3_rows<4>, cgd, cb, CR_LDS, st, g); break;
      }
    } else if (dc_stem && g.cW <= 128 && getenv_conv_rows()) {  // the stem's row-ring form (k_conv_s2d_rows)
      long cg = std::min<long>(3L * ncu_s, (long)g.cN * g.cHo);
      if (g.col_stats) cg = std::min<long>(cg, blocks);
      const dim3 cgd((unsigned)cg), cb(CR_NT);
      switch ((g.cWo + 15) >> 4) {
        case 1: hipLaunchKernelGGL(k_conv_s2d_rows<1>, cgd, cb, CS_LDS, st, g); break;
        case 2: hipLaunchKernelGGL(k_conv_s2d_rows<2>, cgd, cb, CS_LDS, st, g); break;
        case 3: hipLaunchKernelGGL(k_conv_s2d_rows<3>, cgd, cb, CS_LDS, st, g); break;
        case 4: hipLaunchKernelGGL(k_conv_s2d_rows<4>, cgd, cb, CS_LDS, st, g); break;
        case 5: hipLaunchKernelGGL(k_conv_s2d_rows<5>, cgd, cb, CS_LDS, st, g); break;
        case 6: hipLaunchKernelGGL(k_conv_s2d_rows<6>, cgd, cb, CS_LDS, st, g); break;
        case 7: hipLaunchKernelGGL(k_conv_s2d_rows<7>, cgd, cb, CS_LDS, st, g); break;
        default: hipLaunchKernelGGL(k_conv_s2d_rows<8>, cgd, cb, CS_LDS, st, g); break;
      }
    } else if (dc_stem) {
      constexpr int lds = DirectConv<16, 4, 4>::LDS;
      hipLaunchKernelGGL((k_direct_conv<16, 4, 4>), dim3((unsigned)grid), dim3(DC_NT), lds, st, g);
    } else {
      constexpr int lds = DirectConv<64, 3, 3>::LDS;
      static bool attr = false;
      if (!attr) {
        OPCK(hipFuncSetAttribute((const void*)k_direct_conv<64, 3, 3>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 lds));
        attr = true;
      }
      hipLaunchKernelGGL((k_direct_conv<64, 3, 3>), dim3((unsigned)grid), dim3(DC_NT), lds, st, g);
    }
    OPCK(hipGetLastError());
    return 0;
  }
  {
    const int sk = getenv_stream();
    const bool conv = g.conv == 1;
    const long long ab = conv ? (long long)g.cN * g.cH * g.cW * g.cC * 2 : ((long long)(g.M - 1) * g.lda + g.K) * 2;
    const long long bb = ((long long)(g.N - 1) * g.ldb + g.K) * 2;
    const long long cbytes = (long long)g.M * g.ldc * 2;
    const int mw = g.N % 128 == 0 ? 1 : 2;  // 128 x 128 tiles, or 256 x 64 for N % 128 == 64
    const bool shape_ok = conv ? (g.cC % 64 == 0 && g.cKH * g.cKW <= 32 &&
                                  (g.N == 64 || g.N == 128 || (g.cKH * g.cKW == 1 && g.N % 128 == 0)) &&
                                  g.orow_S <= 0 &&
                                  g.M < (1 << 24) &&
                                  (sk == 1 || (sk == 2 && STREAM_CONV && g.M >= 16384 &&
                                               (g.N == 128 || (g.cKH * g.cKW == 1 && g.N % 128 == 0)))))
                               : (g.conv == 0 && !g.ta && g.lda % 8 == 0 && g.lda >= g.K &&
                                  (g.N % 128 == 0 || g.N == 64) &&
                                  (sk == 1 || (g.K <= 512 && g.M >= 16384 &&
                                               (g.beta == 0.f || g.K <= 128 || (g.beta_mask && g.K <= 256)))));
    const bool st_ok = sk != 0 && shape_ok && !g.fp8 && !g.tb && g.splits == 1 && g.wperm_T <= 0 && g.orow_S <= 0 &&
                       !(conv && g.beta_mask) &&
                       !g.relu && g.out_bf16 && g.N % 64 == 0 && g.N <= 2048 && g.K % 64 == 0 &&
                       g.K > 0 && g.M > 0 && g.ldb % 8 == 0 && g.ldc % 8 == 0 && g.ldb >= g.K && g.ldc >= g.N &&
                       ((uintptr_t)g.A & 15) == 0 && ((uintptr_t)g.B & 15) == 0 && ((uintptr_t)g.C & 15) == 0 &&
                       ab < (1LL << 31) && bb < (1LL << 31) && cbytes < (1LL << 31) &&
                       (long long)((g.M + GBM - 1) / GBM) * g.N * 8 < (1LL << 31);
    if (st_ok) {
      static int ncu = 0;
      if (!ncu) {
        int dev = 0;
        OPCK(hipGetDevice(&dev));
        OPCK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
      }
      const long tiles = (long)((g.M + GBM * mw - 1) / (GBM * mw)) * (g.N / (128 / mw));
      long grid = std::min<long>(2L * ncu, (tiles + 7) / 8 * 8);  // two resident workgroups per CU
      grid = std::max<long>(8, grid / 8 * 8);
      const int lds = 2 * (GBM * mw * 128 + (128 / mw) * 128) + 2 * g.N * 4;  // 2 x (A | B) + bias | shift
      const dim3 gr((unsigned)grid), bl(ST_NT);
      if (conv) {
        if (mw == 1) hipLaunchKernelGGL((k_gemm_stream<2, 1, true>), gr, bl, lds, st, g);
        else hipLaunchKernelGGL((k_gemm_stream<2, 2, true>), gr, bl, lds, st, g);
      } else {
        if (mw == 1) hipLaunchKernelGGL((k_gemm_stream<2, 1, false>), gr, bl, lds, st, g);
        else hipLaunchKernelGGL((k_gemm_stream<2, 2, false>), gr, bl, lds, st, g);
      }
      OPCK(hipGetLastError());
      return 0;
    }
  }
  if (g.beta_mask) {  // the other kernels read C_old from C: materialise the masked source there first
    hipLaunchKernelGGL(k_masked_copy, dim3(grid_for((long)g.M * (g.N / 8), 256, 4096)), dim3(256), 0, st,
                       (const unsigned short*)g.beta_src, g.beta_mask, (unsigned short*)g.C, g.M, g.N, g.ldc);
    g.beta_mask = nullptr;
    g.beta_src = nullptr;
  }
  // ping-pong 256 x 256 kernel: bf16, K-contiguous operands (plain or the C % 64 implicit conv), no split-K / row
  // remap / fused BN-backward statistics, 16-B aligned rows, operands addressable with 32-bit offsets
  {
    const long long ab = g.conv == 1 ? (long long)g.cN * g.cH * g.cW * g.cC * 2 : ((long long)(g.M - 1) * g.lda + g.K) * 2;
    const long long bb = ((long long)(g.N - 1) * g.ldb + g.K) * 2;
    // shape rule (no wasted MFMA columns, >= 160 of the 256 CUs busy, K >= 1024 to amortise the pipeline fill and
    // the 256-row epilogue): measured 4096^3 779 -> 1037 TF, 3x3 conv 256x14x14x256 109 -> 81.6 us; the ResNet-50
    // batch-256 census (profiles/gemm_pingpong_r2.log) loses on N = 128 (+54 %), 98-tile grids (+38 %) and
    // K = 256 (+20 %), wins on 50176 x 256 x {1024, 2304} (-8 %, -21 %)
    // N % 256 != 0 (e.g. 128): the 256 x 128 tile
    const int ppbn = g.N % 256 == 0 ? 256 : 128;
    const long pp_tiles = (long)((g.M + PP_BM - 1) / PP_BM) * ((g.N + ppbn - 1) / ppbn);
    // (a 256 x 128 tile measured slower than the 128 x 128 kernels on every ResNet-50 N = 128 shape, +12-18 %:
    // 16 MFMAs per barrier interval do not cover the other group's fragment loads; removed in round 5)
    // k_gemm_pp4 (the default) also takes 512 <= K < 1024 (12544 x 2048 x 512 53.3 -> 46.1 us, 12544 x 1024 x 512
    // 34.8 -> 25.4; below 160 tiles it still loses to the 128 x 128 kernels: profiles/gemm_ring_ab_r7.log)
    const bool pp_shape = ppbn == 256 && pp_tiles >= 160 && g.K >= (getenv_pp4() ? 512 : 1024);
    const bool pp = pp_shape && !g.fp8 && !g.ta && !g.tb && g.splits == 1 && g.wperm_T <= 0 && g.orow_S <= 0 &&
                    g.M >= 256 && g.N >= 128 && g.K >= 256 && ab < (1LL << 31) && bb < (1LL << 31) &&
                    (long)g.ldb * 2 % 16 == 0 && ((uintptr_t)g.A & 15) == 0 && ((uintptr_t)g.B & 15) == 0 &&
                    (g.conv == 1 ? (g.cC % 64 == 0 && g.cKH * g.cKW <= 32 && g.M < (1 << 24))
                                 : (g.conv == 0 && (long)g.lda * 2 % 16 == 0 && (long)g.K * 2 % 16 == 0));
    if (pp && g.K % 64 == 0 && getenv_pp4()) {  // the four-slot k32 ring form (k_gemm_pp4)
      if (g.conv == 1) hipLaunchKernelGGL(k_gemm_pp4<true>, dim3((unsigned)pp_tiles), dim3(PP_NT), PP4_LDS, st, g);
      else hipLaunchKernelGGL(k_gemm_pp4<false>, dim3((unsigned)pp_tiles), dim3(PP_NT), PP4_LDS, st, g);
      OPCK(hipGetLastError());
      return 0;
    }
    if (pp) {
      hipLaunchKernelGGL(k_gemm_pp<256>, dim3((unsigned)pp_tiles), dim3(PP_NT), PpTile<256>::LDS, st, g);
      OPCK(hipGetLastError());
      return 0;
    }
  }
  // narrow N (<= 64) with a K-contiguous B operand: the 128x64 tile
  const bool narrow = g.N <= 64 && !g.tb && g.conv != 2;
  const int bn = narrow ? 64 : 128;
  const int tiles = ((g.M + GBM - 1) / GBM) * ((g.N + bn - 1) / bn);
  const dim3 grid(tiles, g.splits);
  g.single = g.k_per_split <= REG_SINGLE_NK * kt ? 1 : 0;  // short K: one buffer, 2x workgroups per CU
  // K-contiguous operands with 16-B aligned rows: direct global -> LDS staging (k_gemm_glds)
  const int esz = g.fp8 ? 1 : 2;
  // (measured, bench/gemm_bench.py: +18..100 % on plain NT GEMMs; bf16 implicit convs only when C % 64 == 0 (one
  // tap per K-tile: a wave-uniform decode); fp8 implicit convs always (the register-staged fp8
  // kernel needs 219 VGPRs: one wave per SIMD); short-K narrow tiles stay on the single-buffer register kernel)
  const bool glds = !g.ta && !g.tb && !(narrow && g.single && !GLDS_NARROW) &&
                    (g.conv == 1 ? (g.fp8 || (g.cC % 64 == 0 && GLDS_CONV))
                                 : (g.conv == 0 && (long)g.lda * esz % 16 == 0 && (long)g.K * esz % 16 == 0)) &&
                    (long)g.ldb * esz % 16 == 0 && ((uintptr_t)g.A & 15) == 0 && ((uintptr_t)g.B & 15) == 0;
  if (glds) {
    g.single = g.k_per_split <= GLDS_SINGLE_NK * kt ? 1 : 0;
    g.stages = g.single ? 1 : GLDS_STAGES;
    const int l64b = g.single ? GemmTile<64>::LDS_SINGLE : g.stages * GemmTile<64>::BUF;
    const int l128b = g.single ? GemmTile<128>::LDS_SINGLE : g.stages * GemmTile<128>::BUF;
    // 8 waves (4 per SIMD at 2 workgroups per CU) for the double-buffered long-K loops: 0.92-0.95x time on the
    // batch-256 long-K convs; the single-buffer short-K launches keep 4 (8 measured 1.13-1.41x there)
    const bool w8 = !g.single;
    const dim3 blk(w8 ? 512 : 256);
    // the epilogue's column-statistics combine uses (threads / (BN / 8)) x BN float2 of LDS
    const int red64 = (w8 ? 512 : 256) / 8 * 64 * 8, red128 = (w8 ? 512 : 256) / 16 * 128 * 8;
    const int l64 = std::max(l64b, red64), l128 = std::max(l128b, red128);
    if (narrow) {
      if (g.fp8) {
        if (w8) hipLaunchKernelGGL((k_gemm_glds<true, 64, 8>), grid, blk, l64, st, g);
        else hipLaunchKernelGGL((k_gemm_glds<true, 64, 4>), grid, blk, l64, st, g);
      } else {
        if (w8) hipLaunchKernelGGL((k_gemm_glds<false, 64, 8>), grid, blk, l64, st, g);
        else hipLaunchKernelGGL((k_gemm_glds<false, 64, 4>), grid, blk, l64, st, g);
      }
    } else {
      if (g.fp8) {
        if (w8) hipLaunchKernelGGL((k_gemm_glds<true, 128, 8>), grid, blk, l128, st, g);
        else hipLaunchKernelGGL((k_gemm_glds<true, 128, 4>), grid, blk, l128, st, g);
      } else {
        if (w8) hipLaunchKernelGGL((k_gemm_glds<false, 128, 8>), grid, blk, l128, st, g);
        else hipLaunchKernelGGL((k_gemm_glds<false, 128, 4>), grid, blk, l128, st, g);
      }
    }
  } else if (narrow) {
    const int lds = g.single ? GemmTile<64>::LDS_SINGLE : GemmTile<64>::LDS;
    if (g.fp8) hipLaunchKernelGGL((k_gemm<true, 64>), grid, dim3(GT), lds, st, g);
    else hipLaunchKernelGGL((k_gemm<false, 64>), grid, dim3(GT), lds, st, g);
  } else {
    const int lds = g.single ? GemmTile<128>::LDS_SINGLE : GemmTile<128>::LDS;
    if (g.fp8) hipLaunchKernelGGL((k_gemm<true, 128>), grid, dim3(GT), lds, st, g);
    else hipLaunchKernelGGL((k_gemm<false, 128>), grid, dim3(GT), lds, st, g);
  }
  if (g.splits > 1 || g.wperm_T > 0)
    hipLaunchKernelGGL(k_gemm_splitk_reduce, dim3(grid_for((long)g.M * g.N, RED_EL, 4096)), dim3(256), 0, st, g);
  OPCK(hipGetLastError());
  return 0;
}

int dca_ops_im2col(const void* x, void* cols, const ConvGeom* geom, void* stream) {
  const ConvGeom g = *geom;
  REQUIRE(g.Kp % 8 == 0 && g.Kp >= g.K && g.K == g.KH * g.KW * g.C, "im2col: bad column geometry");
  const long work = (long)g.N * g.Ho * g.Wo * (g.Kp / 8);
  hipLaunchKernelGGL(k_im2col, dim3(grid_for(work)), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x,
                     (bf16_t*)cols, g);
  OPCK(hipGetLastError());
  return 0;
}

int dca_ops_col2im(const void* dcols, void* dx, const ConvGeom* geom, int accumulate, void* stream) {
  const ConvGeom g = *geom;
  REQUIRE(g.Kp % 8 == 0 && g.Kp >= g.K, "col2im: bad column geometry");
  hipLaunchKernelGGL(k_col2im, dim3(grid_for((long)g.N * g.H * g.W * g.C / ((g.C & 7) == 0 ? 8 : 1))), dim3(256), 0,
                     (hipStream_t)stream,
                     (const bf16_t*)dcols, (bf16_t*)dx, g, accumulate);
  OPCK(hipGetLastError());
  return 0;
}

// BatchNorm train forward fused with ReLU / residual.  part: [ceil(M/256)][C] float2 scratch; stats: [C] float2
// (mean, invstd) kept for the backward.  momentum 0: running stats untouched (but still the shift).
int dca_ops_bn_fwd(const void* x, const void* r, void* out, float* part, float* stats, const float* gamma,
                   const float* beta, float* rm, float* rv, long M, int C, float eps, float momentum, int relu,
                   int res_mode, unsigned* ticket, void* stream) {
  REQUIRE(C % 8 == 0, "bn: C must be a multiple of 8");
  REQUIRE(res_mode == 0 || r != nullptr, "bn: residual missing");
  hipStream_t st = (hipStream_t)stream;
  const int nparts = (int)((M + BN_ROWS - 1) / BN_ROWS);
  hipLaunchKernelGGL(k_bn_stats, dim3((C + 63) / 64, nparts), dim3(256), 0, st, (const bf16_t*)x, rm, (float2*)part,
                     (int)M, C);
  bn_fin_launch<0>(part, nparts, M, C, rm, rv, stats, eps, momentum, 0, ticket, st);
  bn_apply_launch(M, C, st, (const bf16_t*)x, (const bf16_t*)r,
                     (bf16_t*)out, (const float2*)stats, gamma, beta, M, C, relu, res_mode, (uint8_t*)nullptr,
                     (const float*)nullptr, (unsigned*)nullptr, (uint8_t*)nullptr, BnRes{});
  OPCK(hipGetLastError());
  return 0;
}

// BatchNorm forward when the per-tile column partials were produced by the GEMM epilogue (col_stats): finalize
// over `nparts` partial rows + apply.
// q / amax_prev / amax_out (optional): also write an fp8 copy of the output with delayed scaling (k_bn_apply);
// amax_out is zeroed here first.
// mask (optional, res_mode 2 + ReLU): [M C / 8] bytes, the ReLU mask for dca_ops_bn_bwd.
// out == nullptr: statistics only (a BN whose consumer applies it on the fly, BnRes).  rstats / rgamma / rbeta
// (optional, res_mode 2): r is the raw input of another training BN with these statistics, applied on the fly.
int dca_ops_bn_fwd_parts(const void* x, const void* r, void* out, float* part, int nparts, float* stats,
                         const float* gamma, const float* beta, float* rm, float* rv, long M, int C, float eps,
                         float momentum, int relu, int res_mode, void* q, const float* amax_prev, unsigned* amax_out,
                         void* mask, const float* rstats, const float* rgamma, const float* rbeta, unsigned* ticket,
                         void* stream) {
  REQUIRE(C % 8 == 0, "bn: C must be a multiple of 8");
  REQUIRE(res_mode == 0 || r != nullptr, "bn: residual missing");
  REQUIRE(!q || (amax_prev && amax_out), "bn: fp8 output needs amax_prev and amax_out");
  REQUIRE(!mask || (relu && res_mode == 2), "bn: the stored mask is for ReLU(bn + r)");
  hipStream_t st = (hipStream_t)stream;
  REQUIRE(!rstats || (res_mode == 2 && rgamma && rbeta), "bn: an on-the-fly residual BN needs res_mode 2");
  REQUIRE(out || (!q && !mask), "bn: statistics only: no fp8 copy / mask");
  if (q) OPCK(hipMemsetAsync(amax_out, 0, sizeof(unsigned), st));
  bn_fin_launch<0>(part, nparts, M, C, rm, rv, stats, eps, momentum, 0, ticket, st);
  if (out)
    bn_apply_launch(M, C, st, (const bf16_t*)x, (const bf16_t*)r,
                    (bf16_t*)out, (const float2*)stats, gamma, beta, M, C, relu, res_mode, (uint8_t*)q, amax_prev,
                    amax_out, (uint8_t*)mask, BnRes{(const float2*)rstats, rgamma, rbeta});
  OPCK(hipGetLastError());
  return 0;
}

// BatchNorm in eval mode (inference) fused with ReLU / residual: normalises with the running statistics.
// stats: [C] float2 scratch (mean, invstd).  No running-stat update.
int dca_ops_bn_eval(const void* x, const void* r, void* out, float* stats, const float* gamma, const float* beta,
                    const float* rm, const float* rv, long M, int C, float eps, int relu, int res_mode, void* stream) {
  REQUIRE(C % 8 == 0, "bn: C must be a multiple of 8");
  REQUIRE(res_mode == 0 || r != nullptr, "bn: residual missing");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_bn_eval_stats, dim3((C + 255) / 256), dim3(256), 0, st, rm, rv, (float2*)stats, C, eps);
  bn_apply_launch(M, C, st, (const bf16_t*)x, (const bf16_t*)r,
                     (bf16_t*)out, (const float2*)stats, gamma, beta, M, C, relu, res_mode, (uint8_t*)nullptr,
                     (const float*)nullptr, (unsigned*)nullptr, (uint8_t*)nullptr, BnRes{});
  OPCK(hipGetLastError());
  return 0;
}

// mask (optional): the forward's ReLU bit mask (dca_ops_bn_fwd_parts); r is then not read.
int dca_ops_bn_bwd(const void* dy, const void* x, const void* r, const float* stats, const float* gamma,
                   const float* beta, float* part, float* sums, float* dgamma, float* dbeta, void* dx, void* dr,
                   long M, int C, int relu, int res_mode, int accumulate, const void* mask, unsigned* ticket,
                   void* stream) {
  REQUIRE(C % 8 == 0, "bn: C must be a multiple of 8");
  // dr (= dz) may be omitted with the mask: the residual's consumer then reads dy and the mask itself
  REQUIRE(res_mode != 2 || mask != nullptr || (r != nullptr && dr != nullptr), "bn bwd: residual tensors missing");
  // mask: ReLU(bn + r)'s own stored mask (relu, res_mode 2), or -- a plain BN whose output is that r (ResNet
  // downsample branch: no relu, res_mode 0) -- the consumer's mask applied to the consumer's dout, passed as dy
  REQUIRE(!mask || (relu && res_mode == 2) || (!relu && res_mode == 0), "bn bwd: unsupported mask use");
  REQUIRE(res_mode != 2 || relu, "bn bwd: a residual join without ReLU is not supported");
  hipStream_t st = (hipStream_t)stream;
  const int nparts = (int)((M + BN_ROWS - 1) / BN_ROWS);
  const int mode = bn_bwd_mode(relu, res_mode, mask);
  if (C % 128 == 0)
    bn_stats_launch<16>(mode, bn_nt(M, C), dim3(C / 128, nparts), st, (const bf16_t*)dy, (const bf16_t*)x,
                        (const bf16_t*)r, (const float2*)stats, gamma, beta, (float2*)part, (int)M, C,
                        (const uint8_t*)mask);
  else
    bn_stats_launch<8>(mode, false, dim3((C + 63) / 64, nparts), st, (const bf16_t*)dy, (const bf16_t*)x,
                       (const bf16_t*)r, (const float2*)stats, gamma, beta, (float2*)part, (int)M, C,
                       (const uint8_t*)mask);
  bn_fin_launch<1>(part, nparts, M, C, dgamma, dbeta, sums, 0.f, 0.f, accumulate, ticket, st);
  if (C % 128 == 0)
    bn_bwd_apply_launch<16>(mode, bn_bwd_apply_fine(M, C), M, C, st, (const bf16_t*)dy, (const bf16_t*)x,
                            (const bf16_t*)r, (const float2*)stats, gamma, beta, (const float2*)sums, (bf16_t*)dx,
                            (bf16_t*)dr, M, C, (const uint8_t*)mask);
  else
    bn_bwd_apply_launch<8>(mode, false, M, C, st, (const bf16_t*)dy, (const bf16_t*)x, (const bf16_t*)r,
                           (const float2*)stats, gamma, beta, (const float2*)sums, (bf16_t*)dx, (bf16_t*)dr, M, C,
                           (const uint8_t*)mask);
  OPCK(hipGetLastError());
  return 0;
}

// 32-bit pool indexing when every element offset of the input and output (plus one grid stride of slack for the
// loop counter) stays below 2^31
inline bool pool_idx32(const PoolGeom& g) {
  const long in = (long)g.N * g.H * g.W * g.C, out = (long)g.N * g.Ho * g.Wo * g.C;
  return std::max(in, out) + 8192L * 256 < (1L << 31);
}

int dca_ops_maxpool_fwd(const void* x, void* y, void* arg, const PoolGeom* geom, void* stream) {
  const PoolGeom g = *geom;
  REQUIRE(g.K * g.K <= 255 && g.K > 0 && g.S > 0, "maxpool: bad window");
  if (g.K == 3 && g.S == 2 && g.P == 1 && g.H == 2 * g.Ho && g.W == 2 * g.Wo && g.C % 8 == 0 &&
      POOL_K3S2) {
    const dim3 grid(grid_for((long)g.N * g.Ho * g.Wo * g.C / 8));
    if (pool_idx32(g))
      hipLaunchKernelGGL(k_maxpool_fwd_k3s2<unsigned>, grid, dim3(256), 0, (hipStream_t)stream,
                         (const bf16_t*)x, (bf16_t*)y, (uint8_t*)arg, g);
    else
      hipLaunchKernelGGL(k_maxpool_fwd_k3s2<long>, grid, dim3(256), 0, (hipStream_t)stream,
                         (const bf16_t*)x, (bf16_t*)y, (uint8_t*)arg, g);
    OPCK(hipGetLastError());
    return 0;
  }
  const dim3 grid(grid_for((long)g.N * g.Ho * g.Wo * g.C / ((g.C & 7) == 0 ? 8 : 1)));
  if (pool_idx32(g))
    hipLaunchKernelGGL(k_maxpool_fwd<unsigned>, grid, dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)x, (bf16_t*)y, (uint8_t*)arg, g);
  else
    hipLaunchKernelGGL(k_maxpool_fwd<long>, grid, dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)x, (bf16_t*)y, (uint8_t*)arg, g);
  OPCK(hipGetLastError());
  return 0;
}

int dca_ops_maxpool_bwd(const void* dy, const void* arg, void* dx, const PoolGeom* geom, void* stream) {
  const PoolGeom g = *geom;
  if (g.K == 3 && g.S == 2 && g.P == 1 && g.H == 2 * g.Ho && g.W == 2 * g.Wo && g.C % 8 == 0 &&
      POOL_K3S2) {
    const dim3 grid(grid_for((long)g.N * g.Ho * g.Wo * g.C / 8));
    if (pool_idx32(g))
      hipLaunchKernelGGL(k_maxpool_bwd_k3s2<unsigned>, grid, dim3(256), 0, (hipStream_t)stream,
                         (const bf16_t*)dy, (const uint8_t*)arg, (bf16_t*)dx, g);
    else
      hipLaunchKernelGGL(k_maxpool_bwd_k3s2<long>, grid, dim3(256), 0, (hipStream_t)stream,
                         (const bf16_t*)dy, (const uint8_t*)arg, (bf16_t*)dx, g);
    OPCK(hipGetLastError());
    return 0;
  }
  const dim3 grid(grid_for((long)g.N * g.H * g.W * g.C / ((g.C & 7) == 0 ? 8 : 1)));
  if (pool_idx32(g))
    hipLaunchKernelGGL(k_maxpool_bwd<unsigned>, grid, dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)dy, (const uint8_t*)arg, (bf16_t*)dx, g);
  else
    hipLaunchKernelGGL(k_maxpool_bwd<long>, grid, dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)dy, (const uint8_t*)arg, (bf16_t*)dx, g);
  OPCK(hipGetLastError());
  return 0;
}

// The ResNet stem's BatchNorm + ReLU + 3x3/2/1 max pool as one pass over the conv output y [N][H][W][C] (H = 2 Ho,
// W = 2 Wo, C % 64 == 0), the BN column partials coming from the conv GEMM's epilogue (col_stats): finalize + fused
// apply-and-pool into out / arg [N][Ho][Wo][C] (k_bn_pool_fwd).  Same values as dca_ops_bn_fwd_parts followed by
// dca_ops_maxpool_fwd, without the activation in between.
inline bool bn_pool_ok(const PoolGeom& g) {
  return g.K == 3 && g.S == 2 && g.P == 1 && g.H == 2 * g.Ho && g.W == 2 * g.Wo && g.C % 64 == 0 && pool_idx32(g);
}
int dca_ops_bn_pool_fwd_parts(const void* y, float* part, int nparts, float* stats, const float* gamma,
                              const float* beta, float* rm, float* rv, float eps, float momentum, void* out, void* arg,
                              const PoolGeom* geom, unsigned* ticket, void* stream) {
  const PoolGeom g = *geom;
  REQUIRE(bn_pool_ok(g), "bn_pool: 3x3/2/1 pool with H = 2 Ho, W = 2 Wo, C % 64 == 0, 32-bit offsets");
  hipStream_t st = (hipStream_t)stream;
  const long M = (long)g.N * g.H * g.W;
  bn_fin_launch<0>(part, nparts, M, g.C, rm, rv, stats, eps, momentum, 0, ticket, st);
  hipLaunchKernelGGL(k_bn_pool_fwd<unsigned>, dim3(grid_for((long)g.N * g.Ho * g.Wo * g.C / 8)), dim3(256), 0, st,
                     (const bf16_t*)y, (bf16_t*)out, (uint8_t*)arg, g, (const float2*)stats, gamma, beta);
  OPCK(hipGetLastError());
  return 0;
}
// Its backward from the pooled gradient dp and the argmax bytes: dx = d(conv output); dgamma / dbeta written, or
// accumulated (flat gradient sinks).  part: [ceil(N Ho Wo / BNP_OPB)][C] float2 scratch, sums: [C] float2.
int dca_ops_bn_pool_bwd(const void* dp, const void* arg, const void* y, const float* stats, const float* gamma,
                        const float* beta, float* part, float* sums, float* dgamma, float* dbeta, void* dx,
                        int accumulate, const PoolGeom* geom, unsigned* ticket, void* stream) {
  const PoolGeom g = *geom;
  REQUIRE(bn_pool_ok(g), "bn_pool: 3x3/2/1 pool with H = 2 Ho, W = 2 Wo, C % 64 == 0, 32-bit offsets");
  hipStream_t st = (hipStream_t)stream;
  const long npo = (long)g.N * g.Ho * g.Wo;
  const int nparts = (int)((npo + BNP_OPB - 1) / BNP_OPB);
  hipLaunchKernelGGL(k_bn_pool_bwd_stats<unsigned>, dim3(g.C / 64, nparts), dim3(256), 0, st, (const bf16_t*)dp,
                     (const uint8_t*)arg, (const bf16_t*)y, (const float2*)stats, gamma, beta, (float2*)part, g);
  bn_fin_launch<1>(part, nparts, (long)g.N * g.H * g.W, g.C, dgamma, dbeta, sums, 0.f, 0.f, accumulate, ticket, st);
  hipLaunchKernelGGL(k_bn_pool_bwd_apply<unsigned>, dim3(grid_for(npo * g.C / 8)), dim3(256), 0, st,
                     (const bf16_t*)dp, (const uint8_t*)arg, (const bf16_t*)y, (const float2*)stats, gamma, beta,
                     (const float2*)sums, (bf16_t*)dx, g);
  OPCK(hipGetLastError());
  return 0;
}

// y: fp32 [N][C], or bf16 with out_bf16 (the fc GEMM operand directly)
int dca_ops_avgpool_fwd(const void* x, void* y, int N, int HW, int C, int out_bf16, void* stream) {
  const dim3 grid((C + 255) / 256, N);
  if (out_bf16)
    hipLaunchKernelGGL(k_avgpool_fwd<bf16_t>, grid, dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x, (bf16_t*)y,
                       N, HW, C);
  else
    hipLaunchKernelGGL(k_avgpool_fwd<float>, grid, dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x, (float*)y, N,
                       HW, C);
  OPCK(hipGetLastError());
  return 0;
}

// dy: fp32 [N][C], or bf16 with dy_bf16
int dca_ops_avgpool_bwd(const void* dy, void* dx, int N, int HW, int C, int dy_bf16, void* stream) {
  const bool v8 = C % 8 == 0 && (long)N * HW * C + 8192L * 256 * 8 < (1L << 31);
  REQUIRE(v8 || !dy_bf16, "avgpool_bwd: a bf16 dy needs C % 8 == 0");
  if (v8 && dy_bf16)
    hipLaunchKernelGGL(k_avgpool_bwd8<bf16_t>, dim3(grid_for((long)N * HW * C / 8)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)dy, (bf16_t*)dx, N, HW, C);
  else if (v8)
    hipLaunchKernelGGL(k_avgpool_bwd8<float>, dim3(grid_for((long)N * HW * C / 8)), dim3(256), 0, (hipStream_t)stream,
                       (const float*)dy, (bf16_t*)dx, N, HW, C);
  else
    hipLaunchKernelGGL(k_avgpool_bwd, dim3(grid_for((long)N * HW * C)), dim3(256), 0, (hipStream_t)stream,
                       (const float*)dy, (bf16_t*)dx, N, HW, C);
  OPCK(hipGetLastError());
  return 0;
}

// loss_mean / ticket (optional, both or neither): the batch-mean loss written in the same launch
int dca_ops_cross_entropy(const float* logits, const long* labels, float* loss, float* dlogits, int B, int K,
                          float grad_scale, float* loss_mean, unsigned* ticket, void* stream) {
  REQUIRE(B > 0 && K > 0, "cross_entropy: empty input");
  REQUIRE((loss_mean == nullptr) == (ticket == nullptr), "cross_entropy: loss_mean needs a ticket word");
  hipLaunchKernelGGL(k_cross_entropy, dim3(B), dim3(64), 0, (hipStream_t)stream, logits, labels, loss, dlogits, B, K,
                     grad_scale, loss_mean, ticket);
  OPCK(hipGetLastError());
  return 0;
}

// zero `bytes` bytes on the stream (a gradient buffer before the backward): the runtime's fill, no ATen kernel
int dca_ops_zero(void* p, long bytes, void* stream) {
  OPCK(hipMemsetAsync(p, 0, (size_t)bytes, (hipStream_t)stream));
  return 0;
}

int dca_ops_scale_dev(const float* x, const float* s, float* out, long n, void* stream) {
  hipLaunchKernelGGL(k_scale_dev, dim3(grid_for(n, 256, 2048)), dim3(256), 0, (hipStream_t)stream, x, s, out, n);
  OPCK(hipGetLastError());
  return 0;
}

int dca_ops_cast_bf16(const float* x, void* y, long n, void* stream) {
  hipLaunchKernelGGL(k_cast_bf16, dim3(grid_for(n, 256, 2048)), dim3(256), 0, (hipStream_t)stream, x, (bf16_t*)y, n);
  OPCK(hipGetLastError());
  return 0;
}

int dca_ops_gather_cols(const float* src, int S, const long* idx, int L, float* out, int rows, int accumulate,
                        void* stream) {
  REQUIRE(rows > 0 && L > 0 && (long)rows * L < (1L << 31), "gather_cols: bad shape");
  hipLaunchKernelGGL(k_gather_cols, dim3(grid_for((long)rows * L, 256, 1024)), dim3(256), 0, (hipStream_t)stream, src, S,
                     idx, L, out, rows, accumulate);
  OPCK(hipGetLastError());
  return 0;
}

// ptrs: device array of n int64 pointers
int dca_ops_add_i64(void* ptrs, int n, void* stream) {
  REQUIRE(n > 0, "add_i64: empty");
  hipLaunchKernelGGL(k_add_i64, dim3(1), dim3(64), 0, (hipStream_t)stream, (long long* const*)ptrs, n);
  OPCK(hipGetLastError());
  return 0;
}

// dy [R][N] (dy_bf16: bf16, else fp32), y: optional ReLU mask source [R][N] (y_bf16: bf16, else fp32); dyb: optional
// bf16 copy of the masked dy; db [N] fp32 column sums; part: nchunk * N floats; ticket: ceil(N / 64) zeroed device
// words.
int dca_ops_dy_prep(const void* dy, int dy_bf16, const void* y, int y_bf16, void* dyb, float* part, float* db,
                    unsigned* ticket, long R, int N, int nchunk, int accumulate, void* stream) {
  REQUIRE(R > 0 && N > 0 && nchunk > 0 && nchunk <= 65535 && R < (1L << 31), "dy_prep: bad shape");
  const int rpb = (int)((R + nchunk - 1) / nchunk);
  hipStream_t st = (hipStream_t)stream;
  const dim3 g((N + 63) / 64, nchunk), b(256);
#define DYP(TD, TY) \
  hipLaunchKernelGGL((k_dy_prep<TD, TY>), g, b, 0, st, (const TD*)dy, (const TY*)y, (bf16_t*)dyb, part, db, ticket, \
                     (int)R, N, rpb, accumulate)
  if (dy_bf16 && y_bf16) DYP(bf16_t, bf16_t);
  else if (dy_bf16) DYP(bf16_t, float);
  else if (y_bf16) DYP(float, bf16_t);
  else DYP(float, float);
#undef DYP
  OPCK(hipGetLastError());
  return 0;
}

// first: device int (1 on the first momentum step); cleared after the update.
int dca_ops_sgd(float* p, const float* g, float* buf, long n, float lr, float mu, float wd, int* first, void* stream) {
  REQUIRE(mu == 0.f || buf != nullptr, "sgd: momentum buffer missing");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_sgd, dim3(grid_for(n, 256, 2048)), dim3(256), 0, st, p, g, buf, n, lr, mu, wd, first);
  if (first) hipLaunchKernelGGL(k_clear_flag, dim3(1), dim3(1), 0, st, first);
  OPCK(hipGetLastError());
  return 0;
}

// x (fp32 if is_f32 else bf16, n elements) -> q fp8 e4m3; amax_bits: device uint, zeroed here first.
int dca_ops_quant_fp8(const void* x, int is_f32, long n, void* q, unsigned* amax_bits, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  OPCK(hipMemsetAsync(amax_bits, 0, sizeof(unsigned), st));
  const int grid = grid_for(n, 256, 1024);
  if (is_f32) {
    hipLaunchKernelGGL(k_amax<float>, dim3(grid), dim3(256), 0, st, (const float*)x, n, amax_bits);
    hipLaunchKernelGGL(k_quant_fp8<float>, dim3(grid_for(n / 4 + 1)), dim3(256), 0, st, (const float*)x,
                       (uint8_t*)q, n, amax_bits);
  } else {
    hipLaunchKernelGGL(k_amax<bf16_t>, dim3(grid), dim3(256), 0, st, (const bf16_t*)x, n, amax_bits);
    hipLaunchKernelGGL(k_quant_fp8<bf16_t>, dim3(grid_for(n / 4 + 1)), dim3(256), 0, st, (const bf16_t*)x,
                       (uint8_t*)q, n, amax_bits);
  }
  OPCK(hipGetLastError());
  return 0;
}

int dca_ops_fp8_alpha(const unsigned* amax_a, const unsigned* amax_b, float extra, float* alpha, void* stream) {
  hipLaunchKernelGGL(k_fp8_alpha, dim3(1), dim3(1), 0, (hipStream_t)stream, amax_a, amax_b, extra, alpha);
  OPCK(hipGetLastError());
  return 0;
}

// descs: device array of nd PackDesc (ops/functional.py WeightPack); amax: n_amax device words zeroed first.
int dca_ops_pack_weights(const void* descs, int nd, int blocks_per_layer, unsigned* amax, int n_amax, void* stream) {
  REQUIRE(nd > 0 && blocks_per_layer > 0, "pack_weights: empty");
  REQUIRE(blocks_per_layer <= 4096, "pack_weights: at most 4096 blocks per layer (32-bit grid-stride indices)");
  hipStream_t st = (hipStream_t)stream;
  if (n_amax > 0) OPCK(hipMemsetAsync(amax, 0, sizeof(unsigned) * n_amax, st));
  const dim3 grid(blocks_per_layer, nd);
  hipLaunchKernelGGL(k_pack_weights, grid, dim3(256), 0, st, (const PackDesc*)descs);
  if (n_amax > 0) hipLaunchKernelGGL(k_pack_fp8, grid, dim3(256), 0, st, (const PackDesc*)descs);
  OPCK(hipGetLastError());
  return 0;
}

int dca_ops_pack_desc_size() { return (int)sizeof(PackDesc); }

int dca_ops_nchw_to_nhwc8(const float* x, void* y, int N, int C, long HW, void* stream) {
  REQUIRE(C > 0 && C <= 8, "nchw_to_nhwc8: 1..8 channels");
  hipLaunchKernelGGL(k_nchw_to_nhwc8, dim3(grid_for((long)N * HW)), dim3(256), 0, (hipStream_t)stream, x, (bf16_t*)y,
                     N, C, HW);
  OPCK(hipGetLastError());
  return 0;
}

int dca_ops_nchw_to_s2d16(const float* x, void* y, int N, int C, int H, int W, int Hs, int Ws, int P, void* stream) {
  REQUIRE(C > 0 && C <= 4 && P >= 0 && Hs > 0 && Ws > 0, "nchw_to_s2d16: 1..4 channels");
  hipLaunchKernelGGL(k_nchw_to_s2d16, dim3(grid_for((long)N * Hs * Ws)), dim3(256), 0, (hipStream_t)stream, x,
                     (bf16_t*)y, N, C, H, W, Hs, Ws, P);
  OPCK(hipGetLastError());
  return 0;
}

int dca_ops_pack_gather(const void* descs, int nd, int blocks, void* stream) {
  REQUIRE(nd > 0 && blocks > 0, "pack_gather: empty");
  hipLaunchKernelGGL(k_pack_gather, dim3(blocks, nd), dim3(256), 0, (hipStream_t)stream, (const GatherDesc*)descs);
  OPCK(hipGetLastError());
  return 0;
}

int dca_ops_gather_desc_size() { return (int)sizeof(GatherDesc); }

}  // extern "C"
