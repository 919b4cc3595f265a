// Persistent NetResDeep training step for CDNA4 (gfx950 / MI355X), bf16 MFMA, one workgroup per image.
//
// Why: the multi-kernel engine (netresdeep_kernels.hip) pays a dependent-kernel boundary (~1.5-1.9 us, measured)
// plus a cold reload of activations / weights / BN partials written by other XCDs (~3-5 us, measured) at each of
// its 23 seams.  Here ONE launch runs the whole trunk of a step:
//   stem -> 10 forward blocks -> head (fc1/fc2/cross-entropy fwd+bwd) -> 10 backward blocks -> stem backward
// Each workgroup (1024 threads = 16 waves, one wave per image row) owns one image: its activations stay in
// registers in the MFMA C-fragment layout, the conv weights stay in LDS, and the only cross-workgroup traffic is
// the batch-norm statistics (64 floats per image per block), exchanged in-kernel with an all-gather of tagged
// 8-byte granules (data-as-flag: relaxed agent-scope stores, L1-bypassing sc1 buffer loads, parity
// double-buffered, every spin bounded) -- ~1.4 us per exchange measured (profiles/xchg_calibration.log).
// The trunk weight gradient is accumulated in registers across all 10 applications of the shared conv and
// written once per image; k_pk_reduce then reduces slabs, computes fc grads, and applies SGD.
//
// Element ownership (C layout of v_mfma_f32_16x16x32_bf16): thread (wave w, lane l = 16q + c) owns
//   pixel (row w, col 4q+i), channel 16h + c   for h in {0,1}, i in {0..3}   (8 values)
//
// Reference semantics: model/resnet.py:5-37 (shared ResBlock, skip after ReLU), main.py:27-39 (SGD, CE mean),
// BatchNorm2d training statistics and 10 sequential running-stat updates per forward.

namespace dca {
namespace pk {

constexpr int NTP = 1024;
constexpr int NWV = 16;
constexpr int KSW = 4;                    // granule loads per lane per sweep pass  (batch <= 64)
constexpr unsigned SPIN_LIMIT = 1u << 18; // bounded spin: a missing peer sets an error flag, never hangs
constexpr int ROUNDS = 20;                // exchanges per step (10 forward + 10 backward)

struct PkArgs {
  unsigned long long* gran;  // [2][64][64] granules
  int* epoch;                // device scalar, advanced by k_pk_reduce after every step
  unsigned* err;             // bit r: exchange round r timed out
  float* tslab;              // [B][9216] trunk wgrad (fragment order)
  float* bng;                // [64] dgamma | dbeta  (written by workgroup 0)
  int* ids;                  // [64] dataset ids of the current batch (written by the previous step's reduce)
  uint8_t* simg;             // [2][64][3072] batch images staged contiguously (parity = epoch & 1); each step
  int* slab;                 // [2][64]       stages the NEXT batch into the other parity, see k_pk_step
  unsigned long long* xcc;   // [64] granules: XCD id of each image workgroup (published with round 0)
  int xpack;                 // 1: grid = 8 x batch, only blocks b % 8 == 0 work (one XCD under round-robin dispatch)
  int phase;                 // 0: whole step; split mode: 1 = stem + forward + head, 2 = backward + stem backward
  float* gh;                 // [64][8192] split mode: dL/dx10 of each image (tiled), handed from phase 1 to 2
  int debug;                 // also store DY / G for the numerical diagnostics
};

constexpr int cmax(int a, int b) { return a > b ? a : b; }

// Image / grid size of the persistent launch.  With xpack the grid is 8 x batch and only blocks b % 8 == 0 run:
// blocks b and b + 8 share an XCD under the (observed, never relied on for correctness) round-robin dispatch,
// so all image workgroups sit behind one L2 and the BN exchange can use L2-resident stores (see xchg_publish).
__device__ __forceinline__ int pk_img(int xpack) { return xpack ? (int)(blockIdx.x >> 3) : (int)blockIdx.x; }
__device__ __forceinline__ int pk_grid(int xpack) { return xpack ? (int)(gridDim.x >> 3) : (int)gridDim.x; }
__device__ __forceinline__ unsigned xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
  return v;
}

// diagnostic stamps (DCA_STAMPS builds): global stamp index s -> slot 24 + s/8, entry s%8
#define PK_STAMP(cx, s) DCA_STAMP(cx, 24 + (s) / 8, pk_img(pa.xpack), (s) % 8)

constexpr int P_KSHIFT = 906;  // misc offset of the [10][32] BN shift table (last step's batch means)
constexpr int P_LABEL = 1240; // misc offset of this image's label
constexpr int P_FAST = 1241;  // misc offset of the exchange-protocol flag (1: one XCD, L2-resident publishes)

struct Plan {
  static constexpr int RB = 80;                        // bf16 record = 32 channels (64 B) + 16 B pad
  static constexpr int O_CRED = 0;                     // [2][16][64] f32 combine scratch
  static constexpr int O_STAT = 8192;                  // [10][64] f32: mean[32] | invstd[32]
  static constexpr int O_MISC = O_STAT + 2560;         // [1280] f32 (layout: see k_pk_step)
  static constexpr int O_U = O_MISC + 5120;            // phase union
  // forward
  static constexpr int U_WT = 0;                       // 288 weight records
  static constexpr int U_XR = 288 * RB;                // 18 x 18 conv-input records (zero halo)
  static constexpr int U_XR_END = U_XR + 324 * RB;
  // stem (start of the step)
  static constexpr int U_XIN = U_XR_END;               // [3][34][34] f32 normalised input
  static constexpr int U_SW = U_XIN + 13872;           // [32][32] bf16 stem weight
  static constexpr int U_SB = U_SW + 2048;             // [32] f32 stem bias
  static constexpr int X0S = 36;                       // pixel stride (f32) of the pooled stem output
  static constexpr int U_X0 = U_SB + 128;              // [256][X0S] f32 pooled stem output
  static constexpr int U_SCODE = U_X0 + 256 * X0S * 4; // [256][32] u8 stem pool argmax (re-laid out for global)
  static constexpr int STEM_END = U_SCODE + 8192;
  // head
  static constexpr int U_X10 = 0;                      // [256][32] f32
  static constexpr int U_P = 32768;                    // [2048] f32  (NCHW flatten c*64 + ph*8 + pw)
  static constexpr int U_CODE = U_P + 8192;            // [64][32] u8 pool argmax
  static constexpr int U_DP = U_CODE + 2048;           // [2048] f32
  static constexpr int U_HP = U_DP + 8192;             // [16][32] f32 per-wave fc1 partials
  static constexpr int U_HV = U_HP + 2048;             // h[32] dh[32] logits[16] dl[16]
  static constexpr int U_DPP = U_HV + 384;             // [8 waves max][2048] f32 per-wave dp partials
  static constexpr int HEAD_END = U_DPP + 8 * 2048 * 4;
  // backward
  static constexpr int DYT_S = 256 + 8;
  static constexpr int U_DYT = U_XR_END;               // [32][DYT_S] bf16  dy, pixel-contiguous
  static constexpr int XT_S = 18 * 16 + 8;
  static constexpr int U_XT = U_DYT + 32 * DYT_S * 2;  // [3 kw][32][XT_S] bf16 shifted x copies
  static constexpr int BWD_END = U_XT + 3 * 32 * XT_S * 2;
  // stem backward
  static constexpr int DSP = 1024 + 8;
  static constexpr int U_DST = 0;                      // [32][DSP] bf16 d(stem conv output), pixel-contiguous
  static constexpr int XS_S = 40;                      // row stride (bf16) of the shifted input copies
  static constexpr int U_XS = 32 * DSP * 2;            // [3 kw][3 ci][34 rows][XS_S] bf16: col c holds x[c + kw - 1]
  static constexpr int U_SRED = U_XS + 9 * 34 * XS_S * 2;  // [8 waves][64 lanes][4] f32 stem-wgrad partials
  static constexpr int SBWD_END = U_SRED + 8192;
  static constexpr int UNION = cmax(cmax(STEM_END, HEAD_END), cmax(BWD_END, SBWD_END));
  static constexpr int TOTAL = O_U + UNION;
};
static_assert(Plan::TOTAL <= 160 * 1024, "LDS budget");
static_assert(Plan::U_XIN % 16 == 0 && Plan::U_SW % 16 == 0 && Plan::U_X0 % 16 == 0 && Plan::U_XT % 16 == 0 &&
                  Plan::U_XS % 16 == 0 && Plan::O_U % 16 == 0 && Plan::U_SRED % 16 == 0,
              "16-byte aligned carve");

// Workgroup barrier for LDS-only hand-offs.  __syncthreads() also waits for every outstanding global load and
// store of the wave (vmcnt(0)); here waves share data only through LDS, so global prefetches and write-backs
// stay in flight across the barrier.  Cross-thread hand-offs through GLOBAL memory use __syncthreads().
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Force a loaded value to be materialised here.  hipcc otherwise sinks a load whose only use is a guarded
// LDS store into the guarded branch, where it is waited for on its own: N guarded loads become N serial
// memory round trips.  Pinning after all loads of a phase keeps them in flight together.
__device__ __forceinline__ void pin(float& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void pin(unsigned& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void pin(int& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void pin(uint4& x) { asm volatile("" : "+v"(x.x), "+v"(x.y), "+v"(x.z), "+v"(x.w)); }

// Workgroup geometry: NW waves, each owning RPW consecutive image rows.
template <int NW>
struct Geo {
  static constexpr int NT = 64 * NW;              // threads per workgroup
  static constexpr int RPW = 16 / NW;             // image rows per wave
  static constexpr int KSW = (64 + NW - 1) / NW;  // granule loads per lane per sweep pass (batch <= 64)
  static constexpr int NNT = (18 + NW - 1) / NW;  // wgrad tile columns (ci half x tap) per wave; both co halves
  static constexpr int KPT = 2048 / NT;           // fc1 input features per thread
  static constexpr int SBC = 16 / NW;             // stem-wgrad (tile, row-quarter) combos per wave
  static constexpr int IMW = (768 + NT - 1) / NT; // uint8 image words per thread
};

// offset of the C-layout element (row, h, i) of lane (q, c) inside an NHWC [16][16][32] image (LDS staging)
__device__ __forceinline__ int el(int row, int q, int c, int h, int i) {
  return ((row * 16 + 4 * q + i) << 5) + 16 * h + c;
}
// Global activations (X, Y, DY, G, SCODE) use the fragment-tiled layout [row][h][lane][i]: a thread's four
// values of (row, h) are 16 contiguous bytes, so every global access is one dwordx4 per (row, h) and one wave
// instruction covers a whole 1 KiB line run.  Element (row, col = 4q + i, ch = 16h + c) lives at
// tl(row, h, 16q + c) + i.  (runtime/engine.py: NetResDeepEngine.activations() converts to NHWC.)
__device__ __forceinline__ int tl(int row, int h, int lane) { return row * 512 + h * 256 + lane * 4; }
__device__ __forceinline__ void st4v(float* p, const float (&v)[4]) { *(f32x4*)p = f32x4{v[0], v[1], v[2], v[3]}; }
// X (block inputs) is stored as bf16 in the same tiled order: the backward only uses it as a bf16 MFMA operand
__device__ __forceinline__ void stx(float* xbase, int row, int h, int lane, const float (&v)[4]) {
  *(uint2*)((unsigned short*)xbase + tl(row, h, lane)) =
      uint2{(unsigned)bfbits(v[0]) | ((unsigned)bfbits(v[1]) << 16), (unsigned)bfbits(v[2]) | ((unsigned)bfbits(v[3]) << 16)};
}
__device__ __forceinline__ uint2 ldx(const float* xbase, int row, int h, int lane) {
  return *(const uint2*)((const unsigned short*)xbase + tl(row, h, lane));
}
__device__ __forceinline__ void ld4v(const float* p, float (&v)[4]) {
  const f32x4 u = *(const f32x4*)p;
  v[0] = u[0]; v[1] = u[1]; v[2] = u[2]; v[3] = u[3];
}

// per-image channel sums of two per-thread C-layout partials (a0: channel c, a1: channel 16+c; same for b);
// results oa[32], ob[32] in LDS, valid after the call.  Two LDS barriers.
template <int NW>
__device__ __forceinline__ void img_csum2(float a0, float a1, float b0, float b1, float* cred, float* oa, float* ob) {
  const int t = threadIdx.x, w = t >> 6, lane = t & 63, c = lane & 15;
  a0 += __shfl_xor(a0, 16);
  a0 += __shfl_xor(a0, 32);
  a1 += __shfl_xor(a1, 16);
  a1 += __shfl_xor(a1, 32);
  b0 += __shfl_xor(b0, 16);
  b0 += __shfl_xor(b0, 32);
  b1 += __shfl_xor(b1, 16);
  b1 += __shfl_xor(b1, 32);
  if (lane < 16) {
    cred[w * 32 + c] = a0;
    cred[w * 32 + 16 + c] = a1;
    cred[512 + w * 32 + c] = b0;
    cred[512 + w * 32 + 16 + c] = b1;
  }
  lds_barrier();
  if (t < 64) {
    const int ch = t & 31, off = t < 32 ? 0 : 512;
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NW; ++k) s += cred[off + k * 32 + ch];
    (t < 32 ? oa : ob)[ch] = s;
  }
  lds_barrier();
}

// one sweep pass over the granules of a round: KS loads per lane, all issued before any is waited for (a
// guarded load per slot would be compiled into KS serial round trips).  Slots past the grid read a valid granule
// (clamped index) and are then replaced by a neutral (0, tag) pair.  Split in issue / evaluate halves so a pass
// can be issued early and evaluated after independent work.
template <int NW, int KS>
__device__ __forceinline__ void sweep_load(const __amdgpu_buffer_rsrc_t rs, int w, int lane, int G, unsigned (&lo)[KS],
                                           unsigned (&hi)[KS]) {
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) {
    const int k = w + NW * kk, kc = k < G ? k : G - 1;
    const auto x = __builtin_amdgcn_raw_buffer_load_b64(rs, (kc * 64 + lane) * 8, 0, 16);  // sc1
    lo[kk] = x[0];
    hi[kk] = x[1];
  }
}
template <int NW, int KS>
__device__ __forceinline__ bool sweep_eval(int w, int G, unsigned tag, const unsigned (&lo)[KS], const unsigned (&hi)[KS],
                                           float& s1) {
  bool ok = true;
  s1 = 0.f;
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) {
    const bool valid = w + NW * kk < G;
    ok &= !valid || hi[kk] == tag;
    s1 += valid ? __uint_as_float(lo[kk]) : 0.f;
  }
  return ok;
}
template <int NW, int KS>
__device__ __forceinline__ bool sweep(const __amdgpu_buffer_rsrc_t rs, int w, int lane, int G, unsigned tag,
                                      float& s1) {
  unsigned lo[KS], hi[KS];
  sweep_load<NW, KS>(rs, w, lane, G, lo, hi);
  return sweep_eval<NW, KS>(w, G, tag, lo, hi, s1);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t gran_rsrc(const PkArgs& pa, int round) {
  return __builtin_amdgcn_make_buffer_rsrc(pa.gran + (size_t)(round & 1) * 64 * 64, (short)0, 64 * 64 * 8, 0x00020000);
}

// Per-image channel sums of per-thread C-layout partials, delivered straight to the publishing threads: on
// return thread t < 64 holds  t < 32: sum of a (channel t),  t >= 32: sum of b (channel t - 32)
// (a0/b0: channel c, a1/b1: channel 16 + c).  One LDS barrier.
template <int NW>
__device__ __forceinline__ float img_csum_pub(float a0, float a1, float b0, float b1, float* cred) {
  const int t = threadIdx.x, w = t >> 6, lane = t & 63, c = lane & 15;
  a0 += __shfl_xor(a0, 16);
  a0 += __shfl_xor(a0, 32);
  a1 += __shfl_xor(a1, 16);
  a1 += __shfl_xor(a1, 32);
  b0 += __shfl_xor(b0, 16);
  b0 += __shfl_xor(b0, 32);
  b1 += __shfl_xor(b1, 16);
  b1 += __shfl_xor(b1, 32);
  float* r = cred + 1024;  // [NW][64], disjoint from the sweep's cred[0 .. NW*64)
  if (lane < 16) {
    r[w * 64 + c] = a0;
    r[w * 64 + 16 + c] = a1;
    r[w * 64 + 32 + c] = b0;
    r[w * 64 + 48 + c] = b1;
  }
  lds_barrier();
  float v = 0.f;
  if (t < 64) {
#pragma unroll
    for (int k = 0; k < NW; ++k) v += r[k * 64 + t];
  }
  return v;
}

// In-kernel all-gather + sum, in two halves so that independent work can run between them:
//   xchg_publish: thread t < 64 of every workgroup contributes `v` to round `round`;
//   xchg_wait:    on return thread t < 64 of every workgroup holds the sum of slot t over all workgroups.
// One LDS barrier (the cross-wave combine).  The sweep is split over the waves (wave w reads workgroups
// w, w + NW, ...).
// fast: every image workgroup was found on ONE XCD (checked with round 0), so a plain store -- which stays in
// that XCD's L2, where the sc1 polls of the other workgroups read -- is enough; otherwise a write-through (sc1)
// agent-scope store.
__device__ __forceinline__ void xchg_publish(const PkArgs& pa, int epoch, int round, float v, bool fast) {
  const int t = threadIdx.x;
  const unsigned tag = (unsigned)(epoch * 64 + round + 1);
  unsigned long long* dst = pa.gran + (size_t)(round & 1) * 64 * 64 + pk_img(pa.xpack) * 64 + t;
  const unsigned long long g = ((unsigned long long)tag << 32) | __float_as_uint(v);
  if (t < 64) {
    if (fast) *(volatile unsigned long long*)dst = g;
    else __hip_atomic_store(dst, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (round == 0 && t == 64)  // this workgroup's XCD, for the fast-path decision
    __hip_atomic_store(pa.xcc + pk_img(pa.xpack), ((unsigned long long)tag << 32) | xcc_id(), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
// After round 0: 1 if every image workgroup reported the same XCD (identical answer in every workgroup).
// Wave 0 only; bounded spin like the exchange.
__device__ __forceinline__ int xcc_all_same(const PkArgs& pa, int epoch) {
  const int lane = threadIdx.x & 63, G = pk_grid(pa.xpack);
  const unsigned tag = (unsigned)(epoch * 64 + 1);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(pa.xcc, (short)0, 64 * 8, 0x00020000);
  unsigned id = 0;
  for (unsigned spins = 0;; ++spins) {
    asm volatile("" ::: "memory");
    const auto x = __builtin_amdgcn_raw_buffer_load_b64(rs, (lane < G ? lane : 0) * 8, 0, 16);  // sc1
    id = x[0];
    if (__all(lane >= G || x[1] == tag)) break;
    if (spins >= SPIN_LIMIT) {
      if (lane == 0) atomicOr(pa.err, 1u << 31);
      return 0;
    }
  }
  const unsigned id0 = __builtin_amdgcn_readfirstlane(id);
  return __all(lane >= G || id == id0) ? 1 : 0;
}
// Early pass for xchg_wait (batch <= 32): issue it, do independent work, then hand it to xchg_wait.
template <int NW>
struct EarlyPass {
  static constexpr int KS = (32 + NW - 1) / NW;
  unsigned lo[KS], hi[KS];
};
template <int NW>
__device__ __forceinline__ void xchg_early(const PkArgs& pa, int round, EarlyPass<NW>& ep) {
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int G = pk_grid(pa.xpack);
  if (G <= 32) sweep_load<NW, EarlyPass<NW>::KS>(gran_rsrc(pa, round), w, threadIdx.x & 63, G, ep.lo, ep.hi);
}
template <int NW>
__device__ float xchg_wait(const PkArgs& pa, int epoch, int round, float* cred, const EarlyPass<NW>* ep = nullptr) {
  constexpr int KSW = Geo<NW>::KSW, KSH = (32 + NW - 1) / NW;
  const int t = threadIdx.x, lane = t & 63, G = pk_grid(pa.xpack);
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);  // wave-uniform -> scalar branches in the sweep
  const unsigned tag = (unsigned)(epoch * 64 + round + 1);
  const __amdgpu_buffer_rsrc_t rs = gran_rsrc(pa, round);
  float s1 = 0.f;
  bool done = false;
  if (ep != nullptr && G <= 32) done = __all(sweep_eval<NW, KSH>(w, G, tag, ep->lo, ep->hi, s1));
  for (unsigned spins = 0; !done; ++spins) {
    asm volatile("" ::: "memory");  // the granule loads are re-issued every pass (no hoisting out of the spin)
    const bool ok = G <= 32 ? sweep<NW, KSH>(rs, w, lane, G, tag, s1) : sweep<NW, KSW>(rs, w, lane, G, tag, s1);
    if (__all(ok)) break;
    if (spins >= SPIN_LIMIT) {
      if (lane == 0) atomicOr(pa.err, 1u << (round & 31));
      break;
    }
  }
  cred[w * 64 + lane] = s1;
  lds_barrier();
  float a = 0.f;
  if (t < 64) {
#pragma unroll
    for (int k = 0; k < NW; ++k) a += cred[k * 64 + t];
  }
  return a;
}
template <int NW>
__device__ __forceinline__ float xchg(const PkArgs& pa, int epoch, int round, float v, float* cred, bool fast) {
  xchg_publish(pa, epoch, round, v, fast);
  return xchg_wait<NW>(pa, epoch, round, cred);
}

// Records are 80 bytes (32 bf16 channels + 16 B pad, which also staggers the banks of neighbouring
// records), so every tap is the per-lane base address plus a compile-time immediate offset.
__device__ __forceinline__ void st1r(char* xr, int rec, int ch, float v) {
  *(unsigned short*)(xr + rec * Plan::RB + ch * 2) = bfbits(v);
}
// whole-image 3x3 conv on MFMA: rows r0 .. r0+RPW-1, both channel halves.  xr: 18x18 records, wt: 288 records.
template <int RPW>
__device__ __forceinline__ void conv_img(const char* xr, const char* wt, f32x4 (&acc)[RPW][2], int r0, int lane) {
  const int c = lane & 15, q = lane >> 4;
  const char* abase = xr + (r0 * 18 + c) * Plan::RB + q * 16;
  const char* bbase = wt + c * Plan::RB + q * 16;
#pragma unroll
  for (int rr = 0; rr < RPW; ++rr) {
    acc[rr][0] = z4();
    acc[rr][1] = z4();
  }
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int kh = tap / 3, kw = tap % 3;
    const bf16x8 b0 = *(const bf16x8*)(bbase + (tap * 32) * Plan::RB);
    const bf16x8 b1 = *(const bf16x8*)(bbase + (tap * 32 + 16) * Plan::RB);
#pragma unroll
    for (int rr = 0; rr < RPW; ++rr) {
      const bf16x8 a = *(const bf16x8*)(abase + ((rr + kh) * 18 + kw) * Plan::RB);
      acc[rr][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b0, acc[rr][0], 0, 0, 0);
      acc[rr][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b1, acc[rr][1], 0, 0, 0);
    }
  }
}

// forward BN statistics of y (C layout) for block `blk`: one pass of shifted sums S1 = sum(y - K),
// S2 = sum((y - K)^2) per image, all-gathered; K (kshift) is this block's batch mean from the previous step (0 at
// the first), identical in every workgroup, so the shifted sums combine exactly and the E[d^2] - E[d]^2
// cancellation is negligible.  Finalise: scale/shift -> misc[192..256), (mean, invstd) -> stat[blk]; workgroup 0
// updates the running stats and STATS.  Ends with a barrier.
template <int NW>
__device__ void bn_fwd_stats(const Ctx& cx, const PkArgs& pa, int epoch, int blk,
                             const float (&y)[Geo<NW>::RPW][2][4], float* cred, float* misc, float* stat) {
  constexpr int RPW = Geo<NW>::RPW;
  const int t = threadIdx.x, lane = t & 63, c = lane & 15;
  const float* kshift = misc + P_KSHIFT;
  const float K0 = kshift[blk * 32 + c], K1 = kshift[blk * 32 + 16 + c];
  float a0 = 0.f, a1 = 0.f, b0 = 0.f, b1 = 0.f;
#pragma unroll
  for (int rr = 0; rr < RPW; ++rr)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float d0 = y[rr][0][i] - K0, d1 = y[rr][1][i] - K1;
      a0 += d0;
      a1 += d1;
      b0 += d0 * d0;
      b1 += d1 * d1;
    }
  const float v = img_csum_pub<NW>(a0, a1, b0, b1, cred);
  if (blk == 5) PK_STAMP(cx, 25);
  const float tot = xchg<NW>(pa, epoch, blk, v, cred, blk > 0 && misc[P_FAST] != 0.f);
  if (blk == 5) PK_STAMP(cx, 26);
  if (blk == 0 && threadIdx.x < 64) {  // decide the exchange protocol of rounds 1.. (same answer everywhere)
    const int same = xcc_all_same(pa, epoch);
    if (threadIdx.x == 0) misc[P_FAST] = same ? 1.f : 0.f;  // read after the barrier at the end of this function
  }
  const float sq = __shfl(tot, (lane & 31) + 32);  // wave 0: lane t < 32 also gets slot 32 + t
  if (t < 32) {
    const float N = (float)pk_grid(pa.xpack) * 256.f;
    const float dm = tot / N;
    const float mean = kshift[blk * 32 + t] + dm;
    const float var = fmaxf(sq / N - dm * dm, 0.f);
    const float invstd = rsqrtf(var + cx.bn_eps);
    const float gam = misc[320 + t], bet = misc[352 + t];
    misc[192 + t] = gam * invstd;
    misc[224 + t] = bet - mean * gam * invstd;
    stat[blk * 64 + t] = mean;
    stat[blk * 64 + 32 + t] = invstd;
    if (pk_img(pa.xpack) == 0) {  // running stats live in LDS (misc[448..512)) for the whole forward
      cx.STATS[blk * 32 + t] = make_float2(mean, invstd);
      const float unb = var * N / (N - 1.f), mo = cx.bn_mom;
      misc[448 + t] = misc[448 + t] * (1.f - mo) + mean * mo;
      misc[480 + t] = misc[480 + t] * (1.f - mo) + unb * mo;
    }
  }
  lds_barrier();
}

// wgrad of the shared conv for one application (dyT / xT staged in LDS), accumulated in registers.  Wave w
// owns tile columns nt = w, w + NW, ... (ci half x tap) for BOTH co halves: per K step the two dy fragments are
// read once and each x fragment feeds two MFMAs.
template <int NW>
__device__ __forceinline__ void wgrad_acc(const unsigned short* dyT, const unsigned short* xT,
                                          f32x4 (&wacc)[Geo<NW>::NNT][2], int w, int lane) {
  const int c = lane & 15, q = lane >> 4;
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int row = 2 * s + (q >> 1), c0 = 8 * (q & 1);
    const bf16x8 a0 = *(const bf16x8*)(dyT + c * Plan::DYT_S + row * 16 + c0);
    const bf16x8 a1 = *(const bf16x8*)(dyT + (16 + c) * Plan::DYT_S + row * 16 + c0);
#pragma unroll
    for (int j = 0; j < Geo<NW>::NNT; ++j) {
      const int nt = w + NW * j;
      if (nt < 18) {
        const int tap = nt >> 1, cih = nt & 1, kh = tap / 3, kw = tap % 3;
        const bf16x8 b = *(const bf16x8*)(xT + (kw * 32 + 16 * cih + c) * Plan::XT_S + (row + kh) * 16 + c0);
        wacc[j][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b, wacc[j][0], 0, 0, 0);
        wacc[j][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b, wacc[j][1], 0, 0, 0);
      }
    }
  }
}

template <int NW>
__device__ __forceinline__ void zero_xr_halo(char* xr) {
  // rows 0 and 17 (18 records each) + columns 0 and 17 of rows 1..16 -> 68 records x 4 chunks
  for (int idx = threadIdx.x; idx < 68 * 4; idx += 64 * NW) {
    const int r = idx >> 2, ch = idx & 3;
    const int rec = r < 18 ? r : (r < 36 ? 17 * 18 + (r - 18) : ((r - 36) / 2 + 1) * 18 + ((r - 36) & 1) * 17);
    *(uint4*)(xr + rec * Plan::RB + ch * 16) = uint4{0u, 0u, 0u, 0u};
  }
}
// stage_wt split in a load half and a store half (three named registers, not an array: a uint4 array that
// lives across a loop is demoted to scratch by the compiler).  512 threads x 3 chunks >= 1152.
__device__ __forceinline__ void stage_wt_load3(uint4& v0, uint4& v1, uint4& v2, const void* src) {
  const uint4* s = (const uint4*)src;
  const int i0 = threadIdx.x, i2 = i0 + 1024;
  v0 = s[i0];
  v1 = s[i0 + 512];
  v2 = s[i2 < 1152 ? i2 : 1151];
}
__device__ __forceinline__ void stage_wt_store3(char* wt, const uint4& v0, const uint4& v1, const uint4& v2) {
  const int i0 = threadIdx.x, i1 = i0 + 512, i2 = i0 + 1024;
  *(uint4*)(wt + (i0 >> 2) * Plan::RB + (i0 & 3) * 16) = v0;
  *(uint4*)(wt + (i1 >> 2) * Plan::RB + (i1 & 3) * 16) = v1;
  if (i2 < 1152) *(uint4*)(wt + (i2 >> 2) * Plan::RB + (i2 & 3) * 16) = v2;
}
template <int NW>
__device__ __forceinline__ void stage_wt(char* wt, const void* src) {
  constexpr int M = (1152 + 64 * NW - 1) / (64 * NW);
  const uint4* s = (const uint4*)src;
  uint4 v[M];
#pragma unroll
  for (int m = 0; m < M; ++m) {  // unconditional (clamped) loads: all in flight together, no scratch
    const int idx = threadIdx.x + 64 * NW * m;
    v[m] = s[idx < 1152 ? idx : 1151];
  }
#pragma unroll
  for (int m = 0; m < M; ++m) pin(v[m]);
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const int idx = threadIdx.x + 64 * NW * m;
    if (idx < 1152) *(uint4*)(wt + (idx >> 2) * Plan::RB + (idx & 3) * 16) = v[m];
  }
}
// stage_input in two halves, so the global loads can be issued long before the LDS region is free
template <int NW>
__device__ __forceinline__ void stage_input_load(unsigned (&wd)[Geo<NW>::IMW], const uint8_t* img) {
  constexpr int NTH = 64 * NW;
#pragma unroll
  for (int m = 0; m < Geo<NW>::IMW; ++m) {
    const int idx = threadIdx.x + NTH * m;
    wd[m] = ((const unsigned*)img)[idx < 768 ? idx : 767];
  }
}
template <int NW>
__device__ __forceinline__ void stage_input_store(float* xin, const unsigned (&wd)[Geo<NW>::IMW]) {
  constexpr int NTH = 64 * NW;
  const int t = threadIdx.x;
  for (int idx = t; idx < 3 * 34 * 34; idx += NTH) {
    const int rem = idx % (34 * 34), r = rem / 34, cc = rem % 34;
    if (r == 0 || r == 33 || cc == 0 || cc == 33) xin[idx] = 0.f;
  }
#pragma unroll
  for (int m = 0; m < Geo<NW>::IMW; ++m) {
    const int idx = t + NTH * m;
    if (idx < 768) {
      const int ch = idx >> 8, y = (idx >> 3) & 31, x0 = 4 * (idx & 7);
      float* dst = xin + ch * 34 * 34 + (y + 1) * 34 + 1 + x0;
#pragma unroll
      for (int b = 0; b < 4; ++b) dst[b] = norm_px((wd[m] >> (8 * b)) & 255u, ch);
    }
  }
}
// normalised input image [3][34][34] f32 (zero border) from the uint8 CHW image
template <int NW>
__device__ __forceinline__ void stage_input(float* xin, const uint8_t* img) {
  constexpr int NTH = 64 * NW, M = (768 + NTH - 1) / NTH;
  const int t = threadIdx.x;
  unsigned wd[M];
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const int idx = t + NTH * m;
    wd[m] = ((const unsigned*)img)[idx < 768 ? idx : 767];
  }
#pragma unroll
  for (int m = 0; m < M; ++m) pin(wd[m]);
  for (int idx = t; idx < 3 * 34 * 34; idx += NTH) {
    const int rem = idx % (34 * 34), r = rem / 34, cc = rem % 34;
    if (r == 0 || r == 33 || cc == 0 || cc == 33) xin[idx] = 0.f;
  }
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const int idx = t + NTH * m;
    if (idx < 768) {
      const int ch = idx >> 8, y = (idx >> 3) & 31, x0 = 4 * (idx & 7);
      float* dst = xin + ch * 34 * 34 + (y + 1) * 34 + 1 + x0;
#pragma unroll
      for (int b = 0; b < 4; ++b) dst[b] = norm_px((wd[m] >> (8 * b)) & 255u, ch);
    }
  }
}

// ============================================================================================================
template <int NW>
__global__ void __launch_bounds__(64 * NW) k_pk_step(Ctx cx, PkArgs pa) {
  static_assert(NW == 8, "8 waves per workgroup: 2 image rows (one pool row) per wave, 4 fc1 rows per wave");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  using P = Plan;
  using Gm = Geo<NW>;
  constexpr int RPW = Gm::RPW, NTH = Gm::NT;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63, c = lane & 15, q = lane >> 4;
  const int r0 = w * RPW;  // first image row owned by this wave
  if (pa.xpack && (blockIdx.x & 7)) return;  // placement filler (see pk_img)
  const int n = pk_img(pa.xpack);
  float* cred = (float*)(smem + P::O_CRED);
  float* stat = (float*)(smem + P::O_STAT);
  float* misc = (float*)(smem + P::O_MISC);  // [0,64) publish | [64,192) sums | [192,256) scale/shift | ...
  char* U = smem + P::O_U;
  char* WT = U + P::U_WT;
  char* XR = U + P::U_XR;
  const int epoch = *pa.epoch;
  const size_t img = (size_t)n * 8192;
  const int B = cx.B;
  const int par = epoch & 1;
  const uint8_t* my_img = pa.simg + (size_t)(par * 64 + n) * 3072;  // staged by the previous step
  const int next_id = sample_id(cx, B + n);  // image n of the NEXT batch (staged at the end of this step)
  PK_STAMP(cx, 0);

  float g[RPW][2][4];   // dL/dx of the current block input (backward), starting with dL/dx10 from the head
  float yb[RPW][2][4];  // the backward's y_i tile and its x_i tile (packed bf16), y_9 / x_9 loaded by the head
  uint2 xb[RPW][2];
  if (pa.phase != 2) {  // ---------------- stem, forward, head (whole step, or split-mode phase 1) ----------------
  // ======================= stem: gather + normalise + conv1 + bias + ReLU + 2x2 max-pool =================
  // Input staged as bf16 NHWC4 pixels (3 channels + a zero), so an MFMA K-group of 4 is one tap of one pixel:
  // v_mfma_f32_16x16x16_bf16 with K = (tap, channel), 3 MFMAs cover the 9 taps (taps 9..11 have zero weights).
  {
    uint2* xin4 = (uint2*)(U + P::U_XIN);  // [34][34] pixels, zero halo
    const float* sb = misc + 874;
    float* x0i = (float*)(U + P::U_X0);
    // step constants -> misc: k < 64: BN gamma|beta -> misc[320 + k]; k >= 64 -> misc[384 + k]: running
    // mean|var (rank 0's base under DDP, reference CC4) [448,512), fc1 bias [512,544), W2 [544,864),
    // b2 [864,874), conv1 bias [874,906), BN shifts [906,1226) (= P_KSHIFT).  Every global load of the
    // prologue is issued before any is waited for.
    constexpr int NKC = 842, KCM = (NKC + NTH - 1) / NTH;
    float kc[KCM];
#pragma unroll
    for (int m = 0; m < KCM; ++m) {
      const int k = min(t + NTH * m, NKC - 1);
      const float* rsm = cx.ws > 1 ? cx.rs_base : cx.rm;
      const float* rsv = cx.ws > 1 ? cx.rs_base + 32 : cx.rv;
      const float* src = k < 64 ? cx.params + OFF_BNW + k
                       : k < 96 ? rsm + (k - 64)
                       : k < 128 ? rsv + (k - 96)
                       : k < 160 ? cx.params + OFF_FC1B + (k - 128)
                       : k < 480 ? cx.params + OFF_FC2W + (k - 160)
                       : k < 490 ? cx.params + OFF_FC2B + (k - 480)
                       : k < 522 ? cx.params + OFF_C1B + (k - 490)
                                 : (const float*)cx.STATS + 2 * (k - 522);  // BN shifts (.x = mean)
      kc[m] = *src;
    }
    int lab = pa.slab[par * 64 + n];
    const int tq = t & 255;  // threads < 256: pixels (y = tq >> 3, x = 4 (tq & 7) .. +3), all 3 channels
    const unsigned* imw = (const unsigned*)my_img;
    unsigned iw0 = imw[tq], iw1 = imw[256 + tq], iw2 = imw[512 + tq];
    uint4 wt0, wt1, wt2;
    stage_wt_load3(wt0, wt1, wt2, cx.wt_f);
    // B fragments (conv1 weights) for the whole stem, prepared by the SGD kernels: lane (co = 16h + c,
    // k-group q) of MFMA m holds W[co][ci = 0..2][tap = 4m + q] and a zero (4th channel / taps 9..11)
    uint2 bwr[2][3];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int m = 0; m < 3; ++m) bwr[h][m] = ((const uint2*)cx.swf)[(h * 3 + m) * 64 + lane];
#pragma unroll
    for (int m = 0; m < KCM; ++m) pin(kc[m]);
    pin(lab);
    pin(iw0);
    pin(iw1);
    pin(iw2);
    pin(wt0);
    pin(wt1);
    pin(wt2);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int m = 0; m < 3; ++m) {
        pin(bwr[h][m].x);
        pin(bwr[h][m].y);
      }
#pragma unroll
    for (int m = 0; m < KCM; ++m) {
      const int k = t + NTH * m;
      if (k < NKC) misc[(k < 64 ? 320 : 384) + k] = k >= 522 && !(fabsf(kc[m]) < 1e30f) ? 0.f : kc[m];
    }
    if (t == 0) misc[P_LABEL] = __int_as_float(lab);  // label for the head's cross-entropy
    if (t < 256) {
      const int y = tq >> 3, x0 = 4 * (tq & 7);
#pragma unroll
      for (int b2 = 0; b2 < 4; ++b2) {
        const unsigned c0 = bfbits(norm_px((iw0 >> (8 * b2)) & 255u, 0));
        const unsigned c1 = bfbits(norm_px((iw1 >> (8 * b2)) & 255u, 1));
        const unsigned c2 = bfbits(norm_px((iw2 >> (8 * b2)) & 255u, 2));
        xin4[(y + 1) * 34 + x0 + 1 + b2] = uint2{c0 | (c1 << 16), c2};
      }
    } else if (tq < 132) {  // the 132 halo pixels: rows 0 / 33 (34 each), cols 0 / 33 of rows 1..32
      const int px = tq < 34 ? tq : tq < 68 ? 33 * 34 + (tq - 34) : ((tq - 68) / 2 + 1) * 34 + ((tq - 68) & 1) * 33;
      xin4[px] = uint2{0u, 0u};
    }
    stage_wt_store3(WT, wt0, wt1, wt2);
    zero_xr_halo<NW>(XR);
    lds_barrier();
    PK_STAMP(cx, 29);
    s4v bw[2][3];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int m = 0; m < 3; ++m) bw[h][m] = __builtin_bit_cast(s4v, bwr[h][m]);
    uint8_t* scl = (uint8_t*)(U + P::U_SCODE);
    PK_STAMP(cx, 43);
#pragma unroll 1
    for (int j = 0; j < 32 / NW; ++j) {
      if (j == 1) PK_STAMP(cx, 44);
      const int u = w + NW * j, pr = u >> 1, chalf = u & 1;  // pool row pr, image cols 16 chalf .. +15
      f32x4 acc[2][2];
#pragma unroll
      for (int rw = 0; rw < 2; ++rw) {
        acc[rw][0] = z4();
        acc[rw][1] = z4();
#pragma unroll
        for (int m = 0; m < 3; ++m) {
          const int tap = 4 * m + q, tc = tap < 9 ? tap : 0, kh = tc / 3, kw = tc % 3;
          const uint2 av = xin4[(2 * pr + rw + kh) * 34 + 16 * chalf + c + kw];
          const s4v a = __builtin_bit_cast(s4v, av);
          acc[rw][0] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, bw[0][m], acc[rw][0], 0, 0, 0);
          acc[rw][1] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, bw[1][m], acc[rw][1], 0, 0, 0);
        }
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int co = 16 * h + c;
        const float bias = sb[co];
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
          const float v00 = fmaxf(acc[0][h][2 * pp] + bias, 0.f), v01 = fmaxf(acc[0][h][2 * pp + 1] + bias, 0.f);
          const float v10 = fmaxf(acc[1][h][2 * pp] + bias, 0.f), v11 = fmaxf(acc[1][h][2 * pp + 1] + bias, 0.f);
          float best = v00;
          int code = 0;
          if (v01 > best) { best = v01; code = 1; }
          if (v10 > best) { best = v10; code = 2; }
          if (v11 > best) { best = v11; code = 3; }
          if (best > 0.f) code |= 4;
          const int pc = 8 * chalf + 2 * q + pp, po = (pr * 16 + pc) * 32 + co;
          x0i[(pr * 16 + pc) * P::X0S + co] = best;
          scl[po] = (uint8_t)code;
          st1r(XR, (pr + 1) * 18 + pc + 1, co, best);
        }
      }
    }
    PK_STAMP(cx, 30);
    lds_barrier();
  }
  PK_STAMP(cx, 1);
  float x[RPW][2][4], y[RPW][2][4];
  {
    const float* x0i = (const float*)(U + P::U_X0);
#pragma unroll
    for (int rr = 0; rr < RPW; ++rr)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i) x[rr][h][i] = x0i[((r0 + rr) * 16 + 4 * q + i) * P::X0S + 16 * h + c];
    // x0 and the stem pool codes go to global in the tiled layout, written by the very threads that read them
    // back in the backward (so no workgroup-wide memory barrier is ever needed for them)
    const uint8_t* scl = (const uint8_t*)(U + P::U_SCODE);
#pragma unroll
    for (int rr = 0; rr < RPW; ++rr)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        stx(cx.X + img / 2, r0 + rr, h, lane, x[rr][h]);
        unsigned cw = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) cw |= (unsigned)scl[el(r0 + rr, q, c, h, i)] << (8 * i);
        *(unsigned*)(cx.SCODE + img + tl(r0 + rr, h, lane)) = cw;
      }
  }

  // ======================= forward: 10 applications of the shared ResBlock =================================
#pragma unroll 1
  for (int i = 0; i < NBLK; ++i) {
    if (i > 0) {
      bn_fwd_stats<NW>(cx, pa, epoch, i - 1, y, cred, misc, stat);
      float* Xo = cx.X + ((size_t)i * B * 8192 + img) / 2;  // bf16 tiles
      float* Yo = cx.Y + (size_t)(i - 1) * B * 8192 + img;  // y_{i-1}, written now that its exchange is done
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int ch = 16 * h + c;
        const float sc = misc[192 + ch], sh = misc[224 + ch];
#pragma unroll
        for (int rr = 0; rr < RPW; ++rr) {
#pragma unroll
          for (int i2 = 0; i2 < 4; ++i2) {
            const float v = fmaxf(y[rr][h][i2] * sc + sh, 0.f) + x[rr][h][i2];
            x[rr][h][i2] = v;
            st1r(XR, (r0 + rr + 1) * 18 + 4 * q + i2 + 1, ch, v);
          }
          st4v(Yo + tl(r0 + rr, h, lane), y[rr][h]);
          stx(Xo, r0 + rr, h, lane, x[rr][h]);
        }
      }
      lds_barrier();
    }
    if (i == 6) PK_STAMP(cx, 39);
    f32x4 acc[RPW][2];
    conv_img<RPW>(XR, WT, acc, r0, lane);
#pragma unroll
    for (int rr = 0; rr < RPW; ++rr)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i2 = 0; i2 < 4; ++i2) y[rr][h][i2] = acc[rr][h][i2];
    PK_STAMP(cx, 2 + i);
  }
  // fc1 weight slice of this wave (bf16 copy): all 32 rows x features 256w + 4l .. +3 (lane l) = 64 VGPRs,
  // loaded once (issued before the last BN exchange, whose wait hides the latency), used by fc1 AND its
  // transpose (dp), so W1 is read once per step
  uint2 wv[32];
  {
    const uint2* W1b = (const uint2*)cx.w1b;
#pragma unroll
    for (int j = 0; j < 32; ++j) wv[j] = W1b[j * 512 + w * 64 + lane];
  }

  bn_fwd_stats<NW>(cx, pa, epoch, NBLK - 1, y, cred, misc, stat);
  if (n == 0 && t < 32) {
    cx.rm[t] = misc[448 + t];
    cx.rv[t] = misc[480 + t];
  }
  {
    float* Yo = cx.Y + (size_t)(NBLK - 1) * B * 8192 + img;
#pragma unroll
    for (int rr = 0; rr < RPW; ++rr)
#pragma unroll
      for (int h = 0; h < 2; ++h) st4v(Yo + tl(r0 + rr, h, lane), y[rr][h]);
  }
  PK_STAMP(cx, 12);

  // ======================= head =============================================================================
  // x10 = relu(bn(y9)) + x9, 2x2 max-pool, fc1 + ReLU, fc2, cross-entropy (mean over the batch) and their
  // backward down to g = dL/dx10, all inside the workgroup.
  {
    float* Pv = (float*)(U + P::U_P);      // [2048] pooled features, NCHW flatten order c*64 + ph*8 + pw
    float* dp = (float*)(U + P::U_DP);     // [2048] dL/dpooled
    float* hp = (float*)(U + P::U_HP);     // [8 waves][32] fc1 partial sums; [256, 288) dh
    // pool straight from registers: the wave's two rows are one pool row; cols 4q..4q+3 are two windows
    unsigned codes = 0;  // 2-bit argmax per (h, window)
    float pooled[4];     // this thread's pooled outputs (stored for the reduce kernel after the loss)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int ch = 16 * h + c;
      const float sc = misc[192 + ch], sh = misc[224 + ch];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {  // window order (0,0) (0,1) (1,0) (1,1): first maximum wins
          const int rr = e >> 1, i2 = 2 * k + (e & 1);
          v[e] = fmaxf(y[rr][h][i2] * sc + sh, 0.f) + x[rr][h][i2];
        }
        float best = v[0];
        unsigned id = 0;
        if (v[1] > best) { best = v[1]; id = 1; }
        if (v[2] > best) { best = v[2]; id = 2; }
        if (v[3] > best) { best = v[3]; id = 3; }
        codes |= id << (2 * (2 * h + k));
        Pv[ch * 64 + w * 8 + 2 * q + k] = best;  // pool row = w, pool col = 2q + k
        pooled[2 * h + k] = best;
      }
    }
    lds_barrier();
    PK_STAMP(cx, 31);
    // fc1 partial sums over this wave's 256 features for all 32 rows, then a butterfly reduce-scatter across the
    // lanes (31 shuffles): lane l ends with the wave's sum for row (l >> 1) & 31
    {
      const f32x4 pv = ld4(Pv + 256 * w + 4 * lane);
      float v[32];
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        const uint2 u = wv[j];
        v[j] = __uint_as_float(u.x << 16) * pv[0] + __uint_as_float(u.x & 0xffff0000u) * pv[1] +
               __uint_as_float(u.y << 16) * pv[2] + __uint_as_float(u.y & 0xffff0000u) * pv[3];
      }
#pragma unroll
      for (int step = 0; step < 5; ++step) {
        const int half = 16 >> step, off = 32 >> step;
        const bool upper = (lane & off) != 0;
#pragma unroll
        for (int r = 0; r < half; ++r) {
          const float keep = upper ? v[half + r] : v[r], give = upper ? v[r] : v[half + r];
          v[r] = keep + __shfl_xor(give, off);
        }
      }
      const float tot = v[0] + __shfl_xor(v[0], 1);
      if ((lane & 1) == 0) hp[w * 32 + (lane >> 1)] = tot;
    }
    lds_barrier();
    PK_STAMP(cx, 32);
    if (w == 0) {
      // wave 0: fc1 bias + ReLU, fc2, softmax cross-entropy and dh, lane-parallel with shuffles (no barriers)
      float hh = 0.f;
      if (lane < 32) {
        hh = misc[512 + lane];
#pragma unroll
        for (int k2 = 0; k2 < NW; ++k2) hh += hp[k2 * 32 + lane];
      }
      PK_STAMP(cx, 40);
      const float hr = fmaxf(hh, 0.f);
      const int o = lane < 10 ? lane : 0;
      float logit = misc[864 + o];
#pragma unroll
      for (int j = 0; j < 32; ++j)
        logit += misc[544 + o * 32 + j] * __int_as_float(__builtin_amdgcn_readlane(__float_as_int(hr), j));
      PK_STAMP(cx, 41);
      float lg[10];  // the 10 logits, broadcast to every lane (scalar reads, no LDS shuffles)
#pragma unroll
      for (int oo = 0; oo < 10; ++oo) lg[oo] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(logit), oo));
      float mx = lg[0];
#pragma unroll
      for (int oo = 1; oo < 10; ++oo) mx = fmaxf(mx, lg[oo]);
      float ex[10], se = 0.f;
#pragma unroll
      for (int oo = 0; oo < 10; ++oo) {
        ex[oo] = __expf(lg[oo] - mx);
        se += ex[oo];
      }
      const float lse = mx + __logf(se), rse = 1.f / se;
      const int label = __float_as_int(misc[P_LABEL]);
      float lt = lg[0];
#pragma unroll
      for (int oo = 1; oo < 10; ++oo) lt = label == oo ? lg[oo] : lt;
      if (lane == 0) cx.HLOSS[n] = lse - lt;
      const float invB = 1.f / (float)B;
      float sd = 0.f, dl = 0.f;
#pragma unroll
      for (int oo = 0; oo < 10; ++oo) {
        const float dlo = (ex[oo] * rse - (oo == label ? 1.f : 0.f)) * invB;
        sd += misc[544 + oo * 32 + (lane & 31)] * dlo;
        dl = lane == oo ? dlo : dl;
      }
      const float dh = hh > 0.f ? sd : 0.f;
      PK_STAMP(cx, 42);
      if (lane < 32) {
        hp[256 + lane] = dh;
        cx.HDH[n * 32 + lane] = dh;
        cx.HH[n * 32 + lane] = hr;
      }
      if (lane < 10) cx.HDL[n * 10 + lane] = dl;
    } else {
      // waves 1..7 meanwhile: the backward conv weights (taps flipped, ci <-> co transposed) re-laid out from
      // the forward copy still in WT -- no global reload.  Chunk o: record R = (8 - tap) * 32 + ci, co 8(o&3)..+7
      unsigned wtr[3][4];
#pragma unroll
      for (int m = 0; m < 3; ++m) {
        const int o0 = t - 64 + (NTH - 64) * m, o = o0 < 1152 ? o0 : 1151, R = o >> 2, co0 = 8 * (o & 3);
        const int tap = 8 - (R >> 5), ci = R & 31;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const unsigned lo = *(const unsigned short*)(WT + (tap * 32 + co0 + 2 * e) * P::RB + 2 * ci);
          const unsigned hi = *(const unsigned short*)(WT + (tap * 32 + co0 + 2 * e + 1) * P::RB + 2 * ci);
          wtr[m][e] = lo | (hi << 16);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // waves 1..7: all WT reads done
#pragma unroll
      for (int m = 0; m < 3; ++m) {
        const int o = t - 64 + (NTH - 64) * m;
        if (o < 1152) *(uint4*)(WT + (o >> 2) * P::RB + (o & 3) * 16) = uint4{wtr[m][0], wtr[m][1], wtr[m][2], wtr[m][3]};
      }
    }
    if (w == 0) asm volatile("s_barrier" ::: "memory");  // wave 0's side of the waves-1..7 barrier above
    lds_barrier();
    PK_STAMP(cx, 33);
#pragma unroll
    for (int hk = 0; hk < 4; ++hk)  // fc1 input for the weight gradient (k_pk_reduce)
      cx.HP[(size_t)n * 2048 + (16 * (hk >> 1) + c) * 64 + w * 8 + 2 * q + (hk & 1)] = pooled[hk];
    // dp = W1^T dh for this wave's features (complete per lane: all 32 rows are in its registers)
    {
      f32x4 d = z4();
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        const float dhj = hp[256 + j];
        const uint2 u = wv[j];
        d[0] += dhj * __uint_as_float(u.x << 16);
        d[1] += dhj * __uint_as_float(u.x & 0xffff0000u);
        d[2] += dhj * __uint_as_float(u.y << 16);
        d[3] += dhj * __uint_as_float(u.y & 0xffff0000u);
      }
      st4(dp + 256 * w + 4 * lane, d);
    }
    {  // y_9 / x_9 for the first backward block (this thread's own stores: no cross-thread hand-off)
      const float* yp = cx.Y + (size_t)(NBLK - 1) * B * 8192 + img;
      const float* xp = cx.X + ((size_t)(NBLK - 1) * B * 8192 + img) / 2;
#pragma unroll
      for (int rr = 0; rr < RPW; ++rr)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          ld4v(yp + tl(r0 + rr, h, lane), yb[rr][h]);
          xb[rr][h] = ldx(xp, r0 + rr, h, lane);
        }
    }
    lds_barrier();
    // g = max-pool backward of dp, routed by the saved argmax
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const float dpv = dp[(16 * h + c) * 64 + w * 8 + 2 * q + k];
        const unsigned id = (codes >> (2 * (2 * h + k))) & 3u;
#pragma unroll
        for (int e = 0; e < 4; ++e) g[e >> 1][h][2 * k + (e & 1)] = id == (unsigned)e ? dpv : 0.f;
      }
    if (pa.debug) {
#pragma unroll
      for (int rr = 0; rr < RPW; ++rr)
#pragma unroll
        for (int h = 0; h < 2; ++h) st4v(cx.G + img + tl(r0 + rr, h, lane), g[rr][h]);
    }
  }
  if (pa.phase == 1) {  // split mode: hand dL/dx10 to phase 2 (own-thread layout) and end here
#pragma unroll
    for (int rr = 0; rr < RPW; ++rr)
#pragma unroll
      for (int h = 0; h < 2; ++h) st4v(pa.gh + img + tl(r0 + rr, h, lane), g[rr][h]);
    return;
  }
  } else {  // ---------------- split-mode phase 2: restore what phase 1 left in LDS / registers ----------------
#pragma unroll
    for (int rr = 0; rr < RPW; ++rr)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        ld4v(pa.gh + img + tl(r0 + rr, h, lane), g[rr][h]);
        ld4v(cx.Y + (size_t)(NBLK - 1) * B * 8192 + img + tl(r0 + rr, h, lane), yb[rr][h]);
        xb[rr][h] = ldx(cx.X + ((size_t)(NBLK - 1) * B * 8192 + img) / 2, r0 + rr, h, lane);
      }
    if (t < NBLK * 32) {  // batch (mean, invstd) of every block, written by workgroup 0 of phase 1
      const float2 st = cx.STATS[t];
      stat[(t >> 5) * 64 + (t & 31)] = st.x;
      stat[(t >> 5) * 64 + 32 + (t & 31)] = st.y;
    }
    if (t < 64) misc[320 + t] = cx.params[OFF_BNW + t];  // gamma | beta
    if (t == 0) misc[P_FAST] = 0.f;
    stage_wt<NW>(WT, cx.wt_d);
  }
  PK_STAMP(cx, 13);
  lds_barrier();  // every wave is done with the head's LDS before the backward's tiles overwrite it

  // ======================= backward: 10 applications, newest first ========================================
  unsigned short* dyT = (unsigned short*)(U + P::U_DYT);
  unsigned short* xT = (unsigned short*)(U + P::U_XT);
  zero_xr_halo<NW>(XR);
  for (int idx = t; idx < 3 * 32 * P::XT_S * 2 / 16; idx += NTH) ((uint4*)xT)[idx] = uint4{0u, 0u, 0u, 0u};

  f32x4 wacc[Gm::NNT][2];
#pragma unroll
  for (int j = 0; j < Gm::NNT; ++j) wacc[j][0] = wacc[j][1] = z4();
  uint4 nxt = uint4{0u, 0u, 0u, 0u};  // next batch's image n (+ label): loaded during the last backward block,
  int nxt_lab = 0;                    // stored into the other staging parity at the end of the step
  float dgam = 0.f, dbet = 0.f;
  unsigned codew[RPW][2];                         // stem-backward prefetch (filled during block 0)
  unsigned imgw[Gm::IMW];
  lds_barrier();
  const float Ntot = (float)B * 256.f;
#pragma unroll 1
  for (int i = NBLK - 1; i >= 0; --i) {
    // yb / xb hold y_i / x_i (loaded during the previous block)
    float sa[2] = {0.f, 0.f}, sbv[2] = {0.f, 0.f}, dz[RPW][2][4], xh[RPW][2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int ch = 16 * h + c;
      const float mean = stat[i * 64 + ch], inv = stat[i * 64 + 32 + ch];
      const float gam = misc[320 + ch], bet = misc[352 + ch];
      const float sc = gam * inv, sh = bet - mean * sc;
#pragma unroll
      for (int rr = 0; rr < RPW; ++rr)
#pragma unroll
        for (int i2 = 0; i2 < 4; ++i2) {
          xh[rr][h][i2] = (yb[rr][h][i2] - mean) * inv;
          dz[rr][h][i2] = (yb[rr][h][i2] * sc + sh) > 0.f ? g[rr][h][i2] : 0.f;
          sa[h] += dz[rr][h][i2];
          sbv[h] += dz[rr][h][i2] * xh[rr][h][i2];
        }
    }
    const float pv = img_csum_pub<NW>(sa[0], sa[1], sbv[0], sbv[1], cred);  // image sums -> publish value
    xchg_publish(pa, epoch, NBLK + (NBLK - 1 - i), pv, misc[P_FAST] != 0.f);
    if (i == 5) PK_STAMP(cx, 36);
    // While the exchange is in flight: the weight gradient of the PREVIOUS application (block i + 1), whose
    // dy / x tiles are still staged in dyT / xT.  Then the barrier retires every wave's reads of them (and of
    // XR by block i + 1's dgrad) before x_i replaces them.
    if (i < NBLK - 1) wgrad_acc<NW>(dyT, xT, wacc, w, lane);
    if (i == 5) PK_STAMP(cx, 38);
    EarlyPass<NW> ep;  // first sweep pass issued now, evaluated after the x tile writes
    xchg_early<NW>(pa, NBLK + (NBLK - 1 - i), ep);
    lds_barrier();
#pragma unroll
    for (int rr = 0; rr < RPW; ++rr)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int ch = 16 * h + c, rowoff = (r0 + rr + 1) * 16 + 4 * q;
        const unsigned b0 = xb[rr][h].x & 0xffffu, b1 = xb[rr][h].x >> 16;
        const unsigned b2 = xb[rr][h].y & 0xffffu, b3 = xb[rr][h].y >> 16;
        unsigned short* p1 = xT + (32 + ch) * P::XT_S + rowoff;  // kw = 1: x at the same column
        *(uint2*)p1 = uint2{b0 | (b1 << 16), b2 | (b3 << 16)};
        unsigned short* p0 = xT + ch * P::XT_S + rowoff;  // kw = 0: column + 1
        p0[1] = (unsigned short)b0;
        *(unsigned*)(p0 + 2) = b1 | (b2 << 16);
        if (q < 3) p0[4] = (unsigned short)b3;
        unsigned short* p2 = xT + (64 + ch) * P::XT_S + rowoff;  // kw = 2: column - 1
        if (q > 0) p2[-1] = (unsigned short)b0;
        *(unsigned*)p2 = b1 | (b2 << 16);
        p2[2] = (unsigned short)b3;
      }
    if (i == 5) PK_STAMP(cx, 27);
    {
      const float tot = xchg_wait<NW>(pa, epoch, NBLK + (NBLK - 1 - i), cred, &ep);
      if (t < 64) misc[64 + t] = tot;  // batch sums: [64, 96) sum dz, [96, 128) sum dz * xhat
      lds_barrier();
    }
    if (i == 5) PK_STAMP(cx, 28);
    if (i > 0) {  // prefetch y_{i-1} / x_{i-1}; the loads land while this block's convolutions run
      const float* yp = cx.Y + (size_t)(i - 1) * B * 8192 + img;
      const float* xp = cx.X + ((size_t)(i - 1) * B * 8192 + img) / 2;
#pragma unroll
      for (int rr = 0; rr < RPW; ++rr)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          ld4v(yp + tl(r0 + rr, h, lane), yb[rr][h]);
          xb[rr][h] = ldx(xp, r0 + rr, h, lane);
        }
    } else {  // last block: prefetch what the stem backward needs (pool codes, raw image words)
#pragma unroll
      for (int rr = 0; rr < RPW; ++rr)
#pragma unroll
        for (int h = 0; h < 2; ++h) codew[rr][h] = *(const unsigned*)(cx.SCODE + img + tl(r0 + rr, h, lane));
      stage_input_load<NW>(imgw, my_img);
      nxt = ((const uint4*)(cx.data + (size_t)next_id * 3072))[t < 192 ? t : 0];
      nxt_lab = cx.labels[next_id];
    }
    if (n == 0 && t < 32) {
      dbet += misc[64 + t];
      dgam += misc[96 + t];
    }
    float* dyo = cx.DY + (size_t)i * B * 8192 + img;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int ch = 16 * h + c;
      const float Sa = misc[64 + ch], Sb = misc[96 + ch];
      const float k1 = misc[320 + ch] * stat[i * 64 + 32 + ch] / Ntot;
#pragma unroll
      for (int rr = 0; rr < RPW; ++rr) {
        const int row = r0 + rr;
        unsigned bits[4];
        float dyv4[4];
#pragma unroll
        for (int i2 = 0; i2 < 4; ++i2) {
          const float dyv = k1 * (Ntot * dz[rr][h][i2] - Sa - xh[rr][h][i2] * Sb);
          dyv4[i2] = dyv;
          const int col = 4 * q + i2;
          st1r(XR, (row + 1) * 18 + col + 1, ch, dyv);
          bits[i2] = bfbits(dyv);
        }
        if (pa.debug) st4v(dyo + tl(row, h, lane), dyv4);
        *(uint2*)(dyT + ch * P::DYT_S + row * 16 + 4 * q) = uint2{bits[0] | (bits[1] << 16), bits[2] | (bits[3] << 16)};
      }
    }
    lds_barrier();
    if (i == 5) PK_STAMP(cx, 37);
    // dgrad: g_i = g_{i+1} + conv(dy, W^T flipped)
    {
      f32x4 acc[RPW][2];
      conv_img<RPW>(XR, WT, acc, r0, lane);
#pragma unroll
      for (int rr = 0; rr < RPW; ++rr)
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int i2 = 0; i2 < 4; ++i2) g[rr][h][i2] += acc[rr][h][i2];
    }
    PK_STAMP(cx, 14 + (NBLK - 1 - i));
    if (pa.debug && i >= 1) {
      float* gout = cx.G + (size_t)((10 - i) & 1) * B * 8192 + img;
#pragma unroll
      for (int rr = 0; rr < RPW; ++rr)
#pragma unroll
        for (int h = 0; h < 2; ++h) st4v(gout + tl(r0 + rr, h, lane), g[rr][h]);
    }
  }
  wgrad_acc<NW>(dyT, xT, wacc, w, lane);  // application 0 (its dyT / xT are staged by the last iteration)
  if (n == 0 && t < 32) {
    pa.bng[t] = dgam;
    pa.bng[32 + t] = dbet;
  }

  // ======================= stem backward: max-pool bwd (saved argmax) -> ReLU mask -> conv1 wgrad ==========
  lds_barrier();  // every wave is done with the backward's LDS regions
  {
    unsigned short* dsT = (unsigned short*)(U + P::U_DST);  // [32 co][DSP] bf16 d(stem conv output)
    unsigned short* xs = (unsigned short*)(U + P::U_XS);
    // d(conv1 output): every 2x2 pool window written whole (value at the argmax if the ReLU was active, zeros
    // elsewhere), so dsT needs no clearing pass
    float db0 = 0.f, db1 = 0.f;
#pragma unroll
    for (int rr = 0; rr < RPW; ++rr)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i2 = 0; i2 < 4; ++i2) {
          const unsigned code = (codew[rr][h] >> (8 * i2)) & 255u, pos = code & 3u;
          const float val = (code & 4u) ? g[rr][h][i2] : 0.f;
          const unsigned vb = bfbits(val);
          const int ch = 16 * h + c, sr = 2 * (r0 + rr), sc = 2 * (4 * q + i2);
          unsigned short* d0 = dsT + ch * P::DSP + sr * 32 + sc;
          *(unsigned*)d0 = (pos == 0 ? vb : 0u) | ((pos == 1 ? vb : 0u) << 16);
          *(unsigned*)(d0 + 32) = (pos == 2 ? vb : 0u) | ((pos == 3 ? vb : 0u) << 16);
          if (h == 0) db0 += val;
          else db1 += val;
        }
    // three column-shifted bf16 copies of the normalised input (copy kw, col c holds x[c + kw - 1]); row r + 1
    // holds image row r, rows 0 / 33 are the zero halo
#pragma unroll
    for (int m = 0; m < Gm::IMW; ++m) {
      const int idx = t + NTH * m;
      if (idx < 768) {
        const int ch = idx >> 8, row = ((idx >> 3) & 31) + 1, x0 = 4 * (idx & 7);
        unsigned bb[4];
#pragma unroll
        for (int b2 = 0; b2 < 4; ++b2) bb[b2] = bfbits(norm_px((imgw[m] >> (8 * b2)) & 255u, ch));
        unsigned short* p1 = xs + ((3 + ch) * 34 + row) * P::XS_S + x0;  // kw = 1
        *(uint2*)p1 = uint2{bb[0] | (bb[1] << 16), bb[2] | (bb[3] << 16)};
        unsigned short* p0 = xs + ((0 + ch) * 34 + row) * P::XS_S + x0;  // kw = 0: col c holds x[c - 1]
        p0[1] = (unsigned short)bb[0];
        *(unsigned*)(p0 + 2) = bb[1] | (bb[2] << 16);
        if (x0 + 4 < 32) p0[4] = (unsigned short)bb[3];
        unsigned short* p2 = xs + ((6 + ch) * 34 + row) * P::XS_S + x0;  // kw = 2: col c holds x[c + 1]
        if (x0 > 0) p2[-1] = (unsigned short)bb[0];
        *(unsigned*)p2 = bb[1] | (bb[2] << 16);
        p2[2] = (unsigned short)bb[3];
      }
    }
    if (t < 72) {  // halo rows 0 and 33 of the 9 planes (32 cols = 4 x 16 B each)
      const int plane = t >> 3, row = (t >> 2) & 1 ? 33 : 0, part = t & 3;
      *(uint4*)(xs + (plane * 34 + row) * P::XS_S + 8 * part) = uint4{0u, 0u, 0u, 0u};
    } else if (t < 72 + 192) {  // kw = 0: col 0 (x[-1]); kw = 2: col 31 (x[32]) of rows 1..32
      const int e = t - 72, kwe = e < 96 ? 0 : 2, ci = (e % 96) >> 5, row = (e & 31) + 1;
      xs[((kwe * 3 + ci) * 34 + row) * P::XS_S + (kwe ? 31 : 0)] = 0;
    }
    img_csum2<NW>(db0, db1, 0.f, 0.f, cred, misc + 384, misc + 416);  // also the barrier before the MFMAs
    PK_STAMP(cx, 34);
    float* ss = cx.SSLAB + (size_t)n * SSLAB_N;
    if (t < 32) ss[1024 + t] = misc[384 + t];
    // D[co][k] = sum over the 1024 stem pixels of ds[p][co] * im2col[p][k], K step = one image row.
    // Wave w: tile w & 3 (mt = co half, nt = k tile), rows 16 (w >> 2) .. +15; k >= 27 columns are discarded.
    {
      const int tile = w & 3, mt = tile & 1, nt = tile >> 1, r0s = 16 * (w >> 2);
      const int kidx = 16 * nt + c, kk = kidx < 27 ? kidx : 0, ci = kk / 9, kh = (kk % 9) / 3, kw = kk % 3;
      const unsigned short* abase = dsT + (16 * mt + c) * P::DSP + 8 * q;
      const unsigned short* bbase = xs + ((kw * 3 + ci) * 34 + kh) * P::XS_S + 8 * q;
      f32x4 acc2 = z4();
#pragma unroll 4
      for (int sr = r0s; sr < r0s + 16; ++sr) {
        const bf16x8 a = *(const bf16x8*)(abase + sr * 32);
        const bf16x8 b = *(const bf16x8*)(bbase + sr * P::XS_S);
        acc2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc2, 0, 0, 0);
      }
      float* sred = (float*)(U + P::U_SRED);
      st4(sred + ((w * 64 + lane) << 2), acc2);  // [8 waves][64 lanes][4]
    }
    PK_STAMP(cx, 35);
    lds_barrier();
    if (t < 256) {
      const float* sred = (const float*)(U + P::U_SRED);
      const int tile = t >> 6, ln = t & 63;
      st4(ss + ((tile * 64 + ln) << 2), ld4(sred + ((tile * 64 + ln) << 2)) + ld4(sred + (((tile + 4) * 64 + ln) << 2)));
    }
  }
  if (t < 192) ((uint4*)(pa.simg + (size_t)((par ^ 1) * 64 + n) * 3072))[t] = nxt;
  if (t == 192) pa.slab[(par ^ 1) * 64 + n] = nxt_lab;
  // trunk wgrad slab (accumulated over the 10 applications)
#pragma unroll
  for (int j = 0; j < Gm::NNT; ++j) {
    const int nt = w + NW * j;
    if (nt < 18) {  // slab tile tt = 2 nt + mt (layout read by k_pk_reduce)
      st4(pa.tslab + (size_t)n * WSLAB_N + (((2 * nt) * 64 + lane) << 2), wacc[j][0]);
      st4(pa.tslab + (size_t)n * WSLAB_N + (((2 * nt + 1) * 64 + lane) << 2), wacc[j][1]);
    }
  }
  PK_STAMP(cx, 24);
}

// ============================================================================================================
// Reduction + SGD after the persistent step.  Grid: 36 trunk chunks | 5 stem chunks | 32 fc1 column blocks |
// 1 bookkeeping workgroup (fc2, biases, BN, loss, cursor, epoch).  256 threads.
// ============================================================================================================
// Batch ids for the first step after the host moved the cursor or replaced the index list.
// Stage image / label / id of batch position `b` (= cursor + b) into staging parity `par`.
__device__ __forceinline__ void stage_sample(const Ctx& cx, const PkArgs& pa, int b, int par) {
  const int t = threadIdx.x, id = sample_id(cx, b);
  if (t < 192)
    ((uint4*)(pa.simg + (size_t)(par * 64 + b) * 3072))[t] = ((const uint4*)(cx.data + (size_t)id * 3072))[t];
  if (t == 192) {
    pa.slab[par * 64 + b] = cx.labels[id];
    pa.ids[b] = id;
  }
}
// The first batch after the host moved the cursor or replaced the index list (grid 64 x 256).
__global__ void __launch_bounds__(256) k_pk_prime_ids(Ctx cx, PkArgs pa) {
  stage_sample(cx, pa, blockIdx.x, *pa.epoch & 1);
}

constexpr int R_TRUNK = 36, R_STEM = 5, R_FC = 32, R_WORK = R_TRUNK + R_STEM + R_FC + 1;
constexpr int R_GRID = R_WORK;

__device__ __forceinline__ void sgd_put(const Ctx& cx, int pidx, float gval) {
  cx.grads[pidx] = gval;
  if (cx.fuse_sgd) cx.params[pidx] -= cx.lr * gval;
}
// same with the old parameter value loaded up front (no load -> store round trip after the reduction);
// returns the value the parameter now has
__device__ __forceinline__ float sgd_put_pre(const Ctx& cx, int pidx, float gval, float oldp) {
  cx.grads[pidx] = gval;
  if (cx.fuse_sgd) {
    const float np = oldp - cx.lr * gval;
    cx.params[pidx] = np;
    return np;
  }
  return oldp;
}

// slab reduction + SGD of the shared trunk conv (36 chunks of 256 outputs) and of conv1 (5 chunks)
__device__ __forceinline__ void pk_red_trunk_stem(const Ctx& cx, const PkArgs& pa, int bid, f32x4* red) {
  const int t = threadIdx.x, B = cx.B;
  const bool stem = bid >= R_TRUNK;
  const int chunk = stem ? bid - R_TRUNK : bid;
  const int slot = t & 63, grp = t >> 6, e0 = chunk * 256 + slot * 4;
  const float* src = stem ? cx.SSLAB : pa.tslab;
  const int stride = stem ? SSLAB_N : WSLAB_N, lim = stem ? SSLAB_N : WSLAB_N;
  // parameter index of each of this thread's 4 outputs (slab fragment order -> flat layout), -1 if none
  int pix[4];
  float pold[4];
#pragma unroll
  for (int ii = 0; ii < 4; ++ii) {
    const int e = e0 + ii;
    int pidx = -1;
    if (e < lim) {
      if (!stem) {
        const int tt = e >> 8, ln = (e >> 2) & 63, mt = tt & 1, nt = tt >> 1, tap = nt >> 1, cih = nt & 1;
        pidx = OFF_CONVW + (16 * mt + 4 * (ln >> 4) + ii) * 288 + (16 * cih + (ln & 15)) * 9 + tap;
      } else if (e < 1024) {
        const int tt = e >> 8, ln = (e >> 2) & 63, mt = tt & 1, nt = tt >> 1, k = 16 * nt + (ln & 15);
        if (k < 27) pidx = OFF_C1W + (16 * mt + 4 * (ln >> 4) + ii) * 27 + k;
      } else if (e < 1056) {
        pidx = OFF_C1B + (e - 1024);
      }
    }
    pix[ii] = pidx;
    pold[ii] = cx.params[pidx >= 0 ? pidx : 0];  // issued with the slab loads
  }
  f32x4 s = z4();
  {  // every load unconditional (clamped index), all in flight together; out-of-range ones are dropped after
    const int ec = e0 < lim ? e0 : lim - 4;
    f32x4 v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int k = grp + 4 * u;
      v[u] = ld4(src + (size_t)(k < B ? k : B - 1) * stride + ec);
    }
#pragma unroll
    for (int u = 0; u < 16; ++u)
      if (grp + 4 * u < B) s += v[u];
  }
  red[t] = s;
  __syncthreads();
  if (t < 64 && e0 < lim) {
    const f32x4 tot = red[t] + red[64 + t] + red[128 + t] + red[192 + t];
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      const int pidx = pix[ii];
      if (pidx < 0) continue;
      const float wv = sgd_put_pre(cx, pidx, tot[ii], pold[ii]);
      if (!cx.fuse_sgd) continue;
      if (pidx >= OFF_CONVW && pidx < OFF_CONVW + 9216) {
        const int r = pidx - OFF_CONVW, co = r / 288, ci = (r / 9) % 32, tap = r % 9;
        ((unsigned short*)cx.wt_f)[(tap * 32 + co) * 32 + ci] = bfbits(wv);
        ((unsigned short*)cx.wt_d)[((8 - tap) * 32 + ci) * 32 + co] = bfbits(wv);
      } else if (pidx >= OFF_C1W && pidx < OFF_C1W + 864) {
        const int r = pidx - OFF_C1W, co = r / 27, k = r % 27;
        const unsigned short wb = bfbits(wv);
        ((unsigned short*)cx.sw)[co * 32 + k] = wb;
        ((unsigned short*)cx.swf)[swf_slot(co, k)] = wb;
      }
    }
  }
  }

// dW1[j][64f .. 64f+63] = sum_b dh[b][j] * p[b][k] (+ SGD and the head's bf16 copy)
__device__ __forceinline__ void pk_red_fc1(const Ctx& cx, int f, float* stage) {
  const int t = threadIdx.x, B = cx.B;
  float* dh_s = stage;          // [B][32]
  float* p_s = stage + 64 * 32; // [B][64]
  f32x4 dh4[2], p4[4];
  const int j = t >> 3, kk = 8 * (t & 7);
  const int base = OFF_FC1W + j * 2048 + 64 * f + kk;
  const f32x4 o0 = ld4(cx.params + base), o1 = ld4(cx.params + base + 4);  // old weights, fetched early
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const int idx = t + 256 * m;
    dh4[m] = ld4(cx.HDH + 4 * (idx < B * 8 ? idx : 0));
  }
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int idx = t + 256 * m, ic = idx < B * 16 ? idx : 0, b = ic >> 4, k4 = ic & 15;
    p4[m] = ld4(cx.HP + (size_t)b * 2048 + 64 * f + 4 * k4);
  }
#pragma unroll
  for (int m = 0; m < 2; ++m)
    if (t + 256 * m < B * 8) st4(dh_s + 4 * (t + 256 * m), dh4[m]);
#pragma unroll
  for (int m = 0; m < 4; ++m)
    if (t + 256 * m < B * 16) st4(p_s + 4 * (t + 256 * m), p4[m]);
  __syncthreads();
  f32x4 a0 = z4(), a1 = z4();
#pragma unroll 8
  for (int b = 0; b < B; ++b) {
    const float dh = dh_s[b * 32 + j];
    a0 += dh * ld4(p_s + b * 64 + kk);
    a1 += dh * ld4(p_s + b * 64 + kk + 4);
  }
  st4(cx.grads + base, a0);
  st4(cx.grads + base + 4, a1);
  if (cx.fuse_sgd) {
    const f32x4 n0 = o0 - cx.lr * a0, n1 = o1 - cx.lr * a1;
    st4(cx.params + base, n0);
    st4(cx.params + base + 4, n1);
    *(uint4*)((unsigned short*)cx.w1b + base - OFF_FC1W) =
        uint4{pk2(n0[0], n0[1]), pk2(n0[2], n0[3]), pk2(n1[0], n1[1]), pk2(n1[2], n1[3])};
  }
  }

// fc1 bias, fc2 weight / bias gradients (+ SGD) from the head's per-image vectors
__device__ __forceinline__ void pk_red_fc_small(const Ctx& cx, float* stage) {
  const int t = threadIdx.x, B = cx.B;
  float* hh_s = stage;             // [B][32]
  float* dl_s = stage + 64 * 32;   // [B][16]
  float* dh_s = dl_s + 64 * 16;    // [B][32]
  {  // all loads first (clamped, unconditional), then the LDS stores
  float hv[8], dv[8], lv[3];
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const int idx = t + 256 * m, ic = idx < B * 32 ? idx : 0;
    hv[m] = cx.HH[ic];
    dv[m] = cx.HDH[ic];
  }
#pragma unroll
  for (int m = 0; m < 3; ++m) {
    const int idx = t + 256 * m;
    lv[m] = cx.HDL[idx < B * 10 ? idx : 0];
  }
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const int idx = t + 256 * m;
    if (idx < B * 32) {
      hh_s[idx] = hv[m];
      dh_s[idx] = dv[m];
    }
  }
#pragma unroll
  for (int m = 0; m < 3; ++m) {
    const int idx = t + 256 * m;
    if (idx < B * 10) dl_s[(idx / 10) * 16 + idx % 10] = lv[m];
  }
  }
  __syncthreads();
  for (int idx = t; idx < 32 + 320 + 10; idx += 256) {
  float s = 0.f;
  if (idx < 32) {
#pragma unroll 8
    for (int b = 0; b < B; ++b) s += dh_s[b * 32 + idx];
    sgd_put(cx, OFF_FC1B + idx, s);
  } else if (idx < 352) {
    const int o = (idx - 32) >> 5, jj = (idx - 32) & 31;
#pragma unroll 8
    for (int b = 0; b < B; ++b) s += dl_s[b * 16 + o] * hh_s[b * 32 + jj];
    sgd_put(cx, OFF_FC2W + o * 32 + jj, s);
  } else {
    const int o = idx - 352;
#pragma unroll 8
    for (int b = 0; b < B; ++b) s += dl_s[b * 16 + o];
    sgd_put(cx, OFF_FC2B + o, s);
  }
  }
}

// BN affine grads (+ SGD), loss, cursor, step count, num_batches_tracked, epoch, CC4 running-stat segment
__device__ __forceinline__ void pk_bookkeeping(const Ctx& cx, const PkArgs& pa, float* red) {
  const int t = threadIdx.x, B = cx.B;
  const float lo = cx.HLOSS[t < B ? t : 0];
  const float bg = pa.bng[t & 63];
  red[t] = t < B ? lo : 0.f;
  if (t < 64) sgd_put(cx, (t < 32 ? OFF_BNW : OFF_BNB) + (t & 31), bg);  // 0..31 dgamma, 32..63 dbeta
  __syncthreads();
  if (t == 0) {
    float s = 0.f;
    for (int k = 0; k < B; ++k) s += red[k];
    *cx.loss_acc += (double)(s / (float)B);
    *cx.cursor += B;
    *cx.step_count += 1;
    *cx.nbt += NBLK;  // BatchNorm num_batches_tracked: +1 per application
    *pa.epoch += 1;
  }
  if (!cx.fuse_sgd && t < 64) {
    const float v = t < 32 ? cx.rm[t] : cx.rv[t - 32];
    cx.grads[OFF_RS + t] = cx.rank == 0 ? v : 0.f;
  }
}

// Reduction + SGD after the persistent step.  with_fc = 1: grid R_GRID (trunk | stem | fc1 | bookkeeping incl.
// the small fc grads); with_fc = 0 (split mode, the fc part runs as k_pk_fc on the comm stream): grid
// R_TRUNK + R_STEM + 1.
__global__ void __launch_bounds__(256) k_pk_reduce(Ctx cx, PkArgs pa, int with_fc) {
  __shared__ f32x4 red[256];
  __shared__ float stage[64 * 32 + 64 * 64];
  const int bid = blockIdx.x;
  if (bid < R_TRUNK + R_STEM) {
    pk_red_trunk_stem(cx, pa, bid, red);
  } else if (with_fc && bid < R_TRUNK + R_STEM + R_FC) {
    pk_red_fc1(cx, bid - R_TRUNK - R_STEM, stage);
  } else {
    if (with_fc) pk_red_fc_small(cx, stage);
    __syncthreads();
    pk_bookkeeping(cx, pa, (float*)red);
  }
}

// Split mode: the fc gradients (bucket A, 86 % of the gradient bytes) as soon as the head has run, so their
// all-reduce overlaps the trunk backward.  Grid R_FC + 1.
__global__ void __launch_bounds__(256) k_pk_fc(Ctx cx) {
  __shared__ float stage[64 * 32 + 64 * 64];
  if (blockIdx.x < R_FC) pk_red_fc1(cx, blockIdx.x, stage);
  else pk_red_fc_small(cx, stage);
}

}  // namespace pk
}  // namespace dca
