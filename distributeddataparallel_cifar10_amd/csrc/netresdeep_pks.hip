// Image-sliced persistent NetResDeep training step for CDNA4 (gfx950 / MI355X): ONE launch per step, every image
// split over S = 4 workgroups of 4 image rows, so a batch of 32 runs on 128 CUs instead of the 32 of a
// one-workgroup-per-image design (rounds 1-2; retired).  A workgroup has 8 waves: wave (row w, channel half
// h) owns one image row and 16 of the 32 channels, so every latency-bound phase of a block is short.
//
//   stem (+ 1 halo pooled row each side, recomputed, no exchange) -> 10 forward blocks -> head -> 10 backward
//   blocks -> stem backward; then k_pks_reduce (slab reduction + SGD + bookkeeping).
//
// Cross-workgroup traffic, all as data-as-flag granules {tag, f32} written by ONE sc1 store (8 or 16 B) and read
// by sc1 loads (MI355X guide, Guideline 16 R2; no fences), double-buffered by round parity, every spin bounded:
//   * per block, one round: the 64 BatchNorm partial sums of every workgroup (all-to-all sweep) PLUS the two
//     boundary rows of the conv output (forward: y) or of the BN-masked gradient (backward: dz) for the
//     neighbouring slices' halos -- the halo rides in the same round, so slicing adds no extra hand-off latency;
//   * once, in the head: the 32 fc1 partial sums of the S slices of an image.
// The halo row of x is kept by the halo waves themselves (x_{i+1} = relu(bn(y_i)) + x_i needs only the neighbour's
// y_i row and the global BN statistics).  The backward recovers x_i = x_{i+1} - relu(bn(y_i)) (reversible
// residual) instead of storing every block input.
//
// Precision P: 0 = bf16 MFMA operands (fp32 accumulate, BatchNorm / loss / SGD in fp32); 1 = fp32-accurate
// "3xbf16": every operand a = a_hi + a_lo (two bf16), every product a_hi*b_hi + a_hi*b_lo + a_lo*b_hi on
// v_mfma_f32_16x16x32_bf16 (relative product error ~2^-17, not IEEE fp32 products), fc1 in plain fp32.  Measured
// against the plain-PyTorch fp32 oracle: <= 1e-5 per tensor (flip-aware), 8-step trajectory <= 1e-4.
//
// Element ownership (C layout of v_mfma_f32_16x16x32_bf16): thread (wave 4h + w, lane l = 16q + c) owns
//   pixel (image row 4s + w, col 4q + i), channel 16h + c   for i in {0..3}   (4 values)
// Global activations keep the tiled row layout [row][h][lane][i] (one f32x4 per thread and row).
//
// Reference semantics: model/resnet.py:5-37 (one shared ResBlock applied 10x, skip after the ReLU),
// main.py:27-39 (SGD, CrossEntropy mean), BatchNorm2d training statistics + 10 running-stat EMAs per forward.

namespace dca {
// stamps build: which forward / backward block gets the detailed stamps (slots 6 / 7)
#ifndef DCA_DETAIL_FWD
#define DCA_DETAIL_FWD 5
#endif
#ifndef DCA_DETAIL_BWD
#define DCA_DETAIL_BWD 5
#endif
namespace pks {

constexpr int S = 4;                   // workgroups (row slices) per image
constexpr int RS = 16 / S;             // image rows per slice
constexpr int NW = 2 * RS;             // waves per workgroup: (row, channel half)
constexpr int NTH = 64 * NW;           // threads per workgroup
constexpr int GSTR = 64 + 2 * 512;     // granules per workgroup per round: 64 (head partials) | top row | bottom row
constexpr int LMAX = 64 * S;           // logical workgroups (batch <= 64)
constexpr int NNT = (18 + NW - 1) / NW;  // wgrad tile columns (ci half x tap) per wave
constexpr int RND_HEAD = 10;           // rounds: 0..9 forward BN, 10 head (fc1 partials), 11..20 backward BN
constexpr unsigned SPIN_LIMIT = 1u << 17;
constexpr int RB = 64;                 // bf16 record: 32 channels, 16-B chunks swizzled (rec_chunk)
constexpr int cmax(int a, int b) { return a > b ? a : b; }

struct Args {
  unsigned long long* gran;  // [2][LMAX][GSTR] granules (halo rows, head partials)
  unsigned* bnx;             // [2][LMAX][64] BatchNorm partials, 4-byte self-tagged values (see bn_tag)
  unsigned long long* hdone; // [LMAX] head-done granules {tagof(epoch, RND_HDONE), 0} (fc workers' start signal)
  int* epoch;                // device scalar, advanced by the reduce kernel after every step
  unsigned* err;             // bit r: exchange round r timed out
  float* tslab;              // [LMAX][WSLAB_N] trunk wgrad per workgroup (fragment order, read by k_pks_reduce)
  float* bng;                // [64] dgamma | dbeta (written by logical workgroup 0)
  uint8_t* simg;             // [2][64][3072] batch images staged by the previous step (parity = epoch & 1)
  int* slab;                 // [2][64] their labels
  float* yh;                 // [10][LMAX][2][512] halo rows of y received in the forward (for the backward)
  float* c1;                 // debug: [B][32][32][32] conv1 pre-activation (NCHW), for the flip-aware oracle
  int debug;                 // also store X / DY / G / C1 for the numerical diagnostics
};

// ---- LDS plan (bytes; every region 16-byte aligned) ---------------------------------------------------------
template <int P>
struct Plan {
  static constexpr int NP = P + 1;                       // precision planes: hi (+ lo)
  static constexpr int O_CRED = 0;                       // [2][NW][64] f32 combine scratch
  static constexpr int O_STAT = O_CRED + 2 * NW * 64 * 4;  // [10][32] f32x4: mean, invstd, BN scale, shift of every
                                                         // block (one 16-B LDS read per channel in the backward)
  static constexpr int O_MISC = O_STAT + 5120;           // [1280] f32 step constants (layout: k_pks_step)
  static constexpr int O_U = O_MISC + 5120;              // phase union
  // trunk, forward and backward
  static constexpr int WT_PL = 288 * RB;                 // conv weight records [tap][co | ci] x 32
  static constexpr int U_WT = 0;
  static constexpr int XR_PL = (RS + 2) * 18 * RB;       // conv input records, rows -1..RS, cols -1..16
  static constexpr int U_XR = U_WT + NP * WT_PL;
  static constexpr int U_XR_END = U_XR + NP * XR_PL;
  static constexpr int DYT_S = RS * 16 + 8;              // dy, channel-major (wgrad A operand)
  static constexpr int DYT_PL = 32 * DYT_S * 2;
  static constexpr int U_DYT = U_XR_END;
  static constexpr int XT_S = (RS + 2) * 16 + 8;         // x, channel-major, 3 column-shifted copies
  static constexpr int XT_PL = 3 * 32 * XT_S * 2;
  static constexpr int U_XT = U_DYT + NP * DYT_PL;
  static constexpr int BWD_END = U_XT + NP * XT_PL;
  // stem (start of the step; WT and XR live)
  static constexpr int XIN_ROWS = 2 * RS + 6, XIN_COLS = 34;  // input rows 8s-3 .. 8s+10, cols -1..32
  static constexpr int XIN_PL = XIN_ROWS * XIN_COLS * 8;      // NHWC4 bf16 pixels
  static constexpr int U_XIN = U_XR_END;
  static constexpr int X0S = 36;
  static constexpr int U_X0 = U_XIN + NP * XIN_PL;             // [RS + 2][16][X0S] f32 pooled stem output
  static constexpr int U_SCODE = U_X0 + (RS + 2) * 16 * X0S * 4;  // [RS][16][32] u8 stem pool codes
  static constexpr int STEM_END = U_SCODE + RS * 16 * 32;
  // head (WT live -- it receives the dgrad weights meanwhile -- XR / dyT / xT free)
  static constexpr int X10S = 33;
  static constexpr int U_X10 = U_XR;                           // [RS][16][X10S] f32
  static constexpr int X10_BYTES = RS * 16 * X10S * 4;
  static constexpr int W1S = P == 1 ? 516 : 520;               // fc1 slice row stride (elements)
  static constexpr int W1_BYTES = 32 * W1S * (P == 1 ? 4 : 2); // [32 rows][512 local features] (f32 | bf16)
  static constexpr int U_W1 = (cmax(U_XR_END, U_X10 + X10_BYTES) + 15) / 16 * 16;
  static constexpr int U_PCODE = U_W1 + W1_BYTES;              // [512] u8 pool argmax
  static constexpr int U_DP = U_PCODE + 512;                   // [512] f32 dL/dpooled
  static constexpr int U_PL = U_DP + 2048;                     // [512] f32 pooled features
  static constexpr int U_HP = U_PL + 2048;                     // [32] fc1 partials | [32, 64) dh
  static constexpr int HEAD_END = U_HP + 256;
  // stem backward (WT / XR free)
  static constexpr int DSP = 2 * RS * 32 + 8;                  // d(conv1 out), channel-major, own conv rows
  static constexpr int DST_PL = 32 * DSP * 2;
  static constexpr int U_DST = 0;
  static constexpr int XSR = 2 * RS + 2;                       // input rows 8s-1 .. 8s+8
  static constexpr int XS_S = 40;
  static constexpr int XS_PL = 9 * XSR * XS_S * 2;             // [3 kw][3 ci][XSR][XS_S] shifted input copies
  static constexpr int U_XS = U_DST + NP * DST_PL;
  static constexpr int U_SRED = U_XS + NP * XS_PL;             // [NW][64][4] f32 stem-wgrad partials (written
                                                               // after the barrier that retires the last wgrad)
  static constexpr int SBWD_END = U_SRED + NW * 64 * 16;
  static constexpr int UNION = cmax(cmax(BWD_END, STEM_END), cmax(HEAD_END, SBWD_END));
  static constexpr int TOTAL = O_U + UNION;
};
static_assert(Plan<1>::TOTAL <= 160 * 1024, "LDS budget");
static_assert(Plan<0>::U_W1 >= Plan<0>::U_X10 + Plan<0>::X10_BYTES, "x10 clear of the fc1 slice");
// dsT / xs are written while other waves may still run the last wgrad (dyT / xT); SRED only after the barrier
static_assert(Plan<0>::U_SRED <= Plan<0>::U_DYT, "stem-backward staging clear of dyT / xT (last wgrad)");
static_assert(Plan<1>::U_SRED <= Plan<1>::U_DYT, "stem-backward staging clear of dyT / xT (last wgrad)");

// ---- helpers ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ __forceinline__ void pin(float& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void pin(unsigned& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void pin(int& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void pin(uint2& x) { asm volatile("" : "+v"(x.x), "+v"(x.y)); }
__device__ __forceinline__ void pin(uint4& x) { asm volatile("" : "+v"(x.x), "+v"(x.y), "+v"(x.z), "+v"(x.w)); }

typedef unsigned v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned short bf_lo(float v, unsigned short hi) {
  return bfbits(v - __uint_as_float((unsigned)hi << 16));
}
// Record layout of the conv operands (inputs XR, weights WT): record r = 32 bf16 channels = four 16-B chunks; chunk
// q of record r sits at chunk position q ^ 2((r >> 2) & 1).  An MFMA operand read (ds_read_b128, lane 16q + c
// reads chunk q of record base + c) then touches 16 distinct 16-B bank groups in each of the instruction's four
// 16-lane groups, for ANY base (an unswizzled record stride cannot: 80-B records conflicted 2-way).
__device__ __forceinline__ int rec_chunk(int rec, int q) { return ((rec << 6) | (q << 4)) ^ ((rec & 4) << 3); }
__device__ __forceinline__ int rec_elem(int rec, int ch) { return rec_chunk(rec, ch >> 3) + ((ch & 7) << 1); }
// one value into channel `ch` of record `rec` (both planes)
template <int P>
__device__ __forceinline__ void st1r(char* xr, int plane, int rec, int ch, float v) {
  const unsigned short hi = bfbits(v);
  const int o = rec_elem(rec, ch);
  *(unsigned short*)(xr + o) = hi;
  if constexpr (P == 1) *(unsigned short*)(xr + plane + o) = bf_lo(v, hi);
}
template <int P>
__device__ __forceinline__ f32x4 mma3(const bf16x8& ah, const bf16x8& al, const bf16x8& bh, const bf16x8& bl,
                                      f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc, 0, 0, 0);
  if constexpr (P == 1) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc, 0, 0, 0);
  }
  return acc;
}
template <int P>
__device__ __forceinline__ f32x4 mma3s(const s4v& ah, const s4v& al, const s4v& bh, const s4v& bl, f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ah, bh, acc, 0, 0, 0);
  if constexpr (P == 1) {
    acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ah, bl, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(al, bh, acc, 0, 0, 0);
  }
  return acc;
}

// The B fragments of one conv weight (9 taps, lane 16q + c: record tap*32 + 16h + c, chunk q).  P = 0 keeps them
// in registers for a whole pass (forward / backward): the conv then reads only its A operand from LDS.
__device__ __forceinline__ int wrec_off(int h, int lane) {
  return rec_chunk(16 * h + (lane & 15), lane >> 4);  // + tap * 32 * RB (a multiple of 8 records: same swizzle)
}
__device__ __forceinline__ void load_bfrag(const char* wt, int h, int lane, bf16x8 (&bw)[9]) {
  const char* bb = wt + wrec_off(h, lane);
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) bw[tap] = *(const bf16x8*)(bb + tap * 32 * RB);
}
// 3x3 conv of one output row (slice row w), output channels 16h .. 16h+15, on MFMA.  xr: (RS+2) x 18 records,
// wt: 288 records (tap-major); P=1 reads the lo planes at +XR_PL / +WT_PL and the B operands from LDS, P=0 takes
// its B operands from registers (bw).
template <int P>
__device__ __forceinline__ f32x4 conv_row(const char* xr, const char* wt, const bf16x8 (&bw)[9], int w, int h,
                                          int lane) {
  using PL = Plan<P>;
  const int c = lane & 15, q = lane >> 4;
  const char* bbase = wt + wrec_off(h, lane);
  f32x4 acc = z4();
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int kh = tap / 3, kw = tap % 3;
    const int ao = rec_chunk((w + kh) * 18 + kw + c, q);
    const bf16x8 a = *(const bf16x8*)(xr + ao);
    bf16x8 b, bl, al = a;
    if constexpr (P == 1) {
      b = *(const bf16x8*)(bbase + tap * 32 * RB);
      bl = *(const bf16x8*)(bbase + PL::WT_PL + tap * 32 * RB);
      al = *(const bf16x8*)(xr + PL::XR_PL + ao);
    } else {
      b = bw[tap];
      bl = b;
    }
    acc = mma3<P>(a, al, b, bl, acc);
  }
  return acc;
}

// a + a[lane ^ 16], then + the same of lane ^ 32: the value every lane of a 16-lane column group ends with, summed in
// the order of two __shfl_xor steps (bitwise the same; fp addition is commutative) but on the gfx950 cross-row VALU
// swaps (v_permlane16_swap / v_permlane32_swap) instead of two dependent ds_bpermute LDS round trips
__device__ __forceinline__ float xsum_rows(float a) {
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(a), false, false);
  a = __uint_as_float(p[0]) + __uint_as_float(p[1]);
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(a), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// sum over the 16 lanes of a row, every lane ending with it: the xor-1 / 2 / 4 / 8 butterfly of __shfl_xor (the same
// pairings, so bitwise the same sums) on DPP lane moves -- quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror,
// row_mirror -- instead of four dependent ds_bpermute round trips
__device__ __forceinline__ float xsum_row16(float a) {
  a += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(a), 0xB1, 0xF, 0xF, false));
  a += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(a), 0x4E, 0xF, 0xF, false));
  a += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(a), 0x141, 0xF, 0xF, false));
  a += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(a), 0x140, 0xF, 0xF, false));
  return a;
}

// per-workgroup channel sums of per-thread partials (a, b: channel 16h + c of wave 4h + w), delivered to the
// publishing threads: thread t < 64 returns slot t (t < 32: sum of a for channel t, else sum of b for channel
// t - 32).  One LDS barrier.
// FRESH: re-derive the thread's LDS offsets here (an opaque copy of threadIdx.x) instead of letting the compiler keep
// them live from the kernel's start -- the stem backward's call is the only use after the 20 blocks, and holding its
// address through them spilled a VGPR to scratch.
template <bool FRESH = false>
__device__ __forceinline__ float wg_csum(float a, float b, float* cred) {
  int t = threadIdx.x;
  if constexpr (FRESH) asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"(t));
  const int wv = t >> 6, lane = t & 63, c = lane & 15;
  a = xsum_rows(a);
  b = xsum_rows(b);
  // [2 halves][32: a | b of 16 channels][RS rows], disjoint from the sweep combine area: a publishing thread reads
  // its RS row partials as one 16-B LDS read (summed in row order)
  float* r = cred + NW * 64;
  if (lane < 16) {
    r[((wv / RS) * 32 + c) * RS + wv % RS] = a;
    r[((wv / RS) * 32 + 16 + c) * RS + wv % RS] = b;
  }
  lds_barrier();
  float v = 0.f;
  if (t < 64) {
    const int ch = t & 31, hh = ch >> 4, off = (t >> 5) * 16 + (ch & 15);
    const f32x4 x = *(const f32x4*)(r + (hh * 32 + off) * RS);
    v = x[0];
    v += x[1];
    v += x[2];
    v += x[3];
  }
  return v;
}

// The step epoch (device scalar) runs 0 .. EPOCH_WRAP - 1 and wraps (pks_bookkeeping): EPOCH_WRAP is a multiple of 6,
// so the epoch parity (staging) and the bn_tag cycle (epoch mod 3) continue seamlessly across the wrap, and
// epoch * 64 + round + 1 < 2^32 never overflows (unsigned arithmetic throughout: no signed-overflow UB after hours of
// stepping).  Consecutive epochs -- the only ones a granule can hold -- still give distinct tags at the wrap.
constexpr unsigned EPOCH_WRAP = 6u << 23;
static_assert((unsigned long long)EPOCH_WRAP * 64 + 64 < (1ull << 32), "granule tags fit 32 bits");
__device__ __forceinline__ unsigned tagof(int epoch, int round) {
  return (unsigned)epoch * 64u + (unsigned)round + 1u;
}
__device__ __forceinline__ unsigned long long* gslot(const Args& pa, int round, int L) {
  return pa.gran + ((size_t)(round & 1) * LMAX + L) * GSTR;
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t grsrc(const Args& pa, int round) {
  return __builtin_amdgcn_make_buffer_rsrc(pa.gran + (size_t)(round & 1) * LMAX * GSTR, (short)0,
                                           LMAX * GSTR * 8, 0x00020000);
}
// one granule, one sc1 store
__device__ __forceinline__ void gput(unsigned long long* g, unsigned tag, float v) {
  __hip_atomic_store(g, ((unsigned long long)tag << 32) | __float_as_uint(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
// publish this lane's 4 values (channel half h) of a boundary row (which: 0 = my top row, 1 = my bottom row):
// 2 x 16-B sc1 stores, each holding two whole granules
__device__ __forceinline__ void publish_row(const Args& pa, int round, int L, int which, int h, unsigned tag,
                                            const float (&v)[4], int lane) {
  const __amdgpu_buffer_rsrc_t rs = grsrc(pa, round);
  const int base = (L * GSTR + 64 + which * 512 + h * 256 + lane * 4) * 8;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const v4u x = v4u{__float_as_uint(v[2 * p]), tag, __float_as_uint(v[2 * p + 1]), tag};
    __builtin_amdgcn_raw_buffer_store_b128(x, rs, base + 2 * p * 8, 0, 16);
  }
}

// BatchNorm partials travel as 4-byte self-tagged fp32 values: the 2 low mantissa bits of every value carry the
// tag (a <= 3 ulp perturbation of a partial sum, identical for every reader), so one 16-B sc1 load returns four
// validated values -- half the bytes per sweep pass of {value, tag} granules (profiles/bnx_variants_r3.log: 1.73 vs
// 2.05 us per exchange round at 128 workgroups).  Slot parity = round & 1; consecutive writes of a slot carry
// consecutive tags of the cycle 1, 2, 3 (each parity is written 10 times per step: c = 10 epoch + k, tag =
// 1 + c mod 3), so a reader can never accept the previous write; 0 never matches (the host zeroes the buffer
// whenever the batch size changes, so slots of workgroups absent from earlier steps are never stale-valid).
// (10 epoch + k) mod 3 = (epoch mod 3 + k) mod 3, in unsigned arithmetic (EPOCH_WRAP % 3 == 0 keeps the cycle).
__host__ __device__ __forceinline__ unsigned bn_tag(int epoch, int rnd) {
  const unsigned k = rnd < RND_HEAD ? (unsigned)rnd >> 1 : 5u + ((unsigned)(rnd - RND_HEAD - 1) >> 1);
  return 1u + ((unsigned)epoch % 3u + k) % 3u;
}
static_assert(EPOCH_WRAP % 6 == 0, "epoch wrap keeps parity and the bn_tag cycle");
__device__ __forceinline__ void bn_put(const Args& pa, int rnd, int L, int slot, unsigned tag, float v) {
  __hip_atomic_store(pa.bnx + ((size_t)(rnd & 1) * LMAX + L) * 64 + slot, (__float_as_uint(v) & ~3u) | tag,
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// BN sweep: lane 16 sub + q4 of wave wv reads slots 4 q4 .. 4 q4 + 3 of workgroups 4 wv + sub + 32 k (one 16-B sc1
// load), k < KS.  A pass re-reads only the loads whose four values were not all valid yet (per lane: exec-masked;
// per wave: skipped once no lane needs it), so after the first pass the polling traffic is the stragglers' slots
// only and every later pass is a short round trip.  The values are summed once at the end, in k order: the same
// sums in every workgroup, whatever order they arrived in.
__device__ __forceinline__ void sleep_units(int n) {
  for (int k = 0; k < n; ++k) __builtin_amdgcn_s_sleep(1);  // 64 cycles each
}
// Halo waves poll the neighbour slice's boundary row (2 x 16-B sc1 loads of {value, tag} granules) in the SAME
// passes (need bit 8 .. 9): its data arrive with the BN partials instead of costing one more round trip after them.
template <int KS>
__device__ __forceinline__ void sweep_wait(const Args& pa, int round, int wv, int lane, int G, unsigned tag,
                                           float (&sv)[4], bool halo, int Lsrc, int which, int h, unsigned htag,
                                           float (&hv)[4]) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(pa.bnx + (size_t)(round & 1) * LMAX * 64,
                                                                      (short)0, LMAX * 64 * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rh = grsrc(pa, round);
  const int hbase = (Lsrc * GSTR + 64 + which * 512 + h * 256 + lane * 4) * 8;
  const int q4 = lane & 15, sub = lane >> 4;
  v4u xa[KS], xh[2];
  unsigned need = 0;  // bit k: load k of this lane still lacks a valid value; bits 8, 9: the halo row
#pragma unroll
  for (int k = 0; k < KS; ++k) {
    xa[k] = v4u{0u, 0u, 0u, 0u};
    if (4 * wv + sub + 4 * NW * k < G) need |= 1u << k;
  }
  xh[0] = xh[1] = v4u{0u, 0u, 0u, 0u};
  if (halo) need |= 3u << 8;
  for (unsigned spins = 0;; ++spins) {
    asm volatile("" ::: "memory");  // re-issued every pass (never hoisted out of the spin)
#pragma unroll
    for (int p = 0; p < 2; ++p)
      if (need & (1u << (8 + p))) xh[p] = __builtin_amdgcn_raw_buffer_load_b128(rh, hbase + 2 * p * 8, 0, 16);
#pragma unroll
    for (int k = 0; k < KS; ++k)
      if (need & (1u << k))
        xa[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, ((4 * wv + sub + 4 * NW * k) * 64 + 4 * q4) * 4, 0, 16);
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      const bool ok = (xa[k][0] & 3u) == tag && (xa[k][1] & 3u) == tag && (xa[k][2] & 3u) == tag &&
                      (xa[k][3] & 3u) == tag;
      if (ok) need &= ~(1u << k);
    }
#pragma unroll
    for (int p = 0; p < 2; ++p)
      if (xh[p][1] == htag && xh[p][3] == htag) need &= ~(1u << (8 + p));
    if (__all(need == 0)) break;  // (re-issued at once: any sleep between passes measured slower)
    if (spins >= SPIN_LIMIT) {
      if (lane == 0) atomicOr(pa.err, 1u << (round & 31));
      break;
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) sv[e] = 0.f;
#pragma unroll
  for (int k = 0; k < KS; ++k) {
    const bool valid = 4 * wv + sub + 4 * NW * k < G;
#pragma unroll
    for (int e = 0; e < 4; ++e) sv[e] += valid ? __uint_as_float(xa[k][e]) : 0.f;
  }
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    hv[2 * p] = __uint_as_float(xh[p][0]);
    hv[2 * p + 1] = __uint_as_float(xh[p][2]);
  }
}
// All-to-all BN exchange wait + (halo waves) the neighbour's boundary row.  On return cred[0 .. NW*64) holds every
// wave's partial totals slot-major (the caller's barrier makes them visible): tot(slot) = sum_k cred[slot * NW + k],
// two 16-B LDS reads per slot.  (A conflict-free one-write-per-lane form, wave k of a slot at position k ^ (slot >> 3),
// sums in a slot-dependent order: it moved the fp32 flip-aware batch-64 check past its 1e-4 bound, so not used.)
__device__ __forceinline__ void xchg_wait(const Args& pa, int round, int epoch, int G, float* cred, bool halo,
                                          int Lsrc, int which, int h, float (&hv)[4]) {
  const int t = threadIdx.x, lane = t & 63;
  const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
  const unsigned tag = tagof(epoch, round);
  float sv[4];
  const unsigned btag = bn_tag(epoch, round);
  if (G <= 4 * NW) sweep_wait<1>(pa, round, wv, lane, G, btag, sv, halo, Lsrc, which, h, tag, hv);
  else if (G <= 8 * NW) sweep_wait<2>(pa, round, wv, lane, G, btag, sv, halo, Lsrc, which, h, tag, hv);
  else if (G <= 16 * NW) sweep_wait<4>(pa, round, wv, lane, G, btag, sv, halo, Lsrc, which, h, tag, hv);
  else sweep_wait<8>(pa, round, wv, lane, G, btag, sv, halo, Lsrc, which, h, tag, hv);
#pragma unroll
  for (int e = 0; e < 4; ++e) {  // the four 16-lane groups read different workgroups
    sv[e] = xsum_rows(sv[e]);
  }
  if (lane < 16) {
#pragma unroll
    for (int e = 0; e < 4; ++e) cred[(4 * lane + e) * NW + wv] = sv[e];
  }
}
__device__ __forceinline__ float slot_total(const float* cred, int slot) {
  static_assert(NW == 8 && RS == 4, "slot-major combine layout: 8 waves, 4 rows");
  const f32x4 u = *(const f32x4*)(cred + slot * NW), w = *(const f32x4*)(cred + slot * NW + 4);
  float a = u[0];  // wave order, as the per-wave sums were added before
  a += u[1];
  a += u[2];
  a += u[3];
  a += w[0];
  a += w[1];
  a += w[2];
  a += w[3];
  return a;
}

// this thread's 4 values of one image row in the tiled global layout [h][lane][i]
// Write-through (sc1) 16-B store: the line leaves the XCD's L2 instead of staying dirty there.  Used for the bulk
// data this kernel writes (per-block y, halo rows, weight-gradient slabs, pooled features, the next batch): dirty
// L2 lines are written back at the kernel boundary (MI355X guide "boundary": + dirty bytes / ~6 TB/s), ~15 MB
// per step here, which the following reduction kernel would wait for.
__device__ __forceinline__ void st4_wt(void* p, f32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st2_wt(float* p, float a, float b) {
  typedef float f2_ __attribute__((ext_vector_type(2)));
  asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(p), "v"(f2_{a, b}) : "memory");
}
__device__ __forceinline__ void st1_wt(float* p, float v) {
  __hip_atomic_store((unsigned*)p, __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st4r_wt(float* rowp, int h, int lane, const float (&v)[4]) {
  st4_wt(rowp + h * 256 + lane * 4, f32x4{v[0], v[1], v[2], v[3]});
}
__device__ __forceinline__ void st4r(float* rowp, int h, int lane, const float (&v)[4]) {
  *(f32x4*)(rowp + h * 256 + lane * 4) = f32x4{v[0], v[1], v[2], v[3]};
}
__device__ __forceinline__ void ld4r(const float* rowp, int h, int lane, float (&v)[4]) {
  const f32x4 u = *(const f32x4*)(rowp + h * 256 + lane * 4);
  v[0] = u[0];
  v[1] = u[1];
  v[2] = u[2];
  v[3] = u[3];
}

// wgrad of one application, accumulated in registers: D[co][ci,tap] += sum over this slice's pixels of
// dy[p][co] x[p + tap][ci].  Wave wv owns tile columns nt = wv, wv + NW, ... (ci half x tap), both co halves; K
// steps of 32 pixels = two image rows.
template <int P>
__device__ __forceinline__ void wgrad_acc(const unsigned short* dyT, const unsigned short* xT, f32x4 (&wacc)[NNT][2],
                                          int wv, int lane) {
  using PL = Plan<P>;
  const int c = lane & 15, q = lane >> 4;
  constexpr int DYO = PL::DYT_PL / 2, XTO = PL::XT_PL / 2;  // lo-plane offsets (elements)
#pragma unroll
  for (int s = 0; s < RS / 2; ++s) {
    const int row = 2 * s + (q >> 1), c0 = 8 * (q & 1);
    const int ao0 = c * PL::DYT_S + row * 16 + c0, ao1 = (16 + c) * PL::DYT_S + row * 16 + c0;
    const bf16x8 a0 = *(const bf16x8*)(dyT + ao0);
    const bf16x8 a1 = *(const bf16x8*)(dyT + ao1);
    bf16x8 a0l = a0, a1l = a1;
    if constexpr (P == 1) {
      a0l = *(const bf16x8*)(dyT + DYO + ao0);
      a1l = *(const bf16x8*)(dyT + DYO + ao1);
    }
#pragma unroll
    for (int j = 0; j < NNT; ++j) {
      const int nt = wv + NW * j;
      if (nt < 18) {
        const int tap = nt >> 1, cih = nt & 1, kh = tap / 3, kw = tap % 3;
        const int bo = (kw * 32 + 16 * cih + c) * PL::XT_S + (row + kh) * 16 + c0;
        const bf16x8 b = *(const bf16x8*)(xT + bo);
        bf16x8 bl = b;
        if constexpr (P == 1) bl = *(const bf16x8*)(xT + XTO + bo);
        wacc[j][0] = mma3<P>(a0, a0l, b, bl, wacc[j][0]);
        wacc[j][1] = mma3<P>(a1, a1l, b, bl, wacc[j][1]);
      }
    }
  }
}
// one lane's 4 consecutive columns (4q .. 4q+3) of x, channel ch, into the three column-shifted copies of xT row
// `xrow` (copy kw holds x[col + kw - 1] at col)
__device__ __forceinline__ void xt_put(unsigned short* xT, int XT_S, int xrow, int ch, int q, unsigned b0, unsigned b1,
                                       unsigned b2, unsigned b3) {
  const int rowoff = xrow * 16 + 4 * q;
  unsigned short* p1 = xT + (32 + ch) * XT_S + rowoff;
  *(uint2*)p1 = uint2{b0 | (b1 << 16), b2 | (b3 << 16)};
  unsigned short* p0 = xT + ch * XT_S + rowoff;
  p0[1] = (unsigned short)b0;
  *(unsigned*)(p0 + 2) = b1 | (b2 << 16);
  if (q < 3) p0[4] = (unsigned short)b3;
  unsigned short* p2 = xT + (64 + ch) * XT_S + rowoff;
  if (q > 0) p2[-1] = (unsigned short)b0;
  *(unsigned*)p2 = b1 | (b2 << 16);
  p2[2] = (unsigned short)b3;
}
template <int P>
__device__ __forceinline__ void xt_row(unsigned short* xT, int xrow, int q, int ch, const float (&x)[4]) {
  using PL = Plan<P>;
  unsigned hb[4], lb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const unsigned short hi = bfbits(x[i]);
    hb[i] = hi;
    lb[i] = P == 1 ? bf_lo(x[i], hi) : 0u;
  }
  xt_put(xT, PL::XT_S, xrow, ch, q, hb[0], hb[1], hb[2], hb[3]);
  if constexpr (P == 1) xt_put(xT + PL::XT_PL / 2, PL::XT_S, xrow, ch, q, lb[0], lb[1], lb[2], lb[3]);
}
// this lane's 4 records-entries (channel ch, cols 4q .. 4q+3) of XR row `xrow`
template <int P>
__device__ __forceinline__ void xr_row(char* XR, int xrow, int q, int ch, const float (&v)[4]) {
  using PL = Plan<P>;
#pragma unroll
  for (int i = 0; i < 4; ++i) st1r<P>(XR, PL::XR_PL, xrow * 18 + 4 * q + i + 1, ch, v[i]);
}

// weight staging: the NP planes (hi, lo) of one conv weight, stored in global memory in the LDS record layout
// (common.h PKW_*), copied into WT by LDS-DMA -- no registers, no scratch; the issuing waves' vmcnt covers it.
// 1 KB per wave instruction, chunks dealt round-robin to the waves; P = 0's 22.5 KB end in a half chunk.
template <int P>
__device__ __forceinline__ void wt_dma(char* wt, const unsigned short* src, int wv, int lane) {
  constexpr int BYTES = (P + 1) * PKW_PLANE * 2, NCH = (BYTES + 1023) / 1024;
  static_assert(BYTES == (P + 1) * Plan<P>::WT_PL, "record layout of pkw matches the LDS weight planes");
#pragma unroll
  for (int m = 0; m < (NCH + NW - 1) / NW; ++m) {
    const int ck = wv + NW * m;
    if (ck < NCH && ck * 1024 + lane * 16 < BYTES)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)((const char*)src + ck * 1024 + lane * 16),
                                       (__attribute__((address_space(3))) void*)(wt + ck * 1024), 16, 0, 0);
  }
}
// The same planes when the prologue reduction wrote them in this launch: sc1 16-B buffer loads into registers, then
// LDS stores (the guide's validated consumer form; LDS-DMA is not one of them)
template <int P>
__device__ __forceinline__ void wt_copy_sc1(char* wt, const unsigned short* src) {
  constexpr int BYTES = (P + 1) * PKW_PLANE * 2, N16 = BYTES / 16, R = (N16 + NTH - 1) / NTH;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, BYTES, 0x00020000);
  v4u v[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int idx = (int)threadIdx.x + NTH * r;
    v[r] = __builtin_amdgcn_raw_buffer_load_b128(rs, (idx < N16 ? idx : 0) * 16, 0, 16);
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int idx = (int)threadIdx.x + NTH * r;
    if (idx < N16) *(v4u*)(wt + idx * 16) = v[r];
  }
}
// conv1 B fragment of MFMA m (taps 4m + q), channel half h for this lane, plane p, from the fp32 weights (sc1 dword
// loads: written in this launch by the prologue reduction) -- the swf_slot record the next launches read from pkw
template <int P>
__device__ __forceinline__ uint2 stem_bfrag_sc1(const Ctx& cx, int p, int h, int m, int lane) {
  const int co = 16 * h + (lane & 15), tap = 4 * m + (lane >> 4);
  unsigned short u[3];
#pragma unroll
  for (int ci = 0; ci < 3; ++ci) {
    const float x = tap < 9 ? __hip_atomic_load(cx.params + OFF_C1W + co * 27 + ci * 9 + tap, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT) : 0.f;
    const unsigned short hi = bfbits(x);
    u[ci] = p == 0 ? hi : bf_lo(x, hi);
  }
  return uint2{(unsigned)u[0] | ((unsigned)u[1] << 16), (unsigned)u[2]};
}

// fc1 slice of slice s: 32 rows x 512 local features (u = ch*16 + pr*8 + pw <-> global ch*64 + (2s + pr)*8 + pw),
// row j at w1l + j * W1S elements; one lane-linear 1 KB LDS-DMA per bf16 row (P=0) / half f32 row (P=1)
template <int P>
__device__ __forceinline__ void w1_dma(const Ctx& cx, char* w1l, int s, int wv, int lane) {
  constexpr int IPR = P == 1 ? 2 : 1, NI = 32 * IPR / NW;
#pragma unroll
  for (int m = 0; m < NI; ++m) {
    const int ins = wv * NI + m, j = ins / IPR, h = ins % IPR;
    const void* src;
    if constexpr (P == 1) {
      const int u = 256 * h + 4 * lane;
      src = cx.params + OFF_FC1W + j * 2048 + (u >> 4) * 64 + (2 * s + ((u >> 3) & 1)) * 8 + (u & 7);
    } else {
      const int u = 8 * lane;
      src = (const unsigned short*)cx.w1b + j * 2048 + (u >> 4) * 64 + (2 * s + ((u >> 3) & 1)) * 8;
    }
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(w1l + j * Plan<P>::W1S * (P == 1 ? 4 : 2) + h * 1024),
                                     16, 0, 0);
  }
}

// ============================================================================================================
// Gradient segments: reduction + gradient all-reduce + SGD.  Every segment is one slice of the gradient: a 64-element
// chunk of the trunk conv or of conv1 (slab fragment order, summed over the B x S workgroup slabs), a 16-row x
// 64-feature block of fc1 (1024), the fc tail (fc1 bias, fc2 weight and bias; 362) or the BN tail (BN affine and
// the CC4 running-stat segment; 128).  A segment is
//   mode 0 (world size 1): reduced, then SGD (fused);
//   mode 1 (RCCL): reduced and written to the gradient only (ncclAllReduce + k_apply_sgd follow in the graph);
//   mode 2 (xGMI): reduced, exchanged one-shot with the peers (write-through slab + per-segment flags in the second
//     half of every rank's IPC region, peers read all W slabs, sum in rank order -- bitwise identical on every
//     rank), then the averaging SGD: ~227 concurrent small all-reduces instead of one all-reduce launch after the
//     reduction (reference: DDP's single NCCL bucket after the whole backward, main.py:63);
//   mode 3: the same exchange on a caller pattern (collective self-test of this path).
// The fc1 blocks and the fc tail are final after the head: with `fc_in_step` the step kernel runs them on 65
// extra workgroups ("fc workers", on CUs the 128 step workgroups leave idle) beside the trunk backward --
// including their xGMI exchange, i.e. 86.6 % of the gradient bytes all-reduced while the backward runs (the
// reference's DDP bucket becomes ready only after the last backward op: zero overlap).  k_pks_reduce_ar
// then handles the trunk, conv1 and BN-tail segments.
// Memory ordering as in xgmi_allreduce.hip (system-coherent stores to uncached memory, s_waitcnt vmcnt(0) +
// barrier before the flag, cache-bypassing loads; per-segment epochs, slab parity = epoch & 1).
// ============================================================================================================
// Segment layout, chosen per launch: trunk / conv1 chunks of `ch` = 64 elements (B x S slabs of 256 B per
// workgroup; 227 segments) or 256 (41 chunks, 107 segments: the layout for ranks sharing one device, whose reduction
// grid must leave room for another rank's step kernel -- a CU holding a reduction workgroup has too few VGPRs left
// for a step workgroup).  256-element chunks read 128 KB through one CU (3.9 us, profiles/stamps_pks_bf16_r3f.log).
constexpr int R_FC1 = 64;
// LDS staging of the fc segments at batch B: fc1 block dh [B][32] + p [B][64]; fc tail h [B][32] + dlogits [B][16]
// + dh [B][32].  Sized per launch (dynamic LDS of k_pks_reduce_ar): the reduction grids of ranks sharing a device
// spin side by side and must leave a step workgroup's LDS free on every CU.
__host__ __device__ constexpr int stage_floats(int B) { return B * 96; }
constexpr int FCT_LEN = 364, BNT_LEN = 128;        // fc tail 362 (+2 pad), BN tail
constexpr int SEG_MAX = 1024;
constexpr int NSEG_MAX = WSLAB_N / 64 + (SSLAB_N + 63) / 64 + R_FC1 + 2;  // 227: flag-array stride per rank
constexpr int N_FCW = R_FC1 + 1;                   // fc workers of the step kernel
constexpr int RND_HDONE = 30;                      // tag round of the head-done granules (fc workers' start)
struct SegLayout {
  int ch, r_trunk, r_ts, fct, bnt, nseg, off_fc1, off_fct, off_bnt;
};
__host__ __device__ constexpr SegLayout seg_layout(int ch) {
  return SegLayout{ch,
                   WSLAB_N / ch,
                   WSLAB_N / ch + (SSLAB_N + ch - 1) / ch,
                   WSLAB_N / ch + (SSLAB_N + ch - 1) / ch + R_FC1,
                   WSLAB_N / ch + (SSLAB_N + ch - 1) / ch + R_FC1 + 1,
                   WSLAB_N / ch + (SSLAB_N + ch - 1) / ch + R_FC1 + 2,
                   (WSLAB_N / ch + (SSLAB_N + ch - 1) / ch) * ch,
                   (WSLAB_N / ch + (SSLAB_N + ch - 1) / ch) * ch + R_FC1 * 1024,
                   (WSLAB_N / ch + (SSLAB_N + ch - 1) / ch) * ch + R_FC1 * 1024 + FCT_LEN};
}
static_assert(WSLAB_N % 256 == 0, "trunk slab splits into whole chunks");
static_assert(seg_layout(64).nseg == NSEG_MAX && seg_layout(128).nseg <= NSEG_MAX && seg_layout(256).nseg <= NSEG_MAX,
              "flag stride");
static_assert(seg_layout(128).off_bnt + BNT_LEN >= FLAT_N && seg_layout(128).off_bnt + BNT_LEN <= (int)xg::SLAB_FLOATS,
              "the 128-element layout covers the flat buffer and fits one slab");
static_assert((size_t)NSEG_MAX * xg::MAXR * 4 <= xg::FLAG_BYTES, "one flag per segment and rank");
static_assert(seg_layout(64).off_bnt + BNT_LEN >= FLAT_N && seg_layout(256).off_bnt + BNT_LEN >= FLAT_N &&
                  seg_layout(256).off_bnt + BNT_LEN <= (int)xg::SLAB_FLOATS,
              "segments cover the flat buffer (self-test) and fit one slab");
__device__ __forceinline__ int seg_off(const SegLayout& G, int b) {
  return b < G.r_ts ? b * G.ch : b < G.fct ? G.off_fc1 + (b - G.r_ts) * 1024 : b == G.fct ? G.off_fct : G.off_bnt;
}
__device__ __forceinline__ int seg_len(const SegLayout& G, int b) {
  return b < G.r_ts ? G.ch : b < G.fct ? 1024 : b == G.fct ? FCT_LEN : BNT_LEN;
}

struct RedAr {
  xg::Peers peers;            // every rank's IPC region; the segments use its SECOND half (xg::REGION_BYTES on)
  unsigned* err;              // bit 31: a peer wait expired
  unsigned long long deadline;  // s_memrealtime ticks
  const float* st_src;        // mode 3: the pattern (st_n floats, slab offsets)
  float* st_dst;
  int st_n;
  int mode;
  int fc_in_step;             // flags (ra_fc / ra_prev / ra_s / ra_chunk): bit 0 the fc1 / fc-tail segments run on
                              // the step kernel's fc workers; bit 1 (step kernel) the prologue reduction of the
                              // previous step runs in this launch; bits 8..15 the step's index s in its chunk;
                              // bits 16..23 (reduction kernel) the chunk length C it closes.  One int: a larger
                              // kernel argument once pushed the 256-VGPR step kernel into scratch spills
  int seg_ch;                 // segment layout (seg_layout): 64, 128 or 256
};

__host__ __device__ __forceinline__ int ra_fc(const RedAr& ra) { return ra.fc_in_step & 1; }
__host__ __device__ __forceinline__ int ra_prev(const RedAr& ra) { return (ra.fc_in_step >> 1) & 1; }
__host__ __device__ __forceinline__ int ra_s(const RedAr& ra) { return (ra.fc_in_step >> 8) & 255; }
__host__ __device__ __forceinline__ int ra_chunk(const RedAr& ra) { return (ra.fc_in_step >> 16) & 255; }
__host__ __device__ __forceinline__ int ra_flags(int fc, int prev, int s, int chunk) {
  return (fc ? 1 : 0) | (prev ? 2 : 0) | (s << 8) | (chunk << 16);
}
// The step's epoch and batch position: a chunk of C steps shares one device epoch / cursor base, advanced by C
// (and C x B) by the reduction kernel that closes the chunk; step s of the chunk runs at base + s.
__device__ __forceinline__ int step_epoch(const Args& pa, const RedAr& ra) {
  return (int)(((unsigned)*pa.epoch + (unsigned)ra_s(ra)) % EPOCH_WRAP);
}
__device__ __forceinline__ char* rbase(const RedAr& ra, int q) { return ra.peers.base[q] + xg::REGION_BYTES; }
__device__ __forceinline__ float* rslab(const RedAr& ra, int q, int par) {
  return (float*)(rbase(ra, q) + xg::FLAG_BYTES) + (size_t)par * xg::SLAB_FLOATS;
}

// one-shot exchange of segment b (segv[0 .. len), len % 4 == 0) with every peer; on return segv holds the sum
// ep0: this segment's last epoch (own flag), loaded by the caller early so its latency hides under the reduction
// (thread 0's value; broadcast here through s_ep[0]).  Returns false (workgroup-uniform) when the sum must not be
// used: the exchange word was already set on entry or a wait expired.
// Failing together: once this rank's exchange word is set (a peer wait expired), later exchanges neither publish
// nor wait -- the flag stops advancing, so every peer's next wait for this rank expires too and every rank reports
// the error -- instead of publishing ahead, which let a slow peer pass its wait on a later epoch's slab and run
// SGD on a sum mixing epochs without noticing.
template <int NTH>
__device__ bool seg_exchange(const Ctx& cx, const RedAr& ra, int b, float* segv, int len, int off, int ep0, int* s_ep) {
  const int t = threadIdx.x, W = cx.ws, me = cx.rank;
  int* myflags = (int*)rbase(ra, me);
  const unsigned long long t_in = __builtin_amdgcn_s_memrealtime();
  if (t == 0) {
    s_ep[0] = xg::next_ep(ep0);
    s_ep[1] = xg::failed(ra.err);
  }
  __syncthreads();
  const int ep = s_ep[0], par = ep & 1;
  if (s_ep[1]) return false;
  constexpr int SYS = 17;  // sc0 | sc1: write-through store / cache-bypassing load
  const __amdgpu_buffer_rsrc_t mine =
      __builtin_amdgcn_make_buffer_rsrc(rslab(ra, me, par), (short)0, (int)(xg::SLAB_FLOATS * 4), 0x00020000);
  for (int k = 4 * t; k < len; k += 4 * NTH)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(xg::v4u, *(const f32x4*)(segv + k)), mine,
                                           4 * (off + k), 0, SYS);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's slab stores are performed
  __syncthreads();                                    // ... and every thread's
  if (t < W) xg::flag_store((int*)rbase(ra, t) + me * NSEG_MAX + b, ep);
  if (t < W) xg::wait_flag(myflags + t * NSEG_MAX + b, ep, ra.deadline, ra.err);
  __syncthreads();
  if (t == 0) s_ep[1] = xg::failed(ra.err);  // this wait (or any other of this rank) expired
  __syncthreads();
  if (s_ep[1]) return false;
  // metrics: exchange wait of the trunk / conv1 segments (the reduction's, on the step's critical path; the fc
  // segments exchange beside the backward) -- ticks and count per segment, so comm_time() gives the mean wait of
  // one segment exchange, i.e. the exposed exchange time of a step (the segments exchange in parallel)
  if (t == 0 && b < seg_layout(ra.seg_ch).r_ts && ra.peers.ticks != nullptr) {
    atomicAdd(ra.peers.ticks, __builtin_amdgcn_s_memrealtime() - t_in);
    atomicAdd(ra.peers.ticks + 1, 1ull);
  }
  for (int k = 4 * t; k < len; k += 4 * NTH) {  // exactly W loads in flight, one per peer link (rank_sum.h)
    *(f32x4*)(segv + k) = rank_sum(W, [&](int q) {
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(rslab(ra, q, par), (short)0,
                                                                          (int)(xg::SLAB_FLOATS * 4), 0x00020000);
      return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, 4 * (off + k), 0, SYS));
    });
  }
  __syncthreads();
  return true;
}

// parameter index of element k of segment b: >= 0 a parameter; -1 none; -2 - k: CC4 running-stat slot k
__device__ __forceinline__ int seg_pidx(const SegLayout& G, int b, int k) {
  if (b < G.r_ts) {  // slab fragment order
    const bool stem = b >= G.r_trunk;
    const int e = (stem ? b - G.r_trunk : b) * G.ch + k, ii = k & 3;
    if (e >= (stem ? SSLAB_N : WSLAB_N)) return -1;
    const int tt = e >> 8, ln = (e >> 2) & 63, mt = tt & 1, nt = tt >> 1;
    if (!stem) return OFF_CONVW + (16 * mt + 4 * (ln >> 4) + ii) * 288 + (16 * (nt & 1) + (ln & 15)) * 9 + (nt >> 1);
    if (e < 1024) {
      const int kk = 16 * nt + (ln & 15);
      return kk < 27 ? OFF_C1W + (16 * mt + 4 * (ln >> 4) + ii) * 27 + kk : -1;
    }
    return e < 1056 ? OFF_C1B + (e - 1024) : -1;
  }
  if (b < G.fct) {
    const int fb = b - G.r_ts;  // fc1 block: features 64 (fb >> 1) .., rows 16 (fb & 1) ..
    return OFF_FC1W + (16 * (fb & 1) + (k >> 6)) * 2048 + 64 * (fb >> 1) + (k & 63);
  }
  if (b == G.fct) {
    if (k < 32) return OFF_FC1B + k;
    if (k < 352) return OFF_FC2W + ((k - 32) >> 5) * 32 + ((k - 32) & 31);
    return k < 362 ? OFF_FC2B + (k - 352) : -1;
  }
  return k < 64 ? (k < 32 ? OFF_BNW : OFF_BNB) + (k & 31) : -2 - (k - 64);
}

// 16-B load bypassing L1 (sc1): the head outputs are read by the fc workers inside the launch that writes them
__device__ __forceinline__ f32x4 ld4_sc1(const float* base, int bytes, int off_floats) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, bytes, 0x00020000);
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, 4 * off_floats, 0, 16));
}

// trunk / stem chunk b of CH outputs in slab fragment order, summed over the nslab workgroup slabs in ONE order for
// every block size (the 512-thread prologue reducers and the 256-thread reduction kernel give bitwise-equal sums):
// VG = 2048 / CH virtual groups, group gv sums float4 `slot` of slabs gv, gv + VG, ... in slab order; the chunk
// total is sum_g (acc(g) + acc(g + VG / 2)) over g < VG / 2, in g order.  A 512-thread workgroup runs one virtual
// group per thread, a 256-thread one two (gv = grp, grp + VG / 2: it adds the pair before the LDS combine).
template <int NTH, int CH>
__device__ __forceinline__ void seg_chunk(const Ctx& cx, const Args& pa, const SegLayout& Ls, int b, int nslab,
                                          float* segv, f32x4* red) {
  constexpr int NS = CH / 4, VG = 2048 / CH, NG = NTH / NS, VPG = VG / NG, NU = 128 / VG, HG = VG / 2;
  static_assert(NG * VPG == VG && (VPG == 1 || VPG == 2), "512- or 256-thread reducers");
  const int t = threadIdx.x;
  const bool stem = b >= Ls.r_trunk;
  const int chunk = stem ? b - Ls.r_trunk : b;
  const int slot = t % NS, grp = t / NS, e0 = chunk * CH + slot * 4;
  const float* src = stem ? cx.SSLAB : pa.tslab;
  const int stride = stem ? SSLAB_N : WSLAB_N;
  const int ec = e0 < stride ? e0 : stride - 4;  // conv1's last 256-chunk is partial (1088 = 4.25 x 256)
  f32x4 sacc[VPG];
#pragma unroll
  for (int vp = 0; vp < VPG; ++vp) sacc[vp] = z4();
  for (int k0 = 0; k0 < nslab; k0 += 128) {
#pragma unroll
    for (int vp = 0; vp < VPG; ++vp) {
      const int gv = grp + NG * vp;
      f32x4 v[NU];
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int k = k0 + gv + VG * u;
        const int kc = k < nslab ? k : nslab - 1;
        v[u] = ld4(src + (size_t)kc * stride + ec);  // plain loads: the slabs were written before the kernel boundary
      }
#pragma unroll
      for (int u = 0; u < NU; ++u)
        if (k0 + gv + VG * u < nslab) sacc[vp] += v[u];
    }
  }
  red[t] = VPG == 2 ? sacc[0] + sacc[VPG - 1] : sacc[0];  // (VPG = 2: groups grp and grp + HG)
  __syncthreads();
  if (t < NS) {
    f32x4 tot;
    if constexpr (VPG == 2) {
      tot = red[t];
#pragma unroll
      for (int g = 1; g < HG; ++g) tot += red[NS * g + t];
    } else {
      tot = red[t] + red[NS * HG + t];
#pragma unroll
      for (int g = 1; g < HG; ++g) tot += red[NS * g + t] + red[NS * (g + HG) + t];
    }
    *(f32x4*)(segv + slot * 4) = e0 < stride ? tot : z4();
  }
}

// Write-through stores of the SGD results when the readers run in the SAME launch (the prologue reduction: the step
// workgroups read the new weights after the ready granules).  Only the hand-off forms the MI355X guide validates
// (Guideline 16 / "Valid forms", table row 1): every byte stored sc1 by a 4- or 16-B store and drained before the
// ready granule, every consumer load an sc1 global / buffer load into registers.  So the fp32 parameters and the CC4
// base are dword sc1 stores, and the trunk's bf16 hi / lo weight records are written as whole 16-B chunks: a
// 128-element trunk chunk (slab fragment order) is 8 output x 16 input channels of one tap = 16 forward chunks
// (record tap*32 + co, channels ci) and 16 dgrad chunks (record (8 - tap)*32 + ci, channels co) per plane.  (The
// first version stored every bf16 element with a 2-byte store and let the step workgroups LDS-DMA the records:
// the forms the guide has no measurement for, and the trajectory drifted.)  conv1's records are scattered 2-byte slots:
// written plainly for the NEXT launches; the step workgroups of this launch derive their conv1 fragments from the
// fp32 weights instead (stem_bfrag_sc1).
template <int NTH>
__device__ __forceinline__ void pkw_trunk_chunks_wt(const Ctx& cx, const float* wnew, int e_base, int len) {
  for (int t = threadIdx.x; t < 64 * (len / 128); t += NTH) {
    const int hf = t >> 6, j = t & 63, kind = j >> 4, idx = j & 15;
    const int e0 = e_base + hf * 128, tt = e0 >> 8, h = (e0 >> 7) & 1, mt = tt & 1, nt = tt >> 1;
    const int tap = nt >> 1, cih = nt & 1;
    const float* w = wnew + hf * 128;
    unsigned short v[8];
    int dst;
    if (kind < 2) {  // forward record tap*32 + co, channels 16 cih + 8 qq .. +7
      const int col = idx >> 1, qq = idx & 1, co = 16 * mt + 8 * h + col;
#pragma unroll
      for (int j8 = 0; j8 < 8; ++j8) {
        const float x = w[64 * (col >> 2) + 4 * (8 * qq + j8) + (col & 3)];
        const unsigned short hi = bfbits(x);
        v[j8] = kind == 0 ? hi : bf_lo(x, hi);
      }
      dst = (kind == 1 ? PKW_PLANE : 0) + pkw_elem(tap * 32 + co, 16 * cih + 8 * qq);
    } else {  // dgrad record (8 - tap)*32 + ci, channels 16 mt + 8 h .. +7
      const int cl = idx;
#pragma unroll
      for (int c8 = 0; c8 < 8; ++c8) {
        const float x = w[64 * (c8 >> 2) + 4 * cl + (c8 & 3)];
        const unsigned short hi = bfbits(x);
        v[c8] = kind == 2 ? hi : bf_lo(x, hi);
      }
      dst = PKW_DGRAD + (kind == 3 ? PKW_PLANE : 0) + pkw_elem((8 - tap) * 32 + 16 * cih + cl, 16 * mt + 8 * h);
    }
    st4_wt(cx.pkw + dst, __builtin_bit_cast(f32x4, v4u{v[0] | ((unsigned)v[1] << 16), v[2] | ((unsigned)v[3] << 16),
                                                       v[4] | ((unsigned)v[5] << 16), v[6] | ((unsigned)v[7] << 16)}));
  }
}

// Segment b on this workgroup (NTH threads): reduce / compute into segv, exchange (mode 2), SGD.  LDS: segv
// [SEG_MAX], red [NTH] f32x4, stage [stage_floats(B)], s_ep[2].  WT: the SGD results are read inside this launch
// (prologue reduction; trunk / conv1 / BN-tail segments only).
// LEAN 1: mode 0 with the fc segments on the step kernel's fc workers (world size 1): trunk / conv1 chunks and the BN
// tail only, no exchange; LEAN 2: the same segments in mode 2 (the xGMI exchange) -- each compiled without the other
// modes' code.
template <int NTH, bool WT = false, int LEAN = 0>
__device__ void seg_process(const Ctx& cx, const Args& pa, const RedAr& ra, int b, int nslab, float* segv,
                            f32x4* red, float* stage, int* s_ep, int sslot, int swg) {
  const int t = threadIdx.x, B = cx.B;
  const int mode = LEAN == 1 ? 0 : (LEAN == 2 ? 2 : ra.mode);
  const SegLayout Ls = seg_layout(ra.seg_ch);
  const int len = seg_len(Ls, b), off = seg_off(Ls, b);
  // this segment's exchange epoch (own flag), and this thread's SGD elements (k = t + NTH i): parameter indices
  // and old values, loaded first so their latency hides under the reduction
  const int ep0 = mode >= 2 && t == 0 ? xg::flag_load((const int*)rbase(ra, cx.rank) + cx.rank * NSEG_MAX + b) : 0;
  constexpr int KMAX = SEG_MAX / NTH;
  int pid[KMAX];
  float pold[KMAX];
#pragma unroll
  for (int i = 0; i < KMAX; ++i) {
    const int k = t + NTH * i;
    pid[i] = k < len && mode != 3 ? seg_pidx(Ls, b, k) : -1;
    pold[i] = cx.params[pid[i] >= 0 ? pid[i] : 0];
  }
  if (mode == 3) {
    for (int k = t; k < len; k += NTH) segv[k] = off + k < ra.st_n ? ra.st_src[off + k] : 0.f;
  } else if (b < Ls.r_ts) {
    if (Ls.ch == 128) seg_chunk<NTH, 128>(cx, pa, Ls, b, nslab, segv, red);
    else seg_chunk<NTH, 256>(cx, pa, Ls, b, nslab, segv, red);
  } else if (!LEAN && b < Ls.fct) {
    // fc1 block: dW1[j][64f + kk .. +3] = sum_b dh[b][j] p[b][64f + kk ..], rows j = 16 h .. 16 h + 15
    const int fb = b - Ls.r_ts, f = fb >> 1, j0 = 16 * (fb & 1);
    float* dh_s = stage;           // [B][32]
    float* p_s = stage + B * 32;   // [B][64]
    constexpr int MD = (64 * 8 + NTH - 1) / NTH, MP = (64 * 16 + NTH - 1) / NTH;
    f32x4 dh4[MD], p4[MP];
#pragma unroll
    for (int m = 0; m < MD; ++m) {
      const int idx = t + NTH * m;
      dh4[m] = ld4_sc1(cx.HDH, 64 * 32 * 4, 4 * (idx < B * 8 ? idx : 0));
    }
#pragma unroll
    for (int m = 0; m < MP; ++m) {
      const int idx = t + NTH * m, ic = idx < B * 16 ? idx : 0, bb = ic >> 4, k4 = ic & 15;
      p4[m] = ld4_sc1(cx.HP, 64 * 2048 * 4, bb * 2048 + 64 * f + 4 * k4);
    }
#pragma unroll
    for (int m = 0; m < MD; ++m)
      if (t + NTH * m < B * 8) st4(dh_s + 4 * (t + NTH * m), dh4[m]);
#pragma unroll
    for (int m = 0; m < MP; ++m)
      if (t + NTH * m < B * 16) st4(p_s + 4 * (t + NTH * m), p4[m]);
    __syncthreads();
    if (t < 256) {
      const int jl = t >> 4, kk = 4 * (t & 15);
      f32x4 a0 = z4();
#pragma unroll 8
      for (int bb = 0; bb < B; ++bb) a0 += dh_s[bb * 32 + j0 + jl] * ld4(p_s + bb * 64 + kk);
      st4(segv + jl * 64 + kk, a0);
    }
  } else if (!LEAN && b == Ls.fct) {
    // fc tail: fc1 bias [0,32), fc2 weight [32,352), fc2 bias [352,362), pad
    float* hh_s = stage;            // [B][32]
    float* dl_s = stage + B * 32;   // [B][16]
    float* dh_s = dl_s + B * 16;    // [B][32]
    for (int idx = t; idx < B * 8; idx += NTH) {
      st4(hh_s + 4 * idx, ld4_sc1(cx.HH, 64 * 32 * 4, 4 * idx));
      st4(dh_s + 4 * idx, ld4_sc1(cx.HDH, 64 * 32 * 4, 4 * idx));
    }
    for (int idx = t; idx < B * 10; idx += NTH) {
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)cx.HDL, (short)0, 64 * 16 * 4, 0x00020000);
      dl_s[(idx / 10) * 16 + idx % 10] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, 4 * idx, 0, 16));
    }
    __syncthreads();
    for (int idx = t; idx < FCT_LEN; idx += NTH) {  // (parameter indices: seg_pidx)
      float sv = 0.f;
      if (idx < 32) {
#pragma unroll 8
        for (int bb = 0; bb < B; ++bb) sv += dh_s[bb * 32 + idx];
      } else if (idx < 352) {
        const int o = (idx - 32) >> 5, jj = (idx - 32) & 31;
#pragma unroll 8
        for (int bb = 0; bb < B; ++bb) sv += dl_s[bb * 16 + o] * hh_s[bb * 32 + jj];
      } else if (idx < 362) {
        const int o = idx - 352;
#pragma unroll 8
        for (int bb = 0; bb < B; ++bb) sv += dl_s[bb * 16 + o];
      }
      segv[idx] = sv;
    }
  } else {
    // BN tail: gamma | beta gradients [0, 64), CC4 running mean | var [64, 128) (rank 0's buffers; others 0)
    for (int idx = t; idx < BNT_LEN; idx += NTH) {
      float sv;
      if (idx < 64) {
        sv = pa.bng[idx];
      } else {
        const int k = idx - 64;
        sv = cx.rank == 0 ? (k < 32 ? cx.rm[k] : cx.rv[k - 32]) : 0.f;
      }
      segv[idx] = sv;
    }
  }
  __syncthreads();
  DCA_STAMP(cx, sslot, swg, 1);
  if (mode >= 2 && !seg_exchange<NTH>(cx, ra, b, segv, len, off, ep0, s_ep)) return;  // no SGD on a failed sum
  DCA_STAMP(cx, sslot, swg, 2);
#pragma unroll
  for (int i = 0; i < KMAX; ++i) {
    const int k = t + NTH * i;
    if (k >= len) break;
    const int pidx = pid[i];
    const float g = segv[k];
    if (mode == 3) {
      if (off + k < ra.st_n) ra.st_dst[off + k] = g;
      continue;
    }
    if (pidx >= 0) {
      cx.grads[pidx] = g;
      if (mode == 1) continue;
      const float oldp = pold[i];
      float wv;
      if (mode == 0) {
        wv = __builtin_fmaf(-cx.lr, g, oldp);
      } else {
        wv = oldp;
        wv -= cx.lr * g * cx.inv_ws;  // same rounding as k_apply_sgd / k_xgmi_ar_sgd
      }
      if constexpr (WT) {
        st1_wt(cx.params + pidx, wv);
        if (b < Ls.r_trunk) segv[k] = wv;             // the records: whole 16-B chunks below
        else derive_param<true>(cx, pidx, wv);        // conv1 records: for the next launches (plain stores)
      } else {
        cx.params[pidx] = wv;
        derive_param<true>(cx, pidx, wv);
      }
    } else if (pidx <= -2) {  // CC4: rank 0's running stats become every rank's base (rides the all-reduce)
      const int kk = -2 - pidx;
      if (mode == 1) cx.grads[OFF_RS + kk] = g;
      else if (mode == 2) {
        if constexpr (WT) st1_wt(cx.rs_base + kk, g);
        else cx.rs_base[kk] = g;
      }
    }
  }
  if constexpr (WT) {
    if (b < Ls.r_trunk && mode != 1 && mode != 3) {  // this chunk's weight records (segv = the new weights)
      __syncthreads();
      pkw_trunk_chunks_wt<NTH>(cx, segv, b * Ls.ch, len);
    }
  }
  DCA_STAMP(cx, sslot, swg, 3);
}

// The finished step's batch-mean loss, step / BN-batch counters: independent of every segment, so it runs beside
// them.  chunk > 0 (the reduction kernel closing a chunk of `chunk` steps): also the epoch / cursor base, advanced by
// the chunk; 0 (a prologue reduction inside the chunk): they stay (the chunk's steps run at base + s).
__device__ __forceinline__ void pks_bookkeeping(const Ctx& cx, const Args& pa, int chunk) {
  const int t = threadIdx.x, B = cx.B;
  if (t >= 64) return;
  float l = t < B ? cx.HLOSS[t] : 0.f;  // B <= 64
  double acc = 0.0;
  int cur = 0, stp = 0, ep = 0;
  long long nb = 0;
  if (t == 0) {  // issued together with the loss loads: one memory round trip, not five dependent ones
    ep = *pa.epoch;
    acc = *cx.loss_acc;
    cur = *cx.cursor;
    stp = *cx.step_count;
    nb = *cx.nbt;
  }
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) l += __shfl_xor(l, m);  // fixed tree: identical every step
  if (t == 0) {
    *cx.loss_acc = acc + (double)(l / (float)B);
    *cx.step_count = stp + 1;
    *cx.nbt = nb + NBLK;  // BatchNorm num_batches_tracked: +1 per application
    if (chunk > 0) {
      *cx.cursor = cur + chunk * B;
      *pa.epoch = (int)(((unsigned)ep + (unsigned)chunk) % EPOCH_WRAP);
    }
  }
}

// fc worker fb (0 .. R_FC1 - 1: fc1 block fb; R_FC1: fc tail) of the step kernel: waits until every main workgroup
// has published its head-done granule (its pooled features HP and, slice 0, the image's dh / h / dlogits are
// written through and drained), then runs the segment (compute, xGMI exchange, SGD) beside the trunk backward.
template <int P>
__device__ void fc_segment(const Ctx& cx, const Args& pa, const RedAr& ra, int fb, char* smem) {
  const int t = threadIdx.x, lane = t & 63, G = cx.B * S;
  const int epoch = step_epoch(pa, ra);
  DCA_STAMP(cx, 9, fb, 0);
  if (t < 64) {  // ONE wave polls (sleeping between passes): the CU's other work is the step's, on other CUs
    const unsigned tag = tagof(epoch, RND_HDONE);
    for (unsigned spins = 0;; ++spins) {
      bool ok = true;
      for (int k = lane; k < G; k += 64)
        ok &= (unsigned)(__hip_atomic_load(pa.hdone + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 32) == tag;
      if (__all(ok)) break;
      if (spins >= SPIN_LIMIT) {
        if (lane == 0) atomicOr(pa.err, 1u << 30);
        break;
      }
      __builtin_amdgcn_s_sleep(8);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  float* segv = (float*)smem;
  f32x4* red = (f32x4*)(smem + SEG_MAX * 4);
  float* stage = (float*)(smem + SEG_MAX * 4 + NTH * 16);
  int* s_ep = (int*)(smem + SEG_MAX * 4 + NTH * 16 + stage_floats(cx.B) * 4);  // [2]
  const SegLayout Ls = seg_layout(ra.seg_ch);
  seg_process<NTH>(cx, pa, ra, fb < R_FC1 ? Ls.r_ts + fb : Ls.fct, G, segv, red, stage, s_ep, 9, fb);
}

// ============================================================================================================
// Prologue reduction (k_pks_step with ra_prev): the gradient segments of the PREVIOUS step -- its trunk / conv1 chunks
// and the BN tail, i.e. what k_pks_reduce_ar would do after it -- run at the start of this launch on the reducer
// workgroups (the fc workers first, then extras), while the step workgroups stage their input images.  Each segment
// is reduced, exchanged (xGMI), applied (SGD, write-through: the readers are in this launch) and announced by a
// ready granule {tagof(epoch, RND_RDONE)}; the step workgroups wait for all of them before they load the weights
// and step constants (sc1 loads).  A chunk of C steps is then C step launches and ONE reduction kernel (the last
// step's segments, closing the chunk): one kernel boundary per step instead of two (MI355X guide "boundary",
// ~1.8 us each), and the reduction's own latency overlaps the stem's input staging.  The previous step's slabs,
// BN-affine gradient and losses are read here before any step workgroup of this launch can write them again (they
// write only after the ready wait).  Not used with RCCL / host all-reduce (mode 1: the collective must sit between
// the reduction and the SGD) nor when the reducers do not fit beside the step (engine.hip prologue_ok).
// ============================================================================================================
constexpr int RND_RDONE = 29;  // tag round of the ready granules
__host__ __device__ inline int prologue_segments(int seg_ch) { return seg_layout(seg_ch).r_ts + 1; }
__device__ __forceinline__ unsigned long long* rdone(const Args& pa) { return pa.hdone + LMAX; }

template <int P>
__device__ void prologue_reduce(const Ctx& cx, const Args& pa, const RedAr& ra, int r, char* smem) {
  const SegLayout Ls = seg_layout(ra.seg_ch);
  const int nred = prologue_segments(ra.seg_ch);
  if (r >= nred) return;
  const int epoch = step_epoch(pa, ra);
  float* segv = (float*)smem;
  f32x4* red = (f32x4*)(smem + SEG_MAX * 4);
  float* stage = (float*)(smem + SEG_MAX * 4 + NTH * 16);
  int* s_ep = (int*)(smem + SEG_MAX * 4 + NTH * 16 + stage_floats(cx.B) * 4);  // [2]
  DCA_STAMP(cx, 8, r, 0);
  seg_process<NTH, true>(cx, pa, ra, r < Ls.r_ts ? r : Ls.bnt, cx.B * S, segv, red, stage, s_ep, 8, r);
  if (r == nred - 1) pks_bookkeeping(cx, pa, 0);  // the previous step's loss and counters
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's write-through stores are performed
  __syncthreads();                                    // ... and every thread's of this workgroup
  if (threadIdx.x == 0) gput(rdone(pa) + r, tagof(epoch, RND_RDONE), 0.f);
}
// Step workgroups: wait (one wave, bounded) until every reducer of this launch has announced its segment.  At world
// size 1 the reducers never wait on anything, so a spin count bounds it; with the xGMI exchange (mode 2) a reducer
// may itself wait up to ra.deadline for a lagging peer, so this wait is bounded by the same s_memrealtime deadline
// (a spin count would expire first and let the step read weights the reducers are still writing).
__device__ __forceinline__ void wait_ready(const Args& pa, const RedAr& ra, int epoch) {
  const int t = threadIdx.x, lane = t & 63;
  if (t < 64) {
    const int nred = prologue_segments(ra.seg_ch);
    const unsigned tag = tagof(epoch, RND_RDONE);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (unsigned spins = 0;; ++spins) {
      bool ok = true;
      for (int k = lane; k < nred; k += 64)
        ok &= (unsigned)(__hip_atomic_load(rdone(pa) + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 32) == tag;
      if (__all(ok)) break;
      const bool expired = ra.mode == 2 ? (__builtin_amdgcn_s_memrealtime() - t0 > ra.deadline + (ra.deadline >> 3))
                                        : spins >= SPIN_LIMIT;
      if (expired) {
        if (lane == 0) atomicOr(pa.err, 1u << 28);
        break;
      }
      if (ra.mode == 2) __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
}

constexpr int P_KSHIFT = 906;  // misc: [10][32] BN shifts (last step's batch means)
constexpr int P_LABEL = 1240;  // misc: this image's label

// ============================================================================================================
// The step of one main workgroup (slice s of image n).  PRO: the prologue-reduction form (compiled separately, so
// the default form carries none of its code: the shared form ran ~1 us per step slower, profiles/pks_split_r6.log).
template <int P, bool PRO>
__device__ __forceinline__ void step_main(const Ctx& cx, const Args& pa, const RedAr& ra, char* smem) {
  using PL = Plan<P>;
  const int t = threadIdx.x, wv = t >> 6, lane = t & 63, c = lane & 15, q = lane >> 4;
  const int w = wv & (RS - 1), hh = wv / RS, ch = 16 * hh + c;  // image row (in the slice), channel half, channel
  // Placement (speed only, never correctness): blocks b and b + 8 share an XCD under the observed round-robin
  // dispatch, so the S slices of an image get block ids 8 apart and their halo hand-offs stay in one L2.
  const int b = blockIdx.x, s = (b >> 3) % S, n = (b >> 3) / S * 8 + (b & 7);
  const int B = cx.B;
  if (n >= B) return;
  const int L = n * S + s, G = B * S;
  const int row = s * RS + w;  // image row of this wave
  const bool halo = (w == 0 && s > 0) || (w == RS - 1 && s < S - 1);  // this wave keeps a neighbour row
  const int hwhich = w == 0 ? 0 : 1;                  // the boundary row this wave publishes: 0 top, 1 bottom
  const int hsrc = w == 0 ? L - 1 : L + 1;            // ... and whose boundary row it receives
  const int hxrow = w == 0 ? 0 : RS + 1;              // XR / xT row of the received halo
  float* cred = (float*)(smem + PL::O_CRED);
  f32x4* stat = (f32x4*)(smem + PL::O_STAT);
  float* misc = (float*)(smem + PL::O_MISC);
  char* U = smem + PL::O_U;
  char* WT = U + PL::U_WT;
  char* XR = U + PL::U_XR;
  const int epoch = step_epoch(pa, ra);
  const int par = epoch & 1;
  const bool prev = PRO && ra_prev(ra);  // the previous step's gradient segments are applied in this launch
  const uint8_t* my_img = pa.simg + (size_t)(par * 64 + n) * 3072;
  const int next_id = sample_id(cx, (ra_s(ra) + 1) * B + n);
  const float Ntot = (float)B * 256.f;
  const unsigned short* pkw = (const unsigned short*)cx.pkw;
  const size_t img8 = (size_t)n * 8192 + (size_t)row * 512;  // this row inside an image of a block's tensor
  DCA_STAMP(cx, 0, L, 0);

  float x[4];        // this thread's values of the current block input (forward), x_{i+1} (backward)
  float xo[4] = {};  // halo waves: the neighbour row of the same
  float y[4];        // conv output of the current block

  // ======================= stem: gather + normalise + conv1 + bias + ReLU + 2x2 max-pool ======================
  // Pooled rows 4s-1 .. 4s+4 (own + one halo row each side, recomputed here: the input image is read-only).
  // Input staged as bf16 NHWC4 pixels (3 channels + a zero): an MFMA K-group of 4 is one tap of one pixel
  // (v_mfma_f32_16x16x16_bf16, K = (tap, channel), 3 MFMAs cover the 9 taps; taps 9..11 have zero weights).
  {
    uint2* xin4 = (uint2*)(U + PL::U_XIN);
    float* x0i = (float*)(U + PL::U_X0);
    uint8_t* scl = (uint8_t*)(U + PL::U_SCODE);
    // step constants -> misc: k < 64: BN gamma|beta -> misc[320 + k]; k >= 64 ->
    // misc[384 + k]: running mean|var [448,512) (rank 0's base under DDP, CC4), fc1 bias [512,544), W2
    // [544,864), b2 [864,874), conv1 bias [874,906), BN shifts [906,1226)
    constexpr int NKC = 842, KCM = (NKC + NTH - 1) / NTH;
    float kc[KCM];
    int lab = 0;
    // input words: thread t < 112 -> xin4 row j = t >> 3 (image row 8s-3+j), 4 columns 4 (t & 7) .., 3 channels
    const int jr = (t >> 3) < 14 ? (t >> 3) : 13, yimg = 8 * s - 3 + jr, xq = t & 7;
    const bool ivalid = t < 112 && yimg >= 0 && yimg < 32;
    const unsigned* imw = (const unsigned*)my_img;
    const int yc = yimg < 0 ? 0 : (yimg > 31 ? 31 : yimg);
    unsigned iw0 = 0u, iw1 = 0u, iw2 = 0u;
    auto image_loads = [&] {
      lab = pa.slab[par * 64 + n];
      iw0 = imw[yc * 8 + xq];
      iw1 = imw[256 + yc * 8 + xq];
      iw2 = imw[512 + yc * 8 + xq];
    };
    if constexpr (PRO) {
      // prologue reduction: the weights / constants below are the reducers' (this launch): wait for their ready
      // granules (the image loads stay in flight), then read them with sc1 loads
      image_loads();
      if (prev) wait_ready(pa, ra, epoch);
    }
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
                                 : (const float*)cx.STATS + 2 * (k - 522);
      kc[m] = prev ? __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *src;
    }
    if constexpr (!PRO) image_loads();  // (after the constants: the round-4 order)
    // forward trunk weights, records [tap][co] x ci (hi, lo)
    if (prev) wt_copy_sc1<P>(WT, pkw);
    else wt_dma<P>(WT, pkw, wv, lane);
    uint2 bwr[P + 1][2][3];        // conv1 B fragments: lane (co = 16h + c, k-group q) of MFMA m
#pragma unroll
    for (int p = 0; p <= P; ++p)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int m = 0; m < 3; ++m)
          bwr[p][h][m] = prev ? stem_bfrag_sc1<P>(cx, p, h, m, lane)
                              : ((const uint2*)(pkw + PKW_STEM + p * 1536))[(h * 3 + m) * 64 + lane];
#pragma unroll
    for (int m = 0; m < KCM; ++m) pin(kc[m]);
    pin(lab);
    pin(iw0);
    pin(iw1);
    pin(iw2);
#pragma unroll
    for (int p = 0; p <= P; ++p)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int m = 0; m < 3; ++m) pin(bwr[p][h][m]);
#pragma unroll
    for (int m = 0; m < KCM; ++m) {
      const int k = t + NTH * m;
      if (k < NKC) misc[(k < 64 ? 320 : 384) + k] = k >= 522 && !(fabsf(kc[m]) < 1e30f) ? 0.f : kc[m];
    }
    if (t == 0) misc[P_LABEL] = __int_as_float(lab);
    if (t < 112) {
#pragma unroll
      for (int b2 = 0; b2 < 4; ++b2) {
        const float v0 = ivalid ? norm_px((iw0 >> (8 * b2)) & 255u, 0) : 0.f;
        const float v1 = ivalid ? norm_px((iw1 >> (8 * b2)) & 255u, 1) : 0.f;
        const float v2 = ivalid ? norm_px((iw2 >> (8 * b2)) & 255u, 2) : 0.f;
        const unsigned short h0 = bfbits(v0), h1 = bfbits(v1), h2 = bfbits(v2);
        const int px = jr * 34 + 4 * xq + 1 + b2;
        xin4[px] = uint2{(unsigned)h0 | ((unsigned)h1 << 16), (unsigned)h2};
        if constexpr (P == 1)
          xin4[PL::XIN_PL / 8 + px] = uint2{(unsigned)bf_lo(v0, h0) | ((unsigned)bf_lo(v1, h1) << 16),
                                            (unsigned)bf_lo(v2, h2)};
      }
    } else if (t < 112 + 28) {  // columns 0 and 33 of the 14 rows
      const int k = t - 112, px = (k >> 1) * 34 + ((k & 1) ? 33 : 0);
      xin4[px] = uint2{0u, 0u};
      if constexpr (P == 1) xin4[PL::XIN_PL / 8 + px] = uint2{0u, 0u};
    }
    for (int idx = t; idx < PL::NP * PL::XR_PL / 16; idx += NTH) ((uint4*)XR)[idx] = uint4{0u, 0u, 0u, 0u};
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's weight DMA has landed in LDS
    lds_barrier();
    DCA_STAMP(cx, 0, L, 2);
    s4v bw[P + 1][2][3];
#pragma unroll
    for (int p = 0; p <= P; ++p)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int m = 0; m < 3; ++m) bw[p][h][m] = __builtin_bit_cast(s4v, bwr[p][h][m]);
    const float* sb = misc + 874;
    // units: (pooled row 4s-1+ur, column half), ur = 0..RS+1; wave wv takes units wv, wv + NW, ...
#pragma unroll 1
    for (int u = wv; u < 2 * (RS + 2); u += NW) {
      const int ur = u >> 1, chalf = u & 1, pr = 4 * s - 1 + ur;
      if (pr < 0 || pr > 15) continue;  // wave-uniform: the image border (XR rows stay zero)
      f32x4 acc[2][2];
#pragma unroll
      for (int rw = 0; rw < 2; ++rw) {
        acc[rw][0] = z4();
        acc[rw][1] = z4();
#pragma unroll
        for (int m = 0; m < 3; ++m) {
          const int tap = 4 * m + q, tc = tap < 9 ? tap : 0, kh = tc / 3, kw = tc % 3;
          const int px = (2 * ur + rw + kh) * 34 + 16 * chalf + c + kw;
          const s4v a = __builtin_bit_cast(s4v, xin4[px]);
          s4v al = a;
          if constexpr (P == 1) al = __builtin_bit_cast(s4v, xin4[PL::XIN_PL / 8 + px]);
          acc[rw][0] = mma3s<P>(a, al, bw[0][0][m], bw[P][0][m], acc[rw][0]);
          acc[rw][1] = mma3s<P>(a, al, bw[0][1][m], bw[P][1][m], acc[rw][1]);
        }
      }
      if (pa.debug && ur >= 1 && ur <= RS) {  // conv1 + bias before the ReLU, own rows (NCHW)
#pragma unroll
        for (int rw = 0; rw < 2; ++rw)
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int i2 = 0; i2 < 4; ++i2)
              pa.c1[(((size_t)n * 32 + 16 * h + c) * 32 + 2 * pr + rw) * 32 + 16 * chalf + 4 * q + i2] =
                  acc[rw][h][i2] + sb[16 * h + c];
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
          const int pc = 8 * chalf + 2 * q + pp;
          x0i[(ur * 16 + pc) * PL::X0S + co] = best;
          if (ur >= 1 && ur <= RS) scl[((ur - 1) * 16 + pc) * 32 + co] = (uint8_t)code;
          st1r<P>(XR, PL::XR_PL, ur * 18 + pc + 1, co, best);
        }
      }
    }
    lds_barrier();
    DCA_STAMP(cx, 0, L, 3);
    unsigned cw = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      x[i] = x0i[((w + 1) * 16 + 4 * q + i) * PL::X0S + ch];
      if (halo) xo[i] = x0i[(hxrow * 16 + 4 * q + i) * PL::X0S + ch];
      cw |= (unsigned)scl[(w * 16 + 4 * q + i) * 32 + ch] << (8 * i);
    }
    // stem pool codes, read back by this very thread in the stem backward
    *(unsigned*)(cx.SCODE + img8 + hh * 256 + lane * 4) = cw;
    if (pa.debug) st4r(cx.X + img8, hh, lane, x);
  }
  DCA_STAMP(cx, 0, L, 1);

  // ======================= forward: 10 applications of the shared ResBlock ===================================
  // fc1 weights of this slice's 512 pooled features (local index u = ch*16 + pr*8 + pw <-> global feature
  // ch*64 + (2s + pr)*8 + pw: per row, 32 runs of 16 contiguous elements): copied into their LDS region (unused by
  // the forward) by LDS-DMA right after block 6's exchange, read by
  // fc1 (reduction over features) and its transpose dp (reduction over rows).  The dgrad weights replace the
  // forward ones in WT by LDS-DMA right after block 9's exchange (block 9's conv was WT's last reader).
  const float gam = misc[320 + ch], bet = misc[352 + ch];  // BN affine of this thread's channel (registers)
  bf16x8 bw[9];  // P = 0: this wave's B fragments of the conv weight (forward here, dgrad in the backward)
  if constexpr (P == 0) load_bfrag(WT, hh, lane, bw);
#pragma unroll 1
  for (int i = 0; i < NBLK; ++i) {
    // shifted one-pass sums S1 = sum(y - K), S2 = sum((y - K)^2); K = this block's batch mean of the previous
    // step (0 at the first), identical in every workgroup, so the partials combine exactly (read ahead of the conv:
    // its LDS latency hides under the conv's)
    const float K = misc[P_KSHIFT + i * 32 + ch];
    {
      const f32x4 acc = conv_row<P>(XR, WT, bw, w, hh, lane);
#pragma unroll
      for (int i2 = 0; i2 < 4; ++i2) y[i2] = acc[i2];
    }
    if (i == DCA_DETAIL_FWD) DCA_STAMP(cx, 6, L, 0);
    float a = 0.f, bsq = 0.f;
#pragma unroll
    for (int i2 = 0; i2 < 4; ++i2) {
      const float d = y[i2] - K;
      a += d;
      bsq += d * d;
    }
    const float pv = wg_csum(a, bsq, cred);
    const unsigned tag = tagof(epoch, i);
    if (t < 64) bn_put(pa, i, L, t, bn_tag(epoch, i), pv);
    if (halo) publish_row(pa, i, L, hwhich, hh, tag, y, lane);
    float yo[4];
    if (i == DCA_DETAIL_FWD) DCA_STAMP(cx, 6, L, 1);
    xchg_wait(pa, i, epoch, G, cred, halo, hsrc, hwhich ^ 1, hh, yo);
    if (i == DCA_DETAIL_FWD) DCA_STAMP(cx, 6, L, 2);
    st4r_wt(cx.Y + (size_t)i * B * 8192 + img8, hh, lane, y);  // this block's y for the backward (after the sweep)
    // the fc1 slice for the head, straight into its LDS region (free during the forward) by LDS-DMA, issued right
    // AFTER an exchange: vmcnt is in order, so loads in flight when a sweep starts hold up its first pass (register
    // loads before the exchange + an LDS store a block later cost ~1.4 us in each of the two blocks, stamps)
    if (i == NBLK - 4) w1_dma<P>(cx, U + PL::U_W1, s, wv, lane);
    if (i == NBLK - 1) {  // dgrad weights, records [8 - tap][ci] x co (sc1 loads: the prologue reduction wrote them)
      if (prev) wt_copy_sc1<P>(WT, pkw + PKW_DGRAD);
      else wt_dma<P>(WT, pkw + PKW_DGRAD, wv, lane);
    }
    lds_barrier();
    if (i == DCA_DETAIL_FWD) DCA_STAMP(cx, 6, L, 3);
    if (halo) st4r_wt(pa.yh + ((size_t)(i * LMAX + L) * 2 + hwhich) * 512, hh, lane, yo);
    // every thread finalises the statistics of its own channel (same sums, same order everywhere)
    const float S1 = slot_total(cred, ch), S2 = slot_total(cred, 32 + ch);
    const float dm = S1 / Ntot;
    const float mean = K + dm;
    const float var = fmaxf(S2 / Ntot - dm * dm, 0.f);
    const float invstd = rsqrtf(var + cx.bn_eps);
    const float scv = gam * invstd;
    const float shv = bet - mean * scv;
    if (w == 0 && q == 0) {
      stat[i * 32 + ch] = f32x4{mean, invstd, scv, shv};
      if (L == 0) {  // BN running statistics (10 EMAs per forward) and the batch stats for the next step
        const float unb = var * Ntot / (Ntot - 1.f), mo = cx.bn_mom;
        misc[448 + ch] = misc[448 + ch] * (1.f - mo) + mean * mo;
        misc[480 + ch] = misc[480 + ch] * (1.f - mo) + unb * mo;
        cx.STATS[i * 32 + ch] = make_float2(mean, invstd);
        if (i == NBLK - 1) {
          cx.rm[ch] = misc[448 + ch];
          cx.rv[ch] = misc[480 + ch];
        }
      }
    }
    // x_{i+1} = relu(bn(y_i)) + x_i, own row and (halo waves) the neighbour row
#pragma unroll
    for (int i2 = 0; i2 < 4; ++i2) {
      x[i2] = fmaxf(__builtin_fmaf(y[i2], scv, shv), 0.f) + x[i2];
      if (halo) xo[i2] = fmaxf(__builtin_fmaf(yo[i2], scv, shv), 0.f) + xo[i2];
    }
    if (i < NBLK - 1) {
      xr_row<P>(XR, w + 1, q, ch, x);
      if (halo) xr_row<P>(XR, hxrow, q, ch, xo);
      if (pa.debug) st4r(cx.X + (size_t)(i + 1) * B * 8192 + img8, hh, lane, x);
      lds_barrier();
    }
    DCA_STAMP(cx, 1 + i / 8, L, i % 8);
  }

  // ======================= head ==============================================================================
  // x10 (registers) -> LDS -> 2x2 max-pool -> fc1 partial over this slice's 512 features -> the S slices of the
  // image exchange their partials -> fc1 + ReLU, fc2, cross-entropy (mean over the batch) and their backward
  // (every slice, redundantly) -> dp = W1^T dh for this slice's features -> max-pool backward -> g = dL/dx10.
  float g[4];
  float yv[4], yo[4] = {};  // y_i of this row / of the halo row (backward)
  {
    float* x10 = (float*)(U + PL::U_X10);
    uint8_t* pcode = (uint8_t*)(U + PL::U_PCODE);
    float* dpl = (float*)(U + PL::U_DP);
    float* pl = (float*)(U + PL::U_PL);
    float* hp = (float*)(U + PL::U_HP);
    char* w1l = U + PL::U_W1;
#pragma unroll
    for (int i2 = 0; i2 < 4; ++i2) x10[(w * 16 + 4 * q + i2) * PL::X10S + ch] = x[i2];
    lds_barrier();
    // pool: thread t < 256 -> channel t >> 3, local pool row pr = (t >> 2) & 1, pool cols 2 (t & 3) + {0, 1}
    if (t < 256) {
      const int pch = t >> 3, pr = (t >> 2) & 1;
      float pv[2];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int pc = 2 * (t & 3) + k;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e)  // window order (0,0) (0,1) (1,0) (1,1): first maximum wins
          v[e] = x10[((2 * pr + (e >> 1)) * 16 + 2 * pc + (e & 1)) * PL::X10S + pch];
        float best = v[0];
        unsigned id = 0;
        if (v[1] > best) { best = v[1]; id = 1; }
        if (v[2] > best) { best = v[2]; id = 2; }
        if (v[3] > best) { best = v[3]; id = 3; }
        pv[k] = best;
        pcode[2 * t + k] = (uint8_t)id;  // local feature u = ch*16 + pr*8 + pc = 2t + k
      }
      *(float2*)(pl + 2 * t) = make_float2(pv[0], pv[1]);
      // fc1 input for the weight gradient: global feature ch*64 + (2s + pr)*8 + pc
      st2_wt(cx.HP + (size_t)n * 2048 + pch * 64 + (2 * s + pr) * 8 + 2 * (t & 3), pv[0], pv[1]);
    }
    lds_barrier();
    // block 9's y for the first backward block, loaded now: the fc1 partial below hides the latency (the head
    // exchange is polled by wave 0 only, after that)
    ld4r(cx.Y + (size_t)(NBLK - 1) * B * 8192 + img8, hh, lane, yv);
    if (halo) ld4r(pa.yh + ((size_t)((NBLK - 1) * LMAX + L) * 2 + hwhich) * 512, hh, lane, yo);
    // fc1 partial over this slice's features: thread (row j = t >> 4, part k = t & 15) sums features
    // u = 64m + 4k .. +3 (one 8 / 16-B weight read and one 16-B feature read per 4 features), then the 16 parts by
    // DPP (fixed order: identical in every workgroup)
    {
      const int j = t >> 4, k = t & 15;
      float a = 0.f;
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const int u0 = 64 * m + 4 * k;
        float wv4[4];
        if constexpr (P == 1) {
          const f32x4 w4 = *(const f32x4*)((const float*)w1l + j * PL::W1S + u0);
          wv4[0] = w4[0];
          wv4[1] = w4[1];
          wv4[2] = w4[2];
          wv4[3] = w4[3];
        } else {
          const uint2 w4 = *(const uint2*)((const unsigned short*)w1l + j * PL::W1S + u0);
          wv4[0] = __uint_as_float(w4.x << 16);
          wv4[1] = __uint_as_float(w4.x & 0xffff0000u);
          wv4[2] = __uint_as_float(w4.y << 16);
          wv4[3] = __uint_as_float(w4.y & 0xffff0000u);
        }
        const f32x4 p4 = *(const f32x4*)(pl + u0);
#pragma unroll
        for (int e = 0; e < 4; ++e) a += wv4[e] * p4[e];
      }
      a = xsum_row16(a);
      if (k == 0) hp[j] = a;
    }
    lds_barrier();
    DCA_STAMP(cx, 3, L, 1);
    const unsigned tag = tagof(epoch, RND_HEAD);
    if (t < 32) gput(gslot(pa, RND_HEAD, L) + t, tag, hp[t]);
    if (wv == 0) {
      // the image's S partials, summed in slice order (bitwise identical in every slice); fc1 bias + ReLU, fc2,
      // softmax cross-entropy and dh, lane-parallel with shuffles
      float hsum = 0.f;
      {
        const __amdgpu_buffer_rsrc_t rs = grsrc(pa, RND_HEAD);
        const int sl = lane & 31;
        for (unsigned spins = 0;; ++spins) {
          asm volatile("" ::: "memory");
          bool ok = true;
          float a = 0.f;
#pragma unroll
          for (int s2 = 0; s2 < S; ++s2) {
            const auto xg = __builtin_amdgcn_raw_buffer_load_b64(rs, ((n * S + s2) * GSTR + sl) * 8, 0, 16);
            ok &= xg[1] == tag;
            a += __uint_as_float(xg[0]);
          }
          hsum = a;
          if (__all(ok)) break;
          if (spins >= SPIN_LIMIT) {
            if (lane == 0) atomicOr(pa.err, 1u << RND_HEAD);
            break;
          }
        }
      }
      DCA_STAMP(cx, 3, L, 2);
      hsum += misc[512 + (lane & 31)];
      const float hr = fmaxf(hsum, 0.f);
      const int o = lane < 10 ? lane : 0;
      float logit = misc[864 + o];
#pragma unroll
      for (int j4 = 0; j4 < 8; ++j4) {  // W2 row o as 8 x 16-B LDS reads (same summation order)
        const f32x4 w4 = *(const f32x4*)(misc + 544 + o * 32 + 4 * j4);
#pragma unroll
        for (int e = 0; e < 4; ++e)
          logit += w4[e] * __int_as_float(__builtin_amdgcn_readlane(__float_as_int(hr), 4 * j4 + e));
      }
      float lg[10];
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
      const float invB = 1.f / (float)B;
      float sd = 0.f, dl = 0.f;
#pragma unroll
      for (int oo = 0; oo < 10; ++oo) {
        const float dlo = (ex[oo] * rse - (oo == label ? 1.f : 0.f)) * invB;
        sd += misc[544 + oo * 32 + (lane & 31)] * dlo;
        dl = lane == oo ? dlo : dl;
      }
      const float dh = hsum > 0.f ? sd : 0.f;
      if (lane < 32) hp[32 + lane] = dh;
      if (s == 0) {  // write-through (sc1): the fc workers read them inside this launch
        if (lane == 0) st1_wt(cx.HLOSS + n, lse - lt);
        if (lane < 32) {
          st1_wt(cx.HDH + n * 32 + lane, dh);
          st1_wt(cx.HH + n * 32 + lane, hr);
        }
        if (lane < 10) st1_wt(cx.HDL + n * 10 + lane, dl);
      }
    }
    lds_barrier();
    DCA_STAMP(cx, 3, L, 3);
    {  // dp = W1^T dh for this thread's local feature u = t (dh read as 8 broadcast 16-B LDS reads)
      float d0 = 0.f;
#pragma unroll
      for (int j4 = 0; j4 < 8; ++j4) {
        const f32x4 dh4 = *(const f32x4*)(hp + 32 + 4 * j4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int j = 4 * j4 + e;
          const float wvv = P == 1 ? ((const float*)w1l)[j * PL::W1S + t]
                                   : __uint_as_float((unsigned)((const unsigned short*)w1l)[j * PL::W1S + t] << 16);
          d0 += dh4[e] * wvv;
        }
      }
      dpl[t] = d0;
    }
    lds_barrier();
    // g = max-pool backward of dp, routed by the saved argmax (this thread's pixels)
#pragma unroll
    for (int i2 = 0; i2 < 4; ++i2) {
      const int col = 4 * q + i2, u = ch * 16 + (w >> 1) * 8 + (col >> 1);
      const unsigned pos = (unsigned)((w & 1) * 2 + (col & 1));
      g[i2] = pcode[u] == pos ? dpl[u] : 0.f;
    }
    if (pa.debug) st4r(cx.G + img8, hh, lane, g);
  }
  DCA_STAMP(cx, 3, L, 0);

  // ======================= backward: 10 applications, newest first ===========================================
  unsigned short* dyT = (unsigned short*)(U + PL::U_DYT);
  unsigned short* xT = (unsigned short*)(U + PL::U_XT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the dgrad weight DMA (block 9) has landed
  lds_barrier();  // every wave is done with the head's LDS (X10 / W1 / DP overlap XR / dyT / xT)
  if constexpr (P == 0) load_bfrag(WT, hh, lane, bw);  // dgrad B fragments
  for (int idx = t; idx < PL::NP * PL::XR_PL / 16; idx += NTH) ((uint4*)XR)[idx] = uint4{0u, 0u, 0u, 0u};
  for (int idx = t; idx < PL::NP * PL::XT_PL / 16; idx += NTH) ((uint4*)xT)[idx] = uint4{0u, 0u, 0u, 0u};
  f32x4 wacc[NNT][2];
#pragma unroll
  for (int j = 0; j < NNT; ++j) wacc[j][0] = wacc[j][1] = z4();
  float dgam = 0.f, dbet = 0.f;
  unsigned codew = 0;  // stem-backward prefetch (during block 0)
  unsigned imgw = 0;
  uint4 nxt = uint4{0u, 0u, 0u, 0u};
  int nxt_lab = 0;
  lds_barrier();
  f32x4 st4n = stat[(NBLK - 1) * 32 + ch];  // this channel's statistics of the next backward block, read ahead
#pragma unroll 1
  for (int i = NBLK - 1; i >= 0; --i) {
    // recover x_i = x_{i+1} - relu(bn(y_i)) (same fma, same scale / shift as the forward); BN-backward inputs
    float dz[4], xh[4], xho[4];
    float sa = 0.f, sbv = 0.f;
    const f32x4 st4 = st4n;
    const float mean = st4[0], inv = st4[1], sc = st4[2], sh = st4[3];
#pragma unroll
    for (int i2 = 0; i2 < 4; ++i2) {
      const float z = __builtin_fmaf(yv[i2], sc, sh);
      x[i2] = x[i2] - fmaxf(z, 0.f);
      xh[i2] = (yv[i2] - mean) * inv;
      dz[i2] = z > 0.f ? g[i2] : 0.f;
      sa += dz[i2];
      sbv += dz[i2] * xh[i2];
      if (halo) {
        const float zo = __builtin_fmaf(yo[i2], sc, sh);
        xo[i2] = xo[i2] - fmaxf(zo, 0.f);
        xho[i2] = (yo[i2] - mean) * inv;
      }
    }
    const int rnd = RND_HEAD + 1 + (NBLK - 1 - i);
    const unsigned tag = tagof(epoch, rnd);
    if (i == DCA_DETAIL_BWD) DCA_STAMP(cx, 7, L, 0);
    const float pv = wg_csum(sa, sbv, cred);
    if (t < 64) bn_put(pa, rnd, L, t, bn_tag(epoch, rnd), pv);
    if (halo) publish_row(pa, rnd, L, hwhich, hh, tag, dz, lane);
    if (i == DCA_DETAIL_BWD) DCA_STAMP(cx, 7, L, 1);
    // while the exchange is in flight: the weight gradient of the PREVIOUS application (block i + 1), whose dy /
    // x tiles are still staged; then the barrier retires every wave's reads of them before x_i replaces them
    if (i < NBLK - 1) wgrad_acc<P>(dyT, xT, wacc, wv, lane);
    if (i == DCA_DETAIL_BWD) DCA_STAMP(cx, 7, L, 2);
    lds_barrier();
    xt_row<P>(xT, w + 1, q, ch, x);
    if (halo) xt_row<P>(xT, hxrow, q, ch, xo);
    float dzo[4];
    if (i == DCA_DETAIL_BWD) DCA_STAMP(cx, 7, L, 3);
    xchg_wait(pa, rnd, epoch, G, cred, halo, hsrc, hwhich ^ 1, hh, dzo);
    if (i == DCA_DETAIL_BWD) DCA_STAMP(cx, 7, L, 4);
    // loads for the next block, issued AFTER the exchange (vmcnt is in order: a load in flight when a sweep
    // starts holds up its first pass); they land during this block's dgrad
    if (i > 0) {  // y_{i-1}
      ld4r(cx.Y + (size_t)(i - 1) * B * 8192 + img8, hh, lane, yv);
    } else {      // last block: what the stem backward needs (pool codes, raw input words, next batch's image)
      codew = *(const unsigned*)(cx.SCODE + img8 + hh * 256 + lane * 4);
      {
        const int ci = t / 80, rem = t % 80, xr_ = rem >> 3, yimg = 8 * s - 1 + xr_;
        const int yc = yimg < 0 ? 0 : (yimg > 31 ? 31 : yimg);
        imgw = ((const unsigned*)my_img)[(ci < 3 ? ci : 2) * 256 + yc * 8 + (rem & 7)];
      }
      if (t < 48) nxt = ((const uint4*)(cx.data + (size_t)next_id * 3072 + 768 * s))[t];
      if (t == 48) nxt_lab = cx.labels[next_id];
    }
    if (halo && i > 0) ld4r(pa.yh + ((size_t)((i - 1) * LMAX + L) * 2 + hwhich) * 512, hh, lane, yo);
    lds_barrier();
    // head outputs done: every wave's head stores (write-through) were retired by its sweep's waits (vmcnt counts
    // stores and loads in order) before this barrier -> one granule releases the fc workers
    if (i == NBLK - 1 && ra_fc(ra) && t == 0) gput(pa.hdone + L, tagof(epoch, RND_HDONE), 0.f);
    if (i == DCA_DETAIL_BWD) DCA_STAMP(cx, 7, L, 5);
    if (L == 0 && t < 32) {  // BN affine gradients: dbeta = sum dz, dgamma = sum dz * xhat
      dbet += slot_total(cred, t);
      dgam += slot_total(cred, 32 + t);
    }
    float dyv[4], dyo[4];
    {
      const float Sa = slot_total(cred, ch), Sb = slot_total(cred, 32 + ch);
      const float k1 = sc / Ntot;  // gamma * invstd: the forward's scale, bitwise
#pragma unroll
      for (int i2 = 0; i2 < 4; ++i2) {
        dyv[i2] = k1 * (Ntot * dz[i2] - Sa - xh[i2] * Sb);
        if (halo) dyo[i2] = k1 * (Ntot * dzo[i2] - Sa - xho[i2] * Sb);
      }
    }
    xr_row<P>(XR, w + 1, q, ch, dyv);
    if (halo) xr_row<P>(XR, hxrow, q, ch, dyo);
    {
      unsigned hb[4], lb[4];
#pragma unroll
      for (int i2 = 0; i2 < 4; ++i2) {
        const unsigned short hi = bfbits(dyv[i2]);
        hb[i2] = hi;
        lb[i2] = P == 1 ? bf_lo(dyv[i2], hi) : 0u;
      }
      *(uint2*)(dyT + ch * PL::DYT_S + w * 16 + 4 * q) = uint2{hb[0] | (hb[1] << 16), hb[2] | (hb[3] << 16)};
      if constexpr (P == 1)
        *(uint2*)(dyT + PL::DYT_PL / 2 + ch * PL::DYT_S + w * 16 + 4 * q) =
            uint2{lb[0] | (lb[1] << 16), lb[2] | (lb[3] << 16)};
    }
    if (pa.debug) {
      st4r(cx.DY + (size_t)i * B * 8192 + img8, hh, lane, dyv);
      st4r(cx.X + (size_t)i * B * 8192 + img8, hh, lane, x);
    }
    lds_barrier();
    if (i == DCA_DETAIL_BWD) DCA_STAMP(cx, 7, L, 6);
    // dgrad: g_i = g_{i+1} + conv(dy, W^T flipped)
    if (i > 0) st4n = stat[(i - 1) * 32 + ch];
    {
      const f32x4 acc = conv_row<P>(XR, WT, bw, w, hh, lane);
#pragma unroll
      for (int i2 = 0; i2 < 4; ++i2) g[i2] += acc[i2];
    }
    if (pa.debug && (i == 2 || i == 1)) st4r(cx.G + (size_t)(i == 2 ? 0 : 1) * B * 8192 + img8, hh, lane, g);
    DCA_STAMP(cx, 4 + (NBLK - 1 - i) / 8, L, (NBLK - 1 - i) % 8);
  }
  if (L == 0 && t < 32) {
    pa.bng[t] = dgam;
    pa.bng[32 + t] = dbet;
  }

  // ======================= stem backward: max-pool bwd (saved argmax) -> ReLU mask -> conv1 wgrad ============
  lds_barrier();  // every wave is done with XR / WT (the last dgrad); dyT / xT stay for the last wgrad
  wgrad_acc<P>(dyT, xT, wacc, wv, lane);  // application 0
  DCA_STAMP(cx, 5, L, 2);
  {
    // the lane indices re-derived from an opaque copy of threadIdx.x: nothing this phase addresses is held live
    // (and spilled) through the 20 blocks
    int tf = threadIdx.x;
    asm volatile("v_mov_b32 %0, %1" : "=v"(tf) : "v"(tf));
    const int t = tf, wv = tf >> 6, lane = tf & 63, c = lane & 15, q = lane >> 4;
    const int w = wv & (RS - 1), ch = 16 * (wv / RS) + c;
    unsigned short* dsT = (unsigned short*)(U + PL::U_DST);
    unsigned short* xs = (unsigned short*)(U + PL::U_XS);
    float* sred = (float*)(U + PL::U_SRED);
    // d(conv1 output) of this row's two conv rows, channel ch: every 2x2 window written whole (value at the
    // argmax if the ReLU was active, zeros elsewhere)
    float db = 0.f;
#pragma unroll
    for (int i2 = 0; i2 < 4; ++i2) {
      const unsigned code = (codew >> (8 * i2)) & 255u, pos = code & 3u;
      const float val = (code & 4u) ? g[i2] : 0.f;
      const unsigned short vh = bfbits(val);
      const unsigned vb = vh, vl = P == 1 ? (unsigned)bf_lo(val, vh) : 0u;
      const int so = ch * PL::DSP + (2 * w) * 32 + 2 * (4 * q + i2);
      *(unsigned*)(dsT + so) = (pos == 0 ? vb : 0u) | ((pos == 1 ? vb : 0u) << 16);
      *(unsigned*)(dsT + so + 32) = (pos == 2 ? vb : 0u) | ((pos == 3 ? vb : 0u) << 16);
      if constexpr (P == 1) {
        *(unsigned*)(dsT + PL::DST_PL / 2 + so) = (pos == 0 ? vl : 0u) | ((pos == 1 ? vl : 0u) << 16);
        *(unsigned*)(dsT + PL::DST_PL / 2 + so + 32) = (pos == 2 ? vl : 0u) | ((pos == 3 ? vl : 0u) << 16);
      }
      db += val;
    }
    // three column-shifted copies of the normalised input rows 8s-1 .. 8s+8 (copy kw holds x[col + kw - 1])
    if (t < 240) {
      const int ci = t / 80, rem = t % 80, xr_ = rem >> 3, x0 = 4 * (rem & 7), yimg = 8 * s - 1 + xr_;
      const bool valid = yimg >= 0 && yimg < 32;
      unsigned hb[4], lb[4];
#pragma unroll
      for (int b2 = 0; b2 < 4; ++b2) {
        const float v = valid ? norm_px((imgw >> (8 * b2)) & 255u, ci) : 0.f;
        const unsigned short hi = bfbits(v);
        hb[b2] = hi;
        lb[b2] = P == 1 ? bf_lo(v, hi) : 0u;
      }
#pragma unroll
      for (int p = 0; p <= P; ++p) {
        const unsigned* bb = p ? lb : hb;
        unsigned short* base = xs + p * (PL::XS_PL / 2);
        unsigned short* p1 = base + ((3 + ci) * PL::XSR + xr_) * PL::XS_S + x0;  // kw = 1
        *(uint2*)p1 = uint2{bb[0] | (bb[1] << 16), bb[2] | (bb[3] << 16)};
        unsigned short* p0 = base + ((0 + ci) * PL::XSR + xr_) * PL::XS_S + x0;  // kw = 0: col c holds x[c - 1]
        p0[1] = (unsigned short)bb[0];
        *(unsigned*)(p0 + 2) = bb[1] | (bb[2] << 16);
        if (x0 + 4 < 32) p0[4] = (unsigned short)bb[3];
        if (x0 == 0) p0[0] = 0;
        unsigned short* p2 = base + ((6 + ci) * PL::XSR + xr_) * PL::XS_S + x0;  // kw = 2: col c holds x[c + 1]
        if (x0 > 0) p2[-1] = (unsigned short)bb[0];
        *(unsigned*)p2 = bb[1] | (bb[2] << 16);
        p2[2] = (unsigned short)bb[3];
        if (x0 == 28) p2[3] = 0;
      }
    }
    // conv1 bias gradient partial of this workgroup (also the barrier before the MFMAs)
    const float dbv = wg_csum<true>(db, 0.f, cred);
    DCA_STAMP(cx, 5, L, 3);
    float* ss = cx.SSLAB + (size_t)L * SSLAB_N;
    if (t < 32) ss[1024 + t] = dbv;
    // D[co][k] = sum over this slice's conv pixels of ds[p][co] * im2col[p][k]; K step = one conv row (32 px).
    // Wave wv: tile wv & 3 (mt = co half, nt = k tile), conv rows 4 (wv >> 2) .. +3; k >= 27 columns are
    // discarded by the reduce
    {
      const int tile = wv & 3, mt = tile & 1, nt = tile >> 1, sr0 = 4 * (wv >> 2);
      const int kidx = 16 * nt + c, kk = kidx < 27 ? kidx : 0, ci = kk / 9, kh = (kk % 9) / 3, kw = kk % 3;
      const unsigned short* abase = dsT + (16 * mt + c) * PL::DSP + 8 * q;
      const unsigned short* bbase = xs + ((kw * 3 + ci) * PL::XSR + kh) * PL::XS_S + 8 * q;
      f32x4 acc2 = z4();
#pragma unroll
      for (int sr = sr0; sr < sr0 + 4; ++sr) {
        const bf16x8 a = *(const bf16x8*)(abase + sr * 32);
        const bf16x8 bb = *(const bf16x8*)(bbase + sr * PL::XS_S);
        bf16x8 al = a, bl = bb;
        if constexpr (P == 1) {
          al = *(const bf16x8*)(abase + PL::DST_PL / 2 + sr * 32);
          bl = *(const bf16x8*)(bbase + PL::XS_PL / 2 + sr * PL::XS_S);
        }
        acc2 = mma3<P>(a, al, bb, bl, acc2);
      }
      st4(sred + ((wv * 64 + lane) << 2), acc2);
    }
    lds_barrier();
    if (t < 256) {
      const int tile = t >> 6, ln = t & 63;
      st4_wt(ss + ((tile * 64 + ln) << 2), ld4(sred + ((tile * 64 + ln) << 2)) + ld4(sred + (((tile + 4) * 64 + ln) << 2)));
    }
  }
  DCA_STAMP(cx, 5, L, 4);
  // the next batch's image n (this slice's quarter) and label, staged into the other parity
  if (t < 48) st4_wt((uint4*)(pa.simg + (size_t)((par ^ 1) * 64 + n) * 3072 + 768 * s) + t, __builtin_bit_cast(f32x4, nxt));
  if (t == 48 && s == 0) pa.slab[(par ^ 1) * 64 + n] = nxt_lab;
  // trunk wgrad slab (accumulated over the 10 applications): tile tt = 2 nt + mt, the layout the reduction reads.
  // (Issued here, last: stored right after application 0's wgrad instead, the write-through stores held up the stem
  // backward's own waits -- vmcnt retires in order -- and the step was no faster.)
  int wvf = wv;  // opaque copy: the slab offsets are re-derived here, not held live (spilled) since the forward
  asm volatile("v_mov_b32 %0, %1" : "=v"(wvf) : "v"(wvf));
#pragma unroll
  for (int j = 0; j < NNT; ++j) {
    const int nt = wvf + NW * j;
    if (nt < 18) {
      st4_wt(pa.tslab + (size_t)L * WSLAB_N + (((2 * nt) * 64 + lane) << 2), wacc[j][0]);
      st4_wt(pa.tslab + (size_t)L * WSLAB_N + (((2 * nt + 1) * 64 + lane) << 2), wacc[j][1]);
    }
  }
  DCA_STAMP(cx, 5, L, 7);
}

template <int P, bool PRO>
__global__ void __launch_bounds__(NTH) k_pks_step(Ctx cx, Args pa, RedAr ra) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int gmain = (cx.B + 7) / 8 * 8 * S;
  if ((int)blockIdx.x < gmain) {
    step_main<P, PRO>(cx, pa, ra, smem);
    return;
  }
  // past the main grid: the reducers of the prologue reduction (ra_prev; the previous step's segments), then the fc
  // workers (ra_fc); one fc segment each in a training step (nfw == N_FCW); the self-test on a shared device launches
  // fewer workers (its per-rank CU budget), which then take the segments in turn
  const int fb = (int)blockIdx.x - gmain;
  if constexpr (PRO) {
    if (ra_prev(ra)) {
      prologue_reduce<P>(cx, pa, ra, fb, smem);
      __syncthreads();  // its LDS is reused by the fc segment
    }
  }
  if (!ra_fc(ra)) return;
  const int nfw = min((int)gridDim.x - gmain, N_FCW);
  for (int f = fb; f < N_FCW; f += nfw) {
    if (f != fb) __syncthreads();
    fc_segment<P>(cx, pa, ra, f, smem);
  }
}


// The first batch after the host moved the cursor or replaced the index list (grid 64 x 256): image and label of
// batch position b into the current staging parity (every later batch is staged by the step before it).
__global__ void __launch_bounds__(256) k_pks_prime(Ctx cx, Args pa) {
  const int t = threadIdx.x, b = blockIdx.x, par = *pa.epoch & 1, id = sample_id(cx, b);  // (a chunk's first step)
  if (t < 192)
    ((uint4*)(pa.simg + (size_t)(par * 64 + b) * 3072))[t] = ((const uint4*)(cx.data + (size_t)id * 3072))[t];
  if (t == 192) pa.slab[par * 64 + b] = cx.labels[id];
}

// ============================================================================================================
// The reduction kernel after the step: the trunk / conv1 chunks and the BN tail (plus the fc1 blocks and the fc
// tail when the step kernel did not run them), each followed by its exchange and SGD; one more workgroup does the
// step's bookkeeping.  mode 3 (self-test): every segment, no bookkeeping.
// ============================================================================================================
// grid: reduce_grid(ra) + 1
__host__ __device__ inline int reduce_segments(int fc_in_step, int seg_ch) {
  return fc_in_step ? seg_layout(seg_ch).r_ts + 1 : seg_layout(seg_ch).nseg;
}

// dynamic LDS: stage_floats(cx.B) * 4 bytes (fc-segment staging)
// Grid: nred + 1 workgroups (one segment each, the last one the bookkeeping), or -- ranks sharing one device
// (shared-GPU rehearsal) -- at most the per-rank CU budget: workgroup b then runs segments b, b + grid, ... in turn
// and the last workgroup also does the bookkeeping.  Every segment's exchange only waits for the SAME segment of the
// peers, and each rank visits its segments in the same order, so the looped form cannot deadlock among reductions;
// its point is that a rank's spinning reduction never holds more CUs than its step kernel (a step workgroup needs a
// whole CU: 256 VGPRs), so a late peer always finds room for its step.
template <int LEAN>
__global__ void __launch_bounds__(256) k_pks_reduce_ar(Ctx cx, Args pa, int nslab, RedAr ra) {
  __shared__ __attribute__((aligned(16))) float segv[SEG_MAX];
  __shared__ f32x4 red[256];
  extern __shared__ __attribute__((aligned(16))) float stage[];
  __shared__ int s_ep[2];
  const int nred = reduce_segments(ra_fc(ra), ra.seg_ch), b = blockIdx.x, nwg = gridDim.x;
  const SegLayout Ls = seg_layout(ra.seg_ch);
  if (nwg > nred) {
    if (b >= nred) {
      if (ra.mode != 3) pks_bookkeeping(cx, pa, ra_chunk(ra));
      return;
    }
    const int seg = !ra_fc(ra) || b < Ls.r_ts ? b : Ls.bnt;
    DCA_STAMP(cx, 8, b, 0);
    seg_process<256, false, LEAN>(cx, pa, ra, seg, nslab, segv, red, stage, s_ep, 8, b);
    return;
  }
  for (int k = b; k < nred; k += nwg) {
    const int seg = !ra_fc(ra) || k < Ls.r_ts ? k : Ls.bnt;
    seg_process<256, false, LEAN>(cx, pa, ra, seg, nslab, segv, red, stage, s_ep, 8, k);
    __syncthreads();  // segv / red / stage are reused by the next segment
  }
  if (b == nwg - 1 && ra.mode != 3) pks_bookkeeping(cx, pa, ra_chunk(ra));
}

}  // namespace pks
}  // namespace dca
