// Native runtime of the NetResDeep training engine: owns the device workspace, enqueues the fused kernel
// sequence of one training step, captures it (including the RCCL gradient collectives) into a hipGraph per
// batch size and replays it.  Exposed to Python through a small C ABI (ctypes), see runtime/engine.py.
//
// DDP semantics (reference main.py:63, torch DDP):
//   * gradients are averaged over ranks: sum all-reduce + 1/world_size scaling fused into the SGD kernel;
//   * bucket A (fc1/fc2, 86.6 % of the bytes) is all-reduced on a comm stream while the 10 trunk backward kernels
//     run (the reference's single 25 MiB bucket gives zero overlap);
//   * bucket B (trunk conv, BN affine, stem) carries rank 0's BN running statistics in a 64-float tail segment,
//     which replaces DDP's per-forward buffer broadcast (CC4) at zero extra collective latency.
#include <rccl/rccl.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "netresdeep_kernels.hip"
#include "xgmi_allreduce.hip"
#include "netresdeep_pks.hip"

namespace {

thread_local std::string g_err;

#define HIPCK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      g_err = std::string(#x) + ": " + hipGetErrorString(e_);                      \
      return -1;                                                                   \
    }                                                                              \
  } while (0)
#define NCCK(x)                                                                    \
  do {                                                                             \
    ncclResult_t r_ = (x);                                                         \
    if (r_ != ncclSuccess) {                                                       \
      g_err = std::string(#x) + ": " + ncclGetErrorString(r_);                     \
      return -1;                                                                   \
    }                                                                              \
  } while (0)

}  // namespace

extern "C" {

// Must match runtime/engine.py::_DcaInit field by field.
struct DcaInit {
  float* params;
  float* grads;
  float* rm;
  float* rv;
  long long* nbt;
  const uint8_t* data;
  const int* labels;
  int n_data;
  int bmax;
  int bf16;
  int rows;  // trunk tile rows R (2 or 4)
  float lr;
  float bn_mom;
  float bn_eps;
  int world_size;
  int rank;
  const char* nccl_id;  // 128 bytes (world_size > 1)
  int persistent;       // 1: the one-launch image-sliced persistent step kernel (netresdeep_pks.hip)
  int debug;            // persistent engine: also store X / DY / G / conv1 pre-activations for diagnostics
  int pk_waves;         // unused (kept for ABI layout; must be 0 or 8)
  int comm_mode;        // world_size > 1: 0 = RCCL inside the step; 1 = external (host drives the all-reduce
                        // between dca_engine_run_part(.., 1) and (.., 2); test/debug path, no RCCL communicator);
                        // 2 = xGMI one-shot (peer-to-peer reads of IPC-mapped gradient slabs, fused with SGD)
  int force_comm;       // comm_mode 0 at world_size 1: still run the RCCL all-reduce + averaging SGD (tests)
  int auto_engine;      // the persistent engine was chosen automatically: keep one workgroup of co-residency
                        // slack (else the caller asked for it explicitly and may use every CU)
  int loopback;         // world_size 1, comm_mode 2: run the xGMI exchange path with this rank as its own single
                        // peer (uncached region, slab write-through, flags, peer reads, averaging SGD), so the
                        // protocol's per-step cost is measurable on one device (bench.py --loopback)
};

}  // extern "C"

namespace dca {

struct Engine {
  DcaInit in{};
  Ctx base{};
  int R = 4, RW = 16, TPI = 4;
  bool bf = true;
  hipStream_t st = nullptr, cst = nullptr;
  hipEvent_t evA = nullptr, evB = nullptr, evC = nullptr;
  char* wsp = nullptr;
  size_t ws_bytes = 0;
  int* indices = nullptr;
  int n_indices = 0;
  // dca_engine_run_checked: pinned host copies of the two error words per in-flight chunk + their events
  unsigned* err_host = nullptr;  // [CHK_RING][2]
  hipEvent_t chk_ev[4] = {};
  ncclComm_t comm = nullptr;
  // comm_mode 2 (xGMI one-shot): this rank's shared region and every rank's mapping of it
  char* xregion = nullptr;
  xg::Peers peers{};
  bool peers_open = false;
  unsigned long long ar_deadline = 300ull * 100000000ull;  // 300 s in 100 MHz ticks (a peer may be in host code)
  std::map<int, hipGraphExec_t> graphs;
  bool persistent = false;  // the image-sliced persistent step kernel (netresdeep_pks.hip; default)
  pks::Args qa{};
  bool comm_on = false;  // the step ends with a gradient collective (world_size > 1, or force_comm)
  int resident = 0;      // persistent engine: live step workgroups allowed in one grid (coresident_budget, 1 rank)
  int per_cu = 0, ncu = 0;  // persistent engine: step workgroups per CU (occupancy) and CUs of the device
  int staged_b = 0;  // persistent engine: batch slots of the current staging parity that hold the next batch
  int last_b = 0;    // batch size of the last enqueued step (BN slots are re-zeroed when it changes)
  int fc_in_step = 1;  // the fc1 / fc-tail gradient segments run on the step kernel's fc workers (pks::N_FCW extra
                       // workgroups beside the backward); off: in the reduction kernel.  Off whenever the step and
                       // its fc workers would exceed the co-resident budget, and when xGMI peers share this device
  // chunks apply each step's gradient segments in the next step's launch (prologue_ok).  Off by default: same box,
  // 300 steps bf16, 84.3 / 84.7 us with it against 83.3 / 83.0 us without (profiles/prologue_ab_r5h.log); the
  // reducers' latency lands on the stem's critical path.  DCA_PKS_PROLOGUE=1 turns it on (bitwise equal: tests).
  int prologue = 0;
  int shared_device = 0;  // set by the host: number of xGMI ranks on this device (shared-GPU rehearsal; 0/1: not
                          // shared): the coarse 107-segment layout, and fc workers only when every co-scheduled
                          // grid fits (fc_in_step_for), so a spinning kernel always leaves CUs for a peer's step
  std::map<std::string, void*> regions;
  // dynamic LDS sizes
  size_t s_stem = 0, s_fwd = 0, s_head1 = 0, s_head2 = 0, s_dgrad = 0, s_dgrad0 = 0, s_wgrad = 0, s_fc = 0;
  // kernel entry points for the selected (BF, R, RW) instantiation
  void (*kstem)(Ctx) = nullptr;
  void (*kfwd)(Ctx, int) = nullptr;
  void (*khead1)(Ctx) = nullptr;
  void (*khead2)(Ctx) = nullptr;
  void (*kbwd)(Ctx, int) = nullptr;
  void (*kred)(Ctx, int, int) = nullptr;
  void (*kapply)(Ctx, int) = nullptr;
};

static size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

template <bool BF, int R, int RW>
static void bind_kernels(Engine* e) {
  e->kstem = k_stem_block0<BF, R>;
  e->kfwd = k_fwd_block<BF, R>;
  e->khead1 = k_head1<R>;
  e->khead2 = k_head2<R>;
  using L = LdsPlan<BF, R, RW>;
  e->s_stem = L::stem;
  e->s_fwd = L::fwd;
  e->s_head1 = L::head1;
  e->s_head2 = L::head2;
  e->s_dgrad = L::dgrad;
  e->s_dgrad0 = L::dgrad0;
  e->s_wgrad = L::wgrad;
  e->s_fc = L::fc;
  e->kbwd = k_bwd_block<BF, R, RW>;
  e->kred = k_reduce<BF>;
  e->kapply = k_apply_sgd<BF>;
}

static int alloc_workspace(Engine* e) {
  const size_t bmax = e->in.bmax;
  const size_t pstride = bmax * e->TPI;
  const size_t nslab = 9 * bmax * (16 / e->RW) + pstride;
  const size_t esz = e->bf ? 2 : 4;
  struct R_ {
    const char* name;
    size_t bytes;
  } regs[] = {
      {"X", 10 * bmax * 8192 * 4},   {"Y", 10 * bmax * 8192 * 4},     {"DY", 10 * bmax * 8192 * 4},
      {"G", 2 * bmax * 8192 * 4},    {"SCODE", bmax * 8192},          {"FPART", 10 * pstride * 32 * 8},
      {"STATS", 10 * 32 * 8},        {"BPART", 2 * pstride * 32 * 8}, {"WSLAB", nslab * WSLAB_N * 4},
      {"SSLAB", pstride * SSLAB_N * 4}, {"HP", bmax * 2048 * 4},      {"HH", bmax * 32 * 4},
      {"HDH", bmax * 32 * 4},        {"HDL", bmax * 16 * 4},          {"HLOSS", bmax * 4},
      {"HPART", pstride * 32 * 4},   {"HCODE", bmax * 2048},
      {"WT_F", 9216 * esz},          {"WT_D", 9216 * esz},            {"SW", 1024 * esz},
      {"RS_BASE", 64 * 4},           {"CURSOR", 16},                  {"STEPS", 16},
      {"LOSS", 16},                  {"STAMPS", 32 * 256 * 8 * 2 * 8},
      {"EPOCH", 16},                 {"ERR", 16},
      {"TSLAB", bmax * pks::S * WSLAB_N * 4}, {"BNG", 64 * 4}, {"W1B", 65536 * 2}, {"SIMG", 2 * 64 * 3072},
      {"SLAB", 2 * 64 * 4},
      {"COMMT", 16}, {"PKW", PKW_N * 2},
      {"PKS_GRAN", 2 * (size_t)pks::LMAX * pks::GSTR * 8}, {"PKS_YH", 10 * (size_t)pks::LMAX * 2 * 512 * 4},
      {"PKS_BNX", 2 * (size_t)pks::LMAX * 64 * 4},
      {"PKS_HDONE", (size_t)pks::LMAX * 8 + 256 * 8},  // head-done | prologue ready granules
      {"C1", e->in.debug ? bmax * 32 * 1024 * 4 : 16},
  };
  size_t total = 0;
  for (auto& r : regs) total += align_up(r.bytes, 256);
  HIPCK(hipMalloc(&e->wsp, total));
  HIPCK(hipMemset(e->wsp, 0, total));
  e->ws_bytes = total;
  size_t off = 0;
  for (auto& r : regs) {
    e->regions[r.name] = e->wsp + off;
    off += align_up(r.bytes, 256);
  }
  Ctx& c = e->base;
  c.X = (float*)e->regions["X"];
  c.Y = (float*)e->regions["Y"];
  c.DY = (float*)e->regions["DY"];
  c.G = (float*)e->regions["G"];
  c.SCODE = (uint8_t*)e->regions["SCODE"];
  c.FPART = (float2*)e->regions["FPART"];
  c.STATS = (float2*)e->regions["STATS"];
  c.BPART = (float2*)e->regions["BPART"];
  c.WSLAB = (float*)e->regions["WSLAB"];
  c.SSLAB = (float*)e->regions["SSLAB"];
  c.HP = (float*)e->regions["HP"];
  c.HH = (float*)e->regions["HH"];
  c.HDH = (float*)e->regions["HDH"];
  c.HDL = (float*)e->regions["HDL"];
  c.HLOSS = (float*)e->regions["HLOSS"];
  c.HPART = (float*)e->regions["HPART"];
  c.HCODE = (uint8_t*)e->regions["HCODE"];
  c.wt_f = e->regions["WT_F"];
  c.wt_d = e->regions["WT_D"];
  c.sw = e->regions["SW"];
  c.rs_base = (float*)e->regions["RS_BASE"];
  c.cursor = (int*)e->regions["CURSOR"];
  c.step_count = (int*)e->regions["STEPS"];
  c.loss_acc = (double*)e->regions["LOSS"];
  c.pstride = (int)pstride;
  c.stamps = (unsigned long long*)e->regions["STAMPS"];
  // derived weight copies: each engine writes only the layouts its kernels read (derive_param skips null ones)
  c.swf = nullptr;
  if (e->persistent) {
    c.w1b = e->regions["W1B"];
    c.pkw = (unsigned short*)e->regions["PKW"];
    c.wt_f = c.wt_d = c.sw = nullptr;
  } else {
    c.w1b = nullptr;
    c.pkw = nullptr;
  }
  pks::Args& qa = e->qa;
  qa.gran = (unsigned long long*)e->regions["PKS_GRAN"];
  qa.bnx = (unsigned*)e->regions["PKS_BNX"];
  qa.hdone = (unsigned long long*)e->regions["PKS_HDONE"];
  qa.epoch = (int*)e->regions["EPOCH"];
  qa.err = (unsigned*)e->regions["ERR"];
  qa.tslab = (float*)e->regions["TSLAB"];
  qa.bng = (float*)e->regions["BNG"];
  qa.simg = (uint8_t*)e->regions["SIMG"];
  qa.slab = (int*)e->regions["SLAB"];
  qa.yh = (float*)e->regions["PKS_YH"];
  qa.c1 = (float*)e->regions["C1"];
  qa.debug = e->in.debug;
  return 0;
}

static int set_lds_limits(Engine* e) {
  const size_t dg = std::max(std::max(e->s_dgrad, e->s_dgrad0), std::max(e->s_wgrad, e->s_fc));
  HIPCK(hipFuncSetAttribute((const void*)e->kstem, hipFuncAttributeMaxDynamicSharedMemorySize, (int)e->s_stem));
  HIPCK(hipFuncSetAttribute((const void*)e->kfwd, hipFuncAttributeMaxDynamicSharedMemorySize, (int)e->s_fwd));
  HIPCK(hipFuncSetAttribute((const void*)e->khead1, hipFuncAttributeMaxDynamicSharedMemorySize, (int)e->s_head1));
  HIPCK(hipFuncSetAttribute((const void*)e->khead2, hipFuncAttributeMaxDynamicSharedMemorySize, (int)e->s_head2));
  HIPCK(hipFuncSetAttribute((const void*)e->kbwd, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dg));
  HIPCK(hipFuncSetAttribute((const void*)pks::k_pks_step<0, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            pks::Plan<0>::TOTAL));
  HIPCK(hipFuncSetAttribute((const void*)pks::k_pks_step<1, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            pks::Plan<1>::TOTAL));
  HIPCK(hipFuncSetAttribute((const void*)pks::k_pks_step<0, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            pks::Plan<0>::TOTAL));
  HIPCK(hipFuncSetAttribute((const void*)pks::k_pks_step<1, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            pks::Plan<1>::TOTAL));

  return 0;
}

// comm_mode 2: the one-shot xGMI all-reduce fused with the averaging SGD (replaces all-reduce + k_apply_sgd)
static int enqueue_xgmi_sgd(Engine* e, const Ctx& cx) {
  if (!e->peers_open) {
    g_err = "xGMI all-reduce: peers not mapped (call dca_engine_ipc_open first)";
    return -1;
  }
  if (e->bf)
    hipLaunchKernelGGL(xg::k_xgmi_ar_sgd<true>, dim3(xg::AR_NB), dim3(xg::AR_T), 0, e->st, cx, e->peers,
                       (const float*)cx.grads, (float*)nullptr, e->qa.err + 1, 1, e->ar_deadline);
  else
    hipLaunchKernelGGL(xg::k_xgmi_ar_sgd<false>, dim3(xg::AR_NB), dim3(xg::AR_T), 0, e->st, cx, e->peers,
                       (const float*)cx.grads, (float*)nullptr, e->qa.err + 1, 1, e->ar_deadline);
  HIPCK(hipGetLastError());
  return 0;
}

// Persistent path: the sliced step kernel, then ONE kernel for reduction + all-reduce + SGD (mode: see
// k_pks_reduce_ar).  `part`: 0 = the whole step; 1 = compute up to (not including) the gradient all-reduce;
// 2 = what follows it (averaging SGD + CC4 base).  Parts 1/2 exist for comm_mode 1, where the host runs the
// all-reduce in between.
// grid of the sliced step: S workgroups per image, image slots rounded up to a multiple of 8 (see k_pks_step)
static int pks_grid(int B) { return (B + 7) / 8 * 8 * pks::S; }
// the step workgroups that stay resident and spin in its exchanges (the padding ids of pks_grid exit at once)
static int pks_live(int B) { return B * pks::S; }

// Co-residency budget: how many spinning workgroups ONE rank may have resident at once -- one rule for a device of
// its own and a device shared by n ranks (the shared-GPU rehearsal).  Every workgroup of a persistent grid must be
// resident together; the occupancy answer can be one block per CU high near register edges (MI355X guide,
// Residency), so a margin stays free: one block per CU when several fit, else one CU -- unless the caller asked
// for the whole (dedicated) device explicitly.  Ranks sharing the device split what is left evenly: a rank's step
// (+ fc workers) and its reduction grid stay within its share, so a late rank always finds room for its step
// however the others are spread over their steps and reductions.  (Before round 5 the shared share was
// slots / n with no margin; 8 ranks x batch 8 filled it exactly and a BN exchange timed out.)
// Mirrored in Python: runtime/engine.py coresident_budget (CPU-tested).
static int coresident_budget(int per_cu, int ncu, int n_share, bool full_device) {
  const int slots = per_cu * ncu;
  const int margin = per_cu > 1 ? ncu : (full_device && n_share <= 1 ? 0 : 1);
  return (slots - margin) / std::max(n_share, 1);
}
static int share_budget(const Engine* e) {
  return e->shared_device > 1 ? coresident_budget(e->per_cu, e->ncu, e->shared_device, false) : e->resident;
}
// gradient-segment layout (pks::seg_layout): trunk / conv1 chunks of 128 elements, 256 on a shared device (fewer
// reduction workgroups: they must leave CUs for a peer's step)
static int seg_ch(const Engine* e) { return e->shared_device > 1 ? 256 : 128; }

// Whether the step at batch B runs the fc gradient segments on fc workers (the live step + N_FCW fits the budget).
static bool fc_in_step_for(const Engine* e, int B) {
  return e->fc_in_step && pks_live(B) + pks::N_FCW <= share_budget(e);
}
// Reduction grid: one workgroup per segment + the bookkeeping one; shared device: capped at the rank's budget
// (k_pks_reduce_ar then loops over the segments).
static int reduce_grid(const Engine* e, int nred_plus) {
  return e->shared_device > 1 ? std::min(nred_plus, share_budget(e)) : nred_plus;
}

// Whether a chunk of steps at batch B may apply each step's gradient segments in the NEXT step's launch (the
// prologue reduction, netresdeep_pks.hip): the SGD must be fused into the segments (world size 1 or xGMI; RCCL and
// the host all-reduce sit between reduction and SGD), the fc workers run in the step (the prologue leaves the fc
// segments to them), and the reducers fit beside the live step within the co-residency budget.
// Off by default (one reduction kernel after every step); DCA_PKS_PROLOGUE=1 turns it on.  With the xGMI exchange the
// step's ready wait is bounded by the exchange deadline (netresdeep_pks.hip wait_ready), and the form is covered by a
// two-rank shared-device test (tests/test_ddp_engine_gpu.py::test_xgmi_prologue_two_ranks_one_gpu).
static bool prologue_ok(const Engine* e, int B) {
  if (!e->persistent || !e->prologue) return false;
  if (e->comm_on && e->in.comm_mode != 2) return false;
  if (!fc_in_step_for(e, B)) return false;
  return pks_live(B) + std::max(pks::N_FCW, pks::prologue_segments(seg_ch(e))) <= share_budget(e);
}

// The sliced step kernel: step s of its chunk; prev: the previous step's segments are applied in its prologue.
static int enqueue_pks_step(Engine* e, int B, int s, bool prev) {
  Ctx cx = e->base;
  cx.B = B;
  const bool multi = e->comm_on, xgmi = multi && e->in.comm_mode == 2;
  if (xgmi && !e->peers_open) {
    g_err = "xGMI all-reduce: peers not mapped (call dca_engine_ipc_open first)";
    return -1;
  }
  if (pks_live(B) > share_budget(e)) {  // (set_shared_device already refused batch_max; kept as the last guard)
    g_err = "persistent engine: " + std::to_string(pks_live(B)) + " step workgroups (batch " + std::to_string(B) +
            ") exceed the co-residency budget of " + std::to_string(share_budget(e)) + " per rank";
    return -1;
  }
  pks::RedAr ra{};
  ra.peers = e->peers;
  ra.err = e->qa.err + 1;
  ra.deadline = e->ar_deadline;
  ra.mode = !multi ? 0 : (xgmi ? 2 : 1);
  const bool fc = fc_in_step_for(e, B);
  ra.fc_in_step = pks::ra_flags(fc, prev, s, 0);
  ra.seg_ch = seg_ch(e);
  const int extra = fc ? std::max(pks::N_FCW, prev ? pks::prologue_segments(ra.seg_ch) : 0) : 0;
  const dim3 grid(pks_grid(B) + extra);
  // (the prologue form only where this launch applies the previous step's segments)
  const dim3 blk(pks::NTH);
  if (e->bf && prev)
    hipLaunchKernelGGL((pks::k_pks_step<0, true>), grid, blk, pks::Plan<0>::TOTAL, e->st, cx, e->qa, ra);
  else if (e->bf)
    hipLaunchKernelGGL((pks::k_pks_step<0, false>), grid, blk, pks::Plan<0>::TOTAL, e->st, cx, e->qa, ra);
  else if (prev)
    hipLaunchKernelGGL((pks::k_pks_step<1, true>), grid, blk, pks::Plan<1>::TOTAL, e->st, cx, e->qa, ra);
  else
    hipLaunchKernelGGL((pks::k_pks_step<1, false>), grid, blk, pks::Plan<1>::TOTAL, e->st, cx, e->qa, ra);
  HIPCK(hipGetLastError());
  return 0;
}

// The reduction kernel closing a chunk of `chunk` steps (the last step's segments + its bookkeeping, epoch and
// cursor advanced by the chunk); then, RCCL / host all-reduce (mode 1), the collective and the averaging SGD.
// part: 0 whole; 1 up to the all-reduce; 2 the SGD after it (comm_mode 1, the host runs the all-reduce between).
static int enqueue_pks_reduce(Engine* e, int B, int chunk, int part) {
  Ctx cx = e->base;
  cx.B = B;
  const bool multi = e->comm_on, xgmi = multi && e->in.comm_mode == 2;
  if (part != 2) {
    pks::RedAr ra{};
    ra.peers = e->peers;
    ra.err = e->qa.err + 1;
    ra.deadline = e->ar_deadline;
    ra.mode = !multi ? 0 : (xgmi ? 2 : 1);
    const bool fc = fc_in_step_for(e, B);
    ra.fc_in_step = pks::ra_flags(fc, false, 0, chunk);
    ra.seg_ch = seg_ch(e);
    const dim3 rgrid(reduce_grid(e, pks::reduce_segments(fc, ra.seg_ch) + 1));
    // the lean forms (no fc segments, one exchange mode): world size 1, or the xGMI exchange (also on a shared
    // device, so the multi-rank rehearsals run the form a multi-GPU node runs)
    const int lean = !fc ? 0 : (ra.mode == 0 ? 1 : (ra.mode == 2 ? 2 : 0));
    const size_t lds = pks::stage_floats(B) * 4;
    if (lean == 1)
      hipLaunchKernelGGL(pks::k_pks_reduce_ar<1>, rgrid, dim3(256), lds, e->st, cx, e->qa, B * pks::S, ra);
    else if (lean == 2)
      hipLaunchKernelGGL(pks::k_pks_reduce_ar<2>, rgrid, dim3(256), lds, e->st, cx, e->qa, B * pks::S, ra);
    else
      hipLaunchKernelGGL(pks::k_pks_reduce_ar<0>, rgrid, dim3(256), lds, e->st, cx, e->qa, B * pks::S, ra);
  }
  if (multi && !xgmi) {  // RCCL (comm_mode 0, captured) or the host (comm_mode 1, between parts 1 and 2)
    if (part == 0) NCCK(ncclAllReduce(cx.grads, cx.grads, FLAT_N, ncclFloat32, ncclSum, e->comm, e->st));
    if (part != 1) hipLaunchKernelGGL(e->kapply, dim3(64), dim3(NT), 0, e->st, cx, 1);
  }
  HIPCK(hipGetLastError());
  return 0;
}

// One step followed by its own reduction (a chunk of 1): eager runs, the host all-reduce, RCCL.
static int enqueue_step_persistent(Engine* e, int B, int part) {
  if (part != 2 && enqueue_pks_step(e, B, 0, false)) return -1;
  return enqueue_pks_reduce(e, B, 1, part);
}

// Enqueue one full training step for batch B on e->st (and e->cst for the collectives).
static int enqueue_step(Engine* e, int B, int part = 0);
// Enqueue `chunk` consecutive steps: with the prologue reduction `chunk` step kernels and one reduction kernel (one
// kernel boundary per step), else step + reduction each.
static int enqueue_chunk(Engine* e, int B, int chunk) {
  if (!prologue_ok(e, B)) {
    for (int s = 0; s < chunk; ++s)
      if (enqueue_step(e, B)) return -1;
    return 0;
  }
  for (int s = 0; s < chunk; ++s)
    if (enqueue_pks_step(e, B, s, s > 0)) return -1;
  return enqueue_pks_reduce(e, B, chunk, 0);
}

static int enqueue_step(Engine* e, int B, int part) {
  if (e->persistent) return enqueue_step_persistent(e, B, part);
  Ctx cx = e->base;
  cx.B = B;
  if (part == 2) {  // external all-reduce done: averaging SGD + CC4 base
    hipLaunchKernelGGL(e->kapply, dim3(64), dim3(NT), 0, e->st, cx, 1);
    HIPCK(hipGetLastError());
    return 0;
  }
  const int nparts = B * e->TPI, nw = B * (16 / e->RW);
  const int nslab = 9 * nw + nparts;
  const dim3 blk(NT);
  hipLaunchKernelGGL(e->kstem, dim3(nparts), blk, e->s_stem, e->st, cx);
  for (int i = 1; i < NBLK; ++i) hipLaunchKernelGGL(e->kfwd, dim3(nparts), blk, e->s_fwd, e->st, cx, i);
  hipLaunchKernelGGL(e->khead1, dim3(nparts), blk, e->s_head1, e->st, cx);
  hipLaunchKernelGGL(e->khead2, dim3(nparts), blk, e->s_head2, e->st, cx);
  for (int i = NBLK - 1; i >= 0; --i) {
    const int extra = (i == NBLK - 1) ? N_FC_WG : nw;
    size_t lds = (i == 0) ? e->s_dgrad0 : e->s_dgrad;
    lds = std::max(lds, (i < NBLK - 1) ? e->s_wgrad : e->s_fc);
    hipLaunchKernelGGL(e->kbwd, dim3(nparts + extra), blk, lds, e->st, cx, i);
    if (i == NBLK - 1 && e->comm_on && part == 0 && e->in.comm_mode == 0) {  // bucket A ready: overlap its all-reduce with the trunk bwd
      HIPCK(hipEventRecord(e->evA, e->st));
      HIPCK(hipStreamWaitEvent(e->cst, e->evA, 0));
      NCCK(ncclAllReduce(cx.grads, cx.grads, BUCKET_A_END, ncclFloat32, ncclSum, e->comm, e->cst));
    }
  }
  const int nother = cx.fuse_sgd ? 64 : 0;
  hipLaunchKernelGGL(e->kred, dim3(N_TRUNK_RED_WG + N_STEM_RED_WG + nother + 1), blk, 0, e->st, cx, nslab, nparts);
  if (e->comm_on && part == 0 && e->in.comm_mode == 2) return enqueue_xgmi_sgd(e, cx);
  if (e->comm_on && part == 0) {
    HIPCK(hipEventRecord(e->evB, e->st));
    HIPCK(hipStreamWaitEvent(e->cst, e->evB, 0));
    NCCK(ncclAllReduce(cx.grads + OFF_CONVW, cx.grads + OFF_CONVW, FLAT_N - OFF_CONVW, ncclFloat32, ncclSum, e->comm,
                       e->cst));
    HIPCK(hipEventRecord(e->evC, e->cst));
    HIPCK(hipStreamWaitEvent(e->st, e->evC, 0));
    hipLaunchKernelGGL(e->kapply, dim3(64), blk, 0, e->st, cx, 1);
  }
  HIPCK(hipGetLastError());
  return 0;
}

}  // namespace dca


using dca::Engine;

extern "C" {

const char* dca_last_error() { return g_err.c_str(); }

int dca_abi_version() { return 7; }  // bump with every DcaInit / signature change

int dca_nccl_unique_id(char* out128) {
  ncclUniqueId id;
  NCCK(ncclGetUniqueId(&id));
  static_assert(sizeof(ncclUniqueId) == 128, "unexpected ncclUniqueId size");
  memcpy(out128, &id, 128);
  return 0;
}

static int prime_ids(Engine* e);
static void engine_free(Engine* e);

// Body of dca_engine_create; on failure the caller frees whatever was acquired (engine_free handles a partially
// built engine), so every early return of HIPCK / NCCK is leak-free.
static int engine_init(Engine* e, const DcaInit* in, int n_indices) {
  e->in = *in;
  e->bf = in->bf16 != 0;
  e->R = in->rows;
  e->RW = e->bf ? 16 : 8;
  if (in->bmax < 1 || in->bmax > dca::BMAX_LIMIT) {
    g_err = "batch_max must be in [1, 64]";
    return -1;
  }
  if (e->R != 2 && e->R != 4) {
    g_err = "rows must be 2 or 4";
    return -1;
  }
  e->TPI = 16 / e->R;
  e->persistent = in->persistent != 0;
  if (in->pk_waves != 0 && in->pk_waves != 8) {
    g_err = "persistent engine: pk_waves must be 8";
    return -1;
  }
  // comm_on: the step ends with a gradient collective + the averaging SGD kernel.  force_comm runs that path at
  // world_size 1 (a 1-rank RCCL communicator) so the graph-captured collective is testable on one GPU; loopback
  // does the same for the xGMI exchange (this rank as its only peer).
  if (in->loopback && (in->world_size != 1 || in->comm_mode != 2)) {
    g_err = "loopback needs world_size 1 and comm_mode 2 (xGMI)";
    return -1;
  }
  e->comm_on = in->world_size > 1 || (in->force_comm && in->comm_mode == 0) || in->loopback;
  if (e->bf && e->R == 4) dca::bind_kernels<true, 4, 16>(e);
  else if (e->bf) dca::bind_kernels<true, 2, 16>(e);
  else if (e->R == 4) dca::bind_kernels<false, 4, 8>(e);
  else dca::bind_kernels<false, 2, 8>(e);
  if (dca::set_lds_limits(e)) return -1;
  if (e->persistent) {
    // Co-residency: the persistent step spins on in-kernel exchanges, so every one of its bmax workgroups must be
    // resident at once.  The occupancy answer can be one block per CU high near register edges (MI355X guide,
    // Residency): require a margin of one block per CU below it.
    int dev = 0, ncu = 0, per_cu = 0;
    HIPCK(hipGetDevice(&dev));
    HIPCK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    if (e->bf)
      HIPCK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)dca::pks::k_pks_step<0, false>, dca::pks::NTH,
                                                        dca::pks::Plan<0>::TOTAL));
    else
      HIPCK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)dca::pks::k_pks_step<1, false>, dca::pks::NTH,
                                                        dca::pks::Plan<1>::TOTAL));
    // one step workgroup per CU (256 VGPRs): a grid of every CU would leave no slack for anything else on the
    // device (another stream's kernel, another process), so an automatically chosen engine keeps a margin of one
    // workgroup -- batch 64 (256 workgroups) then falls back to the multi-kernel engine with a warning; an
    // explicit persistent=True may use every CU (coresident_budget)
    const int resident = dca::coresident_budget(per_cu, ncu, 1, !in->auto_engine);
    const int need = dca::pks_live(in->bmax);
    e->per_cu = per_cu;
    e->ncu = ncu;
    if (resident < need) {
      g_err = "persistent engine: " + std::to_string(need) + " workgroups cannot all be resident (" +
              std::to_string(per_cu) + " per CU x " + std::to_string(ncu) + " CUs); use the multi-kernel engine";
      return -1;
    }
    e->resident = resident;
    if (const char* fo = getenv("DCA_PKS_FC_IN_STEP")) e->fc_in_step = fo[0] != '0';
    if (const char* po = getenv("DCA_PKS_PROLOGUE")) e->prologue = po[0] != '0';
    if (e->prologue) {  // the prologue form is a separate instantiation: it must be as resident as the default one
      int per_cu_pro = 0;
      HIPCK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
          &per_cu_pro, e->bf ? (const void*)dca::pks::k_pks_step<0, true> : (const void*)dca::pks::k_pks_step<1, true>,
          dca::pks::NTH, e->bf ? dca::pks::Plan<0>::TOTAL : dca::pks::Plan<1>::TOTAL));
      if (per_cu_pro < per_cu) e->prologue = 0;
    }
  }
  HIPCK(hipStreamCreateWithFlags(&e->st, hipStreamNonBlocking));
  HIPCK(hipStreamCreateWithFlags(&e->cst, hipStreamNonBlocking));
  HIPCK(hipEventCreateWithFlags(&e->evA, hipEventDisableTiming));
  HIPCK(hipEventCreateWithFlags(&e->evB, hipEventDisableTiming));
  HIPCK(hipEventCreateWithFlags(&e->evC, hipEventDisableTiming));
  for (auto& ev : e->chk_ev) HIPCK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  HIPCK(hipHostMalloc((void**)&e->err_host, 4 * 2 * sizeof(unsigned), hipHostMallocDefault));
  memset(e->err_host, 0, 4 * 2 * sizeof(unsigned));
  if (dca::alloc_workspace(e)) return -1;
  e->n_indices = n_indices;
  HIPCK(hipMalloc(&e->indices, sizeof(int) * (size_t)std::max(n_indices, 1)));
  HIPCK(hipMemset(e->indices, 0, sizeof(int) * (size_t)std::max(n_indices, 1)));
  dca::Ctx& c = e->base;
  c.ws = in->world_size;
  c.rank = in->rank;
  c.fuse_sgd = e->comm_on ? 0 : 1;
  c.lr = in->lr;
  c.bn_mom = in->bn_mom;
  c.bn_eps = in->bn_eps;
  c.inv_ws = 1.f / (float)in->world_size;
  c.params = in->params;
  c.grads = in->grads;
  c.rm = in->rm;
  c.rv = in->rv;
  c.nbt = in->nbt;
  c.data = in->data;
  c.labels = in->labels;
  c.indices = e->indices;
  c.n_data = in->n_data;
  c.n_idx = std::max(n_indices, 1);
  e->peers.ticks = (unsigned long long*)e->regions["COMMT"];
  if ((in->world_size > 1 || in->loopback) && in->comm_mode == 2) {
    if (in->world_size > dca::xg::MAXR) {
      g_err = "xGMI all-reduce: world_size > 8 (one node) -- use RCCL";
      return -1;
    }
    // uncached device memory: peers read it over xGMI and no L2 may hold a stale line of it
    // two halves: [0, REGION_BYTES) k_xgmi_ar_sgd (multi-kernel / per-image engines); [REGION_BYTES, 2x) the
    // sliced engine's fused reduce + all-reduce (own flags and slabs: their epochs never mix)
    if (hipExtMallocWithFlags((void**)&e->xregion, 2 * dca::xg::REGION_BYTES, hipDeviceMallocUncached) != hipSuccess) {
      (void)hipGetLastError();
      HIPCK(hipMalloc(&e->xregion, 2 * dca::xg::REGION_BYTES));
    }
    HIPCK(hipMemset(e->xregion, 0, 2 * dca::xg::REGION_BYTES));
    HIPCK(hipDeviceSynchronize());
    const char* dl = getenv("DCA_XGMI_TIMEOUT_S");
    if (dl) e->ar_deadline = (unsigned long long)(atof(dl) * 1e8);
    if (in->loopback) {  // the rank is its own (only) peer: no IPC mapping
      e->peers.base[0] = e->xregion;
      e->peers_open = true;
    }
  }
  if (e->comm_on && in->comm_mode == 0) {
    ncclUniqueId id;
    if (in->world_size == 1) NCCK(ncclGetUniqueId(&id));  // force_comm: a private 1-rank communicator
    else memcpy(&id, in->nccl_id, 128);
    NCCK(ncclCommInitRank(&e->comm, in->world_size, id, in->rank));
  }
  if (prime_ids(e)) return -1;
  HIPCK(hipStreamSynchronize(e->st));
  return 0;
}

int dca_engine_create(const DcaInit* in, int n_indices, void** out) {
  Engine* e = new Engine();
  if (engine_init(e, in, n_indices)) {
    const std::string err = g_err;
    engine_free(e);
    g_err = err;
    return -1;
  }
  *out = e;
  return 0;
}

// Release everything an Engine holds; safe on a partially initialised engine.
static void engine_free(Engine* e) {
  if (e->st) (void)hipStreamSynchronize(e->st);
  if (e->cst) (void)hipStreamSynchronize(e->cst);
  for (auto& kv : e->graphs) (void)hipGraphExecDestroy(kv.second);
  if (e->comm) (void)ncclCommDestroy(e->comm);
  for (int q = 0; q < dca::xg::MAXR; ++q)
    if (e->peers_open && !e->in.loopback && q != e->in.rank && q < e->in.world_size && e->peers.base[q])
      (void)hipIpcCloseMemHandle(e->peers.base[q]);
  if (e->xregion) (void)hipFree(e->xregion);
  if (e->wsp) (void)hipFree(e->wsp);
  if (e->indices) (void)hipFree(e->indices);
  if (e->err_host) (void)hipHostFree(e->err_host);
  for (auto& ev : e->chk_ev)
    if (ev) (void)hipEventDestroy(ev);
  if (e->evA) (void)hipEventDestroy(e->evA);
  if (e->evB) (void)hipEventDestroy(e->evB);
  if (e->evC) (void)hipEventDestroy(e->evC);
  if (e->st) (void)hipStreamDestroy(e->st);
  if (e->cst) (void)hipStreamDestroy(e->cst);
  delete e;
}

int dca_engine_destroy(void* h) {
  if (h) engine_free((Engine*)h);
  return 0;
}

// Rebuild the MFMA-layout weight copies from the fp32 parameters (after init / load_state_dict / broadcast)
// and snapshot the running stats as the rank-0 base.  Synchronous.
int dca_engine_derive(void* h) {
  Engine* e = (Engine*)h;
  hipLaunchKernelGGL(e->kapply, dim3(64), dim3(dca::NT), 0, e->st, e->base, 0);
  HIPCK(hipGetLastError());
  HIPCK(hipStreamSynchronize(e->st));
  return 0;
}

// persistent engine: the batch ids of the next step are produced by the previous step; re-derive them whenever
// the host moves the cursor or replaces the index list
static int prime_ids(Engine* e) {
  if (!e->persistent) return 0;  // the multi-kernel engine gathers its batch inside the stem kernel
  hipLaunchKernelGGL(dca::pks::k_pks_prime, dim3(64), dim3(256), 0, e->st, e->base, e->qa);
  HIPCK(hipGetLastError());
  e->staged_b = 64;
  return 0;
}
// A persistent step of batch B stages only B slots of the next batch; a following larger batch re-primes.
static int ensure_staged(Engine* e, int B) {
  if (e->persistent && B > e->staged_b && prime_ids(e)) return -1;
  if (e->persistent) e->staged_b = B;
  // sliced engine: a workgroup absent from the last steps (smaller batch) left BN slots whose 2-bit tags could
  // match again; zeroed slots (tag 0) never match (bn_tag)
  if (e->persistent && B != e->last_b) {
    HIPCK(hipMemsetAsync(e->qa.bnx, 0, 2 * (size_t)dca::pks::LMAX * 64 * 4, e->st));
  }
  e->last_b = B;
  return 0;
}

int dca_engine_set_indices(void* h, const int* host_idx, int n) {
  Engine* e = (Engine*)h;
  if (n > e->n_indices) {
    g_err = "too many indices";
    return -1;
  }
  HIPCK(hipMemcpyAsync(e->indices, host_idx, sizeof(int) * (size_t)n, hipMemcpyHostToDevice, e->st));
  if (prime_ids(e)) return -1;
  HIPCK(hipStreamSynchronize(e->st));
  return 0;
}

int dca_engine_set_cursor(void* h, int v) {
  Engine* e = (Engine*)h;
  HIPCK(hipMemcpyAsync(e->base.cursor, &v, sizeof(int), hipMemcpyHostToDevice, e->st));
  if (prime_ids(e)) return -1;
  HIPCK(hipStreamSynchronize(e->st));
  return 0;
}

// Seed the step epoch (and, xGMI, every exchange flag of this rank's region) -- the epoch-wrap test hook: e.g.
// EPOCH_WRAP - 3 and 2^32 - 3, so the next steps cross both wraps (pks::EPOCH_WRAP for the device epoch: staging
// parity, BN tags, granule tags; 2^32 for the per-segment / per-workgroup exchange flags).  Every tag holder whose
// validity depends on the epoch (BN partial slots, halo / head granules, head-done granules) is zeroed, because an
// arbitrary jump could make a stale slot's tag match (a zero tag never does); the next batch is re-staged into the
// new epoch's parity.  xGMI: collective -- every rank seeds the same flag value while no rank is stepping (barrier
// before and after), since peers write into this rank's flag area.  Synchronous.
int dca_engine_set_epoch(void* h, int device_epoch, int flag_epoch) {
  Engine* e = (Engine*)h;
  if (!e->persistent) {
    g_err = "set_epoch: the sliced (persistent) engine only";
    return -1;
  }
  if (device_epoch < 0 || (unsigned)device_epoch >= dca::pks::EPOCH_WRAP) {
    g_err = "set_epoch: device epoch outside [0, EPOCH_WRAP)";
    return -1;
  }
  HIPCK(hipStreamSynchronize(e->st));
  HIPCK(hipMemcpy(e->qa.epoch, &device_epoch, sizeof(int), hipMemcpyHostToDevice));
  HIPCK(hipMemset(e->qa.gran, 0, 2 * (size_t)dca::pks::LMAX * dca::pks::GSTR * 8));
  HIPCK(hipMemset(e->qa.bnx, 0, 2 * (size_t)dca::pks::LMAX * 64 * 4));
  HIPCK(hipMemset(e->qa.hdone, 0, (size_t)dca::pks::LMAX * 8 + 256 * 8));
  if (e->xregion) {
    std::vector<int> f(dca::xg::FLAG_BYTES / 4, flag_epoch);
    HIPCK(hipMemcpy(e->xregion, f.data(), dca::xg::FLAG_BYTES, hipMemcpyHostToDevice));                 // k_xgmi_ar_sgd
    HIPCK(hipMemcpy(e->xregion + dca::xg::REGION_BYTES, f.data(), dca::xg::FLAG_BYTES, hipMemcpyHostToDevice));  // segments
  }
  if (prime_ids(e)) return -1;
  HIPCK(hipStreamSynchronize(e->st));
  return 0;
}

// The current device epoch (synchronous).
int dca_engine_epoch(void* h, int* out) {
  Engine* e = (Engine*)h;
  HIPCK(hipStreamSynchronize(e->st));
  HIPCK(hipMemcpy(out, e->qa.epoch, sizeof(int), hipMemcpyDeviceToHost));
  return 0;
}

// Device-side error flags: flags[0] of the persistent engine (bit r: BN exchange round r timed out),
// flags[1] of the xGMI all-reduce (bit 31: a peer-flag wait timed out).  Synchronises; reset clears them.
int dca_engine_errors(void* h, unsigned* flags, int reset) {
  Engine* e = (Engine*)h;
  HIPCK(hipStreamSynchronize(e->st));
  HIPCK(hipMemcpy(flags, e->qa.err, 2 * sizeof(unsigned), hipMemcpyDeviceToHost));
  if (reset) HIPCK(hipMemset(e->qa.err, 0, 2 * sizeof(unsigned)));
  return 0;
}

// Read (and optionally reset) the device-side loss accumulator.  Synchronises the engine stream.
int dca_engine_read_loss(void* h, double* loss, int* steps, int reset) {
  Engine* e = (Engine*)h;
  HIPCK(hipStreamSynchronize(e->st));
  HIPCK(hipMemcpy(loss, e->base.loss_acc, sizeof(double), hipMemcpyDeviceToHost));
  HIPCK(hipMemcpy(steps, e->base.step_count, sizeof(int), hipMemcpyDeviceToHost));
  if (reset) {
    HIPCK(hipMemset(e->base.loss_acc, 0, sizeof(double)));
    HIPCK(hipMemset(e->base.step_count, 0, sizeof(int)));
  }
  return 0;
}

// Enqueue `nsteps` training steps of batch B.  use_graph: replay a captured hipGraph (captured on first use).
constexpr int GRAPH_CHUNK = 16;  // steps per graph replay (remainders: 8 / 4 / 2 / 1-step graphs, <= 4 extra launches)

// The executable graph of `chunk` consecutive steps of batch B (captured and instantiated on first use).
static hipGraphExec_t capture_graph(Engine* e, int B, int chunk) {
  const int key = B * 1024 + chunk;
  auto it = e->graphs.find(key);
  if (it != e->graphs.end()) return it->second;
  hipGraph_t g;
  hipError_t ec = hipStreamBeginCapture(e->st, hipStreamCaptureModeThreadLocal);
  if (ec != hipSuccess) {
    g_err = std::string("hipStreamBeginCapture: ") + hipGetErrorString(ec);
    return nullptr;
  }
  const int rc = dca::enqueue_chunk(e, B, chunk);
  ec = hipStreamEndCapture(e->st, &g);
  if (rc) {
    if (ec == hipSuccess) (void)hipGraphDestroy(g);
    return nullptr;
  }
  if (ec != hipSuccess) {
    g_err = std::string("hipStreamEndCapture: ") + hipGetErrorString(ec);
    return nullptr;
  }
  hipGraphExec_t ex;
  ec = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  if (ec != hipSuccess) {
    g_err = std::string("hipGraphInstantiate: ") + hipGetErrorString(ec);
    return nullptr;
  }
  // upload now (stream-ordered), so the first replay -- possibly inside a timed region -- does not pay it
  ec = hipGraphUpload(ex, e->st);
  if (ec != hipSuccess) {
    (void)hipGraphExecDestroy(ex);
    g_err = std::string("hipGraphUpload: ") + hipGetErrorString(ec);
    return nullptr;
  }
  e->graphs.emplace(key, ex);
  return ex;
}

int dca_engine_run(void* h, int B, int nsteps, int use_graph) {
  Engine* e = (Engine*)h;
  if (B < 1 || B > e->in.bmax) {
    g_err = "batch out of range";
    return -1;
  }
  if (e->in.world_size > 1 && e->in.comm_mode == 1) {
    g_err = "comm_mode 1 (external all-reduce): drive steps with dca_engine_run_part";
    return -1;
  }
  if (nsteps > 0 && ensure_staged(e, B)) return -1;
  if (!use_graph) {
    for (int s = 0; s < nsteps; ++s)
      if (dca::enqueue_step(e, B)) return -1;
    return 0;
  }
  // Steps are replayed from graphs holding GRAPH_CHUNK consecutive steps (the data cursor / batch ids advance
  // on the device, so consecutive steps need no host input): launching one graph per step leaves a ~5-8 us
  // gap between graph launches on the GPU (rocprofv3, profiles/), inside a graph consecutive kernels are
  // back to back.
  int done = 0;
  for (const int chunk : {GRAPH_CHUNK, 8, 4, 2, 1}) {
    const int reps = (nsteps - done) / chunk;
    if (reps == 0) continue;
    hipGraphExec_t ex = capture_graph(e, B, chunk);
    if (ex == nullptr) return -1;
    for (int r = 0; r < reps; ++r) HIPCK(hipGraphLaunch(ex, e->st));
    done += reps * chunk;
  }
  return 0;
}

// dca_engine_run with the device error words checked after EVERY graph chunk, without stalling the GPU: behind each
// chunk an async copy of the two words into pinned host memory and an event; before launching chunk k + 2 the host
// waits for chunk k's event (chunk k + 1 keeps the GPU busy meanwhile) and reads its words.  An exchange timeout
// (BN exchange of the step, or a peer that stopped stepping in the xGMI all-reduce) therefore stops the run within
// two 8-step chunks (< 16 steps) instead of at the epoch end; after the first timed-out wait the kernels do not wait
// again (fail fast on the error word), so those steps are quick.  Returns 0, or 1 when an error word was set (*steps_done:
// steps of the chunks enqueued before stopping; the words stay set for dca_engine_errors); -1 on a HIP error.
// Synchronous: the stream is drained before returning.
int dca_engine_run_checked(void* h, int B, int nsteps, int* steps_done) {
  Engine* e = (Engine*)h;
  constexpr int RING = 4;
  *steps_done = 0;
  if (B < 1 || B > e->in.bmax || nsteps < 0) {
    g_err = "batch out of range";
    return -1;
  }
  if (e->in.world_size > 1 && e->in.comm_mode == 1) {
    g_err = "comm_mode 1 (external all-reduce): drive steps with dca_engine_run_part";
    return -1;
  }
  if (nsteps > 0 && ensure_staged(e, B)) return -1;
  int left = nsteps;
  std::vector<int> order;  // graph chunk sizes in launch order (16s, then 8 / 4 / 2 / 1)
  for (const int chunk : {8, 4, 2, 1})  // 8-step chunks: a failure is seen within < 16 steps (2 chunks in flight)
    for (; left >= chunk; left -= chunk) order.push_back(chunk);
  int launched = 0, rc = 0;
  size_t k = 0, checked = 0;
  auto check = [&](size_t j) -> int {  // chunk j's words (its event first)
    hipEvent_t ev = e->chk_ev[j % RING];
    if (hipEventSynchronize(ev) != hipSuccess) return -1;
    const unsigned* w = e->err_host + 2 * (j % RING);
    return (w[0] | w[1]) ? 1 : 0;
  };
  for (; k < order.size(); ++k) {
    if (k >= 2) {  // keep <= 2 chunks in flight behind the check
      const int r = check(checked++);
      if (r < 0) HIPCK(hipGetLastError());
      if (r) {
        rc = 1;
        break;
      }
    }
    hipGraphExec_t ex = capture_graph(e, B, order[k]);
    if (ex == nullptr) return -1;
    HIPCK(hipGraphLaunch(ex, e->st));
    HIPCK(hipMemcpyAsync(e->err_host + 2 * (k % RING), e->qa.err, 2 * sizeof(unsigned), hipMemcpyDeviceToHost, e->st));
    HIPCK(hipEventRecord(e->chk_ev[k % RING], e->st));
    launched += order[k];
  }
  while (rc == 0 && checked < k) {
    const int r = check(checked++);
    if (r < 0) HIPCK(hipGetLastError());
    if (r) rc = 1;
  }
  HIPCK(hipStreamSynchronize(e->st));
  *steps_done = launched;
  return rc;
}

// Capture (without running) the graphs dca_engine_run replays for batch B, so a later timed run never pays
// capture + instantiate.  Synchronous.
int dca_engine_precapture(void* h, int B) {
  Engine* e = (Engine*)h;
  if (B < 1 || B > e->in.bmax) {
    g_err = "batch out of range";
    return -1;
  }
  if (e->in.world_size > 1 && e->in.comm_mode == 1) return 0;  // external all-reduce: eager only
  for (const int chunk : {GRAPH_CHUNK, 8, 4, 2, 1})
    if (capture_graph(e, B, chunk) == nullptr) return -1;
  HIPCK(hipStreamSynchronize(e->st));
  return 0;
}

// Time spent inside the gradient all-reduce kernel (xGMI path: workgroup 0 of k_xgmi_ar_sgd, entry to exit,
// including the wait for the slowest peer), summed since the last reset: microseconds and calls.
int dca_engine_comm_time(void* h, double* us, long long* calls, int reset) {
  Engine* e = (Engine*)h;
  HIPCK(hipStreamSynchronize(e->st));
  unsigned long long v[2] = {0, 0};
  HIPCK(hipMemcpy(v, e->peers.ticks, sizeof(v), hipMemcpyDeviceToHost));
  *us = (double)v[0] / 100.0;  // s_memrealtime: 100 MHz
  *calls = (long long)v[1];
  if (reset) HIPCK(hipMemset(e->peers.ticks, 0, sizeof(v)));
  return 0;
}

// comm_mode 2: the IPC handle (64 bytes) of this rank's shared region, to be all-gathered by the host.
int dca_engine_ipc_handle(void* h, char* out64) {
  Engine* e = (Engine*)h;
  if (!e->xregion) {
    g_err = "ipc_handle: engine not created with comm_mode 2";
    return -1;
  }
  static_assert(sizeof(hipIpcMemHandle_t) == 64, "unexpected hipIpcMemHandle_t size");
  hipIpcMemHandle_t hd;
  HIPCK(hipIpcGetMemHandle(&hd, e->xregion));
  memcpy(out64, &hd, 64);
  return 0;
}

// comm_mode 2: map every peer's region (`all` = world_size handles of 64 bytes, in rank order).
int dca_engine_ipc_open(void* h, const char* all, int world) {
  Engine* e = (Engine*)h;
  if (!e->xregion || world != e->in.world_size) {
    g_err = "ipc_open: engine not created with comm_mode 2, or world size mismatch";
    return -1;
  }
  for (int q = 0; q < world; ++q) {
    if (q == e->in.rank) {
      e->peers.base[q] = e->xregion;
      continue;
    }
    hipIpcMemHandle_t hd;
    memcpy(&hd, all + 64 * q, 64);
    void* p = nullptr;
    HIPCK(hipIpcOpenMemHandle(&p, hd, hipIpcMemLazyEnablePeerAccess));
    e->peers.base[q] = (char*)p;
  }
  e->peers_open = true;
  return 0;
}

// comm_mode 2 self-test: one all-reduce (no SGD) of `n = FLAT_N` floats from device `src` into device `dst`
// through the same protocol, epochs and slabs as a training step.  Collective: every rank must call it.
// timeout_s bounds the flag waits; returns 1 in *timed_out when a wait expired.  Synchronous.
int dca_engine_ipc_selftest(void* h, const float* src, float* dst, float timeout_s, int* timed_out) {
  Engine* e = (Engine*)h;
  if (!e->peers_open) {
    g_err = "ipc_selftest: peers not mapped";
    return -1;
  }
  HIPCK(hipMemsetAsync(e->qa.err + 1, 0, sizeof(unsigned), e->st));
  const unsigned long long dl = (unsigned long long)((double)timeout_s * 1e8);
  if (e->persistent) {  // the path a sliced training step uses: per-segment exchange inside the fused reduce kernel
    dca::pks::RedAr ra{};
    ra.peers = e->peers;
    ra.peers.ticks = nullptr;
    ra.err = e->qa.err + 1;
    ra.deadline = dl;
    ra.st_src = src;
    ra.st_dst = dst;
    ra.st_n = dca::FLAT_N;
    ra.mode = 3;
    ra.fc_in_step = 0;  // every segment in the reduction kernel
    ra.seg_ch = dca::seg_ch(e);
    dca::Ctx cx = e->base;
    cx.B = 1;
    hipLaunchKernelGGL(dca::pks::k_pks_reduce_ar<0>, dim3(dca::reduce_grid(e, dca::pks::seg_layout(ra.seg_ch).nseg)),
                       dim3(256), dca::pks::stage_floats(1) * 4, e->st, cx, e->qa, 1, ra);
  } else {
    dca::xg::Peers P = e->peers;
    P.ticks = nullptr;  // a self-test is not training-step communication (metrics)
    if (e->bf)
      hipLaunchKernelGGL(dca::xg::k_xgmi_ar_sgd<true>, dim3(dca::xg::AR_NB), dim3(dca::xg::AR_T), 0, e->st,
                         e->base, P, src, dst, e->qa.err + 1, 0, dl);
    else
      hipLaunchKernelGGL(dca::xg::k_xgmi_ar_sgd<false>, dim3(dca::xg::AR_NB), dim3(dca::xg::AR_T), 0, e->st,
                         e->base, P, src, dst, e->qa.err + 1, 0, dl);
  }
  HIPCK(hipGetLastError());
  HIPCK(hipStreamSynchronize(e->st));
  unsigned f = 0;
  HIPCK(hipMemcpy(&f, e->qa.err + 1, sizeof(unsigned), hipMemcpyDeviceToHost));
  HIPCK(hipMemset(e->qa.err + 1, 0, sizeof(unsigned)));
  *timed_out = (f & 0x80000000u) ? 1 : 0;
  return 0;
}

// comm_mode 2, sliced engine: the same collective self-test through the STEP kernel's fc workers (the in-step
// exchange of the fc1 blocks and the fc tail that runs beside the trunk backward): k_pks_step launched with batch 0,
// i.e. N_FCW fc workers and no step workgroups, in self-test mode.  Only the fc segments' slab range is written to
// dst: [*lo, *hi).  Each fc worker waits only for the same segment of its peers, so ranks sharing a device need no
// co-residency budget here.  Collective; synchronous.
int dca_engine_ipc_selftest_fc(void* h, const float* src, float* dst, float timeout_s, int* timed_out, int* lo,
                               int* hi) {
  Engine* e = (Engine*)h;
  if (!e->peers_open || !e->persistent) {
    g_err = "ipc_selftest_fc: needs the sliced engine with mapped peers";
    return -1;
  }
  HIPCK(hipMemsetAsync(e->qa.err, 0, 2 * sizeof(unsigned), e->st));
  dca::pks::RedAr ra{};
  ra.peers = e->peers;
  ra.peers.ticks = nullptr;
  ra.err = e->qa.err + 1;
  ra.deadline = (unsigned long long)((double)timeout_s * 1e8);
  ra.st_src = src;
  ra.st_dst = dst;
  ra.st_n = dca::FLAT_N;
  ra.mode = 3;
  ra.fc_in_step = 1;
  ra.seg_ch = dca::seg_ch(e);
  dca::Ctx cx = e->base;
  cx.B = 0;  // no step workgroups: the whole grid is fc workers
  // one workgroup per fc segment, or (ranks sharing the device) the rank's CU budget: every rank's workgroup f waits
  // for its peers' workgroup f, so all ranks' grids must be co-resident (a step-kernel workgroup takes a whole CU)
  const dim3 grid(std::min(dca::pks::N_FCW, dca::share_budget(e)));
  if (e->bf)
    hipLaunchKernelGGL((dca::pks::k_pks_step<0, false>), grid, dim3(dca::pks::NTH), dca::pks::Plan<0>::TOTAL, e->st, cx, e->qa,
                       ra);
  else
    hipLaunchKernelGGL((dca::pks::k_pks_step<1, false>), grid, dim3(dca::pks::NTH), dca::pks::Plan<1>::TOTAL, e->st, cx, e->qa,
                       ra);
  HIPCK(hipGetLastError());
  HIPCK(hipStreamSynchronize(e->st));
  unsigned f[2] = {0, 0};
  HIPCK(hipMemcpy(f, e->qa.err, sizeof(f), hipMemcpyDeviceToHost));
  HIPCK(hipMemset(e->qa.err, 0, sizeof(f)));
  *timed_out = ((f[1] & 0x80000000u) || f[0]) ? 1 : 0;
  const dca::pks::SegLayout L = dca::pks::seg_layout(ra.seg_ch);
  *lo = L.off_fc1;
  *hi = std::min(L.off_fct + 362, (int)dca::FLAT_N);
  return 0;
}

// comm_mode 2 protocol latency: `iters` back-to-back all-reduces (no SGD) of FLAT_N floats; writes the mean
// microseconds per all-reduce (HIP events around the loop).  Collective: every rank must call it.
int dca_engine_ipc_bench(void* h, const float* src, float* dst, int iters, float* us) {
  Engine* e = (Engine*)h;
  if (!e->peers_open || iters < 1) {
    g_err = "ipc_bench: peers not mapped or iters < 1";
    return -1;
  }
  hipEvent_t a, b;
  HIPCK(hipEventCreate(&a));
  HIPCK(hipEventCreate(&b));
  HIPCK(hipEventRecord(a, e->st));
  dca::xg::Peers P = e->peers;
  P.ticks = nullptr;  // benchmark traffic stays out of the training comm-time counters
  for (int i = 0; i < iters; ++i) {
    if (e->persistent) {  // the exchange a sliced training step runs: every gradient segment, self-test mode
      dca::pks::RedAr ra{};
      ra.peers = P;
      ra.err = e->qa.err + 1;
      ra.deadline = e->ar_deadline;
      ra.st_src = src;
      ra.st_dst = dst;
      ra.st_n = dca::FLAT_N;
      ra.mode = 3;
      ra.fc_in_step = 0;
      ra.seg_ch = dca::seg_ch(e);
      dca::Ctx cx = e->base;
      cx.B = 1;
      hipLaunchKernelGGL(dca::pks::k_pks_reduce_ar<0>, dim3(dca::reduce_grid(e, dca::pks::seg_layout(ra.seg_ch).nseg)),
                         dim3(256), dca::pks::stage_floats(1) * 4, e->st, cx, e->qa, 1, ra);
    } else if (e->bf) {
      hipLaunchKernelGGL(dca::xg::k_xgmi_ar_sgd<true>, dim3(dca::xg::AR_NB), dim3(dca::xg::AR_T), 0, e->st,
                         e->base, P, src, dst, e->qa.err + 1, 0, e->ar_deadline);
    } else {
      hipLaunchKernelGGL(dca::xg::k_xgmi_ar_sgd<false>, dim3(dca::xg::AR_NB), dim3(dca::xg::AR_T), 0, e->st,
                         e->base, P, src, dst, e->qa.err + 1, 0, e->ar_deadline);
    }
  }
  HIPCK(hipEventRecord(b, e->st));
  HIPCK(hipEventSynchronize(b));
  float ms = 0.f;
  HIPCK(hipEventElapsedTime(&ms, a, b));
  *us = 1e3f * ms / (float)iters;
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return 0;
}

// comm_mode 1: one part of a step, eager (see enqueue_step_persistent)
int dca_engine_run_part(void* h, int B, int part) {
  Engine* e = (Engine*)h;
  if (B < 1 || B > e->in.bmax || part < 1 || part > 2 || e->in.world_size < 2 || e->in.comm_mode != 1) {
    g_err = "run_part: needs world_size > 1, comm_mode 1, part 1 or 2, batch in range";
    return -1;
  }
  if (part == 1 && ensure_staged(e, B)) return -1;
  return dca::enqueue_step(e, B, part);
}

int dca_engine_sync(void* h) {
  Engine* e = (Engine*)h;
  HIPCK(hipStreamSynchronize(e->st));
  HIPCK(hipStreamSynchronize(e->cst));
  return 0;
}

// Sliced engine: the host reports that `n` xGMI ranks share this device (shared-GPU rehearsal; the largest such
// count over all devices, so every rank picks the same layout): the coarse gradient-segment layout and the
// co-residency rule of fc_in_step_for.  Collective in effect: every rank must make the same call before
// stepping.  Drops the captured graphs.
int dca_engine_set_shared_device(void* h, int n) {
  Engine* e = (Engine*)h;
  if (e->persistent && n > 1) {
    const int budget = dca::coresident_budget(e->per_cu, e->ncu, n, false);
    if (dca::pks_live(e->in.bmax) > budget) {
      g_err = "shared device: " + std::to_string(n) + " ranks x " + std::to_string(dca::pks_live(e->in.bmax)) +
              " step workgroups (batch_max " + std::to_string(e->in.bmax) + ") exceed the per-rank co-residency budget " +
              "of " + std::to_string(budget) + " of the device's " + std::to_string(e->per_cu * e->ncu) +
              " workgroup slots (one kept free); use batch_max <= " + std::to_string(budget / dca::pks::S);
      return -1;
    }
  }
  HIPCK(hipStreamSynchronize(e->st));
  for (auto& kv : e->graphs) (void)hipGraphExecDestroy(kv.second);
  e->graphs.clear();
  e->shared_device = n > 1 ? n : 0;
  return 0;
}

// Sliced engine: 1 if a step at batch B runs the fc gradient segments on the step kernel's fc workers.
int dca_engine_fc_in_step(void* h, int B) {
  Engine* e = (Engine*)h;
  return e->persistent && fc_in_step_for(e, B) ? 1 : 0;
}

// Whether graph chunks at batch B apply each step's gradient segments in the next step's launch (prologue_ok).
int dca_engine_prologue(void* h, int B) { return dca::prologue_ok((Engine*)h, B) ? 1 : 0; }

// Handle of the engine stream (so Python can order torch work against it).
void* dca_engine_stream(void* h) { return ((Engine*)h)->st; }

// Device pointer of a named workspace region (tests / debugging).
void* dca_engine_region(void* h, const char* name) {
  Engine* e = (Engine*)h;
  auto it = e->regions.find(name);
  return it == e->regions.end() ? nullptr : it->second;
}

size_t dca_engine_workspace_bytes(void* h) { return ((Engine*)h)->ws_bytes; }

// 0: multi-kernel engine; 2: persistent, image-sliced (S workgroups per image).  (1, the retired
// one-workgroup-per-image kernel, is never returned.)
int dca_engine_kind(void* h) {
  Engine* e = (Engine*)h;
  return e->persistent ? 2 : 0;
}


}  // extern "C"
