// C ABI of the generic xGMI collective library (libdca_comm.so), driven from parallel/xgmi.py.
//
// A communicator = this rank's IPC-exported shared region (csrc/xgmi_comm.hip layout) + its peers' regions
// mapped into this process.  Handles are exchanged by the host over the torch process group (RCCL or gloo);
// all-reduces are enqueued on the caller's HIP stream and are graph-capturable (no host sync, no memset).
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>

#include "xgmi_comm.hip"

namespace {
thread_local std::string g_err;
#define CMCK(x)                                               \
  do {                                                        \
    hipError_t e_ = (x);                                      \
    if (e_ != hipSuccess) {                                   \
      g_err = std::string(#x) + ": " + hipGetErrorString(e_); \
      return -1;                                              \
    }                                                         \
  } while (0)
#define REQUIRE(c, msg) \
  do {                  \
    if (!(c)) {         \
      g_err = msg;      \
      return -1;        \
    }                   \
  } while (0)

using namespace dca::comm;

struct Comm {
  int rank = 0, W = 1, nb = 0;
  long long slab_bytes = 0;
  char* region = nullptr;
  char* base[MAXR] = {};
  bool mapped[MAXR] = {};
  bool open = false;
  unsigned* err = nullptr;
};

// Modelled crossover between one-shot ((W-1)*S bytes in per rank, one flag round trip) and two-shot
// (2(W-1)/W*S bytes, two round trips): one-shot while (W-1)(1-2/W)*S <= L*B, with L ~ 5 us per flag round trip
// and B ~ 350 GB/s of peer-read bandwidth per GPU (7 links).  W <= 2: one-shot always moves no more bytes.
constexpr double ROUND_TRIP_BYTES = 5e-6 * 350e9;
}  // namespace

extern "C" {

const char* dca_comm_last_error() { return g_err.c_str(); }
int dca_comm_abi_version() { return 1; }
long long dca_comm_flag_bytes() { return (long long)FLAG_BYTES; }

// slab_bytes: largest bucket on the wire (n * 4 for fp32, n * 2 for bf16), rounded up to 4 KiB internally.
// nb: workgroups per call (every call launches exactly nb).
int dca_comm_create(int rank, int world, long long slab_bytes, int nb, void** out) {
  REQUIRE(world >= 1 && world <= MAXR && rank >= 0 && rank < world, "comm_create: 1 <= world <= 8, 0 <= rank < world");
  REQUIRE(nb >= 1 && nb <= NB_MAX, "comm_create: 1 <= nb <= 1024");
  REQUIRE(slab_bytes > 0 && slab_bytes <= (1ll << 30), "comm_create: 0 < slab_bytes <= 1 GiB");
  Comm* c = new Comm();
  c->rank = rank;
  c->W = world;
  c->nb = nb;
  c->slab_bytes = (slab_bytes + 4095) / 4096 * 4096;
  const size_t bytes = FLAG_BYTES + 4 * (size_t)c->slab_bytes;
  hipError_t e = hipExtMallocWithFlags((void**)&c->region, bytes, hipDeviceMallocUncached);
  if (e == hipSuccess) e = hipMemset(c->region, 0, bytes);
  if (e == hipSuccess) e = hipMalloc(&c->err, sizeof(unsigned));
  if (e == hipSuccess) e = hipMemset(c->err, 0, sizeof(unsigned));
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    g_err = std::string("comm_create: ") + hipGetErrorString(e);
    if (c->region) (void)hipFree(c->region);
    if (c->err) (void)hipFree(c->err);
    delete c;
    return -1;
  }
  c->base[rank] = c->region;
  *out = c;
  return 0;
}

int dca_comm_ipc_handle(void* h, char* out64) {
  Comm* c = (Comm*)h;
  static_assert(sizeof(hipIpcMemHandle_t) == 64, "unexpected hipIpcMemHandle_t size");
  hipIpcMemHandle_t hd;
  CMCK(hipIpcGetMemHandle(&hd, c->region));
  memcpy(out64, &hd, 64);
  return 0;
}

// all: world x 64-byte handles in rank order (this rank's own entry is ignored).
int dca_comm_open(void* h, const char* all) {
  Comm* c = (Comm*)h;
  REQUIRE(!c->open, "comm_open: already open");
  for (int q = 0; q < c->W; ++q) {
    if (q == c->rank) continue;
    hipIpcMemHandle_t hd;
    memcpy(&hd, all + 64 * q, 64);
    void* p = nullptr;
    CMCK(hipIpcOpenMemHandle(&p, hd, hipIpcMemLazyEnablePeerAccess));
    c->base[q] = (char*)p;
    c->mapped[q] = true;
  }
  c->open = true;
  return 0;
}

// algo: 0 auto (modelled crossover), 1 one-shot, 2 two-shot.  Writes the chosen algorithm to *used (may be null).
int dca_comm_allreduce(void* h, const float* src, float* dst, long long n, int wire_bf16, int algo, float scale,
                       float timeout_s, void* stream, int* used) {
  Comm* c = (Comm*)h;
  REQUIRE(c->open || c->W == 1, "allreduce: peers not mapped (call open first)");
  REQUIRE(n > 0, "allreduce: empty buffer");
  REQUIRE(((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0, "allreduce: src/dst must be 16-byte aligned");
  const long long wire = wire_bf16 ? 2 : 4;
  REQUIRE((n + 3) / 4 * 4 * wire <= c->slab_bytes, "allreduce: bucket larger than the communicator's slab");
  REQUIRE(algo >= 0 && algo <= 2, "allreduce: algo must be 0 (auto), 1 (one-shot) or 2 (two-shot)");
  if (algo == 0) {
    const double S = (double)n * wire, W = c->W;
    algo = (W <= 2 || (W - 1) * (1 - 2 / W) * S <= ROUND_TRIP_BYTES) ? 1 : 2;
  }
  if (used) *used = algo;
  Args a{};
  for (int q = 0; q < MAXR; ++q) a.base[q] = c->base[q < c->W ? q : c->rank];
  a.src = src;
  a.dst = dst;
  a.n = n;
  a.slab_bytes = c->slab_bytes;
  a.err = c->err;
  a.deadline = (unsigned long long)((double)timeout_s * 1e8);
  a.scale = scale;
  a.W = c->W;
  a.me = c->rank;
  a.nb = c->nb;
  hipStream_t st = (hipStream_t)stream;
  const dim3 g(c->nb), b(T);
  if (wire_bf16 && algo == 2) hipLaunchKernelGGL((k_allreduce<true, true>), g, b, 0, st, a);
  else if (wire_bf16) hipLaunchKernelGGL((k_allreduce<true, false>), g, b, 0, st, a);
  else if (algo == 2) hipLaunchKernelGGL((k_allreduce<false, true>), g, b, 0, st, a);
  else hipLaunchKernelGGL((k_allreduce<false, false>), g, b, 0, st, a);
  CMCK(hipGetLastError());
  return 0;
}

// Synchronous read of the error word (bit 0: a flag wait hit its deadline); reset clears it.
int dca_comm_errors(void* h, unsigned* out, int reset) {
  Comm* c = (Comm*)h;
  CMCK(hipDeviceSynchronize());
  CMCK(hipMemcpy(out, c->err, sizeof(unsigned), hipMemcpyDeviceToHost));
  if (reset) CMCK(hipMemset(c->err, 0, sizeof(unsigned)));
  return 0;
}

// Every rank must have finished all its calls (host barrier) before any rank destroys: peers read this region.
int dca_comm_destroy(void* h) {
  Comm* c = (Comm*)h;
  if (!c) return 0;
  (void)hipDeviceSynchronize();
  for (int q = 0; q < MAXR; ++q)
    if (c->mapped[q]) (void)hipIpcCloseMemHandle(c->base[q]);
  if (c->region) (void)hipFree(c->region);
  if (c->err) (void)hipFree(c->err);
  delete c;
  return 0;
}

}  // extern "C"
