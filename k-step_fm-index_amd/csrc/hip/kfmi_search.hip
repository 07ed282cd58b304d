/*
 * kfmi_search.hip -- MI355X (gfx950) backward search: query packing, the
 * task-per-query and wave64-cooperative LF kernels, device index layouts,
 * and the reference's GPU plugin entry points (common/interface.h:36-41):
 * transferCPUtoGPU, searchIndexGPU, transferGPUtoCPU, free*GPU.
 *
 * Semantics: results are bit-identical to the reference CPU searchers
 * (fmIndexCPUBaseline.c:157-292 for task/coop/packed, -AltCounters.c:145-310
 * for the *-ac backends) -- not to the reference .cu files, which carry the
 * defects B1-B4 of SURVEY.md Appendix B.
 */
#include <hip/hip_runtime.h>
#include <rocprim/device/device_scan.hpp>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../kfmi_internal.h"
#include "kfmi_device.h"
#include "kfmi_coop.h"
#include "kfmi_locate.h"
#include "kfmi_kernels.h"

using namespace kfmi;

/* locate bookkeeping kernels (slot counts, owners, first rows); the walk itself
 * is locate_kernel in kfmi_locate.h */
// Positions each query reports: min(R - L, max_occ) (max_occ 0 = all).  The
// count array has num + 1 slots and the last one is 0, so the exclusive scan's
// last element is the total.
static __global__ __launch_bounds__(256) void loc_count_kernel(const uint32_t* __restrict__ res, uint64_t num,
                                                        uint32_t max_occ, uint64_t* __restrict__ cnt)
{
  const uint64_t q = (uint64_t) blockIdx.x * 256 + threadIdx.x;
  if (q > num) return;
  uint64_t c = 0;
  if (q < num) {
    const uint2 lr = *reinterpret_cast<const uint2*>(res + 2 * q);
    c = lr.y > lr.x ? (uint64_t) (lr.y - lr.x) : 0u;
    if (max_occ && c > max_occ) c = max_occ;
  }
  cnt[q] = c;
}

// Owner of each output slot without a per-slot search: every query with at
// least one position writes its id at its first slot (owner[] zeroed first),
// and an inclusive max-scan spreads it over the query's slots.
static __global__ __launch_bounds__(256) void loc_heads_kernel(const uint64_t* __restrict__ cnt,
                                                        const uint64_t* __restrict__ off, uint64_t num,
                                                        uint32_t* __restrict__ owner)
{
  const uint64_t q = (uint64_t) blockIdx.x * 256 + threadIdx.x;
  if (q < num && cnt[q]) owner[off[q]] = (uint32_t) q;
}

// First row of every output slot, in place over the owner array:
// rows[i] = L of its query + the slot's rank inside the query.
static __global__ __launch_bounds__(256) void loc_rows_kernel(const uint32_t* __restrict__ res,
                                                       const uint64_t* __restrict__ off, uint64_t total,
                                                       uint32_t* __restrict__ own_rows)
{
  for (uint64_t i = (uint64_t) blockIdx.x * 256 + threadIdx.x; i < total; i += (uint64_t) gridDim.x * 256) {
    const uint32_t q = own_rows[i];   /* grid-stride: a batch may hold more than 2^32 positions */
    own_rows[i] = res[2 * (uint64_t) q] + (uint32_t) (i - off[q]);
  }
}

/* ------------------------------------------------------------------------ */
/* backend registry and per-thread state                                    */
/* ------------------------------------------------------------------------ */

static const char* kBackendNames[KFMI_BK_COUNT] = {
    "task", "coop", "task-ac", "coop-ac", "task-packed", "coop-packed", "task-mid", "coop-mid",
    "task-ac128", "coop-ac128"};

static thread_local int t_backend = -1;
static thread_local int t_device = -1;
static thread_local int32_t t_last_error = KFMI_SUCCESS;
static thread_local double t_ms[3] = {0, 0, 0};
static thread_local int t_ftab = -1;   /* ftab bases for the task kernels; -1: KFMI_FTAB, else 0 */

static int backend_from_name(const char* n)
{
  if (!n) return -1;
  for (int i = 0; i < KFMI_BK_COUNT; ++i)
    if (!strcmp(n, kBackendNames[i])) return i;
  /* reference binary names (makefile:177-207) */
  if (!strcmp(n, "task-2step") || !strcmp(n, "task-1step")) return KFMI_BK_TASK;
  if (!strcmp(n, "coop-2step") || !strcmp(n, "coop-1step")) return KFMI_BK_COOP;
  if (!strcmp(n, "task-2step-ac")) return KFMI_BK_TASK_AC;
  if (!strcmp(n, "coop-2step-ac")) return KFMI_BK_COOP_AC;
  if (!strcmp(n, "packed")) return KFMI_BK_TASK_PACKED;
  return -1;
}

extern "C" kfmi_backend_t kfmi_backend(void)
{
  if (t_backend < 0) {
    int b = backend_from_name(getenv("KFMI_BACKEND"));
    t_backend = b >= 0 ? b : KFMI_BK_TASK_MID;
  }
  return (kfmi_backend_t) t_backend;
}

extern "C" uint32_t kfmi_backend_tag(kfmi_backend_t b)
{
  return (b == KFMI_BK_TASK_AC || b == KFMI_BK_COOP_AC || b == KFMI_BK_TASK_AC128 || b == KFMI_BK_COOP_AC128)
             ? 201u : 101u;
}

extern "C" int32_t kfmi_set_backend(const char* name)
{
  int b = backend_from_name(name);
  if (b < 0) return KFMI_E_BAD_ARGUMENT;
  t_backend = b;
  return KFMI_SUCCESS;
}

extern "C" const char* kfmi_get_backend(void) { return kBackendNames[kfmi_backend()]; }

extern "C" int32_t kfmi_device_count(void)
{
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

static int group_devices(int* devs);

extern "C" int32_t kfmi_current_device(void)
{
  if (t_device < 0) {
    const char* e = getenv("KFMI_DEVICE");
    int devs[16];
    t_device = e ? atoi(e) : (group_devices(devs) == 1 ? devs[0] : 0);
  }
  return t_device;
}

extern "C" int32_t kfmi_set_device(int32_t device)
{
  int n = kfmi_device_count();
  if (device < 0 || device >= n) return KFMI_E_NO_DEVICE;
  t_device = device;
  return KFMI_SUCCESS;
}

extern "C" void kfmi_set_last_error(int32_t e) { t_last_error = e; }

extern "C" int32_t kfmi_set_ftab(uint32_t bases)
{
  if (bases > 16) return KFMI_E_BAD_ARGUMENT;
  t_ftab = (int) bases;
  return KFMI_SUCCESS;
}

static uint32_t ftab_bases(void)
{
  if (t_ftab >= 0) return (uint32_t) t_ftab;
  const char* e = getenv("KFMI_FTAB");
  const int v = e ? atoi(e) : 0;
  return v > 0 && v <= 16 ? (uint32_t) v : 0u;
}
extern "C" int32_t kfmi_last_error(void) { return t_last_error; }

extern "C" int32_t kfmi_last_timing(double* ms_total, double* ms_pack, double* ms_lf)
{
  if (ms_total) *ms_total = t_ms[0];
  if (ms_pack) *ms_pack = t_ms[1];
  if (ms_lf) *ms_lf = t_ms[2];
  return KFMI_SUCCESS;
}

/* One non-blocking stream and a set of timing events per device. */
struct DevCtx {
  bool init = false;
  hipStream_t st = nullptr;
  hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
};
static DevCtx g_ctx[64];
static std::mutex g_ctx_mu;

static int32_t ctx_for(int dev, DevCtx** out)
{
  if (dev < 0 || dev >= 64) return KFMI_E_NO_DEVICE;
  std::lock_guard<std::mutex> lk(g_ctx_mu);
  DevCtx& c = g_ctx[dev];
  if (hipSetDevice(dev) != hipSuccess) return KFMI_E_NO_DEVICE;
  if (!c.init) {
    if (hipStreamCreateWithFlags(&c.st, hipStreamNonBlocking) != hipSuccess) return KFMI_E_NO_DEVICE;
    for (int i = 0; i < 3; ++i)
      if (hipEventCreate(&c.ev[i]) != hipSuccess) return KFMI_E_NO_DEVICE;
    c.init = true;
  }
  *out = &c;
  return KFMI_SUCCESS;
}

#define HIP_OK(x)                                                                   \
  do {                                                                              \
    hipError_t _e = (x);                                                            \
    if (_e != hipSuccess) {                                                         \
      fprintf(stderr, "kstepfmi: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(_e), \
              __FILE__, __LINE__);                                                  \
      return KFMI_E_KERNEL;                                                         \
    }                                                                               \
  } while (0)

/* ------------------------------------------------------------------------ */
/* device-side handles                                                      */
/* ------------------------------------------------------------------------ */

struct kfmi_dev_index {
  int device = -1;
  int backend = -1;
  int layout = -1;
  uint32_t K = 0, d = 0, nb = 0, bwtsize = 0, nentries = 0;
  DollarArgs dl{};
  uint32_t* ent = nullptr;     /* device entries */
  uint64_t ent_bytes = 0;
  uint32_t* sb = nullptr;      /* packed: superblock counters */
  uint64_t sb_bytes = 0;
  uint32_t* sa = nullptr;      /* locate: row-sampled suffix array */
  uint64_t sa_bytes = 0;
  uint32_t sa_log2 = 0, sa_gen = 0;
  uint2* ftab = nullptr;       /* jump-start table of ftab_chars bases (0 = none) */
  uint32_t ftab_chars = 0;
};

struct kfmi_dev_queries {
  int device = -1;
  uint8_t* ascii = nullptr;    /* num*size bytes, plain layout */
  uint32_t* packed = nullptr;  /* nwords x num u32 codes */
  uint64_t num = 0;
  uint32_t size = 0, K = 0, steps = 0, nwords = 0;
};

/* ------------------------------------------------------------------------ */
/* query packing: ASCII [num][m] -> codes [nwords][num], step t of query q in */
/* word t/SPW, bits 2K*(t%SPW)..; step t consumes chars m-1-K*t-i (i<K), the  */
/* order of fmIndexCPUBaseline.c:200-226.                                   */
/* ------------------------------------------------------------------------ */

template <int K>
__global__ __launch_bounds__(256) void pack_queries_kernel(const uint8_t* __restrict__ q, uint64_t num,
                                                           uint32_t m, uint32_t steps, uint32_t nwords,
                                                           uint32_t tq, uint32_t* __restrict__ out)
{
  extern __shared__ __attribute__((aligned(16))) uint8_t tile[];
  constexpr int SPW = 32 / (2 * K);
  const uint64_t q0 = (uint64_t) blockIdx.x * tq;
  const uint64_t nq = (num - q0) < tq ? (num - q0) : tq;
  const uint64_t bytes = nq * m;
  const uint8_t* src = q + q0 * m;   /* q0*m is a multiple of 64*m: 16-byte aligned when m%... */
  if ((((uintptr_t) src) & 15u) == 0) {
    const uint64_t n16 = bytes / 16;
    for (uint64_t i = threadIdx.x; i < n16; i += blockDim.x)
      reinterpret_cast<uint4*>(tile)[i] = reinterpret_cast<const uint4*>(src)[i];
    for (uint64_t i = n16 * 16 + threadIdx.x; i < bytes; i += blockDim.x) tile[i] = src[i];
  } else {
    for (uint64_t i = threadIdx.x; i < bytes; i += blockDim.x) tile[i] = src[i];
  }
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < nq; t += blockDim.x) {
    const uint8_t* p = tile + (uint64_t) t * m;
    for (uint32_t w = 0; w < nwords; ++w) {
      uint32_t word = 0;
#pragma unroll
      for (int j = 0; j < SPW; ++j) {
        const uint32_t st = w * SPW + j;
        if (st < steps) {
          const int pos = (int) m - 1 - (int) (K * st);
          uint32_t c = 0;
#pragma unroll
          for (int i = 0; i < K; ++i) c |= code_of(p[pos - i]) << (2 * i);
          word |= c << (2 * K * j);
        }
      }
      out[(uint64_t) w * num + q0 + t] = word;
    }
  }
}


/* ------------------------------------------------------------------------ */
/* packed layout construction from tag-101 entries (on the device)          */
/* ------------------------------------------------------------------------ */

template <int K, int NB>
__global__ __launch_bounds__(256) void build_packed_kernel(const uint32_t* __restrict__ inter, uint32_t nentries,
                                                           uint32_t* __restrict__ packed, uint32_t* __restrict__ sb,
                                                           uint32_t* __restrict__ overflow)
{
  using GI = Geo<K, NB, LAY_INTER>;
  using GP = Geo<K, NB, LAY_PACKED>;
  constexpr int S = sb_shift_for(GI::D);
  const uint64_t b = (uint64_t) blockIdx.x * 256 + threadIdx.x;
  if (b >= nentries) return;
  const uint32_t* src = inter + b * GI::EW;
  const uint32_t* sup = inter + ((b >> S) << S) * GI::EW;
  uint32_t* dst = packed + b * GP::EW;
  for (int i = 0; i < GI::BMW; ++i) dst[i] = src[i];
  uint16_t* d16 = reinterpret_cast<uint16_t*>(dst);
  for (int c = 0; c < GI::NC; ++c) {
    const uint32_t delta = src[GI::BMW + c] - sup[GI::BMW + c];
    if (delta > 0xFFFFu) atomicAdd(overflow, 1u);
    d16[GP::DELTA16 + c] = (uint16_t) delta;
  }
  for (int i = GI::BMW + GI::NC / 2; i < GP::EW; ++i) dst[i] = 0;
  if ((b & ((1u << S) - 1)) == 0)
    for (int c = 0; c < GI::NC; ++c) sb[(b >> S) * GI::NC + c] = src[GI::BMW + c];
}

/* MID layout construction from tag-101 entries: line p holds the planes of
 * blocks 2p and 2p+1 and the counters sampled at its midpoint (= cnt_{2p+1}).
 * The last odd-count line and one padding line take host-computed counters
 * (rows past n+1 read as code 0, see mid_ext_counters). */
template <int K, int NB>
__global__ __launch_bounds__(256) void build_mid_kernel(const uint32_t* __restrict__ inter, uint32_t nentries,
                                                        uint32_t nlines, uint32_t* __restrict__ lines,
                                                        const uint32_t* __restrict__ ext_last,
                                                        const uint32_t* __restrict__ ext_pad)
{
  using GI = Geo<K, NB, LAY_INTER>;
  using GM = Geo<K, NB, LAY_MID>;
  const uint64_t p = (uint64_t) blockIdx.x * 256 + threadIdx.x;
  if (p >= nlines) return;
  uint32_t* dst = lines + p * GM::EW;
  for (int h = 0; h < 2; ++h) {
    const uint64_t b = 2 * p + h;
    for (int i = 0; i < GI::BMW; ++i) dst[h * GI::BMW + i] = b < nentries ? inter[b * GI::EW + i] : 0u;
  }
  for (int c = 0; c < GI::NC; ++c) {
    uint32_t v;
    if (2 * p + 1 < nentries) v = inter[(2 * p + 1) * GI::EW + GI::BMW + c];
    else if (2 * p < nentries) v = ext_last[c];
    else v = ext_pad[c];
    dst[GM::MIDCNT + c] = v;
  }
  for (int i = GM::MIDCNT + GI::NC; i < GM::EW; ++i) dst[i] = 0;
}

/* AC128 layout construction from tag-201 entries (E + 1 of them, the last
 * being the sentinel): line b = [planes of b | cnt_half_b | cnt_half_{b+1}],
 * the counters of entries past the sentinel read as 0 (as the AC backend's
 * zero padding entries do).  Lines 0 .. E plus one padding line. */
template <int K, int NB>
__global__ __launch_bounds__(256) void build_ac128_kernel(const uint32_t* __restrict__ ac, uint32_t nent,
                                                          uint32_t nlines, uint32_t* __restrict__ lines)
{
  using GA = Geo<K, NB, LAY_AC>;
  using GL = Geo<K, NB, LAY_AC128>;
  const uint64_t b = (uint64_t) blockIdx.x * 256 + threadIdx.x;
  if (b >= nlines) return;
  uint32_t* dst = lines + b * GL::EW;
  const uint32_t* src = ac + b * GA::EW;
  const uint32_t* nxt = ac + (b + 1) * GA::EW;
  for (int i = 0; i < GA::BMW; ++i) dst[i] = b < nent ? src[GA::BOFF + i] : 0u;
  for (int c = 0; c < GA::HALF; ++c) {
    dst[GA::BMW + c] = b < nent ? src[c] : 0u;
    dst[GA::BMW + GA::HALF + c] = b + 1 < nent ? nxt[c] : 0u;
  }
  for (int i = GA::BMW + 2 * GA::HALF; i < GL::EW; ++i) dst[i] = 0;
}

/* Code registers the task kernel needs to pack a query itself (0: use the
 * pack kernel).  KFMI_FUSED=0 forces the separate pack launch. */
static bool is_coop(int backend);

static int fused_maxw(int backend, uint32_t nwords)
{
  (void) backend;   /* task and coop kernels both pack in-kernel (m <= 256 fits either's LDS staging) */
  const char* e = getenv("KFMI_FUSED");
  if (e && !atoi(e)) return 0;
  return nwords <= 8 ? 8 : (nwords <= 16 ? 16 : 0);
}

static bool nb_supported(uint32_t nb)
{
  return nb == 1 || nb == 2 || nb == 4 || nb == 6 || nb == 8 || nb == 14 || nb == 30;
}

/* dispatch_one<K, NB, LAY> is compiled in kfmi_inst_*.hip (one unit per K and
 * layout, built in parallel). */
namespace kfmi {
KFMI_FOR_NB(KFMI_EXTERN, 1, LAY_INTER)
KFMI_FOR_NB(KFMI_EXTERN, 2, LAY_INTER)
KFMI_FOR_NB(KFMI_EXTERN, 1, LAY_AC)
KFMI_FOR_NB(KFMI_EXTERN, 2, LAY_AC)
KFMI_FOR_NB(KFMI_EXTERN, 1, LAY_PACKED)
KFMI_FOR_NB(KFMI_EXTERN, 2, LAY_PACKED)
KFMI_FOR_NB(KFMI_EXTERN, 1, LAY_MID)
KFMI_FOR_NB(KFMI_EXTERN, 2, LAY_MID)
KFMI_FOR_NB(KFMI_EXTERN, 1, LAY_AC128)
KFMI_FOR_NB(KFMI_EXTERN, 2, LAY_AC128)
}  // namespace kfmi

static hipError_t dispatch(Op op, uint32_t K, uint32_t nb, int lay, const SearchLaunch& a,
                           unsigned long long* d_total = nullptr)
{
#define KFMI_CASE(KK, NBV, LAYV)                                   \
  if (K == KK && nb == NBV && lay == LAYV) return dispatch_one<KK, NBV, LAYV>(op, a, d_total);
  KFMI_FOR_NB(KFMI_CASE, 1, LAY_INTER)
  KFMI_FOR_NB(KFMI_CASE, 2, LAY_INTER)
  KFMI_FOR_NB(KFMI_CASE, 1, LAY_AC)
  KFMI_FOR_NB(KFMI_CASE, 2, LAY_AC)
  KFMI_FOR_NB(KFMI_CASE, 1, LAY_PACKED)
  KFMI_FOR_NB(KFMI_CASE, 2, LAY_PACKED)
  KFMI_FOR_NB(KFMI_CASE, 1, LAY_MID)
  KFMI_FOR_NB(KFMI_CASE, 2, LAY_MID)
  KFMI_FOR_NB(KFMI_CASE, 1, LAY_AC128)
  KFMI_FOR_NB(KFMI_CASE, 2, LAY_AC128)
#undef KFMI_CASE
  return hipErrorInvalidValue;
}

/* Whether the backend's kernel exists for this geometry (the cooperative
 * kernel needs 16-byte-aligned chunks, CoopCfg::OK). */
static bool geometry_supported(int backend, uint32_t K, uint32_t nb, int lay)
{
  if (!nb_supported(nb) || (K != 1 && K != 2)) return false;
  if (!is_coop(backend)) return true;
#define KFMI_OKC(KK, NBV, LAYV) \
  if (K == KK && nb == NBV && lay == LAYV) return CoopCfg<Geo<KK, NBV, LAYV>>::OK;
  KFMI_FOR_NB(KFMI_OKC, 1, LAY_INTER)
  KFMI_FOR_NB(KFMI_OKC, 2, LAY_INTER)
  KFMI_FOR_NB(KFMI_OKC, 1, LAY_AC)
  KFMI_FOR_NB(KFMI_OKC, 2, LAY_AC)
  KFMI_FOR_NB(KFMI_OKC, 1, LAY_PACKED)
  KFMI_FOR_NB(KFMI_OKC, 2, LAY_PACKED)
  KFMI_FOR_NB(KFMI_OKC, 1, LAY_MID)
  KFMI_FOR_NB(KFMI_OKC, 2, LAY_MID)
  KFMI_FOR_NB(KFMI_OKC, 1, LAY_AC128)
  KFMI_FOR_NB(KFMI_OKC, 2, LAY_AC128)
#undef KFMI_OKC
  return false;
}

static hipError_t dispatch_build_packed(uint32_t K, uint32_t nb, const uint32_t* inter, uint32_t nentries,
                                        uint32_t* packed, uint32_t* sb, uint32_t* overflow, hipStream_t st)
{
  const uint32_t blocks = (nentries + 255) / 256;
#define KFMI_BP(KK, NBV, LAYV)                                                                  \
  if (K == KK && nb == NBV) {                                                                   \
    hipLaunchKernelGGL((build_packed_kernel<KK, NBV>), dim3(blocks), dim3(256), 0, st, inter, nentries, \
                       packed, sb, overflow);                                                   \
    return hipGetLastError();                                                                   \
  }
  KFMI_FOR_NB(KFMI_BP, 1, 0)
  KFMI_FOR_NB(KFMI_BP, 2, 0)
#undef KFMI_BP
  return hipErrorInvalidValue;
}

static hipError_t dispatch_build_mid(uint32_t K, uint32_t nb, const uint32_t* inter, uint32_t nentries,
                                     uint32_t nlines, uint32_t* lines, const uint32_t* ext_last,
                                     const uint32_t* ext_pad, hipStream_t st)
{
  const uint32_t blocks = (nlines + 255) / 256;
#define KFMI_BM(KK, NBV, LAYV)                                                                         \
  if (K == KK && nb == NBV) {                                                                          \
    hipLaunchKernelGGL((build_mid_kernel<KK, NBV>), dim3(blocks), dim3(256), 0, st, inter, nentries, nlines, \
                       lines, ext_last, ext_pad);                                                      \
    return hipGetLastError();                                                                          \
  }
  KFMI_FOR_NB(KFMI_BM, 1, 0)
  KFMI_FOR_NB(KFMI_BM, 2, 0)
#undef KFMI_BM
  return hipErrorInvalidValue;
}

static hipError_t dispatch_build_ac128(uint32_t K, uint32_t nb, const uint32_t* ac, uint32_t nent, uint32_t nlines,
                                       uint32_t* lines, hipStream_t st)
{
  const uint32_t blocks = (nlines + 255) / 256;
#define KFMI_BA(KK, NBV, LAYV)                                                                          \
  if (K == KK && nb == NBV) {                                                                           \
    hipLaunchKernelGGL((build_ac128_kernel<KK, NBV>), dim3(blocks), dim3(256), 0, st, ac, nent, nlines, lines); \
    return hipGetLastError();                                                                           \
  }
  KFMI_FOR_NB(KFMI_BA, 1, 0)
  KFMI_FOR_NB(KFMI_BA, 2, 0)
#undef KFMI_BA
  return hipErrorInvalidValue;
}

static int layout_of(int backend)
{
  switch (backend) {
    case KFMI_BK_TASK: case KFMI_BK_COOP: return LAY_INTER;
    case KFMI_BK_TASK_AC: case KFMI_BK_COOP_AC: return LAY_AC;
    case KFMI_BK_TASK_MID: case KFMI_BK_COOP_MID: return LAY_MID;
    case KFMI_BK_TASK_AC128: case KFMI_BK_COOP_AC128: return LAY_AC128;
    default: return LAY_PACKED;
  }
}

static bool is_coop(int backend)
{
  return backend == KFMI_BK_COOP || backend == KFMI_BK_COOP_AC || backend == KFMI_BK_COOP_PACKED ||
         backend == KFMI_BK_COOP_MID || backend == KFMI_BK_COOP_AC128;
}

/* ------------------------------------------------------------------------ */
/* host helpers for the device layouts                                      */
/* ------------------------------------------------------------------------ */

/* Counters at row n+1 (one past the last row) from a tag-100/101 index:
 * cnt_{E-1} + rows of each code in the last block, $ rows excluded.  Used for
 * the padding entry that keeps R/d == nentries in bounds when (n+1) % d == 0
 * (reference defect B5: it reads past the end there). */
static void end_counters(const kfmi_fmi_t* f, uint32_t* out)
{
  const uint32_t nc = 1u << (2 * f->steps), nb = f->nbitmaps;
  const uint32_t last = f->nentries - 1;
  const uint32_t* e = f->h_index + (uint64_t) last * f->entry_words;
  const uint32_t o = f->bwtsize - last * f->chunk;  /* rows of the last block, in (0, d] */
  for (uint32_t c = 0; c < nc; ++c) {
    uint32_t pop = 0;
    for (uint32_t w = 0; w < nb; ++w) {
      int sh = (int) o - 32 * (int) w;
      sh = sh < 0 ? 0 : (sh > 32 ? 32 : sh);
      uint32_t m = (uint32_t) (0xFFFFFFFF00000000ull >> sh);
      for (uint32_t s = 0; s < f->steps; ++s)
        for (uint32_t t = 0; t < 2; ++t) {
          uint32_t p = e[kfmi_plane_index(f->tag, f->steps, nb, s, t, w)];
          m &= ((c >> (2 * s + t)) & 1u) ? p : ~p;
        }
      pop += (uint32_t) __builtin_popcount(m);
    }
    for (uint32_t s = 0; s < f->steps; ++s)
      if (f->modposdollarBWT[s] == last && f->dollarBaseBWT[s] == c && f->bwtsize > f->dollarPositionBWT[s]) pop--;
    out[c] = e[2 * nb * f->steps + c] + pop;
  }
}

/* Host image of the entries for a layout, converting tags as needed.
 * INTER/PACKED need plain counters (tag 100/101); AC needs tag 201 (a
 * tag-100/101 input goes through the tfmiAC transform first). */
static int32_t host_entries_for(const kfmi_fmi_t* f, int lay, kfmi_fmi_t** owned, const kfmi_fmi_t** use)
{
  *owned = nullptr;
  *use = f;
  if (lay == LAY_INTER || lay == LAY_PACKED || lay == LAY_MID) {
    /* tag 101 as is; tag 100 is interleaved on the device (upload_entries) */
    if (f->tag == 101 || f->tag == 100) return KFMI_SUCCESS;
    return KFMI_INDEX_VER_INTERLEAVE;   /* an AC file cannot feed a plain-counter backend */
  }
  /* AC, AC128 */
  if (f->tag == 201) return KFMI_SUCCESS;
  kfmi_fmi_t* t100 = nullptr;
  const kfmi_fmi_t* src100 = f;
  if (f->tag == 101) {
    /* de-interleave to tag 100 first */
    int32_t e = kfmi_index_alloc(100, f->steps, f->bwtsize, f->nentries, f->chunk, f->dollarPositionBWT,
                                 f->dollarBaseBWT, &t100);
    if (e) return e;
    const uint32_t nb = f->nbitmaps, K = f->steps, nbw = 2 * nb * K;
    for (uint64_t i = 0; i < f->nentries; ++i) {
      const uint32_t* s = f->h_index + i * f->entry_words;
      uint32_t* d = t100->h_index + i * t100->entry_words;
      for (uint32_t w = 0; w < nb; ++w)
        for (uint32_t st = 0; st < K; ++st)
          for (uint32_t t = 0; t < 2; ++t)
            d[kfmi_plane_index(100, K, nb, st, t, w)] = s[kfmi_plane_index(101, K, nb, st, t, w)];
      for (uint32_t c = 0; c < f->ncounters; ++c) d[nbw + c] = s[nbw + c];
    }
    src100 = t100;
  } else if (f->tag == 200) {
    /* permute the bit planes of every entry into tag-201 order */
    int32_t e = kfmi_index_alloc(201, f->steps, f->bwtsize, f->nentries, f->chunk, f->dollarPositionBWT,
                                 f->dollarBaseBWT, owned);
    if (e) return e;
    const uint32_t nb = f->nbitmaps, K = f->steps, half = f->ncounters;
    for (uint64_t i = 0; i < f->nentries; ++i) {
      const uint32_t* s = f->h_index + i * f->entry_words;
      uint32_t* d = (*owned)->h_index + i * (*owned)->entry_words;
      for (uint32_t c = 0; c < half; ++c) d[c] = s[c];
      for (uint32_t w = 0; w < nb; ++w)
        for (uint32_t st = 0; st < K; ++st)
          for (uint32_t t = 0; t < 2; ++t)
            d[half + kfmi_plane_index(201, K, nb, st, t, w)] = s[half + kfmi_plane_index(200, K, nb, st, t, w)];
    }
    *use = *owned;
    return KFMI_SUCCESS;
  }
  int32_t e = kfmi_transform_ac((void*) src100, nullptr, (void**) owned);
  if (t100) freeIndex((void**) &t100);
  if (e) return e;
  *use = *owned;
  return KFMI_SUCCESS;
}

static void free_dev_index(kfmi_dev_index* di)
{
  if (!di) return;
  if (di->device >= 0) (void) hipSetDevice(di->device);
  if (di->ent) (void) hipFree(di->ent);
  if (di->sb) (void) hipFree(di->sb);
  if (di->sa) (void) hipFree(di->sa);
  if (di->ftab) (void) hipFree(di->ftab);
  delete di;
}

namespace {
bool host_pinned(const void* p);
void par_copy(void* dst, const void* src, uint64_t bytes);
}  // namespace

/* Large host-to-device copy.  hipMemcpy from pageable memory runs at a few
 * GB/s; above 256 MB the source is staged through two pinned 64 MB buffers
 * (filled by the host workers) so that the copy runs at PCIe speed.  Returns
 * with the copy complete when staged, else queued on `st`. */
static hipError_t h2d(void* dst, const void* src, uint64_t bytes, hipStream_t st)
{
  constexpr uint64_t CH = 64ull << 20;
  if (bytes < (256ull << 20) || host_pinned(src)) return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st);
  void* buf[2] = {nullptr, nullptr};
  hipEvent_t ev[2] = {nullptr, nullptr};
  hipError_t e = hipSuccess;
  for (int b = 0; b < 2 && e == hipSuccess; ++b) {
    e = hipHostMalloc(&buf[b], CH, hipHostMallocDefault);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ev[b], hipEventDisableTiming);
  }
  for (uint64_t off = 0, i = 0; off < bytes && e == hipSuccess; off += CH, ++i) {
    const int b = (int) (i & 1);
    if (i >= 2) e = hipEventSynchronize(ev[b]);
    if (e != hipSuccess) break;
    const uint64_t len = bytes - off < CH ? bytes - off : CH;
    par_copy(buf[b], (const uint8_t*) src + off, len);
    e = hipMemcpyAsync((uint8_t*) dst + off, buf[b], len, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipEventRecord(ev[b], st);
  }
  const hipError_t es = hipStreamSynchronize(st);
  for (int b = 0; b < 2; ++b) {
    if (ev[b]) (void) hipEventDestroy(ev[b]);
    if (buf[b]) (void) hipHostFree(buf[b]);
  }
  return e != hipSuccess ? e : es;
}

/* tag-100 -> tag-101 entries (kfmi_transform_interleave's plane order,
 * transformIndexBitmaps.c) on the device: out word p of an entry is in word
 * perm[p] of the same entry. */
constexpr uint32_t KFMI_MAX_ENTRY_WORDS = 160;   /* K <= 2, d <= 960: 2*30*2 + 16 = 136 */
struct EntryPerm {
  uint32_t p[KFMI_MAX_ENTRY_WORDS];
};

__global__ __launch_bounds__(256) void interleave_entries_kernel(const uint32_t* __restrict__ in,
                                                                 uint32_t* __restrict__ out, uint64_t words,
                                                                 uint32_t ew, EntryPerm perm)
{
  for (uint64_t i = (uint64_t) blockIdx.x * 256 + threadIdx.x; i < words; i += (uint64_t) gridDim.x * 256) {
    const uint64_t e = i / ew;
    out[i] = in[e * ew + perm.p[i - e * ew]];
  }
}

/* The entries of `src` as tag 101 (plain family) or as stored, into device
 * memory at dst (`body` bytes). */
static hipError_t upload_entries(void* dst, const kfmi_fmi_t* src, uint64_t body, hipStream_t st)
{
  if (src->tag != 100) return h2d(dst, src->h_index, body, st);
  const uint32_t ew = src->entry_words, K = src->steps, nb = src->nbitmaps;
  if (ew > KFMI_MAX_ENTRY_WORDS) return hipErrorInvalidValue;
  EntryPerm perm;
  for (uint32_t p = 0; p < ew; ++p) perm.p[p] = p;   /* counters keep their place */
  for (uint32_t w = 0; w < nb; ++w)
    for (uint32_t k = 0; k < K; ++k)
      for (uint32_t t = 0; t < 2; ++t) perm.p[kfmi_plane_index(101, K, nb, k, t, w)] = kfmi_plane_index(100, K, nb, k, t, w);
  uint32_t* tmp = nullptr;
  hipError_t e = hipMalloc((void**) &tmp, body ? body : 4);
  if (e != hipSuccess) return e;
  e = h2d(tmp, src->h_index, body, st);
  const uint64_t words = body / 4, blocks = (words + 255) / 256;
  if (e == hipSuccess && words) {
    hipLaunchKernelGGL(interleave_entries_kernel, dim3((uint32_t) (blocks < (1u << 20) ? blocks : (1u << 20))),
                       dim3(256), 0, st, tmp, (uint32_t*) dst, words, ew, perm);
    e = hipGetLastError();
  }
  const hipError_t es = hipStreamSynchronize(st);
  (void) hipFree(tmp);
  return e != hipSuccess ? e : es;
}

/* Device copy of the index's SA samples (locate); none when it has none. */
static int32_t upload_sa(const kfmi_fmi_t* f, kfmi_dev_index* di, DevCtx* ctx)
{
  if (di->sa) (void) hipFree(di->sa);
  di->sa = nullptr;
  di->sa_bytes = 0;
  di->sa_gen = f->sa_gen;
  if (!f->h_sa || !f->sa_rate) return KFMI_SUCCESS;
  const uint64_t bytes = 4ull * f->sa_count;
  if (hipMalloc((void**) &di->sa, bytes + 4) != hipSuccess) {
    di->sa = nullptr;
    return KFMI_E_DEVICE_ALLOC;
  }
  if (h2d(di->sa, f->h_sa, bytes, ctx->st) != hipSuccess ||
      hipStreamSynchronize(ctx->st) != hipSuccess) {
    (void) hipFree(di->sa);
    di->sa = nullptr;
    return KFMI_E_KERNEL;
  }
  di->sa_bytes = bytes;
  di->sa_log2 = (uint32_t) __builtin_ctz(f->sa_rate);
  return KFMI_SUCCESS;
}

/* Uploads f for `backend` to `dev`: into f->dev, or into *out (group replicas). */
static int32_t upload_index(kfmi_fmi_t* f, int backend, int dev, DevCtx* ctx, kfmi_dev_index** out = nullptr)
{
  if (f->steps < 1 || f->steps > 2) return KFMI_E_BAD_ARGUMENT;   /* GPU kernels: K in {1,2} */
  if (!nb_supported(f->nbitmaps)) return KFMI_E_BAD_ARGUMENT;
  const int lay = layout_of(backend);
  if (!geometry_supported(backend, f->steps, f->nbitmaps, lay)) return KFMI_E_BAD_ARGUMENT;
  kfmi_fmi_t* owned = nullptr;
  const kfmi_fmi_t* src = nullptr;
  int32_t err = host_entries_for(f, lay, &owned, &src);
  if (err) return err;

  kfmi_dev_index* di = new (std::nothrow) kfmi_dev_index();   /* no C++ exception crosses the C ABI */
  if (!di) {
    if (owned) freeIndex((void**) &owned);
    return KFMI_E_ALLOCATING_FMI;
  }
  di->device = dev;
  di->backend = backend;
  di->layout = lay;
  di->K = f->steps;
  di->d = f->chunk;
  di->nb = f->nbitmaps;
  di->bwtsize = f->bwtsize;
  di->nentries = src->nentries;
  for (uint32_t s = 0; s < 2; ++s) {
    di->dl.dpos[s] = s < f->steps ? f->dollarPositionBWT[s] : 0xFFFFFFFFu;
    di->dl.dbase[s] = s < f->steps ? f->dollarBaseBWT[s] : 0xFFFFFFFFu;
    di->dl.dblk[s] = s < f->steps ? f->dollarPositionBWT[s] / f->chunk : 0xFFFFFFFFu;
  }
  const uint64_t ew = src->entry_words;
  const uint64_t body = 4ull * ew * src->nentries;
  const uint32_t nc = 1u << (2 * f->steps);
  std::vector<uint32_t> pad(ew * 2, 0);

  auto fail = [&](int32_t code) {
    if (owned) freeIndex((void**) &owned);
    free_dev_index(di);
    return code;
  };

  if (lay == LAY_INTER || lay == LAY_AC) {
    /* entries + 2 padding entries (B5 guard; AC may look at b+1 of the sentinel) */
    di->ent_bytes = body + 4ull * ew * 2;
    if (hipMalloc((void**) &di->ent, di->ent_bytes) != hipSuccess) return fail(KFMI_E_DEVICE_ALLOC);
    if (lay == LAY_INTER) end_counters(src, pad.data() + 2 * f->nbitmaps * f->steps);
    if (upload_entries(di->ent, src, body, ctx->st) != hipSuccess ||
        hipMemcpyAsync((uint8_t*) di->ent + body, pad.data(), 4ull * ew * 2, hipMemcpyHostToDevice, ctx->st) !=
            hipSuccess ||
        hipStreamSynchronize(ctx->st) != hipSuccess)
      return fail(KFMI_E_KERNEL);
  } else if (lay == LAY_AC128) {
    /* one line per tag-201 entry (sentinel included) + one padding line, built on
     * the device from the entries; padding entry b+1 of the sentinel reads 0 */
    const uint32_t E = src->nentries;                 /* tag-201 entries incl. the sentinel */
    const uint32_t nl = E + 1;
    const uint32_t lw = (uint32_t) pow2ceil((int) (2 * f->nbitmaps * f->steps + nc));
    uint32_t* tmp = nullptr;
    di->ent_bytes = 4ull * lw * nl;
    if (hipMalloc((void**) &tmp, body + 16) != hipSuccess) return fail(KFMI_E_DEVICE_ALLOC);
    if (hipMalloc((void**) &di->ent, di->ent_bytes) != hipSuccess) {
      (void) hipFree(tmp);
      return fail(KFMI_E_DEVICE_ALLOC);
    }
    bool ok = upload_entries(tmp, src, body, ctx->st) == hipSuccess &&
              dispatch_build_ac128(f->steps, f->nbitmaps, tmp, E, nl, di->ent, ctx->st) == hipSuccess &&
              hipStreamSynchronize(ctx->st) == hipSuccess;
    (void) hipFree(tmp);
    if (!ok) return fail(KFMI_E_KERNEL);
  } else if (lay == LAY_MID) {
    /* MID: pairs of blocks per line, built on the device from tag-101 entries;
     * counters of the last line (odd block count) and of one padding line are
     * "rows past n+1 read as A" extensions of the end counters. */
    const uint32_t E = src->nentries;
    const uint32_t nreal = (E + 1) / 2;
    const uint32_t nl = nreal + 1;
    const uint32_t lw = (uint32_t) pow2ceil((int) (2 * 2 * f->nbitmaps * f->steps + nc));
    std::vector<uint32_t> endc(nc), ext(2 * nc);
    end_counters(src, endc.data());
    const uint64_t n1 = f->bwtsize;                                   /* n + 1 */
    const uint64_t mid_last = (uint64_t) E * f->chunk;               /* midpoint of line nreal-1 when E is odd */
    const uint64_t mid_pad = (uint64_t) nreal * 2 * f->chunk + f->chunk;
    for (uint32_t c = 0; c < nc; ++c) {
      ext[c] = endc[c] + (c == 0 ? (uint32_t) (mid_last - n1) : 0u);
      ext[nc + c] = endc[c] + (c == 0 ? (uint32_t) (mid_pad - n1) : 0u);
    }
    uint32_t *tmp = nullptr, *d_ext = nullptr;
    di->ent_bytes = 4ull * lw * nl;
    if (hipMalloc((void**) &tmp, body + 16) != hipSuccess) return fail(KFMI_E_DEVICE_ALLOC);
    if (hipMalloc((void**) &di->ent, di->ent_bytes) != hipSuccess ||
        hipMalloc((void**) &d_ext, 8ull * nc) != hipSuccess) {
      (void) hipFree(tmp);
      if (d_ext) (void) hipFree(d_ext);
      return fail(KFMI_E_DEVICE_ALLOC);
    }
    bool ok = upload_entries(tmp, src, body, ctx->st) == hipSuccess &&
              hipMemcpyAsync(d_ext, ext.data(), 8ull * nc, hipMemcpyHostToDevice, ctx->st) == hipSuccess &&
              dispatch_build_mid(f->steps, f->nbitmaps, tmp, E, nl, di->ent, d_ext, d_ext + nc, ctx->st) ==
                  hipSuccess &&
              hipStreamSynchronize(ctx->st) == hipSuccess;
    (void) hipFree(tmp);
    (void) hipFree(d_ext);
    if (!ok) return fail(KFMI_E_KERNEL);
  } else {
    /* packed: build on the device from tag-101 entries (+ the padding entry) */
    const uint32_t ne = src->nentries + 1;
    uint32_t* tmp = nullptr;
    uint32_t* d_over = nullptr;
    const uint32_t pw = (uint32_t) pow2ceil((int) (2 * f->nbitmaps * f->steps + nc / 2));
    const int S = sb_shift_for((int) f->chunk);
    const uint64_t nsb = ((uint64_t) ne + (1u << S) - 1) >> S;
    end_counters(src, pad.data() + 2 * f->nbitmaps * f->steps);
    di->ent_bytes = 4ull * pw * (ne + 1);
    di->sb_bytes = 4ull * nc * nsb;
    if (hipMalloc((void**) &tmp, 4ull * ew * ne) != hipSuccess) return fail(KFMI_E_DEVICE_ALLOC);
    if (hipMalloc((void**) &di->ent, di->ent_bytes) != hipSuccess ||
        hipMalloc((void**) &di->sb, di->sb_bytes) != hipSuccess || hipMalloc((void**) &d_over, 4) != hipSuccess) {
      (void) hipFree(tmp);
      if (d_over) (void) hipFree(d_over);
      return fail(KFMI_E_DEVICE_ALLOC);
    }
    uint32_t over = 0;
    bool ok = upload_entries(tmp, src, body, ctx->st) == hipSuccess &&
              hipMemcpyAsync((uint8_t*) tmp + body, pad.data(), 4ull * ew, hipMemcpyHostToDevice, ctx->st) ==
                  hipSuccess &&
              hipMemsetAsync(d_over, 0, 4, ctx->st) == hipSuccess &&
              hipMemsetAsync(di->ent, 0, di->ent_bytes, ctx->st) == hipSuccess &&
              dispatch_build_packed(f->steps, f->nbitmaps, tmp, ne, di->ent, di->sb, d_over, ctx->st) ==
                  hipSuccess &&
              hipMemcpyAsync(&over, d_over, 4, hipMemcpyDeviceToHost, ctx->st) == hipSuccess &&
              hipStreamSynchronize(ctx->st) == hipSuccess;
    (void) hipFree(tmp);
    (void) hipFree(d_over);
    if (!ok) return fail(KFMI_E_KERNEL);
    if (over) {
      fprintf(stderr, "kstepfmi: packed layout delta overflow (%u) -- corrupt counters\n", over);
      return fail(KFMI_E_READING_FMI);
    }
  }
  if (owned) freeIndex((void**) &owned);
  if (f->h_sa) {
    err = upload_sa(f, di, ctx);
    if (err) {
      free_dev_index(di);
      return err;
    }
  }
  if (out) {
    *out = di;
    return KFMI_SUCCESS;
  }
  if (f->dev) free_dev_index(f->dev);
  f->dev = di;
  return KFMI_SUCCESS;
}

static IdxArgs idx_args(const kfmi_dev_index* di)
{
  IdxArgs ix;
  ix.ent = di->ent;
  ix.sb = di->sb;
  ix.bwtsize = di->bwtsize;
  const char* e = getenv("KFMI_NT_FROM");   /* K-step from which index loads are non-temporal */
  ix.nt_from = e ? (uint32_t) atoi(e) : 0xFFFFFFFFu;
  ix.dl = di->dl;
  ix.ftab = nullptr;
  ix.ftab_steps = 0;
  ix.ftab_mask = 0;
  return ix;
}

/* The ftab of `bases` bases, (re)built on the device from the uploaded layout
 * with the search's own LF steps; sets ix.ftab (null when off or when bases is
 * not a multiple of K). */
static int32_t use_ftab(kfmi_dev_index* di, hipStream_t st, IdxArgs& ix, uint32_t bases)
{
  ix.ftab = nullptr;
  ix.ftab_steps = 0;
  ix.ftab_mask = 0;
  if (!bases || bases % di->K) return KFMI_SUCCESS;
  if (di->ftab_chars != bases) {
    if (di->ftab) (void) hipFree(di->ftab);
    di->ftab = nullptr;
    di->ftab_chars = 0;
    const uint64_t n = 1ull << (2 * bases);
    if (hipMalloc((void**) &di->ftab, 8 * n) != hipSuccess) {
      di->ftab = nullptr;
      return KFMI_E_DEVICE_ALLOC;
    }
    SearchLaunch a{};
    a.st = st;
    a.ix = idx_args(di);
    a.ftab_out = di->ftab;
    a.ftab_steps = bases / di->K;
    a.ftab_n = n;
    if (dispatch(Op::Ftab, di->K, di->nb, di->layout, a) != hipSuccess || hipStreamSynchronize(st) != hipSuccess)
      return KFMI_E_KERNEL;
    di->ftab_chars = bases;
  }
  ix.ftab = di->ftab;
  ix.ftab_steps = bases / di->K;
  ix.ftab_mask = bases >= 16 ? 0xFFFFFFFFu : (1u << (2 * bases)) - 1u;
  return KFMI_SUCCESS;
}

static void free_dev_queries(kfmi_dev_queries* dq)
{
  if (!dq) return;
  if (dq->device >= 0) (void) hipSetDevice(dq->device);
  if (dq->ascii) (void) hipFree(dq->ascii);
  if (dq->packed) (void) hipFree(dq->packed);
  delete dq;
}

static int32_t upload_queries(kfmi_qrys_t* q, uint32_t K, int dev, DevCtx* ctx)
{
  if (q->size == 0 || (q->size % K) != 0) return KFMI_E_BAD_ARGUMENT;   /* B6 */
  if (64ull * q->size > 160ull * 1024) return KFMI_E_BAD_ARGUMENT;       /* pack tile must fit LDS */
  kfmi_dev_queries* dq = new (std::nothrow) kfmi_dev_queries();
  if (!dq) return KFMI_E_ALLOCATING_MFASTA;
  dq->device = dev;
  dq->num = q->num;
  dq->size = q->size;
  dq->K = K;
  dq->steps = q->size / K;
  const uint32_t spw = 32 / (2 * K);
  dq->nwords = (dq->steps + spw - 1) / spw;
  const uint64_t abytes = q->num * (uint64_t) q->size;
  if (hipMalloc((void**) &dq->ascii, abytes + 16) != hipSuccess ||
      hipMalloc((void**) &dq->packed, 4ull * dq->nwords * (q->num ? q->num : 1)) != hipSuccess) {
    free_dev_queries(dq);
    return KFMI_E_DEVICE_ALLOC;
  }
  if (abytes && (h2d(dq->ascii, q->h_queries, abytes, ctx->st) != hipSuccess ||
                 hipStreamSynchronize(ctx->st) != hipSuccess)) {
    free_dev_queries(dq);
    return KFMI_E_KERNEL;
  }
  if (q->dev) free_dev_queries(q->dev);
  q->dev = dq;
  return KFMI_SUCCESS;
}

static hipError_t launch_pack(const kfmi_dev_queries* dq, hipStream_t st)
{
  if (dq->num == 0) return hipSuccess;
  uint32_t tq = 256;
  while ((uint64_t) tq * dq->size > 64 * 1024 && tq > 64) tq >>= 1;
  const uint64_t blocks = (dq->num + tq - 1) / tq;
  const size_t lds = (size_t) tq * dq->size + 16;
  if (dq->K == 1)
    hipLaunchKernelGGL((pack_queries_kernel<1>), dim3((uint32_t) blocks), dim3(256), lds, st, dq->ascii, dq->num,
                       dq->size, dq->steps, dq->nwords, tq, dq->packed);
  else
    hipLaunchKernelGGL((pack_queries_kernel<2>), dim3((uint32_t) blocks), dim3(256), lds, st, dq->ascii, dq->num,
                       dq->size, dq->steps, dq->nwords, tq, dq->packed);
  return hipGetLastError();
}

/* ------------------------------------------------------------------------ */
/* device groups (SURVEY 8(b) device selection, 8(e) partitioning).  The     */
/* reference fixes one GPU at compile time (-DDEVICE); KFMI_DEVICES=0,1,...  */
/* or kfmi_set_devices spreads the same handles over several: the index      */
/* replicated on every device, the queries cut into contiguous slices        */
/* (multiples of 64 reads), each device searching its slice on its own       */
/* stream, results copied back into disjoint slices of h_results.  No        */
/* exchange between devices on the data path.                               */
/* ------------------------------------------------------------------------ */

constexpr int KFMI_MAX_GROUP = 16;
static thread_local int t_ngroup = -1;   /* -1: read KFMI_DEVICES */
static thread_local int t_group[KFMI_MAX_GROUP];

/* The device list (0 or 1 entry: single-device mode). */
static int group_devices(int* devs)
{
  if (t_ngroup < 0) {
    t_ngroup = 0;
    const char* p = getenv("KFMI_DEVICES");
    while (p && *p && t_ngroup < KFMI_MAX_GROUP) {
      char* end = nullptr;
      const long v = strtol(p, &end, 10);
      if (end == p) break;
      t_group[t_ngroup++] = (int) v;
      p = end;
      while (*p == ',' || *p == ' ') ++p;
    }
  }
  for (int i = 0; i < t_ngroup; ++i) devs[i] = t_group[i];
  return t_ngroup;
}

struct GroupIndex {
  int n = 0, backend = -1;
  int dev[KFMI_MAX_GROUP] = {};
  kfmi_dev_index* di[KFMI_MAX_GROUP] = {};
  hipStream_t st[KFMI_MAX_GROUP] = {};
  hipEvent_t ev[KFMI_MAX_GROUP][3] = {};
};

/* queries or results of a group: one contiguous slice per member */
struct GroupSlices {
  int n = 0;
  int dev[KFMI_MAX_GROUP] = {};
  uint64_t q0[KFMI_MAX_GROUP] = {}, num[KFMI_MAX_GROUP] = {};
  kfmi_dev_queries* dq[KFMI_MAX_GROUP] = {};
  uint32_t* d_res[KFMI_MAX_GROUP] = {};
};

static GroupSlices* group_slices(uint64_t num, const int* devs, int n)
{
  GroupSlices* g = new (std::nothrow) GroupSlices();
  if (!g) return nullptr;
  g->n = n;
  uint64_t per = (num + n - 1) / n;
  per = (per + 63) & ~63ull;
  for (int i = 0; i < n; ++i) {
    g->dev[i] = devs[i];
    const uint64_t a = per * i < num ? per * i : num, b = per * (i + 1) < num ? per * (i + 1) : num;
    g->q0[i] = a;
    g->num[i] = b - a;
  }
  return g;
}

static void group_free_index(kfmi_fmi_t* f)
{
  GroupIndex* g = (GroupIndex*) f->grp;
  if (!g) return;
  for (int i = 0; i < g->n; ++i) {
    (void) hipSetDevice(g->dev[i]);
    if (g->st[i]) (void) hipStreamSynchronize(g->st[i]);
    free_dev_index(g->di[i]);
    for (int k = 0; k < 3; ++k)
      if (g->ev[i][k]) (void) hipEventDestroy(g->ev[i][k]);
    if (g->st[i]) (void) hipStreamDestroy(g->st[i]);
  }
  delete g;
  f->grp = nullptr;
}

static void free_dev_queries(kfmi_dev_queries* dq);

static void group_free_queries(kfmi_qrys_t* q)
{
  GroupSlices* g = (GroupSlices*) q->grp;
  if (!g) return;
  for (int i = 0; i < g->n; ++i) free_dev_queries(g->dq[i]);
  delete g;
  q->grp = nullptr;
}

static void group_free_results(kfmi_res_t* r)
{
  GroupSlices* g = (GroupSlices*) r->grp;
  if (!g) return;
  for (int i = 0; i < g->n; ++i)
    if (g->d_res[i]) {
      (void) hipSetDevice(g->dev[i]);
      (void) hipFree(g->d_res[i]);
    }
  delete g;
  r->grp = nullptr;
}

static int32_t upload_queries(kfmi_qrys_t* q, uint32_t K, int dev, DevCtx* ctx);

static int32_t group_transfer(kfmi_fmi_t* f, kfmi_qrys_t* q, kfmi_res_t* r, const int* devs, int n)
{
  const int backend = kfmi_backend();
  int32_t err = KFMI_SUCCESS;
  if (f) {
    GroupIndex* g = (GroupIndex*) f->grp;
    bool same = g && g->backend == backend && g->n == n;
    for (int i = 0; same && i < n; ++i) same = g->dev[i] == devs[i];
    if (!same) {
      group_free_index(f);
      g = new (std::nothrow) GroupIndex();
      if (!g) return KFMI_E_ALLOCATING_FMI;
      g->n = n;
      g->backend = backend;
      f->grp = g;
      for (int i = 0; i < n && !err; ++i) {
        g->dev[i] = devs[i];
        DevCtx* ctx = nullptr;
        err = ctx_for(devs[i], &ctx);
        if (!err) err = upload_index(f, backend, devs[i], ctx, &g->di[i]);
        if (!err && hipStreamCreateWithFlags(&g->st[i], hipStreamNonBlocking) != hipSuccess) err = KFMI_E_NO_DEVICE;
        for (int k = 0; k < 3 && !err; ++k)
          if (hipEventCreate(&g->ev[i][k]) != hipSuccess) err = KFMI_E_NO_DEVICE;
      }
      if (err) {
        group_free_index(f);
        return err;
      }
    }
    if (f->dev) {   /* one mode per handle: the single-device copy goes */
      free_dev_index(f->dev);
      f->dev = nullptr;
    }
  }
  if (q) {
    if (!f) return KFMI_E_BAD_ARGUMENT;
    group_free_queries(q);
    if (q->dev) {
      free_dev_queries(q->dev);
      q->dev = nullptr;
    }
    GroupSlices* g = group_slices(q->num, devs, n);
    if (!g) return KFMI_E_ALLOCATING_MFASTA;
    q->grp = g;
    for (int i = 0; i < n && !err; ++i) {
      DevCtx* ctx = nullptr;
      err = ctx_for(devs[i], &ctx);
      kfmi_qrys_t sh{};
      sh.num = g->num[i];
      sh.size = q->size;
      sh.h_queries = q->h_queries + g->q0[i] * q->size;
      if (!err) err = upload_queries(&sh, f->steps, devs[i], ctx);
      g->dq[i] = sh.dev;
    }
    if (err) {
      group_free_queries(q);
      return err;
    }
  }
  if (r) {
    group_free_results(r);
    if (r->d_results) {
      (void) hipFree(r->d_results);
      r->d_results = nullptr;
    }
    GroupSlices* g = group_slices(r->num, devs, n);
    if (!g) return KFMI_E_ALLOCATING_RESULTS;
    r->grp = g;
    for (int i = 0; i < n && !err; ++i) {
      DevCtx* ctx = nullptr;
      err = ctx_for(devs[i], &ctx);
      if (!err && hipMalloc((void**) &g->d_res[i], 8ull * (g->num[i] ? g->num[i] : 1)) != hipSuccess) {
        g->d_res[i] = nullptr;
        err = KFMI_E_DEVICE_ALLOC;
      }
      if (!err && (hipMemsetAsync(g->d_res[i], 0, 8ull * g->num[i], ctx->st) != hipSuccess ||
                   hipStreamSynchronize(ctx->st) != hipSuccess))
        err = KFMI_E_KERNEL;
    }
    if (err) {
      group_free_results(r);
      return err;
    }
  }
  return KFMI_SUCCESS;
}

static int32_t search_enqueue(kfmi_dev_index* di, kfmi_dev_queries* dq, uint32_t* d_res, hipStream_t st,
                              hipEvent_t* ev, uint32_t ftab);
static int32_t search_finish(hipStream_t st, hipEvent_t* ev, double* ms);

/* Every member queues its slice, then all are waited for; the timings are the
 * slowest member's. */
static int32_t group_search(kfmi_fmi_t* f, kfmi_qrys_t* q, kfmi_res_t* r)
{
  GroupIndex* gi = (GroupIndex*) f->grp;
  GroupSlices* gq = (GroupSlices*) q->grp;
  GroupSlices* gr = (GroupSlices*) r->grp;
  if (!gi || !gq || !gr) return KFMI_E_NOT_ON_DEVICE;   /* handles moved to different modes */
  if (gq->n != gi->n || gr->n != gi->n) return KFMI_E_BAD_ARGUMENT;
  for (int i = 0; i < gi->n; ++i)
    if (gq->dev[i] != gi->dev[i] || gr->dev[i] != gi->dev[i] || gq->num[i] != gr->num[i]) return KFMI_E_BAD_ARGUMENT;
  const uint32_t ftab = ftab_bases();
  int32_t err = KFMI_SUCCESS;
  int queued = 0;
  for (int i = 0; i < gi->n && !err; ++i) {
    if (hipSetDevice(gi->dev[i]) != hipSuccess) {
      err = KFMI_E_NO_DEVICE;
      break;
    }
    err = search_enqueue(gi->di[i], gq->dq[i], gr->d_res[i], gi->st[i], gi->ev[i], ftab);
    if (!err) ++queued;
  }
  double worst[3] = {0, 0, 0};
  for (int i = 0; i < queued; ++i) {
    (void) hipSetDevice(gi->dev[i]);
    double ms[3] = {0, 0, 0};
    const int32_t e = search_finish(gi->st[i], gi->ev[i], ms);
    if (e && !err) err = e;
    for (int k = 0; k < 3; ++k) worst[k] = ms[k] > worst[k] ? ms[k] : worst[k];
  }
  for (int k = 0; k < 3; ++k) t_ms[k] = worst[k];
  return err;
}

static int32_t group_to_host(kfmi_res_t* r)
{
  GroupSlices* g = (GroupSlices*) r->grp;
  for (int i = 0; i < g->n; ++i) {
    DevCtx* ctx = nullptr;
    int32_t err = ctx_for(g->dev[i], &ctx);
    if (err) return err;
    if (g->num[i])
      HIP_OK(hipMemcpyAsync(r->h_results + 2 * g->q0[i], g->d_res[i], 8ull * g->num[i], hipMemcpyDeviceToHost,
                            ctx->st));
  }
  for (int i = 0; i < g->n; ++i) {
    DevCtx* ctx = nullptr;
    int32_t err = ctx_for(g->dev[i], &ctx);
    if (err) return err;
    HIP_OK(hipStreamSynchronize(ctx->st));
  }
  return KFMI_SUCCESS;
}

extern "C" int32_t kfmi_set_devices(const int32_t* devices, int32_t n)
{
  if (n < 0 || n > KFMI_MAX_GROUP || (n && !devices)) return KFMI_E_BAD_ARGUMENT;
  const int avail = kfmi_device_count();
  for (int i = 0; i < n; ++i)
    if (devices[i] < 0 || devices[i] >= avail) return KFMI_E_NO_DEVICE;
  for (int i = 0; i < n; ++i) t_group[i] = devices[i];
  t_ngroup = n;
  if (n == 1) t_device = devices[0];
  return KFMI_SUCCESS;
}

extern "C" int32_t kfmi_get_devices(int32_t* devices, int32_t cap)
{
  int devs[KFMI_MAX_GROUP];
  const int n = group_devices(devs);
  for (int i = 0; i < n && i < cap && devices; ++i) devices[i] = devs[i];
  return n;
}

/* ------------------------------------------------------------------------ */
/* C ABI: the reference's GPU plugin entry points                           */
/* ------------------------------------------------------------------------ */

/* interface.h:40, e.g. fmIndexGPU-Coop-2Step.cu:250-285 (index, $ arrays,
 * queries and zeroed results to the device; the index is re-laid-out for the
 * selected backend). */
extern "C" int32_t transferCPUtoGPU(void* index, void* queries, void* results)
{
  kfmi_fmi_t* f = (kfmi_fmi_t*) index;
  kfmi_qrys_t* q = (kfmi_qrys_t*) queries;
  kfmi_res_t* r = (kfmi_res_t*) results;
  int devs[KFMI_MAX_GROUP];
  const int ng = group_devices(devs);
  if (ng > 1) return group_transfer(f, q, r, devs, ng);
  if (f) group_free_index(f);   /* one mode per handle */
  if (q) group_free_queries(q);
  if (r) group_free_results(r);
  const int dev = kfmi_current_device();
  DevCtx* ctx = nullptr;
  int32_t err = ctx_for(dev, &ctx);
  if (err) return err;
  const int backend = kfmi_backend();
  if (f && (!f->dev || f->dev->backend != backend || f->dev->device != dev)) {
    err = upload_index(f, backend, dev, ctx);
    if (err) return err;
  }
  if (q) {
    if (!f) return KFMI_E_BAD_ARGUMENT;
    err = upload_queries(q, f->steps, dev, ctx);
    if (err) return err;
  }
  if (r) {
    if (r->d_results) { (void) hipFree(r->d_results); r->d_results = nullptr; }
    if (hipMalloc((void**) &r->d_results, 8ull * (r->num ? r->num : 1)) != hipSuccess) return KFMI_E_DEVICE_ALLOC;
    if (hipMemsetAsync(r->d_results, 0, 8ull * r->num, ctx->st) != hipSuccess ||
        hipStreamSynchronize(ctx->st) != hipSuccess)
      return KFMI_E_KERNEL;
  }
  return KFMI_SUCCESS;
}

/* Queues pack (if not fused) + LF of one device batch on `st`, bracketed by
 * ev[0..2]; search_finish waits and reads the timings. */
static int32_t search_enqueue(kfmi_dev_index* di, kfmi_dev_queries* dq, uint32_t* d_res, hipStream_t st,
                              hipEvent_t* ev, uint32_t ftab)
{
  if (dq->device != di->device || dq->K != di->K) return KFMI_E_BAD_ARGUMENT;
  SearchLaunch a{};
  a.st = st;
  a.ix = idx_args(di);
  int32_t err = use_ftab(di, st, a.ix, ftab);
  if (err) return err;
  a.qp = dq->packed;
  a.ascii = dq->ascii;
  a.m = dq->size;
  a.maxw = fused_maxw(di->backend, dq->nwords);
  a.num = dq->num;
  a.steps = dq->steps;
  a.nwords = dq->nwords;
  a.res = d_res;
  HIP_OK(hipEventRecord(ev[0], st));
  if (!a.maxw) HIP_OK(launch_pack(dq, st));
  HIP_OK(hipEventRecord(ev[1], st));
  if (dq->num) {
    const Op op = is_coop(di->backend) ? Op::Coop : Op::Task;
    HIP_OK(dispatch(op, di->K, di->nb, di->layout, a));
  }
  HIP_OK(hipEventRecord(ev[2], st));
  return KFMI_SUCCESS;
}

static int32_t search_finish(hipStream_t st, hipEvent_t* ev, double* ms)
{
  HIP_OK(hipStreamSynchronize(st));
  float ms01 = 0, ms12 = 0;
  HIP_OK(hipEventElapsedTime(&ms01, ev[0], ev[1]));
  HIP_OK(hipEventElapsedTime(&ms12, ev[1], ev[2]));
  ms[0] = ms01 + ms12;
  ms[1] = ms01;
  ms[2] = ms12;
  return KFMI_SUCCESS;
}

static int32_t group_search(kfmi_fmi_t* f, kfmi_qrys_t* q, kfmi_res_t* r);

extern "C" int32_t kfmi_search(void* index, void* queries, void* results)
{
  kfmi_fmi_t* f = (kfmi_fmi_t*) index;
  kfmi_qrys_t* q = (kfmi_qrys_t*) queries;
  kfmi_res_t* r = (kfmi_res_t*) results;
  if (!f || !q || !r) return KFMI_E_BAD_ARGUMENT;
  if (q->num != r->num) return KFMI_E_BAD_ARGUMENT;
  if (f->grp || q->grp || r->grp) return group_search(f, q, r);
  if (!f->dev || !q->dev || !r->d_results) return KFMI_E_NOT_ON_DEVICE;
  kfmi_dev_index* di = f->dev;
  DevCtx* ctx = nullptr;
  int32_t err = ctx_for(di->device, &ctx);
  if (!err) err = search_enqueue(di, q->dev, r->d_results, ctx->st, ctx->ev, ftab_bases());
  if (!err) err = search_finish(ctx->st, ctx->ev, t_ms);
  return err;
}

/* interface.h:31: synchronous like the reference (cudaThreadSynchronize,
 * Task-2Step.cu:209) but its status is kept (kfmi_last_error) instead of
 * being dropped. */
extern "C" void searchIndexGPU(void* index, void* queries, void* resIntervals)
{
  int32_t e = kfmi_search(index, queries, resIntervals);
  t_last_error = e;
  if (e) fprintf(stderr, "kstepfmi: searchIndexGPU failed: %s\n", errorCommon(e));
}

extern "C" int32_t kfmi_count_blocks(void* index, void* queries, uint64_t* blocks)
{
  kfmi_fmi_t* f = (kfmi_fmi_t*) index;
  kfmi_qrys_t* q = (kfmi_qrys_t*) queries;
  if (!f || !q || !blocks) return KFMI_E_BAD_ARGUMENT;
  if (f->grp || q->grp) return KFMI_E_NOT_IMPLEMENTED;   /* single-device API */
  if (!f->dev || !q->dev) return KFMI_E_NOT_ON_DEVICE;
  kfmi_dev_index* di = f->dev;
  kfmi_dev_queries* dq = q->dev;
  DevCtx* ctx = nullptr;
  int32_t err = ctx_for(di->device, &ctx);
  if (err) return err;
  unsigned long long* d_total = nullptr;
  HIP_OK(hipMalloc((void**) &d_total, sizeof(unsigned long long)));
  SearchLaunch a;
  a.st = ctx->st;
  a.ix = idx_args(di);
  a.qp = dq->packed;
  a.ascii = dq->ascii;
  a.m = dq->size;
  a.maxw = 0;
  a.num = dq->num;
  a.steps = dq->steps;
  a.nwords = dq->nwords;
  a.res = nullptr;
  unsigned long long total = 0;
  bool ok = hipMemsetAsync(d_total, 0, sizeof(total), ctx->st) == hipSuccess &&
            launch_pack(dq, ctx->st) == hipSuccess &&
            (dq->num == 0 || dispatch(Op::Count, di->K, di->nb, di->layout, a, d_total) == hipSuccess) &&
            hipMemcpyAsync(&total, d_total, sizeof(total), hipMemcpyDeviceToHost, ctx->st) == hipSuccess &&
            hipStreamSynchronize(ctx->st) == hipSuccess;
  (void) hipFree(d_total);
  if (!ok) return KFMI_E_KERNEL;
  *blocks = total;
  return KFMI_SUCCESS;
}

/* interface.h:39, Coop-2Step.cu:287-293 */
extern "C" int32_t transferGPUtoCPU(void* results)
{
  kfmi_res_t* r = (kfmi_res_t*) results;
  if (r && r->grp) return group_to_host(r);
  if (!r || !r->d_results) return KFMI_E_NOT_ON_DEVICE;
  DevCtx* ctx = nullptr;
  int32_t err = ctx_for(kfmi_current_device(), &ctx);
  if (err) return err;
  HIP_OK(hipMemcpyAsync(r->h_results, r->d_results, 8ull * r->num, hipMemcpyDeviceToHost, ctx->st));
  HIP_OK(hipStreamSynchronize(ctx->st));
  return KFMI_SUCCESS;
}

/* interface.h:38, Task-1Step.cu:236-256: releases and NULLs the device copy */
extern "C" int32_t freeIndexGPU(void** index)
{
  kfmi_fmi_t* f = index ? (kfmi_fmi_t*) *index : nullptr;
  if (f) group_free_index(f);
  if (f && f->dev) {
    free_dev_index(f->dev);
    f->dev = nullptr;
  }
  return KFMI_SUCCESS;
}

extern "C" int32_t freeQueriesGPU(void** queries)
{
  kfmi_qrys_t* q = queries ? (kfmi_qrys_t*) *queries : nullptr;
  if (q) group_free_queries(q);
  if (q && q->dev) {
    free_dev_queries(q->dev);
    q->dev = nullptr;
  }
  return KFMI_SUCCESS;
}

extern "C" int32_t freeResultsGPU(void** results)
{
  kfmi_res_t* r = results ? (kfmi_res_t*) *results : nullptr;
  if (r) group_free_results(r);
  if (r && r->d_results) {
    (void) hipFree(r->d_results);
    r->d_results = nullptr;
  }
  return KFMI_SUCCESS;
}

extern "C" uint64_t kfmi_device_index_bytes(void* index)
{
  kfmi_fmi_t* f = (kfmi_fmi_t*) index;
  if (f && f->grp) {   /* all replicas of a device group */
    const GroupIndex* g = (const GroupIndex*) f->grp;
    uint64_t b = 0;
    for (int i = 0; i < g->n; ++i) b += g->di[i]->ent_bytes + g->di[i]->sb_bytes + g->di[i]->sa_bytes;
    return b;
  }
  if (!f || !f->dev) return 0;
  return f->dev->ent_bytes + f->dev->sb_bytes + f->dev->sa_bytes;
}

/* ------------------------------------------------------------------------ */
/* locate: [L, R) of every query -> text positions          */
/* ------------------------------------------------------------------------ */

struct kfmi_locations {
  uint64_t num = 0, total = 0;
  uint64_t* h_off = nullptr;   /* num + 1 */
  uint32_t* h_pos = nullptr;   /* total */
};

extern "C" int32_t kfmi_locations_free(void** locations)
{
  kfmi_locations* L = locations ? (kfmi_locations*) *locations : nullptr;
  if (L) {
    free(L->h_off);
    free(L->h_pos);
    delete L;
    *locations = nullptr;
  }
  return KFMI_SUCCESS;
}

extern "C" uint64_t kfmi_locations_total(void* locations)
{
  return locations ? ((kfmi_locations*) locations)->total : 0;
}

extern "C" const uint64_t* kfmi_locations_offsets(void* locations)
{
  return locations ? ((kfmi_locations*) locations)->h_off : nullptr;
}

extern "C" const uint32_t* kfmi_locations_positions(void* locations)
{
  return locations ? ((kfmi_locations*) locations)->h_pos : nullptr;
}

/* Locate of the `num` results at d_res (device of di) into *locations. */
static int32_t locate_on(kfmi_fmi_t* f, kfmi_dev_index* di, uint32_t* d_res, uint64_t num, uint32_t max_occ,
                         kfmi_locations** locations)
{
  DevCtx* ctx = nullptr;
  int32_t err = ctx_for(di->device, &ctx);
  if (err) return err;
  if (!di->sa || di->sa_gen != f->sa_gen) {
    err = upload_sa(f, di, ctx);
    if (err) return err;
  }
  kfmi_locations* L = new (std::nothrow) kfmi_locations();
  if (!L) return KFMI_E_ALLOCATING_RESULTS;
  L->num = num;
  L->h_off = (uint64_t*) malloc(8 * (num + 1));
  if (!L->h_off) {
    kfmi_locations_free((void**) &L);
    return KFMI_E_ALLOCATING_RESULTS;
  }
  uint64_t *d_cnt = nullptr, *d_off = nullptr;
  uint32_t *d_pos = nullptr, *d_own = nullptr;
  void *tmp = nullptr, *tmp2 = nullptr;
  size_t tb = 0, tb2 = 0;
  uint64_t total = 0;
  auto done = [&](int32_t code) {
    if (d_cnt) (void) hipFree(d_cnt);
    if (d_off) (void) hipFree(d_off);
    if (d_pos) (void) hipFree(d_pos);
    if (d_own) (void) hipFree(d_own);
    if (tmp) (void) hipFree(tmp);
    if (tmp2) (void) hipFree(tmp2);
    if (code) kfmi_locations_free((void**) &L);
    else *locations = L;
    return code;
  };
  const hipStream_t st = ctx->st;
  bool ok = hipMalloc((void**) &d_cnt, 8 * (num + 1)) == hipSuccess &&
            hipMalloc((void**) &d_off, 8 * (num + 1)) == hipSuccess &&
            rocprim::exclusive_scan(nullptr, tb, d_cnt, d_off, (uint64_t) 0, (size_t) (num + 1),
                                    rocprim::plus<uint64_t>(), st) == hipSuccess &&
            hipMalloc(&tmp, tb ? tb : 1) == hipSuccess;
  if (!ok) return done(KFMI_E_DEVICE_ALLOC);
  if (hipEventRecord(ctx->ev[0], st) != hipSuccess) return done(KFMI_E_KERNEL);
  hipLaunchKernelGGL(loc_count_kernel, dim3((uint32_t) ((num + 1 + 255) / 256)), dim3(256), 0, st, d_res, num,
                     max_occ, d_cnt);
  ok = hipGetLastError() == hipSuccess &&
       rocprim::exclusive_scan(tmp, tb, d_cnt, d_off, (uint64_t) 0, (size_t) (num + 1), rocprim::plus<uint64_t>(),
                               st) == hipSuccess &&
       hipMemcpyAsync(&total, d_off + num, 8, hipMemcpyDeviceToHost, st) == hipSuccess &&
       hipStreamSynchronize(st) == hipSuccess;
  if (!ok) return done(KFMI_E_KERNEL);
  L->total = total;
  L->h_pos = (uint32_t*) malloc(4 * total + 4);
  if (!L->h_pos) return done(KFMI_E_ALLOCATING_RESULTS);
  if (hipMalloc((void**) &d_pos, 4 * total + 4) != hipSuccess ||
      hipMalloc((void**) &d_own, 4 * total + 4) != hipSuccess ||
      rocprim::inclusive_scan(nullptr, tb2, d_pos, d_own, (size_t) total, rocprim::maximum<uint32_t>(), st) !=
          hipSuccess ||
      hipMalloc(&tmp2, tb2 ? tb2 : 1) != hipSuccess)
    return done(KFMI_E_DEVICE_ALLOC);
  if (total) {   /* owner[i] = query of slot i: heads at each query's first slot, then a max-scan */
    if (hipMemsetAsync(d_pos, 0, 4 * total, st) != hipSuccess) return done(KFMI_E_KERNEL);   /* heads in d_pos */
    hipLaunchKernelGGL(loc_heads_kernel, dim3((uint32_t) ((num + 255) / 256)), dim3(256), 0, st, d_cnt, d_off, num,
                       d_pos);
    if (hipGetLastError() != hipSuccess ||
        rocprim::inclusive_scan(tmp2, tb2, d_pos, d_own, (size_t) total, rocprim::maximum<uint32_t>(), st) !=
            hipSuccess)
      return done(KFMI_E_KERNEL);
    const uint64_t rb = (total + 255) / 256;
    hipLaunchKernelGGL(loc_rows_kernel, dim3((uint32_t) (rb < (1u << 20) ? rb : (1u << 20))), dim3(256), 0, st,
                       d_res, d_off, total, d_own);   /* owner -> first row of each slot, in place */
    if (hipGetLastError() != hipSuccess) return done(KFMI_E_KERNEL);
  }
  SearchLaunch a{};
  a.st = st;
  a.ix = idx_args(di);
  a.res = d_res;
  a.num = num;
  a.sa = di->sa;
  a.sa_log2 = di->sa_log2;
  a.off = d_off;
  a.owner = d_own;
  a.total = total;
  a.pos = d_pos;
  ok = hipEventRecord(ctx->ev[1], st) == hipSuccess &&
       (total == 0 || dispatch(Op::Locate, di->K, di->nb, di->layout, a) == hipSuccess) &&
       hipEventRecord(ctx->ev[2], st) == hipSuccess &&
       hipMemcpyAsync(L->h_off, d_off, 8 * (num + 1), hipMemcpyDeviceToHost, st) == hipSuccess &&
       (total == 0 || hipMemcpyAsync(L->h_pos, d_pos, 4 * total, hipMemcpyDeviceToHost, st) == hipSuccess) &&
       hipStreamSynchronize(st) == hipSuccess;
  if (!ok) return done(KFMI_E_KERNEL);
  float ms01 = 0, ms12 = 0;
  (void) hipEventElapsedTime(&ms01, ctx->ev[0], ctx->ev[1]);
  (void) hipEventElapsedTime(&ms12, ctx->ev[1], ctx->ev[2]);
  t_ms[0] = ms01 + ms12;   /* scan + walk (the host read of the total sits between) */
  t_ms[1] = ms01;
  t_ms[2] = ms12;          /* the locate kernel alone */
  return done(KFMI_SUCCESS);
}

extern "C" int32_t kfmi_locate(void* index, void* results, uint32_t max_occ, void** locations)
{
  kfmi_fmi_t* f = (kfmi_fmi_t*) index;
  kfmi_res_t* r = (kfmi_res_t*) results;
  if (!locations) return KFMI_E_BAD_ARGUMENT;
  *locations = nullptr;
  if (!f || !r) return KFMI_E_BAD_ARGUMENT;
  if (!f->h_sa || !f->sa_rate) return KFMI_E_BAD_ARGUMENT;   /* index built without SA samples */
  if (!f->grp && !r->grp) {
    if (!f->dev || !r->d_results) return KFMI_E_NOT_ON_DEVICE;
    return locate_on(f, f->dev, r->d_results, r->num, max_occ, (kfmi_locations**) locations);
  }
  /* device group: every member locates its slice, the lists are concatenated */
  GroupIndex* gi = (GroupIndex*) f->grp;
  GroupSlices* gr = (GroupSlices*) r->grp;
  if (!gi || !gr) return KFMI_E_NOT_ON_DEVICE;
  if (gr->n != gi->n) return KFMI_E_BAD_ARGUMENT;
  kfmi_locations* part[KFMI_MAX_GROUP] = {};
  int32_t err = KFMI_SUCCESS;
  double ms[3] = {0, 0, 0};
  uint64_t total = 0;
  for (int i = 0; i < gi->n && !err; ++i) {
    if (gr->dev[i] != gi->dev[i]) err = KFMI_E_BAD_ARGUMENT;
    if (!err) err = locate_on(f, gi->di[i], gr->d_res[i], gr->num[i], max_occ, &part[i]);
    if (!err) {
      total += part[i]->total;
      for (int k = 0; k < 3; ++k) ms[k] += t_ms[k];
    }
  }
  kfmi_locations* L = err ? nullptr : new (std::nothrow) kfmi_locations();
  if (!err && !L) err = KFMI_E_ALLOCATING_RESULTS;
  if (!err) {
    L->num = r->num;
    L->total = total;
    L->h_off = (uint64_t*) malloc(8 * (r->num + 1));
    L->h_pos = (uint32_t*) malloc(4 * total + 4);
    if (!L->h_off || !L->h_pos) err = KFMI_E_ALLOCATING_RESULTS;
  }
  if (!err) {
    uint64_t base = 0;
    for (int i = 0; i < gi->n; ++i) {
      for (uint64_t j = 0; j < gr->num[i]; ++j) L->h_off[gr->q0[i] + j] = base + part[i]->h_off[j];
      if (part[i]->total) memcpy(L->h_pos + base, part[i]->h_pos, 4 * part[i]->total);
      base += part[i]->total;
    }
    L->h_off[r->num] = total;
    *locations = L;
    for (int k = 0; k < 3; ++k) t_ms[k] = ms[k];
  } else if (L) {
    kfmi_locations_free((void**) &L);
  }
  for (int i = 0; i < gi->n; ++i)
    if (part[i]) kfmi_locations_free((void**) &part[i]);
  return err;
}

/* ------------------------------------------------------------------------ */
/* streamed search from host memory: query H2D, packing, LF  */
/* and result D2H of successive chunks overlap on NSLOT HIP streams.  By    */
/* default the host packs each chunk to 2-bit code words (qpack.c) while    */
/* the GPU works on the previous ones, so PCIe carries 4 bytes per 16 bases */
/* (KFMI_STREAM_HOSTPACK=0: ASCII H2D and packing on the device).  Pinned   */
/* ASCII is DMA'd directly; pageable goes through pinned staging.           */
/* ------------------------------------------------------------------------ */

namespace {

constexpr int NSLOT = 3;

struct StreamSlot {
  hipStream_t st = nullptr;
  hipEvent_t done = nullptr;
  kfmi_dev_queries dq;         /* device ascii + packed of one chunk */
  uint32_t* d_res = nullptr;
  uint8_t* h_in = nullptr;     /* pinned staging */
  uint32_t* h_out = nullptr;
  uint32_t* h_pk = nullptr;    /* pinned host-packed code words */
  uint64_t cap_q = 0, cap_in = 0, cap_words = 0;
  uint64_t q0 = 0, n = 0;
  bool busy = false;
};

struct StreamPool {
  bool init = false;
  StreamSlot slot[NSLOT];
};
StreamPool g_pool[64];

void pool_free(int dev)
{
  StreamPool& p = g_pool[dev];
  if (!p.init) return;
  (void) hipSetDevice(dev);
  for (StreamSlot& s : p.slot) {
    if (s.st) (void) hipStreamSynchronize(s.st);
    if (s.dq.ascii) (void) hipFree(s.dq.ascii);
    if (s.dq.packed) (void) hipFree(s.dq.packed);
    if (s.d_res) (void) hipFree(s.d_res);
    if (s.h_in) (void) hipHostFree(s.h_in);
    if (s.h_out) (void) hipHostFree(s.h_out);
    if (s.h_pk) (void) hipHostFree(s.h_pk);
    if (s.done) (void) hipEventDestroy(s.done);
    if (s.st) (void) hipStreamDestroy(s.st);
    s = StreamSlot();
  }
  p.init = false;
}

/* Grows slot buffers to hold `cq` queries of `size` bytes packed in `words` words. */
int32_t slot_reserve(StreamSlot& s, uint64_t cq, uint32_t size, uint32_t words, bool stage_in, bool stage_out,
                     bool host_pack)
{
  if (!s.st) {
    if (hipStreamCreateWithFlags(&s.st, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&s.done, hipEventDisableTiming) != hipSuccess)
      return KFMI_E_NO_DEVICE;
  }
  const uint64_t in = cq * size + 16;
  if (in > s.cap_in) {
    if (s.dq.ascii) (void) hipFree(s.dq.ascii);
    if (s.h_in) { (void) hipHostFree(s.h_in); s.h_in = nullptr; }
    s.dq.ascii = nullptr;
    s.cap_in = 0;
    if (hipMalloc((void**) &s.dq.ascii, in) != hipSuccess) return KFMI_E_DEVICE_ALLOC;
    s.cap_in = in;
  }
  if (stage_in && !s.h_in && hipHostMalloc((void**) &s.h_in, s.cap_in, hipHostMallocDefault) != hipSuccess)
    return KFMI_E_ALLOCATING_MFASTA;
  if (cq > s.cap_q || (uint64_t) words * cq > s.cap_words) {
    if (s.dq.packed) (void) hipFree(s.dq.packed);
    if (s.d_res) (void) hipFree(s.d_res);
    if (s.h_out) { (void) hipHostFree(s.h_out); s.h_out = nullptr; }
    if (s.h_pk) { (void) hipHostFree(s.h_pk); s.h_pk = nullptr; }
    s.dq.packed = nullptr;
    s.d_res = nullptr;
    s.cap_q = s.cap_words = 0;
    if (hipMalloc((void**) &s.dq.packed, 4ull * words * cq) != hipSuccess ||
        hipMalloc((void**) &s.d_res, 8ull * cq) != hipSuccess)
      return KFMI_E_DEVICE_ALLOC;
    s.cap_q = cq;
    s.cap_words = (uint64_t) words * cq;
  }
  if (stage_out && !s.h_out && hipHostMalloc((void**) &s.h_out, 8ull * s.cap_q, hipHostMallocDefault) != hipSuccess)
    return KFMI_E_ALLOCATING_RESULTS;
  if (host_pack && !s.h_pk && hipHostMalloc((void**) &s.h_pk, 4ull * s.cap_words, hipHostMallocDefault) != hipSuccess)
    return KFMI_E_ALLOCATING_MFASTA;
  return KFMI_SUCCESS;
}

bool host_pinned(const void* p)
{
  hipPointerAttribute_t at;
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void) hipGetLastError();
    return false;
  }
  return at.type == hipMemoryTypeHost;
}

/* Persistent host workers for the streamed search (a chunk every few hundred
 * microseconds: spawning threads per chunk would cost as much as the work).
 * KFMI_HOST_THREADS (default min(16, cores)) threads including the caller. */
class HostPool {
 public:
  static HostPool& get()
  {
    static HostPool p;
    return p;
  }
  int size() const { return (int) th_.size() + 1; }
  /* fn(i) for i in [0, n) over the workers and the caller; returns when all are
   * done.  Calls from several host threads (one per device) take turns. */
  void run(int n, const std::function<void(int)>& fn)
  {
    if (n <= 1 || th_.empty()) {
      for (int i = 0; i < n; ++i) fn(i);
      return;
    }
    std::lock_guard<std::mutex> turn(run_mu_);
    {
      std::lock_guard<std::mutex> lk(mu_);
      fn_ = &fn;
      n_ = n;
      next_ = 0;
      left_ = n;
      ++gen_;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [&] { return left_ == 0; });
    fn_ = nullptr;
  }

 private:
  HostPool()
  {
    const char* e = getenv("KFMI_HOST_THREADS");
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    int v = e ? atoi(e) : (int) std::min(16u, hw);
    v = std::max(1, std::min(v, 64));
    for (int i = 0; i + 1 < v; ++i) th_.emplace_back([this] { loop(); });
  }
  ~HostPool()
  {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  void loop()
  {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      work();
    }
  }
  void work()
  {
    for (;;) {
      const std::function<void(int)>* f;
      int i;
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (!fn_ || next_ >= n_) return;
        i = next_++;
        f = fn_;
      }
      (*f)(i);
      std::lock_guard<std::mutex> lk(mu_);
      if (--left_ == 0) done_.notify_all();
    }
  }
  std::vector<std::thread> th_;
  std::mutex run_mu_, mu_;
  std::condition_variable cv_, done_;
  const std::function<void(int)>* fn_ = nullptr;
  int n_ = 0, next_ = 0, left_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

/* memcpy split over the host workers (pageable <-> pinned staging) */
void par_copy(void* dst, const void* src, uint64_t bytes)
{
  HostPool& hp = HostPool::get();
  const int nt = hp.size();
  if (nt == 1 || bytes < (8u << 20)) {
    memcpy(dst, src, bytes);
    return;
  }
  const uint64_t part = ((bytes + nt - 1) / nt + 4095) & ~4095ull;
  hp.run(nt, [&](int t) {
    const uint64_t b = part * t;
    if (b >= bytes) return;
    const uint64_t len = bytes - b < part ? bytes - b : part;
    memcpy((uint8_t*) dst + b, (const uint8_t*) src + b, len);
  });
}

/* ASCII rows -> word-major code words of one chunk, over the host workers */
void par_pack(const char* src, uint64_t n, uint32_t size, uint32_t* out)
{
  HostPool& hp = HostPool::get();
  const int parts = n < 4096 ? 1 : hp.size();
  hp.run(parts, [&](int t) {
    const uint64_t r0 = n * t / parts, r1 = n * (t + 1) / parts;
    kfmi_pack_rows((const uint8_t*) src + r0 * size, r1 - r0, size, out + r0, n);
  });
}

}  // namespace

extern "C" int32_t kfmi_host_alloc(uint64_t bytes, void** p)
{
  if (!p) return KFMI_E_BAD_ARGUMENT;
  *p = nullptr;
  if (hipSetDevice(kfmi_current_device()) != hipSuccess) return KFMI_E_NO_DEVICE;
  if (hipHostMalloc(p, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) return KFMI_E_ALLOCATING_MFASTA;
  return KFMI_SUCCESS;
}

extern "C" int32_t kfmi_host_free(void* p)
{
  if (p && hipHostFree(p) != hipSuccess) return KFMI_E_BAD_ARGUMENT;
  return KFMI_SUCCESS;
}

extern "C" int32_t kfmi_stream_release(void)
{
  const int dev = kfmi_current_device();
  if (dev < 0 || dev >= 64) return KFMI_E_NO_DEVICE;
  std::lock_guard<std::mutex> lk(g_ctx_mu);
  pool_free(dev);
  return KFMI_SUCCESS;
}

extern "C" int32_t kfmi_search_stream(void* index, const char* ascii, uint64_t num, uint32_t size,
                                      uint32_t* results, uint64_t chunk)
{
  kfmi_fmi_t* f = (kfmi_fmi_t*) index;
  if (!f || (!ascii && num) || (!results && num)) return KFMI_E_BAD_ARGUMENT;
  if (!f->dev) return KFMI_E_NOT_ON_DEVICE;
  kfmi_dev_index* di = f->dev;
  const uint32_t K = di->K;
  if (size == 0 || size % K || 64ull * size > 160ull * 1024) return KFMI_E_BAD_ARGUMENT;
  DevCtx* ctx = nullptr;
  int32_t err = ctx_for(di->device, &ctx);
  if (err) return err;
  if (num == 0) return KFMI_SUCCESS;
  const char* hp = getenv("KFMI_STREAM_HOSTPACK");
  const bool host_pack = !hp || atoi(hp) != 0;
  const uint64_t def_chunk = host_pack ? (1ull << 19) : (1ull << 16);   /* profiles/r01/e2e_sweep*.jsonl */
  if (chunk == 0) {
    const char* e = getenv("KFMI_STREAM_CHUNK");
    chunk = e ? strtoull(e, nullptr, 10) : def_chunk;
  }
  if (chunk == 0) chunk = def_chunk;
  if (chunk > num) chunk = num;
  const uint32_t steps = size / K, spw = 32 / (2 * K), nwords = (steps + spw - 1) / spw;
  const bool pin_in = host_pinned(ascii), pin_out = host_pinned(results);

  std::lock_guard<std::mutex> lk(g_ctx_mu);   /* one streamed search per device at a time */
  StreamPool& pool = g_pool[di->device];
  pool.init = true;
  for (StreamSlot& s : pool.slot) {
    err = slot_reserve(s, chunk, size, nwords, !pin_in && !host_pack, !pin_out, host_pack);
    if (err) return err;
    s.busy = false;
  }
  const auto t0 = std::chrono::steady_clock::now();
  const Op op = is_coop(di->backend) ? Op::Coop : Op::Task;
  IdxArgs ix = idx_args(di);
  err = use_ftab(di, ctx->st, ix, ftab_bases());
  if (err) return err;
  int32_t status = KFMI_SUCCESS;
  using clk = std::chrono::steady_clock;
  double host_ms = 0, wait_ms = 0;   /* host packing/staging; blocked on the GPU */
  auto since = [](clk::time_point t) { return std::chrono::duration<double, std::milli>(clk::now() - t).count(); };
  auto retire = [&](StreamSlot& s) {
    if (!s.busy) return;
    const auto tw = clk::now();
    const bool ok = hipEventSynchronize(s.done) == hipSuccess;
    wait_ms += since(tw);
    if (!ok) status = KFMI_E_KERNEL;
    else if (!pin_out) par_copy(results + 2 * s.q0, s.h_out, 8ull * s.n);
    s.busy = false;
  };
  const uint64_t nchunks = (num + chunk - 1) / chunk;
  for (uint64_t i = 0; i < nchunks && status == KFMI_SUCCESS; ++i) {
    StreamSlot& s = pool.slot[i % NSLOT];
    retire(s);
    if (status) break;
    s.q0 = i * chunk;
    s.n = num - s.q0 < chunk ? num - s.q0 : chunk;
    const char* src = ascii + s.q0 * size;
    const uint64_t bytes = s.n * size;
    const void* hsrc = src;
    const auto th = clk::now();
    if (host_pack) par_pack(src, s.n, size, s.h_pk);
    else if (!pin_in) {
      par_copy(s.h_in, src, bytes);
      hsrc = s.h_in;
    }
    host_ms += since(th);
    s.dq.device = di->device;
    s.dq.num = s.n;
    s.dq.size = size;
    s.dq.K = K;
    s.dq.steps = steps;
    s.dq.nwords = nwords;
    SearchLaunch a;
    a.st = s.st;
    a.ix = ix;
    a.qp = s.dq.packed;
    a.ascii = s.dq.ascii;
    a.m = size;
    a.maxw = host_pack ? 0 : fused_maxw(di->backend, nwords);
    a.num = s.n;
    a.steps = steps;
    a.nwords = nwords;
    a.res = s.d_res;
    void* hdst = pin_out ? (void*) (results + 2 * s.q0) : (void*) s.h_out;
    const bool up_ok = host_pack
                           ? hipMemcpyAsync(s.dq.packed, s.h_pk, 4ull * nwords * s.n, hipMemcpyHostToDevice, s.st) ==
                                 hipSuccess
                           : (hipMemcpyAsync(s.dq.ascii, hsrc, bytes, hipMemcpyHostToDevice, s.st) == hipSuccess &&
                              (a.maxw || launch_pack(&s.dq, s.st) == hipSuccess));
    if (!up_ok || dispatch(op, K, di->nb, di->layout, a) != hipSuccess ||
        hipMemcpyAsync(hdst, s.d_res, 8ull * s.n, hipMemcpyDeviceToHost, s.st) != hipSuccess ||
        hipEventRecord(s.done, s.st) != hipSuccess) {
      status = KFMI_E_KERNEL;
      break;
    }
    s.busy = true;
  }
  for (StreamSlot& s : pool.slot) retire(s);
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  t_ms[0] = ms;
  t_ms[1] = host_ms;   /* host packing or staging copies */
  t_ms[2] = wait_ms;   /* blocked on chunks in flight */
  return status;
}
