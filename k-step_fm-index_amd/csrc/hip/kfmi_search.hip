/*
 * kfmi_search.hip -- MI355X (gfx950) backward search: backend and device
 * selection, device index layouts and their upload, query packing, the
 * kernel dispatch tables, and the reference's GPU plugin entry points
 * (common/interface.h:36-41): transferCPUtoGPU, searchIndexGPU,
 * transferGPUtoCPU, free*GPU.  The kernels are in kfmi_kernels.h /
 * kfmi_coop.h / kfmi_locate.h (instantiated in kfmi_inst_*.hip); device
 * groups, locate and streaming in kfmi_group.hip, kfmi_locate.hip and
 * kfmi_stream.hip.
 *
 * Semantics: results are bit-identical to the reference CPU searchers
 * (fmIndexCPUBaseline.c:157-292 for task/coop/mid, -AltCounters.c:145-310
 * for the *-ac backends) -- not to the reference .cu files, which carry the
 * defects B1-B4 of SURVEY.md Appendix B.
 */
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <atomic>
#include <mutex>
#include <new>
#include <vector>

#include "../kfmi_internal.h"
#include "kfmi_device.h"
#include "kfmi_coop.h"
#include "kfmi_locate.h"
#include "kfmi_runtime.h"

namespace kfmi {

/* ------------------------------------------------------------------------ */
/* backend registry and per-thread state                                    */
/* ------------------------------------------------------------------------ */

static const char* kBackendNames[KFMI_BK_COUNT] = {
    "task", "coop", "task-ac", "coop-ac", "task-mid", "coop-mid", "task-ac-mid", "coop-ac-mid", "task-grp", "coop-grp"};

static thread_local int t_backend = -1;
static thread_local bool t_backend_implicit = true;   /* neither KFMI_BACKEND nor kfmi_set_backend chose it */
thread_local int t_device = -1;
thread_local int32_t t_last_error = KFMI_SUCCESS;
thread_local double t_ms[3] = {0, 0, 0};
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
  return -1;
}

extern "C" kfmi_backend_t kfmi_backend(void)
{
  if (t_backend < 0) {
    int b = backend_from_name(getenv("KFMI_BACKEND"));
    t_backend = b >= 0 ? b : KFMI_BK_TASK_MID;
    t_backend_implicit = b < 0;
  }
  return (kfmi_backend_t) t_backend;
}

/* The backend an index of K-steps is uploaded for: the selected one, except
 * that the implicit default (task-mid, K <= 2) becomes coop-grp for K = 3, 4
 * indexes, the one layout those run on at speed. */
int backend_for(uint32_t K)
{
  const int b = kfmi_backend();
  return (t_backend_implicit && (K == 3 || K == 4)) ? (int) KFMI_BK_COOP_GRP : b;
}

extern "C" uint32_t kfmi_backend_tag(kfmi_backend_t b)
{
  return (b == KFMI_BK_TASK_AC || b == KFMI_BK_COOP_AC || b == KFMI_BK_TASK_AC_MID || b == KFMI_BK_COOP_AC_MID)
             ? 201u : 101u;
}

extern "C" int32_t kfmi_set_backend(const char* name)
{
  int b = backend_from_name(name);
  if (b < 0) return KFMI_E_BAD_ARGUMENT;
  t_backend = b;
  t_backend_implicit = false;
  return KFMI_SUCCESS;
}

extern "C" const char* kfmi_get_backend(void) { return kBackendNames[kfmi_backend()]; }

extern "C" int32_t kfmi_device_count(void)
{
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

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

/* The physical GPU behind a device number: HIP_VISIBLE_DEVICES renumbers the
 * devices per process, the PCI bus id does not (bench.py's ranks compare it). */
extern "C" int32_t kfmi_device_pci_bus_id(int32_t device, char* buf, int32_t len)
{
  if (!buf || len < 13) return KFMI_E_BAD_ARGUMENT;
  if (device < 0 || device >= kfmi_device_count()) return KFMI_E_NO_DEVICE;
  if (hipDeviceGetPCIBusId(buf, len, device) != hipSuccess) {
    (void) hipGetLastError();
    return KFMI_E_NO_DEVICE;
  }
  return KFMI_SUCCESS;
}

RwLock& index_lock(const void* f)
{
  static_assert(sizeof(RwLock) == sizeof(pthread_rwlock_t), "RwLock is the handle's pthread lock");
  return *reinterpret_cast<RwLock*>(&static_cast<kfmi_fmi_t*>(const_cast<void*>(f))->rw);
}

extern "C" void kfmi_set_last_error(int32_t e) { t_last_error = e; }

extern "C" int32_t kfmi_set_ftab(uint32_t bases)
{
  if (bases > 16) return KFMI_E_BAD_ARGUMENT;
  t_ftab = (int) bases;
  return KFMI_SUCCESS;
}

uint32_t ftab_bases(void)
{
  if (t_ftab >= 0) return (uint32_t) t_ftab;
  static const uint32_t env = [] {   /* KFMI_FTAB, read once per process */
    const char* e = getenv("KFMI_FTAB");
    const int v = e ? atoi(e) : 0;
    return v > 0 && v <= 16 ? (uint32_t) v : 0u;
  }();
  return env;
}

/* Test knobs of the search path: read from the environment once per process
 * (KFMI_SPLIT, KFMI_FUSED) and switched through their setters afterwards, so
 * no search reads the environment.  -2 = not read yet. */
static std::atomic<int> g_split_class{-2};   /* 0 = by table size (split_for), 1/2/4 = that class */
static std::atomic<int> g_fused{-2};         /* 1 = fused packing where it fits, 0 = pack kernel */

static int knob_once(std::atomic<int>& k, int (*read_env)())
{
  int v = k.load(std::memory_order_relaxed);
  if (v == -2) {
    int expect = -2;
    k.compare_exchange_strong(expect, read_env(), std::memory_order_relaxed);
    v = k.load(std::memory_order_relaxed);
  }
  return v;
}

static int split_class_from_env()
{
  const char* e = getenv("KFMI_SPLIT");
  if (!e || !*e) return 0;
  const int v = atoi(e);
  if (v != 1 && v != 2 && v != 4)
    fprintf(stderr, "kstepfmi: KFMI_SPLIT=%s: only 1, 2 or 4 (table-size class) are read; using 1\n", e);
  return (v == 2 || v == 4) ? v : 1;
}

static int fused_from_env()
{
  const char* e = getenv("KFMI_FUSED");
  return (e && !atoi(e)) ? 0 : 1;
}

extern "C" int32_t kfmi_set_split_class(uint32_t cls)
{
  if (cls != 0 && cls != 1 && cls != 2 && cls != 4) return KFMI_E_BAD_ARGUMENT;
  g_split_class.store((int) cls, std::memory_order_relaxed);
  return KFMI_SUCCESS;
}

extern "C" int32_t kfmi_set_fused(int32_t on)
{
  g_fused.store(on ? 1 : 0, std::memory_order_relaxed);
  return KFMI_SUCCESS;
}
extern "C" int32_t kfmi_last_error(void) { return t_last_error; }

extern "C" int32_t kfmi_last_timing(double* ms_total, double* ms_pack, double* ms_lf)
{
  if (ms_total) *ms_total = t_ms[0];
  if (ms_pack) *ms_pack = t_ms[1];
  if (ms_lf) *ms_lf = t_ms[2];
  return KFMI_SUCCESS;
}

static DevCtx g_ctx[64];
static std::mutex g_ctx_mu;   /* guards the one-time creation of g_ctx[dev] only */

int32_t ctx_for(int dev, DevCtx** out)
{
  if (dev < 0 || dev >= 64) return KFMI_E_NO_DEVICE;
  if (hipSetDevice(dev) != hipSuccess) return KFMI_E_NO_DEVICE;
  DevCtx& c = g_ctx[dev];
  {
    std::lock_guard<std::mutex> lk(g_ctx_mu);
    if (!c.init) {
      if (hipStreamCreateWithFlags(&c.st, hipStreamNonBlocking) != hipSuccess) return KFMI_E_NO_DEVICE;
      c.init = true;
    }
  }
  *out = &c;
  return KFMI_SUCCESS;
}

/* Per calling thread and device: a search stream and three timing events.
 * Searches from different threads therefore run concurrently (small,
 * latency-bound batches overlap on the device); uploads stay on the shared
 * per-device stream and complete before they return.  Released when the
 * thread exits. */
struct ThreadRes {
  hipStream_t st[64] = {};
  hipEvent_t ev[64][3] = {};
  ~ThreadRes()
  {
    for (int d = 0; d < 64; ++d) {
      if (!st[d] && !ev[d][0] && !ev[d][1] && !ev[d][2]) continue;
      if (hipSetDevice(d) != hipSuccess) continue;
      if (st[d]) (void) hipStreamDestroy(st[d]);
      for (hipEvent_t& e : ev[d])
        if (e) (void) hipEventDestroy(e);
    }
  }
};
static thread_local ThreadRes t_res;

hipEvent_t* thread_events(int dev)
{
  if (dev < 0 || dev >= 64) return nullptr;
  hipEvent_t* ev = t_res.ev[dev];
  for (int i = 0; i < 3; ++i)
    if (!ev[i] && hipEventCreate(&ev[i]) != hipSuccess) {
      ev[i] = nullptr;
      return nullptr;
    }
  return ev;
}

hipStream_t thread_stream(int dev)
{
  if (dev < 0 || dev >= 64) return nullptr;
  if (!t_res.st[dev] && hipStreamCreateWithFlags(&t_res.st[dev], hipStreamNonBlocking) != hipSuccess)
    t_res.st[dev] = nullptr;
  return t_res.st[dev];
}

/* ------------------------------------------------------------------------ */
/* query packing: ASCII [num][m] -> codes [nwords][num], step t of query q in */
/* word t/SPW, bits 2K*(t%SPW)..; step t consumes chars m-1-K*t-i (i<K), the  */
/* order of fmIndexCPUBaseline.c:200-226.                                   */
/*                                                                          */
/* Reads of any length: block (x, y) packs the tq rows q0 = x*tq .. and the   */
/* word chunk y (words [y*wc, (y+1)*wc)), staging only the bytes of those     */
/* rows that chunk reads -- [m-rem-K*s1, m-rem-K*s0) for its steps [s0, s1),  */
/* at most K*SPW*wc <= 1 KiB per row -- HBM -> LDS with 16-byte loads where   */
/* the slice is aligned, then one thread per row builds the chunk's words     */
/* (writes of a word row: consecutive queries, coalesced).                   */
/* ------------------------------------------------------------------------ */

/* LDS row pitch of the pack kernel: whole rows stay contiguous (pitch m), a
 * slice of a longer row takes a 16-B multiple (the launch sizes LDS with the
 * largest slice, wc words) */
__host__ __device__ constexpr uint32_t pack_pitch(uint32_t m, uint32_t len)
{
  return len == m ? m : ((len + 15u) & ~15u);
}

template <int K>
__global__ __launch_bounds__(256) void pack_queries_kernel(const uint8_t* __restrict__ q, uint64_t num,
                                                           uint32_t m, uint32_t steps, uint32_t nwords,
                                                           uint32_t tq, uint32_t wc, uint32_t* __restrict__ out,
                                                           uint32_t rem)
{
  extern __shared__ __attribute__((aligned(16))) uint8_t tile[];
  constexpr int SPW = 32 / (2 * K);
  const uint64_t q0 = (uint64_t) blockIdx.x * tq;
  const uint64_t nq = (num - q0) < tq ? (num - q0) : tq;
  const uint32_t w0 = blockIdx.y * wc;
  const uint32_t w1 = w0 + wc < nwords ? w0 + wc : nwords;
  const uint32_t s0 = w0 * SPW, s1 = (w1 * SPW < steps ? w1 * SPW : steps);
  /* one chunk (reads up to ~1 KiB): whole rows, one contiguous piece of nq
   * rows; else row r's slice [lo, lo + len) at tile + r * pitch */
  const bool whole = gridDim.y == 1;
  const uint32_t lo = whole ? 0u : (m - rem) - K * s1, len = whole ? m : K * (s1 - s0);
  const uint32_t pitch = pack_pitch(m, len);
  /* 16-B copies only where the whole slice is 16-B words (K = 3 slices are
   * 15-base words: a 1,020-byte chunk, or a short last one, takes bytes) */
  const bool al = ((m | lo | len) & 15u) == 0 && ((((uintptr_t) q) & 15u) == 0);
  if (whole) {
    const uint64_t bytes = nq * m;
    const uint8_t* src = q + q0 * m;
    if ((((uintptr_t) src) & 15u) == 0) {
      const uint64_t n16 = bytes / 16;
      for (uint64_t i = threadIdx.x; i < n16; i += blockDim.x)
        reinterpret_cast<uint4*>(tile)[i] = reinterpret_cast<const uint4*>(src)[i];
      for (uint64_t i = n16 * 16 + threadIdx.x; i < bytes; i += blockDim.x) tile[i] = src[i];
    } else {
      for (uint64_t i = threadIdx.x; i < bytes; i += blockDim.x) tile[i] = src[i];
    }
  } else if (al) {
    const uint32_t n16 = len / 16;
    for (uint64_t i = threadIdx.x; i < nq * n16; i += blockDim.x) {
      const uint64_t r = i / n16, k = i % n16;
      reinterpret_cast<uint4*>(tile + r * pitch)[k] = reinterpret_cast<const uint4*>(q + (q0 + r) * m + lo)[k];
    }
  } else {
    for (uint64_t i = threadIdx.x; i < nq * len; i += blockDim.x) {
      const uint64_t r = i / len, k = i % len;
      tile[r * pitch + k] = q[(q0 + r) * m + lo + k];
    }
  }
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < nq; t += blockDim.x) {
    const uint8_t* p = tile + (uint64_t) t * pitch;   /* p[pos - lo] for pos in [lo, lo + len) */
    for (uint32_t w = w0; w < w1; ++w) {
      uint32_t word = 0;
#pragma unroll
      for (int j = 0; j < SPW; ++j) {
        const uint32_t st = w * SPW + j;
        if (st < steps) {
          const int pos = (int) (m - rem) - 1 - (int) (K * st);
          uint32_t c = 0;
#pragma unroll
          for (int i = 0; i < K; ++i) c |= code_of(p[pos - i - (int) lo]) << (2 * i);
          word |= c << (2 * K * j);
        }
      }
      out[(uint64_t) w * num + q0 + t] = word;
    }
    /* remainder table index: the last rem bases, read from HBM (chunk 0 only) */
    if (rem && blockIdx.y == 0) out[(uint64_t) nwords * num + q0 + t] = rem_code(q + (q0 + t) * m + m - rem, rem);
  }
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

/* GRP layout construction from tag-101 entries (plus the padding entry with
 * the end counters): line b * NGRP + g = [planes of entry b | cnt_b[NCG g ..]]. */
/* Reads the entries as stored (tag 100 or 101: plane word i of the tag-101
 * order is word perm[i] of the stored entry), so neither a second copy nor an
 * interleave pass is needed; entry nent (the padding block) comes from `pad`. */
struct PlanePerm {
  uint32_t p[32];
};

template <int K, int NB>
__global__ __launch_bounds__(256) void build_grp_kernel(const uint32_t* __restrict__ ent, uint64_t nent,
                                                        const uint32_t* __restrict__ pad, PlanePerm perm,
                                                        uint64_t nlines, uint32_t* __restrict__ lines)
{
  using GI = Geo<K, NB, LAY_INTER>;
  using GG = Geo<K, NB, LAY_GRP>;
  static_assert(GI::BMW <= 32, "plane permutation table");
  const uint64_t l = (uint64_t) blockIdx.x * 256 + threadIdx.x;
  if (l >= nlines) return;
  const uint64_t b = l / GG::NGRP, g = l % GG::NGRP;
  const uint32_t* src = b < nent ? ent + b * GI::EW : pad;
  uint32_t* dst = lines + l * GG::EW;
  for (int i = 0; i < GI::BMW; ++i) dst[i] = src[perm.p[i]];
  for (int c = 0; c < GG::NCG; ++c) dst[GI::BMW + c] = src[GI::BMW + g * GG::NCG + c];
  for (int i = GI::BMW + GG::NCG; i < GG::EW; ++i) dst[i] = 0;
}

/* Code registers the task kernel needs to pack a query itself (0: use the
 * pack kernel).  KFMI_FUSED=0 / kfmi_set_fused(0) forces the separate pack launch. */
/* Fused packing keeps 16 bases per register word (MAXW words): 8 words up to
 * 128 K-step bases, 16 up to 256, else the pack kernel. */
int fused_maxw(int backend, uint32_t bases)
{
  (void) backend;   /* task and coop kernels both pack in-kernel (m <= 256 fits either's LDS staging) */
  if (!knob_once(g_fused, fused_from_env)) return 0;
  return bases <= 128 ? 8 : (bases <= 256 ? 16 : 0);
}

static bool nb_supported(uint32_t nb)
{
  return nb == 1 || nb == 2 || nb == 4 || nb == 6 || nb == 8 || nb == 14 || nb == 30;
}

/* dispatch_one<K, NB, LAY> is compiled in kfmi_inst_*.hip (one unit per K and
 * layout, built in parallel). */
KFMI_FOR_NB(KFMI_EXTERN, 1, LAY_INTER)
KFMI_FOR_NB(KFMI_EXTERN, 2, LAY_INTER)
KFMI_FOR_NB(KFMI_EXTERN, 1, LAY_AC)
KFMI_FOR_NB(KFMI_EXTERN, 2, LAY_AC)
KFMI_FOR_NB(KFMI_EXTERN, 1, LAY_MID)
KFMI_FOR_NB(KFMI_EXTERN, 2, LAY_MID)
KFMI_FOR_NB(KFMI_EXTERN, 1, LAY_MIDAC)
KFMI_FOR_NB(KFMI_EXTERN, 2, LAY_MIDAC)
KFMI_EXTERN(4, 2, LAY_GRP)
KFMI_EXTERN(3, 2, LAY_GRP)

hipError_t dispatch(Op op, uint32_t K, uint32_t nb, int lay, const SearchLaunch& a, unsigned long long* d_total)
{
#define KFMI_CASE(KK, NBV, LAYV)                                   \
  if (K == KK && nb == NBV && lay == LAYV) return dispatch_one<KK, NBV, LAYV>(op, a, d_total);
  KFMI_FOR_NB(KFMI_CASE, 1, LAY_INTER)
  KFMI_FOR_NB(KFMI_CASE, 2, LAY_INTER)
  KFMI_FOR_NB(KFMI_CASE, 1, LAY_AC)
  KFMI_FOR_NB(KFMI_CASE, 2, LAY_AC)
  KFMI_FOR_NB(KFMI_CASE, 1, LAY_MID)
  KFMI_FOR_NB(KFMI_CASE, 2, LAY_MID)
  KFMI_FOR_NB(KFMI_CASE, 1, LAY_MIDAC)
  KFMI_FOR_NB(KFMI_CASE, 2, LAY_MIDAC)
  KFMI_CASE(4, 2, LAY_GRP)
  KFMI_CASE(3, 2, LAY_GRP)
#undef KFMI_CASE
  return hipErrorInvalidValue;
}

bool is_coop(int backend);

/* Whether the backend's kernel exists for this geometry (the cooperative
 * kernel needs 16-byte-aligned chunks, CoopCfg::OK). */
static bool geometry_supported(int backend, uint32_t K, uint32_t nb, int lay)
{
  if (lay == LAY_GRP) {   /* instantiated for K = 3, 4 with d = 64 (K <= 2 has the MID128 lines) */
    if ((K != 3 && K != 4) || nb != 2) return false;
    return !is_coop(backend) || (K == 4 ? CoopCfg<Geo<4, 2, LAY_GRP>>::OK : CoopCfg<Geo<3, 2, LAY_GRP>>::OK);
  }
  if (!nb_supported(nb) || (K != 1 && K != 2)) return false;
  if (!is_coop(backend)) return true;
#define KFMI_OKC(KK, NBV, LAYV) \
  if (K == KK && nb == NBV && lay == LAYV) return CoopCfg<Geo<KK, NBV, LAYV>>::OK;
  KFMI_FOR_NB(KFMI_OKC, 1, LAY_INTER)
  KFMI_FOR_NB(KFMI_OKC, 2, LAY_INTER)
  KFMI_FOR_NB(KFMI_OKC, 1, LAY_AC)
  KFMI_FOR_NB(KFMI_OKC, 2, LAY_AC)
  KFMI_FOR_NB(KFMI_OKC, 1, LAY_MID)
  KFMI_FOR_NB(KFMI_OKC, 2, LAY_MID)
  KFMI_FOR_NB(KFMI_OKC, 1, LAY_MIDAC)
  KFMI_FOR_NB(KFMI_OKC, 2, LAY_MIDAC)
#undef KFMI_OKC
  return false;
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

static hipError_t dispatch_build_grp(uint32_t K, uint32_t nb, uint32_t tag, const uint32_t* ent, uint64_t nent,
                                     const uint32_t* pad, uint64_t nlines, uint32_t* lines, hipStream_t st)
{
  if ((K != 3 && K != 4) || nb != 2 || (tag != 100 && tag != 101)) return hipErrorInvalidValue;
  PlanePerm perm;
  for (uint32_t w = 0; w < nb; ++w)
    for (uint32_t s = 0; s < K; ++s)
      for (uint32_t t = 0; t < 2; ++t)
        perm.p[kfmi_plane_index(101, K, nb, s, t, w)] = kfmi_plane_index(tag, K, nb, s, t, w);
  const dim3 grid((uint32_t) ((nlines + 255) / 256));
  if (K == 4)
    hipLaunchKernelGGL((build_grp_kernel<4, 2>), grid, dim3(256), 0, st, ent, nent, pad, perm, nlines, lines);
  else
    hipLaunchKernelGGL((build_grp_kernel<3, 2>), grid, dim3(256), 0, st, ent, nent, pad, perm, nlines, lines);
  return hipGetLastError();
}

static int layout_of(int backend)
{
  switch (backend) {
    case KFMI_BK_TASK: case KFMI_BK_COOP: return LAY_INTER;
    case KFMI_BK_TASK_AC: case KFMI_BK_COOP_AC: return LAY_AC;
    case KFMI_BK_TASK_MID: case KFMI_BK_COOP_MID: return LAY_MID;
    case KFMI_BK_TASK_AC_MID: case KFMI_BK_COOP_AC_MID: return LAY_MIDAC;
    default: return LAY_GRP;   /* KFMI_BK_TASK_GRP, KFMI_BK_COOP_GRP */
  }
}

bool is_coop(int backend)
{
  return backend == KFMI_BK_COOP || backend == KFMI_BK_COOP_AC || backend == KFMI_BK_COOP_MID ||
         backend == KFMI_BK_COOP_AC_MID || backend == KFMI_BK_COOP_GRP;
}

/* ------------------------------------------------------------------------ */
/* host helpers for the device layouts                                      */
/* ------------------------------------------------------------------------ */

/* The host entries, or null while they live only in HBM; acquire pairs with
 * the release in kfmi_host_entries (another thread may be fetching them). */
static inline const uint32_t* host_index(const kfmi_fmi_t* f)
{
  return __atomic_load_n(&f->h_index, __ATOMIC_ACQUIRE);
}

/* Locate walks need the plain LF.  On the AltCounters layouts a step taken
 * backward from the sentinel -- in the last real block L, for the codes the
 * AC rule sends to entry L+1 -- differs from it by a constant per code c: the
 * sentinel holds cnt_L[c] plus (n+1) mod d rows of block L read from the
 * planes ('$' rows included) plus the padding rows for code 0
 * (kfmi_transform_ac; when (n+1) mod d == 0, B5, the transform's masked read
 * adds no rows and the padding is a whole block), where the plain LF counts
 * every row of block L below X and leaves each D_s out.  out[c] = that
 * difference, which kfmi_locate.h lf_row takes off such a step. */
static bool ac_locate_fix(const kfmi_fmi_t* f, uint32_t* out)
{
  const uint32_t nc = 1u << (2 * f->steps), nb = f->nbitmaps, d = f->chunk;
  const uint32_t last = (uint32_t) (((uint64_t) f->bwtsize + d - 1) / d) - 1u, rem = f->bwtsize % d;
  const uint32_t poff = f->tag >= 200 ? nc / 2 : 0u;   /* tag 200/201 entries: [counters | planes] */
  std::vector<uint32_t> ent;
  const uint32_t* e;
  if (last >= f->nentries) return false;
  if (const uint32_t* hi = host_index(f)) {
    e = hi + (uint64_t) last * f->entry_words;
  } else {   /* entries only in HBM: fetch that one */
    ent.assign(f->entry_words, 0u);
    DeviceGuard dg;
    if (hipSetDevice(f->d_entries_dev) != hipSuccess ||
        hipMemcpy(ent.data(), f->d_entries + (uint64_t) last * f->entry_words, 4ull * f->entry_words,
                  hipMemcpyDeviceToHost) != hipSuccess)
      return false;
    e = ent.data();
  }
  for (uint32_t c = 0; c < nc; ++c) {
    uint32_t all = 0, head = 0;   /* rows of code c in the block, in its first rem rows */
    for (uint32_t w = 0; w < nb; ++w) {
      uint32_t m = 0xFFFFFFFFu;
      for (uint32_t st = 0; st < f->steps; ++st)
        for (uint32_t t = 0; t < 2; ++t) {
          const uint32_t pl = e[poff + kfmi_plane_index(f->tag, f->steps, nb, st, t, w)];
          m &= ((c >> (2 * st + t)) & 1u) ? pl : ~pl;
        }
      int sh = (int) rem - 32 * (int) w;
      sh = sh < 0 ? 0 : (sh > 32 ? 32 : sh);
      all += (uint32_t) __builtin_popcount(m);
      head += (uint32_t) __builtin_popcount(m & (uint32_t) (0xFFFFFFFF00000000ull >> sh));
    }
    uint32_t dollar = 0;
    for (uint32_t st = 0; st < f->steps; ++st)
      dollar += (f->dollarPositionBWT[st] / d == last && f->dollarBaseBWT[st] == c) ? 1u : 0u;
    const uint32_t added = head + (c == 0 ? d - rem : 0u);   /* what the transform adds to cnt_L */
    out[c] = added - all + dollar;
  }
  return true;
}

/* Counters at row n+1 (one past the last row) from a tag-100/101 index:
 * cnt_{E-1} + rows of each code in the last block, $ rows excluded -- each
 * distinct row once, as the builder's counters exclude them (a 'ref'-mode index
 * can put two D_s on one row), so the padding entry is the next
 * block the builder would have written and every layout agrees past the end:
 * INTER's line-local step from entry E-1, GRP/MID's stored copies and
 * MID's backward steps (corrected by dollar_dup like every other block).  Used
 * for the padding entry that keeps R/d == nentries in bounds when
 * (n+1) % d == 0 (reference defect B5: it reads past the end there). */
static bool end_counters(const kfmi_fmi_t* f, uint32_t* out)
{
  const uint32_t nc = 1u << (2 * f->steps), nb = f->nbitmaps;
  const uint32_t last = f->nentries - 1;
  std::vector<uint32_t> dev_last;
  const uint32_t* e;
  if (const uint32_t* hi = host_index(f)) {
    e = hi + (uint64_t) last * f->entry_words;
  } else {   /* entries only in HBM: fetch the last one */
    dev_last.assign(f->entry_words, 0u);
    DeviceGuard dg;
    if (hipSetDevice(f->d_entries_dev) != hipSuccess) return false;
    const hipError_t ce = hipMemcpy(dev_last.data(), f->d_entries + (uint64_t) last * f->entry_words,
                                    4ull * f->entry_words, hipMemcpyDeviceToHost);
    if (ce != hipSuccess) return false;
    e = dev_last.data();
  }
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
    for (uint32_t s = 0; s < f->steps; ++s) {
      bool first = true;   /* the first s of its row */
      for (uint32_t t = 0; t < s; ++t) first = first && f->dollarPositionBWT[t] != f->dollarPositionBWT[s];
      if (first && f->modposdollarBWT[s] == last && f->dollarBaseBWT[s] == c && f->bwtsize > f->dollarPositionBWT[s])
        pop--;
    }
    out[c] = e[2 * nb * f->steps + c] + pop;
  }
  return true;
}

/* Host image of the entries for a layout, converting tags as needed.
 * INTER/MID/GRP need plain counters (tag 100/101); MIDAC takes those or
 * an AltCounters file (tag 200/201, turned back into its tag-100 file); AC
 * needs tag 201 (a tag-100/101 input goes through the tfmiAC transform first). */
static int32_t host_entries_for(const kfmi_fmi_t* f, int lay, kfmi_fmi_t** owned, const kfmi_fmi_t** use)
{
  *owned = nullptr;
  *use = f;
  if (lay == LAY_INTER || lay == LAY_MID || lay == LAY_MIDAC || lay == LAY_GRP) {
    /* tag 101 as is; tag 100 is interleaved on the device (upload_entries),
     * or on the host with KFMI_HOST_INTERLEAVE=1 (A/B experiment) */
    if (f->tag == 100 && getenv("KFMI_HOST_INTERLEAVE") && atoi(getenv("KFMI_HOST_INTERLEAVE"))) {
      int32_t e = kfmi_transform_interleave((void*) f, (void**) owned);
      if (e) return e;
      *use = *owned;
      return KFMI_SUCCESS;
    }
    if (f->tag == 101 || f->tag == 100) return KFMI_SUCCESS;
    if (lay == LAY_MIDAC) {
      /* AltCounters semantics from an AltCounters file (the reference's -AC
       * searchers' input): its tag-100 file back (kfmi_transform_plain), whose
       * MID128 lines and AC tail the layout is built from */
      int32_t e = kfmi_transform_plain((void*) f, (void**) owned);
      if (e) return e;
      *use = *owned;
      return KFMI_SUCCESS;
    }
    return KFMI_INDEX_VER_INTERLEAVE;   /* an AC file cannot feed a plain-counter backend */
  }
  /* AC */
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

void free_dev_index(kfmi_dev_index* di)
{
  if (!di) return;
  if (di->device >= 0) (void) hipSetDevice(di->device);
  if (di->ent) (void) hipFree(di->ent);
  if (di->sa) (void) hipFree(di->sa);
  if (di->ac_tail) (void) hipFree(di->ac_tail);
  for (uint2* t : di->ftab)
    if (t) (void) hipFree(t);
  for (uint2* t : di->rtab)
    if (t) (void) hipFree(t);
  delete di;
}

/* Host-to-device copy of a whole buffer, queued on `st`.  Pageable and pinned
 * sources alike go straight to hipMemcpyAsync: on this ROCm a 1.5 GB copy
 * from pageable memory runs at 56.5 GB/s against 57.6 from pinned memory,
 * while staging through two pinned 64 MB buffers allocated per call (the
 * earlier form) paid 42 ms for the allocation alone
 * (`bin/copy_probe`, profiles/r04/copy_probe_r4m.jsonl). */
hipError_t h2d(void* dst, const void* src, uint64_t bytes, hipStream_t st)
{
  return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st);
}

/* tag-100 -> tag-101 entries (kfmi_transform_interleave's plane order,
 * transformIndexBitmaps.c) on the device: out word p of an entry is in word
 * perm[p] of the same entry. */
constexpr uint32_t KFMI_MAX_ENTRY_WORDS = 320;   /* K <= 2, d <= 960: 2*30*2 + 16 = 136; K = 4, d = 64: 272 */
struct EntryPerm {
  uint32_t p[KFMI_MAX_ENTRY_WORDS];
};

/* In place, a batch of whole entries per workgroup staged through LDS; no
 * second copy of the index is allocated (the LF kernels measured 3.5 % slower
 * when the upload went through an extra 4.5 GB buffer, profiles/r01). */
constexpr uint32_t IL_LDS_WORDS = 8192;

__global__ __launch_bounds__(256) void interleave_entries_kernel(uint32_t* __restrict__ ent, uint64_t nent, uint32_t ew,
                                                                 EntryPerm perm)
{
  __shared__ uint32_t buf[IL_LDS_WORDS];
  const uint32_t epb = IL_LDS_WORDS / ew;   /* entries per batch */
  const uint64_t nbatch = (nent + epb - 1) / epb;
  for (uint64_t b = blockIdx.x; b < nbatch; b += gridDim.x) {
    const uint64_t e0 = b * epb;
    const uint32_t ne = (uint32_t) (nent - e0 < epb ? nent - e0 : epb);
    const uint32_t nw = ne * ew;
    uint32_t* g = ent + e0 * ew;
    for (uint32_t i = threadIdx.x; i < nw; i += 256) buf[i] = g[i];
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nw; i += 256) {
      const uint32_t e = i / ew;
      g[i] = buf[e * ew + perm.p[i - e * ew]];
    }
    __syncthreads();
  }
}

/* The stored entries of `src` into device memory at dst: from the host image,
 * or device to device when they only live in HBM (built there). */
static hipError_t entries_in(void* dst, const kfmi_fmi_t* src, uint64_t body, hipStream_t st)
{
  if (const uint32_t* hi = host_index(src)) return h2d(dst, hi, body, st);
  if (!src->d_entries) return hipErrorInvalidValue;
  int cur = 0;
  hipError_t e = hipGetDevice(&cur);
  if (e != hipSuccess) return e;
  if (cur == src->d_entries_dev) return hipMemcpyAsync(dst, src->d_entries, body, hipMemcpyDeviceToDevice, st);
  return hipMemcpyPeerAsync(dst, cur, src->d_entries, src->d_entries_dev, body, st);
}

/* The entries of `src` as tag 101 (plain family) or as stored, into device
 * memory at dst (`body` bytes). */
static hipError_t upload_entries(void* dst, const kfmi_fmi_t* src, uint64_t body, hipStream_t st)
{
  if (src->tag != 100) return entries_in(dst, src, body, st);
  const uint32_t ew = src->entry_words, K = src->steps, nb = src->nbitmaps;
  if (ew > KFMI_MAX_ENTRY_WORDS || ew == 0) return hipErrorInvalidValue;
  EntryPerm perm;
  for (uint32_t p = 0; p < ew; ++p) perm.p[p] = p;   /* counters keep their place */
  for (uint32_t w = 0; w < nb; ++w)
    for (uint32_t k = 0; k < K; ++k)
      for (uint32_t t = 0; t < 2; ++t) perm.p[kfmi_plane_index(101, K, nb, k, t, w)] = kfmi_plane_index(100, K, nb, k, t, w);
  hipError_t e = entries_in(dst, src, body, st);
  const uint64_t nent = body / (4ull * ew), nbatch = (nent + IL_LDS_WORDS / ew - 1) / (IL_LDS_WORDS / ew);
  if (e == hipSuccess && nent) {
    hipLaunchKernelGGL(interleave_entries_kernel, dim3(grid_blocks(nbatch, 1u << 16)),
                       dim3(256), 0, st, (uint32_t*) dst, nent, ew, perm);
    e = hipGetLastError();
  }
  const hipError_t es = hipStreamSynchronize(st);
  return e != hipSuccess ? e : es;
}

/* Device copy of the index's SA samples (locate); none when it has none. */
int32_t upload_sa(const kfmi_fmi_t* f, kfmi_dev_index* di, DevCtx* ctx)
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
int32_t upload_index(kfmi_fmi_t* f, int backend, int dev, DevCtx* ctx, kfmi_dev_index** out)
{
  if (f->steps == 2 && layout_of(backend) == LAY_GRP) {
    /* a K = 2 file (the reference's GPU index) on the grouped-counter layout:
     * its K = 4 index derived on the device, laid out, and dropped again
     * (DESIGN.md 5d'); the handle keeps the K = 4 device copy.  The K = 4
     * geometry and row limits are checked first, so a file the layout cannot
     * take fails before the derivation's buffers are allocated. */
    if (!geometry_supported(backend, 4, f->nbitmaps, LAY_GRP) ||
        ((uint64_t) f->nentries + 3u) * f->chunk > 0xFFFFFFFFull)
      return KFMI_E_BAD_ARGUMENT;
    kfmi_fmi_t* g = nullptr;
    int32_t e = derive_index(f, 4, dev, false, &g);
    if (e) return e;
    kfmi_dev_index* di = nullptr;
    e = upload_index(g, backend, dev, ctx, &di);
    freeIndex((void**) &g);
    if (e) return e;
    if (out) {
      *out = di;
      return KFMI_SUCCESS;
    }
    if (f->dev) free_dev_index(f->dev);
    f->dev = di;
    return KFMI_SUCCESS;
  }
  if (f->steps < 1 || f->steps > 4) return KFMI_E_BAD_ARGUMENT;   /* GPU kernels: K in {1,2}; 4 on LAY_GRP */
  if (!nb_supported(f->nbitmaps)) return KFMI_E_BAD_ARGUMENT;
  const int lay = layout_of(backend);
  if (!geometry_supported(backend, f->steps, f->nbitmaps, lay)) return KFMI_E_BAD_ARGUMENT;
  /* rows are u32 on the device: every layout's padding blocks and the
   * AltCounters cap, (S+2)*d - 1 (ac_clamp), must stay below 2^32 -- which
   * leaves out only the last ~3d rows of the u32 range */
  if (((uint64_t) f->nentries + 3u) * f->chunk > 0xFFFFFFFFull) return KFMI_E_BAD_ARGUMENT;
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
  /* LAY_AC: the last real block E-1 (tag-201 entries end with the sentinel E):
   * steps from there on keep the reference's counter (line_local_prev) */
  if (lay == LAY_AC) di->ac_tail_b0 = src->nentries >= 2 ? src->nentries - 2 : 0;
  di->K = f->steps;
  di->d = f->chunk;
  di->nb = f->nbitmaps;
  di->bwtsize = f->bwtsize;
  di->nentries = src->nentries;
  for (uint32_t s = 0; s < 4; ++s) {
    di->dl.dpos[s] = s < f->steps ? f->dollarPositionBWT[s] : 0xFFFFFFFFu;
    di->dl.dbase[s] = s < f->steps ? f->dollarBaseBWT[s] : 0xFFFFFFFFu;
    di->dl.dblk[s] = s < f->steps ? f->dollarPositionBWT[s] / f->chunk : 0xFFFFFFFFu;
  }
  di->dl.duniq = 0;
  for (uint32_t s = 0; s < f->steps && s < 4; ++s) {
    bool first = true;
    for (uint32_t t = 0; t < s; ++t) first = first && f->dollarPositionBWT[t] != f->dollarPositionBWT[s];
    if (first) di->dl.duniq |= 1u << s;
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
    if (lay == LAY_INTER && !end_counters(src, pad.data() + 2 * f->nbitmaps * f->steps)) return fail(KFMI_E_KERNEL);
    if (upload_entries(di->ent, src, body, ctx->st) != hipSuccess ||
        hipMemcpyAsync((uint8_t*) di->ent + body, pad.data(), 4ull * ew * 2, hipMemcpyHostToDevice, ctx->st) !=
            hipSuccess ||
        hipStreamSynchronize(ctx->st) != hipSuccess)
      return fail(KFMI_E_KERNEL);
  } else if (lay == LAY_GRP) {
    /* NGRP lines per block (planes repeated, one counter group each), built on
     * the device from the tag-101 entries plus one padding entry carrying the
     * end counters (B5: R/d == nentries) */
    const uint32_t ngrp = nc < 16 ? 1u : nc / 16;
    const uint32_t lw = (uint32_t) pow2ceil((int) (2 * f->nbitmaps * f->steps + (nc < 16 ? nc : 16)));
    const uint64_t nlines = (uint64_t) (src->nentries + 1) * ngrp;
    if (!end_counters(src, pad.data() + 2 * f->nbitmaps * f->steps)) return fail(KFMI_E_KERNEL);
    /* entries that already live on this device (built here, no host image) are
     * read in place; otherwise one staging copy as stored (no interleave pass) */
    const bool in_place = !host_index(src) && src->d_entries && src->d_entries_dev == dev;
    uint32_t *tmp = nullptr, *d_pad = nullptr;
    di->ent_bytes = 4ull * lw * nlines;
    if ((!in_place && hipMalloc((void**) &tmp, body + 16) != hipSuccess) ||
        hipMalloc((void**) &d_pad, 4ull * ew) != hipSuccess || hipMalloc((void**) &di->ent, di->ent_bytes) != hipSuccess) {
      if (tmp) (void) hipFree(tmp);
      if (d_pad) (void) hipFree(d_pad);
      return fail(KFMI_E_DEVICE_ALLOC);
    }
    bool ok = (in_place || entries_in(tmp, src, body, ctx->st) == hipSuccess) &&
              hipMemcpyAsync(d_pad, pad.data(), 4ull * ew, hipMemcpyHostToDevice, ctx->st) == hipSuccess &&
              dispatch_build_grp(f->steps, f->nbitmaps, src->tag, in_place ? src->d_entries : tmp, src->nentries, d_pad,
                                 nlines, di->ent, ctx->st) == hipSuccess &&
              hipStreamSynchronize(ctx->st) == hipSuccess;
    if (tmp) (void) hipFree(tmp);
    (void) hipFree(d_pad);
    if (!ok) return fail(KFMI_E_KERNEL);
  } else {   /* LAY_MID, LAY_MIDAC */
    /* MID: pairs of blocks per line, built on the device from tag-101 entries;
     * counters of the last line (odd block count) and of one padding line are
     * "rows past n+1 read as A" extensions of the end counters. */
    const uint32_t E = src->nentries;
    const uint32_t nreal = (E + 1) / 2;
    const uint32_t nl = nreal + 1;
    const uint32_t lw = (uint32_t) pow2ceil((int) (2 * 2 * f->nbitmaps * f->steps + nc));
    std::vector<uint32_t> endc(nc), ext(2 * nc);
    if (!end_counters(src, endc.data())) return fail(KFMI_E_KERNEL);
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
  }
  if (lay == LAY_AC || lay == LAY_MIDAC) {
    /* 4 x NC words: LAY_MIDAC's AltCounters counters of entries E-1, E, E+1
     * (kfmi_ac_tail), and on every AltCounters layout row 3, the locate walk's
     * correction of a backward step from the sentinel (ac_locate_fix) */
    std::vector<uint32_t> tail(4 * nc, 0u);
    if (lay == LAY_MIDAC && kfmi_ac_tail(src, tail.data(), &di->ac_tail_b0) != KFMI_SUCCESS)
      return fail(KFMI_E_BAD_ARGUMENT);
    if (!ac_locate_fix(src, tail.data() + 3 * nc)) return fail(KFMI_E_KERNEL);
    if (hipMalloc((void**) &di->ac_tail, 16ull * nc) != hipSuccess) {
      di->ac_tail = nullptr;
      return fail(KFMI_E_DEVICE_ALLOC);
    }
    if (hipMemcpyAsync(di->ac_tail, tail.data(), 16ull * nc, hipMemcpyHostToDevice, ctx->st) != hipSuccess ||
        hipStreamSynchronize(ctx->st) != hipSuccess)
      return fail(KFMI_E_KERNEL);
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

/* Gather split for the per-lane (task) kernels (IdxArgs::split): how many
 * exec-masked lane groups issue each step's index gathers (launch_task,
 * kfmi_kernels.h, turns it into a fetch form per geometry).  Auto values:
 * 4 = every task kernel splits; 2 = only the fused kernel for reads of <= 128
 * bases, except where the asm fetch (fetch_ends_x4) applies, which splits
 * in two groups whenever this is 2 or 4; 1 = none.
 *  - tables over 3.5 GB: 4.  Past the translation reach the per-instruction
 *    page cliff costs up to 2.7x (task-grp 96 GB: 17.6 -> 6.8 ms at 100 bp,
 *    25.1 -> 9.1 at 150 bp; the retired AC128 layout's 6.4 GB: 18.1 -> 10.0, 26.1 -> 15.5);
 *  - 2-3.5 GB, one line per LF (MID128 / MIDAC): 2 (task-mid 9.53 -> 9.45 at
 *    100 bp, but 14.41 -> 14.83 ms with the 16-word kernel at 150 bp);
 *  - 2-3.5 GB, other layouts: 4 (task-ac 12.87 -> 11.81 at 100 bp,
 *    18.93 -> 17.94 at 150 bp; the retired packed layout 14.0 -> 13.3).
 * profiles/r02/sweep_split_r2ah.jsonl, sweep_split150_r2aj.jsonl; the asm
 * forms: profiles/r03/sweep_r3n.jsonl, sweep150_r3n.jsonl.  The ftab lookup
 * (one gather per read) is never split: that measured slower.
 * KFMI_SPLIT=1|2|4 / kfmi_set_split_class (a test knob) answers in place of the table size, so that
 * a small test index runs the fetch form a table of that size class gets
 * (launch_task: one form per geometry and class). */
/* Knobs of earlier rounds' experiments that no longer exist, and KFMI_SPLIT
 * values of the old fetch-form meaning (4/6/7/8 picked a form; it now names a
 * table-size class 1/2/4): one message per process, so a rerun of an old
 * sweep does not quietly time the default path under another label. */
static void warn_stale_knobs_once()
{
  static std::once_flag once;
  std::call_once(once, [] {
    for (const char* k : {"KFMI_REORDER", "KFMI_LDS_PAD", "KFMI_COOP_ISSUE", "KFMI_QPT", "KFMI_NT_FROM"})
      if (getenv(k)) fprintf(stderr, "kstepfmi: %s is no longer read (removed experiment knob); ignored\n", k);
  });
}

static uint32_t split_for(uint64_t table_bytes, int layout)
{
  warn_stale_knobs_once();
  const int cls = knob_once(g_split_class, split_class_from_env);
  if (cls) return (uint32_t) cls;
  if (table_bytes > 3500000000ull) return 4u;
  if (table_bytes > 2000000000ull) return (layout == LAY_MID || layout == LAY_MIDAC) ? 2u : 4u;
  return 1u;
}

IdxArgs idx_args(const kfmi_dev_index* di)
{
  IdxArgs ix;
  ix.ent = di->ent;
  ix.bwtsize = di->bwtsize;
  ix.dl = di->dl;
  ix.ftab = nullptr;
  ix.ftab_steps = 0;
  ix.ftab_mask = 0;
  ix.ac_tail = di->ac_tail;
  ix.ac_tail_b0 = di->ac_tail_b0;
  ix.rtab = nullptr;
  ix.rem = 0;
  ix.split = split_for(di->ent_bytes, di->layout);
  /* the last row of block nentries, which every layout holds (INTER / AC: 2
   * padding entries, MID: the padding line, GRP: the padding entry); on the
   * AltCounters layouts ac_clamp's bound, block ceil(n+1 / d) + 1 */
  const uint64_t d = di->d;
  const uint64_t cap = (di->layout == LAY_AC || di->layout == LAY_MIDAC)
                           ? ((di->bwtsize + d - 1) / d + 2) * d - 1
                           : ((uint64_t) di->nentries + 1) * d - 1;
  ix.lf_cap = (uint32_t) std::min<uint64_t>(cap, 0xFFFFFFFFull);
  return ix;
}

/* Pointer jumping over the successor array: out[X] = next[next[X]]. */
__global__ __launch_bounds__(256) void jump_kernel(const uint32_t* __restrict__ next, uint64_t rows,
                                                   uint32_t* __restrict__ out)
{
  for (uint64_t i = (uint64_t) blockIdx.x * 256 + threadIdx.x; i < rows; i += (uint64_t) gridDim.x * 256)
    out[i] = next[next[i]];
}

/* After the jumps every row's successor must be a '$' row D_s. */
__global__ __launch_bounds__(256) void walk_end_kernel(const uint32_t* __restrict__ next, uint64_t rows, DollarArgs dl,
                                                       uint32_t K, uint32_t* __restrict__ bad)
{
  for (uint64_t i = (uint64_t) blockIdx.x * 256 + threadIdx.x; i < rows; i += (uint64_t) gridDim.x * 256) {
    const uint32_t e = next[i];
    bool d = false;
    for (uint32_t s = 0; s < K; ++s) d = d || dl.dpos[s] == e;
    if (!d) atomicOr(bad, 2u);
  }
}

/* ---- the sampled walk check (large indexes) --------------------------------
 * Rows whose hashed index has its low 8 bits zero are "samples" (1 in 256,
 * independent of the LF order); a sample's walk runs over the successor array
 * to the next sample or '$' row, marking the rows it passes (next[] := WSENT)
 * and leaving the sample's skeleton successor in next[sample].  Every row
 * then lies on a sample's path, or is an "orphan" (the few rows before the
 * first sample of each chain, or a cycle with no sample), and each orphan
 * walks forward to a stop.  Pointer jumping over the skeleton decides the
 * rest.  Walks past kWalkLimit steps, a walk running into a marked row (LF not
 * injective) or list overflow fall back to full pointer jumping. */
constexpr uint32_t WSENT = 0xFFFFFFFFu;
constexpr uint32_t kWalkLimit = 1u << 16;
constexpr uint32_t kOrphanCap = 1u << 16;
enum : uint32_t { WALK_BAD_IMAGE = 1u, WALK_CYCLE = 2u, WALK_FALLBACK = 4u };

__device__ __forceinline__ bool walk_sample(uint32_t x)
{
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return (x & 255u) == 0;
}

__device__ __forceinline__ bool walk_dollar(uint32_t x, const DollarArgs& dl, uint32_t K)
{
  bool d = false;
  for (uint32_t s = 0; s < K; ++s) d = d || dl.dpos[s] == x;
  return d;
}

/* Appends row i to list (wave-aggregated) when want; overflow sets the fallback flag. */
__device__ __forceinline__ void walk_append(bool want, uint32_t i, uint32_t* __restrict__ list, uint32_t cap,
                                            uint32_t* __restrict__ count, uint32_t* __restrict__ flags)
{
  const uint64_t m = __ballot(want);
  if (!m) return;
  const uint32_t lane = threadIdx.x & 63u;
  const int leader = __ffsll((unsigned long long) m) - 1;
  uint32_t base = 0;
  if ((int) lane == leader) base = atomicAdd(count, (uint32_t) __popcll(m));
  base = __shfl(base, leader);
  if (want) {
    const uint32_t slot = base + __builtin_amdgcn_mbcnt_hi((uint32_t) (m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t) m, 0u));
    if (slot < cap) list[slot] = i;
    else atomicOr(flags, WALK_FALLBACK);
  }
}

/* The sample list: every non-'$' row with walk_sample(row).  One block per
 * kSampleChunk rows gathers its ~256 samples in LDS and claims their slots
 * with one global atomic (one counter shared by 12 M per-wave atomics was
 * 118 ms at 3 Gbase, all of it contention). */
constexpr uint32_t kSampleChunk = 1u << 16;
constexpr uint32_t kSampleBuf = 1024;   /* Binomial(65536, 1/256): mean 256, sd 16 */

__global__ __launch_bounds__(256) void walk_samples_kernel(uint64_t rows, DollarArgs dl, uint32_t K,
                                                           uint32_t* __restrict__ list, uint32_t cap,
                                                           uint32_t* __restrict__ count, uint32_t* __restrict__ flags)
{
  __shared__ uint32_t buf[kSampleBuf];
  __shared__ uint32_t n, base;
  for (uint64_t c0 = (uint64_t) blockIdx.x * kSampleChunk; c0 < rows; c0 += (uint64_t) gridDim.x * kSampleChunk) {
    if (threadIdx.x == 0) n = 0;
    __syncthreads();
    const uint64_t c1 = min(rows, c0 + kSampleChunk);
    for (uint64_t i = c0 + threadIdx.x; i < c1; i += 256)
      if (walk_sample((uint32_t) i) && !walk_dollar((uint32_t) i, dl, K)) {
        const uint32_t s = atomicAdd(&n, 1u);
        if (s < kSampleBuf) buf[s] = (uint32_t) i;
      }
    __syncthreads();
    const uint32_t m = min(n, kSampleBuf);
    if (threadIdx.x == 0) {
      if (n > kSampleBuf) atomicOr(flags, WALK_FALLBACK);
      base = atomicAdd(count, m);
    }
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < m; t += 256) {
      if (base + t < cap) list[base + t] = buf[t];
      else atomicOr(flags, WALK_FALLBACK);
    }
    __syncthreads();
  }
}

/* Each sample's walk to the next stop, marking the rows passed. */
__global__ __launch_bounds__(256) void walk_paths_kernel(uint32_t* __restrict__ next, const uint32_t* __restrict__ list,
                                                         const uint32_t* __restrict__ count, uint32_t cap, DollarArgs dl,
                                                         uint32_t K, uint32_t* __restrict__ flags)
{
  const uint32_t n = min(*count, cap);
  for (uint32_t t = blockIdx.x * 256 + threadIdx.x; t < n; t += gridDim.x * 256) {
    const uint32_t s = list[t];
    uint32_t j = next[s], steps = 0;
    while (!walk_dollar(j, dl, K) && !walk_sample(j)) {
      const uint32_t nj = next[j];
      if (nj == WSENT || ++steps > kWalkLimit) {   /* two walks meet (LF not injective) or a long gap */
        atomicOr(flags, WALK_FALLBACK);
        break;
      }
      next[j] = WSENT;
      j = nj;
    }
    next[s] = j;
  }
}

/* Rows on no sample's path: neither marked, a sample nor a '$' row. */
__global__ __launch_bounds__(256) void walk_orphans_kernel(const uint32_t* __restrict__ next, uint64_t rows, DollarArgs dl,
                                                           uint32_t K, uint32_t* __restrict__ list,
                                                           uint32_t* __restrict__ count, uint32_t* __restrict__ flags)
{
  for (uint64_t base = (uint64_t) blockIdx.x * 256 + (threadIdx.x & ~63u); base < rows; base += (uint64_t) gridDim.x * 256) {
    const uint64_t i = base + (threadIdx.x & 63u);
    bool want = false;
    if (i < rows) {
      const uint32_t x = (uint32_t) i;
      want = next[i] != WSENT && !walk_sample(x) && !walk_dollar(x, dl, K);
    }
    walk_append(want, (uint32_t) i, list, kOrphanCap, count, flags);
  }
}

/* Each orphan walks over unmarked rows to a stop; coming back to itself is a
 * cycle with no sample and no '$' row. */
__global__ __launch_bounds__(256) void walk_orphan_paths_kernel(const uint32_t* __restrict__ next, uint64_t rows,
                                                                const uint32_t* __restrict__ list,
                                                                const uint32_t* __restrict__ count, DollarArgs dl,
                                                                uint32_t K, uint32_t* __restrict__ flags)
{
  const uint32_t n = min(*count, kOrphanCap);
  for (uint32_t t = blockIdx.x * 256 + threadIdx.x; t < n; t += gridDim.x * 256) {
    const uint32_t o = list[t];
    uint32_t j = o;
    for (uint32_t steps = 0;; ++steps) {
      const uint32_t nj = next[j];
      if ((uint64_t) nj >= rows) {   /* never: j is unmarked and lf_next_kernel keeps images in range */
        atomicOr(flags, WALK_FALLBACK);
        break;
      }
      if (nj == o) {
        atomicOr(flags, WALK_CYCLE);
        break;
      }
      if (walk_dollar(nj, dl, K) || walk_sample(nj) || next[nj] == WSENT) break;   /* a stop, or a sample's path */
      if (steps >= kWalkLimit) {
        atomicOr(flags, WALK_FALLBACK);
        break;
      }
      j = nj;
    }
  }
}

/* One round of pointer jumping over the samples' skeleton successors (in
 * place: a pointer read mid-round is at least as far along as the round's
 * start value, so each round still at least doubles every distance). */
__global__ __launch_bounds__(256) void walk_skeleton_kernel(uint32_t* __restrict__ next, uint64_t rows,
                                                            const uint32_t* __restrict__ list,
                                                            const uint32_t* __restrict__ count, uint32_t cap,
                                                            DollarArgs dl, uint32_t K, uint32_t* __restrict__ flags,
                                                            bool last)
{
  const uint32_t n = min(*count, cap);
  for (uint32_t t = blockIdx.x * 256 + threadIdx.x; t < n; t += gridDim.x * 256) {
    const uint32_t s = list[t];
    const uint32_t j = next[s];
    if (walk_dollar(j, dl, K)) continue;
    if ((uint64_t) j >= rows) {   /* a mark, not a row: only after a walk broke off (the host skips us then) */
      atomicOr(flags, WALK_FALLBACK);
      continue;
    }
    if (last) atomicOr(flags, WALK_CYCLE);
    else next[s] = next[j];
  }
}

/* Whether every LF_K walk of di ends at a '$' row -- true of every index of a
 * text (LF_K takes the row of suffix p to the row of p - K) -- kept in
 * di->lf_perm.  A 'ref'-mode index of a text with bytes other than A/C/G/T
 * (the reference builder counts the raw bytes in one order and the codes in
 * another, genFMindex.c:283-309, :402-424) has LF_K cycles that never reach a
 * '$' row: locate walks on it need not end and a derivation would compose a
 * map that is not the text's.  The successor of every row (lf_next_kernel,
 * '$' rows fixed), then, below 2^22 rows or when the sampled check falls
 * back, ceil(log2 rows) rounds of full pointer jumping (8 bytes per row of
 * scratch, ~32 random-gather passes at 3 Gbase: 2.0 s); otherwise the sampled
 * check above (4 bytes per row, about one random gather and one random store
 * per row). */
static std::atomic<int> g_walk_mode{0};   /* 0 = by size, 1 = full pointer jumping, 2 = sampled */
static std::atomic<int> g_walk_last{0};   /* 1 = full, 2 = sampled, 3 = sampled then full */

extern "C" int32_t kfmi_set_walk_check(uint32_t mode)
{
  if (mode > 2) return KFMI_E_BAD_ARGUMENT;
  g_walk_mode.store((int) mode, std::memory_order_relaxed);
  return KFMI_SUCCESS;
}

extern "C" int32_t kfmi_walk_check_last(void) { return g_walk_last.load(std::memory_order_relaxed); }

int32_t check_lf_walks(kfmi_dev_index* di, hipStream_t st)
{
  const uint64_t rows = di->bwtsize;
  const int mode = g_walk_mode.load(std::memory_order_relaxed);
  const bool sampled = mode == 2 || (mode == 0 && rows >= (1ull << 22));
  const uint32_t cap = (uint32_t) std::min<uint64_t>(rows / 128 + 4096, rows);
  uint32_t *next = nullptr, *tmp = nullptr, *bad = nullptr;
  auto done = [&](int32_t code) {
    if (next) (void) hipFree(next);
    if (tmp) (void) hipFree(tmp);
    if (bad) (void) hipFree(bad);
    return code;
  };
  /* bad[0] flags, bad[1] sample count, bad[2] orphan count, then the lists */
  const uint64_t tmp_words = sampled ? 3 + (uint64_t) cap + kOrphanCap : 4;
  if (hipMalloc((void**) &next, 4 * rows) != hipSuccess || hipMalloc((void**) &bad, 4 * tmp_words) != hipSuccess)
    return done(KFMI_E_DEVICE_ALLOC);
  SearchLaunch a{};
  a.st = st;
  a.ix = idx_args(di);
  a.num = rows;
  a.perm_next = next;
  a.perm_bad = bad;
  auto fetch_flags = [&](uint32_t& h) {
    return hipGetLastError() == hipSuccess && hipMemcpyAsync(&h, bad, 4, hipMemcpyDeviceToHost, st) == hipSuccess &&
           hipStreamSynchronize(st) == hipSuccess;
  };
  if (hipMemsetAsync(bad, 0, 12, st) != hipSuccess || dispatch(Op::PermCheck, di->K, di->nb, di->layout, a) != hipSuccess)
    return done(KFMI_E_KERNEL);
  const dim3 grid(grid_blocks((rows + 255) / 256, 65536));
  uint32_t h_bad = 0;
  if (sampled) {
    uint32_t* list = bad + 3;
    uint32_t* orphans = list + cap;
    const dim3 wgrid(grid_blocks((cap + 255) / 256, 8192));
    hipLaunchKernelGGL(walk_samples_kernel, dim3(grid_blocks((rows + kSampleChunk - 1) / kSampleChunk, 65536)), dim3(256), 0,
                       st, rows, di->dl, di->K, list, cap, bad + 1, bad);
    hipLaunchKernelGGL(walk_paths_kernel, wgrid, dim3(256), 0, st, next, list, bad + 1, cap, di->dl, di->K, bad);
    hipLaunchKernelGGL(walk_orphans_kernel, grid, dim3(256), 0, st, next, rows, di->dl, di->K, orphans, bad + 2, bad);
    hipLaunchKernelGGL(walk_orphan_paths_kernel, dim3(256), dim3(256), 0, st, next, rows, orphans, bad + 2, di->dl, di->K,
                       bad);
    if (!fetch_flags(h_bad)) return done(KFMI_E_KERNEL);
    if (!h_bad) {   /* every walk reached a stop: the skeleton decides (after a broken walk it may hold marks) */
      for (uint64_t span = 1; span <= cap; span <<= 1)   /* skeleton paths are at most cap long */
        hipLaunchKernelGGL(walk_skeleton_kernel, wgrid, dim3(256), 0, st, next, rows, list, bad + 1, cap, di->dl, di->K,
                           bad, false);
      hipLaunchKernelGGL(walk_skeleton_kernel, wgrid, dim3(256), 0, st, next, rows, list, bad + 1, cap, di->dl, di->K, bad,
                         true);
      if (!fetch_flags(h_bad)) return done(KFMI_E_KERNEL);
    }
    if ((h_bad & (WALK_BAD_IMAGE | WALK_CYCLE)) || !(h_bad & WALK_FALLBACK)) {
      g_walk_last.store(2, std::memory_order_relaxed);
      di->lf_perm.store((h_bad & (WALK_BAD_IMAGE | WALK_CYCLE)) ? 0 : 1);
      return done(KFMI_SUCCESS);
    }
    /* undecided: the successors again, then full pointer jumping */
    if (hipMemsetAsync(bad, 0, 4, st) != hipSuccess || dispatch(Op::PermCheck, di->K, di->nb, di->layout, a) != hipSuccess)
      return done(KFMI_E_KERNEL);
  }
  if (hipMalloc((void**) &tmp, 4 * rows) != hipSuccess) return done(KFMI_E_DEVICE_ALLOC);
  for (uint64_t span = 1; span < rows; span <<= 1) {   /* after round r every row looks 2^r steps ahead */
    hipLaunchKernelGGL(jump_kernel, grid, dim3(256), 0, st, next, rows, tmp);
    std::swap(next, tmp);
  }
  hipLaunchKernelGGL(walk_end_kernel, grid, dim3(256), 0, st, next, rows, di->dl, di->K, bad);
  if (!fetch_flags(h_bad)) return done(KFMI_E_KERNEL);
  g_walk_last.store(sampled ? 3 : 1, std::memory_order_relaxed);
  di->lf_perm.store(h_bad ? 0 : 1);
  return done(KFMI_SUCCESS);
}

/* Reads with m % K = rem != 0 (the reference reads P[-1] there, defect B6):
 * their last rem bases are resolved by the remainder table, built once per
 * (index, rem) from the uploaded layout (rem_tab_kernel), and the K-steps
 * cover bases 0 .. m-rem-1.  The result is the reads' suffix-array interval,
 * which is what every plain-semantics backend returns for m % K = 0; the
 * AltCounters-semantics backends keep rejecting such reads (their intervals
 * differ from the true ones where the reference's sentinel counts, and the
 * reference defines no result here).  The ftab is not combined with it. */
bool rem_supported(int layout)
{
  return layout == LAY_INTER || layout == LAY_MID || layout == LAY_GRP;
}

int32_t use_rtab(kfmi_dev_index* di, hipStream_t st, IdxArgs& ix, uint32_t rem)
{
  ix.rtab = nullptr;
  ix.rem = 0;
  if (!rem) return KFMI_SUCCESS;
  if (rem >= di->K || rem > 3 || !rem_supported(di->layout)) return KFMI_E_BAD_ARGUMENT;
  {
    std::lock_guard<std::mutex> lk(di->ftab_mu);
    if (!di->rtab[rem]) {
      uint2* t = nullptr;
      if (hipMalloc((void**) &t, 8ull << (2 * rem)) != hipSuccess) return KFMI_E_DEVICE_ALLOC;
      SearchLaunch a{};
      a.st = st;
      a.ix = idx_args(di);
      a.ftab_out = t;
      a.rem = rem;
      if (dispatch(Op::RemTab, di->K, di->nb, di->layout, a) != hipSuccess || hipStreamSynchronize(st) != hipSuccess) {
        (void) hipFree(t);
        return KFMI_E_KERNEL;
      }
      di->rtab[rem] = t;   /* published complete; never replaced */
    }
  }
  ix.rtab = di->rtab[rem];
  ix.rem = rem;
  ix.ftab = nullptr;
  ix.ftab_steps = 0;
  ix.ftab_mask = 0;
  return KFMI_SUCCESS;
}

/* The ftab of `bases` bases, (re)built on the device from the uploaded layout
 * with the search's own LF steps; sets ix.ftab (null when off or when bases is
 * not a multiple of K). */
int32_t use_ftab(kfmi_dev_index* di, hipStream_t st, IdxArgs& ix, uint32_t bases)
{
  ix.ftab = nullptr;
  ix.ftab_steps = 0;
  ix.ftab_mask = 0;
  if (!bases || bases % di->K || bases > 16) return KFMI_SUCCESS;
  {
    std::lock_guard<std::mutex> lk(di->ftab_mu);
    if (!di->ftab[bases]) {
      const uint64_t n = 1ull << (2 * bases);
      uint2* t = nullptr;
      if (hipMalloc((void**) &t, 8 * n) != hipSuccess) return KFMI_E_DEVICE_ALLOC;
      SearchLaunch a{};
      a.st = st;
      a.ix = idx_args(di);
      a.ftab_out = t;
      a.ftab_steps = bases / di->K;
      a.ftab_n = n;
      if (dispatch(Op::Ftab, di->K, di->nb, di->layout, a) != hipSuccess || hipStreamSynchronize(st) != hipSuccess) {
        (void) hipFree(t);
        return KFMI_E_KERNEL;
      }
      di->ftab[bases] = t;   /* published complete; never replaced */
    }
  }
  ix.ftab = di->ftab[bases];
  ix.ftab_steps = bases / di->K;
  ix.ftab_mask = bases >= 16 ? 0xFFFFFFFFu : (1u << (2 * bases)) - 1u;
  return KFMI_SUCCESS;
}

void free_dev_queries(kfmi_dev_queries* dq)
{
  if (!dq) return;
  if (dq->device >= 0) (void) hipSetDevice(dq->device);
  if (dq->ascii) (void) hipFree(dq->ascii);
  if (dq->packed) (void) hipFree(dq->packed);
  delete dq;
}

void query_geometry(kfmi_dev_queries* dq, uint32_t K)
{
  dq->K = K;
  dq->rem = dq->size % K;
  dq->steps = (dq->size - dq->rem) / K;
  const uint32_t spw = 32 / (2 * K);
  dq->nwords = (dq->steps + spw - 1) / spw;
}

/* Host-packed upload (KFMI_UPLOAD=packed, DESIGN.md 6a'): for K in {1, 2, 4}
 * the reads are packed to their 2-bit code words on the host workers (the
 * streamed search's packer, qpack.c) chunk by chunk into pinned buffers while
 * the previous chunks' DMAs run, so a quarter of the bytes cross PCIe, and the
 * device keeps only the code words the LF kernels read when packing is not
 * fused.  Opt-in: it wins where the host workers out-pack the link (16 workers
 * on a fast box: 1 GB in 12.4 ms against 18.3 ms for the ASCII DMA) and loses
 * where they do not (a slower box of the same pool: 18.8 ms; config #5's
 * 1.5 GB 72 ms against ~45), so the default upload is the ASCII one. */
static bool upload_host_packed(const kfmi_qrys_t* q, uint32_t K)
{
  const char* e = getenv("KFMI_UPLOAD");
  return e && !strcmp(e, "packed") && (K == 1 || K == 2 || K == 4) && q->num && q->h_queries;
}

/* The device's two pinned chunk buffers, kept between uploads (pinning costs
 * ~0.3 ms per MB, copy_probe: 42 ms for 2 x 64 MB), grown to `need` bytes
 * each, and their events.  The caller holds ctx->up_mu while it uses them and
 * leaves the copies from them complete. */
hipError_t upload_staging(DevCtx* ctx, uint64_t need)
{
  hipError_t e = hipSuccess;
  if (ctx->up_cap < need) {
    for (int b = 0; b < 2; ++b)
      if (ctx->up_buf[b]) {
        (void) hipHostFree(ctx->up_buf[b]);
        ctx->up_buf[b] = nullptr;
      }
    ctx->up_cap = 0;
    for (int b = 0; b < 2 && e == hipSuccess; ++b) e = hipHostMalloc(&ctx->up_buf[b], need, hipHostMallocDefault);
    if (e != hipSuccess) return e;
    ctx->up_cap = need;
  }
  for (int b = 0; b < 2 && e == hipSuccess; ++b)
    if (!ctx->up_ev[b]) e = hipEventCreateWithFlags(&ctx->up_ev[b], hipEventDisableTiming);
  return e;
}

static hipError_t h2d_packed(kfmi_dev_queries* dq, const char* src, DevCtx* ctx)
{
  /* reads per chunk: 100 MB of 100-bp ASCII in, 28 MB of words out (KFMI_UPLOAD_CHUNK: tests) */
  const char* ce = getenv("KFMI_UPLOAD_CHUNK");
  const uint64_t rows = dq->nwords + (dq->rem ? 1 : 0);
  uint64_t CQ = ce && atoll(ce) > 0 ? (uint64_t) atoll(ce) : 1ull << 20;
  /* long reads: 64 MB buffers; a requested chunk is held to 1 GB of words */
  const uint64_t cap = (ce ? 1ull << 30 : 64ull << 20) / (4 * rows);
  if (CQ > cap) CQ = cap;
  if (CQ < 1) CQ = 1;   /* one read per chunk at least: the loop below always advances */
  const uint64_t cq = dq->num < CQ ? dq->num : CQ;
  const uint64_t need = 4 * rows * cq;
  hipStream_t st = ctx->st;
  std::lock_guard<std::mutex> lk(ctx->up_mu);
  hipError_t e = upload_staging(ctx, need);
  for (uint64_t q0 = 0, i = 0; q0 < dq->num && e == hipSuccess; q0 += cq, ++i) {
    const int b = (int) (i & 1);
    if (i >= 2) e = hipEventSynchronize(ctx->up_ev[b]);
    if (e != hipSuccess) break;
    const uint64_t n = dq->num - q0 < cq ? dq->num - q0 : cq;
    par_pack(src + q0 * dq->size, n, dq->size, dq->rem, (uint32_t*) ctx->up_buf[b]);
    /* chunk rows (stride n) into the batch's word-major rows (stride num) */
    e = hipMemcpy2DAsync(dq->packed + q0, 4 * dq->num, ctx->up_buf[b], 4 * n, 4 * n, rows, hipMemcpyHostToDevice,
                         st);
    if (e == hipSuccess) e = hipEventRecord(ctx->up_ev[b], st);
  }
  const hipError_t es = hipStreamSynchronize(st);   /* the buffers are free again before the lock goes */
  return e != hipSuccess ? e : es;
}

/* kfmi_stream_release: the upload staging of every device */
void release_upload_staging()
{
  DeviceGuard dg;
  for (int dev = 0; dev < 64; ++dev) {
    DevCtx& c = g_ctx[dev];
    std::lock_guard<std::mutex> lk(c.up_mu);
    if (!c.up_cap) continue;
    (void) hipSetDevice(dev);
    for (int b = 0; b < 2; ++b) {
      if (c.up_buf[b]) (void) hipHostFree(c.up_buf[b]);
      c.up_buf[b] = nullptr;
      if (c.up_ev[b]) (void) hipEventDestroy(c.up_ev[b]);
      c.up_ev[b] = nullptr;
    }
    c.up_cap = 0;
  }
}

int32_t upload_queries(kfmi_qrys_t* q, uint32_t K, int dev, DevCtx* ctx)
{
  if (q->size == 0 || K == 0) return KFMI_E_BAD_ARGUMENT;
  kfmi_dev_queries* dq = new (std::nothrow) kfmi_dev_queries();
  if (!dq) return KFMI_E_ALLOCATING_MFASTA;
  dq->device = dev;
  dq->num = q->num;
  dq->size = q->size;
  query_geometry(dq, K);
  const uint64_t abytes = q->num * (uint64_t) q->size;
  const bool hp = upload_host_packed(q, K);
  if ((!hp && hipMalloc((void**) &dq->ascii, abytes + 16) != hipSuccess) ||
      hipMalloc((void**) &dq->packed, 4ull * (dq->nwords + 1) * (q->num ? q->num : 1)) != hipSuccess) {
    free_dev_queries(dq);
    return KFMI_E_DEVICE_ALLOC;
  }
  dq->packed_rows = dq->nwords + 1;
  if (abytes && ((hp ? h2d_packed(dq, q->h_queries, ctx) : h2d(dq->ascii, q->h_queries, abytes, ctx->st)) !=
                     hipSuccess ||
                 hipStreamSynchronize(ctx->st) != hipSuccess)) {
    free_dev_queries(dq);
    return KFMI_E_KERNEL;
  }
  if (q->dev) free_dev_queries(q->dev);
  q->dev = dq;
  return KFMI_SUCCESS;
}

hipError_t launch_pack(const kfmi_dev_queries* dq, hipStream_t st)
{
  if (dq->num == 0 || !dq->ascii) return hipSuccess;   /* no ASCII: packed by the host on upload */
  /* word chunks of at most 1 KiB of row bytes (K * SPW bases per word), rows
   * per block so that one block stages <= 64 KiB; m == rem (no K-step) runs
   * one empty chunk for the remainder codes */
  const uint32_t bpw = dq->K * (32u / (2u * dq->K));      /* bases per word: 16 (K = 1, 2, 4), 15 (K = 3) */
  const uint32_t wc = 1024u / bpw;
  const uint32_t nchunks = dq->nwords ? (dq->nwords + wc - 1) / wc : 1u;
  /* the largest slice a chunk stages: whole rows when one chunk covers them */
  const uint32_t pitch = nchunks == 1 ? dq->size : pack_pitch(dq->size, wc * bpw);
  uint32_t tq = 256;
  while ((uint64_t) tq * pitch > 64 * 1024 && tq > 64) tq >>= 1;
  const uint64_t blocks = (dq->num + tq - 1) / tq;
  if (blocks > 0xFFFFFFFFull || nchunks > 65535u) return hipErrorInvalidValue;
  const size_t lds = (size_t) tq * pitch + 16;
  const dim3 grid((uint32_t) blocks, nchunks);
  if (dq->K == 1)
    hipLaunchKernelGGL((pack_queries_kernel<1>), grid, dim3(256), lds, st, dq->ascii, dq->num, dq->size, dq->steps,
                       dq->nwords, tq, wc, dq->packed, dq->rem);
  else if (dq->K == 4)
    hipLaunchKernelGGL((pack_queries_kernel<4>), grid, dim3(256), lds, st, dq->ascii, dq->num, dq->size, dq->steps,
                       dq->nwords, tq, wc, dq->packed, dq->rem);
  else if (dq->K == 3)
    hipLaunchKernelGGL((pack_queries_kernel<3>), grid, dim3(256), lds, st, dq->ascii, dq->num, dq->size, dq->steps,
                       dq->nwords, tq, wc, dq->packed, dq->rem);
  else
    hipLaunchKernelGGL((pack_queries_kernel<2>), grid, dim3(256), lds, st, dq->ascii, dq->num, dq->size, dq->steps,
                       dq->nwords, tq, wc, dq->packed, dq->rem);
  return hipGetLastError();
}

/* ------------------------------------------------------------------------ */
/* C ABI: the reference's GPU plugin entry points                           */
/* ------------------------------------------------------------------------ */

/* interface.h:40, e.g. fmIndexGPU-Coop-2Step.cu:250-285 (index, $ arrays,
 * queries and zeroed results to the device; the index is re-laid-out for the
 * selected backend). */
uint32_t device_steps(const kfmi_fmi_t* f)
{
  if (f->dev) return f->dev->K;
  if (f->grp && ((const GroupIndex*) f->grp)->di[0]) return ((const GroupIndex*) f->grp)->di[0]->K;
  return f->steps;
}

extern "C" int32_t transferCPUtoGPU(void* index, void* queries, void* results)
{
  kfmi_fmi_t* f = (kfmi_fmi_t*) index;
  kfmi_qrys_t* q = (kfmi_qrys_t*) queries;
  kfmi_res_t* r = (kfmi_res_t*) results;
  DeviceGuard dg;
  int devs[KFMI_MAX_GROUP];
  const int ng = group_devices(devs);
  if (ng > 1) {
    std::unique_lock<RwLock> lk;
    if (f) lk = std::unique_lock<RwLock>(index_lock(f));
    return group_transfer(f, q, r, devs, ng);
  }
  if (q) group_free_queries(q);
  if (r) group_free_results(r);
  const int dev = kfmi_current_device();
  DevCtx* ctx = nullptr;
  int32_t err = ctx_for(dev, &ctx);
  if (err) return err;
  const int backend = f ? backend_for(f->steps) : kfmi_backend();
  uint32_t qk = f ? f->steps : 0;   /* K of the device copy, read under the handle's lock */
  if (f) {
    /* the index's device copy is replaced only under the handle's exclusive
     * lock (searches on other threads hold it shared); when it already fits,
     * nothing waits */
    auto fits = [&] { return !f->grp && f->dev && f->dev->backend == backend && f->dev->device == dev; };
    bool ok;
    {
      std::shared_lock<RwLock> sl(index_lock(f));
      ok = fits();
      if (ok) qk = device_steps(f);
    }
    if (!ok) {
      std::unique_lock<RwLock> ul(index_lock(f));
      if (!fits()) {
        group_free_index(f);   /* one mode per handle */
        err = upload_index(f, backend, dev, ctx);
        if (err) return err;
      }
      qk = device_steps(f);
    }
  }
  if (q) {
    if (!f) return KFMI_E_BAD_ARGUMENT;
    if (!q->h_queries && q->num) {   /* parsed on the device (kfmi_load_queries_gpu): already there */
      if (!q->dev) return KFMI_E_NOT_ON_DEVICE;
      if (q->dev->device != dev) return KFMI_E_BAD_ARGUMENT;
      query_geometry(q->dev, qk);
      kfmi_dev_queries* dq = q->dev;
      if (dq->nwords + 1 > dq->packed_rows) {   /* K = 3 packs 15 bases per word: a few more rows */
        (void) hipFree(dq->packed);
        dq->packed = nullptr;
        dq->packed_rows = 0;
        if (hipMalloc((void**) &dq->packed, 4ull * (dq->nwords + 1) * (dq->num ? dq->num : 1)) != hipSuccess)
          return KFMI_E_DEVICE_ALLOC;
        dq->packed_rows = dq->nwords + 1;
      }
    } else {
      err = upload_queries(q, qk, dev, ctx);
      if (err) return err;
    }
  }
  if (r) {
    if (r->d_results) {
      (void) hipSetDevice(r->d_device);
      (void) hipFree(r->d_results);
      r->d_results = nullptr;
      (void) hipSetDevice(dev);
    }
    if (hipMalloc((void**) &r->d_results, 8ull * (r->num ? r->num : 1)) != hipSuccess) return KFMI_E_DEVICE_ALLOC;
    r->d_device = dev;
    if (hipMemsetAsync(r->d_results, 0, 8ull * r->num, ctx->st) != hipSuccess ||
        hipStreamSynchronize(ctx->st) != hipSuccess)
      return KFMI_E_KERNEL;
  }
  return KFMI_SUCCESS;
}

/* Queues pack (if not fused) + LF of one device batch on `st`, bracketed by
 * ev[0..2]; search_finish waits and reads the timings. */
int32_t search_enqueue(kfmi_dev_index* di, kfmi_dev_queries* dq, uint32_t* d_res, hipStream_t st,
                              hipEvent_t* ev, uint32_t ftab)
{
  if (dq->device != di->device || dq->K != di->K) return KFMI_E_BAD_ARGUMENT;
  SearchLaunch a{};
  a.st = st;
  a.ix = idx_args(di);
  int32_t err = use_ftab(di, st, a.ix, ftab);
  if (!err) err = use_rtab(di, st, a.ix, dq->rem);
  if (err) return err;
  a.qp = dq->packed;
  a.ascii = dq->ascii;
  a.m = dq->size;
  a.maxw = dq->ascii ? fused_maxw(di->backend, dq->K * dq->steps) : 0;
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

int32_t search_finish(hipStream_t st, hipEvent_t* ev, double* ms)
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

extern "C" int32_t kfmi_search(void* index, void* queries, void* results)
{
  kfmi_fmi_t* f = (kfmi_fmi_t*) index;
  kfmi_qrys_t* q = (kfmi_qrys_t*) queries;
  kfmi_res_t* r = (kfmi_res_t*) results;
  if (!f || !q || !r) return KFMI_E_BAD_ARGUMENT;
  if (q->num != r->num) return KFMI_E_BAD_ARGUMENT;
  DeviceGuard dg;
  std::shared_lock<RwLock> lk(index_lock(f));
  if (f->grp || q->grp || r->grp) return group_search(f, q, r);
  if (!f->dev || !q->dev || !r->d_results) return KFMI_E_NOT_ON_DEVICE;
  kfmi_dev_index* di = f->dev;
  if (r->d_device != di->device) return KFMI_E_BAD_ARGUMENT;   /* handles transferred to different devices */
  DevCtx* ctx = nullptr;
  int32_t err = ctx_for(di->device, &ctx);
  hipEvent_t* ev = err ? nullptr : thread_events(di->device);
  hipStream_t st = err ? nullptr : thread_stream(di->device);
  if (!err && (!ev || !st)) err = KFMI_E_NO_DEVICE;
  if (!err) err = search_enqueue(di, q->dev, r->d_results, st, ev, ftab_bases());
  if (!err) err = search_finish(st, ev, t_ms);
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

static int32_t count_on(kfmi_dev_index* di, kfmi_dev_queries* dq, Op op, uint64_t* out, int nout);

/* A statistics launch over the batch (Op::Count: one total; Op::CountLines:
 * four), on a device group summed over the members' slices. */
static int32_t count_stat(void* index, void* queries, Op op, uint64_t* out, int nout)
{
  kfmi_fmi_t* f = (kfmi_fmi_t*) index;
  kfmi_qrys_t* q = (kfmi_qrys_t*) queries;
  if (!f || !q || !out) return KFMI_E_BAD_ARGUMENT;
  DeviceGuard dg;
  std::shared_lock<RwLock> lk(index_lock(f));
  if (f->grp || q->grp) {
    GroupIndex* gi = (GroupIndex*) f->grp;
    GroupSlices* gq = (GroupSlices*) q->grp;
    if (!gi || !gq) return KFMI_E_NOT_ON_DEVICE;   /* handles moved to different modes */
    if (gq->n != gi->n) return KFMI_E_BAD_ARGUMENT;
    for (int j = 0; j < nout; ++j) out[j] = 0;
    for (int i = 0; i < gi->n; ++i) {
      uint64_t part[4] = {0, 0, 0, 0};
      const int32_t e = count_on(gi->di[i], gq->dq[i], op, part, nout);
      if (e) return e;
      for (int j = 0; j < nout; ++j) out[j] += part[j];
    }
    return KFMI_SUCCESS;
  }
  if (!f->dev || !q->dev) return KFMI_E_NOT_ON_DEVICE;
  return count_on(f->dev, q->dev, op, out, nout);
}

/* Distinct d-blocks the batch's LF steps touch (SURVEY 8(d) algorithmic bytes);
 * on a device group the sum over the members' slices. */
extern "C" int32_t kfmi_count_blocks(void* index, void* queries, uint64_t* blocks)
{
  return count_stat(index, queries, Op::Count, blocks, 1);
}

/* The 128-B lines the backend's task-kernel fetches touch over the batch
 * (count_lines_kernel): out[0] distinct lines per K-step summed, out[1] ends
 * whose counter lies outside their planes' line, out[2] ends fetched, out[3]
 * ends counted forward from block b-1. */
extern "C" int32_t kfmi_count_lines(void* index, void* queries, uint64_t* out)
{
  return count_stat(index, queries, Op::CountLines, out, 4);
}

static int32_t count_on(kfmi_dev_index* di, kfmi_dev_queries* dq, Op op, uint64_t* out, int nout)
{
  DevCtx* ctx = nullptr;
  int32_t err = ctx_for(di->device, &ctx);
  if (err) return err;
  SearchLaunch a{};
  a.st = ctx->st;
  a.ix = idx_args(di);
  if (dq->device != di->device || dq->K != di->K) return KFMI_E_BAD_ARGUMENT;
  err = use_rtab(di, ctx->st, a.ix, dq->rem);
  if (err) return err;
  unsigned long long* d_total = nullptr;
  HIP_OK(hipMalloc((void**) &d_total, 4 * sizeof(unsigned long long)));
  a.qp = dq->packed;
  a.ascii = dq->ascii;
  a.m = dq->size;
  a.maxw = 0;
  a.num = dq->num;
  a.steps = dq->steps;
  a.nwords = dq->nwords;
  a.res = nullptr;
  unsigned long long total[4] = {0, 0, 0, 0};
  bool ok = hipMemsetAsync(d_total, 0, sizeof(total), ctx->st) == hipSuccess &&
            launch_pack(dq, ctx->st) == hipSuccess &&
            (dq->num == 0 || dispatch(op, di->K, di->nb, di->layout, a, d_total) == hipSuccess) &&
            hipMemcpyAsync(total, d_total, sizeof(total), hipMemcpyDeviceToHost, ctx->st) == hipSuccess &&
            hipStreamSynchronize(ctx->st) == hipSuccess;
  (void) hipFree(d_total);
  if (!ok) return KFMI_E_KERNEL;
  for (int j = 0; j < nout && j < 4; ++j) out[j] = total[j];
  return KFMI_SUCCESS;
}

/* How the reads of `queries` sit on the device: 0 not there, 1 ASCII, 2 code
 * words packed by the host on upload (of the first member for a group). */
extern "C" int32_t kfmi_queries_upload_form(void* queries)
{
  const kfmi_qrys_t* q = (const kfmi_qrys_t*) queries;
  if (!q) return 0;
  const kfmi_dev_queries* dq = q->dev;
  const GroupSlices* g = (const GroupSlices*) q->grp;
  if (g && g->n > 0) dq = g->dq[0];
  if (!dq) return 0;
  return dq->ascii ? 1 : 2;
}

/* interface.h:39, Coop-2Step.cu:287-293 */
extern "C" int32_t transferGPUtoCPU(void* results)
{
  kfmi_res_t* r = (kfmi_res_t*) results;
  DeviceGuard dg;
  if (r) r->origin = KFMI_RES_FROM_GPU;
  if (r && r->grp) return group_to_host(r);
  if (!r || !r->d_results) return KFMI_E_NOT_ON_DEVICE;
  DevCtx* ctx = nullptr;
  int32_t err = ctx_for(r->d_device, &ctx);   /* the device the results live on, not the caller's current one */
  if (err) return err;
  HIP_OK(hipMemcpyAsync(r->h_results, r->d_results, 8ull * r->num, hipMemcpyDeviceToHost, ctx->st));
  HIP_OK(hipStreamSynchronize(ctx->st));
  return KFMI_SUCCESS;
}

/* interface.h:38, Task-1Step.cu:236-256: releases and NULLs the device copy */
extern "C" int32_t freeIndexGPU(void** index)
{
  kfmi_fmi_t* f = index ? (kfmi_fmi_t*) *index : nullptr;
  if (!f) return KFMI_SUCCESS;
  DeviceGuard dg;
  std::unique_lock<RwLock> lk(index_lock(f));
  group_free_index(f);
  if (f->dev) {
    free_dev_index(f->dev);
    f->dev = nullptr;
  }
  return KFMI_SUCCESS;
}

extern "C" int32_t freeQueriesGPU(void** queries)
{
  DeviceGuard dg;
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
  DeviceGuard dg;
  kfmi_res_t* r = results ? (kfmi_res_t*) *results : nullptr;
  if (r) group_free_results(r);
  if (r && r->d_results) {
    (void) hipSetDevice(r->d_device);
    (void) hipFree(r->d_results);
    r->d_results = nullptr;
  }
  return KFMI_SUCCESS;
}

extern "C" uint64_t kfmi_device_index_bytes(void* index)
{
  kfmi_fmi_t* f = (kfmi_fmi_t*) index;
  if (!f) return 0;
  std::shared_lock<RwLock> lk(index_lock(f));
  if (f->grp) {   /* all replicas of a device group */
    const GroupIndex* g = (const GroupIndex*) f->grp;
    uint64_t b = 0;
    for (int i = 0; i < g->n; ++i) b += g->di[i]->ent_bytes + g->di[i]->sa_bytes;
    return b;
  }
  if (!f || !f->dev) return 0;
  return f->dev->ent_bytes + f->dev->sa_bytes;
}

}  // namespace kfmi
