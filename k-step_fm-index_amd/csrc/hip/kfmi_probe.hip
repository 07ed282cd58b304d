/*
 * kfmi_probe.hip -- replay probe (diagnostic; DESIGN.md 5 "The ceiling,
 * measured on the kernel's own requests").  Is the LF kernel at the memory
 * system's request ceiling, or is it held below it by its dependent chain?
 *
 * gather_probe measures uniformly random lines; the LF kernel's requests are
 * a mix (its first K-steps touch a few thousand lines that stay in L2, the
 * next ones ~10^5-10^6 lines that live in the Infinity Cache, the rest are
 * HBM).  This probe replays that exact mix: a trace launch walks the batch with
 * the search's own LF and records, for every (K-step, read), the MID128 line
 * each end reads (kfmi_probe_replay, MID layouts at K = 2, d = 64 only); the
 * replay launch then issues the same loads per line as the task kernel (both
 * 16-byte plane chunks and the counter word), with the addresses read from
 * the trace instead of computed from the previous step -- no dependence, and
 * `unroll` K-steps of loads in flight per lane.  Its line rate bounds what any
 * issue order can get from the request stream the search must make.
 *
 * Trace entry (u32 per end): line index (bits 0-24), block parity (25), code
 * c (26-29), bit 31 = R in L's block (the kernel loads nothing for it).
 * Layout [wave][step][lane][end]: 8 bytes per read per K-step, a wave's 512 B
 * per step contiguous and its steps adjacent, so each wave streams its own
 * 25.6 KB (100 bp) -- a few pages per wave, not one per step (the table's
 * gathers already press on the translation reach); reported as trace_bytes.
 * The gathers are issued as `groups` (1 or 2) exec-masked lane groups, as the
 * task kernel issues them (two 32-lane groups on tables over 2 GB, DESIGN.md
 * 5): the two groups' loads name two copies of the table pointer, so the
 * compiler cannot merge them into one instruction.
 */
#include <hip/hip_runtime.h>

#include "kfmi_runtime.h"

namespace kfmi {
namespace {

using GM = Geo<2, 2, LAY_MID>;
constexpr uint32_t LINE_BITS = 25;

__global__ __launch_bounds__(256) void trace_lines_kernel(IdxArgs ix, const uint32_t* __restrict__ qp, uint64_t num,
                                                          uint32_t steps, uint32_t* __restrict__ trace)
{
  const uint64_t q = (uint64_t) blockIdx.x * 256 + threadIdx.x;
  if (q >= num) return;
  uint32_t L = 0, R = ix.bwtsize;
  for (uint32_t t = 0; t < steps; ++t) {
    const uint32_t word = qp[(uint64_t) (t / GM::SPW) * num + q];
    const uint32_t c = (word >> (2 * GM::K * (t % GM::SPW))) & (uint32_t) (GM::NC - 1);
    const uint32_t bl = L / (uint32_t) GM::D, br = R / (uint32_t) GM::D;
    uint2 e;
    e.x = (bl >> 1) | ((bl & 1u) << LINE_BITS) | (c << 26);
    e.y = (br >> 1) | ((br & 1u) << LINE_BITS) | (c << 26) | (br == bl ? 0x80000000u : 0u);
    reinterpret_cast<uint2*>(trace)[((q >> 6) * steps + t) * 64 + (q & 63)] = e;
    uint32_t sx[2 * GM::K];
    plane_xor<GM::K>(c, sx);
    L = lf_stream<GM>(ix, L, c, sx);
    R = lf_stream<GM>(ix, R, c, sx);
  }
}

struct EndLoads {
  uint4 a, b;
  uint32_t cnt;
};

/* the task kernel's loads for one end: block b's two 16-B plane chunks and the
 * counter word of code c in its MID128 line */
__device__ __forceinline__ EndLoads replay_end(const uint32_t* __restrict__ ent, uint32_t e)
{
  const uint32_t* line = ent + (uint64_t) (e & ((1u << LINE_BITS) - 1u)) * GM::EW;
  const uint32_t* pl = line + ((e >> LINE_BITS) & 1u) * GM::BMW;
  return {*reinterpret_cast<const uint4*>(pl), *reinterpret_cast<const uint4*>(pl + 4), line[GM::MIDCNT + ((e >> 26) & 15u)]};
}

template <int U>
__device__ __forceinline__ void replay_issue(const uint32_t* __restrict__ ent, const uint2 (&e)[U], EndLoads (&l)[U],
                                             EndLoads (&r)[U])
{
#pragma unroll
  for (int u = 0; u < U; ++u) {
    l[u] = replay_end(ent, e[u].x);
    if (!(e[u].y >> 31)) r[u] = replay_end(ent, e[u].y);
    else r[u] = EndLoads{make_uint4(0u, 0u, 0u, 0u), make_uint4(0u, 0u, 0u, 0u), 0u};
  }
}

template <int U, int GR>
__global__ __launch_bounds__(256) void replay_lines_kernel(const uint32_t* __restrict__ ent_a,
                                                           const uint32_t* __restrict__ ent_b,
                                                           const uint32_t* __restrict__ trace, uint64_t num,
                                                           uint32_t steps, uint32_t* __restrict__ sink)
{
  const uint64_t q = (uint64_t) blockIdx.x * 256 + threadIdx.x;
  if (q >= num) return;
  const uint2* tr = reinterpret_cast<const uint2*>(trace) + (q >> 6) * steps * 64 + (q & 63);
  const bool hi = (threadIdx.x & 32) != 0;
  uint32_t acc = 0;
  for (uint32_t t = 0; t < steps; t += U) {
    uint2 e[U];
#pragma unroll
    for (int u = 0; u < U; ++u) e[u] = t + u < steps ? tr[(uint64_t) (t + u) * 64] : make_uint2(0u, 0x80000000u);
    EndLoads l[U], r[U];
    if (GR == 1 || !hi) replay_issue<U>(ent_a, e, l, r);   // lanes 0-31 (all lanes: GR 1)
    else replay_issue<U>(ent_b, e, l, r);                    // lanes 32-63, their own instructions
#pragma unroll
    for (int u = 0; u < U; ++u)
      acc ^= l[u].a.x ^ l[u].a.y ^ l[u].a.z ^ l[u].a.w ^ l[u].b.x ^ l[u].b.y ^ l[u].b.z ^ l[u].b.w ^ l[u].cnt ^
             r[u].a.x ^ r[u].a.y ^ r[u].a.z ^ r[u].a.w ^ r[u].b.x ^ r[u].b.y ^ r[u].b.z ^ r[u].b.w ^ r[u].cnt;
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;   /* keeps the loads; practically never stored */
}

/* unroll 0: the task kernel's own fetch (fetch_ends_x4, the asm block that
 * issues both ends' loads under per-group exec masks and waits once), one
 * K-step per lane in flight as in the kernel, on rows rebuilt from the trace
 * (any row of the recorded block gives the same addresses); the next step's
 * trace entry is loaded before each fetch */
template <int SPLIT>
__global__ __launch_bounds__(256) void replay_fetch_kernel(IdxArgs ix, const uint32_t* __restrict__ trace,
                                                           uint64_t num, uint32_t steps, uint32_t* __restrict__ sink)
{
  const uint64_t q = (uint64_t) blockIdx.x * 256 + threadIdx.x;
  if (q >= num) return;
  const uint2* tr = reinterpret_cast<const uint2*>(trace) + (q >> 6) * steps * 64 + (q & 63);
  uint32_t acc = 0;
  uint2 e = tr[0];
  for (uint32_t t = 0; t < steps; ++t) {
    const uint2 en = t + 1 < steps ? tr[(uint64_t) (t + 1) * 64] : e;
    const uint32_t bl = 2u * (e.x & ((1u << LINE_BITS) - 1u)) + ((e.x >> LINE_BITS) & 1u);
    const uint32_t br = 2u * (e.y & ((1u << LINE_BITS) - 1u)) + ((e.y >> LINE_BITS) & 1u);
    const uint32_t c = (e.x >> 26) & 15u;
    const uint32_t L = bl * (uint32_t) GM::D, R = (e.y >> 31) ? L : br * (uint32_t) GM::D;
    Blk<GM> kl, kr;
    fetch_ends_x4<GM, SPLIT>(ix, L, R, c, kl, kr);
#pragma unroll
    for (int i = 0; i < GM::BMW; ++i) acc ^= kl.bm[i] ^ kr.bm[i];
    acc ^= kl.cnt ^ kr.cnt;
    e = en;
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;
}

template <int U>
hipError_t launch_replay(int groups, const uint32_t* ent, const uint32_t* trace, uint64_t num, uint32_t steps,
                         uint32_t* sink, hipStream_t st)
{
  const uint64_t blocks = (num + 255) / 256;
  if (groups == 2)
    hipLaunchKernelGGL((replay_lines_kernel<U, 2>), dim3((uint32_t) blocks), dim3(256), 0, st, ent, ent, trace, num,
                       steps, sink);
  else
    hipLaunchKernelGGL((replay_lines_kernel<U, 1>), dim3((uint32_t) blocks), dim3(256), 0, st, ent, ent, trace, num,
                       steps, sink);
  return hipGetLastError();
}

}  // namespace
}  // namespace kfmi

using namespace kfmi;

/* Diagnostic (not in the reference): replays the MID128 line requests of a
 * search of `queries` on `index` (uploaded for task-mid or coop-mid, K = 2,
 * d = 64, m % K == 0).  `unroll` (1, 2, 4 or 8): K-steps of loads in flight
 * per lane (C++ loads); 0: the task kernel's own asm fetch, one K-step in
 * flight; `groups` (1, 2): exec-masked lane groups of the gathers; `reps`
 * timed launches after one warm-up.  Out: mean replay launch
 * time (ms), the lines the replay fetches per launch (L's line every step, R's
 * where it lies in another block -- the fetches of the task kernel), and the
 * trace bytes it streams beside them. */
extern "C" int32_t kfmi_probe_replay(void* index, void* queries, int32_t unroll, int32_t groups, int32_t reps,
                                     double* ms, uint64_t* lines, uint64_t* trace_bytes)
{
  kfmi_fmi_t* f = (kfmi_fmi_t*) index;
  kfmi_qrys_t* q = (kfmi_qrys_t*) queries;
  if (!f || !q || !ms || !lines || !trace_bytes || reps < 1) return KFMI_E_BAD_ARGUMENT;
  if (unroll != 0 && unroll != 1 && unroll != 2 && unroll != 4 && unroll != 8) return KFMI_E_BAD_ARGUMENT;
  if (groups != 1 && groups != 2) return KFMI_E_BAD_ARGUMENT;
  DeviceGuard dg;
  std::shared_lock<RwLock> lk(index_lock(f));
  if (!f->dev || !q->dev || f->grp || q->grp) return KFMI_E_NOT_ON_DEVICE;
  kfmi_dev_index* di = f->dev;
  kfmi_dev_queries* dq = q->dev;
  if (di->layout != LAY_MID || di->K != 2 || di->nb != 2 || dq->K != 2 || dq->rem) return KFMI_E_BAD_ARGUMENT;
  if (dq->device != di->device || di->ent_bytes / (GM::EW * 4) >= (1ull << LINE_BITS)) return KFMI_E_BAD_ARGUMENT;
  DevCtx* ctx = nullptr;
  int32_t err = ctx_for(di->device, &ctx);
  if (err) return err;
  const uint64_t num = dq->num, steps = dq->steps, tbytes = 8ull * steps * ((num + 63) / 64 * 64);
  uint32_t* trace = nullptr;
  uint32_t* sink = nullptr;
  unsigned long long* d_total = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  HIP_OK(hipMalloc((void**) &trace, tbytes ? tbytes : 8));
  bool ok = hipMalloc((void**) &sink, 4) == hipSuccess && hipMalloc((void**) &d_total, 8) == hipSuccess &&
            hipEventCreate(&e0) == hipSuccess && hipEventCreate(&e1) == hipSuccess &&
            hipMemsetAsync(d_total, 0, 8, ctx->st) == hipSuccess && launch_pack(dq, ctx->st) == hipSuccess;
  const IdxArgs ix = idx_args(di);
  const uint64_t blocks = (num + 255) / 256;
  if (ok && num) {
    hipLaunchKernelGGL(trace_lines_kernel, dim3((uint32_t) blocks), dim3(256), 0, ctx->st, ix, dq->packed, num,
                       (uint32_t) steps, trace);
    /* the fetched lines: count_blocks' distinct blocks (L's, and R's when it differs) */
    SearchLaunch a{};
    a.st = ctx->st;
    a.ix = ix;
    a.qp = dq->packed;
    a.num = num;
    a.steps = dq->steps;
    a.nwords = dq->nwords;
    ok = hipGetLastError() == hipSuccess && dispatch(Op::Count, 2, 2, LAY_MID, a, d_total) == hipSuccess;
  }
  auto run = [&]() -> bool {
    if (unroll == 0) {
      const uint64_t blocks2 = (num + 255) / 256;
      if (groups == 2)
        hipLaunchKernelGGL((replay_fetch_kernel<7>), dim3((uint32_t) blocks2), dim3(256), 0, ctx->st, ix, trace, num,
                           (uint32_t) steps, sink);
      else
        hipLaunchKernelGGL((replay_fetch_kernel<8>), dim3((uint32_t) blocks2), dim3(256), 0, ctx->st, ix, trace, num,
                           (uint32_t) steps, sink);
      return hipGetLastError() == hipSuccess;
    }
    switch (unroll) {
      case 1: return launch_replay<1>(groups, di->ent, trace, num, (uint32_t) steps, sink, ctx->st) == hipSuccess;
      case 2: return launch_replay<2>(groups, di->ent, trace, num, (uint32_t) steps, sink, ctx->st) == hipSuccess;
      case 4: return launch_replay<4>(groups, di->ent, trace, num, (uint32_t) steps, sink, ctx->st) == hipSuccess;
      default: return launch_replay<8>(groups, di->ent, trace, num, (uint32_t) steps, sink, ctx->st) == hipSuccess;
    }
  };
  float total_ms = 0.f;
  unsigned long long total = 0;
  if (ok && num) {
    ok = run() && hipEventRecord(e0, ctx->st) == hipSuccess;
    for (int i = 0; ok && i < reps; ++i) ok = run();
    ok = ok && hipEventRecord(e1, ctx->st) == hipSuccess && hipEventSynchronize(e1) == hipSuccess &&
         hipEventElapsedTime(&total_ms, e0, e1) == hipSuccess &&
         hipMemcpy(&total, d_total, 8, hipMemcpyDeviceToHost) == hipSuccess;
  }
  if (e0) (void) hipEventDestroy(e0);
  if (e1) (void) hipEventDestroy(e1);
  (void) hipFree(d_total);
  (void) hipFree(sink);
  (void) hipFree(trace);
  if (!ok) return KFMI_E_KERNEL;
  *ms = (double) total_ms / reps;
  *lines = total;
  *trace_bytes = tbytes;
  return KFMI_SUCCESS;
}
